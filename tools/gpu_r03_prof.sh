# Round-3 evidence: walk step statistics, one-step timeline, kernel stats + PMC passes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_W2_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-e2e > gpurun_out/w2stats.log 2>&1 || { tail -5 gpurun_out/w2stats.log; exit 1; }
grep w2stats gpurun_out/w2stats.log | tail -32 > gpurun_out/w2stats.txt; cat gpurun_out/w2stats.txt
bash tools/gpu_timeline.sh > /dev/null && tail -3 gpurun_out/trace.txt
bash tools/gpu_prof_r.sh > gpurun_out/prof_r.log 2>&1 || { tail -20 gpurun_out/prof_r.log; exit 1; }
python3 tools/pmc_main.py gpurun_out/prof > gpurun_out/prof/pmc_main.json
head -12 gpurun_out/prof/kt_summary.txt
