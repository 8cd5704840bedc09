# Round evidence (through gpurun): kernel stats + PMC passes, one-step timeline, default bench with CPU baseline
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_prof_r.sh > gpurun_out/prof_r.log 2>&1 || { tail -20 gpurun_out/prof_r.log; exit 1; }
python3 tools/pmc_main.py gpurun_out/prof > gpurun_out/prof/pmc_main.json
# the bench line below reads its traffic from this run's counters
PMCF=$(python3 -c "import bench; print(bench.PMC_FILE)")
cp gpurun_out/prof/pmc_main.json profiles/$PMCF
bash tools/gpu_timeline.sh > /dev/null
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log | cut -c1-300
