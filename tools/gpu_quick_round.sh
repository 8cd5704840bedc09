# Full GPU suite + default bench + kernel-trace stats (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gpu.log 2>&1 || { tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
rm -rf gpurun_out/kt; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/kt.log 2>&1
python3 tools/kstats.py gpurun_out/kt/kt_kernel_stats.csv > gpurun_out/kt_summary.txt && grep -E "nhr|run_bin|finalize" gpurun_out/kt_summary.txt
