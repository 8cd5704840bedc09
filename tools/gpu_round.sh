# Round check (run through gpurun from the repo root): GPU tests, default bench, kernel trace stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gpu.log 2>&1 || { tail -60 gpurun_out/t_gpu.log; exit 1; }
tail -3 gpurun_out/t_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
rm -rf gpurun_out/kt; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/kt.log 2>&1
python3 tools/kstats.py gpurun_out/kt/kt_kernel_stats.csv > gpurun_out/kt_summary.txt && head -30 gpurun_out/kt_summary.txt
