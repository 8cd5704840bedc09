# kernel trace of the default bench (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/kt; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/kt.log 2>&1
python3 tools/kstats.py gpurun_out/kt/kt_kernel_stats.csv > gpurun_out/kt_summary.txt && head -60 gpurun_out/kt_summary.txt
