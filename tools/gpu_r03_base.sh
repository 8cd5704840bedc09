set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/base_bench.log 2>&1 || { tail -20 gpurun_out/base_bench.log; exit 1; }
tail -1 gpurun_out/base_bench.log | cut -c1-400
rm -rf gpurun_out/kt; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/kt.log 2>&1
python3 tools/kstats.py gpurun_out/kt/kt_kernel_stats.csv > gpurun_out/kt_summary.txt && head -40 gpurun_out/kt_summary.txt
