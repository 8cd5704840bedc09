# Kernel timeline of the last bench step (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/kt2; timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt2 -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-e2e --no-check > gpurun_out/kt2.log 2>&1
python3 tools/ktrace.py gpurun_out/kt2/kt_kernel_trace.csv > gpurun_out/trace.txt
cat gpurun_out/trace.txt
