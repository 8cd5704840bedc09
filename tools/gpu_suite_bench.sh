# Round 4, box I: the full -m gpu suite on the candidate build, then the
# default bench line (with the CPU baseline and the end-to-end leg).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_gpu_suite.log 2>&1 || { tail -60 gpurun_out/r04i_gpu_suite.log; exit 1; }
tail -2 gpurun_out/r04i_gpu_suite.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04i_bench.log 2>&1 || { tail -30 gpurun_out/r04i_bench.log; exit 1; }
tail -1 gpurun_out/r04i_bench.log | cut -c1-1500
