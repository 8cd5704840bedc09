# The full -m gpu suite on the candidate build, then the default bench line
# (with the CPU baseline and the end-to-end leg); TAG names the logs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-suite}
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || { tail -60 gpurun_out/${TAG}_gpu_suite.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_suite.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-1500
