# A/B of library variants (tools/gpu_ab.sh), then the full -m gpu suite on
# the candidate build (cms-bwt_amd/build).  Usage: bash tools/gpu_ab_suite.sh TAG variant...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=$1; shift
bash tools/gpu_ab.sh "$@" 2>&1 | tee gpurun_out/${tag}_ab.log || exit 1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_suite.log 2>&1 || { tail -60 gpurun_out/${tag}_gpu_suite.log; exit 1; }
tail -2 gpurun_out/${tag}_gpu_suite.log
