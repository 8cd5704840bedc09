# Tests + end-to-end timing (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTSEL:+-k "$TESTSEL"} > gpurun_out/t_gpu.log 2>&1 || { tail -60 gpurun_out/t_gpu.log; exit 1; }
tail -3 gpurun_out/t_gpu.log
grep -E "c5p|config5|reader" gpurun_out/t_gpu.log | tail -30 || true
bash tools/gpu_e2e.sh
