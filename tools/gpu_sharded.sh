# sharded-merge tests (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_sh.log 2>&1 || { tail -80 gpurun_out/t_sh.log; exit 1; }
tail -5 gpurun_out/t_sh.log
