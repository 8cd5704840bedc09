# Sharded merge: its GPU tests, then the W=1 bench line and one-step timeline (through gpurun)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_dist.py -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sharded.log 2>&1 || { grep -E "Error|error|assert" gpurun_out/t_sharded.log | head -20; tail -30 gpurun_out/t_sharded.log; exit 1; }
tail -1 gpurun_out/t_sharded.log
bash tools/gpu_r03_sharded_tl.sh
