# Sharded merge + sharded ingest: GPU tests, then W=1 bench + kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_dist.py tests/test_gpu_reader.py -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sh.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/t_sh.log | head -20; tail -40 gpurun_out/t_sh.log; exit 1; }
tail -2 gpurun_out/t_sh.log
bash tools/gpu_sharded1_prof.sh
