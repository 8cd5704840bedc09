# Sharded merge: composite-key grouping paths and the 4-rank config-5 proxy (plain .bwt)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py -x -v -m gpu -k "composite_key or config5 or world1_matches" --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sh5.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/t_sh5.log | head -20; tail -40 gpurun_out/t_sh5.log; exit 1; }
tail -2 gpurun_out/t_sh5.log
