# Round 4, box G: the counter stream-path parity tests, then the round
# evidence (kernel stats, PMC passes, one-step timeline, default bench line).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "counter_stream or doubling_group" --timeout 120 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1 || { tail -40 gpurun_out/r04g_tests.log; exit 1; }
tail -1 gpurun_out/r04g_tests.log
bash tools/gpu_round_prof.sh
