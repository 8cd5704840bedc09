# Round 4, box J: the full -m gpu suite, smoke() and the default bench line on
# the final tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j_gpu_suite.log 2>&1 || { tail -60 gpurun_out/r04j_gpu_suite.log; exit 1; }
tail -2 gpurun_out/r04j_gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04j_smoke.log 2>&1 || { tail -20 gpurun_out/r04j_smoke.log; exit 1; }
tail -1 gpurun_out/r04j_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r04j_bench.log 2>&1 || { tail -20 gpurun_out/r04j_bench.log; exit 1; }
tail -1 gpurun_out/r04j_bench.log | cut -c1-400
