# Full GPU suite + smoke, then round-3 profiling evidence
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gpu.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/t_gpu.log | head -20; tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
bash tools/gpu_r03_prof.sh
