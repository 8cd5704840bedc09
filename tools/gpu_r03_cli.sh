# Boundary tests + bench (e2e leg) on one box
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_parity.py -x -v -m gpu -k "cli or config1 or small_cases_rle" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_cli.log 2>&1 || { tail -60 gpurun_out/t_cli.log; exit 1; }
tail -3 gpurun_out/t_cli.log
timeout -k 10 500 python bench.py > gpurun_out/bench_e2e.log 2>&1 || { tail -20 gpurun_out/bench_e2e.log; exit 1; }
tail -1 gpurun_out/bench_e2e.log
