# Round 4, first box: the CLI's multi-GPU path (-n) on one GPU, config 4
# through bench.py's N>1 path at W=2/4/8 (gloo), config-5 walk sizing, and a
# short N=1 bench with the parity check.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cli_multi.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_cli_multi.log 2>&1 || { tail -60 gpurun_out/r04_cli_multi.log; exit 1; }
tail -3 gpurun_out/r04_cli_multi.log
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/r04_bench1.log 2>&1 || { tail -30 gpurun_out/r04_bench1.log; exit 1; }
tail -1 gpurun_out/r04_bench1.log | cut -c1-400
timeout -k 10 300 python -u tools/c5_size.py > gpurun_out/r04_c5.log 2>&1 || { tail -30 gpurun_out/r04_c5.log; exit 1; }
tail -2 gpurun_out/r04_c5.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py -x -v -s --timeout 580 --timeout-method thread > gpurun_out/r04_c4.log 2>&1 || { tail -40 gpurun_out/r04_c4.log; exit 1; }
grep -E "passed|failed|world" gpurun_out/r04_c4.log | cut -c1-600
