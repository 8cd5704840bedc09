# Parity + sharded tests of the single-GPU path, default bench (+ optional env A/B), through gpurun
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_par.log 2>&1 || { tail -40 gpurun_out/t_par.log; exit 1; }
tail -2 gpurun_out/t_par.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['stages_ms'])"
if [ -n "$AB_ENV" ]; then
  env $AB_ENV timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('AB',d['ms_per_step'],d['stages_ms'])"
fi
