# Default bench + optional env A/B (no tests), through gpurun
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['stages_ms'])"
if [ -n "$AB_ENV" ]; then
  env $AB_ENV timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print('AB',d['ms_per_step'],d['stages_ms'])"
fi
