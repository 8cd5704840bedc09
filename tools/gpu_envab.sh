# A/B of environment settings on the default bench (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$TESTSEL" ]; then
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "$TESTSEL" > gpurun_out/t_ab.log 2>&1 || { tail -40 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
fi
IFS=';' read -ra CFGS <<< "${CFGS:-X=1}"
for cfg in "${CFGS[@]}"; do
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/b_ab.log 2>&1 || { tail -20 gpurun_out/b_ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/b_ab.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
done
