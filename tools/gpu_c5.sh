# End-to-end CLI (GPU reader + device index) and config-5-shaped bench runs
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -n "$SKIP_E2E" ] || E2E_CONFIGS="${E2E_CONFIGS:-10000000 1000 0.001 4 c3}" bash tools/gpu_e2e.sh
for c in ${C5_COPIES:-4 20 60}; do
    timeout -k 10 400 python bench.py --ref-len 100000000 --copies $c --p 0.01 --seed 5 --plain --steps 1 --warmup 1 --no-cpu --no-e2e > gpurun_out/c5_$c.json 2> gpurun_out/c5_$c.err || { tail -5 gpurun_out/c5_$c.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c5_$c.json').read().strip().splitlines()[-1]); print('c5 copies $c', d['value'], 'MB/s', d['ms_per_step'], 'ms', d['config']['heads'], 'heads', d['stages_ms'])"
done
