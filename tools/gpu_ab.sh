# A/B helper (run through gpurun from the repo root): GPU tests, bench variants
set -e
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu --timeout 300 -p no:cacheprovider -x -k "not config3" > gpurun_out/t_v2.log 2>&1 || { tail -50 gpurun_out/t_v2.log; exit 1; }
tail -1 gpurun_out/t_v2.log
CMSBWT_W2_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/b.log 2> gpurun_out/stats.log || { cat gpurun_out/b.log gpurun_out/stats.log; exit 1; }
grep w2stats gpurun_out/stats.log
for cfg in "X=1"; do
    echo "== $cfg"
    env $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b.log 2>&1 || { cat gpurun_out/b.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'])"
done
