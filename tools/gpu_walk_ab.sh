# walk change check: walk parity tests, config-3 golden, bench timing, walk step stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_par.log 2>&1 || { tail -60 gpurun_out/t_par.log; exit 1; }
tail -2 gpurun_out/t_par.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
CMSBWT_W2_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/b_st.log 2> gpurun_out/w2stats.log || { tail -20 gpurun_out/w2stats.log; exit 1; }
grep w2stats gpurun_out/w2stats.log
