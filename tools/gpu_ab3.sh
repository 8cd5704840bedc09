# A/B of library builds under exp/ (run through gpurun from the repo root):
# walk-path parity on the default build, then the bench per variant.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${TESTSEL:-gpu_index or small_cases or chunk_restarts or large_reference or config1 or config3_full or config2}" > gpurun_out/t_walk.log 2>&1 || { tail -40 gpurun_out/t_walk.log; exit 1; }
tail -1 gpurun_out/t_walk.log
fi
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then lib=""; else lib="$PWD/exp/$v/libcmsbwt.so"; fi
  CMSBWT_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
done
if [ -n "$STATS" ]; then
CMSBWT_W2_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/b_st.log 2> gpurun_out/w2stats.log || { tail -20 gpurun_out/b_st.log gpurun_out/w2stats.log; exit 1; }
grep w2stats gpurun_out/w2stats.log
fi
