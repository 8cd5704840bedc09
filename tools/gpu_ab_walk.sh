# A/B of builds (libraries under cms-bwt_amd/build/var, VARIANTS) against the default library "base";
# PMCV: variants whose walk L2 counters are collected; TSTATS=1: counter wave-record statistics
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in base ${VARIANTS}; do
  if [ "$v" = base ]; then unset CMSBWT_LIB; else export CMSBWT_LIB=$GRAFT_REPO_ROOT/cms-bwt_amd/build/var/libcmsbwt_$v.so; fi
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "bench_workload_full or (walk_table_paths and (copies or identical)) or chunk_restarts or config2" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_t_$v.log 2>&1 || { echo "variant $v FAILED"; tail -20 gpurun_out/ab_t_$v.log; exit 1; }
  echo "variant $v tests: $(tail -1 gpurun_out/ab_t_$v.log)"
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu --no-e2e > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('variant $v', d['ms_per_step'], d['stages_ms'])"
  if [[ " $PMCV " == *" $v "* ]]; then
    rm -rf gpurun_out/abp_$v; timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d gpurun_out/abp_$v -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e > gpurun_out/abp_$v.log 2>&1
    python3 tools/pmc_walk.py gpurun_out/abp_$v $v
  fi
done
unset CMSBWT_LIB
if [ -n "$TSTATS" ]; then
  CMSBWT_LIB=$GRAFT_REPO_ROOT/cms-bwt_amd/build/var/libcmsbwt_ts.so CMSBWT_COUNTER_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-e2e > gpurun_out/ab_ts.log 2>&1 || { tail -5 gpurun_out/ab_ts.log; exit 1; }
  grep "\[counter\]" gpurun_out/ab_ts.log | tail -2
fi
