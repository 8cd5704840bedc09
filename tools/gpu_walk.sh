# walk-kernel experiments (run through gpurun from the repo root)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmcw; rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "ms_walk2|counter_win" -d $OUT/p$i -o p$i --output-format csv -- $B > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
for cfg in "CMSBWT_WALK_LANES=131072" "CMSBWT_WALK_LANES=262144" "CMSBWT_WALK_LANES=1048576"; do
    echo "== $cfg"
    env $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b.log 2>&1 || { cat gpurun_out/b.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'])"
done
