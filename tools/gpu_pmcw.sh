# PMC passes for the walk kernel only (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcw; rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "ms_walk2" -d $OUT/p$i -o p$i --output-format csv -- $B > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
python3 -c "
import json; d=json.load(open('$OUT/pmc_summary.json'))
for k in d: print(k, {c: '%.4g'%v['per_launch'] for c,v in d[k].items()})"
