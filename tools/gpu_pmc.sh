# PMC passes over the default bench (run through gpurun from the repo root);
# each counter group in its own rocprofv3 run (no traces combined with --pmc)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B > $OUT/kt.log 2>&1
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "WRITE_SIZE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- $B > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
ls -R $OUT | head -50
