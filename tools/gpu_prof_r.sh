# Round profile (run through gpurun from the repo root): kernel trace stats of
# the default bench and PMC passes (one counter group per rocprofv3 run, no
# traces combined with --pmc) for the walk and counter kernels.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof; rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B > $OUT/kt.log 2>&1
python3 tools/kstats.py $OUT/kt/kt_kernel_stats.csv > $OUT/kt_summary.txt
python3 tools/launches.py $OUT/kt/kt_kernel_trace.csv > $OUT/launches.txt
B1="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "ms_walk2|counter_tgt" -d $OUT/p$i -o p$i --output-format csv -- $B1 > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
head -30 $OUT/kt_summary.txt
