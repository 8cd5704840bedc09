# PMC passes of the walk kernel only (run through gpurun from the repo root);
# one counter group per rocprofv3 run, no traces combined with --pmc.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcw2; rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_IFETCH" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-ms_walk2}" -d $OUT/p$i -o p$i --output-format csv -- $B > $OUT/p$i.log 2>&1 || echo "pass $i failed: $grp"
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/pmcw2/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        rows[(r["Dispatch_Id"], r["Kernel_Name"][:40])][r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in rows.items():
    print(k, {c: f"{x:.4g}" for c, x in v.items()})
PY
