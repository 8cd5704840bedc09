# Counter kernel split (staging only / no searches / full) and PMC passes (through gpurun)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/cp; rm -rf $OUT; mkdir -p $OUT
for dbg in 0 2 4; do
  CMSBWT_TGT_DEBUG=$dbg timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 > $OUT/b$dbg.log 2>&1 || true
  python3 -c "import json;d=json.loads(open('$OUT/b$dbg.log').read().strip().splitlines()[-1]);print('dbg $dbg', d['stages_ms'])" || tail -3 $OUT/b$dbg.log
done
B1="python3 bench.py --steps 1 --warmup 0 --no-cpu"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "counter_tgt" -d $OUT/p$i -o p$i --output-format csv -- $B1 > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.json || true
python3 tools/pmc_main.py $OUT > $OUT/pmc_main.json || true
cat $OUT/pmc_main.json | head -60
