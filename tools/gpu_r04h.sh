# Round 4, box H: attribution of k_counter_tgt's LDS bank conflicts and time to
# its phases (attribution builds exp/ph1: staging only, exp/ph2: + record
# walks and re-tests; new: + binary searches).  Counters of the ph builds are
# wrong by construction (--no-check).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/attr; rm -rf $OUT; mkdir -p $OUT
lib() { case $1 in new) echo cms-bwt_amd/build/libcmsbwt.so;; *) echo exp/$1/libcmsbwt.so;; esac; }
for v in new ph1 ph2; do
  mkdir -p $OUT/$v
  CMSBWT_LIB=$(lib $v) timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --no-check > $OUT/$v/bench.log 2>&1 || { tail -20 $OUT/$v/bench.log; exit 1; }
  echo "$v $(tail -1 $OUT/$v/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("counter", d["stages_ms"]["counter_kernel"], "step", d["ms_per_step"])')"
  CMSBWT_LIB=$(lib $v) timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS --kernel-include-regex "counter_tgt" -d $OUT/$v/p1 -o p1 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > $OUT/$v/p1.log 2>&1 || { tail -20 $OUT/$v/p1.log; exit 1; }
  python3 tools/pmc_main.py $OUT/$v > $OUT/$v/pmc.json
  python3 -c "import json; d=json.load(open('$OUT/$v/pmc.json'))['k_counter_tgt']; print('$v', {k: d[k] for k in d if not k.startswith('_')})"
done
