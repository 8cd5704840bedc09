# Round 4, box E: walk A/B of the alignment memo (with temporal text, without
# refill); step counts; FETCH/WRITE and L2 request PMC of the walk; SA round
# timing end to end; then the full -m gpu suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
lib() { case $1 in new) echo cms-bwt_amd/build/libcmsbwt.so;; *) echo exp/$1/libcmsbwt.so;; esac; }
for v in new memotnt memonoref new memotnt memonoref; do
  CMSBWT_LIB=$(lib $v) timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > gpurun_out/r04e_ab_$v.log 2>&1
  rc=$?
  if [ $rc = 1 ]; then echo "$v FAILED: $(tail -1 gpurun_out/r04e_ab_$v.log)"; continue; fi
  [ $rc = 0 ] || { tail -30 gpurun_out/r04e_ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r04e_ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages_ms"]; print(d["ms_per_step"], s["ms_walk"], s["ms_walk_kernel"], s["counter_kernel"], d["parity"]["verdict"])')"
done
CMSBWT_W2_STATS=1 timeout -k 10 240 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > gpurun_out/r04e_stats.log 2>&1 || { tail -30 gpurun_out/r04e_stats.log; exit 1; }
grep -E "w2stats" gpurun_out/r04e_stats.log | tr '\n' ' '; echo
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "ms_walk2|counter_tgt" -d gpurun_out/r04e_pmc/p$i -o p$i --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > gpurun_out/r04e_pmc_p$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/r04e_pmc_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/r04e_pmc > gpurun_out/r04e_pmc_summary.json && python3 tools/pmc_walk.py gpurun_out/r04e_pmc/p3 new
W=/tmp/r04e2e; mkdir -p $W
timeout -k 10 120 cms-bwt_amd/build/gen_synth 10000000 1000 0.001 4 $W/w > /dev/null || { echo gen failed; exit 1; }
for ov in 1 0; do
  CMSBWT_TIMING=1 CMSBWT_OVERLAP_UPLOAD=$ov timeout -k 10 120 cms-bwt_amd/build/cmsbwt -r -v -o $W/o $W/w.list > $W/cli.out 2> gpurun_out/r04e_e2e_ov$ov.err || { echo cli failed; tail -5 gpurun_out/r04e_e2e_ov$ov.err; exit 1; }
  echo "e2e overlap=$ov: $(tail -1 $W/cli.out)"; grep "\[index\]" gpurun_out/r04e_e2e_ov$ov.err | head -12; tail -1 gpurun_out/r04e_e2e_ov$ov.err
done
rm -rf $W
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04e_gpu_suite.log 2>&1 || { tail -40 gpurun_out/r04e_gpu_suite.log; exit 1; }
tail -2 gpurun_out/r04e_gpu_suite.log
