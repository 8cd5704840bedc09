# Round 4, box D: walk / counter A/B
# (refill + no-skip vs refill vs base) with the full-size parity check; step
# counts; L2 request counters of the walk per variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
true

lib() { case $1 in new) echo cms-bwt_amd/build/libcmsbwt.so;; *) echo exp/$1/libcmsbwt.so;; esac; }
for v in new memo tnt cbase refill base new memo tnt cbase refill base; do
  CMSBWT_LIB=$(lib $v) timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > gpurun_out/r04c_ab_$v.log 2>&1
  rc=$?
  if [ $rc = 1 ]; then echo "$v FAILED: $(tail -1 gpurun_out/r04c_ab_$v.log)"; continue; fi
  [ $rc = 0 ] || { tail -30 gpurun_out/r04c_ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r04c_ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages_ms"]; print(d["ms_per_step"], s["ms_walk"], s["ms_walk_kernel"], s["counter_kernel"], d["parity"]["verdict"])')"
done
CMSBWT_W2_STATS=1 timeout -k 10 240 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > gpurun_out/r04c_stats_new.log 2>&1 || { tail -30 gpurun_out/r04c_stats_new.log; exit 1; }
grep -E "w2stats" gpurun_out/r04c_stats_new.log | tail -30
for v in new memo refill; do
  CMSBWT_LIB=$(lib $v) timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex ms_walk2 -d gpurun_out/r04c_pmc_$v -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > gpurun_out/r04c_pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/r04c_pmc_$v.log; exit 1; }
  python3 tools/pmc_walk.py gpurun_out/r04c_pmc_$v $v
done
# end to end (Metric 1) stage breakdown of the CLI on the bench workload's FASTA
W=/tmp/r04e2e; mkdir -p $W
timeout -k 10 120 cms-bwt_amd/build/gen_synth 10000000 1000 0.001 4 $W/w > /dev/null || { echo gen failed; exit 1; }
for run in a b; do
  for ov in 1 0; do
    CMSBWT_TIMING=1 CMSBWT_OVERLAP_UPLOAD=$ov timeout -k 10 120 cms-bwt_amd/build/cmsbwt -r -v -o $W/o $W/w.list > $W/cli.out 2> gpurun_out/r04_e2e_${run}_ov$ov.err || { echo cli failed; tail -5 gpurun_out/r04_e2e_${run}_ov$ov.err; exit 1; }
    echo "e2e $run overlap=$ov: $(tail -1 $W/cli.out) | $(grep -E 'first launch|\] sa ' gpurun_out/r04_e2e_${run}_ov$ov.err | tr '\n' ' ') | $(tail -1 gpurun_out/r04_e2e_${run}_ov$ov.err)"
  done
done
sha256sum $W/o.rl_bwt | cut -c1-16
for n in 2 4; do
  timeout -k 10 180 cms-bwt_amd/build/cmsbwt -r -v -n $n -o $W/o$n $W/w.list > $W/cli$n.out 2> gpurun_out/r04_e2e_n$n.err || { echo cli -n $n failed; tail -5 gpurun_out/r04_e2e_n$n.err; exit 1; }
  echo "e2e -n $n: $(tail -1 $W/cli$n.out) | $(tail -1 gpurun_out/r04_e2e_n$n.err) | $(sha256sum $W/o$n.rl_bwt | cut -c1-16)"
done
rm -rf $W
