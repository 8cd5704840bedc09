# Round 4, box B: the CLI's multi-GPU path (-n); walk A/B (cooperative slot
# refill vs fixed groups of four) with the bench's full-size parity check;
# config-5 walk sizing; config 4 through bench.py's N>1 path at W=2/4/8.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cli_multi.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r04_cli_multi.log 2>&1 || { tail -60 gpurun_out/r04_cli_multi.log; exit 1; }
tail -1 gpurun_out/r04_cli_multi.log
B="python -u bench.py --steps 10 --warmup 2 --no-cpu --no-e2e"
for v in new old new old; do
  if [ $v = old ]; then L=exp/norefill/libcmsbwt.so; else L=cms-bwt_amd/build/libcmsbwt.so; fi
  CMSBWT_LIB=$L timeout -k 10 240 $B > gpurun_out/r04_ab_$v.log 2>&1 || { tail -30 gpurun_out/r04_ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r04_ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stages_ms"], d["parity"]["verdict"])')"
done
for v in new old; do
  if [ $v = old ]; then L=exp/norefill/libcmsbwt.so; else L=cms-bwt_amd/build/libcmsbwt.so; fi
  CMSBWT_W2_STATS=1 CMSBWT_LIB=$L timeout -k 10 240 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > gpurun_out/r04_stats_$v.log 2>&1 || { tail -30 gpurun_out/r04_stats_$v.log; exit 1; }
  grep -E "coop_steps|wave_steps" gpurun_out/r04_stats_$v.log | tail -2
done
timeout -k 10 300 python -u tools/c5_size.py > gpurun_out/r04_c5.log 2>&1 || { tail -30 gpurun_out/r04_c5.log; exit 1; }
tail -2 gpurun_out/r04_c5.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py -x -v -s --timeout 580 --timeout-method thread > gpurun_out/r04_c4.log 2>&1 || { tail -40 gpurun_out/r04_c4.log; exit 1; }
grep -E "passed|failed|world" gpurun_out/r04_c4.log | cut -c1-600
