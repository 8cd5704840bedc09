# Where the in-process multi-rank merge spends its time:
# the group bench at N = 1, 2, 4 on one GPU with per-stage host timing of
# the sharded merge (CMSBWT_MULTI_TIMING=1), plus cmsbwt -n 2 on config 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 2; do
  CMSBWT_BENCH_REHEARSAL=1 CMSBWT_MULTI_TIMING=1 CMSBWT_DM_TIMING=1 timeout -k 10 300 python -u bench.py --gpus $n --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/mt_g$n.log 2> gpurun_out/mt_g$n.err || { tail -20 gpurun_out/mt_g$n.err; exit 1; }
  echo "gpus $n: $(tail -1 gpurun_out/mt_g$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step", d["ms_per_step"], d["stages_ms"], d["parity"]["verdict"])')"
  grep timing gpurun_out/mt_g$n.err | tail -12
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/mt_g1.log 2>&1 || exit 1
echo "gpus 1: $(tail -1 gpurun_out/mt_g1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step", d["ms_per_step"], d["stages_ms"])')"
