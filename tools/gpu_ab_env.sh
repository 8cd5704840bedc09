# A/B of one build under environment settings (through gpurun from the repo
# root): bash tools/gpu_ab_env.sh "" "CMSBWT_X=1" ...  ("" = defaults); each
# setting runs the default bench twice, interleaved, with the parity check.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  k=0
  for e in "$@"; do
    k=$((k+1))
    env $e timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > gpurun_out/abe_$k.log 2>&1
    rc=$?
    if [ $rc = 1 ]; then echo "[$e] FAILED: $(tail -1 gpurun_out/abe_$k.log)"; continue; fi
    [ $rc = 0 ] || { tail -30 gpurun_out/abe_$k.log; exit 1; }
    echo "[$e] $(tail -1 gpurun_out/abe_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages_ms"]; print("step", d["ms_per_step"], "walk stage", s["ms_walk"], "walk", s["ms_walk_kernel"], "counter", s["counter_kernel"], "merge", s["merge"], d["parity"]["verdict"])')"
  done
done
