# A/B of library builds on one box (run through gpurun from the repo root):
#   make lib OUT=exp/<name> XFLAGS="-D..."   (CPU side, once per variant)
#   gpurun -- 'bash tools/gpu_ab.sh new <name> ...'
# "new" is cms-bwt_amd/build; each variant runs the default bench twice,
# interleaved, with the full-size parity check.  A variant whose bench raises
# (Python exit 1) is reported and skipped; anything else stops the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
lib() { case $1 in new) echo cms-bwt_amd/build/libcmsbwt.so;; *) echo exp/$1/libcmsbwt.so;; esac; }
for rep in 1 2; do
  for v in "$@"; do
    CMSBWT_LIB=$(lib $v) timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > gpurun_out/ab_$v.log 2>&1
    rc=$?
    if [ $rc = 1 ]; then echo "$v FAILED: $(tail -1 gpurun_out/ab_$v.log)"; continue; fi
    [ $rc = 0 ] || { tail -30 gpurun_out/ab_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stages_ms"]; print("step", d["ms_per_step"], "walk", s["ms_walk_kernel"], "counter", s["counter_kernel"], "merge", s["merge"], d["parity"]["verdict"])')"
  done
done
