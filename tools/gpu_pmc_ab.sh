# PMC A/B of library builds on one box (through gpurun from the repo root):
#   bash tools/gpu_pmc_ab.sh <regex> new <name> ...   (exp/<name>/libcmsbwt.so)
# one bench step per pass, L2/fabric counters then SQ counters of the kernels
# matching <regex>; tools/pmc_walk.py prints the largest dispatch's values.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rx=$1; shift
lib() { case $1 in new) echo cms-bwt_amd/build/libcmsbwt.so;; *) echo exp/$1/libcmsbwt.so;; esac; }
B1="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check"
for v in "$@"; do
  i=0
  for grp in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES"; do
    i=$((i+1))
    rm -rf gpurun_out/pa_$v$i
    CMSBWT_LIB=$(lib $v) timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "$rx" -d gpurun_out/pa_$v$i -o p --output-format csv -- $B1 > gpurun_out/pa_$v$i.log 2>&1 || { echo "$v pass $i failed"; tail -5 gpurun_out/pa_$v$i.log; exit 1; }
    python3 tools/pmc_walk.py gpurun_out/pa_$v$i $v
  done
done
