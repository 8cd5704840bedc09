# e2e overlap A/B, counter variant A/B, then the 2-rank bench rehearsal (one gpurun call)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/e2e_ab.py 5 > gpurun_out/e2e_ab.txt 2>&1 || { tail -5 gpurun_out/e2e_ab.txt; exit 1; }
tail -2 gpurun_out/e2e_ab.txt
VARIANTS="${VARIANTS:-nop8 cvalu}" STEPS=10 bash tools/gpu_ab_walk.sh
bash tools/gpu_r03_bench2.sh
