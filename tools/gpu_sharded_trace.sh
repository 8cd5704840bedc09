# Kernel trace of the sharded merge at one rank's head share of W = 8 (125
# copies, CMSBWT_DIST=sharded1, all n positions owned): which kernels the
# per-rank fixed cost is made of (through gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/shtr; rm -rf $OUT; mkdir -p $OUT
CMSBWT_DIST=sharded1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --copies 125 --steps 3 --warmup 1 --no-cpu --no-e2e --no-check > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
python3 tools/kstats.py $OUT/kt/kt_kernel_stats.csv > $OUT/kt_summary.txt
head -45 $OUT/kt_summary.txt
