set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_DBL_STATS=1 CMSBWT_COUNTER_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/b_st3.log 2> gpurun_out/dstats.log || { tail gpurun_out/dstats.log; exit 1; }
grep -E "dbl|counter" gpurun_out/dstats.log | head -40
