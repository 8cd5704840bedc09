set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_COUNTER_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/b_st2.log 2> gpurun_out/cstats.log || { tail gpurun_out/cstats.log; exit 1; }
grep counter gpurun_out/cstats.log | head -3
