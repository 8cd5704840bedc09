# walk step statistics (CMSBWT_W2_STATS=1) on the default workload
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_W2_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/b_st.log 2> gpurun_out/w2stats.log || { tail -20 gpurun_out/b_st.log gpurun_out/w2stats.log; exit 1; }
grep w2stats gpurun_out/w2stats.log
CMSBWT_COUNTER_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/b_st2.log 2> gpurun_out/cstats.log || true
grep counter gpurun_out/cstats.log | head -3
