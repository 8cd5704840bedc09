# Round 4, box E: first-sort probe, counter pair shape, A/B new vs base, then
# the full -m gpu suite on the candidate build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 ./exp/sort_first > gpurun_out/r04e_sortfirst.log 2>&1 || { cat gpurun_out/r04e_sortfirst.log; exit 1; }
cat gpurun_out/r04e_sortfirst.log
CMSBWT_COUNTER_STATS=2 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check > gpurun_out/r04e_shape.log 2>&1 || { tail -20 gpurun_out/r04e_shape.log; exit 1; }
grep "counter" gpurun_out/r04e_shape.log
bash tools/gpu_ab_suite.sh r04e new base prio claim nhr1k
