# FETCH_SIZE / WRITE_SIZE of every kernel of one bench step (run through
# gpurun from the repo root); one rocprofv3 run per counter, no traces.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmca; rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/p1 -o p1 --output-format csv -- $B > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/p2 -o p2 --output-format csv -- $B > $OUT/p2.log 2>&1
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
echo done
