# Whole -m gpu suite on one box, then the sharded-merge timing of the
# in-process group (--gpus 2) and the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -5 gpurun_out/suite.log
[ $rc -le 1 ] || exit 1
CMSBWT_BENCH_REHEARSAL=1 CMSBWT_MULTI_TIMING=1 CMSBWT_DM_TIMING=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/mt_g2.log 2> gpurun_out/mt_g2.err || { tail -20 gpurun_out/mt_g2.err; exit 1; }
grep timing gpurun_out/mt_g2.err | tail -6
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], d["roofline"]["frac"], d["stages_ms"], d["parity"]["verdict"], d.get("e2e",{}).get("wall_median_s"), d["cpu_baseline"].get("value"))'
