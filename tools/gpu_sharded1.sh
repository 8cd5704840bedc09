# Sharded merge path at N=1 (CMSBWT_DIST=sharded1) vs the one-GPU merge, through gpurun
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_DIST=sharded1 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_sh1.log 2>&1 || { tail -20 gpurun_out/bench_sh1.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_sh1.log').read().strip().splitlines()[-1]);print('sharded1',d['ms_per_step'],d['stages_ms'])"
rm -rf gpurun_out/kt3; CMSBWT_DIST=sharded1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt3 -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/kt3.log 2>&1
python3 tools/ktrace.py gpurun_out/kt3/kt_kernel_trace.csv > gpurun_out/trace_sh1.txt
tail -1 gpurun_out/trace_sh1.txt
