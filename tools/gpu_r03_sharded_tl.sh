# Sharded merge at W=1 on the headline workload: bench line and a one-step kernel timeline (through gpurun)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_DIST=sharded1 timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 10 --warmup 3 > gpurun_out/bench_s1.log 2>&1 || { tail -20 gpurun_out/bench_s1.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_s1.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['stages_ms'])"
rm -rf gpurun_out/kts1; CMSBWT_DIST=sharded1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kts1 -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-e2e > gpurun_out/kts1.log 2>&1
python3 tools/ktrace.py gpurun_out/kts1/kt_kernel_trace.csv > gpurun_out/trace_s1.txt
tail -3 gpurun_out/trace_s1.txt
