# Sharded merge at W=1 on the headline workload: bench + kernel stats (through gpurun)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_DIST=sharded1 timeout -k 10 300 python bench.py --no-cpu --no-e2e > gpurun_out/bench_s1.log 2>&1 || { tail -20 gpurun_out/bench_s1.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_s1.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['stages_ms'])"
rm -rf gpurun_out/ks1; CMSBWT_DIST=sharded1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks1 -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-e2e > gpurun_out/ks1.log 2>&1
python3 tools/kstats.py gpurun_out/ks1/kt_kernel_stats.csv > gpurun_out/ks1_summary.txt && head -40 gpurun_out/ks1_summary.txt
