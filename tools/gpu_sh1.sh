# sharded merge at world 1 on the headline workload: golden test + timing vs the single-GPU merge
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k config3 > gpurun_out/t_sh3.log 2>&1 || { tail -60 gpurun_out/t_sh3.log; exit 1; }
tail -2 gpurun_out/t_sh3.log
CMSBWT_DIST=sharded1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b_sh1.log 2>&1 || { tail -20 gpurun_out/b_sh1.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/b_sh1.log').read().strip().splitlines()[-1]); print('sharded1', d['ms_per_step'], d['config']['runs'])"
rm -rf gpurun_out/kt1; CMSBWT_DIST=sharded1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt1 -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/kt1.log 2>&1
python3 tools/kstats.py gpurun_out/kt1/kt_kernel_stats.csv > gpurun_out/kt1_summary.txt && head -40 gpurun_out/kt1_summary.txt
