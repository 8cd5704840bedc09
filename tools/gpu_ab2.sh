# A/B of env settings on the default bench + timeline of the default build
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "X=1" "CMSBWT_GROUP_SORT=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['stages_ms'])"
done
rm -rf gpurun_out/kt2; timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt2 -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/kt2.log 2>&1
python3 tools/ktrace.py gpurun_out/kt2/kt_kernel_trace.csv > gpurun_out/trace.txt
