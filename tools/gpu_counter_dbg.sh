set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for d in 0 2 4 6; do
CMSBWT_TGT_DEBUG=$d timeout -k 10 300 python bench.py --no-cpu --steps 2 > gpurun_out/bench_d$d.log 2>&1 || { tail -5 gpurun_out/bench_d$d.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_d$d.log').read().strip().splitlines()[-1]);print('dbg $d', d['stages_ms']['counter_kernel'])"
done
