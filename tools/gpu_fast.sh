# Parity subset + default bench (through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${TESTSEL:-small_cases or config1 or config2 or chunk_restarts or large_reference or sharded_small}" > gpurun_out/t_fast.log 2>&1 || { tail -40 gpurun_out/t_fast.log; exit 1; }
tail -1 gpurun_out/t_fast.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['stages_ms'])"
rm -rf gpurun_out/kt; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/kt.log 2>&1
python3 tools/kstats.py gpurun_out/kt/kt_kernel_stats.csv > gpurun_out/kt_summary.txt && head -24 gpurun_out/kt_summary.txt
