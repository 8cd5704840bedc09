# Parity subset + bench (run through gpurun from the repo root)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTSEL:-small or config1 or config2 or window or counter}" > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
