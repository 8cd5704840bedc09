# std::map replay tests first, then the round check (full GPU suite, bench, kernel stats) and PMC passes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu -k "ambiguity or forced_map_replay" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_replay.log 2>&1 || { grep -E "Error|error|assert" gpurun_out/t_replay.log | head -30; tail -30 gpurun_out/t_replay.log; exit 1; }
tail -2 gpurun_out/t_replay.log
bash tools/gpu_round.sh
bash tools/gpu_prof_r.sh > gpurun_out/prof_r.log 2>&1
python3 tools/pmc_main.py gpurun_out/prof > gpurun_out/prof/pmc_main.json
