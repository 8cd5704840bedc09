# Sharded-merge attribution: in-process group at --gpus 2 (one GPU) and the
# torch.distributed path at W = 1 (CMSBWT_DIST=sharded1), sub-stage host
# timing with allocator misses (CMSBWT_DM_TIMING=1), against the one-GPU step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_BENCH_REHEARSAL=1 CMSBWT_MULTI_TIMING=1 CMSBWT_DM_TIMING=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/dm_g2.log 2> gpurun_out/dm_g2.err || { tail -20 gpurun_out/dm_g2.err; exit 1; }
tail -1 gpurun_out/dm_g2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("gpus2", d["ms_per_step"], d["stages_ms"]["merge"], d["parity"]["verdict"])'
grep timing gpurun_out/dm_g2.err | tail -6
CMSBWT_DIST=sharded1 CMSBWT_DM_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/dm_s1.log 2> gpurun_out/dm_s1.err || { tail -20 gpurun_out/dm_s1.err; exit 1; }
tail -1 gpurun_out/dm_s1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("sharded1", d["ms_per_step"], d["stages_ms"]["merge"], d["parity"]["verdict"])'
grep timing gpurun_out/dm_s1.err | tail -3
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > gpurun_out/dm_1.log 2>&1 || exit 1
tail -1 gpurun_out/dm_1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("one-gpu", d["ms_per_step"], d["stages_ms"]["merge"])'
