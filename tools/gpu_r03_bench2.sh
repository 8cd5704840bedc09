# Rehearsal of the driver's N>1 bench command on a one-GPU box: two ranks on
# device 0 over gloo (CMSBWT_BENCH_SAME_GPU=1), the full config-4 workload
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_BENCH_SAME_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2.log 2>&1 || { tail -30 gpurun_out/bench_n2.log; exit 1; }
tail -1 gpurun_out/bench_n2.log | cut -c1-700
