set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=/tmp/e2e; mkdir -p $W
timeout -k 10 300 oracle/_build/gen_synth 100000000 2 0.01 5 $W/c5 > /dev/null
CMSBWT_TIMING=1 timeout -k 10 300 cms-bwt_amd/build/cmsbwt -v -o $W/c5_out $W/c5.list > /dev/null 2> gpurun_out/idx.err || true
cat gpurun_out/idx.err
