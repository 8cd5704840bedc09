# Reader/writer thread and chunk sweep on the 10 GB file, plus config-5-shape e2e (plain .bwt)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
W=/tmp/e2e; mkdir -p $W
timeout -k 10 300 oracle/_build/gen_synth 10000000 1000 0.001 4 $W/c3 > /dev/null
for cfg in "8 32" "16 32" "16 16" "32 16" "16 64"; do
    set -- $cfg
    for rep in 1 2; do
        CMSBWT_READ_THREADS=$1 CMSBWT_WRITE_THREADS=$1 CMSBWT_READ_CHUNK_MB=$2 timeout -k 10 300 cms-bwt_amd/build/cmsbwt -r -v -o $W/c3_out $W/c3.list > /dev/null 2> gpurun_out/sw.err
        echo "threads $1 chunk $2 rep $rep: $(tail -1 gpurun_out/sw.err)"
    done
done
rm -f $W/c3*
timeout -k 10 300 oracle/_build/gen_synth 100000000 20 0.01 5 $W/c5 > /dev/null
for rep in 1 2; do
    t0=$(date +%s.%N)
    timeout -k 10 300 cms-bwt_amd/build/cmsbwt -v -o $W/c5_out $W/c5.list > /dev/null 2> gpurun_out/c5e.err
    t1=$(date +%s.%N)
    echo "c5-shape 100MB x 20 @1% plain rep $rep: wall $(python3 -c "print(round($t1 - $t0, 3))") s; $(tail -1 gpurun_out/c5e.err); out $(stat -c %s $W/c5_out.bwt) B"
done
rm -f $W/c5*
