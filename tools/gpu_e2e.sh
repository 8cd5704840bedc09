# End-to-end CLI timing (run through gpurun from the repo root): the cmsbwt
# process from start to .rl_bwt closed, on FASTA files written by the
# deterministic generator (SURVEY.md §8d metric 1, file-inclusive).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
df -h /tmp | tail -1
W=${E2E_DIR:-/tmp/e2e}
mkdir -p $W
IFS=';' read -ra CFGS <<< "${E2E_CONFIGS:-10000000 100 0.001 3 c2;10000000 1000 0.001 4 c3}"
for cfg in "${CFGS[@]}"; do
    set -- $cfg
    avail=$(df --output=avail -B1 /tmp | tail -1)
    need=$(( $1 * $2 * 13 / 10 ))
    if [ "$avail" -lt "$need" ]; then echo "skip $5: /tmp has $avail B, needs $need"; continue; fi
    t0=$(date +%s.%N)
    timeout -k 10 300 oracle/_build/gen_synth $1 $2 $3 $4 $W/$5 > /dev/null
    t1=$(date +%s.%N)
    echo "$5: generated $(stat -c %s $W/$5.coll.fa) B in $(python3 -c "print(round($t1 - $t0, 2))") s"
    sync
    for rep in 1 2 3; do
        [ $rep = 3 ] && export CMSBWT_HOST_READER=1
        t0=$(date +%s.%N)
        timeout -k 10 300 cms-bwt_amd/build/cmsbwt -r -v -o $W/$5_out $W/$5.list > gpurun_out/e2e_$5.out 2> gpurun_out/e2e_$5.err
        t1=$(date +%s.%N)
        echo "$5 rep $rep: wall $(python3 -c "print(round($t1 - $t0, 3))") s; $(tail -1 gpurun_out/e2e_$5.err); out $(stat -c %s $W/$5_out.rl_bwt) B"
    done
    unset CMSBWT_HOST_READER
    sha256sum $W/$5_out.rl_bwt | cut -c1-16
    rm -f $W/$5*
done
