set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
W=/tmp/e2e; mkdir -p $W
timeout -k 10 300 oracle/_build/gen_synth 100000000 20 0.01 5 $W/c5 > /dev/null
for rep in 1 2; do
    t0=$(date +%s.%N)
    timeout -k 10 300 cms-bwt_amd/build/cmsbwt -v -o $W/c5_out $W/c5.list > /dev/null 2> gpurun_out/c5e.err
    t1=$(date +%s.%N)
    echo "c5-shape 100MB x 20 @1% plain rep $rep: wall $(python3 -c "print(round($t1 - $t0, 3))") s; $(tail -1 gpurun_out/c5e.err); out $(stat -c %s $W/c5_out.bwt) B"
done
sha256sum $W/c5_out.bwt | cut -c1-16
rm -f $W/c5*
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "config2 or config3 or config5 or repeated" > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
