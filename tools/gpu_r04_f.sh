# Round 4, box F: which walk change breaks raw_reference_with_N (bisect by
# variant builds), then the SA first-sort timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
lib() { case $1 in new) echo cms-bwt_amd/build/libcmsbwt.so;; *) echo exp/$1/libcmsbwt.so;; esac; }
for v in new nomemo skip norefill; do
  CMSBWT_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "small_cases" --timeout 120 --timeout-method thread > gpurun_out/r04f_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/r04f_$v.log)"
  grep -E "^FAILED" gpurun_out/r04f_$v.log | head -8
  [ $rc -le 1 ] || exit 1
done
W=/tmp/r04e2e; mkdir -p $W
timeout -k 10 120 cms-bwt_amd/build/gen_synth 10000000 20 0.001 4 $W/w > /dev/null || { echo gen failed; exit 1; }
for ov in 1 0; do
  CMSBWT_TIMING=1 CMSBWT_OVERLAP_UPLOAD=$ov timeout -k 10 120 cms-bwt_amd/build/cmsbwt -r -v -o $W/o $W/w.list > $W/cli.out 2> gpurun_out/r04f_e2e_ov$ov.err || { echo cli failed; tail -5 gpurun_out/r04f_e2e_ov$ov.err; exit 1; }
  echo "e2e overlap=$ov"; grep "\[index\]" gpurun_out/r04f_e2e_ov$ov.err | head -8
done
rm -rf $W
