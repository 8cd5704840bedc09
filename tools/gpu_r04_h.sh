# Round 4, box H: the alignment memo's claims checked against the bytes (debug build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CMSBWT_LIB=exp/verify/libcmsbwt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "small_cases_rle and raw_reference" --timeout 120 --timeout-method thread > gpurun_out/r04h.log 2>&1
echo "rc=$?"; grep -c "memo bad" gpurun_out/r04h.log; grep "memo bad" gpurun_out/r04h.log | head -20; tail -2 gpurun_out/r04h.log
