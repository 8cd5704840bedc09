# Round 4, box G: bisect the alignment-memo failure (use / record modes);
# SA sort timing on a second index build in the same process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in m1 m2 m4 m8; do
  CMSBWT_LIB=exp/$v/libcmsbwt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "small_cases" --timeout 120 --timeout-method thread > gpurun_out/r04g_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/r04g_$v.log)"
  [ $rc -le 1 ] || exit 1
done
CMSBWT_TIMING=1 timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0, 'cms-bwt_amd'); sys.path.insert(0, '.')
import cmsbwt, bench
ref = bench.synth_reference(10_000_000, 4)
e = cmsbwt.Engine(0)
for k in range(3):
    e.load_reference_bytes(ref)
    print('build', k, 'index', round(e.stats().t_index_s, 3), flush=True)
" > gpurun_out/r04g_sa.log 2>&1 || { tail -20 gpurun_out/r04g_sa.log; exit 1; }
grep -E "sort|build|first" gpurun_out/r04g_sa.log
