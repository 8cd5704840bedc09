# time experiment builds under exp/*/ (run through gpurun from the repo root)
set -e
export TMPDIR=/tmp
for lib in cms-bwt_amd/build exp/*; do
  echo "== $lib"
  CMSBWT_LIB=$PWD/$lib/libcmsbwt.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; continue; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms'])"
done
