# Alignment-memo reproducer on one box: the walk's head
# records of every small case, generic and default instance, for each build.
#   make lib OUT=exp/mg  XFLAGS="-DCMSBWT_MEMO_GENERIC=1"
#   make lib OUT=exp/mgc XFLAGS="-DCMSBWT_MEMO_GENERIC=1 -DCMSBWT_MEMO_CHECK=1"
#   make lib OUT=exp/mfc XFLAGS="-DCMSBWT_MEMO_CHECK=1"
#   gpurun -- 'bash tools/gpu_memo.sh new mg mgc mfc'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
lib() { case $1 in new) echo cms-bwt_amd/build/libcmsbwt.so;; *) echo exp/$1/libcmsbwt.so;; esac; }
for v in "$@"; do
  CMSBWT_LIB=$(lib $v) timeout -k 10 ${MEMO_TIMEOUT:-300} python -u tools/memo_repro.py $MEMO_CASES > gpurun_out/memo_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"; grep -E "DIFF|\[memo\]|ALL OK|SOME|Error|error" gpurun_out/memo_$v.log | head -30
  [ $rc -le 1 ] || exit 1
done
