# Builds a library variant whose walk kernel (ms_walk2.hip) is compiled in two
# separate halves, so that the optimiser and the code generator can be judged
# apart:
#   1. clang -cc1 -O3 -emit-llvm: the optimised IR, exactly what -O3 hands to
#      the backend (kept as exp/<name>/walk2.ll for inspection);
#   2. llc <llc options> on that IR: the machine code.
# Every other object comes from the normal build (make lib).
#   bash tools/memo_isa.sh <name> "<XFLAGS>" <llc options...>
# e.g. bash tools/memo_isa.sh l3 "-DCMSBWT_MEMO_GENERIC_BARRIER=0" -O3
#      bash tools/memo_isa.sh l1 "-DCMSBWT_MEMO_GENERIC_BARRIER=0" -O1
# CPU only (cross-compiles for gfx950); run the result with tools/gpu_memo.sh.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; xflags=$2; shift 2
OUT=$ROOT/exp/$name
mkdir -p "$OUT"
B=$ROOT/cms-bwt_amd/build
LLC=/opt/rocm/lib/llvm/bin/llc
# the device cc1 line's backend options (hipcc -###)
LLCF="-amdgpu-internalize-symbols -simplifycfg-sink-common=false"
cmds=$(cd "$ROOT/cms-bwt_amd/csrc" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall \
  -mllvm -simplifycfg-sink-common=false -DCMSBWT_W2_WAVES=4 $xflags -c -o "$OUT/ms_walk2.o" ms_walk2.hip -### 2>&1 | grep '^ "')
dev=$(echo "$cmds" | sed -n 1p)
devobj=$(echo "$dev" | grep -o '"-o" "[^"]*"' | sed 's/"-o" "\(.*\)"/\1/')
# step 1: the device compile, stopped after the IR pipeline
ir=$(echo "$dev" | sed 's/"-emit-obj"/"-emit-llvm"/' | sed "s#\"-o\" \"$devobj\"#\"-o\" \"$OUT/walk2.ll\"#")
(cd "$ROOT/cms-bwt_amd/csrc" && eval "$ir")
# step 2: the backend alone
"$LLC" -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 $LLCF "$@" -filetype=obj "$OUT/walk2.ll" -o "$devobj"
"$LLC" -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 $LLCF "$@" -filetype=asm "$OUT/walk2.ll" -o "$OUT/walk2.s"
# link, bundle, host compile: unchanged
(cd "$ROOT/cms-bwt_amd/csrc" && echo "$cmds" | sed -n '2,$p' | while read -r c; do eval "$c"; done)
objs=""
for o in engine multi dist_kernels ms_walk merge synth coll_read ref_index host_index host_reader; do objs="$objs $B/$o.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libcmsbwt.so" $objs "$OUT/ms_walk2.o"
echo "built $OUT/libcmsbwt.so (llc $*)"
