// synth.hip — SURVEY.md §8(d) workload generated straight into HBM.
// Byte-identical to tools/gen_synth (same counter-based hash, synth.h).
#include <hip/hip_runtime.h>
#include "kernels.h"
#include "synth.h"

namespace cmsbwt {

// copy c (1-based: copy_begin + d) is written at base + d*(L+1), followed by
// the 0x02 separator.  One thread per 8 output bytes.
__global__ void k_synth(uint8_t* __restrict__ text, uint64_t L, uint64_t seed, uint64_t copy_begin,
                        uint64_t ncopies, uint64_t pthr, uint64_t base) {
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t total = ncopies * (L + 1);
  uint64_t o = g * 8;
  for (int k = 0; k < 8 && o + k < total; k++) {
    uint64_t e = o + k;
    uint64_t d = e / (L + 1), q = e % (L + 1);
    uint8_t ch;
    if (q == L) ch = 2;
    else ch = (uint8_t)synth_acgt(synth_copy_code(seed, copy_begin + d, q, pthr));
    text[base + e] = ch;
  }
}

void launch_synth_collection(uint8_t* text, uint64_t L, uint64_t seed, uint64_t copy_begin, uint64_t ncopies,
                             uint64_t pthr, uint64_t base, hipStream_t st) {
  uint64_t total = ncopies * (L + 1);
  uint64_t threads = (total + 7) / 8;
  if (!threads) return;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, text, L, seed,
                     copy_begin, ncopies, pthr, base);
}

}  // namespace cmsbwt
