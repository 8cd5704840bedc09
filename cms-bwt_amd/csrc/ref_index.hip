// ref_index.hip — the reference index built on the GPU (SURVEY.md §8a row a1,
// §8f row 1): SA, ISA, Φ-PLCP, LCP, max-neighbour PLCP and BWT of the
// augmented reference x (FN:231-297).  libsais is absent from the image, and
// the reference's SA is unique (x ends in the unique smallest byte \0,
// FN:236-237), so any exact construction reproduces libsais' output.
//
// SA: prefix doubling.  Keys start as 7 symbols of 9 bits (byte + 1; 0 past
// the end, so the end of the string sorts first as in libsais), then each
// round sorts only the still-tied suffixes by (rank[i], rank[i+h] + 1) with
// rank = the SA slot of the suffix's group head; h doubles until every group
// is a singleton.  LCP: Kasai's Φ method over chunks of kIdxChunk positions
// per thread (PLCP[i+1] >= PLCP[i] - 1 inside a chunk; each chunk starts from
// zero, so the work is n + the sum of PLCP at chunk starts).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace cmsbwt {

static inline dim3 gidx(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

__global__ void k_ix_init(const uint8_t* __restrict__ x, uint32_t n, unsigned long long* __restrict__ key,
                          uint32_t* __restrict__ idx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long k = 0;
#pragma unroll
  for (uint32_t j = 0; j < kIdxH0; j++) {
    const uint32_t p = i + j;
    k = (k << 9) | (p < n ? (unsigned long long)x[p] + 1 : 0ull);
  }
  key[i] = k;
  idx[i] = i;
}

// over a sorted run of m keys at slots slot[u] (slot == nullptr: slot = u):
// head[u] = slot of u's group start (max-scan input), tie[u] = group size > 1
__global__ void k_ix_heads(const unsigned long long* __restrict__ key, const uint32_t* __restrict__ slot, uint32_t m,
                           uint32_t* __restrict__ headIn, uint32_t* __restrict__ tie) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= m) return;
  const unsigned long long k = key[u];
  const bool first = u == 0 || key[u - 1] != k;
  const bool last = u + 1 == m || key[u + 1] != k;
  headIn[u] = first ? (slot ? slot[u] : u) : 0u;
  tie[u] = (first && last) ? 0u : 1u;
}

// SA[slot[u]] = val[u]; rank[val[u]] = head[u]
__global__ void k_ix_place(const uint32_t* __restrict__ val, const uint32_t* __restrict__ slot,
                           const uint32_t* __restrict__ head, uint32_t m, int32_t* __restrict__ sa,
                           uint32_t* __restrict__ rank) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= m) return;
  const uint32_t i = val[u];
  sa[slot ? slot[u] : u] = (int32_t)i;
  rank[i] = head[u];
}

// doubling keys of the tied slots act[0..U)
__global__ void k_ix_keys(const uint32_t* __restrict__ act, uint32_t U, const int32_t* __restrict__ sa,
                          const uint32_t* __restrict__ rank, uint32_t n, uint32_t h,
                          unsigned long long* __restrict__ key, uint32_t* __restrict__ val) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const uint32_t i = (uint32_t)sa[act[u]];
  const uint64_t j = (uint64_t)i + h;
  key[u] = ((unsigned long long)rank[i] << 32) | (j < n ? (unsigned long long)rank[j] + 1 : 0ull);
  val[u] = i;
}

__global__ void k_ix_isa_phi(const int32_t* __restrict__ sa, uint32_t n, uint32_t* __restrict__ isa,
                             int32_t* __restrict__ phi) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int32_t s = sa[r];
  isa[s] = r;
  phi[s] = r ? sa[r - 1] : -1;
}

__global__ void k_ix_plcp(const uint8_t* __restrict__ x, uint32_t n, const int32_t* __restrict__ phi,
                          int32_t* __restrict__ plcp) {
  const uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kIdxChunk;
  if (i0 >= n) return;
  const uint64_t i1 = i0 + kIdxChunk < n ? i0 + kIdxChunk : n;
  uint64_t l = 0;
  for (uint64_t i = i0; i < i1; i++) {
    const int32_t j = phi[i];
    if (j < 0) { plcp[i] = 0; l = 0; continue; }
    while (i + l < n && (uint64_t)j + l < n && x[i + l] == x[j + l]) l++;
    plcp[i] = (int32_t)l;
    if (l > 0) l--;
  }
}

// LCP[r] = PLCP[SA[r]] (LCP[n] = -1), BWT[r] = x[SA[r]-1] (0 at SA = 0)
__global__ void k_ix_lcp_bwt(const uint8_t* __restrict__ x, const int32_t* __restrict__ sa, uint32_t n,
                             const int32_t* __restrict__ plcp, int32_t* __restrict__ lcp, uint8_t* __restrict__ bwt) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n) return;
  if (r == n) { lcp[n] = -1; return; }
  const int32_t s = sa[r];
  lcp[r] = plcp[s];
  bwt[r] = s > 0 ? x[s - 1] : 0;
}

// FN:272-274: PLCP[i] = max(LCP[ISA[i]], LCP[ISA[i]+1])
__global__ void k_ix_plcp_max(const uint32_t* __restrict__ isa, const int32_t* __restrict__ lcp, uint32_t n,
                              int32_t* __restrict__ plcp) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = isa[i];
  const int32_t a = lcp[r], b = lcp[r + 1];
  plcp[i] = a > b ? a : b;
}

void launch_ix_init(const uint8_t* x, uint32_t n, unsigned long long* key, uint32_t* idx, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_ix_init, gidx(n), dim3(256), 0, st, x, n, key, idx);
}
void launch_ix_heads(const unsigned long long* key, const uint32_t* slot, uint32_t m, uint32_t* headIn, uint32_t* tie,
                     hipStream_t st) {
  if (m) hipLaunchKernelGGL(k_ix_heads, gidx(m), dim3(256), 0, st, key, slot, m, headIn, tie);
}
void launch_ix_place(const uint32_t* val, const uint32_t* slot, const uint32_t* head, uint32_t m, int32_t* sa,
                     uint32_t* rank, hipStream_t st) {
  if (m) hipLaunchKernelGGL(k_ix_place, gidx(m), dim3(256), 0, st, val, slot, head, m, sa, rank);
}
void launch_ix_keys(const uint32_t* act, uint32_t U, const int32_t* sa, const uint32_t* rank, uint32_t n, uint32_t h,
                    unsigned long long* key, uint32_t* val, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_ix_keys, gidx(U), dim3(256), 0, st, act, U, sa, rank, n, h, key, val);
}
void launch_ix_lcp(const uint8_t* x, const int32_t* sa, uint32_t n, uint32_t* isa, int32_t* phi, int32_t* plcpRaw,
                   int32_t* lcp, uint8_t* bwt, int32_t* plcp, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_ix_isa_phi, gidx(n), dim3(256), 0, st, sa, n, isa, phi);
  const uint64_t chunks = ((uint64_t)n + kIdxChunk - 1) / kIdxChunk;
  hipLaunchKernelGGL(k_ix_plcp, gidx(chunks), dim3(256), 0, st, x, n, phi, plcpRaw);
  hipLaunchKernelGGL(k_ix_lcp_bwt, gidx((uint64_t)n + 1), dim3(256), 0, st, x, sa, n, plcpRaw, lcp, bwt);
  hipLaunchKernelGGL(k_ix_plcp_max, gidx(n), dim3(256), 0, st, isa, lcp, n, plcp);
}

}  // namespace cmsbwt
