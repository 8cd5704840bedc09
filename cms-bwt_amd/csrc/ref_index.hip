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

#include <algorithm>

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

// LCP[r] = PLCP[SA[r]] (LCP[n] = -1)
__global__ void k_ix_lcp(const int32_t* __restrict__ sa, uint32_t n, const int32_t* __restrict__ plcp,
                         int32_t* __restrict__ lcp) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n) return;
  if (r == n) { lcp[n] = -1; return; }
  lcp[r] = plcp[sa[r]];
}

// FN:294-297: BWT[r] = x[SA[r]-1] (0 at SA = 0)
__global__ void k_ix_bwt(const uint8_t* __restrict__ x, const int32_t* __restrict__ sa, uint32_t n,
                         uint8_t* __restrict__ bwt) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int32_t s = sa[r];
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
// FN:258-263 (ISA) with the Phi array of the PLCP pass
void launch_ix_isa(const int32_t* sa, uint32_t n, uint32_t* isa, int32_t* phi, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_ix_isa_phi, gidx(n), dim3(256), 0, st, sa, n, isa, phi);
}
// FN:270-274: PLCP by Phi, LCP, then the max-neighbour PLCP
void launch_ix_lcp(const uint8_t* x, const int32_t* sa, uint32_t n, const uint32_t* isa, const int32_t* phi,
                   int32_t* plcpRaw, int32_t* lcp, int32_t* plcp, hipStream_t st) {
  if (!n) return;
  const uint64_t chunks = ((uint64_t)n + kIdxChunk - 1) / kIdxChunk;
  hipLaunchKernelGGL(k_ix_plcp, gidx(chunks), dim3(256), 0, st, x, n, phi, plcpRaw);
  hipLaunchKernelGGL(k_ix_lcp, gidx((uint64_t)n + 1), dim3(256), 0, st, sa, n, plcpRaw, lcp);
  hipLaunchKernelGGL(k_ix_plcp_max, gidx(n), dim3(256), 0, st, isa, lcp, n, plcp);
}
void launch_ix_bwt(const uint8_t* x, const int32_t* sa, uint32_t n, uint8_t* bwt, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_ix_bwt, gidx(n), dim3(256), 0, st, x, sa, n, bwt);
}
}  // namespace cmsbwt

// ---------------------------------------------------------------- walk tables
// Device builds of the tables engine.h's host staging fills (same layouts):
// LCP block minima, child table, adjacency records, prefix-rank tables and the
// PLCP skip precondition.
namespace cmsbwt {

__global__ void k_ix_plcp_check(const int32_t* __restrict__ plcp, uint32_t n, uint32_t* __restrict__ err) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q + 1 >= n) return;
  if ((int64_t)plcp[q + 1] + 1 < (int64_t)plcp[q]) atomicOr(err, 1u);
}

__global__ void k_ix_level(const int32_t* __restrict__ prev, uint32_t prevLen, int32_t* __restrict__ cur,
                           uint32_t curLen) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= curLen) return;
  int32_t m = INT32_MAX;
  const uint64_t e = (uint64_t)i * 64 + 64 < prevLen ? (uint64_t)i * 64 + 64 : prevLen;
  for (uint64_t k = (uint64_t)i * 64; k < e; k++) m = prev[k] < m ? prev[k] : m;
  cur[i] = m;
}

__device__ __forceinline__ uint32_t ix_chr(const uint8_t* x, const int32_t* sa, uint32_t n, uint32_t k, int32_t l) {
  const uint64_t at = (uint64_t)(uint32_t)sa[k] + (uint32_t)(l > 0 ? l : 0);
  return at < n ? x[at] : 0u;
}

__global__ void k_ix_child(const uint8_t* __restrict__ x, const int32_t* __restrict__ sa,
                           const int32_t* __restrict__ lcp, uint32_t n, uint32_t* __restrict__ ld) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int32_t l = lcp[k] > 0 ? lcp[k] : 0;
  const uint32_t d = k ? ix_chr(x, sa, n, k, l) : 0u;
  const uint32_t u = lcp[k + 1] >= 0 ? ix_chr(x, sa, n, k, lcp[k + 1]) : 0u;
  ld[k] = ((uint32_t)(l < 0xffff ? l : 0xffff) << 16) | (d << 8) | u;
}

__device__ __forceinline__ uint32_t ix_lc(const int32_t* lcp, uint32_t n, int64_t k) {
  if (k < 0 || k > (int64_t)n) return 0;
  const int32_t v = lcp[k];
  return v < 0 ? 0u : (uint32_t)(v < 255 ? v : 255);
}

__device__ __forceinline__ void ix_rec(const int32_t* lcp, uint32_t n, uint32_t r, uint4* o) {
  uint32_t w[3] = {0, 0, 0};
#pragma unroll
  for (int j = 0; j < 6; j++) w[j / 4] |= ix_lc(lcp, n, (int64_t)r - j) << (8 * (j % 4));
#pragma unroll
  for (int j = 0; j < 6; j++) w[(6 + j) / 4] |= ix_lc(lcp, n, (int64_t)r + 1 + j) << (8 * ((6 + j) % 4));
  *o = make_uint4(r, w[0], w[1], w[2]);
}

__global__ void k_ix_adjacency(const int32_t* __restrict__ sa, const uint32_t* __restrict__ isa,
                               const int32_t* __restrict__ lcp, uint32_t n, uint4* __restrict__ pr,
                               uint4* __restrict__ ir) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t s = (uint32_t)sa[k];
  if (s == n - 1) pr[k] = make_uint4(0xffffffffu, 0, 0, 0);
  else ix_rec(lcp, n, isa[s + 1], &pr[k]);
  ix_rec(lcp, n, isa[k], &ir[k]);
}

// prefix-rank tables, one length l per launch (state cur/term carried over l)
__global__ void k_ix_pfx_count(const uint8_t* __restrict__ x, uint32_t n, uint32_t l, uint32_t B,
                               const uint8_t* __restrict__ map, const uint32_t* __restrict__ below,
                               uint32_t* __restrict__ cur, uint8_t* __restrict__ term, uint32_t* __restrict__ cf,
                               uint32_t* __restrict__ ct) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint32_t sym = 0;
  uint8_t t = term[p];
  if (!t) {
    const uint64_t at = (uint64_t)p + l - 1;
    if (at >= n) {
      t = 1;
    } else {
      const uint8_t b = x[at];
      if (map[b] == 0xff) { t = 1; sym = below[b]; }
      else sym = map[b];
    }
    term[p] = t;
  }
  const uint32_t c = (cur[p] << B) + sym;
  cur[p] = c;
  atomicAdd(t ? &ct[c] : &cf[c], 1u);
}

// same, for short lengths (E1 <= kPfxLds): block-private histograms in LDS
// (a few hundred bins would serialise 1e8 global atomics), flushed once
constexpr uint32_t kPfxLds = 4097;
__global__ void __launch_bounds__(256) k_ix_pfx_count_lds(const uint8_t* __restrict__ x, uint32_t n, uint32_t l,
                                                          uint32_t B, const uint8_t* __restrict__ map,
                                                          const uint32_t* __restrict__ below,
                                                          uint32_t* __restrict__ cur, uint8_t* __restrict__ term,
                                                          uint32_t* __restrict__ cf, uint32_t* __restrict__ ct,
                                                          uint32_t E1) {
  __shared__ uint32_t hf[kPfxLds], ht[kPfxLds];
  for (uint32_t i = threadIdx.x; i < E1; i += blockDim.x) hf[i] = ht[i] = 0;
  __syncthreads();
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t sym = 0;
    uint8_t t = term[p];
    if (!t) {
      const uint64_t at = p + l - 1;
      if (at >= n) {
        t = 1;
      } else {
        const uint8_t b = x[at];
        if (map[b] == 0xff) { t = 1; sym = below[b]; }
        else sym = map[b];
      }
      term[p] = t;
    }
    const uint32_t c = (cur[p] << B) + sym;
    cur[p] = c;
    atomicAdd(t ? &ht[c] : &hf[c], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < E1; i += blockDim.x) {
    if (hf[i]) atomicAdd(&cf[i], hf[i]);
    if (ht[i]) atomicAdd(&ct[i], ht[i]);
  }
}

__global__ void k_ix_pfx_write(const uint32_t* __restrict__ cfEx, const uint32_t* __restrict__ ctIn,
                               const uint32_t* __restrict__ cf, uint64_t E1, uint32_t* __restrict__ o) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= E1) return;
  o[2 * c] = cfEx[c] + ctIn[c];
  o[2 * c + 1] = cf[c];
}

// Answer entries of level l (device_common.h), from level l-1 (already
// final) and level l's own insertion points: a P that does not occur either
// inherits its parent's answer (the parent does not occur either) or, when
// the parent P[0..l-1) occurs with interval [S, S+C), gets l-1, the insertion
// point Start_l(P) of FN:65-76 and pos = SA of it.
__global__ void k_ix_pfx_answer(uint32_t* __restrict__ tab, const uint32_t* __restrict__ par, uint64_t E,
                                uint32_t B, const int32_t* __restrict__ sa, uint32_t n, uint32_t l) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= E) return;
  const uint32_t cnt = tab[2 * c + 1];
  if (cnt) return;  // occurs (counts never carry kPfxAns: n < 2^31)
  uint32_t S = 0, C = n;
  if (par) {
    const uint32_t p0 = par[2 * (c >> B)], p1 = par[2 * (c >> B) + 1];
    if (p1 & kPfxAns) { tab[2 * c] = p0; tab[2 * c + 1] = p1; return; }
    S = p0;
    C = p1;
  }
  uint32_t mm = tab[2 * c], f = kPfxAns | kPfxSmaller;
  if (mm >= S + C) { mm = S + C - 1; f = kPfxAns; }
  if (C == 1) f |= kPfxSingle;
  tab[2 * c] = (uint32_t)sa[mm];
  tab[2 * c + 1] = f | (l - 1);
}

// after every level's answers: occurring strings with one suffix store its
// reference position (kPfxOne)
__global__ void k_ix_pfx_one(uint32_t* __restrict__ tab, uint64_t E, const int32_t* __restrict__ sa) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= E) return;
  if (tab[2 * c + 1] == 1u) {
    tab[2 * c] = (uint32_t)sa[tab[2 * c]];
    tab[2 * c + 1] = kPfxOne | 1u;
  }
}

static inline dim3 gix(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

// paired level-K table (device_common.h DevRef::pfk): entry s of line Z
__global__ void k_ix_pfx_pair(const uint32_t* __restrict__ tabK, uint32_t K, uint64_t nent,
                              uint2* __restrict__ out) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nent) return;
  const uint64_t Z = e >> 3;
  const uint32_t s = (uint32_t)e & 7u;
  const uint64_t code = s < 4 ? ((uint64_t)s << (2 * (K - 1))) | Z : (Z << 2) | (s - 4);
  out[e] = make_uint2(tabK[2 * code], tabK[2 * code + 1]);
}
void launch_ix_pfx_pair(const uint32_t* tabK, uint32_t K, uint32_t* out, hipStream_t st) {
  const uint64_t nent = 8ull << (2 * (K - 1));
  hipLaunchKernelGGL(k_ix_pfx_pair, gix(nent), dim3(256), 0, st, tabK, K, nent, (uint2*)out);
}

__global__ void k_ix_plcp8(const int32_t* __restrict__ plcp, uint32_t n, uint8_t* __restrict__ out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) out[q] = (uint8_t)min(max(plcp[q], 0), 255);
}
void launch_ix_plcp8(const int32_t* plcp, uint32_t n, uint8_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_ix_plcp8, dim3((n + 255) / 256), dim3(256), 0, st, plcp, n, out);
}
void launch_ix_plcp_check(const int32_t* plcp, uint32_t n, uint32_t* err, hipStream_t st) {
  if (n > 1) hipLaunchKernelGGL(k_ix_plcp_check, gix(n), dim3(256), 0, st, plcp, n, err);
}
void launch_ix_level(const int32_t* prev, uint32_t prevLen, int32_t* cur, uint32_t curLen, hipStream_t st) {
  if (curLen) hipLaunchKernelGGL(k_ix_level, gix(curLen), dim3(256), 0, st, prev, prevLen, cur, curLen);
}
void launch_ix_child(const uint8_t* x, const int32_t* sa, const int32_t* lcp, uint32_t n, uint32_t* ld,
                     hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_ix_child, gix(n), dim3(256), 0, st, x, sa, lcp, n, ld);
}
void launch_ix_adjacency(const int32_t* sa, const uint32_t* isa, const int32_t* lcp, uint32_t n, uint32_t* pr,
                         uint32_t* ir, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_ix_adjacency, gix(n), dim3(256), 0, st, sa, isa, lcp, n, (uint4*)pr, (uint4*)ir);
}
void launch_ix_pfx_count(const uint8_t* x, uint32_t n, uint32_t l, uint32_t B, const uint8_t* map,
                         const uint32_t* below, uint32_t* cur, uint8_t* term, uint32_t* cf, uint32_t* ct,
                         hipStream_t st) {
  if (!n) return;
  const uint64_t E1 = (1ull << (B * l)) + 1;
  if (E1 <= kPfxLds) {
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_ix_pfx_count_lds, dim3((unsigned)blocks), dim3(256), 0, st, x, n, l, B, map, below, cur,
                       term, cf, ct, (uint32_t)E1);
  } else {
    hipLaunchKernelGGL(k_ix_pfx_count, gix(n), dim3(256), 0, st, x, n, l, B, map, below, cur, term, cf, ct);
  }
}
void launch_ix_pfx_write(const uint32_t* cfEx, const uint32_t* ctIn, const uint32_t* cf, uint64_t E1, uint32_t* o,
                         hipStream_t st) {
  if (E1) hipLaunchKernelGGL(k_ix_pfx_write, gix(E1), dim3(256), 0, st, cfEx, ctIn, cf, E1, o);
}

void launch_ix_pfx_answer(uint32_t* tab, const uint32_t* par, uint64_t E, uint32_t B, const int32_t* sa, uint32_t n,
                          uint32_t l, hipStream_t st) {
  if (E) hipLaunchKernelGGL(k_ix_pfx_answer, gix(E), dim3(256), 0, st, tab, par, E, B, sa, n, l);
}
void launch_ix_pfx_one(uint32_t* tab, uint64_t E, const int32_t* sa, hipStream_t st) {
  if (E) hipLaunchKernelGGL(k_ix_pfx_one, gix(E), dim3(256), 0, st, tab, E, sa);
}

}  // namespace cmsbwt
