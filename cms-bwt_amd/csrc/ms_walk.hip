// ms_walk.hip — the walk's bookkeeping around k_ms_walk2 (ms_walk2.hip) and
// head finalisation on gfx950.
//
// Reference semantics (CMS-BWT-functions.cpp = FN): per-document walk
// FN:1151-1212 (pool records -> document order, end-of-document phrases),
// j-scan FN:1359-1385 (k_finalize), buckets FN:1162-1185 (run difference
// arrays through position bins).
#include <algorithm>

#include "device_common.h"
#include "kernels.h"

namespace cmsbwt {

// ------------------------------------------------------------ pool -> idx order
__global__ void k_chunk_with_end(const Chunk* __restrict__ chunks, const uint32_t* __restrict__ chunkCount,
                                 uint32_t nch, unsigned long long* __restrict__ out) {
  uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nch) out[c] = (unsigned long long)chunkCount[c] + chunks[c].last;
}

__global__ void k_scatter_heads(Pool pool, uint32_t blocksUsed, const uint32_t* __restrict__ chunkCount,
                                const unsigned long long* __restrict__ chunkBase, HeadsSoA h,
                                const Chunk* __restrict__ chunks, const uint8_t* __restrict__ text,
                                const uint64_t* __restrict__ docOff, uint32_t* __restrict__ hdoc) {
  uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t blk = slot / kPoolB;
  if (blk >= blocksUsed) return;
  const uint2 bm = pool.blkMeta[blk];
  const uint32_t cid = bm.x;
  if (cid == 0xffffffffu) return;  // reserved by a lane, never started
  uint32_t local = bm.y * kPoolB + (uint32_t)(slot % kPoolB);
  if (local >= chunkCount[cid]) return;
  uint32_t idx = (uint32_t)chunkBase[cid] + local;
  HeadRec r = pool.rec[slot];
  h.start[idx] = r.start;
  h.pos[idx] = r.pos;
  h.len[idx] = r.len;
  h.smaller[idx] = (uint8_t)(r.flags & 1u);
  // (CMSBWT_WALK_LCHAR) the BWT character when the walk had it: 0x100 | byte,
  // or 0; parked in tonext, which k_finalize reads before writing it
  if (kWalkLchar) h.tonext[idx] = r.flags >> 8;
  // (the BWT character before the phrase is read by k_finalize, whose
  // document-ordered threads read the text lines coalesced)
  hdoc[idx] = chunks[cid].doc;
}

// End-of-document phrase (FN:1198-1212): (docLen, n-1, 0, false), char =
// last sequence byte or 0x02 for an empty document.
__global__ void k_end_phrases(const uint8_t* __restrict__ text, const uint64_t* __restrict__ docOff,
                              uint32_t ndocs, const uint32_t* __restrict__ docLastChunk,
                              const uint32_t* __restrict__ chunkCount,
                              const unsigned long long* __restrict__ chunkBase, uint32_t n, HeadsSoA h,
                              uint32_t* __restrict__ docEndIdx, uint32_t* __restrict__ hdoc) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  uint32_t c = docLastChunk[d];
  uint32_t idx = (uint32_t)chunkBase[c] + chunkCount[c];
  uint64_t len = docOff[d + 1] - docOff[d] - 1;
  h.start[idx] = (uint32_t)len;
  h.pos[idx] = n - 1;
  h.len[idx] = 0;
  h.smaller[idx] = 0;
  h.lchar[idx] = len ? text[docOff[d] + len - 1] : kSep;
  docEndIdx[d] = idx;
  hdoc[idx] = d;
}

// ------------------------------------------------------------ j-scan (FN:1359-1385)
// For head i: j = first k > i (within its document) with end_k > end_i or k the
// end phrase; ends are non-decreasing inside a document (MS(q+1) >= MS(q)-1), so
// the reference's monotone pointer equals this search.  Also: toNext, isaNext,
// nextHead (uint16, FN:1128/1379), and the run (pos, start_{i+1}-start_i) that
// replaces the per-position bucket increments.
__global__ void k_finalize(DevRef R, HeadsSoA h, uint32_t H, const uint32_t* __restrict__ docEndIdx,
                           uint32_t ndocs, const uint8_t* __restrict__ text, const uint64_t* __restrict__ docOff,
                           uint32_t* __restrict__ errFlags, const uint32_t* __restrict__ hdoc,
                           const uint32_t* __restrict__ isax) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H) return;
  const uint32_t leni = h.len[i];
  if (leni == 0) {  // end phrase: isaNext = ISA[n-1] = 0, toNext = 0, nextHead = 0
    h.isa[i] = 0;
    h.tonext[i] = 0;
    h.nexthead[i] = 0;
    return;
  }
  const uint32_t lk = kWalkLchar ? h.tonext[i] : 0u;  // the walk's BWT character (0x100 | byte) or 0
  const uint32_t lo = hdoc[i];  // document of i (written by the scatter)
  const uint32_t de = docEndIdx[lo];
  const uint32_t si = h.start[i];
  const uint32_t ei = si + leni;
  // monotone ends check (the search below relies on it)
  if (i + 1 < de && h.start[i + 1] + h.len[i + 1] < ei) atomicOr(errFlags, 1u);
  auto cond = [&](uint32_t k) -> bool { return h.len[k] == 0 || h.start[k] + h.len[k] > ei; };
  uint32_t l = i, k = i + 1, step = 1;
  while (!cond(k)) {
    l = k;
    uint64_t nk = (uint64_t)k + step;
    k = nk > de ? de : (uint32_t)nk;
    step <<= 1;
  }
  while (k - l > 1) {  // cond(l) false (or l == i), cond(k) true
    uint32_t m = l + ((k - l) >> 1);
    if (cond(m)) k = m; else l = m;
  }
  const uint32_t j = k;
  const uint32_t s1 = h.start[i + 1];
  h.tonext[i] = s1 - si - 1;
  const uint32_t sj = h.start[j];
  uint32_t q = h.pos[j] + (ei - sj);
  if (q >= R.n) { atomicOr(errFlags, 2u); q = R.n - 1; }
  // isax (n < 2^24): ISA[q] | x[q] << 24, one random line instead of two
  const uint32_t ix = isax ? isax[q] : 0u;
  h.isa[i] = isax ? ix & 0xffffffu : R.isa[q];
  // Order invariant: the isaNext suffix starts with the mismatching text byte
  // (or the head ends at the document separator and isaNext is the smallest
  // suffix).  When it holds for every head and the reference has no byte >=
  // 0x80 (FN:55's signed compare then agrees with the suffix order; checked
  // on the host), MatchInSet::operator< is a strict weak order on every
  // position's keys and queries.
  const uint8_t* dt = text + docOff[lo];
  // (CMSBWT_WALK_LCHAR) t[ei] lies in head j's match when sj <= ei (ei < sj +
  // len_j by the search) and then equals x[q] by that match: the text is read
  // only for the others
  if (!kWalkLchar || sj > ei || h.len[j] == 0) {
    const uint8_t c = dt[ei];
    const uint8_t xq = isax ? (uint8_t)(ix >> 24) : R.x[q];
    if (!(c == xq || (c == kSep && q == R.n - 1))) atomicOr(errFlags, 8u);
  }
  // BWT character of the phrase (FN:1158-1161): the text byte before it, 0x02
  // at a document start.  Read here rather than in k_scatter_heads: heads are
  // in document order, so a wave reads the same text lines as for the check.
  h.lchar[i] = si == 0 ? (uint8_t)kSep : (lk & 0x100u) ? (uint8_t)lk : dt[si - 1];
  h.nexthead[i] = (uint16_t)(j - i);
  if ((uint64_t)h.pos[i] + (s1 - si) > R.n) atomicOr(errFlags, 4u);
}

// ------------------------------------------------------------ run buckets (FN:1162-1171, 1203)
// Every head i covers the reference positions [pos_i, pos_i + start_{i+1} -
// start_i) with one bucket increment each; an end phrase covers [n-1, n).
// diff = (#runs starting at p) - (#runs ending at p) and hasHead[p] = (#runs
// starting at p) > 0.  Instead of two random device-scope atomics and a random
// byte store per head, the run endpoints (pos << 1 | isEnd) are scattered into
// bins of 2^kRunBinShift positions (count, scan, scatter) and every bin is
// counted in LDS and written out coalesced.
// bins are 2^sh positions, sh <= kRunBinShift (smaller only to test bin edges)
__device__ __forceinline__ bool run_of(const HeadsSoA& h, uint32_t i, uint32_t n, uint32_t& p, uint32_t& e) {
  if (h.len[i] == 0) { p = n - 1; e = n; return true; }
  p = h.pos[i];
  const uint64_t endp = (uint64_t)p + (h.start[i + 1] - h.start[i]);
  if (endp > n) return false;  // flagged by k_finalize (errFlags 4)
  e = (uint32_t)endp;
  return true;
}

template <bool kLds>
__global__ void k_run_bin_count(HeadsSoA h, uint32_t H, uint32_t n, uint32_t nb, uint32_t sh,
                                uint32_t* __restrict__ binCnt) {
  extern __shared__ uint32_t lds[];
  if (kLds) {
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) lds[j] = 0;
    __syncthreads();
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < H; i += gridDim.x * blockDim.x) {
    uint32_t p, e;
    if (!run_of(h, i, n, p, e)) continue;
    atomicAdd(kLds ? &lds[p >> sh] : &binCnt[p >> sh], 1u);
    atomicAdd(kLds ? &lds[e >> sh] : &binCnt[e >> sh], 1u);
  }
  if (kLds) {
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x)
      if (lds[j]) atomicAdd(&binCnt[j], lds[j]);
  }
}

// binCur = exclusive prefix of the counts on entry; each block visits the same
// heads as in k_run_bin_count's launch (same grid), reserves its share of every
// bin once, then places its endpoints through LDS cursors.
template <bool kLds>
__global__ void k_run_bin_scatter(HeadsSoA h, uint32_t H, uint32_t n, uint32_t nb, uint32_t sh,
                                  uint32_t* __restrict__ binCur, uint32_t* __restrict__ vals) {
  extern __shared__ uint32_t lds[];
  if (kLds) {
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) lds[j] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < H; i += gridDim.x * blockDim.x) {
      uint32_t p, e;
      if (!run_of(h, i, n, p, e)) continue;
      atomicAdd(&lds[p >> sh], 1u);
      atomicAdd(&lds[e >> sh], 1u);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x)
      if (lds[j]) lds[j] = atomicAdd(&binCur[j], lds[j]);
    __syncthreads();
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < H; i += gridDim.x * blockDim.x) {
    uint32_t p, e;
    if (!run_of(h, i, n, p, e)) continue;
    vals[atomicAdd(kLds ? &lds[p >> sh] : &binCur[p >> sh], 1u)] = p << 1;
    vals[atomicAdd(kLds ? &lds[e >> sh] : &binCur[e >> sh], 1u)] = e << 1 | 1u;
  }
}

__global__ __launch_bounds__(1024) void k_run_bin_emit(const uint32_t* __restrict__ vals,
                                                       const uint32_t* __restrict__ binOff, uint32_t n,
                                                       uint32_t sh, int32_t* __restrict__ diff,
                                                       uint8_t* __restrict__ hasHead) {
  constexpr uint32_t kW = 1u << kRunBinShift;
  __shared__ uint32_t cs[kW], ce[kW];
  const uint32_t W = 1u << sh;
  for (uint32_t j = threadIdx.x; j < W; j += blockDim.x) cs[j] = ce[j] = 0;
  __syncthreads();
  const uint32_t b = blockIdx.x, k1 = binOff[b + 1];
  for (uint32_t k = binOff[b] + threadIdx.x; k < k1; k += blockDim.x) {
    const uint32_t v = vals[k], j = (v >> 1) & (W - 1);
    atomicAdd((v & 1u) ? &ce[j] : &cs[j], 1u);
  }
  __syncthreads();
  const uint64_t base = (uint64_t)b << sh;
  for (uint32_t j = threadIdx.x; j < W; j += blockDim.x) {
    const uint64_t q = base + j;
    if (q <= n) diff[q] = (int32_t)(cs[j] - ce[j]);
    if (q < n) hasHead[q] = cs[j] != 0;
  }
}

// ------------------------------------------------------------ host launchers
void launch_chunk_with_end(const Chunk* chunks, const uint32_t* chunkCount, uint32_t nch, unsigned long long* out,
                           hipStream_t st) {
  if (nch) hipLaunchKernelGGL(k_chunk_with_end, dim3((nch + 255) / 256), dim3(256), 0, st, chunks, chunkCount, nch, out);
}

void launch_scatter_heads(const Pool& pool, uint32_t blocksUsed, const uint32_t* chunkCount,
                          const unsigned long long* chunkBase, const HeadsSoA& h, const Chunk* chunks,
                          const uint8_t* text, const uint64_t* docOff, uint32_t* hdoc, hipStream_t st) {
  uint64_t slots = (uint64_t)blocksUsed * kPoolB;
  if (!slots) return;
  hipLaunchKernelGGL(k_scatter_heads, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, st, pool,
                     blocksUsed, chunkCount, chunkBase, h, chunks, text, docOff, hdoc);
}

void launch_end_phrases(const uint8_t* text, const uint64_t* docOff, uint32_t ndocs,
                        const uint32_t* docLastChunk, const uint32_t* chunkCount,
                        const unsigned long long* chunkBase, uint32_t n, const HeadsSoA& h, uint32_t* docEndIdx,
                        uint32_t* hdoc, hipStream_t st) {
  if (!ndocs) return;
  hipLaunchKernelGGL(k_end_phrases, dim3((ndocs + 255) / 256), dim3(256), 0, st, text, docOff, ndocs,
                     docLastChunk, chunkCount, chunkBase, n, h, docEndIdx, hdoc);
}

__global__ void k_isax(const uint32_t* __restrict__ isa, const uint8_t* __restrict__ x, uint32_t n,
                       uint32_t* __restrict__ out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) out[p] = isa[p] | ((uint32_t)x[p] << 24);
}
void launch_isax(const uint32_t* isa, const uint8_t* x, uint32_t n, uint32_t* out, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_isax, dim3((n + 255) / 256), dim3(256), 0, st, isa, x, n, out);
}
void launch_finalize(const DevRef& R, const HeadsSoA& h, uint32_t H, const uint32_t* docEndIdx,
                     uint32_t ndocs, const uint8_t* text, const uint64_t* docOff, uint32_t* errFlags,
                     const uint32_t* hdoc, hipStream_t st, const uint32_t* isax) {
  if (!H) return;
  hipLaunchKernelGGL(k_finalize, dim3((H + 255) / 256), dim3(256), 0, st, R, h, H, docEndIdx, ndocs, text, docOff,
                     errFlags, hdoc, isax);
}

static unsigned run_bin_grid(uint32_t H) { return std::max(1u, std::min((H + 255) / 256, 1024u)); }

void launch_run_bin_count(const HeadsSoA& h, uint32_t H, uint32_t n, uint32_t nb, uint32_t sh, bool global,
                          uint32_t* binCnt, hipStream_t st) {
  if (!H) return;
  if (nb <= kRunBinLdsMax && !global)
    hipLaunchKernelGGL(k_run_bin_count<true>, dim3(run_bin_grid(H)), dim3(256), nb * 4, st, h, H, n, nb, sh, binCnt);
  else
    hipLaunchKernelGGL(k_run_bin_count<false>, dim3(run_bin_grid(H)), dim3(256), 0, st, h, H, n, nb, sh, binCnt);
}

void launch_run_bin_scatter(const HeadsSoA& h, uint32_t H, uint32_t n, uint32_t nb, uint32_t sh, bool global,
                            uint32_t* binCur, uint32_t* vals, hipStream_t st) {
  if (!H) return;
  if (nb <= kRunBinLdsMax && !global)
    hipLaunchKernelGGL(k_run_bin_scatter<true>, dim3(run_bin_grid(H)), dim3(256), nb * 4, st, h, H, n, nb, sh,
                       binCur, vals);
  else
    hipLaunchKernelGGL(k_run_bin_scatter<false>, dim3(run_bin_grid(H)), dim3(256), 0, st, h, H, n, nb, sh, binCur,
                       vals);
}

void launch_run_bin_emit(const uint32_t* vals, const uint32_t* binOff, uint32_t n, uint32_t nb, uint32_t sh,
                         int32_t* diff, uint8_t* hasHead, hipStream_t st) {
  if (nb) hipLaunchKernelGGL(k_run_bin_emit, dim3(nb), dim3(1024), 0, st, vals, binOff, n, sh, diff, hasHead);
}

}  // namespace cmsbwt
