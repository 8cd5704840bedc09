// ms_walk.hip — the matching-statistics walk and head finalisation on gfx950.
//
// Reference semantics (CMS-BWT-functions.cpp = FN):
//   adjustInterval FN:11-25, contractLeft FN:34-43, computeMSFactorAt FN:45-88,
//   binarySearchLB/RB FN:94-149, PSV/NSV rmq_tree.h:184-225, per-document walk
//   FN:1151-1212, j-scan FN:1359-1385, buckets FN:1162-1185.
//
// Parallel decomposition: the MS triple (pos, len,
// smaller) at a position is a function of the text suffix alone, so every
// document is cut into chunks of `chunk` positions, one lane per chunk.  A
// chunk [a, b) restarts from the SA root at a-1 (to learn pos(a-1) for the
// head test at a) and walks exactly as the reference does.  Two hot loops of
// the reference are replaced by equivalent logarithmic/wide forms:
//   * the PLCP skip loop `while (len > PLCP[pos+1])` (FN:1176-1185) is a
//     search for the first q >= pos+1 with PLCP[q] + q >= len + pos + 1;
//     PLCP[q] + q is non-decreasing (the longest repeated prefix shrinks by at
//     most one per position), so it is a galloping search;
//   * the singleton-interval extension compares 8 bytes per step (LCE).
// Per-position bucket updates become one run (pos, length) per head, turned
// into counts by a difference array (no per-character atomics).
#include <algorithm>

#include "device_common.h"
#include "kernels.h"

namespace cmsbwt {

// ------------------------------------------------------------ PSV / NSV
// psv(i, ub) = max{j <= i : lcp[j] < ub} or -1   (rmq_tree.h:184-205)
__device__ __forceinline__ int32_t d_psv(const DevRef& R, int32_t i, int32_t ub) {
  const int32_t* a = R.lcp;
  int32_t bs = i & ~63;
  for (int32_t j = i; j >= bs; --j)
    if (a[j] < ub) return j;
  uint32_t idx = (uint32_t)i >> 6;
  int L = 0;
  int64_t found = -1;
  for (; L < R.nlvl; ++L) {
    const int32_t* m = R.lvl[L];
    int64_t start = idx & ~63u;
    for (int64_t k = (int64_t)idx - 1; k >= start; --k)
      if (m[k] < ub) { found = k; break; }
    if (found >= 0 || start == 0) break;
    idx >>= 6;
  }
  if (found < 0) return -1;
  uint32_t b = (uint32_t)found;
  for (int l = L - 1; l >= 0; --l) {
    const int32_t* m = R.lvl[l];
    int64_t hi = min((int64_t)b * 64 + 63, (int64_t)R.lvlLen[l] - 1);
    for (int64_t k = hi; k >= (int64_t)b * 64; --k)
      if (m[k] < ub) { b = (uint32_t)k; break; }
  }
  int64_t hi = min((int64_t)b * 64 + 63, (int64_t)R.n - 1);
  for (int64_t k = hi; k >= (int64_t)b * 64; --k)
    if (a[k] < ub) return (int32_t)k;
  return -1;
}

// nsv(i, ub) = min{j >= i, j < n : lcp[j] < ub} or -1   (rmq_tree.h:208-225)
__device__ __forceinline__ int32_t d_nsv(const DevRef& R, int32_t i, int32_t ub) {
  const int32_t* a = R.lcp;
  const int64_t n = R.n;
  if ((int64_t)i >= n) return -1;
  int64_t be = min((int64_t)(i | 63) + 1, n);
  for (int64_t j = i; j < be; ++j)
    if (a[j] < ub) return (int32_t)j;
  uint32_t idx = (uint32_t)i >> 6;
  int L = 0;
  int64_t found = -1;
  for (; L < R.nlvl; ++L) {
    const int32_t* m = R.lvl[L];
    int64_t end = min((int64_t)(idx | 63u) + 1, (int64_t)R.lvlLen[L]);
    for (int64_t k = (int64_t)idx + 1; k < end; ++k)
      if (m[k] < ub) { found = k; break; }
    if (found >= 0 || end == (int64_t)R.lvlLen[L]) break;
    idx >>= 6;
  }
  if (found < 0) return -1;
  uint32_t b = (uint32_t)found;
  for (int l = L - 1; l >= 0; --l) {
    const int32_t* m = R.lvl[l];
    int64_t end = min((int64_t)b * 64 + 64, (int64_t)R.lvlLen[l]);
    for (int64_t k = (int64_t)b * 64; k < end; ++k)
      if (m[k] < ub) { b = (uint32_t)k; break; }
  }
  int64_t end = min((int64_t)b * 64 + 64, n);
  for (int64_t k = (int64_t)b * 64; k < end; ++k)
    if (a[k] < ub) return (int32_t)k;
  return -1;
}

// FN:11-25
__device__ __forceinline__ void d_adjust(const DevRef& R, int32_t lo, int32_t hi, int32_t off,
                                         int32_t& nl, int32_t& nr) {
  int32_t p = d_psv(R, lo, off);
  nl = p == -1 ? 0 : p;
  int32_t q = d_nsv(R, hi + 1, off);
  nr = q == -1 ? (int32_t)R.n - 1 : q - 1;
}

// FN:34-43
__device__ __forceinline__ void d_contract(const DevRef& R, int32_t& lo, int32_t& hi, int32_t off) {
  uint32_t sl = (uint32_t)R.sa[lo], sh = (uint32_t)R.sa[hi];
  if (sl == R.n - 1 || sh == R.n - 1) { lo = 0; hi = (int32_t)R.n - 1; return; }
  d_adjust(R, (int32_t)R.isa[sl + 1], (int32_t)R.isa[sh + 1], off, lo, hi);
}

// First m in [lo, hi+1) with x[SA[m]+off] >= c (FN:94-120 returns this index
// when the symbol is present, else -(this index)-1).
__device__ __forceinline__ int32_t d_lower(const DevRef& R, int32_t lo, int32_t hi, uint32_t off, uint8_t c) {
  int32_t a = lo, b = hi + 1;
  while (a < b) {
    int32_t m = (a + b) >> 1;
    if (R.x[(uint32_t)R.sa[m] + off] < c) a = m + 1; else b = m;
  }
  return a;
}
// First m in [lo, hi+1) with x[SA[m]+off] > c (FN:123-149 returns this - 1).
__device__ __forceinline__ int32_t d_upper(const DevRef& R, int32_t lo, int32_t hi, uint32_t off, uint8_t c) {
  int32_t a = lo, b = hi + 1;
  while (a < b) {
    int32_t m = (a + b) >> 1;
    if (R.x[(uint32_t)R.sa[m] + off] <= c) a = m + 1; else b = m;
  }
  return a;
}

// 8 bytes starting at an arbitrary address (both buffers are padded).
__device__ __forceinline__ uint64_t d_load8(const uint8_t* p) {
  uintptr_t a = (uintptr_t)p;
  const uint64_t* w = (const uint64_t*)(a & ~(uintptr_t)7);
  uint32_t s = (uint32_t)(a & 7) * 8;
  uint64_t lo = w[0];
  if (s == 0) return lo;
  uint64_t hi = w[1];
  return (lo >> s) | (hi << (64 - s));
}

// Longest common extension of x[q..] and t[j..]: stops at the first mismatch,
// which always exists (the document separator 0x02 is absent from x).
__device__ __forceinline__ uint32_t d_lce(const uint8_t* xq, const uint8_t* tj) {
  uint64_t d = d_load8(xq) ^ d_load8(tj);
  if (d) return (uint32_t)(__builtin_ctzll(d) >> 3);
  uint32_t k = 8;
  while (true) {  // 32 bytes per step, loads issued together
    uint64_t d0 = d_load8(xq + k) ^ d_load8(tj + k);
    uint64_t d1 = d_load8(xq + k + 8) ^ d_load8(tj + k + 8);
    uint64_t d2 = d_load8(xq + k + 16) ^ d_load8(tj + k + 16);
    uint64_t d3 = d_load8(xq + k + 24) ^ d_load8(tj + k + 24);
    if (d0) return k + (uint32_t)(__builtin_ctzll(d0) >> 3);
    if (d1) return k + 8 + (uint32_t)(__builtin_ctzll(d1) >> 3);
    if (d2) return k + 16 + (uint32_t)(__builtin_ctzll(d2) >> 3);
    if (d3) return k + 24 + (uint32_t)(__builtin_ctzll(d3) >> 3);
    k += 32;
  }
}

// Smallest s >= 0 with len - s <= PLCP[base + s]  (FN:1176 loop exit).
// With q = base + s the condition is PLCP[q] + q >= base + len =: T, and
// PLCP[q] + q is non-decreasing, so the answer is the first q in [base, T]
// crossing T.  PLCP is short outside long repeats, so the crossing almost
// always lies in the 16 entries just below T: probe that window with
// independent loads first, gallop from `base` only when it does not.
__device__ __forceinline__ uint32_t d_skip(const DevRef& R, uint32_t base, uint32_t len) {
  const int32_t* P = R.plcp;
  if ((int64_t)len <= (int64_t)P[base]) return 0;
  const int64_t T = (int64_t)base + len;
  if (len > 16) {
    const int64_t w0 = T - 16;  // > base
    if ((int64_t)P[w0] + w0 < T) {  // crossing inside (w0, T]: count entries below T
      uint32_t c = 0;
#pragma unroll
      for (int k = 1; k <= 16; k++) c += ((int64_t)P[w0 + k] + w0 + k < T) ? 1u : 0u;
      return (uint32_t)(w0 + 1 + c - base);
    }
  }
  uint32_t lo = 0, hi, step = 1;
  while (true) {
    uint64_t t = (uint64_t)lo + step;
    if (t >= len) { hi = len; break; }
    if ((int64_t)len - (int64_t)t <= (int64_t)P[base + (uint32_t)t]) { hi = (uint32_t)t; break; }
    lo = (uint32_t)t;
    step <<= 1;
  }
  while (hi - lo > 1) {
    uint32_t mid = lo + ((hi - lo) >> 1);
    if ((int64_t)len - (int64_t)mid <= (int64_t)P[base + mid]) hi = mid; else lo = mid;
  }
  return hi;
}

// ------------------------------------------------------------ MS walk kernel
__global__ void __launch_bounds__(256) k_ms_walk(DevRef R, const uint8_t* __restrict__ text,
                                                 const uint64_t* __restrict__ docOff,
                                                 const Chunk* __restrict__ chunks, uint32_t nchunks,
                                                 const uint32_t* __restrict__ laneChunk,
                                                 Pool pool, uint32_t* __restrict__ chunkCount) {
  const uint32_t lane_id = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane_id >= nchunks) return;
  const uint32_t cid = laneChunk[lane_id];
  const Chunk ch = chunks[cid];
  const uint8_t* t = text + docOff[ch.doc];
  const uint32_t a = ch.a, b = ch.b;
  const uint32_t n = R.n;
  uint32_t count = 0, blk = 0xffffffffu, fill = kPoolB, seq = 0;

  uint32_t i = a > 0 ? a - 1 : 0;
  uint32_t len = 0, pos = n - 1;
  int32_t lb = 0, rb = (int32_t)n - 1;
  uint64_t prevPos = (uint64_t)-2;
  bool smaller = false;
  while (i < b) {
    // ---- computeMSFactorAt (FN:45-88)
    {
      uint32_t off = len, j = i + off;
      int32_t nlb = lb, nrb = rb;
      while (true) {
        if (nlb == nrb) {
          uint32_t q = (uint32_t)R.sa[nlb];
          uint32_t m = d_lce(R.x + q + off, t + j);
          off += m;
          j += m;
          smaller = (int8_t)R.x[q + off] > (int8_t)t[j];
          pos = q;
          break;
        }
        uint8_t c = t[j];
        int32_t l2 = d_lower(R, nlb, nrb, off, c);
        if (l2 > nrb || R.x[(uint32_t)R.sa[l2] + off] != c) {
          int32_t mm = l2;
          smaller = true;
          if (mm == nrb + 1) { mm = nrb; smaller = false; }
          pos = (uint32_t)R.sa[mm];
          break;
        }
        int32_t r2 = d_upper(R, l2, nrb, off, c) - 1;
        nlb = l2; nrb = r2;
        lb = nlb; rb = nrb;
        off++; j++;
      }
      len = off;
    }
    // ---- head test and record (FN:1154-1171)
    if (i >= a && (uint64_t)pos != prevPos + 1) {
      if (fill == kPoolB) {
        blk = atomicAdd(pool.used, 1u);
        fill = 0;
        if (blk < pool.capBlocks) { pool.blkChunk[blk] = cid; pool.blkSeq[blk] = seq; }
        seq++;
      }
      if (blk < pool.capBlocks) {
        HeadRec r;
        r.start = i;
        r.pos = pos;
        r.len = len;
        r.flags = smaller ? 1u : 0u;
        pool.rec[(uint64_t)blk * kPoolB + fill] = r;
      }
      fill++;
      count++;
    }
    len--;
    if (lb == rb) {  // FN:1175-1189
      uint32_t s = d_skip(R, pos + 1, len);
      i += s; len -= s; pos += s;
      int32_t v = (int32_t)R.isa[pos + 1];
      d_adjust(R, v, v, (int32_t)len, lb, rb);
    } else {         // FN:1190-1194
      d_contract(R, lb, rb, (int32_t)len);
    }
    i++;
    prevPos = pos;
  }
  chunkCount[cid] = count;
}

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
  uint32_t cid = pool.blkChunk[blk];
  if (cid == 0xffffffffu) return;  // reserved by a lane, never started
  uint32_t local = pool.blkSeq[blk] * kPoolB + (uint32_t)(slot % kPoolB);
  if (local >= chunkCount[cid]) return;
  uint32_t idx = (uint32_t)chunkBase[cid] + local;
  HeadRec r = pool.rec[slot];
  h.start[idx] = r.start;
  h.pos[idx] = r.pos;
  h.len[idx] = r.len;
  h.smaller[idx] = (uint8_t)(r.flags & 1u);
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
                           uint32_t* __restrict__ errFlags, const uint32_t* __restrict__ hdoc) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H) return;
  const uint32_t leni = h.len[i];
  if (leni == 0) {  // end phrase: isaNext = ISA[n-1] = 0, toNext = 0, nextHead = 0
    h.isa[i] = 0;
    h.tonext[i] = 0;
    h.nexthead[i] = 0;
    return;
  }
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
  h.isa[i] = R.isa[q];
  // Order invariant: the isaNext suffix starts with the mismatching text byte
  // (or the head ends at the document separator and isaNext is the smallest
  // suffix).  When it holds for every head, MatchInSet::operator< is a strict
  // weak order on every position's keys and queries.
  const uint8_t* dt = text + docOff[lo];
  {
    const uint8_t c = dt[ei];
    if (!(c == R.x[q] || (c == kSep && q == R.n - 1))) atomicOr(errFlags, 8u);
  }
  // BWT character of the phrase (FN:1158-1161): the text byte before it, 0x02
  // at a document start.  Read here rather than in k_scatter_heads: heads are
  // in document order, so a wave reads the same text lines as for the check.
  h.lchar[i] = si == 0 ? (uint8_t)kSep : dt[si - 1];
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
void launch_ms_walk(const DevRef& R, const uint8_t* text, const uint64_t* docOff, const Chunk* chunks,
                    uint32_t nchunks, const uint32_t* laneChunk, const Pool& pool, uint32_t* chunkCount,
                    hipStream_t st) {
  if (!nchunks) return;
  hipLaunchKernelGGL(k_ms_walk, dim3((nchunks + 255) / 256), dim3(256), 0, st, R, text, docOff, chunks,
                     nchunks, laneChunk, pool, chunkCount);
}

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

void launch_finalize(const DevRef& R, const HeadsSoA& h, uint32_t H, const uint32_t* docEndIdx,
                     uint32_t ndocs, const uint8_t* text, const uint64_t* docOff, uint32_t* errFlags,
                     const uint32_t* hdoc, hipStream_t st) {
  if (!H) return;
  hipLaunchKernelGGL(k_finalize, dim3((H + 255) / 256), dim3(256), 0, st, R, h, H, docEndIdx, ndocs, text, docOff,
                     errFlags, hdoc);
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
