// merge.hip — MS-factor -> BWT-run merge kernels (FN:1387-1777).
//
// Every kernel here is integer/byte work; the heavy lifting between them is
// done by rocPRIM radix sorts and scans driven from engine.hip.
#include <hip/hip_runtime.h>
#include "device_common.h"
#include "kernels.h"
#include "merge_kernels.h"
#include "elem_writer.h"

#include <algorithm>
#include <cstdlib>

namespace cmsbwt {

__global__ void k_iota(uint32_t* p, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

__global__ void k_gather_u32(const uint32_t* __restrict__ src, const uint32_t* __restrict__ perm,
                             uint32_t* __restrict__ dst, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}


// item boundaries over perm sorted by (pos, len, isaNext, idx)
__global__ void k_item_flags(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ pos,
                             const uint32_t* __restrict__ len, const uint32_t* __restrict__ isa,
                             uint32_t* __restrict__ flag, uint64_t H) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  if (k == 0) { flag[k] = 1; return; }
  uint32_t a = perm[k], b = perm[k - 1];
  flag[k] = (pos[a] != pos[b] || len[a] != len[b] || isa[a] != isa[b]) ? 1u : 0u;
}

// Composite grouping key (pos, len, isaNext) in one 64-bit word when the
// fields fit: one stable radix sort replaces three, and item boundaries and
// item fields come from the sorted keys (no per-head gathers).
__global__ void k_group_key(const HeadsSoA h, uint64_t H, int bN, int bL, unsigned long long* __restrict__ key) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H) return;
  key[i] = ((unsigned long long)h.pos[i] << (bN + bL)) | ((unsigned long long)h.len[i] << bN) | h.isa[i];
}
// ---- grouping, position first: after a stable radix sort of the heads by
// pos (HeadKV values in idx order within a position), each position's
// segment is sorted by (len, isaNext) here.  Output: the composite key
// pos|len|isaNext of every sorted head (what the one-sort path produces) and
// its idx.  Segments longer than maxSmall are listed for a radix sort.
constexpr uint32_t kGrpBlock = 256, kGrpHalo = 64;  // segments of <= kGrpHalo heads are ranked in LDS
constexpr uint32_t kGrpEnds = 2048;  // run ends counted in LDS: [first position of the block, + kGrpEnds)
__global__ void __launch_bounds__(256) k_grp_seg(const uint32_t* __restrict__ posS, const uint32_t* __restrict__ hb,
                                                 const HeadKV* __restrict__ kv, uint32_t H, int bN, int bL,
                                                 unsigned long long* __restrict__ key, uint32_t* __restrict__ perm,
                                                 uint32_t* __restrict__ tsOut, uint8_t* __restrict__ smOut,
                                                 uint32_t* __restrict__ bigList, uint32_t maxSmall,
                                                 int32_t* __restrict__ diffEnds, uint32_t n) {
  // one thread per sorted head: its rank inside its position's segment in
  // MAP order (match.h:27-33 on consistent data: smaller=true items by (len,
  // isaNext), then smaller=false items by (len descending, isaNext); members
  // of an item by idx), by counting over the segment staged in LDS with a
  // halo either side.  An item's class is the `smaller` of its first-inserted
  // (lowest idx) member, as the first std::map insertion keeps it.
  constexpr uint32_t W = kGrpBlock + 2 * kGrpHalo;
  __shared__ unsigned long long lk[W], mk[W];
  __shared__ uint32_t lp[W];
  __shared__ uint8_t ls[W];
  __shared__ int32_t endL[kGrpEnds];
  const uint32_t k0 = blockIdx.x * kGrpBlock;
  const int64_t base = (int64_t)k0 - kGrpHalo;
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) {
    const int64_t j = base + i;
    if (j >= 0 && j < (int64_t)H) {
      const HeadKV w = kv[j];
      lk[i] = ((unsigned long long)(w.len & 0x7fffffffu) << bN) | w.isa;
      lp[i] = posS[j];
      ls[i] = (uint8_t)(w.len >> 31);
    } else {
      lp[i] = 0xffffffffu;
    }
  }
  if (diffEnds)
    for (uint32_t i = threadIdx.x; i < kGrpEnds; i += blockDim.x) endL[i] = 0;
  __syncthreads();
  // map key of every staged head: its item's first member is the leftmost
  // entry of its position with the same (len, isaNext) (kv is idx-ascending
  // per position).  Only heads of segments ranked here (<= the halo, inside
  // the window) need it; the scan has fixed bounds (segment start from hb),
  // so its LDS reads pipeline
  const uint32_t lim = min(maxSmall, kGrpHalo);
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) {
    const uint32_t pi = lp[i];
    if (pi == 0xffffffffu) continue;
    const int64_t sb = (int64_t)hb[pi] - base, se = (int64_t)hb[pi + 1] - base;
    if (se - sb > lim || sb < 0 || se > (int64_t)W) continue;
    if (se <= (int64_t)kGrpHalo || sb >= (int64_t)(kGrpHalo + kGrpBlock)) continue;  // no owner in this block
    const unsigned long long me = lk[i];
    uint32_t f = i;
    for (int64_t j = (int64_t)i - 1; j >= sb; j--) f = lk[j] == me ? (uint32_t)j : f;
    const unsigned long long L = me >> bN, I = me & ((1ull << bN) - 1);
    mk[i] = ls[f] ? ((L << bN) | I) : ((1ull << 63) | ((~L & ((1ull << bL) - 1)) << bN) | I);
  }
  __syncthreads();
  const uint32_t k = k0 + threadIdx.x;
  if (diffEnds) {
    // run ends (FN:1162-1171, 1203): head i covers [pos_i, pos_i + start_{i+1}
    // - start_i) = [pos, pos + toNext + 1) (an end phrase: [n-1, n)); ends
    // near the block's first position are counted in LDS, the rest atomically
    const uint32_t pmin = posS[k0];
    if (k < H) {
      const uint64_t e = (uint64_t)posS[k] + kv[k].tonext + 1;
      if (e <= n) {
        if (e - pmin < kGrpEnds) atomicAdd(&endL[e - pmin], 1);
        else atomicAdd(&diffEnds[e], -1);
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kGrpEnds; i += blockDim.x)
      if (endL[i]) atomicAdd(&diffEnds[pmin + i], -endL[i]);
  }
  if (k >= H) return;
  const uint32_t p = posS[k];
  const uint32_t b = hb[p], e = hb[p + 1];
  const unsigned long long hp = (unsigned long long)p << (bN + bL);
  const HeadKV v = kv[k];
  const unsigned long long me = lk[threadIdx.x + kGrpHalo];
  if (e - b > min(maxSmall, kGrpHalo)) {
    key[k] = hp | me;
    perm[k] = v.idx;  // (tonext / smaller of these follow the radix sort: k_grp_big_fields)
    if (k == b) bigList[1 + atomicAdd(bigList, 1u)] = p;
    return;
  }
  // map order; members of an item keep idx order (kv is idx-ascending per position)
  const unsigned long long mme = mk[threadIdx.x + kGrpHalo];
  uint32_t r = 0;
  for (uint32_t j = b; j < e; j++) {
    const unsigned long long mj = mk[j - base];
    r += (mj < mme || (mj == mme && j < k)) ? 1u : 0u;
  }
  key[b + r] = hp | me;
  perm[b + r] = v.idx;
  tsOut[b + r] = v.tonext;
  smOut[b + r] = (uint8_t)(v.len >> 31);
}
// Big segments come out of their radix sort in (len, isaNext, idx) order: one
// block per big position puts its members in map order (smaller=true items as
// sorted, then smaller=false items by len descending, isaNext ascending; an
// item's class from its first, lowest-idx member) through tmp at the
// segment's offset in the big list.  Destinations from one prefix count of the
// smaller=false members: an S member at t goes to t - F(t); an F member of
// the len group [gs, ge) to nS + (nF - F(ge)) + (F(t) - F(gs)).
__global__ void __launch_bounds__(256) k_grp_big_maporder(
    const uint32_t* __restrict__ bpos, uint32_t nb, const uint32_t* __restrict__ hb, const uint32_t* __restrict__ off,
    unsigned long long* __restrict__ key, uint32_t* __restrict__ perm, uint32_t* __restrict__ ts,
    uint8_t* __restrict__ sm, unsigned long long* __restrict__ tKey, uint32_t* __restrict__ tPerm,
    uint32_t* __restrict__ tTs, uint8_t* __restrict__ tSm, uint32_t* __restrict__ tF, int bN) {
  __shared__ uint32_t wsum[4];
  const uint32_t b = hb[bpos[blockIdx.x]], m = hb[bpos[blockIdx.x] + 1] - b, o = off[blockIdx.x];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t c = 0; c < m; c += 256) {
    const uint32_t t = c + threadIdx.x;
    bool f = false;
    if (t < m) {
      const unsigned long long kt = key[b + t];
      tKey[o + t] = kt; tPerm[o + t] = perm[b + t]; tTs[o + t] = ts[b + t]; tSm[o + t] = sm[b + t];
      uint32_t lo = 0, hi = t;  // first member of the item: first entry with key kt
      while (lo < hi) {
        const uint32_t md = (lo + hi) >> 1;
        if (key[b + md] < kt) lo = md + 1; else hi = md;
      }
      f = sm[b + lo] == 0;
    }
    const uint64_t bal = __ballot(f);
    if (lane == 0) wsum[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t pre = carry;
    for (uint32_t x = 0; x < wv; x++) pre += wsum[x];
    if (t < m) tF[o + t] = pre + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
    carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  const uint32_t nF = carry, nS = m - nF;
  auto F = [&](uint32_t t) { return t < m ? tF[o + t] : nF; };
  for (uint32_t t = threadIdx.x; t < m; t += 256) {
    const unsigned long long kt = tKey[o + t];
    const bool isF = F(t + 1) != F(t);
    uint32_t dst;
    if (!isF) {
      dst = t - F(t);
    } else {
      const unsigned long long g = kt >> bN;  // pos | len
      uint32_t lo = 0, hi = t;
      while (lo < hi) {
        const uint32_t md = (lo + hi) >> 1;
        if ((tKey[o + md] >> bN) < g) lo = md + 1; else hi = md;
      }
      const uint32_t gs = lo;
      lo = t + 1; hi = m;
      while (lo < hi) {
        const uint32_t md = (lo + hi) >> 1;
        if ((tKey[o + md] >> bN) <= g) lo = md + 1; else hi = md;
      }
      const uint32_t ge = lo;
      dst = nS + (nF - F(ge)) + (F(t) - F(gs));
    }
    key[b + dst] = kt; perm[b + dst] = tPerm[o + t]; ts[b + dst] = tTs[o + t]; sm[b + dst] = tSm[o + t];
  }
}
__global__ void k_grp_big_fields(const uint32_t* __restrict__ idx, uint32_t B, const uint32_t* __restrict__ perm,
                                 HeadsSoA h, uint32_t* __restrict__ tsOut, uint8_t* __restrict__ smOut) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const uint32_t k = idx[i], a = perm[k];
  tsOut[k] = h.tonext[a];
  smOut[k] = h.smaller[a];
}
// big segments: sizes, then their element indices (positions ascending)
__global__ void k_grp_big_sizes(const uint32_t* __restrict__ pos, uint32_t nb, const uint32_t* __restrict__ hb,
                                uint32_t* __restrict__ sz) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb) sz[i] = hb[pos[i] + 1] - hb[pos[i]];
}
__global__ void k_grp_big_expand(const uint32_t* __restrict__ pos, uint32_t nb, const uint32_t* __restrict__ hb,
                                 const uint32_t* __restrict__ off, uint32_t* __restrict__ idx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  const uint32_t b = hb[pos[i]], e = hb[pos[i] + 1], o = off[i];
  for (uint32_t k = b; k < e; k++) idx[o + (k - b)] = k;
}
__global__ void k_gather_kp(const uint32_t* __restrict__ idx, uint32_t B, const unsigned long long* __restrict__ key,
                            const uint32_t* __restrict__ perm, unsigned long long* __restrict__ keyB,
                            uint32_t* __restrict__ permB) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  keyB[i] = key[idx[i]];
  permB[i] = perm[idx[i]];
}
__global__ void k_scatter_kp(const uint32_t* __restrict__ idx, uint32_t B, const unsigned long long* __restrict__ keyB,
                             const uint32_t* __restrict__ permB, unsigned long long* __restrict__ key,
                             uint32_t* __restrict__ perm) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  key[idx[i]] = keyB[i];
  perm[idx[i]] = permB[i];
}

__global__ void k_item_flags64(const unsigned long long* __restrict__ key, uint32_t* __restrict__ flag, uint64_t H) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H) return;
  flag[k] = (k == 0 || key[k] != key[k - 1]) ? 1u : 0u;
}
__global__ void k_item_fill64(const unsigned long long* __restrict__ key, const uint32_t* __restrict__ perm,
                              const uint32_t* __restrict__ flag, const uint32_t* __restrict__ itemIncl, HeadsSoA h,
                              const uint32_t* __restrict__ tsS, const uint8_t* __restrict__ smS,
                              uint64_t H, int bN, int bL, ItemsSoA it) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H || !flag[k]) return;
  const uint32_t q = itemIncl[k] - 1;
  const uint32_t a = perm[k];
  const unsigned long long v = key[k];
  it.pos[q] = (uint32_t)(v >> (bN + bL));
  it.len[q] = (uint32_t)((v >> bN) & ((1ull << bL) - 1));
  it.isa[q] = (uint32_t)(v & ((1ull << bN) - 1));
  it.smaller[q] = tsS ? smS[k] : h.smaller[a];  // the first member's (sorted order: no gather)
  it.until[q] = tsS ? tsS[k] : h.tonext[a];
  it.first[q] = (uint32_t)k;
}

// One item per flagged position; the first member (smallest idx) supplies
// untilNext and smaller, as the first std::map insertion does (FN:1406-1413).
__global__ void k_item_fill(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ flag,
                            const uint32_t* __restrict__ itemIncl, HeadsSoA h, uint64_t H,
                            ItemsSoA it) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= H || !flag[k]) return;
  uint32_t q = itemIncl[k] - 1;
  uint32_t a = perm[k];
  it.pos[q] = h.pos[a];
  it.len[q] = h.len[a];
  it.isa[q] = h.isa[a];
  it.smaller[q] = h.smaller[a];
  it.until[q] = h.tonext[a];
  it.first[q] = (uint32_t)k;
}

__global__ void k_item_count(const uint32_t* __restrict__ first, uint32_t* __restrict__ count, uint32_t K,
                             uint32_t H) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  uint32_t e = q + 1 < K ? first[q + 1] : H;
  count[q] = e - first[q];
}

// gather item attributes into map order
__global__ void k_item_permute(ItemsSoA in, const uint32_t* __restrict__ order, ItemsSoA out, uint32_t K) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  uint32_t s = order[q];
  out.pos[q] = in.pos[s];
  out.len[q] = in.len[s];
  out.isa[q] = in.isa[s];
  out.smaller[q] = in.smaller[s];
  out.until[q] = in.until[s];
  out.count[q] = in.count[s];
  out.first[q] = in.first[s];
}

// posBegin[p] = first item (map order) with pos >= p, p in [0, n]
// posBegin[p] = first item at a position >= p (p = 0 .. n) from the sorted
// item positions.  Interior gaps (ipos[q-1], ipos[q]] are written by item q's
// thread, or by its whole wave when longer than 64 positions; the two end
// gaps [0, ipos[0]] and (ipos[K-1], n] -- half the positions on each rank of
// a sharded merge, whose items all sit in its own range -- by k_pos_ends, one
// thread per position (one thread writing them serially took ~68 ms per rank
// at config 3 / W = 2).
__global__ void k_pos_begin(const uint32_t* __restrict__ ipos, uint32_t K, uint32_t n,
                            uint32_t* __restrict__ posBegin) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  const bool act = q >= 1 && q < K;  // interior gaps only
  uint32_t lo = 1, hi = 0;
  if (act) {
    lo = ipos[q - 1] + 1;
    hi = ipos[q];
  }
  const bool wide = act && hi >= lo && hi - lo >= 64;
  if (act && !wide)
    for (uint32_t p = lo; p <= hi; p++) posBegin[p] = q;
  uint64_t m = __ballot(wide);
  while (m) {
    const int l = __builtin_ctzll(m);
    m &= m - 1;
    const uint32_t L = __shfl(lo, l), Hh = __shfl(hi, l), Q = __shfl(q, l);
    for (uint32_t p = L + lane; p <= Hh; p += 64) posBegin[p] = Q;
  }
}
__global__ void k_pos_ends(const uint32_t* __restrict__ ipos, uint32_t K, uint32_t n,
                           uint32_t* __restrict__ posBegin) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p > n) return;
  if (K == 0) { posBegin[p] = 0; return; }
  if (p <= ipos[0]) posBegin[p] = 0;
  else if (p > ipos[K - 1]) posBegin[p] = K;
}

// posF[p] = first smaller=false item of position p (= posBegin[p+1] if none)
__global__ void k_pos_f(const uint32_t* __restrict__ ipos, const uint8_t* __restrict__ ism,
                        const uint32_t* __restrict__ posBegin, uint32_t K, uint32_t n,
                        uint32_t* __restrict__ posF) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint32_t b = posBegin[p], e = posBegin[p + 1];
  uint32_t lo = b, hi = e;  // first item in [b, e) with smaller == 0 (T items come first)
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (ism[m]) lo = m + 1; else hi = m;
  }
  posF[p] = lo;
}

// Map-order consistency: for every position, every smaller=true item of
// length L must have isaNext below every smaller=false item of length L,
// otherwise match.h's comparator is not a strict weak order there and
// std::map's layout depends on insertion history.
__global__ void k_check_items(const ItemsSoA it, const uint32_t* __restrict__ posBegin,
                              const uint32_t* __restrict__ posF, uint32_t K,
                              unsigned long long* __restrict__ violations, uint8_t* __restrict__ amb) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K || !it.smaller[q]) return;
  uint32_t p = it.pos[q], L = it.len[q];
  uint32_t f = posF[p], e = posBegin[p + 1];
  if (q + 1 < f && it.len[q + 1] == L) return;  // only the last T item of this length
  // F part sorted by len descending: first item with len <= L
  uint32_t lo = f, hi = e;
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (it.len[m] > L) lo = m + 1; else hi = m;
  }
  if (lo < e && it.len[lo] == L && it.isa[lo] <= it.isa[q]) {
    atomicAdd(violations, 1ull);
    if (amb) amb[p] = 1;  // this position's map layout is replayed on the host
  }
}

// per SA rank: items and heads of position SA[r] (r = 0 -> position n-1 is
// accounted separately: its heads are the end phrases)
__global__ void k_sa_counts(const int32_t* __restrict__ sa, const uint32_t* __restrict__ posBegin,
                            const uint32_t* __restrict__ slot, uint32_t n, uint32_t E,
                            uint32_t* __restrict__ itemsSA, uint32_t* __restrict__ headsSA) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  if (r == 0) { itemsSA[0] = 0; headsSA[0] = E; return; }
  uint32_t p = (uint32_t)sa[r];
  uint32_t b = posBegin[p], e = posBegin[p + 1];
  itemsSA[r] = e - b;
  headsSA[r] = slot[e] - slot[b];
}




// prefix doubling: key = (group of suffix, group of suffix + h)
__global__ void k_dbl_keys(const uint32_t* __restrict__ act, const uint32_t* __restrict__ sa,
                           const uint32_t* __restrict__ grp, uint32_t h, uint32_t U,
                           uint64_t* __restrict__ key, uint32_t* __restrict__ val, uint32_t saMask) {
  uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  uint32_t idx = sa[act[u]] & saMask;  // (k_ranks_slot's unresolved flag cleared)
  key[u] = ((uint64_t)grp[idx] << 32) | grp[idx + h];
  val[u] = idx;
}

// write the sorted members back and compute the new group starts
__global__ void k_dbl_apply(const uint32_t* __restrict__ act, const uint64_t* __restrict__ key,
                            const uint32_t* __restrict__ val, uint32_t U, uint32_t* __restrict__ sa,
                            uint32_t* __restrict__ lab) {
  uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  sa[act[u]] = val[u];
  lab[u] = (u == 0 || key[u] != key[u - 1]) ? act[u] : 0u;
}

// grp update + which members stay unresolved (their new group has >= 2 members)
__global__ void k_dbl_groups(const uint32_t* __restrict__ act, const uint64_t* __restrict__ key,
                             const uint32_t* __restrict__ val, const uint32_t* __restrict__ labMax,
                             uint32_t U, uint32_t* __restrict__ grp, uint32_t* __restrict__ keep) {
  uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  grp[val[u]] = labMax[u];
  bool startHere = (u == 0 || key[u] != key[u - 1]);
  bool endHere = (u + 1 == U || key[u + 1] != key[u]);
  keep[u] = (startHere && endHere) ? 0u : 1u;
}

// ---- map order
// map order of one position's items (sorted by (len, isaNext)): smaller=true
// items in that order, then smaller=false items by len descending, isaNext
// ascending for equal len (match.h:27-33 on consistent data)
__global__ void k_map_order(const uint32_t* __restrict__ posBegin, const uint32_t* __restrict__ len,
                            const uint8_t* __restrict__ sm, uint32_t n, uint32_t* __restrict__ order) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t b = posBegin[p], e = posBegin[p + 1];
  if (b == e) return;
  uint32_t w = b;
  for (uint32_t q = b; q < e; q++)
    if (sm[q]) order[w++] = q;
  uint32_t ge = e;
  while (ge > b) {
    const uint32_t L = len[ge - 1];
    uint32_t gs = ge - 1;
    while (gs > b && len[gs - 1] == L) gs--;
    for (uint32_t q = gs; q < ge; q++)
      if (!sm[q]) order[w++] = q;
    ge = gs;
  }
}

// ---- per-group doubling round.  Keys are in act order and a group is a run
// of equal high words (its label), so each group is a contiguous range: small
// groups are sorted by one thread each, large ones go through a radix sort.
__global__ void k_dbl_gstart(const uint64_t* __restrict__ key, uint32_t U, uint32_t* __restrict__ flag) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < U) flag[u] = (u == 0 || (key[u] >> 32) != (key[u - 1] >> 32)) ? 1u : 0u;
}
// Unresolved members (items with >= 2 heads, end phrases excluded) in sa
// position order, without a sort: per position p its count at rank ISA[p],
// then each position writes its members' sa positions at its rank's offset.
// Group leaders (gflag) sort their group when it has <= maxSmall members;
// members of larger groups are appended to bigList (group by group) for the
// radix path (bigList[0] counts them).
// One thread per unresolved member (act order): its group (a run of equal
// labels = key high words, <= kDblHalo members, found in an LDS copy of the
// keys around the block) is ranked by counting, as k_grp_seg does.  Member u
// moves to sa position act[u0 + rank] (rank by (key, u)), its new label is
// act[u0 + #smaller keys], and it stays unresolved when another member has
// its key.  Members of longer groups are listed for the radix path.
constexpr uint32_t kDblBlock = 256, kDblHalo = 64;
__global__ void __launch_bounds__(256) k_dbl_rank(uint32_t U, const uint32_t* __restrict__ act,
                                                  const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                  uint32_t* __restrict__ sa, uint32_t* __restrict__ grp,
                                                  uint32_t* __restrict__ keep, uint32_t* __restrict__ bigList,
                                                  uint32_t maxSmall) {
  __shared__ uint64_t kL[kDblBlock + 2 * kDblHalo];
  __shared__ uint32_t aL[kDblBlock + 2 * kDblHalo];
  const uint32_t k0 = blockIdx.x * kDblBlock;
  const int64_t base = (int64_t)k0 - kDblHalo;
  for (uint32_t i = threadIdx.x; i < kDblBlock + 2 * kDblHalo; i += blockDim.x) {
    const int64_t j = base + i;
    if (j >= 0 && j < (int64_t)U) { kL[i] = key[j]; aL[i] = act[j]; }
  }
  __syncthreads();
  const uint32_t u = k0 + threadIdx.x;
  if (u >= U) return;
  const uint32_t me = threadIdx.x + kDblHalo;
  const uint64_t kk = kL[me];
  const uint32_t lab = (uint32_t)(kk >> 32);
  const uint32_t lim = min(maxSmall, kDblHalo - 1);
  // group bounds [lo, hi) within lim + 1 steps either side
  uint32_t lo = me, hi = me + 1;
  while (lo > 0 && base + lo > 0 && (uint32_t)(kL[lo - 1] >> 32) == lab && me - lo <= lim) lo--;
  while (hi < kDblBlock + 2 * kDblHalo && base + hi < (int64_t)U && (uint32_t)(kL[hi] >> 32) == lab &&
         hi - me <= lim)
    hi++;
  if (hi - lo > lim) {  // a long group: radix path (wave-aggregated list append)
    const uint64_t bm = __ballot(true);
    const uint32_t lead = __builtin_amdgcn_readfirstlane((uint32_t)__builtin_ctzll(bm));
    uint32_t o = 0;
    if ((threadIdx.x & 63) == lead) o = atomicAdd(bigList, (uint32_t)__popcll(bm));
    o = __shfl(o, (int)lead);
    const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    bigList[1 + o + rk] = u;
    return;
  }
  uint32_t r = 0, rs = 0, eq = 0;
  for (uint32_t j = lo; j < hi; j++) {
    const uint64_t kj = kL[j];
    r += (kj < kk || (kj == kk && j < me)) ? 1u : 0u;
    rs += kj < kk ? 1u : 0u;
    eq += kj == kk ? 1u : 0u;
  }
  const uint32_t v = val[u];
  if (lo + r != me) sa[aL[lo + r]] = v;  // moved by the sort
  if (rs != 0) grp[v] = aL[lo + rs];     // a later part of the group: new label
  // keep is indexed by act position (the member's new sa position): still
  // unresolved while another member has its key
  keep[(uint32_t)(base + lo + r)] = eq > 1 ? 1u : 0u;
}
__global__ void k_dbl_small2(const uint32_t* __restrict__ gflag, uint32_t U, const uint32_t* __restrict__ act,
                             uint64_t* __restrict__ key, uint32_t* __restrict__ val, uint32_t* __restrict__ sa,
                             uint32_t* __restrict__ grp, uint32_t* __restrict__ keep, uint32_t* __restrict__ bigList,
                             uint32_t maxSmall) {
  const uint32_t u0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (u0 >= U || !gflag[u0]) return;
  uint32_t u1 = u0 + 1;
  while (u1 < U && !gflag[u1]) u1++;
  if (u1 - u0 > maxSmall) {
    const uint32_t o = atomicAdd(bigList, u1 - u0);
    for (uint32_t u = u0; u < u1; u++) bigList[1 + o + (u - u0)] = u;
    return;
  }
  // Only changed entries are written: a member keeps its label (the group's
  // first sa position) when it stays in the group's first part, and its sa
  // entry when the sort did not move it (grp writes are random 4-byte stores).
  if (u1 - u0 <= 4) {  // the common case: a sorting network in registers
    uint64_t k[4];
    uint32_t v[4], a4[4], vo[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const bool in = u0 + j < u1;
      k[j] = in ? key[u0 + j] : ~0ull;
      v[j] = in ? val[u0 + j] : 0u;
      a4[j] = in ? act[u0 + j] : 0u;
      vo[j] = v[j];
    }
    auto cs = [&](int x, int y) {
      if (k[y] < k[x]) {
        const uint64_t tk = k[x]; k[x] = k[y]; k[y] = tk;
        const uint32_t tv = v[x]; v[x] = v[y]; v[y] = tv;
      }
    };
    cs(0, 1); cs(2, 3); cs(0, 2); cs(1, 3); cs(1, 2);
    // (equal keys stay in one group: their order is settled by later rounds)
    uint32_t rs = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      if (u0 + j < u1) {
        if (j > 0 && k[j] != k[j - 1]) rs = j;
        const bool endRun = u0 + j + 1 == u1 || k[j + 1 < 4 ? j + 1 : 3] != k[j];
        if (v[j] != vo[j]) sa[a4[j]] = v[j];
        if (rs != 0) grp[v[j]] = a4[rs];
        keep[u0 + j] = (rs == j && endRun) ? 0u : 1u;
      }
    }
    return;
  }
  for (uint32_t a = u0 + 1; a < u1; a++) {  // insertion sort by (label, label of suffix + h)
    const uint64_t kk = key[a];
    const uint32_t vv = val[a];
    uint32_t b = a;
    while (b > u0 && key[b - 1] > kk) {
      key[b] = key[b - 1];
      val[b] = val[b - 1];
      b--;
    }
    key[b] = kk;
    val[b] = vv;
  }
  uint32_t rs = u0;
  for (uint32_t u = u0; u < u1; u++) {
    if (u > u0 && key[u] != key[u - 1]) rs = u;
    const bool endRun = u + 1 == u1 || key[u + 1] != key[u];
    sa[act[u]] = val[u];
    if (rs != u0) grp[val[u]] = act[rs];
    keep[u] = (rs == u && endRun) ? 0u : 1u;
  }
}

__global__ void k_dbl_gather_big(const uint32_t* __restrict__ orig, uint32_t B, const uint32_t* __restrict__ act,
                                 const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                 uint32_t* __restrict__ actB, uint64_t* __restrict__ keyB, uint32_t* __restrict__ valB) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t u = orig[b];
  actB[b] = act[u];
  keyB[b] = key[u];
  valB[b] = val[u];
}
__global__ void k_scatter_u32(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx, uint32_t n,
                              uint32_t* __restrict__ dst) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < n) dst[idx[b]] = src[b];
}



// ---- slot-major members (one thread per head, no per-item loops)
// mark[slot[q]] = 1 for q >= 1; its inclusive scan is the item of each slot
__global__ void k_slot_mark(const uint32_t* __restrict__ slot, uint32_t K, uint32_t* __restrict__ mark) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= 1 && q < K) mark[slot[q]] = 1;
}
// Pm[s] = idx of the member of slot s (members of an item in idx order)
__global__ void k_slot_members(const ItemsSoA it, const uint32_t* __restrict__ itemOfSlot,
                               const uint32_t* __restrict__ perm, uint32_t H, uint32_t* __restrict__ Pm) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= H) return;
  const uint32_t q = itemOfSlot[s];
  Pm[s] = perm[it.first[q] + (s - it.slot[q])];
}
// Ranks of FN:1432-1453 and the initial (first-symbol) order of the head
// string for the suffix sort (FN:1455-1459), one thread per member.
// Per position (mod 2^32): rank(q) = rankBase[p] + q, group g(q) = gBase[p] +
// slot[q] for the items q of p (their SA-rank prefix sums, FN:1436-1449).
__global__ void k_pos_rank_base(const uint32_t* __restrict__ posBegin, const uint32_t* __restrict__ slot,
                                const uint32_t* __restrict__ isaRef, const uint32_t* __restrict__ itemRankBase,
                                const uint32_t* __restrict__ headBase, uint32_t n, uint32_t E,
                                uint32_t* __restrict__ rankBase, uint32_t* __restrict__ gBase) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t b = posBegin[p];
  if (b == posBegin[p + 1]) return;  // no items here
  const uint32_t r = isaRef[p];
  if (rankBase) rankBase[p] = E + 2 + itemRankBase[r] - b;
  gBase[p] = 1 + headBase[r] - slot[b];
}
__global__ void k_ranks_slot(const ItemsSoA it, const uint32_t* __restrict__ itemOfSlot,
                             const uint32_t* __restrict__ Pm, uint32_t H, const uint32_t* __restrict__ rankBase,
                             const uint32_t* __restrict__ gBase, uint32_t n, int32_t* __restrict__ T,
                             uint32_t* __restrict__ sa, uint32_t* __restrict__ grp, uint32_t* __restrict__ actv,
                             uint32_t* __restrict__ gItem, uint8_t* __restrict__ unres, uint32_t saFlag) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= H) return;
  if (unres && s == 0) unres[0] = 0;  // sa position 0: the sentinel
  const uint32_t q = itemOfSlot[s], idx = Pm[s];
  const uint32_t sq = it.slot[q], m = s - sq, p = it.pos[q];
  if (p == n - 1) {  // end phrases: one rank each, in document order
    if (T) T[idx] = (int32_t)(1 + m);
    sa[1 + m] = idx;
    grp[idx] = 1 + m;
    if (actv) actv[s] = 0xffffffffu;
    if (unres) unres[1 + m] = 0;
    if (gItem && m == 0) gItem[q] = 1;
    return;
  }
  const uint32_t g = gBase[p] + sq;
  // the item's members hold the sa positions g .. g + count - 1: its first
  // head rank is g - 1 whatever the suffix sort does inside it
  if (gItem && m == 0) gItem[q] = g;
  if (T) T[idx] = (int32_t)(rankBase[p] + q);  // rank2head: kept for parity copies only
  // unresolved members (items with >= 2 heads): their sa positions, flagged
  // in bit 31 of the sa entry (saFlag, H < 2^31) or in a byte per position
  const bool ur = it.count[q] >= 2;
  sa[g + m] = idx | (ur ? saFlag : 0u);
  grp[idx] = g;
  if (actv) actv[s] = ur ? g + m : 0xffffffffu;
  if (unres) unres[g + m] = ur ? 1 : 0;
}
// next-head rank of each member, in slot order (FN:1480-1494): first per head
// in document order (nexthead is small, so headRank[idx + nexthead] is read
// almost sequentially), then one gather through the slot permutation
__global__ void k_nhr_idx(const uint32_t* __restrict__ headRank, uint32_t sub, const uint16_t* __restrict__ nexthead,
                          uint32_t H, uint32_t* __restrict__ nbi) {
  uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= H) return;
  nbi[idx] = headRank[idx + nexthead[idx]] - sub;
}
// the character before each head at its slot in head-rank order (the
// CMSBWT_NHR_SORT=1 path; the default places them inside k_nhr_rank)
__global__ void k_head_chars_slot(const uint32_t* __restrict__ Pm, const uint32_t* __restrict__ grp,
                                  const uint8_t* __restrict__ lchar, const ItemsSoA it,
                                  const uint32_t* __restrict__ itemOfSlot, const uint32_t* __restrict__ gItem,
                                  uint32_t H, uint8_t* __restrict__ bwtSlot) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= H) return;
  const uint32_t idx = Pm[s], q = itemOfSlot[s];
  bwtSlot[it.slot[q] + grp[idx] - gItem[q]] = lchar[idx];
}
// per head in document order: (next-head rank, head rank, BWT character) for
// k_nhr_rank's one gather per slot (the character then lands at its slot in
// head-rank order, where the writer reads it; no BWTheads gather by rank)
__global__ void k_nhr_rec(const uint32_t* __restrict__ grp, const uint16_t* __restrict__ nexthead,
                          const uint8_t* __restrict__ lchar, uint32_t H, uint4* __restrict__ rec) {
  uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= H) return;
  rec[idx] = make_uint4(grp[idx + nexthead[idx]] - 1, grp[idx] - 1, lchar[idx], 0u);
}
// BWTheads (FN:1471): the character before each head, in head-rank order
__global__ void k_head_chars(const uint32_t* __restrict__ sa, const uint8_t* __restrict__ lchar, uint32_t H,
                             uint8_t* __restrict__ bwtHeads) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < H) bwtHeads[r] = lchar[sa[r + 1]];
}
__global__ void k_nhr_slot(const uint32_t* __restrict__ Pm, const uint32_t* __restrict__ nbi, uint32_t H,
                           uint32_t* __restrict__ nhr) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= H) return;
  nhr[s] = nbi[Pm[s]];
}
// Sort each item's nhr segment: insertion sort in place for <= kSmallSeg
// members; larger items are appended to a list (bigList[0] = their number)
// for one global sort of their members.
constexpr uint32_t kSmallSeg = 32;
// FN:1480-1494 fused: one thread per slot gathers its member's next-head
// rank (nbi, in document order) and ranks it inside its item by counting
// over an LDS copy of the block's slots with a halo (items of <= kSmallSeg
// members, the rest keep their order here and are sorted by the big path).
// Writes the item's members' ranks sorted (std::sort of idxs, FN:1492).
constexpr uint32_t kNhrBlock = 256, kNhrHalo = kSmallSeg + 1;  // the scans go kSmallSeg + 1 slots either way
__global__ void __launch_bounds__(kNhrBlock) k_nhr_rank(const uint32_t* __restrict__ Pm, const uint32_t* __restrict__ nbi,
                                                  const uint32_t* __restrict__ itemOfSlot, uint32_t H,
                                                  uint32_t* __restrict__ nhr, const uint4* __restrict__ rec,
                                                  const uint32_t* __restrict__ slot, const uint32_t* __restrict__ gItem,
                                                  uint8_t* __restrict__ bwtSlot) {
  __shared__ uint32_t vL[kNhrBlock + 2 * kNhrHalo], qL2[kNhrBlock + 2 * kNhrHalo];
  const uint32_t s0 = blockIdx.x * kNhrBlock;
  const int64_t base = (int64_t)s0 - kNhrHalo;
  // rec (one GPU): each block's own slots also place their head's character at
  // slot[q] + rank - first rank of the item (FN:1468-1472)
  for (uint32_t i = threadIdx.x; i < kNhrBlock + 2 * kNhrHalo; i += blockDim.x) {
    const int64_t j = base + i;
    if (j >= 0 && j < (int64_t)H) {
      const uint32_t q = itemOfSlot[j];
      qL2[i] = q;
      if (rec) {
        const uint4 w = rec[Pm[j]];
        vL[i] = w.x;
        if (i >= kNhrHalo && i < kNhrHalo + kNhrBlock) bwtSlot[slot[q] + w.y - (gItem[q] - 1)] = (uint8_t)w.z;
      } else {
        vL[i] = nbi[Pm ? Pm[j] : (uint32_t)j];
      }
    }
  }
  __syncthreads();
  const uint32_t s = s0 + threadIdx.x;
  if (s >= H) return;
  const uint32_t me = threadIdx.x + kNhrHalo, q = qL2[me], v = vL[me];
  uint32_t lo = me, hi = me + 1;
  while (lo > 0 && base + lo > 0 && qL2[lo - 1] == q && me - lo <= kSmallSeg) lo--;
  while (hi < kNhrBlock + 2 * kNhrHalo && base + hi < (int64_t)H && qL2[hi] == q && hi - me <= kSmallSeg) hi++;
  if (hi - lo > kSmallSeg) { nhr[s] = v; return; }  // a long item: the big path sorts it
  uint32_t r = 0;
  for (uint32_t j = lo; j < hi; j++) {
    const uint32_t w = vL[j];
    r += (w < v || (w == v && j < me)) ? 1u : 0u;
  }
  nhr[(uint32_t)(base + lo + r)] = v;
}
__global__ void k_nhr_sort_small(const ItemsSoA it, uint32_t K, uint32_t* __restrict__ nhr,
                                 uint32_t* __restrict__ bigList) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  const uint32_t c = it.count[q];
  if (c > kSmallSeg) bigList[1 + atomicAdd(bigList, 1u)] = q;
  if (c < 2 || c > kSmallSeg) return;
  uint32_t* a = nhr + it.slot[q];
  for (uint32_t x = 1; x < c; x++) {
    const uint32_t v = a[x];
    uint32_t y = x;
    while (y > 0 && a[y - 1] > v) { a[y] = a[y - 1]; y--; }
    a[y] = v;
  }
}
// keys (item, nhr) and slots of the members of the large items (list sorted
// by item, members at the exclusive offsets of their counts): one block per item
__global__ void k_nhr_big_fill(const uint32_t* __restrict__ items, const uint32_t* __restrict__ off,
                               const ItemsSoA it, const uint32_t* __restrict__ nhr,
                               unsigned long long* __restrict__ key, uint32_t* __restrict__ slots) {
  const uint32_t q = items[blockIdx.x], o = off[blockIdx.x], s0 = it.slot[q], c = it.count[q];
  for (uint32_t m = threadIdx.x; m < c; m += blockDim.x) {
    key[o + m] = ((unsigned long long)q << 32) | nhr[s0 + m];
    slots[o + m] = s0 + m;
  }
}
__global__ void k_item_counts_of(const uint32_t* __restrict__ items, uint32_t nb, const uint32_t* __restrict__ count,
                                 uint32_t* __restrict__ out) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < nb) out[b] = count[items[b]];
}
__global__ void k_nhr_big_back(const unsigned long long* __restrict__ sorted, const uint32_t* __restrict__ slots,
                               uint32_t B, uint32_t* __restrict__ nhr) {
  uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < B) nhr[slots[u]] = (uint32_t)sorted[u];
}


// ------------------------------------------------------------ counterSmallerThanHead
// FN:1523-1603.  Work unit (item q, target t = pos+1+k, k < untilNext): the
// non-head suffixes k+1 positions after the item's heads are placed among the
// items of position t with std::map::lower_bound semantics.
//
// Target-major: reference positions are cut into windows whose slots fit in
// LDS.  A block owns one window; the items that reach into it are the items
// starting inside it plus a precomputed crossing list.  One wave per item,
// lanes over consecutive targets; every counter update lands in LDS, and the
// block stores each slot of its window once (no global atomics).  Windows
// whose slots exceed the LDS budget fall back to global u64 atomics.
//
// Items of a position are in map order: smaller=true keys by (len, isa)
// ascending, then smaller=false keys by (~len, isa) ascending, so each class
// is sorted by one 64-bit search key sk and `item < query` is `sk < qk`
// inside the query's class.  CHECK adds the ambiguity tests of DESIGN.md §5
// (only needed when k_finalize's order invariant failed).
constexpr uint32_t kWinSlots = 3584;  // slot cap of an LDS window (see kWinItems)

struct CounterArgs {
  ItemsSoA it;
  const uint32_t* posBegin;
  const uint32_t* posF;
  const uint32_t* nhr;       // sorted next-head ranks, slot order
  const uint32_t* winStart;  // nw + 1
  const uint32_t* crossOff;  // nw + 1
  const uint32_t* crossList;
  unsigned long long* counter;
  unsigned long long* stats; // bad, good, nothing, violations, errors, searched, ambiguous queries
  uint32_t n;
  uint32_t slotCap;          // windows with more slots use global atomics
  HostRoute hr;              // CHECK only: targets answered by the host std::map replay
  EqList eq;                 // k_counter_tgt before the next-head ranks: equal-key queries listed
  const uint4* irec;         // k_counter_tgt: (pos, until, len, count | smaller << 31) per item, or null
};

struct QueryStats {  // per lane; a lane serves far fewer than 2^32 queries per window
  uint32_t bad = 0, good = 0, nothing = 0, viol = 0, slow = 0;
};

__device__ __forceinline__ uint32_t d_upper_u32(const uint32_t* a, uint32_t lo, uint32_t hi, uint32_t v) {
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (a[m] <= v) lo = m + 1; else hi = m;
  }
  return lo;
}

__device__ __forceinline__ uint32_t d_lower_u64(const unsigned long long* a, uint32_t lo, uint32_t hi,
                                                unsigned long long v) {
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1; else hi = m;
  }
  return lo;
}

// Query of one (item, target) pair.  ql/qi/qs/cq/slq: the item's len, isa,
// smaller, count and slot (wave-uniform).  V gives the target's items and
// positions either from LDS (staged window) or from global memory.
template <bool CHECK, class View, class AddFn>
__device__ __forceinline__ void d_counter_query_L(const View& V, uint32_t L, uint32_t qi, bool S, uint32_t cq,
                                                  uint32_t slq, uint32_t t, QueryStats& qs, AddFn add,
                                                  const HostRoute* hr = nullptr, const EqList* eql = nullptr) {
  const uint32_t b0 = V.begin(t), b1 = V.begin(t + 1);
  if (b0 == b1) { qs.nothing++; return; }  // bucket >= 0: no heads at t (FN:1530)
  if (CHECK && hr->mask[t]) {  // answered by the host's std::map replay of t
    const unsigned long long e = atomicAdd(hr->cnt, 1ull);
    if (e < hr->cap) {
      hr->list[2 * e] = slq;
      hr->list[2 * e + 1] = t;
    }
    return;
  }
  const uint32_t f = V.fbeg(t);
  const unsigned long long kT = ((unsigned long long)L << 32) | qi;
  const unsigned long long kF = ((unsigned long long)(~L) << 32) | qi;
  auto lower = [&](uint32_t lo, uint32_t hi, unsigned long long v) {
    while (lo < hi) {
      uint32_t m = (lo + hi) >> 1;
      if (V.sk(m) < v) lo = m + 1; else hi = m;
    }
    return lo;
  };
  uint32_t ans;
  if (S) {
    ans = lower(b0, f, kT);
    if (CHECK) {  // an F item with len == L and isa < I breaks monotonicity
      uint32_t l3 = lower(f, b1, (unsigned long long)(~L) << 32);
      if (l3 < b1 && (uint32_t)~(V.sk(l3) >> 32) == L && (uint32_t)V.sk(l3) < qi) {
        qs.viol++;
        hr->amb[t] = 1;
      }
    }
  } else {
    if (CHECK) {  // a T item with len == L and isa >= I breaks monotonicity
      uint32_t l3 = (unsigned long long)L + 1 > 0xffffffffull ? f
                                                              : lower(b0, f, (unsigned long long)(L + 1u) << 32);
      if (l3 > b0 && (uint32_t)(V.sk(l3 - 1) >> 32) == L && (uint32_t)V.sk(l3 - 1) >= qi) {
        qs.viol++;
        hr->amb[t] = 1;
      }
    }
    ans = lower(f, b1, kF);
  }
  if (ans >= b1) return;  // lower_bound == end(): FN:1535-1536
  const unsigned long long ka = V.sk(ans);
  const bool eq = ka == (ans < f ? kT : kF);  // MatchInSet::operator== (len, isaNext)
  const uint32_t so = V.slot(ans);
  if (eq) {  // same key: FN:1537-1589
    const uint32_t co = V.slot(ans + 1) - so;
    const bool hasNext = ans + 1 < b1;
    if (eql) {  // the next-head ranks do not exist yet: listed for k_counter_eq
      // one atomic per wave for the lanes listing here (a single counter
      // takes every listing of the grid)
      const uint64_t am = __ballot(1);
      const uint32_t lane = __lane_id(), leader = (uint32_t)__builtin_ctzll(am);
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(eql->cnt, (unsigned long long)__popcll(am));
      base = ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(base >> 32), leader) << 32) |
             __builtin_amdgcn_readlane((uint32_t)base, leader);
      const unsigned long long e =
          base + __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
      if ((co | cq) >> 31) atomicAdd(eql->cnt, eql->cap + 1);  // not representable: overflow
      else if (e < eql->cap) eql->rec[e] = make_uint4(slq, cq, so, co | (hasNext ? 0x80000000u : 0u));
      return;
    }
    const uint32_t* me = V.nhr + slq;
    const uint32_t* ot = V.nhr + so;
    if (me[cq - 1] < ot[0]) {
      add(so, cq);
      qs.good++;
    } else if (me[0] > ot[co - 1]) {
      if (hasNext) add(so + co, cq);
      qs.good++;
    } else {
      qs.bad++;
      uint32_t rest = 0;
      for (uint32_t a = 0; a < cq; a++) {
        uint32_t bpos = d_upper_u32(ot, 0, co, me[a]);
        if (bpos < co) add(so + bpos, 1u);
        else rest++;
      }
      if (rest && hasNext) add(so + co, rest);
    }
  } else {
    add(so, cq);
    qs.good++;
  }
}
template <bool CHECK, class View, class AddFn>
__device__ __forceinline__ void d_counter_query(const View& V, uint32_t ql, uint32_t qi, bool S, uint32_t cq,
                                                uint32_t slq, uint32_t k, uint32_t t, QueryStats& qs,
                                                AddFn add, const HostRoute* hr = nullptr) {
  d_counter_query_L<CHECK>(V, ql - 1 - k, qi, S, cq, slq, t, qs, add, hr);  // uint32 wrap as FN:1532
}

// item/position views: global memory, or the block's staged window in LDS
struct GlobalView {
  const ItemsSoA* it;
  const uint32_t* pb;
  const uint32_t* pf;
  const uint32_t* nhr;
  __device__ uint32_t begin(uint32_t t) const { return pb[t]; }
  __device__ uint32_t fbeg(uint32_t t) const { return pf[t]; }
  __device__ unsigned long long sk(uint32_t q) const { return it->sk[q]; }
  __device__ uint32_t slot(uint32_t q) const { return it->slot[q]; }
};
// GlobalView with the query target's item range already known (passed from
// the lane that owns the target): no posBegin / posF loads in the search
struct KnownView {
  const ItemsSoA* it;
  const uint32_t* nhr;
  uint32_t t0, b0, b1, f;
  __device__ uint32_t begin(uint32_t t) const { return t == t0 ? b0 : b1; }
  __device__ uint32_t fbeg(uint32_t) const { return f; }
  __device__ unsigned long long sk(uint32_t q) const { return it->sk[q]; }
  __device__ uint32_t slot(uint32_t q) const { return it->slot[q]; }
};
struct LdsView {  // items and positions rebased to the window
  const unsigned long long* skL;
  const uint32_t* slotL;
  const uint32_t* pbL;
  const uint4* fastL;
  const uint32_t* nhr;
  uint32_t iBeg, T0;
  __device__ uint32_t begin(uint32_t t) const { return pbL[t - T0] ; }
  __device__ uint32_t fbeg(uint32_t t) const { return pbL[t - T0] + ((fastL[t - T0].x >> 16) & 0x1fffu); }
  __device__ unsigned long long sk(uint32_t q) const { return skL[q - iBeg]; }
  __device__ uint32_t slot(uint32_t q) const { return slotL[q - iBeg]; }
};

constexpr uint32_t kWinItems = kWinSlots;  // staged items (= max slots) per window
constexpr uint32_t kWinPositions = 1024;
constexpr uint32_t kFsEnd = 0x40000000u, kFsSearch = 0x40000001u;

template <bool CHECK>
__global__ void __launch_bounds__(512) k_counter_win(CounterArgs A) {
  __shared__ uint32_t cnt[kWinItems + 64];              // 14 KB (+ one dummy per lane); per target the adds sum to <= H < 2^31
  __shared__ unsigned long long skL[kWinItems];         // 28 KB
  __shared__ uint32_t slotL[kWinItems + 1];             // 14 KB
  // per target: its first item (pbL) and the fast-test record fastL:
  //   x: bit 31 no items, bit 30 no smaller=false item, bit 29 no second
  //      smaller=false item, bits 0..11 the first smaller=false item's slot
  //      (window-relative), bits 16..28 its offset from the first item
  //   y: the two longest smaller=true lens (the last two S items: bits 0..15
  //      longest, 16..31 second), 0xffff: that long or longer
  //   z: the two longest smaller=false lens (the first two F items: bits 0..15
  //      first, 16..31 second)
  //   w: slots (window-relative) of the last S item (bits 0..11) and of the
  //      second F item (bits 16..27)
  __shared__ uint32_t pbL[kWinPositions + 1];                       // 4 KB
  __shared__ uint4 fastL[kWinPositions];                            // 16 KB
  __shared__ uint32_t qL[8][64];                                     // 2 KB: per-wave query queues
  __shared__ uint32_t s_next;
  __shared__ unsigned long long red[6];
  const ItemsSoA& it = A.it;
  const uint32_t w = blockIdx.x;
  const uint32_t T0 = A.winStart[w], T1 = A.winStart[w + 1];
  const uint32_t iBeg = A.posBegin[T0], iEnd = A.posBegin[T1];
  const uint32_t sb = it.slot[iBeg], se = it.slot[iEnd];
  const uint32_t nslot = se - sb;
  const bool lds = nslot <= A.slotCap && T1 - T0 <= kWinPositions;
  if (lds) {
    for (uint32_t i = threadIdx.x; i < nslot; i += blockDim.x) cnt[i] = 0;
    for (uint32_t i = threadIdx.x; i < iEnd - iBeg; i += blockDim.x) skL[i] = it.sk[iBeg + i];
    for (uint32_t i = threadIdx.x; i <= iEnd - iBeg; i += blockDim.x) slotL[i] = it.slot[iBeg + i];
    for (uint32_t i = threadIdx.x; i <= T1 - T0; i += blockDim.x) pbL[i] = A.posBegin[T0 + i];
  }
  if (threadIdx.x == 0) s_next = 0;
  if (threadIdx.x < 6) red[threadIdx.x] = 0;
  __syncthreads();
  if (lds) {
    for (uint32_t t = threadIdx.x; t < T1 - T0; t += blockDim.x) {
      const uint32_t b0 = pbL[t] - iBeg, b1 = pbL[t + 1] - iBeg, f = A.posF[T0 + t] - iBeg;
      // S items ascend by len, F items descend: the class maxima are the
      // last S items and the first F items
      auto sat = [](uint32_t v) { return min(v, 0xffffu); };
      const uint32_t mS = f > b0 ? sat((uint32_t)(skL[f - 1] >> 32)) : 0u;
      const uint32_t mS2 = f > b0 + 1 ? sat((uint32_t)(skL[f - 2] >> 32)) : 0u;
      const uint32_t mF = f < b1 ? sat(~(uint32_t)(skL[f] >> 32)) : 0u;
      const uint32_t mF2 = f + 1 < b1 ? sat(~(uint32_t)(skL[f + 1] >> 32)) : 0u;
      const uint32_t x = (b0 == b1 ? 0x80000000u : 0u) | (f < b1 ? slotL[f] - sb : 0x40000000u) |
                         (f + 1 < b1 ? 0u : 0x20000000u) | ((f - b0) << 16);
      const uint32_t wv2 = (f > b0 ? slotL[f - 1] - sb : 0u) | (f + 1 < b1 ? (slotL[f + 1] - sb) << 16 : 0u);
      fastL[t] = make_uint4(x, mS | (mS2 << 16), mF | (mF2 << 16), wv2);
    }
    __syncthreads();
  }
  const uint32_t c0 = A.crossOff[w];
  const uint32_t nCross = A.crossOff[w + 1] - c0;
  const uint32_t nItems = nCross + (iEnd - iBeg);
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  QueryStats qs;
  const LdsView LV{skL, slotL, pbL, fastL, A.nhr, iBeg, T0};
  const GlobalView GV{&A.it, A.posBegin, A.posF, A.nhr};
  auto addLds = [&](uint32_t s, uint32_t v) { atomicAdd(&cnt[s - sb], v); };
  auto addGlb = [&](uint32_t s, uint32_t v) { atomicAdd(&A.counter[s], (unsigned long long)v); };
  // Items are claimed 64 at a time: lane b loads item b's fields with one
  // coalesced load per field, then the wave walks the batch reading them with
  // readlane (no memory latency per item).
  while (true) {
    uint32_t j0 = 0;
    if (lane == 0) j0 = atomicAdd(&s_next, 64u);
    j0 = __builtin_amdgcn_readfirstlane(__shfl(j0, 0));
    if (j0 >= nItems) break;
    const uint32_t nb = min(64u, nItems - j0);
    uint32_t bp = 0, bu = 0, bl = 0, bi = 0, bc = 0, bs = 0, bS = 0;
    if (lane < nb) {
      const uint32_t j = j0 + lane;
      const uint32_t q = j < nCross ? A.crossList[c0 + j] : iBeg + (j - nCross);
      bp = it.pos[q];
      bu = it.until[q];
      bl = it.len[q];
      bi = it.isa[q];
      bc = it.count[q];
      bs = it.slot[q];
      bS = it.smaller[q];
    }
    // queries the fast test cannot settle wait in the wave's queue and run
    // 64 at a time (item fields by bpermute), so the binary searches do not
    // diverge against the cheap lanes
    uint32_t qn = 0;
    auto drain = [&](uint32_t cntq) {
      __builtin_amdgcn_wave_barrier();
      const uint32_t en = lane < cntq ? qL[wv][lane] : 0u;
      const int e = (int)(en & 63u);
      const uint32_t p = __shfl(bp, e), ql = __shfl(bl, e), qi = __shfl(bi, e);
      const uint32_t cq = __shfl(bc, e), slq = __shfl(bs, e), sS = __shfl(bS, e);
      __builtin_amdgcn_wave_barrier();
      if (lane < cntq) {
        qs.slow++;
        const uint32_t t = T0 + (en >> 6);
        d_counter_query<false>(LV, ql, qi, sS != 0, cq, slq, t - p - 1, t, qs, addLds);
      }
    };
    if (lds && !CHECK) {
      for (uint32_t e = 0; e < nb; e++) {
        const uint32_t u = __builtin_amdgcn_readlane(bu, e);
        if (!u) continue;
        const uint32_t p = __builtin_amdgcn_readlane(bp, e);
        const uint32_t ql = __builtin_amdgcn_readlane(bl, e), cq = __builtin_amdgcn_readlane(bc, e);
        const bool S = __builtin_amdgcn_readlane(bS, e) != 0;
        // targets p+1 .. p+u inside [T0, T1) (positions < 2^31: 32-bit is exact)
        const uint32_t lo = max(p + 1, T0);
        const uint32_t hi = (uint32_t)min((uint64_t)p + u, (uint64_t)T1 - 1);
        // the query len at t is ql - 1 - (t - p - 1) = E - t (uint32 wrap as FN:1532)
        const uint32_t E = ql + p;
        for (uint32_t t0 = lo; t0 <= hi; t0 += 64) {
          const uint32_t t = t0 + lane;
          const bool valid = t <= hi;
          const uint4 fw = fastL[min(t, hi) - T0];
          const uint32_t L = E - t;
          const uint32_t mS = fw.y & 0xffffu, mS2 = fw.y >> 16, mF = fw.z & 0xffffu, mF2 = fw.z >> 16;
          // A query longer than every item of its class lands on the first
          // smaller=false item (lower_bound past the smaller=true class, or
          // the first of a class sorted by len descending); an S query there
          // is equal to it (operator== ignores `smaller`) only at its len.
          // One between the two longest of its class lands on the longest S
          // item (S) or on the second F item (F), equal to neither.
          uint32_t dst = kFsEnd;  // kFsEnd: lower_bound == end (no add); kFsSearch: undecided
          if (S) {
            if (mS != 0xffffu && mF != 0xffffu && L > mS && L != mF) dst = fw.x & 0x40000fffu;
            else if (mS != 0xffffu && L < mS && L > mS2) dst = fw.w & 0xfffu;
            else dst = kFsSearch;
          } else {
            if (mF != 0xffffu && L > mF) dst = fw.x & 0x40000fffu;
            else if (mF != 0xffffu && L < mF && L > mF2) dst = (fw.x & 0x20000000u) ? 0x40000000u : fw.w >> 16;
            else dst = kFsSearch;
          }
          const bool none = (fw.x & 0x80000000u) != 0;  // bucket >= 0: no heads at t (FN:1530)
          const bool add = valid && !none && dst < 0x40000000u;
          const bool slow = valid && !none && dst == kFsSearch;
          qs.nothing += (valid && none) ? 1u : 0u;
          qs.good += add ? 1u : 0u;
          // every lane adds: the non-adding ones to a private dummy counter
          atomicAdd(&cnt[add ? dst : kWinItems + lane], cq);
          const uint64_t sm = __ballot(slow);
          if (sm) {
            const uint32_t c = (uint32_t)__popcll(sm), r = (uint32_t)__popcll(sm & ((1ull << lane) - 1));
            const uint32_t room = 64 - qn, en = e | ((t - T0) << 6);
            if (slow && r < room) qL[wv][qn + r] = en;
            if (c >= room) {
              drain(64);
              __builtin_amdgcn_wave_barrier();
              if (slow && r >= room) qL[wv][r - room] = en;
              qn = c - room;
            } else {
              qn += c;
            }
          }
        }
      }
    } else {
      for (uint32_t e = 0; e < nb; e++) {
        const uint32_t u = __builtin_amdgcn_readlane(bu, e);
        if (!u) continue;
        const uint32_t p = __builtin_amdgcn_readlane(bp, e);
        const uint32_t ql = __builtin_amdgcn_readlane(bl, e), qi = __builtin_amdgcn_readlane(bi, e);
        const uint32_t cq = __builtin_amdgcn_readlane(bc, e), slq = __builtin_amdgcn_readlane(bs, e);
        const bool S = __builtin_amdgcn_readlane(bS, e) != 0;
        const uint32_t lo = max(p + 1, T0);
        const uint32_t hi = (uint32_t)min((uint64_t)p + u, (uint64_t)T1 - 1);
        for (uint32_t t0 = lo; t0 <= hi; t0 += 64) {
          const uint32_t t = t0 + lane;
          if (t <= hi) {
            const uint32_t k = t - p - 1;
            if (lds) d_counter_query<CHECK>(LV, ql, qi, S, cq, slq, k, t, qs, addLds, &A.hr);
            else d_counter_query<CHECK>(GV, ql, qi, S, cq, slq, k, t, qs, addGlb, &A.hr);
          }
        }
      }
    }
    if (qn) drain(qn);
  }
  __syncthreads();
  if (lds)
    for (uint32_t i = threadIdx.x; i < nslot; i += blockDim.x) A.counter[sb + i] = cnt[i];
  if (qs.bad) atomicAdd(&red[0], (unsigned long long)qs.bad);
  if (qs.good) atomicAdd(&red[1], (unsigned long long)qs.good);
  if (qs.nothing) atomicAdd(&red[2], (unsigned long long)qs.nothing);
  if (qs.viol) atomicAdd(&red[3], (unsigned long long)qs.viol);
  if (qs.slow) atomicAdd(&red[5], (unsigned long long)qs.slow);
  __syncthreads();
  if (threadIdx.x < 6 && threadIdx.x != 4 && red[threadIdx.x]) atomicAdd(&A.stats[threadIdx.x], red[threadIdx.x]);
}

// ---- counterSmallerThanHead, target-major with register accumulators.
// A block owns a window of <= 256 consecutive targets and a lane owns one of
// them for the whole window (wave w: targets T0 + 64 w ..).  The items
// covering the window (its crossing list, then the items starting inside it)
// are staged in LDS as 16-byte records (match end E = pos + len, the
// window-relative target range, count | smaller << 31, item), each copied to
// the list of every wave whose 64 targets it reaches, and each wave walks its
// list 64 records per LDS read + readlane.  Per (item, target) pair the fast
// tests of k_counter_win compare the query len L = E - t (FN:1532, uint32
// wrap) with the class maxima of the lane's target, held in registers, and a
// decided query adds the item's count to one of the target's three
// accumulators (first smaller=false item, last smaller=true item, second
// smaller=false item): no memory traffic per pair.  Undecided queries are
// appended to the wave's LDS list and searched 64 at a time when it fills
// (items from global memory / L2, adds by global atomics); at the end each
// accumulator is added to its slot.
#ifndef TGT_REC
#define TGT_REC 128
#endif
constexpr uint32_t kTgtRec = TGT_REC;   // item records staged per chunk
constexpr uint32_t kTgtQ = 256;     // undecided queries listed per wave before a search pass
constexpr uint32_t kTgtS = 256;     // queries listed per wave for binary searches
constexpr uint32_t kNoSlot = 0xffffffffu;
// a staged record covering all 64 targets of its wave carries this range word
// (no window-relative range is 0xffff..ffff) and skips the range test
// full-cover records walked apart from the others (CMSBWT_TGT_SPLIT=0: one
// walk per class with the range test for every record; round 4's per-record
// branch between the two forms measured slower, 12.67-12.73 against
// 12.56-12.58 ms)
#ifndef CMSBWT_TGT_SPLIT
#define CMSBWT_TGT_SPLIT 1
#endif
constexpr bool kTgtSplit = CMSBWT_TGT_SPLIT != 0;
// attribution builds only (wrong counters): 1 staging, 2 + record walks and
// re-tests, 3 (default) + binary searches
#ifndef CMSBWT_TGT_PHASES
#define CMSBWT_TGT_PHASES 3
#endif
constexpr int kTgtPhases = CMSBWT_TGT_PHASES;
// attribution builds only (wrong counters): CMSBWT_TGT_SKIP bit 1 drops the
// re-tests (the listed queries are discarded), bit 2 the full-cover walks,
// bit 4 the partial-record walks
#ifndef CMSBWT_TGT_SKIP
#define CMSBWT_TGT_SKIP 0
#endif
constexpr int kTgtSkip = CMSBWT_TGT_SKIP;
// CMSBWT_TGT_L3=1: the record walk settles the third level in registers too
// (round 6): a query landing on the second-longest S item / third F item, or
// past the shortest item of a class with exactly three, is added without
// being listed.  The attribution builds (CMSBWT_TGT_SKIP) put the re-tests
// and searches at 5.65 of 12.4 ms, and ~300 M of their 357 M queries land
// there; but the extra compares on every record cost more (A/B one box,
// bit-exact: counter 12.37-12.43 -> 13.23-13.34 ms), so it stays off
#ifndef CMSBWT_TGT_L3
#define CMSBWT_TGT_L3 0
#endif
constexpr bool kTgtL3 = CMSBWT_TGT_L3 != 0;
// CMSBWT_TGT_THR_LDS=1: the re-tests and searches read a listed query's
// target fields (class lens, flags, first F item) from LDS (two 16-B reads)
// instead of five / two ds_bpermute from the owning lane.  The 8 KB it adds
// leave five blocks per CU instead of seven; measured (round 6, A/B one box,
// bit-exact): counter 12.36-12.39 -> 14.73-14.75 ms, so the shuffles stay
#ifndef CMSBWT_TGT_THR_LDS
#define CMSBWT_TGT_THR_LDS 0
#endif
constexpr bool kThrLds = CMSBWT_TGT_THR_LDS != 0;
// (with the LDS fields: 14.95-14.98 ms, no better than one batch)
#ifndef CMSBWT_TGT_RETEST2
#define CMSBWT_TGT_RETEST2 0
#endif
constexpr bool kRetest2 = CMSBWT_TGT_RETEST2 != 0;


constexpr uint32_t kFullRec = 0xffffffffu;

// stable partition of list[b, e) (one wave, in place): records whose range
// word is kFullRec first; returns their number
__device__ __forceinline__ uint32_t tgt_partition_full(uint4* list, uint32_t b, uint32_t e, uint32_t lane) {
  const uint32_t n = e - b;  // <= 128 (kTgtRec)
  __builtin_amdgcn_wave_barrier();
  uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
  const bool a0 = lane < n, a1 = lane + 64 < n;
  if (a0) v0 = list[b + lane];
  if (a1) v1 = list[b + 64 + lane];
  const bool f0 = a0 && v0.y == kFullRec, f1 = a1 && v1.y == kFullRec;
  const uint64_t m0 = __ballot(f0), m1 = __ballot(f1), p0 = __ballot(a0 && !f0), p1 = __ballot(a1 && !f1);
  const uint32_t nf0 = (uint32_t)__popcll(m0), nf = nf0 + (uint32_t)__popcll(m1);
  const uint32_t np0 = (uint32_t)__popcll(p0);
  const uint64_t below = (1ull << lane) - 1;
  __builtin_amdgcn_wave_barrier();
  if (a0) list[b + (f0 ? (uint32_t)__popcll(m0 & below) : nf + (uint32_t)__popcll(p0 & below))] = v0;
  if (a1) list[b + (f1 ? nf0 + (uint32_t)__popcll(m1 & below) : nf + np0 + (uint32_t)__popcll(p1 & below))] = v1;
  __builtin_amdgcn_wave_barrier();
  return nf;
}

// v (wave-uniform) in the lanes of mask m, 0 elsewhere: one v_cndmask on the
// SGPR-pair mask (keeps decision masks out of VGPRs)
__device__ __forceinline__ uint32_t sel_u32(uint32_t v, uint64_t m) {
  uint32_t r;
  asm volatile("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(v), "s"(m));
  return r;
}
// acc + (lane's bit of m): one v_addc on the VALU (per-lane statistics without
// scalar popcounts: the scalar unit, one per CU, bounds this kernel)
__device__ __forceinline__ uint32_t addc_mask(uint32_t acc, uint64_t m) {
  uint32_t r;
  asm volatile("v_addc_co_u32_e64 %0, vcc, 0, %1, %2" : "=v"(r) : "v"(acc), "s"(m) : "vcc");
  return r;
}
// unsigned compare of each lane, as a wave mask (llvm.amdgcn.icmp predicates)
constexpr int kNE = 33, kUGT = 34, kULT = 36, kULE = 37;  // llvm.amdgcn.icmp predicates
template <int P>
__device__ __forceinline__ uint64_t ucmp(uint32_t a, uint32_t b) {
  return __builtin_amdgcn_uicmp(a, b, P);
}

// 7 waves per SIMD: <= 72 VGPRs, 22 KB of LDS per block (chunks of 128 records)
__global__ void __launch_bounds__(256, 7) k_counter_tgt(CounterArgs A) {
  __shared__ uint4 recG[4][kTgtRec];  // 8 KB: per wave, the records reaching its targets
  __shared__ uint32_t qL[4][kTgtQ];   // 8 KB
  __shared__ uint32_t nG[8];  // per wave: smaller=true records (front), smaller=false (back)
  __shared__ uint32_t accL[6][256];      // 6 KB: adds settled in the search passes, per target
  __shared__ uint32_t qS[4][kTgtS];       // 4 KB: queries left for binary searches
  __shared__ uint64_t noItL[4];           // per wave: targets without items
  __shared__ uint4 thrL[kThrLds ? 2 : 1][kThrLds ? 256 : 1];  // per target: (sl0, sl1, sl2, fl0), (fl1, fl2, flags, fidx)
  const ItemsSoA& it = A.it;
  const uint32_t w = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t T0 = A.winStart[w], T1 = A.winStart[w + 1];
  const uint32_t iBeg = A.posBegin[T0], iEnd = A.posBegin[T1];
  // the lane's target: presence of items, class maxima (S items ascend by
  // len, F items descend) and the three destination slots
  const uint32_t toff = tid, t = T0 + toff;
  // the three longest items of each class: S items ascend by len (the last
  // three, sl0 longest), F items descend (the first three, fl0 longest); a
  // missing item has len 0 and slot kNoSlot
  uint32_t sl0 = 0, sl1 = 0, sl2 = 0, fl0 = 0, fl1 = 0, fl2 = 0;
  uint32_t ss0 = kNoSlot, ss1 = kNoSlot, ss2 = kNoSlot, fs0 = kNoSlot, fs1 = kNoSlot, fs2 = kNoSlot;
  bool has = false, nS3 = false, nF3 = false;
  uint32_t fidx = 0, nS8 = 255, nF8 = 255;  // first F item; class sizes (255: 255 or more)
  if (t < T1) {
    const uint32_t b0 = A.posBegin[t], b1 = A.posBegin[t + 1], f = A.posF[t];
    has = b0 != b1;
    const uint32_t nS = f - b0, nF = b1 - f;
    if (nS >= 1) { sl0 = it.len[f - 1]; ss0 = it.slot[f - 1]; }
    if (nS >= 2) { sl1 = it.len[f - 2]; ss1 = it.slot[f - 2]; }
    if (nS >= 3) { sl2 = it.len[f - 3]; ss2 = it.slot[f - 3]; }
    if (nF >= 1) { fl0 = it.len[f]; fs0 = it.slot[f]; }
    if (nF >= 2) { fl1 = it.len[f + 1]; fs1 = it.slot[f + 1]; }
    if (nF >= 3) { fl2 = it.len[f + 2]; fs2 = it.slot[f + 2]; }
    nS3 = nS == 3;
    nF3 = nF == 3;
    fidx = f;
    nS8 = min(nS, 255u);
    nF8 = min(nF, 255u);
  }
  const bool hasF0 = fs0 != kNoSlot, hasF1 = fs1 != kNoSlot, hasF2 = fs2 != kNoSlot;
  const uint64_t hasF1M = __ballot(hasF1);  // per wave
  const uint64_t hasF0M = __ballot(hasF0);  // (an F item implies items: in-range F lanes = in-range lanes & hasF0M)
  const uint64_t hasM = __ballot(has);
  const uint64_t hasF2M = __ballot(hasF2), nS3M = __ballot(nS3), nF3M = __ballot(nF3);
  const uint32_t flags = (hasF0 ? 1u : 0u) | (hasF1 ? 2u : 0u) | (hasF2 ? 4u : 0u) | (nS3 ? 8u : 0u) |
                         (nF3 ? 16u : 0u) | (nS8 << 8) | (nF8 << 16);
  for (uint32_t k = 0; k < 6; k++) accL[k][tid] = 0;
  if (kThrLds) {
    thrL[0][tid] = make_uint4(sl0, sl1, sl2, fl0);
    thrL[1][tid] = make_uint4(fl1, fl2, flags, fidx);
  }
  // lanes without items never fall in a record's range (their pairs are
  // counted once per staged record: counterDoNothing, FN:1530)
  const uint32_t tofH = has ? toff : 0x40000000u;
  {
    const uint64_t hm = __ballot(has);
    if (lane == 0) noItL[wv] = ~hm;
  }
  // accumulators: first F item (f), S items top 0..2, F items 1..2
  uint32_t aF0 = 0, aS0 = 0, aS1 = 0, aS2 = 0, aF1 = 0, aF2 = 0, nGood = 0, nNothing = 0;
  QueryStats qs;
  const GlobalView GV{&A.it, A.posBegin, A.posF, A.nhr};
  uint32_t* const myQ = qL[wv];
  uint32_t* const myS = qS[wv];
  const uint4* const myR = recG[wv];
  const uint32_t c0 = A.crossOff[w], nCross = A.crossOff[w + 1] - c0;
  const uint32_t nList = nCross + (iEnd - iBeg);
  // binary searches of the wave's listed queries (FN:1534-1597 in full)
  uint32_t nSearch = 0;
  auto search = [&]() {
    __builtin_amdgcn_wave_barrier();
    for (uint32_t d = 0; d < nSearch; d += 64) {
      const bool act = d + lane < nSearch;
      const uint32_t en = act ? myS[d + lane] : 0u;
      // the target's item range from its owning lane
      const int own = (int)((en >> 16) & 63u);
      uint32_t fo, fl;
      if (kThrLds) {
        const uint4 b = thrL[1][(wv << 6) + own];
        fo = b.w;
        fl = b.z;
      } else {
        fo = __shfl(fidx, own);
        fl = __shfl(flags, own);
      }
      if (act) {
        const uint4 rc = myR[en & 0xffffu];
        const uint32_t tq = T0 + ((en >> 16) & 0xffu);
        const uint32_t q = rc.w, L = rc.x - tq;
        const bool S = (en >> 31) != 0;
        qs.slow++;
        auto addG = [&](uint32_t s, uint32_t v) { atomicAdd(&A.counter[s], (unsigned long long)v); };
        const uint32_t nS = (fl >> 8) & 0xffu, nF = (fl >> 16) & 0xffu;
        const EqList* eql = A.eq.rec ? &A.eq : nullptr;
        if (nS < 255u && nF < 255u) {
          const KnownView KV{&A.it, A.nhr, tq, fo - nS, fo + nF, fo};
          d_counter_query_L<false>(KV, L, it.isa[q], S, rc.z & 0x7fffffffu, it.slot[q], tq, qs, addG, nullptr, eql);
        } else {
          d_counter_query_L<false>(GV, L, it.isa[q], S, rc.z & 0x7fffffffu, it.slot[q], tq, qs, addG, nullptr, eql);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    nSearch = 0;
  };
  // one staged record against the wave's 64 targets.  Record: x = match end
  // E, y = aO | span << 16 (targets T0 + aO .. T0 + aO + span), z = count.
  // lower_bound (FN:1534) is settled by the two longest items of the query's
  // class (k_counter_win's fast tests, exact lens).  The decisions are wave
  // masks (SGPR pairs; the per-target flags are loop-invariant masks) and an
  // add is one v_cndmask on its mask; range tests and statistics stay on the
  // VALU (the scalar unit, one per CU, bounds this loop).
  auto rec = [&](auto cls, auto fullc, const uint4& my, uint32_t r, uint32_t e, uint32_t& qn) {
    constexpr bool S = decltype(cls)::value;
    constexpr bool FULL = decltype(fullc)::value;
    const uint32_t cqv = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(my.z, e));
    const uint32_t L = __builtin_amdgcn_readlane(my.x, e) - t;
    uint64_t mIn, mInF;
    if (FULL) {  // the record reaches all 64 targets of the wave: no range test
      mIn = hasM;
      mInF = hasF0M;
    } else {
      const uint32_t ab = __builtin_amdgcn_readlane(my.y, e);
      const uint32_t aO = ab & 0xffffu, span = ab >> 16;
      mIn = ucmp<kULE>(tofH - aO, span);  // targets with items
      mInF = mIn & hasF0M;                // ... and a smaller=false item
    }
    uint64_t mF0, mX, msl, mX3 = 0;
    if (S) {  // smaller=true: S items ascending, then F items
      const uint64_t m1 = ucmp<kUGT>(L, sl0) & ucmp<kNE>(L, fl0);  // past every S item: f (or end)
      const uint64_t m2 = ucmp<kULT>(L, sl0) & ucmp<kUGT>(L, sl1);   // the longest S item
      mF0 = mInF & m1;
      mX = mIn & m2;
      aS0 += sel_u32(cqv, mX);
      if (kTgtL3) {
        // the second-longest S item (the shortest when there are two), or
        // below the shortest of exactly three S items: the third (FN:1534)
        const uint64_t lt1 = ucmp<kULT>(L, sl1);
        const uint64_t m3 = lt1 & ucmp<kUGT>(L, sl2);
        const uint64_t m4 = ucmp<kULT>(L, sl2) & nS3M;
        mX3 = mIn & (m3 | m4);
        aS1 += sel_u32(cqv, mIn & m3);
        aS2 += sel_u32(cqv, mIn & m4);
        msl = mIn & ~(m1 | m2 | m3 | m4);
      } else {
        msl = mIn & ~(m1 | m2);
      }
    } else {  // smaller=false: F items descending
      const uint64_t m1 = ucmp<kUGT>(L, fl0);                       // f
      const uint64_t m2 = ucmp<kULT>(L, fl0) & ucmp<kUGT>(L, fl1);   // the second F item (or end)
      mF0 = mInF & m1;
      mX = mIn & m2 & hasF1M;
      aF1 += sel_u32(cqv, mX);
      if (kTgtL3) {
        // the third F item (or end), or below the shortest of exactly three
        // F items: end (nothing added, FN:1535-1536)
        const uint64_t m3 = ucmp<kULT>(L, fl1) & ucmp<kUGT>(L, fl2);
        const uint64_t m4 = ucmp<kULT>(L, fl2) & nF3M;
        mX3 = mIn & m3 & hasF2M;
        aF2 += sel_u32(cqv, mX3);
        msl = mIn & ~(m1 | m2 | m3 | m4);
      } else {
        msl = mIn & ~(m1 | m2);
      }
    }
    aF0 += sel_u32(cqv, mF0);
    nGood = addc_mask(nGood, mF0 | mX | mX3);  // (disjoint masks)
    if (msl) {
      if ((msl >> lane) & 1) {
        const uint32_t rk =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(msl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)msl, 0u));
        myQ[qn + rk] = (r + e) | (toff << 16);
      }
      qn += (uint32_t)__popcll(msl);
    }
  };
  // search pass over the listed queries: first the three longest items of
  // the class (the target's fields from LDS, or from the owning lane by
  // ds_bpermute); what they do not settle goes to the wave's search list,
  // binary-searched 64 at a time.
  // A listed query's landing by the three longest items of its class (0 f,
  // 1..3 S top 0..2, 4..5 F items 1..2; 6 end / none; 7 search), its count
  auto decide = [&](auto cls, uint32_t en, bool act, uint32_t& cq) -> uint32_t {
    constexpr bool S = decltype(cls)::value;
    const int own = (int)((en >> 16) & 63u);
    uint32_t o0, o1, o2, of0, fl;
    if (kThrLds) {  // (lanes past the list read their wave's target 0: harmless)
      const uint4 a = thrL[0][(wv << 6) + own], b = thrL[1][(wv << 6) + own];
      o0 = S ? a.x : a.w;
      o1 = S ? a.y : b.x;
      o2 = S ? a.z : b.y;
      of0 = a.w;
      fl = b.z;
    } else {
      o0 = __shfl(S ? sl0 : fl0, own);
      o1 = __shfl(S ? sl1 : fl1, own);
      o2 = __shfl(S ? sl2 : fl2, own);
      of0 = __shfl(fl0, own);
      fl = __shfl(flags, own);
    }
    uint32_t dst = 6;
    cq = 0;
    if (act) {
      const uint4 rc = myR[en & 0xffffu];
      const uint32_t L = rc.x - (T0 + (en >> 16));
      cq = rc.z & 0x7fffffffu;
      const bool g0 = L < o0, g1 = L < o1, g2 = L < o2;
      const bool ne = (L != o0) & (L != o1) & (L != o2);
      dst = 7;
      if (S) {
        if (!g0 & ne) dst = (fl & 1u) ? ((L != of0) ? 0u : 7u) : 6u;
        else if (g0 & !g1 & ne) dst = 1;
        else if (g1 & !g2 & ne) dst = 2;
        else if (g2 & ne & ((fl & 8u) != 0)) dst = 3;
      } else {
        if (!g0 & ne) dst = (fl & 1u) ? 0u : 6u;
        else if (g0 & !g1 & ne) dst = (fl & 2u) ? 4u : 6u;
        else if (g1 & !g2 & ne) dst = (fl & 4u) ? 5u : 6u;
        else if (g2 & ne & ((fl & 16u) != 0)) dst = 6;
      }
    }
    return dst;
  };
  // the add of a settled query, or its place in the wave's search list
  auto settle = [&](auto cls, uint32_t en, uint32_t dst, uint32_t cq) {
    constexpr bool S = decltype(cls)::value;
    if (dst < 6) {
      atomicAdd(&accL[dst][en >> 16], cq);
      qs.good++;
    }
    const uint64_t smS = __ballot(dst == 7);
    if (dst == 7) {
      const uint32_t rk =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(smS >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)smS, 0u));
      myS[nSearch + rk] = en | (S ? 0x80000000u : 0u);
    }
    nSearch += (uint32_t)__popcll(smS);
  };
  // the pass, 64 queries at a time (two batches per iteration with
  // CMSBWT_TGT_RETEST2, their LDS reads in flight together)
  auto retest = [&](auto cls, uint32_t qn) {
    __builtin_amdgcn_wave_barrier();
    if (kRetest2) {
      for (uint32_t d = 0; d < qn; d += 128) {
        const bool act0 = d + lane < qn, act1 = d + 64 + lane < qn;
        const uint32_t en0 = act0 ? myQ[d + lane] : 0u, en1 = act1 ? myQ[d + 64 + lane] : 0u;
        uint32_t cq0, cq1;
        const uint32_t dst0 = decide(cls, en0, act0, cq0);
        const uint32_t dst1 = decide(cls, en1, act1, cq1);
        settle(cls, en0, dst0, cq0);
        settle(cls, en1, dst1, cq1);
        if (nSearch >= kTgtS - 128) search();
      }
    } else {
      for (uint32_t d = 0; d < qn; d += 64) {
        const bool act = d + lane < qn;
        const uint32_t en = act ? myQ[d + lane] : 0u;
        uint32_t cq;
        const uint32_t dst = decide(cls, en, act, cq);
        settle(cls, en, dst, cq);
        if (nSearch >= kTgtS - 64) search();
      }
    }
    __builtin_amdgcn_wave_barrier();
  };
  // one walk over a wave's records of one class (smaller=true records from
  // the front of its list, smaller=false ones from the back)
  auto walk = [&](auto cls, auto fullc, uint32_t rb, uint32_t re) {
    uint32_t r = rb;
    while (r < re) {
      uint32_t qn = 0;  // listed undecided queries (wave-uniform)
      while (r < re && qn <= kTgtQ - 64) {
        const uint32_t nb = min(64u, re - r);
        const uint4 my = lane < nb ? myR[r + lane] : make_uint4(0u, 0u, 0u, 0u);
        uint32_t e = 0;
        while (e < nb && qn <= kTgtQ - 64) {
          // records that cannot overflow the query list (<= 64 queries each)
          const uint32_t lim = min(nb, e + ((kTgtQ - qn) >> 6));
          // (unrolled by two: the loop control is scalar work too)
          for (; e + 1 < lim; e += 2) {
            rec(cls, fullc, my, r, e, qn);
            rec(cls, fullc, my, r, e + 1, qn);
          }
          if (e < lim) rec(cls, fullc, my, r, e++, qn);
        }
        r += e;
      }
      if (qn && !(kTgtSkip & 1)) retest(cls, qn);
    }
  };
  for (uint32_t ch = 0; ch < nList; ch += kTgtRec) {
    const uint32_t nr = min(kTgtRec, nList - ch);
    if (tid < 8) nG[tid] = 0;
    __syncthreads();  // the previous chunk's lists are no longer read
    for (uint32_t ti = tid; ti < nr; ti += blockDim.x) {
      // every chunk mixes crossing items (they reach the first waves'
      // targets) and starting items taken from all four quarters of the
      // window, so the four waves get similar lists between two barriers
      const uint32_t j = ch + ti;
      const uint32_t nSt = nList - nCross;
      const uint32_t cj = (uint32_t)((uint64_t)j * nCross / nList);
      const bool isCross = (uint32_t)((uint64_t)(j + 1) * nCross / nList) > cj;
      uint32_t q;
      if (isCross) {
        q = A.crossList[c0 + cj];
      } else {
        const uint32_t sj = j - cj, qs4 = (nSt + 3) >> 2;  // quarter-interleaved starting items
        const uint32_t rq = sj & 3, kq = sj >> 2;
        // the first (nSt mod 4 or 4) quarters hold qs4 items, the rest qs4 - 1
        const uint32_t full = nSt - 4 * (qs4 - 1);  // quarters with qs4 items (1..4)
        q = iBeg + (rq < full ? rq * qs4 : full * qs4 + (rq - full) * (qs4 - 1)) + kq;
      }
      // the item's fields in one 16-byte load (crossing items are random)
      const uint4 iw = A.irec ? A.irec[q] : make_uint4(it.pos[q], it.until[q], 0u, 0u);
      const uint32_t p = iw.x, u = iw.y;
      if (u) {
        const uint32_t lo = max(p + 1, T0);
        const uint32_t hi = (uint32_t)min((uint64_t)p + u, (uint64_t)T1 - 1);
        if (lo <= hi) {
          const uint32_t aO = lo - T0, bO = hi - T0;
          const bool sm = A.irec ? (iw.w >> 31) != 0 : it.smaller[q] != 0;
          const uint32_t ln = A.irec ? iw.z : it.len[q], cnt = A.irec ? iw.w & 0x7fffffffu : it.count[q];
          const uint4 rec = make_uint4(ln + p, aO | ((bO - aO) << 16), cnt, q);
          for (uint32_t k = aO >> 6; k <= (bO >> 6); k++) {
            // pairs of this record whose target has no heads (FN:1530)
            const uint32_t a = k == (aO >> 6) ? (aO & 63u) : 0u, b = k == (bO >> 6) ? (bO & 63u) : 63u;
            nNothing += (uint32_t)__popcll(noItL[k] & (~0ull >> (63u - b)) & (~0ull << a));
            const uint32_t o = atomicAdd(&nG[2 * k + (sm ? 0 : 1)], 1u);
            const bool full = kTgtSplit && aO <= 64 * k && bO >= 64 * k + 63;
            recG[k][sm ? o : kTgtRec - 1 - o] = full ? make_uint4(rec.x, kFullRec, rec.z, rec.w) : rec;
          }
        }
      }
    }
    __syncthreads();
    const uint32_t nS = nG[2 * wv], nF = nG[2 * wv + 1];
    if (kTgtSplit) {
      // full-cover records first in each class's list (a stable partition by
      // the wave, <= 2 x 64 records per class), so the walks over them skip
      // the range test and its decode (80 % of the records, 94 % of the pairs)
      const uint32_t nSf = tgt_partition_full(recG[wv], 0u, nS, lane);
      const uint32_t nFf = tgt_partition_full(recG[wv], kTgtRec - nF, kTgtRec, lane);
      if (kTgtPhases >= 2) {
        if (!(kTgtSkip & 2)) walk(std::true_type{}, std::true_type{}, 0u, nSf);
        if (!(kTgtSkip & 4)) walk(std::true_type{}, std::false_type{}, nSf, nS);
        if (!(kTgtSkip & 2)) walk(std::false_type{}, std::true_type{}, kTgtRec - nF, kTgtRec - nF + nFf);
        if (!(kTgtSkip & 4)) walk(std::false_type{}, std::false_type{}, kTgtRec - nF + nFf, kTgtRec);
      }
    } else if (kTgtPhases >= 2) {
      walk(std::true_type{}, std::false_type{}, 0u, nS);
      walk(std::false_type{}, std::false_type{}, kTgtRec - nF, kTgtRec);
    }
    if (kTgtPhases < 3) nSearch = 0;
    if (nSearch) search();  // before the next chunk replaces the records
  }
  __syncthreads();
  aF0 += accL[0][tid]; aS0 += accL[1][tid]; aS1 += accL[2][tid]; aS2 += accL[3][tid];
  aF1 += accL[4][tid]; aF2 += accL[5][tid];
  if (aF0) atomicAdd(&A.counter[fs0], (unsigned long long)aF0);
  if (aF1) atomicAdd(&A.counter[fs1], (unsigned long long)aF1);
  if (aF2) atomicAdd(&A.counter[fs2], (unsigned long long)aF2);
  if (aS0) atomicAdd(&A.counter[ss0], (unsigned long long)aS0);
  if (aS1) atomicAdd(&A.counter[ss1], (unsigned long long)aS1);
  if (aS2) atomicAdd(&A.counter[ss2], (unsigned long long)aS2);
  qs.good += nGood;
  qs.nothing += nNothing;
  if (qs.bad) atomicAdd(&A.stats[0], (unsigned long long)qs.bad);
  if (qs.good) atomicAdd(&A.stats[1], (unsigned long long)qs.good);
  if (qs.nothing) atomicAdd(&A.stats[2], (unsigned long long)qs.nothing);
  if (qs.slow) atomicAdd(&A.stats[5], (unsigned long long)qs.slow);
}

// statistics only (CMSBWT_COUNTER_STATS=2): per item, its target range cut
// into 64-target groups; out: [0] records, [1] full records, [2] pairs,
// [3] pairs in full records, [8 + b] pairs of items with 2^b <= range < 2^(b+1)
__global__ void k_counter_shape(const ItemsSoA it, uint32_t K, uint32_t n, unsigned long long* __restrict__ out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  const uint32_t p = it.pos[q], u = it.until[q];
  if (!u || p + 1 >= n) return;
  const uint32_t lo = p + 1, hi = (uint32_t)min((uint64_t)p + u, (uint64_t)n - 1);
  const uint32_t g0 = lo >> 6, g1 = hi >> 6, pr = hi - lo + 1;
  uint32_t full = 0;
  for (uint32_t g = g0; g <= g1; g++) full += (64 * g >= lo && 64 * g + 63 <= hi) ? 1u : 0u;
  atomicAdd(&out[0], (unsigned long long)(g1 - g0 + 1));
  atomicAdd(&out[1], (unsigned long long)full);
  atomicAdd(&out[2], (unsigned long long)pr);
  atomicAdd(&out[3], 64ull * full);
  atomicAdd(&out[8 + (31 - __builtin_clz(pr))], (unsigned long long)pr);
}
void mk_counter_shape(const ItemsSoA& it, uint32_t K, uint32_t n, unsigned long long* out, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_counter_shape, dim3((K + 255) / 256), dim3(256), 0, st, it, K, n, out);
}
__global__ void k_item_rec(const ItemsSoA it, uint32_t K, uint4* __restrict__ out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < K)
    out[q] = make_uint4(it.pos[q], it.until[q], it.len[q], (it.count[q] & 0x7fffffffu) | (it.smaller[q] ? 0x80000000u : 0u));
}
void mk_item_rec(const ItemsSoA& it, uint32_t K, uint4* out, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_item_rec, dim3((K + 255) / 256), dim3(256), 0, st, it, K, out);
}
__global__ void k_item_sk(ItemsSoA it, uint32_t K) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  const uint32_t L = it.len[q];
  it.sk[q] = ((unsigned long long)(it.smaller[q] ? L : ~L) << 32) | it.isa[q];
}

// ---- window construction
// boundary at p when the first slot of p enters a new half-window block of
// slots, or every winPos positions
__global__ void k_win_flags(const uint32_t* __restrict__ posBegin, const uint32_t* __restrict__ slot, uint32_t n,
                            uint32_t P0, uint32_t P1, uint32_t winPos, uint32_t half, uint32_t* __restrict__ flag) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (p < P0 || p >= P1) { flag[p] = 0; return; }  // windows cover the target range [P0, P1) only
  if (p == P0 || (p - P0) % winPos == 0) { flag[p] = 1; return; }
  uint32_t a = slot[posBegin[p - 1]] / half, b = slot[posBegin[p]] / half;
  flag[p] = a != b ? 1u : 0u;
}

// fixed windows of winPos targets over [P0, P1): the inclusive window count
// of every position (k_win_flags + scan of the general path) and the starts
__global__ void k_win_fixed(uint32_t n, uint32_t P0, uint32_t P1, uint32_t winPos, uint32_t nw,
                            uint32_t* __restrict__ wincl, uint32_t* __restrict__ winStart) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) wincl[p] = p < P0 ? 0u : (p >= P1 ? nw : (p - P0) / winPos + 1);
  if (p <= nw) winStart[p] = p < nw ? P0 + p * winPos : P1;
}
__global__ void k_set_u32(uint32_t* __restrict__ p, uint32_t v) { *p = v; }
__global__ void k_win_starts(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ winIncl, uint32_t n,
                             uint32_t* __restrict__ winStart) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (flag[p]) winStart[winIncl[p] - 1] = p;
}

// Items crossing the start of later windows, as (window, item) pairs: pass 0
// counts per item, pass 1 writes at the item's exclusive offset; the pairs are
// then radix-sorted by window (no contended atomics).
__global__ void k_win_cross(const ItemsSoA it, uint32_t K, const uint32_t* __restrict__ winIncl, uint32_t n,
                            uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                            uint32_t* __restrict__ keyW, uint32_t* __restrict__ valQ,
                            unsigned long long* __restrict__ errs, int fill) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  const uint32_t p = it.pos[q], u = it.until[q];
  uint32_t c = 0, wf = 0;
  if (u) {
    uint64_t last = (uint64_t)p + u;
    if (last >= n) { if (!fill) atomicAdd(errs, 1ull); last = n - 1; }
    wf = winIncl[p];                         // = window index of p, plus one (0 before the range)
    const uint32_t il = winIncl[last];       // = window of the last target, plus one
    c = il > wf ? il - wf : 0;
  }
  if (!fill) { cnt[q] = c; return; }
  const uint32_t o = off[q];
  for (uint32_t k = 0; k < c; k++) { keyW[o + k] = wf + k; valQ[o + k] = q; }
}

// ---- crossing lists without a sort (round 6).  Item q crosses the windows
// wf_q .. wf_q + c_q - 1 (k_win_cross: wf = its own window + 1, 0 for the
// halo items before P0).  Number the item's "source" sv = wf_q (items of
// window sv - 1; sv = 0: positions before P0) and the distance d = w - sv:
// the items of one source that reach distance d are a filtered run of its
// items, so window w's list is the concatenation over d of the runs of
// source w - d.  Three passes, no sort (the (window, item) pairs were a
// rocPRIM radix sort of ~2 x 10^8 keys, 5.7 ms on the side stream at config
// 3): per source its depth (largest c) and n_sv(d) = #items with c > d; per
// window the counts and the offsets of its runs; per source the placement.
// The order inside a window's list (by distance, then item) differs from the
// sorted order; the counter only sums over it.
constexpr uint32_t kXwHist = kXwMaxDepth;  // depth handled in LDS (deeper sources: the sort path)
__device__ __forceinline__ void xw_items(const uint32_t* posBegin, const uint32_t* winStart, uint32_t P0, uint32_t sv,
                                         uint32_t& ib, uint32_t& ie) {
  const uint32_t ps = sv == 0 ? 0u : winStart[sv - 1], pe = sv == 0 ? P0 : winStart[sv];
  ib = posBegin[ps];
  ie = posBegin[pe];
}
__global__ void __launch_bounds__(256) k_xw_depth(const uint32_t* __restrict__ posBegin,
                                                  const uint32_t* __restrict__ winStart, uint32_t P0,
                                                  const uint32_t* __restrict__ cnt, uint32_t* __restrict__ depth) {
  __shared__ uint32_t mx[4];
  const uint32_t sv = blockIdx.x;
  uint32_t ib, ie;
  xw_items(posBegin, winStart, P0, sv, ib, ie);
  uint32_t m = 0;
  for (uint32_t q = ib + threadIdx.x; q < ie; q += 256) m = max(m, cnt[q]);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) mx[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) depth[sv] = max(max(mx[0], mx[1]), max(mx[2], mx[3]));
}
// n_sv(d) for d < depth[sv] at T[toff[sv] + d] (suffix sums of a histogram
// of c over the source's items)
__global__ void __launch_bounds__(256) k_xw_hist(const uint32_t* __restrict__ posBegin,
                                                 const uint32_t* __restrict__ winStart, uint32_t P0,
                                                 const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ depth,
                                                 const uint32_t* __restrict__ toff, uint32_t* __restrict__ T) {
  __shared__ uint32_t h[kXwHist];
  const uint32_t sv = blockIdx.x, D = depth[sv];
  if (D == 0) return;
  uint32_t ib, ie;
  xw_items(posBegin, winStart, P0, sv, ib, ie);
  for (uint32_t d = threadIdx.x; d < D; d += 256) h[d] = 0;
  __syncthreads();
  for (uint32_t q = ib + threadIdx.x; q < ie; q += 256) {
    const uint32_t c = cnt[q];
    if (c) atomicAdd(&h[c - 1], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    uint32_t* o = T + toff[sv];
    for (uint32_t d = D; d-- > 0;) {
      acc += h[d];
      o[d] = acc;
    }
  }
}
// per target window w: its list length and the offset of each of its runs
// inside it (run (sv, d) at segOff[toff[sv] + d]), distance 0 first
__global__ void k_xw_count(const uint32_t* __restrict__ depth, const uint32_t* __restrict__ toff,
                           const uint32_t* __restrict__ T, uint32_t nw, uint32_t maxDepth,
                           uint32_t* __restrict__ segOff, uint32_t* __restrict__ count) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  uint32_t run = 0;
  const uint32_t dEnd = min(w + 1, maxDepth);
  for (uint32_t d = 0; d < dEnd; d++) {
    const uint32_t sv = w - d;
    if (d < depth[sv]) {
      const uint32_t k = toff[sv] + d;
      segOff[k] = run;
      run += T[k];
    }
  }
  count[w] = run;
}
// per source: each item with c > d goes to window sv + d at its run's offset
// plus its rank among the source's items with c > d (item order)
__global__ void __launch_bounds__(256) k_xw_place(const uint32_t* __restrict__ posBegin,
                                                  const uint32_t* __restrict__ winStart, uint32_t P0,
                                                  const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ depth,
                                                  const uint32_t* __restrict__ toff,
                                                  const uint32_t* __restrict__ segOff,
                                                  const uint32_t* __restrict__ crossOff,
                                                  uint32_t* __restrict__ crossList) {
  __shared__ uint32_t base[kXwHist];
  __shared__ uint32_t wsum[4], cmaxL[4];
  const uint32_t sv = blockIdx.x, D = depth[sv];
  if (D == 0) return;
  uint32_t ib, ie;
  xw_items(posBegin, winStart, P0, sv, ib, ie);
  const uint32_t t0 = toff[sv];
  for (uint32_t d = threadIdx.x; d < D; d += 256) base[d] = crossOff[sv + d] + segOff[t0 + d];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t cb = ib; cb < ie; cb += 256) {
    const uint32_t q = cb + threadIdx.x;
    const uint32_t c = q < ie ? cnt[q] : 0u;
    uint32_t m = c;
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if (lane == 0) cmaxL[wv] = m;
    __syncthreads();  // (also orders the base[] initialisation / previous chunk's updates)
    const uint32_t cm = max(max(cmaxL[0], cmaxL[1]), max(cmaxL[2], cmaxL[3]));
    for (uint32_t d = 0; d < cm; d++) {
      const bool f = c > d;
      const uint64_t b = __ballot(f);
      if (lane == 0) wsum[wv] = (uint32_t)__popcll(b);
      __syncthreads();
      uint32_t before = 0;
      for (uint32_t k = 0; k < wv; k++) before += wsum[k];
      const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
      if (f) crossList[base[d] + before + (uint32_t)__popcll(b & ((1ull << lane) - 1))] = q;
      __syncthreads();  // every read of wsum and base[d] is done
      if (threadIdx.x == 0) base[d] += tot;
    }
    __syncthreads();
  }
}

__global__ void k_win_cross_off(const uint32_t* __restrict__ keyW, uint32_t ncross, uint32_t nw,
                                uint32_t* __restrict__ crossOff) {
  uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w > nw) return;
  uint32_t lo = 0, hi = ncross;
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (keyW[m] < w) lo = m + 1; else hi = m;
  }
  crossOff[w] = lo;
}

// ------------------------------------------------------------ buckets (FN:1162-1171, 1618-1628)
__global__ void k_bucket(const int32_t* __restrict__ countIncl, const uint8_t* __restrict__ hasHead, uint32_t n,
                         int64_t* __restrict__ bucket) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  int64_t c = countIncl[p];
  bucket[p] = hasHead[p] ? -c : c;
}

// ------------------------------------------------------------ writer (FN:1631-1777)
// Segments (character, count) in output order, grouped into runs: a unit /
// element's run count includes its first segment; k_wr_adjust drops that one
// when it continues the previous non-empty unit's run (prevHL = exclusive
// "last non-empty" scan of hl = has << 16 | last << 8 | first)
__global__ void k_wr_adjust(const uint32_t* __restrict__ hl, const uint32_t* __restrict__ prevHL, uint32_t U,
                            uint32_t* __restrict__ runs) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const uint32_t a = hl[u], pv = prevHL[u];
  if ((a >> 16) && (pv >> 16) && (a & 0xff) == ((pv >> 8) & 0xff)) runs[u]--;
}
// 9-byte little-endian records (length u64, char), FN:1708-1709
__global__ void k_wr_records(const unsigned long long* __restrict__ runStart, const uint8_t* __restrict__ runChar,
                             uint64_t R, unsigned long long total, uint8_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= R) return;
  const unsigned long long len = (j + 1 < R ? runStart[j + 1] : total) - runStart[j];
  uint8_t* o = out + 9 * j;
#pragma unroll
  for (int b = 0; b < 8; b++) o[b] = (uint8_t)(len >> (8 * b));
  o[8] = runChar[j];
}

// ---- element writer: one thread per writer element instead of per SA rank.
// Elements in output order: the E end phrases (rank 0), then per SA rank
// r >= 1 its heads in head-rank order (= slot order of its position), or one
// element when it has none.  A rank's heads are contiguous in every array the
// thread reads (counter and cum by slot, bwtHeads by head rank), so a wave
// reads contiguous memory whatever the head count of its ranks; the per-rank
// loops of the round-1 writer diverged over 1..1000+ heads per thread.
// ElemArgs, d_elem_segments: elem_writer.h (shared with the fused scan in engine.h)

// per-rank fields of the element writer: element base, head count, slot
// base of the rank's position, head base; bucket and BWT character
__global__ void k_el_info(const int32_t* __restrict__ sa, const uint8_t* __restrict__ bwt,
                          const int64_t* __restrict__ bucket, const uint32_t* __restrict__ posBegin,
                          const uint32_t* __restrict__ slot, const uint32_t* __restrict__ headBase,
                          const uint32_t* __restrict__ elemBase, uint32_t n, uint32_t E, uint32_t H,
                          uint4* __restrict__ info1, unsigned long long* __restrict__ info2) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t hb = headBase[r];
  const uint32_t nh = (r + 1 < n ? headBase[r + 1] : H) - hb;
  uint32_t s0 = 0;
  unsigned long long j = 0;
  if (r > 0) {
    const uint32_t p = (uint32_t)sa[r];
    const int64_t b = bucket[p];
    if (b < 0 && nh) s0 = slot[posBegin[p]];
    j = ((unsigned long long)b & 0x00ffffffffffffffull) | ((unsigned long long)bwt[r] << 56);
  } else if (E) {
    s0 = slot[posBegin[n - 1]];  // the end phrases' item
  }
  info1[r] = make_uint4(elemBase[r], r == 0 ? E : nh, s0, hb);
  info2[r] = j;
}

// elements per SA rank: E at rank 0, otherwise max(heads, 1)
__global__ void k_el_count(const uint32_t* __restrict__ headBase, uint32_t n, uint32_t E, uint32_t H,
                           uint32_t* __restrict__ m) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t nh = (r + 1 < n ? headBase[r + 1] : H) - headBase[r];
  m[r] = r == 0 ? E : max(nh, 1u);
}
__global__ void k_el_rof(const uint32_t* __restrict__ elemBase, const uint32_t* __restrict__ m, uint32_t n,
                         uint32_t* __restrict__ rOf) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t b = elemBase[r], c = m[r];
  for (uint32_t k = 0; k < c; k++) rOf[b + k] = r;
}
// ---- the writer's run scan in tiles of 256 elements (one block each): the
// tile kernel reduces its elements' run summaries (WrOp, elem_writer.h) to one
// per tile, a scan of the tile summaries gives every tile its prefix, and the
// emit kernel scans its tile's summaries again and emits each element's runs
// at its prefix -- two passes over the elements, no per-element arrays (the
// unfused writer wrote and scanned five of them, CMSBWT_WR_UNFUSED=1)
__device__ __forceinline__ WrState wr_shfl_up(const WrState& v, int d) {
  WrState r;
  r.runs = __shfl_up(v.runs, d);
  r.sym = __shfl_up(v.sym, d);
  r.lastStart = __shfl_up(v.lastStart, d);
  r.hl = __shfl_up(v.hl, d);
  r.pad = 0;
  return r;
}
// block-wide exclusive scan (256 threads) of x; *total = the block's summary
__device__ __forceinline__ WrState wr_block_exscan(WrState x, WrState* total) {
  __shared__ WrState wt[4];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const WrOp op;
  WrState inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const WrState y = wr_shfl_up(inc, d);
    if ((int)lane >= d) inc = op(y, inc);
  }
  if (lane == 63) wt[w] = inc;
  __syncthreads();
  const WrState zero{0ull, 0ull, 0ull, 0u, 0u};
  WrState pre = zero;
  for (uint32_t k = 0; k < w; k++) pre = op(pre, wt[k]);
  WrState ex = wr_shfl_up(inc, 1);
  if (lane == 0) ex = zero;
  if (total) *total = op(op(wt[0], wt[1]), op(wt[2], wt[3]));
  return op(pre, ex);
}
__global__ void __launch_bounds__(256) k_el_wr_tiles(ElemArgs A, uint32_t V, WrState* __restrict__ tileSum,
                                                     uint4* __restrict__ segOut) {
  const uint32_t e = blockIdx.x * 256 + threadIdx.x;
  WrState s{0ull, 0ull, 0ull, 0u, 0u};
  if (e < V) {
    const ElemSegs g = d_elem_collect(A, e);
    if (segOut) segOut[e] = segs_pack(g);  // (element order: coalesced)
    s = g.state();
  }
  WrState tot;
  (void)wr_block_exscan(s, &tot);
  if (threadIdx.x == 0) tileSum[blockIdx.x] = tot;
}
// a 9-byte little-endian record (length u64, char), FN:1708-1709
__device__ __forceinline__ void wr_record(uint8_t* o, unsigned long long len, uint8_t c) {
#pragma unroll
  for (int b = 0; b < 8; b++) o[b] = (uint8_t)(len >> (8 * b));
  o[8] = c;
}
// each element emits its runs at its prefix; a run's record is written by the
// element that starts the next run (its length is then known) or, for the
// last run, by the last element
__global__ void __launch_bounds__(256) k_el_wr_emit_tiles(ElemArgs A, uint32_t V, const WrState* __restrict__ tilePre,
                                                         uint8_t* __restrict__ rec,
                                                         unsigned long long* __restrict__ total,
                                                         const uint4* __restrict__ segIn) {
  const uint32_t e = blockIdx.x * 256 + threadIdx.x;
  ElemSegs g{0u, 0u, 0u, 0u, 0ull, 0ull, 0ull};
  if (e < V) g = segIn ? segs_unpack(segIn[e]) : d_elem_collect(A, e);
  const WrState ex = WrOp{}(tilePre[blockIdx.x], wr_block_exscan(g.state(), nullptr));
  int prev = (ex.hl >> 16) ? (int)((ex.hl >> 8) & 0xffu) : -1;
  unsigned long long j = ex.runs, pos = ex.sym, start = ex.lastStart;
#pragma unroll
  for (uint32_t k = 0; k < 3; k++)
    if (k < g.n) {
      const uint32_t c = g.ch(k);
      if ((int)c != prev) {
        if (j) wr_record(rec + 9 * (j - 1), pos - start, (uint8_t)prev);
        start = pos;
        j++;
      }
      prev = (int)c;
      pos += g.cnt(k);
    }
  if (e + 1 == V) {
    if (j) wr_record(rec + 9 * (j - 1), pos - start, (uint8_t)prev);
    total[0] = j;
    total[1] = pos;
  }
}
void mk_el_wr_tiles(const ElemIn& w, uint32_t V, WrState* tileSum, hipStream_t st, uint4* segOut) {
  if (V)
    hipLaunchKernelGGL(k_el_wr_tiles, dim3((V + 255) / 256), dim3(256), 0, st, elem_args(w), V, tileSum, segOut);
}
void mk_el_wr_emit_tiles(const ElemIn& w, uint32_t V, const WrState* tilePre, uint8_t* rec,
                         unsigned long long* total, hipStream_t st, const uint4* segIn) {
  if (V)
    hipLaunchKernelGGL(k_el_wr_emit_tiles, dim3((V + 255) / 256), dim3(256), 0, st, elem_args(w), V, tilePre, rec,
                       total, segIn);
}

__global__ void k_el_wr_count(ElemArgs A, uint32_t V, uint32_t* __restrict__ runs, unsigned long long* __restrict__ sym,
                              uint32_t* __restrict__ hl, uint4* __restrict__ segs) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= V) return;
  if (segs) {  // the segments kept for the emission (sharded writer, round 6)
    const ElemSegs g = d_elem_collect(A, e);
    const WrState w = g.state();
    runs[e] = (uint32_t)w.runs;
    sym[e] = w.sym;
    hl[e] = w.hl;
    segs[e] = segs_pack(g);
    return;
  }
  int prev = -1, first = -1;
  uint32_t nr = 0;
  unsigned long long ns = 0;
  d_elem_segments(A, e, [&](uint8_t c, unsigned long long cnt) {
    if (first < 0) first = c;
    if ((int)c != prev) nr++;
    prev = c;
    ns += cnt;
  });
  runs[e] = nr;
  sym[e] = ns;
  hl[e] = first < 0 ? 0u : (1u << 16) | ((uint32_t)prev << 8) | (uint32_t)first;
}
__global__ void k_el_wr_emit(ElemArgs A, uint32_t V, const unsigned long long* __restrict__ runOff,
                             const unsigned long long* __restrict__ symOff, const uint32_t* __restrict__ prevHL,
                             unsigned long long* __restrict__ runStart, uint8_t* __restrict__ runChar) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= V) return;
  const uint32_t pv = prevHL[e];
  int prev = (pv >> 16) ? (int)((pv >> 8) & 0xff) : -1;
  // symOff == nullptr: one packed scan, run offset << kPackSymBits | symbol offset
  unsigned long long j, pos;
  if (symOff) {
    j = runOff[e];
    pos = symOff[e];
  } else {
    const unsigned long long v = runOff[e];
    j = v >> kPackSymBits;
    pos = v & ((1ull << kPackSymBits) - 1);
  }
  d_elem_segments(A, e, [&](uint8_t c, unsigned long long cnt) {
    if ((int)c != prev) {
      runStart[j] = pos;
      runChar[j] = c;
      j++;
    }
    prev = c;
    pos += cnt;
  });
}

// ---- element writer of the position-sharded merge (dist_merge.hip): the
// elements of the SA ranks whose position this rank owns (P0 <= SA[r] < P1;
// the E end phrases belong to the owner of position n-1), head characters by
// local slot.  Elements of one SA rank form one writer unit; every element of
// a unit with heads emits its head's character, so all of them are non-empty.
__device__ __forceinline__ bool d_owns(uint32_t p, uint32_t P0, uint32_t P1) { return p >= P0 && p < P1; }

__global__ void k_dm_el_count(const int32_t* __restrict__ sa, const uint32_t* __restrict__ posBegin,
                              const uint32_t* __restrict__ slot, uint32_t n, uint32_t E, uint32_t P0, uint32_t P1,
                              uint32_t* __restrict__ m) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  if (r == 0) { m[0] = d_owns(n - 1, P0, P1) ? E : 0u; return; }
  const uint32_t p = (uint32_t)sa[r];
  if (!d_owns(p, P0, P1)) { m[r] = 0; return; }
  const uint32_t nh = slot[posBegin[p + 1]] - slot[posBegin[p]];
  m[r] = max(nh, 1u);
}

// k_el_info's fields from local slots: heads of rank r, slot base of its
// position (for r = 0: of the end phrases' item at n-1)
__global__ void k_dm_el_info(const int32_t* __restrict__ sa, const uint8_t* __restrict__ bwt,
                             const int64_t* __restrict__ bucket, const uint32_t* __restrict__ posBegin,
                             const uint32_t* __restrict__ slot, const uint32_t* __restrict__ elemBase, uint32_t n,
                             uint32_t E, uint32_t P0, uint32_t P1, uint4* __restrict__ info1,
                             unsigned long long* __restrict__ info2) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint32_t nh = 0, s0 = 0;
  unsigned long long j = 0;
  if (r == 0) {
    if (d_owns(n - 1, P0, P1)) { nh = E; s0 = slot[posBegin[n - 1]]; }
  } else {
    const uint32_t p = (uint32_t)sa[r];
    if (d_owns(p, P0, P1)) {
      const int64_t b = bucket[p];
      nh = slot[posBegin[p + 1]] - slot[posBegin[p]];
      if (b < 0 && nh) s0 = slot[posBegin[p]];
      j = ((unsigned long long)b & 0x00ffffffffffffffull) | ((unsigned long long)bwt[r] << 56);
    }
  }
  info1[r] = make_uint4(elemBase[r], nh, s0, 0u);
  info2[r] = j;
}

// runs of each element less one when its first segment continues the
// previous element of the same unit (SA rank r >= 1)
__global__ void k_dm_el_adj(const uint32_t* __restrict__ rOf, const uint32_t* __restrict__ hl,
                            const uint32_t* __restrict__ runs, uint32_t V, uint32_t* __restrict__ adj) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= V) return;
  const uint32_t a = hl[e];
  uint32_t j = 0;
  if (e > 0 && rOf[e] != 0 && rOf[e - 1] == rOf[e]) {
    const uint32_t pv = hl[e - 1];
    j = ((a >> 16) && (pv >> 16) && (a & 0xff) == ((pv >> 8) & 0xff)) ? 1u : 0u;
  }
  adj[e] = runs[e] - j;
}

// writer units (hl << 32 | runs, symbols) from the elements: units u < E are
// the end phrases (one element each), unit E + r - 1 the elements of SA rank
// r; zero for units of other ranks.  runIn / symIn: inclusive scans over the
// elements of adj and sym.
// inclusive run / symbol scans of the elements: two arrays, or one packed
// array (runs << kPackSymBits | symbols) when sym == nullptr
struct ElemScan {
  const unsigned long long* run;
  const unsigned long long* sym;
  __device__ unsigned long long r(uint32_t i) const { return sym ? run[i] : run[i] >> kPackSymBits; }
  __device__ unsigned long long s(uint32_t i) const {
    return sym ? sym[i] : run[i] & ((1ull << kPackSymBits) - 1);
  }
};
__global__ void k_dm_el_units(const uint32_t* __restrict__ elemBase, const uint32_t* __restrict__ m,
                              const unsigned long long* __restrict__ runIn, const unsigned long long* __restrict__ symIn,
                              const uint32_t* __restrict__ hl, uint32_t n, uint32_t E, uint32_t U,
                              int64_t* __restrict__ out) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  uint32_t e0, e1;
  if (u < E) {
    if (!m[0]) { out[u] = 0; out[(uint64_t)U + u] = 0; return; }
    e0 = elemBase[0] + u;
    e1 = e0 + 1;
  } else {
    const uint32_t r = u - E + 1;
    if (!m[r]) { out[u] = 0; out[(uint64_t)U + u] = 0; return; }
    e0 = elemBase[r];
    e1 = e0 + m[r];
  }
  const ElemScan es{runIn, symIn};
  const unsigned long long rb = e0 ? es.r(e0 - 1) : 0ull, sb = e0 ? es.s(e0 - 1) : 0ull;
  const uint32_t nr = (uint32_t)(es.r(e1 - 1) - rb);
  const unsigned long long ns = es.s(e1 - 1) - sb;
  const uint32_t hf = hl[e0], hlast = hl[e1 - 1];
  const uint32_t h = (hf >> 16) ? ((1u << 16) | (hlast & 0xff00u) | (hf & 0xffu)) : 0u;
  out[u] = (int64_t)(((uint64_t)h << 32) | nr);
  out[(uint64_t)U + u] = (int64_t)ns;
}

// emission: an element's first run index and symbol offset from its unit's
// (unitRunOff: global run index, or the rank-local stream index; the unit's
// first segment continues the previous unit's run when `joined`), the
// character before it from the previous element of its unit or, for a unit's
// first element, from the previous non-empty unit (prevHL, over all ranks)
__global__ void k_dm_el_emit(ElemArgs A, uint32_t V, const uint32_t* __restrict__ elemBase,
                             const unsigned long long* __restrict__ runIn, const unsigned long long* __restrict__ symIn,
                             const unsigned long long* __restrict__ unitRunOff,
                             const unsigned long long* __restrict__ unitSymOff, const uint32_t* __restrict__ prevHL,
                             const uint32_t* __restrict__ unitHL, const uint32_t* __restrict__ hl,
                             unsigned long long* __restrict__ runStart, uint8_t* __restrict__ runChar,
                             const uint4* __restrict__ segs) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= V) return;
  const uint32_t r = A.rOf[e];
  const uint32_t u = r ? A.E + r - 1 : e - elemBase[0];
  const uint32_t e0 = r ? elemBase[r] : e;
  const uint32_t pu = prevHL[u], hu = unitHL[u];
  const ElemScan es{runIn, symIn};
  int prev;
  unsigned long long j = unitRunOff[u];
  if (e == e0) {
    prev = (pu >> 16) ? (int)((pu >> 8) & 0xff) : -1;
  } else {
    prev = (int)((hl[e - 1] >> 8) & 0xff);
    const bool joined = (hu >> 16) && (pu >> 16) && (hu & 0xff) == ((pu >> 8) & 0xff);
    j += es.r(e - 1) - (e0 ? es.r(e0 - 1) : 0ull) - (joined ? 1u : 0u);
  }
  unsigned long long pos = unitSymOff[u] + (e ? es.s(e - 1) : 0ull) - (e0 ? es.s(e0 - 1) : 0ull);
  auto put = [&](uint8_t c, unsigned long long cnt) {
    if ((int)c != prev) {
      runStart[j] = pos;
      runChar[j] = c;
      j++;
    }
    prev = c;
    pos += cnt;
  };
  if (segs) {  // read back sequentially instead of re-gathering the per-slot inputs
    const ElemSegs g = segs_unpack(segs[e]);
#pragma unroll
    for (uint32_t k = 0; k < 3; k++)
      if (k < g.n) put((uint8_t)g.ch(k), g.cnt(k));
  } else {
    d_elem_segments(A, e, put);
  }
}






__global__ void k_count_distinct(const uint32_t* __restrict__ v, uint32_t K, unsigned long long* __restrict__ out) {
  __shared__ unsigned int acc;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  uint32_t c = 0;  // grid-stride: one global atomic per block, few blocks
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < K; q += (uint64_t)gridDim.x * blockDim.x)
    c += (q == 0 || v[q] != v[q - 1]) ? 1u : 0u;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&acc, c);
  __syncthreads();
  if (threadIdx.x == 0 && acc) atomicAdd(out, (unsigned long long)acc);
}

// ------------------------------------------------------------ launchers

// ---- stream compaction (order-preserving select of flagged u32 values).
// Tiles of kSelRows x 256 elements: pass 1 counts each tile's flagged
// elements, an exclusive scan gives the tile offsets, pass 2 ranks each row
// by wave ballots and writes the kept values (replaces rocprim::select, which
// ran at ~1/8 of the bandwidth this needs).
constexpr uint32_t kSelRows = 8, kSelTile = kSelRows * 256;
template <class F>
__global__ void __launch_bounds__(256) k_sel_count(const F* __restrict__ flags, uint32_t n,
                                                   uint32_t* __restrict__ tileCnt) {
  __shared__ uint32_t wc[4];
  const uint64_t t0 = (uint64_t)blockIdx.x * kSelTile;
  uint32_t c = 0;
#pragma unroll
  for (uint32_t j = 0; j < kSelRows; j++) {
    const uint64_t e = t0 + j * 256 + threadIdx.x;
    c += (e < n && flags[e] != 0) ? 1u : 0u;
  }
  for (uint32_t d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, (int)d);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tileCnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}
// in == nullptr: the kept indices themselves
template <class F>
__global__ void __launch_bounds__(256) k_sel_write(const uint32_t* __restrict__ in, const F* __restrict__ flags,
                                                   uint32_t n, const uint32_t* __restrict__ tileOff,
                                                   uint32_t* __restrict__ out) {
  __shared__ uint32_t wc[kSelRows][4];
  const uint64_t t0 = (uint64_t)blockIdx.x * kSelTile;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  bool keep[kSelRows];
  uint32_t rk[kSelRows];
#pragma unroll
  for (uint32_t j = 0; j < kSelRows; j++) {
    const uint64_t e = t0 + j * 256 + threadIdx.x;
    keep[j] = e < n && flags[e] != 0;
    const uint64_t m = __ballot(keep[j]);
    rk[j] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (lane == 0) wc[j][wv] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  uint32_t base = tileOff[blockIdx.x];
#pragma unroll
  for (uint32_t j = 0; j < kSelRows; j++) {
    uint32_t before = 0;
    for (uint32_t w = 0; w < wv; w++) before += wc[j][w];
    const uint32_t e = (uint32_t)(t0 + j * 256 + threadIdx.x);
    if (keep[j]) out[base + before + rk[j]] = in ? in[e] : e;
    base += wc[j][0] + wc[j][1] + wc[j][2] + wc[j][3];
  }
}

// ---- u32 plus scans (exclusive / inclusive), two passes over tiles of 2048:
// tile sums, a scan of the sums, then each thread scans its 8 contiguous
// values (two 16-byte loads) under a block scan of the thread totals.
// (rocprim's lookback scan ran at ~1.3 TB/s on these arrays.)
constexpr uint32_t kScanIpt = 8, kScanTile = 256 * kScanIpt;
__device__ __forceinline__ void scan_load8(const uint32_t* __restrict__ in, uint64_t e, uint64_t n, bool vec,
                                           uint32_t v[kScanIpt]) {
  if (vec && e + kScanIpt <= n) {
    const uint4 a = *reinterpret_cast<const uint4*>(in + e), b = *reinterpret_cast<const uint4*>(in + e + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanIpt; k++) v[k] = e + k < n ? in[e + k] : 0u;
  }
}
__global__ void __launch_bounds__(256) k_scan_sums(const uint32_t* __restrict__ in, uint64_t n, int vec,
                                                   uint32_t* __restrict__ sums) {
  __shared__ uint32_t wsum[4];
  const uint64_t e = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanIpt;
  uint32_t v[kScanIpt];
  scan_load8(in, e, n, vec != 0, v);
  uint32_t c = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanIpt; k++) c += v[k];
  for (uint32_t d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, (int)d);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) sums[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}
__global__ void __launch_bounds__(256) k_scan_tiles(const uint32_t* in, uint32_t* out, uint64_t n, int vec,
                                                    const uint32_t* __restrict__ tileOff, uint32_t init,
                                                    int inclusive) {
  __shared__ uint32_t wsum[4];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t e = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanIpt;
  uint32_t v[kScanIpt];
  scan_load8(in, e, n, vec != 0, v);
  uint32_t tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanIpt; k++) tot += v[k];
  uint32_t inc = tot;  // inclusive scan of the thread totals in the wave
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t base = init + tileOff[blockIdx.x] + (inc - tot);
  for (uint32_t w = 0; w < wv; w++) base += wsum[w];
  uint32_t r[kScanIpt];
#pragma unroll
  for (uint32_t k = 0; k < kScanIpt; k++) {
    if (inclusive) { base += v[k]; r[k] = base; }
    else { r[k] = base; base += v[k]; }
  }
  if (vec != 0 && e + kScanIpt <= n) {
    *reinterpret_cast<uint4*>(out + e) = make_uint4(r[0], r[1], r[2], r[3]);
    *reinterpret_cast<uint4*>(out + e + 4) = make_uint4(r[4], r[5], r[6], r[7]);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanIpt; k++)
      if (e + k < n) out[e + k] = r[k];
  }
}
// the same two passes over u64 values plus a constant: the writer's
// cumulative counters (FN:1504-1515's prefix sums over counter + 1)
__device__ __forceinline__ void scan_load8_u64(const unsigned long long* __restrict__ in, uint64_t e, uint64_t n,
                                               bool vec, uint32_t add, unsigned long long v[kScanIpt]) {
  if (vec && e + kScanIpt <= n) {
    const ulonglong2* i2 = reinterpret_cast<const ulonglong2*>(in + e);
#pragma unroll
    for (uint32_t k = 0; k < kScanIpt / 2; k++) {
      const ulonglong2 a = i2[k];
      v[2 * k] = a.x + add;
      v[2 * k + 1] = a.y + add;
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanIpt; k++) v[k] = e + k < n ? in[e + k] + add : 0ull;
  }
}
__global__ void __launch_bounds__(256) k_scan64_sums(const unsigned long long* __restrict__ in, uint64_t n, int vec,
                                                     uint32_t add, unsigned long long* __restrict__ sums) {
  __shared__ unsigned long long wsum[4];
  const uint64_t e = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanIpt;
  unsigned long long v[kScanIpt];
  scan_load8_u64(in, e, n, vec != 0, add, v);
  unsigned long long c = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanIpt; k++) c += v[k];
  for (uint32_t d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, (int)d);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) sums[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}
__global__ void __launch_bounds__(256) k_scan64_tiles(const unsigned long long* in, unsigned long long* out,
                                                      uint64_t n, int vec,
                                                      const unsigned long long* __restrict__ tileOff, uint32_t add,
                                                      int inclusive) {
  __shared__ unsigned long long wsum[4];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t e = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanIpt;
  unsigned long long v[kScanIpt];
  scan_load8_u64(in, e, n, vec != 0, add, v);
  unsigned long long tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanIpt; k++) tot += v[k];
  unsigned long long inc = tot;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const unsigned long long o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  unsigned long long base = tileOff[blockIdx.x] + (inc - tot);
  for (uint32_t w = 0; w < wv; w++) base += wsum[w];
  unsigned long long r[kScanIpt];
#pragma unroll
  for (uint32_t k = 0; k < kScanIpt; k++) {
    if (inclusive) { base += v[k]; r[k] = base; }
    else { r[k] = base; base += v[k]; }
  }
  if (vec != 0 && e + kScanIpt <= n) {
    ulonglong2* o2 = reinterpret_cast<ulonglong2*>(out + e);
#pragma unroll
    for (uint32_t k = 0; k < kScanIpt / 2; k++) o2[k] = make_ulonglong2(r[2 * k], r[2 * k + 1]);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanIpt; k++)
      if (e + k < n) out[e + k] = r[k];
  }
}
static inline dim3 g1(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }
uint64_t scan_tiles(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }
void mk_scan64_sums(const unsigned long long* in, uint64_t n, uint32_t add, unsigned long long* sums, hipStream_t st) {
  const int vec = (((uintptr_t)in) & 15) == 0;
  if (n) hipLaunchKernelGGL(k_scan64_sums, dim3((unsigned)scan_tiles(n)), dim3(256), 0, st, in, n, vec, add, sums);
}
void mk_scan64_tiles(const unsigned long long* in, unsigned long long* out, uint64_t n, const unsigned long long* tileOff,
                     uint32_t add, bool inclusive, hipStream_t st) {
  const int vec = ((((uintptr_t)in) | ((uintptr_t)out)) & 15) == 0;
  if (n)
    hipLaunchKernelGGL(k_scan64_tiles, dim3((unsigned)scan_tiles(n)), dim3(256), 0, st, in, out, n, vec, tileOff,
                       add, inclusive ? 1 : 0);
}
void mk_scan_sums(const uint32_t* in, uint64_t n, uint32_t* sums, hipStream_t st) {
  const int vec = (((uintptr_t)in) & 15) == 0;
  if (n) hipLaunchKernelGGL(k_scan_sums, dim3((unsigned)scan_tiles(n)), dim3(256), 0, st, in, n, vec, sums);
}
void mk_scan_tiles(const uint32_t* in, uint32_t* out, uint64_t n, const uint32_t* tileOff, uint32_t init,
                   bool inclusive, hipStream_t st) {
  const int vec = ((((uintptr_t)in) | ((uintptr_t)out)) & 15) == 0;
  if (n)
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)scan_tiles(n)), dim3(256), 0, st, in, out, n, vec, tileOff, init,
                       inclusive ? 1 : 0);
}

uint32_t sel_tiles(uint32_t n) { return (uint32_t)(((uint64_t)n + kSelTile - 1) / kSelTile); }
void mk_sel_count(const uint32_t* flags, uint32_t n, uint32_t* tileCnt, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_sel_count<uint32_t>, dim3(sel_tiles(n)), dim3(256), 0, st, flags, n, tileCnt);
}
void mk_sel_write(const uint32_t* in, const uint32_t* flags, uint32_t n, const uint32_t* tileOff, uint32_t* out,
                  hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_sel_write<uint32_t>, dim3(sel_tiles(n)), dim3(256), 0, st, in, flags, n, tileOff, out);
}
// flags in bit 31 of u32 words (k_ranks_slot's sa entries)
struct Bit31 {
  uint32_t v;
  __device__ bool operator!=(int) const { return (v >> 31) != 0; }
};
void mk_sel_count31(const uint32_t* words, uint32_t n, uint32_t* tileCnt, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_sel_count<Bit31>, dim3(sel_tiles(n)), dim3(256), 0, st, (const Bit31*)words, n, tileCnt);
}
void mk_sel_write_idx31(const uint32_t* words, uint32_t n, const uint32_t* tileOff, uint32_t* out, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_sel_write<Bit31>, dim3(sel_tiles(n)), dim3(256), 0, st, nullptr, (const Bit31*)words, n,
                       tileOff, out);
}
__global__ void k_and_u32(uint32_t* __restrict__ p, uint64_t n, uint32_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] &= m;
}
void mk_and_u32(uint32_t* p, uint64_t n, uint32_t m, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_and_u32, g1(n), dim3(256), 0, st, p, n, m);
}
void mk_sel_count8(const uint8_t* flags, uint32_t n, uint32_t* tileCnt, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_sel_count<uint8_t>, dim3(sel_tiles(n)), dim3(256), 0, st, flags, n, tileCnt);
}
void mk_sel_write_idx8(const uint8_t* flags, uint32_t n, const uint32_t* tileOff, uint32_t* out, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_sel_write<uint8_t>, dim3(sel_tiles(n)), dim3(256), 0, st, nullptr, flags, n, tileOff, out);
}


void mk_iota(uint32_t* p, uint64_t n, hipStream_t st) { if (n) hipLaunchKernelGGL(k_iota, g1(n), dim3(256), 0, st, p, n); }
void mk_gather(const uint32_t* src, const uint32_t* perm, uint32_t* dst, uint64_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_gather_u32, g1(n), dim3(256), 0, st, src, perm, dst, n);
}
void mk_item_flags(const uint32_t* perm, const HeadsSoA& h, uint32_t* flag, uint64_t H, hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_item_flags, g1(H), dim3(256), 0, st, perm, h.pos, h.len, h.isa, flag, H);
}
void mk_item_fill(const uint32_t* perm, const uint32_t* flag, const uint32_t* incl, const HeadsSoA& h,
                  uint64_t H, const ItemsSoA& it, hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_item_fill, g1(H), dim3(256), 0, st, perm, flag, incl, h, H, it);
}
void mk_group_key(const HeadsSoA& h, uint64_t H, int bN, int bL, unsigned long long* key, hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_group_key, g1(H), dim3(256), 0, st, h, H, bN, bL, key);
}
void mk_item_flags64(const unsigned long long* key, uint32_t* flag, uint64_t H, hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_item_flags64, g1(H), dim3(256), 0, st, key, flag, H);
}
void mk_item_fill64(const unsigned long long* key, const uint32_t* perm, const uint32_t* flag, const uint32_t* incl,
                    const HeadsSoA& h, const uint32_t* tsS,
                    const uint8_t* smS, uint64_t H, int bN, int bL, const ItemsSoA& it, hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_item_fill64, g1(H), dim3(256), 0, st, key, perm, flag, incl, h, tsS, smS, H, bN, bL, it);
}
void mk_slot_mark(const uint32_t* slot, uint32_t K, uint32_t* mark, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_slot_mark, g1(K), dim3(256), 0, st, slot, K, mark);
}
void mk_slot_members(const ItemsSoA& it, const uint32_t* itemOfSlot, const uint32_t* perm, uint32_t H, uint32_t* Pm,
                     hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_slot_members, g1(H), dim3(256), 0, st, it, itemOfSlot, perm, H, Pm);
}
void mk_pos_rank_base(const uint32_t* posBegin, const uint32_t* slot, const uint32_t* isaRef,
                      const uint32_t* itemRankBase, const uint32_t* headBase, uint32_t n, uint32_t E,
                      uint32_t* rankBase, uint32_t* gBase, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_pos_rank_base, g1(n), dim3(256), 0, st, posBegin, slot, isaRef, itemRankBase, headBase, n, E,
                       rankBase, gBase);
}
void mk_ranks_slot(const ItemsSoA& it, const uint32_t* itemOfSlot, const uint32_t* Pm, uint32_t H,
                   const uint32_t* rankBase, const uint32_t* gBase, uint32_t n, int32_t* T, uint32_t* sa,
                   uint32_t* grp, uint32_t* actv, hipStream_t st, uint32_t* gItem, uint8_t* unres, uint32_t saFlag) {
  if (H)
    hipLaunchKernelGGL(k_ranks_slot, g1(H), dim3(256), 0, st, it, itemOfSlot, Pm, H, rankBase, gBase, n, T, sa, grp,
                       actv, gItem, unres, saFlag);
}
void mk_head_chars_slot(const uint32_t* Pm, const uint32_t* grp, const uint8_t* lchar, const ItemsSoA& it,
                        const uint32_t* itemOfSlot, const uint32_t* gItem, uint32_t H, uint8_t* bwtSlot,
                        hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_head_chars_slot, g1(H), dim3(256), 0, st, Pm, grp, lchar, it, itemOfSlot, gItem, H,
                            bwtSlot);
}
void mk_nhr_rec(const uint32_t* grp, const uint16_t* nexthead, const uint8_t* lchar, uint32_t H, uint4* rec,
                hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_nhr_rec, g1(H), dim3(256), 0, st, grp, nexthead, lchar, H, rec);
}
void mk_head_chars(const uint32_t* sa, const uint8_t* lchar, uint32_t H, uint8_t* bwtHeads, hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_head_chars, g1(H), dim3(256), 0, st, sa, lchar, H, bwtHeads);
}
void mk_nhr_idx(const uint32_t* headRank, uint32_t sub, const uint16_t* nexthead, uint32_t H, uint32_t* nbi,
                hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_nhr_idx, g1(H), dim3(256), 0, st, headRank, sub, nexthead, H, nbi);
}
void mk_nhr_slot(const uint32_t* Pm, const uint32_t* headRank, uint32_t sub, const uint16_t* nexthead, uint32_t H,
                 uint32_t* nbi, uint32_t* nhr, hipStream_t st) {
  if (!H) return;
  hipLaunchKernelGGL(k_nhr_idx, g1(H), dim3(256), 0, st, headRank, sub, nexthead, H, nbi);
  hipLaunchKernelGGL(k_nhr_slot, g1(H), dim3(256), 0, st, Pm, nbi, H, nhr);
}
void mk_nhr_rank(const uint32_t* Pm, const uint32_t* nbi, const uint32_t* itemOfSlot, uint32_t H, uint32_t* nhr,
                 hipStream_t st, const uint4* rec, const uint32_t* slot, const uint32_t* gItem, uint8_t* bwtSlot) {
  if (H) hipLaunchKernelGGL(k_nhr_rank, dim3((H + kNhrBlock - 1) / kNhrBlock), dim3(kNhrBlock), 0, st, Pm, nbi,
                            itemOfSlot, H, nhr, rec, slot, gItem, bwtSlot);
}
// items of more than kSmallSeg members, for the big path
__global__ void k_nhr_big_list(const ItemsSoA it, uint32_t K, uint32_t* __restrict__ bigList) {
  uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < K && it.count[q] > kSmallSeg) bigList[1 + atomicAdd(bigList, 1u)] = q;
}
void mk_nhr_big_list(const ItemsSoA& it, uint32_t K, uint32_t* bigList, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_nhr_big_list, g1(K), dim3(256), 0, st, it, K, bigList);
}
void mk_nhr_sort_small(const ItemsSoA& it, uint32_t K, uint32_t* nhr, uint32_t* bigList, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_nhr_sort_small, g1(K), dim3(256), 0, st, it, K, nhr, bigList);
}
void mk_nhr_big_fill(const uint32_t* items, const uint32_t* off, uint32_t nb, const ItemsSoA& it, const uint32_t* nhr,
                     unsigned long long* key, uint32_t* slots, hipStream_t st) {
  if (nb) hipLaunchKernelGGL(k_nhr_big_fill, dim3(nb), dim3(256), 0, st, items, off, it, nhr, key, slots);
}
void mk_item_counts_of(const uint32_t* items, uint32_t nb, const uint32_t* count, uint32_t* out, hipStream_t st) {
  if (nb) hipLaunchKernelGGL(k_item_counts_of, g1(nb), dim3(256), 0, st, items, nb, count, out);
}
void mk_nhr_big_back(const unsigned long long* sorted, const uint32_t* slots, uint32_t B, uint32_t* nhr,
                     hipStream_t st) {
  if (B) hipLaunchKernelGGL(k_nhr_big_back, g1(B), dim3(256), 0, st, sorted, slots, B, nhr);
}
void mk_item_count(const uint32_t* first, uint32_t* count, uint32_t K, uint32_t H, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_item_count, g1(K), dim3(256), 0, st, first, count, K, H);
}
void mk_item_permute(const ItemsSoA& in, const uint32_t* order, const ItemsSoA& out, uint32_t K, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_item_permute, g1(K), dim3(256), 0, st, in, order, out, K);
}
void mk_pos_begin(const uint32_t* ipos, uint32_t K, uint32_t n, uint32_t* posBegin, hipStream_t st) {
  hipLaunchKernelGGL(k_pos_ends, g1((uint64_t)n + 1), dim3(256), 0, st, ipos, K, n, posBegin);
  if (K > 1) hipLaunchKernelGGL(k_pos_begin, g1(K), dim3(256), 0, st, ipos, K, n, posBegin);
}
void mk_pos_f(const uint32_t* ipos, const uint8_t* ism, const uint32_t* posBegin, uint32_t K, uint32_t n,
              uint32_t* posF, hipStream_t st) {
  hipLaunchKernelGGL(k_pos_f, g1(n), dim3(256), 0, st, ipos, ism, posBegin, K, n, posF);
}
void mk_check_items(const ItemsSoA& it, const uint32_t* posBegin, const uint32_t* posF, uint32_t K,
                    unsigned long long* viol, uint8_t* amb, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_check_items, g1(K), dim3(256), 0, st, it, posBegin, posF, K, viol, amb);
}
void mk_sa_counts(const int32_t* sa, const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t E,
                  uint32_t* itemsSA, uint32_t* headsSA, hipStream_t st) {
  hipLaunchKernelGGL(k_sa_counts, g1(n), dim3(256), 0, st, sa, posBegin, slot, n, E, itemsSA, headsSA);
}
void mk_dbl_keys(const uint32_t* act, const uint32_t* sa, const uint32_t* grp, uint32_t h, uint32_t U,
                 uint64_t* key, uint32_t* val, hipStream_t st, uint32_t saMask) {
  if (U) hipLaunchKernelGGL(k_dbl_keys, g1(U), dim3(256), 0, st, act, sa, grp, h, U, key, val, saMask);
}
void mk_dbl_apply(const uint32_t* act, const uint64_t* key, const uint32_t* val, uint32_t U, uint32_t* sa,
                  uint32_t* lab, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dbl_apply, g1(U), dim3(256), 0, st, act, key, val, U, sa, lab);
}
void mk_dbl_groups(const uint32_t* act, const uint64_t* key, const uint32_t* val, const uint32_t* labMax,
                   uint32_t U, uint32_t* grp, uint32_t* keep, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dbl_groups, g1(U), dim3(256), 0, st, act, key, val, labMax, U, grp, keep);
}
void mk_map_order(const uint32_t* posBegin, const uint32_t* len, const uint8_t* sm, uint32_t n, uint32_t* order,
                  hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_map_order, g1(n), dim3(256), 0, st, posBegin, len, sm, n, order);
}
void mk_dbl_gstart(const uint64_t* key, uint32_t U, uint32_t* flag, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dbl_gstart, g1(U), dim3(256), 0, st, key, U, flag);
}
void mk_dbl_rank(uint32_t U, const uint32_t* act, const uint64_t* key, const uint32_t* val, uint32_t* sa,
                 uint32_t* grp, uint32_t* keep, uint32_t* bigList, uint32_t maxSmall, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dbl_rank, dim3((U + kDblBlock - 1) / kDblBlock), dim3(kDblBlock), 0, st, U, act, key, val,
                            sa, grp, keep, bigList, maxSmall);
}
void mk_dbl_small2(const uint32_t* gflag, uint32_t U, const uint32_t* act, uint64_t* key, uint32_t* val, uint32_t* sa,
                   uint32_t* grp, uint32_t* keep, uint32_t* bigList, uint32_t maxSmall, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dbl_small2, g1(U), dim3(256), 0, st, gflag, U, act, key, val, sa, grp, keep, bigList, maxSmall);
}
void mk_dbl_gather_big(const uint32_t* orig, uint32_t B, const uint32_t* act, const uint64_t* key, const uint32_t* val,
                       uint32_t* actB, uint64_t* keyB, uint32_t* valB, hipStream_t st) {
  if (B) hipLaunchKernelGGL(k_dbl_gather_big, g1(B), dim3(256), 0, st, orig, B, act, key, val, actB, keyB, valB);
}
void mk_scatter_u32(const uint32_t* src, const uint32_t* idx, uint32_t n, uint32_t* dst, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_scatter_u32, g1(n), dim3(256), 0, st, src, idx, n, dst);
}
void mk_win_flags(const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t P0, uint32_t P1,
                  uint32_t winPos, uint32_t slotCap, uint32_t* flag, hipStream_t st) {
  hipLaunchKernelGGL(k_win_flags, g1(n), dim3(256), 0, st, posBegin, slot, n, P0, P1, winPos, std::max(1u, slotCap / 2),
                     flag);
}
void mk_win_starts(const uint32_t* flag, const uint32_t* winIncl, uint32_t n, uint32_t* winStart, hipStream_t st) {
  hipLaunchKernelGGL(k_win_starts, g1(n), dim3(256), 0, st, flag, winIncl, n, winStart);
}
void mk_win_cross(const ItemsSoA& it, uint32_t K, const uint32_t* winIncl, uint32_t n, uint32_t* cnt,
                  const uint32_t* off, uint32_t* keyW, uint32_t* valQ, unsigned long long* errs, int fill,
                  hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_win_cross, g1(K), dim3(256), 0, st, it, K, winIncl, n, cnt, off, keyW, valQ, errs,
                            fill);
}
void mk_xw_depth(const uint32_t* posBegin, const uint32_t* winStart, uint32_t P0, uint32_t nsv, const uint32_t* cnt,
                 uint32_t* depth, hipStream_t st) {
  if (nsv) hipLaunchKernelGGL(k_xw_depth, dim3(nsv), dim3(256), 0, st, posBegin, winStart, P0, cnt, depth);
}
void mk_xw_hist(const uint32_t* posBegin, const uint32_t* winStart, uint32_t P0, uint32_t nsv, const uint32_t* cnt,
                const uint32_t* depth, const uint32_t* toff, uint32_t* T, hipStream_t st) {
  if (nsv) hipLaunchKernelGGL(k_xw_hist, dim3(nsv), dim3(256), 0, st, posBegin, winStart, P0, cnt, depth, toff, T);
}
void mk_xw_count(const uint32_t* depth, const uint32_t* toff, const uint32_t* T, uint32_t nw, uint32_t maxDepth,
                 uint32_t* segOff, uint32_t* count, hipStream_t st) {
  if (nw) hipLaunchKernelGGL(k_xw_count, g1(nw), dim3(256), 0, st, depth, toff, T, nw, maxDepth, segOff, count);
}
void mk_xw_place(const uint32_t* posBegin, const uint32_t* winStart, uint32_t P0, uint32_t nsv, const uint32_t* cnt,
                 const uint32_t* depth, const uint32_t* toff, const uint32_t* segOff, const uint32_t* crossOff,
                 uint32_t* crossList, hipStream_t st) {
  if (nsv)
    hipLaunchKernelGGL(k_xw_place, dim3(nsv), dim3(256), 0, st, posBegin, winStart, P0, cnt, depth, toff, segOff,
                       crossOff, crossList);
}
void mk_win_cross_off(const uint32_t* keyW, uint32_t ncross, uint32_t nw, uint32_t* crossOff, hipStream_t st) {
  hipLaunchKernelGGL(k_win_cross_off, g1((uint64_t)nw + 1), dim3(256), 0, st, keyW, ncross, nw, crossOff);
}
void mk_item_sk(const ItemsSoA& it, uint32_t K, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_item_sk, g1(K), dim3(256), 0, st, it, K);
}
void mk_counter_win(const ItemsSoA& it, const uint32_t* posBegin, const uint32_t* posF, const uint32_t* nhr,
                    const uint32_t* winStart, uint32_t nw, const uint32_t* crossOff, const uint32_t* crossList,
                    unsigned long long* counter, unsigned long long* stats, uint32_t n, uint32_t slotCap,
                    const HostRoute* hr, hipStream_t st) {
  if (!nw) return;
  CounterArgs A{it, posBegin, posF, nhr, winStart, crossOff, crossList, counter, stats, n,
                std::min(slotCap, kWinSlots), hr ? *hr : HostRoute{}};
  if (hr) hipLaunchKernelGGL(k_counter_win<true>, dim3(nw), dim3(512), 0, st, A);
  else hipLaunchKernelGGL(k_counter_win<false>, dim3(nw), dim3(512), 0, st, A);
}
void mk_counter_tgt(const ItemsSoA& it, const uint32_t* posBegin, const uint32_t* posF, const uint32_t* nhr,
                    const uint32_t* winStart, uint32_t nw, const uint32_t* crossOff, const uint32_t* crossList,
                    unsigned long long* counter, unsigned long long* stats, uint32_t n, hipStream_t st,
                    EqList eq, const uint4* irec) {
  if (!nw) return;
  CounterArgs A{it, posBegin, posF, nhr, winStart, crossOff, crossList, counter, stats, n, 0u, HostRoute{}, eq,
                irec};
  hipLaunchKernelGGL(k_counter_tgt, dim3(nw), dim3(256), 0, st, A);
}
// FN:1537-1589 for the listed equal-key queries (the branch of
// d_counter_query_L that reads the next-head ranks)
__global__ void k_counter_eq(const uint4* __restrict__ rec, uint32_t m, const uint32_t* __restrict__ nhr,
                             unsigned long long* __restrict__ counter, unsigned long long* __restrict__ stats) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool good = false, bad = false;
  if (i < m) {
    const uint4 r = rec[i];
    const uint32_t slq = r.x, cq = r.y, so = r.z, co = r.w & 0x7fffffffu;
    const bool hasNext = (r.w >> 31) != 0;
    const uint32_t* me = nhr + slq;
    const uint32_t* ot = nhr + so;
    if (me[cq - 1] < ot[0]) {
      atomicAdd(&counter[so], (unsigned long long)cq);
      good = true;
    } else if (me[0] > ot[co - 1]) {
      if (hasNext) atomicAdd(&counter[so + co], (unsigned long long)cq);
      good = true;
    } else {
      bad = true;
      uint32_t rest = 0;
      for (uint32_t a = 0; a < cq; a++) {
        const uint32_t bpos = d_upper_u32(ot, 0, co, me[a]);
        if (bpos < co) atomicAdd(&counter[so + bpos], 1ull);
        else rest++;
      }
      if (rest && hasNext) atomicAdd(&counter[so + co], (unsigned long long)rest);
    }
  }
  const uint64_t gm = __ballot(good), bm = __ballot(bad);
  if ((threadIdx.x & 63) == 0) {
    if (bm) atomicAdd(&stats[0], (unsigned long long)__popcll(bm));
    if (gm) atomicAdd(&stats[1], (unsigned long long)__popcll(gm));
  }
}
void mk_counter_eq(const uint4* rec, uint32_t m, const uint32_t* nhr, unsigned long long* counter,
                   unsigned long long* stats, hipStream_t st) {
  if (m) hipLaunchKernelGGL(k_counter_eq, dim3((m + 255) / 256), dim3(256), 0, st, rec, m, nhr, counter, stats);
}
__global__ void k_counter_adds(const uint32_t* __restrict__ slot, const unsigned long long* __restrict__ add, uint32_t m,
                               unsigned long long* __restrict__ counter) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) atomicAdd(&counter[slot[i]], add[i]);
}
void mk_counter_adds(const uint32_t* slot, const unsigned long long* add, uint32_t m, unsigned long long* counter,
                     hipStream_t st) {
  if (m) hipLaunchKernelGGL(k_counter_adds, g1(m), dim3(256), 0, st, slot, add, m, counter);
}
__global__ void k_or_mask(uint8_t* __restrict__ mask, const uint8_t* __restrict__ other, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) mask[i] |= other[i];
}
void mk_or_mask(uint8_t* mask, const uint8_t* other, uint32_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_or_mask, g1(n), dim3(256), 0, st, mask, other, n);
}
void mk_count_distinct(const uint32_t* v, uint32_t K, unsigned long long* out, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_count_distinct, dim3(std::min<unsigned>(2048, g1(K).x)), dim3(256), 0, st, v, K, out);
}
void mk_bucket(const int32_t* countIncl, const uint8_t* hasHead, uint32_t n, int64_t* bucket, hipStream_t st) {
  hipLaunchKernelGGL(k_bucket, g1(n), dim3(256), 0, st, countIncl, hasHead, n, bucket);
}
void mk_wr_adjust(const uint32_t* hl, const uint32_t* prevHL, uint32_t U, uint32_t* runs, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_wr_adjust, g1(U), dim3(256), 0, st, hl, prevHL, U, runs);
}
void mk_win_fixed(uint32_t n, uint32_t P0, uint32_t P1, uint32_t winPos, uint32_t nw, uint32_t* wincl,
                  uint32_t* winStart, hipStream_t st) {
  const uint64_t m = std::max<uint64_t>(n, (uint64_t)nw + 1);
  hipLaunchKernelGGL(k_win_fixed, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, n, P0, P1, winPos, nw, wincl,
                     winStart);
}
void mk_set_u32(uint32_t* p, uint32_t v, hipStream_t st) { hipLaunchKernelGGL(k_set_u32, dim3(1), dim3(1), 0, st, p, v); }
void mk_el_info(const ElemIn& w, hipStream_t st) {
  if (w.n) hipLaunchKernelGGL(k_el_info, g1(w.n), dim3(256), 0, st, w.sa, w.bwt, w.bucket, w.posBegin, w.slot,
                              w.headBase, w.elemBase, w.n, w.E, w.H, w.info1, w.info2);
}
void mk_el_count(const uint32_t* headBase, uint32_t n, uint32_t E, uint32_t H, uint32_t* m, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_el_count, g1(n), dim3(256), 0, st, headBase, n, E, H, m);
}
void mk_el_rof(const uint32_t* elemBase, const uint32_t* m, uint32_t n, uint32_t* rOf, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_el_rof, g1(n), dim3(256), 0, st, elemBase, m, n, rOf);
}
void mk_el_wr_count(const ElemIn& w, uint32_t V, uint32_t* runs, unsigned long long* sym, uint32_t* hl,
                    hipStream_t st, uint4* segs) {
  if (V) hipLaunchKernelGGL(k_el_wr_count, g1(V), dim3(256), 0, st, elem_args(w), V, runs, sym, hl, segs);
}
void mk_el_wr_emit(const ElemIn& w, uint32_t V, const unsigned long long* runOff, const unsigned long long* symOff,
                   const uint32_t* prevHL, unsigned long long* runStart, uint8_t* runChar, hipStream_t st) {
  if (V) hipLaunchKernelGGL(k_el_wr_emit, g1(V), dim3(256), 0, st, elem_args(w), V, runOff, symOff, prevHL, runStart,
                            runChar);
}
void mk_dm_el_count(const int32_t* sa, const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t E,
                    uint32_t P0, uint32_t P1, uint32_t* m, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_el_count, g1(n), dim3(256), 0, st, sa, posBegin, slot, n, E, P0, P1, m);
}
void mk_dm_el_info(const ElemIn& w, uint32_t P0, uint32_t P1, hipStream_t st) {
  if (w.n) hipLaunchKernelGGL(k_dm_el_info, g1(w.n), dim3(256), 0, st, w.sa, w.bwt, w.bucket, w.posBegin, w.slot,
                              w.elemBase, w.n, w.E, P0, P1, w.info1, w.info2);
}
void mk_dm_el_adj(const uint32_t* rOf, const uint32_t* hl, const uint32_t* runs, uint32_t V, uint32_t* adj,
                  hipStream_t st) {
  if (V) hipLaunchKernelGGL(k_dm_el_adj, g1(V), dim3(256), 0, st, rOf, hl, runs, V, adj);
}
void mk_dm_el_units(const uint32_t* elemBase, const uint32_t* m, const unsigned long long* runIn,
                    const unsigned long long* symIn, const uint32_t* hl, uint32_t n, uint32_t E, uint32_t U,
                    int64_t* out, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dm_el_units, g1(U), dim3(256), 0, st, elemBase, m, runIn, symIn, hl, n, E, U, out);
}
void mk_dm_el_emit(const ElemIn& w, uint32_t V, const unsigned long long* runIn, const unsigned long long* symIn,
                   const unsigned long long* unitRunOff, const unsigned long long* unitSymOff, const uint32_t* prevHL,
                   const uint32_t* unitHL, const uint32_t* hl, unsigned long long* runStart, uint8_t* runChar,
                   hipStream_t st, const uint4* segs) {
  if (V) hipLaunchKernelGGL(k_dm_el_emit, g1(V), dim3(256), 0, st, elem_args(w), V, w.elemBase, runIn, symIn,
                            unitRunOff, unitSymOff, prevHL, unitHL, hl, runStart, runChar, segs);
}
void mk_grp_big_maporder(const uint32_t* bpos, uint32_t nb, const uint32_t* hb, const uint32_t* off,
                         unsigned long long* key, uint32_t* perm, uint32_t* ts, uint8_t* sm, unsigned long long* tKey,
                         uint32_t* tPerm, uint32_t* tTs, uint8_t* tSm, uint32_t* tF, int bN, hipStream_t st) {
  if (nb) hipLaunchKernelGGL(k_grp_big_maporder, dim3(nb), dim3(256), 0, st, bpos, nb, hb, off, key, perm, ts, sm, tKey,
                             tPerm, tTs, tSm, tF, bN);
}
void mk_grp_seg(const uint32_t* posS, const uint32_t* hb, const HeadKV* kv, uint32_t H, int bN, int bL,
                unsigned long long* key, uint32_t* perm, uint32_t* tsOut, uint8_t* smOut, uint32_t* bigList,
                uint32_t maxSmall, int32_t* diffEnds, uint32_t n, hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_grp_seg, dim3((H + kGrpBlock - 1) / kGrpBlock), dim3(kGrpBlock), 0, st, posS, hb, kv, H, bN,
                            bL, key, perm, tsOut, smOut, bigList, maxSmall, diffEnds, n);
}
// run starts per position from the sorted heads' position offsets:
// diff[p] = #heads at p (ends are subtracted by k_grp_seg), hasHead[p]
__global__ void k_run_starts(const uint32_t* __restrict__ hb, uint32_t n, int32_t* __restrict__ diff,
                             uint8_t* __restrict__ hasHead) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > n) return;
  const uint32_t c = p < n ? hb[p + 1] - hb[p] : 0u;
  diff[p] = (int32_t)c;
  if (p < n) hasHead[p] = c != 0;
}
void mk_run_starts(const uint32_t* hb, uint32_t n, int32_t* diff, uint8_t* hasHead, hipStream_t st) {
  hipLaunchKernelGGL(k_run_starts, g1((uint64_t)n + 1), dim3(256), 0, st, hb, n, diff, hasHead);
}
void mk_grp_big_fields(const uint32_t* idx, uint32_t B, const uint32_t* perm, const HeadsSoA& h, uint32_t* tsOut,
                       uint8_t* smOut, hipStream_t st) {
  if (B) hipLaunchKernelGGL(k_grp_big_fields, g1(B), dim3(256), 0, st, idx, B, perm, h, tsOut, smOut);
}
void mk_grp_big_sizes(const uint32_t* pos, uint32_t nb, const uint32_t* hb, uint32_t* sz, hipStream_t st) {
  if (nb) hipLaunchKernelGGL(k_grp_big_sizes, g1(nb), dim3(256), 0, st, pos, nb, hb, sz);
}
void mk_grp_big_expand(const uint32_t* pos, uint32_t nb, const uint32_t* hb, const uint32_t* off, uint32_t* idx,
                       hipStream_t st) {
  if (nb) hipLaunchKernelGGL(k_grp_big_expand, g1(nb), dim3(256), 0, st, pos, nb, hb, off, idx);
}
void mk_gather_kp(const uint32_t* idx, uint32_t B, const unsigned long long* key, const uint32_t* perm,
                  unsigned long long* keyB, uint32_t* permB, hipStream_t st) {
  if (B) hipLaunchKernelGGL(k_gather_kp, g1(B), dim3(256), 0, st, idx, B, key, perm, keyB, permB);
}
void mk_scatter_kp(const uint32_t* idx, uint32_t B, const unsigned long long* keyB, const uint32_t* permB,
                   unsigned long long* key, uint32_t* perm, hipStream_t st) {
  if (B) hipLaunchKernelGGL(k_scatter_kp, g1(B), dim3(256), 0, st, idx, B, keyB, permB, key, perm);
}
void mk_wr_records(const unsigned long long* runStart, const uint8_t* runChar, uint64_t R, unsigned long long total,
                   uint8_t* out, hipStream_t st) {
  if (R) hipLaunchKernelGGL(k_wr_records, g1(R), dim3(256), 0, st, runStart, runChar, R, total, out);
}

}  // namespace cmsbwt
