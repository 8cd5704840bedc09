// dist_kernels.hip — kernels of the position-sharded merge.
//
// Ranks own contiguous reference-position ranges [P_k, P_k+1).  Heads travel
// from their document's rank to the owner of their position, where they are
// grouped into items exactly as on one GPU (FN:1387-1416); the head-string
// suffix sort (FN:1455-1459) runs as distributed prefix doubling between the
// heads' document ranks and the owners of group-label ranges; counters
// (FN:1523-1603) and writer units (FN:1695-1777) are computed by the position
// owner.  Every kernel here is byte/index work: packing, routing, relabelling.
#include <hip/hip_runtime.h>
#include "device_common.h"
#include "kernels.h"
#include "merge_kernels.h"

namespace cmsbwt {

static inline dim3 g1d(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

__device__ __forceinline__ uint32_t d_owner(const uint32_t* __restrict__ split, uint32_t world, uint32_t v) {
  uint32_t k = 0;  // largest k with split[k] <= v (split[0] = 0 or 1, world <= 64)
  for (uint32_t j = 1; j < world; j++) k += split[j] <= v ? 1u : 0u;
  return k;
}

__global__ void k_dm_owner(const uint32_t* __restrict__ vals, const uint32_t* __restrict__ idx, uint64_t n,
                           const uint32_t* __restrict__ split, uint32_t world, uint32_t* __restrict__ dest) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dest[i] = d_owner(split, world, vals[idx ? idx[i] : i]);
}

// bounds[k] = first index of destination k in a sorted destination array
__global__ void k_dm_bounds(const uint32_t* __restrict__ sorted, uint64_t n, uint32_t world,
                            uint32_t* __restrict__ bounds) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > world) return;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (sorted[m] < k) lo = m + 1; else hi = m;
  }
  bounds[k] = (uint32_t)lo;
}

// head records on the wire: pos, len, isaNext, toNext, smaller | listOfChars << 8
__global__ void k_dm_pack_heads(const uint32_t* __restrict__ perm, HeadsSoA h, uint64_t n, int32_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = perm[j];
  int32_t* o = out + 5 * j;
  o[0] = (int32_t)h.pos[i];
  o[1] = (int32_t)h.len[i];
  o[2] = (int32_t)h.isa[i];
  o[3] = (int32_t)h.tonext[i];
  o[4] = (int32_t)((uint32_t)h.smaller[i] | ((uint32_t)h.lchar[i] << 8));
}

__global__ void k_dm_unpack_heads(const int32_t* __restrict__ in, uint64_t n, HeadsSoA h) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int32_t* o = in + 5 * j;
  h.pos[j] = (uint32_t)o[0];
  h.len[j] = (uint32_t)o[1];
  h.isa[j] = (uint32_t)o[2];
  h.tonext[j] = (uint32_t)o[3];
  h.smaller[j] = (uint8_t)(o[4] & 0xff);
  h.lchar[j] = (uint8_t)((uint32_t)o[4] >> 8);
}

// run buckets (FN:1162-1171) of the received heads when the grouping did not
// take the position-first sort (composite key wider than 64 bits): head j
// covers [pos, pos + toNext + 1) (an end phrase: [n-1, n)); diff and hasHead
// zeroed on entry
__global__ void k_dm_runs(const uint32_t* __restrict__ pos, const uint32_t* __restrict__ tonext, uint64_t H,
                          uint32_t n, int32_t* __restrict__ diff, uint8_t* __restrict__ hasHead) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= H) return;
  const uint32_t p = pos[j];
  const uint64_t e = (uint64_t)p + tonext[j] + 1;
  atomicAdd(&diff[p], 1);
  if (e <= n) atomicAdd(&diff[e], -1);
  hasHead[p] = 1;
}

// per SA rank: this rank's items and heads of position SA[r] (zero for
// positions it does not own; SA rank 0 = position n-1 holds the E end phrases)
__global__ void k_dm_sa_counts(const int32_t* __restrict__ sa, const uint32_t* __restrict__ posBegin,
                               const uint32_t* __restrict__ slot, uint32_t n, uint32_t Eown,
                               uint32_t* __restrict__ out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  if (r == 0) { out[0] = 0; out[n] = Eown; return; }
  const uint32_t p = (uint32_t)sa[r];
  const uint32_t b = posBegin[p], e = posBegin[p + 1];
  out[r] = e - b;
  out[n + r] = slot[e] - slot[b];
}

// Initial group label of every member (its item's first sa position in the
// head-string suffix array, FN:1432-1453): end phrases get 1 + m, others
// gBase[p] + slot[q] (gBase from k_pos_rank_base: 1 + headBase[ISA[p]] minus
// the slot of p's first item; slots ascend with p, so it is read in order).
// Bit 32: unresolved (item with >= 2 members; labels use all 32 bits).
// Written in received order for the return trip.  Labels carry `bias`
// (0 in production; tests set it so that labels cross 2^31 on small inputs,
// CMSBWT_DM_LABEL_BIAS); gItem keeps the unbiased label.
__global__ void k_dm_group_labels(const ItemsSoA it, const uint32_t* __restrict__ itemOfSlot,
                                  const uint32_t* __restrict__ Pm, uint32_t H, const uint32_t* __restrict__ gBase,
                                  uint32_t n, uint32_t bias, unsigned long long* __restrict__ back,
                                  uint32_t* __restrict__ gItem) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= H) return;
  const uint32_t q = itemOfSlot[s], sq = it.slot[q], m = s - sq, p = it.pos[q];
  uint32_t g, act = 0;
  if (p == n - 1) {
    g = 1 + m;
    if (m == 0) gItem[q] = 1;
  } else {
    // members occupy sa positions g .. g + count - 1; their group label is g
    g = gBase[p] + sq;
    if (m == 0) gItem[q] = g;
    act = it.count[q] >= 2 ? 1u : 0u;
  }
  back[Pm[s]] = (unsigned long long)(g + bias) | ((unsigned long long)act << 32);
}

// doc side: labels arrive in send order; flags stay in send order
__global__ void k_dm_grp_init(const uint32_t* __restrict__ perm, const unsigned long long* __restrict__ in, uint64_t n,
                              uint32_t* __restrict__ grp, uint32_t* __restrict__ actFlag) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = perm[j];
  const unsigned long long v = in[j];
  grp[i] = (uint32_t)v;
  actFlag[j] = (uint32_t)(v >> 32);  // send order
}

// doubling keys (group of suffix, group of suffix + h), send order; a
// suffix still unresolved at step h ends inside its document, so idx + h
// stays below this rank's head count (checked)
__global__ void k_dm_dbl_pack(const uint32_t* __restrict__ aPerm, const uint32_t* __restrict__ act,
                              const uint32_t* __restrict__ grp, uint32_t h, uint64_t n, uint32_t H,
                              int32_t* __restrict__ out, uint32_t* __restrict__ err) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = act[aPerm[j]];
  uint32_t g2 = 0;
  if ((uint64_t)i + h < H) g2 = grp[i + h];
  else atomicOr(err, 1u);
  out[2 * j] = (int32_t)grp[i];
  out[2 * j + 1] = (int32_t)g2;
}


// label-range owner, first pass: members keyed by their label's offset in
// the owned range [G0, G1) (the sort needs bits_for(G1 - G0) bits, not the
// full (label, label2) pair), carrying label2 << 32 | received index
__global__ void k_dm_dbl_lkeys(const int32_t* __restrict__ in, uint64_t n, uint32_t G0, uint32_t* __restrict__ key,
                               unsigned long long* __restrict__ val) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  key[j] = (uint32_t)in[2 * j] - G0;
  val[j] = ((unsigned long long)(uint32_t)in[2 * j + 1] << 32) | (uint32_t)j;
}

// second pass over the members sorted by label: a group (equal labels) of at
// most kDblSmall members is ranked by counting over an LDS copy of the block's
// members with a halo; its new label is label + #members with a smaller
// label2 (the sa position where its equal-key run starts, as k_dm_dbl_result),
// unresolved when another member has the same label2.  Larger groups are
// listed (bigList[0] = count) for the full-key sort.
constexpr uint32_t kDblBlock = 256, kDblSmall = 32, kDblHalo = kDblSmall;
__global__ void __launch_bounds__(kDblBlock) k_dm_dbl_rank(const uint32_t* __restrict__ key,
                                                           const unsigned long long* __restrict__ val, uint64_t n,
                                                           uint32_t G0, unsigned long long* __restrict__ res,
                                                           uint32_t* __restrict__ bigList) {
  __shared__ uint32_t kL[kDblBlock + 2 * kDblHalo], l2L[kDblBlock + 2 * kDblHalo];
  const uint64_t u0 = (uint64_t)blockIdx.x * kDblBlock;
  const int64_t base = (int64_t)u0 - kDblHalo;
  for (uint32_t i = threadIdx.x; i < kDblBlock + 2 * kDblHalo; i += blockDim.x) {
    const int64_t j = base + i;
    if (j >= 0 && j < (int64_t)n) {
      kL[i] = key[j];
      l2L[i] = (uint32_t)(val[j] >> 32);
    }
  }
  __syncthreads();
  const uint64_t u = u0 + threadIdx.x;
  if (u >= n) return;
  const uint32_t me = threadIdx.x + kDblHalo, k = kL[me], v = l2L[me];
  uint32_t lo = me, hi = me + 1;
  while (lo > 0 && base + lo > 0 && kL[lo - 1] == k && me - lo <= kDblSmall) lo--;
  while (hi < kDblBlock + 2 * kDblHalo && base + (int64_t)hi < (int64_t)n && kL[hi] == k && hi - me <= kDblSmall) hi++;
  if (hi - lo > kDblSmall) {  // (a group reaching past the halo has more than kDblSmall members)
    bigList[1 + atomicAdd(bigList, 1u)] = (uint32_t)u;
    return;
  }
  uint32_t less = 0, eq = 0;
  for (uint32_t j = lo; j < hi; j++) {
    const uint32_t w = l2L[j];
    less += w < v ? 1u : 0u;
    eq += (w == v && j != me) ? 1u : 0u;
  }
  res[(uint32_t)val[u]] = (unsigned long long)(k + G0 + less) | (eq ? (1ull << 32) : 0ull);
}

// big groups: their members' full (label, label2) keys for the sort path
__global__ void k_dm_dbl_bigkeys(const uint32_t* __restrict__ list, uint32_t B, const uint32_t* __restrict__ key,
                                 const unsigned long long* __restrict__ val, uint32_t G0,
                                 unsigned long long* __restrict__ k64, uint32_t* __restrict__ v2) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t u = list[b];
  const unsigned long long v = val[u];
  k64[b] = ((unsigned long long)(key[u] + G0) << 32) | (v >> 32);
  v2[b] = (uint32_t)v;
}

__global__ void k_dm_dbl_marks(const unsigned long long* __restrict__ key, uint64_t n, uint32_t* __restrict__ gs,
                               uint32_t* __restrict__ ks) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  const bool first = u == 0;
  gs[u] = (first || (key[u] >> 32) != (key[u - 1] >> 32)) ? (uint32_t)u : 0u;
  ks[u] = (first || key[u] != key[u - 1]) ? (uint32_t)u : 0u;
}

// new label = g + (first index of the equal-key run - first index of group
// g), i.e. the sa position the run starts at; bit 32 = still unresolved
__global__ void k_dm_dbl_result(const unsigned long long* __restrict__ key, const uint32_t* __restrict__ val,
                                const uint32_t* __restrict__ gsMax, const uint32_t* __restrict__ ksMax, uint64_t n,
                                unsigned long long* __restrict__ res) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  const unsigned long long k = key[u];
  const uint32_t label = (uint32_t)(k >> 32) + (ksMax[u] - gsMax[u]);
  const bool alone = ksMax[u] == (uint32_t)u && (u + 1 == n || key[u + 1] != k);
  res[val[u]] = (unsigned long long)label | (alone ? 0ull : (1ull << 32));
}

__global__ void k_dm_dbl_apply(const uint32_t* __restrict__ aPerm, const uint32_t* __restrict__ act,
                               const unsigned long long* __restrict__ back, uint64_t n, uint32_t* __restrict__ grp,
                               uint32_t* __restrict__ keep) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t u = aPerm[j];
  const unsigned long long v = back[j];
  grp[act[u]] = (uint32_t)v;
  keep[u] = (uint32_t)(v >> 32);
}

// head rank and next-head rank (FN:1468-1494) of every head, heads send order
// doc side: (head rank, next-head rank, BWT character) per head in send
// order; the character travels here so that the position side places it with
// the ranks it reads anyway (one gather per slot, not two)
__global__ void k_dm_pack_ranks(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ grp,
                                const uint16_t* __restrict__ nexthead, const uint8_t* __restrict__ lchar,
                                uint64_t n, uint32_t H, uint32_t bias, int32_t* __restrict__ out,
                                uint32_t* __restrict__ err) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = perm[j];
  const uint32_t nx = i + nexthead[i];
  uint32_t nv = 0;
  if (nx < H) nv = grp[nx] - 1 - bias;
  else atomicOr(err, 2u);
  out[3 * j] = (int32_t)(grp[i] - 1 - bias);
  out[3 * j + 1] = (int32_t)nv;
  out[3 * j + 2] = (int32_t)lchar[i];
}

// position side: the head characters by slot (the member with head rank hr
// sits at slot slot[q] + hr - (gItem[q] - 1) of its item, which is where the
// writer reads BWTheads[hr], FN:1742-1752) and the next-head ranks in slot
// order (ranked inside their items by k_nhr_rank); one read of the received
// rank pair per slot
__global__ void k_dm_load_ranks(const int32_t* __restrict__ in, const uint32_t* __restrict__ Pm,
                                const uint32_t* __restrict__ itemOfSlot, const ItemsSoA it,
                                const uint32_t* __restrict__ gItem, uint32_t H, uint32_t* __restrict__ nbiS,
                                uint8_t* __restrict__ bwtSlot, uint32_t* __restrict__ err) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= H) return;
  const uint32_t r = Pm[s], q = itemOfSlot[s];
  const int32_t* w = in + 3ull * r;  // (rank, next-head rank, character), one 12-B record
  const uint32_t hr = (uint32_t)w[0], nb = (uint32_t)w[1], ch = (uint32_t)w[2];
  nbiS[s] = nb;
  const uint32_t k = hr - (gItem[q] - 1);
  if (k < it.count[q]) bwtSlot[it.slot[q] + k] = (uint8_t)ch;
  else atomicOr(err, 4u);
}

// ---- halo: items reaching past this rank's last position into later ranks
__global__ void k_dm_halo_count(const ItemsSoA it, uint32_t K, const uint32_t* __restrict__ split, uint32_t world,
                                uint32_t rank, uint32_t n, uint32_t* __restrict__ c) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  const uint32_t u = it.until[q];
  uint32_t cnt = 0;
  if (u) {
    const uint64_t last = min((uint64_t)it.pos[q] + u, (uint64_t)n - 1);
    const uint32_t o = d_owner(split, world, (uint32_t)last);
    cnt = o > rank ? o - rank : 0;
  }
  c[q] = cnt;
}

__global__ void k_dm_halo_fill(const uint32_t* __restrict__ c, const uint32_t* __restrict__ off, uint32_t K,
                               uint32_t rank, uint32_t* __restrict__ dest, uint32_t* __restrict__ item) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= K) return;
  const uint32_t o = off[q];
  for (uint32_t k = 0; k < c[q]; k++) {
    dest[o + k] = rank + 1 + k;
    item[o + k] = q;
  }
}

__global__ void k_dm_pair_words(const uint32_t* __restrict__ item, uint32_t np, const uint32_t* __restrict__ count,
                                uint32_t* __restrict__ w) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < np) w[j] = count[item[j]];
}

// header: pos, len, isaNext, smaller, untilNext, count; then the item's nhr
__global__ void k_dm_halo_pack(const uint32_t* __restrict__ item, uint32_t np, const ItemsSoA it,
                               const uint32_t* __restrict__ nhr, const uint32_t* __restrict__ wOff,
                               int32_t* __restrict__ hdr, int32_t* __restrict__ words) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  const uint32_t q = item[j];
  int32_t* o = hdr + 6 * (uint64_t)j;
  const uint32_t c = it.count[q];
  o[0] = (int32_t)it.pos[q];
  o[1] = (int32_t)it.len[q];
  o[2] = (int32_t)it.isa[q];
  o[3] = (int32_t)it.smaller[q];
  o[4] = (int32_t)it.until[q];
  o[5] = (int32_t)c;
  const uint32_t* src = nhr + it.slot[q];
  int32_t* dst = words + wOff[j];
  for (uint32_t k = 0; k < c; k++) dst[k] = (int32_t)src[k];
}

__global__ void k_dm_halo_unpack(const int32_t* __restrict__ hdr, uint32_t nh, ItemsSoA c) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nh) return;
  const int32_t* o = hdr + 6 * (uint64_t)j;
  c.pos[j] = (uint32_t)o[0];
  c.len[j] = (uint32_t)o[1];
  c.isa[j] = (uint32_t)o[2];
  c.smaller[j] = (uint8_t)o[3];
  c.until[j] = (uint32_t)o[4];
  c.count[j] = (uint32_t)o[5];
}

// ---- writer units: (hl << 32 | runs, symbols) per unit; zero for units of other ranks
__global__ void k_dm_units_pack(const uint32_t* __restrict__ runs, const uint32_t* __restrict__ hl,
                                const unsigned long long* __restrict__ sym, uint32_t U, int64_t* __restrict__ out) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  out[u] = (int64_t)(((uint64_t)hl[u] << 32) | runs[u]);
  out[(uint64_t)U + u] = (int64_t)sym[u];
}

__global__ void k_dm_units_unpack(const int64_t* __restrict__ in, uint32_t U, uint32_t* __restrict__ runs,
                                  uint32_t* __restrict__ hl, unsigned long long* __restrict__ sym) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const uint64_t a = (uint64_t)in[u];
  runs[u] = (uint32_t)a;
  hl[u] = (uint32_t)(a >> 32);
  sym[u] = (unsigned long long)in[(uint64_t)U + u];
}

__device__ __forceinline__ bool d_unit_owned(const int32_t* sa, uint32_t E, uint32_t n, uint32_t u, uint32_t P0,
                                             uint32_t P1) {
  const uint32_t p = u < E ? n - 1 : (uint32_t)sa[u - E + 1];
  return p >= P0 && p < P1;
}

// runs of the units of position range [P0, P1), zero elsewhere (widened)
__global__ void k_dm_own_runs(const uint32_t* __restrict__ runs, uint32_t U, const int32_t* __restrict__ sa,
                              uint32_t E, uint32_t n, uint32_t P0, uint32_t P1, unsigned long long* __restrict__ out) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  out[u] = d_unit_owned(sa, E, n, u, P0, P1) ? runs[u] : 0ull;
}

// rank 0: copy one source rank's runs (its units in unit order) to their
// global run indices
__global__ void k_dm_place(const uint32_t* __restrict__ runs, const unsigned long long* __restrict__ runOff,
                           const unsigned long long* __restrict__ srcOff, uint32_t U, const int32_t* __restrict__ sa,
                           uint32_t E, uint32_t n, uint32_t P0, uint32_t P1,
                           const unsigned long long* __restrict__ srcStart, const uint8_t* __restrict__ srcChar,
                           unsigned long long* __restrict__ runStart, uint8_t* __restrict__ runChar) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const uint32_t c = runs[u];
  if (!c || !d_unit_owned(sa, E, n, u, P0, P1)) return;
  const unsigned long long s = srcOff[u], d = runOff[u];
  for (uint32_t k = 0; k < c; k++) {
    runStart[d + k] = srcStart[s + k];
    runChar[d + k] = srcChar[s + k];
  }
}

// ------------------------------------------------------------ launchers
void mk_dm_owner(const uint32_t* vals, const uint32_t* idx, uint64_t n, const uint32_t* split, uint32_t world,
                 uint32_t* dest, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_owner, g1d(n), dim3(256), 0, st, vals, idx, n, split, world, dest);
}
void mk_dm_bounds(const uint32_t* sorted, uint64_t n, uint32_t world, uint32_t* bounds, hipStream_t st) {
  hipLaunchKernelGGL(k_dm_bounds, g1d((uint64_t)world + 1), dim3(256), 0, st, sorted, n, world, bounds);
}
void mk_dm_pack_heads(const uint32_t* perm, const HeadsSoA& h, uint64_t n, int32_t* out, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_pack_heads, g1d(n), dim3(256), 0, st, perm, h, n, out);
}
void mk_dm_unpack_heads(const int32_t* in, uint64_t n, const HeadsSoA& h, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_unpack_heads, g1d(n), dim3(256), 0, st, in, n, h);
}
void mk_dm_runs(const uint32_t* pos, const uint32_t* tonext, uint64_t H, uint32_t n, int32_t* diff, uint8_t* hasHead,
                hipStream_t st) {
  if (H) hipLaunchKernelGGL(k_dm_runs, g1d(H), dim3(256), 0, st, pos, tonext, H, n, diff, hasHead);
}
void mk_dm_sa_counts(const int32_t* sa, const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t Eown,
                     uint32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_dm_sa_counts, g1d(n), dim3(256), 0, st, sa, posBegin, slot, n, Eown, out);
}
void mk_dm_group_labels(const ItemsSoA& it, const uint32_t* itemOfSlot, const uint32_t* Pm, uint32_t H,
                        const uint32_t* gBase, uint32_t n, uint32_t bias, unsigned long long* back, uint32_t* gItem,
                        hipStream_t st) {
  if (H)
    hipLaunchKernelGGL(k_dm_group_labels, g1d(H), dim3(256), 0, st, it, itemOfSlot, Pm, H, gBase, n, bias, back, gItem);
}
void mk_dm_grp_init(const uint32_t* perm, const unsigned long long* in, uint64_t n, uint32_t* grp, uint32_t* actFlag,
                    hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_grp_init, g1d(n), dim3(256), 0, st, perm, in, n, grp, actFlag);
}
void mk_dm_dbl_pack(const uint32_t* aPerm, const uint32_t* act, const uint32_t* grp, uint32_t h, uint64_t n,
                    uint32_t H, int32_t* out, uint32_t* err, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_dbl_pack, g1d(n), dim3(256), 0, st, aPerm, act, grp, h, n, H, out, err);
}
void mk_dm_dbl_lkeys(const int32_t* in, uint64_t n, uint32_t G0, uint32_t* key, unsigned long long* val,
                     hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_dbl_lkeys, g1d(n), dim3(256), 0, st, in, n, G0, key, val);
}
void mk_dm_dbl_rank(const uint32_t* key, const unsigned long long* val, uint64_t n, uint32_t G0,
                    unsigned long long* res, uint32_t* bigList, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_dbl_rank, dim3((unsigned)((n + kDblBlock - 1) / kDblBlock)), dim3(kDblBlock), 0, st,
                            key, val, n, G0, res, bigList);
}
void mk_dm_dbl_bigkeys(const uint32_t* list, uint32_t B, const uint32_t* key, const unsigned long long* val,
                       uint32_t G0, unsigned long long* k64, uint32_t* v2, hipStream_t st) {
  if (B) hipLaunchKernelGGL(k_dm_dbl_bigkeys, g1d(B), dim3(256), 0, st, list, B, key, val, G0, k64, v2);
}
void mk_dm_dbl_marks(const unsigned long long* key, uint64_t n, uint32_t* gs, uint32_t* ks, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_dbl_marks, g1d(n), dim3(256), 0, st, key, n, gs, ks);
}
void mk_dm_dbl_result(const unsigned long long* key, const uint32_t* val, const uint32_t* gsMax,
                      const uint32_t* ksMax, uint64_t n, unsigned long long* res, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_dbl_result, g1d(n), dim3(256), 0, st, key, val, gsMax, ksMax, n, res);
}
void mk_dm_dbl_apply(const uint32_t* aPerm, const uint32_t* act, const unsigned long long* back, uint64_t n, uint32_t* grp,
                     uint32_t* keep, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_dbl_apply, g1d(n), dim3(256), 0, st, aPerm, act, back, n, grp, keep);
}
void mk_dm_pack_ranks(const uint32_t* perm, const uint32_t* grp, const uint16_t* nexthead, const uint8_t* lchar,
                      uint64_t n, uint32_t H, uint32_t bias, int32_t* out, uint32_t* err, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_dm_pack_ranks, g1d(n), dim3(256), 0, st, perm, grp, nexthead, lchar, n, H, bias, out, err);
}
void mk_dm_load_ranks(const int32_t* in, const uint32_t* Pm, const uint32_t* itemOfSlot, const ItemsSoA& it,
                      const uint32_t* gItem, uint32_t H, uint32_t* nbi, uint8_t* bwtSlot, uint32_t* err, hipStream_t st) {
  if (!H) return;
  hipLaunchKernelGGL(k_dm_load_ranks, g1d(H), dim3(256), 0, st, in, Pm, itemOfSlot, it, gItem, H, nbi, bwtSlot, err);
}
void mk_dm_halo_count(const ItemsSoA& it, uint32_t K, const uint32_t* split, uint32_t world, uint32_t rank,
                      uint32_t n, uint32_t* c, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_dm_halo_count, g1d(K), dim3(256), 0, st, it, K, split, world, rank, n, c);
}
void mk_dm_halo_fill(const uint32_t* c, const uint32_t* off, uint32_t K, uint32_t rank, uint32_t* dest,
                     uint32_t* item, hipStream_t st) {
  if (K) hipLaunchKernelGGL(k_dm_halo_fill, g1d(K), dim3(256), 0, st, c, off, K, rank, dest, item);
}
void mk_dm_pair_words(const uint32_t* item, uint32_t np, const uint32_t* count, uint32_t* w, hipStream_t st) {
  if (np) hipLaunchKernelGGL(k_dm_pair_words, g1d(np), dim3(256), 0, st, item, np, count, w);
}
void mk_dm_halo_pack(const uint32_t* item, uint32_t np, const ItemsSoA& it, const uint32_t* nhr, const uint32_t* wOff,
                     int32_t* hdr, int32_t* words, hipStream_t st) {
  if (np) hipLaunchKernelGGL(k_dm_halo_pack, g1d(np), dim3(256), 0, st, item, np, it, nhr, wOff, hdr, words);
}
void mk_dm_halo_unpack(const int32_t* hdr, uint32_t nh, const ItemsSoA& c, hipStream_t st) {
  if (nh) hipLaunchKernelGGL(k_dm_halo_unpack, g1d(nh), dim3(256), 0, st, hdr, nh, c);
}
void mk_dm_units_pack(const uint32_t* runs, const uint32_t* hl, const unsigned long long* sym, uint32_t U,
                      int64_t* out, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dm_units_pack, g1d(U), dim3(256), 0, st, runs, hl, sym, U, out);
}
void mk_dm_units_unpack(const int64_t* in, uint32_t U, uint32_t* runs, uint32_t* hl, unsigned long long* sym,
                        hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dm_units_unpack, g1d(U), dim3(256), 0, st, in, U, runs, hl, sym);
}
void mk_dm_own_runs(const uint32_t* runs, uint32_t U, const int32_t* sa, uint32_t E, uint32_t n, uint32_t P0,
                    uint32_t P1, unsigned long long* out, hipStream_t st) {
  if (U) hipLaunchKernelGGL(k_dm_own_runs, g1d(U), dim3(256), 0, st, runs, U, sa, E, n, P0, P1, out);
}
void mk_dm_place(const uint32_t* runs, const unsigned long long* runOff, const unsigned long long* srcOff, uint32_t U,
                 const int32_t* sa, uint32_t E, uint32_t n, uint32_t P0, uint32_t P1,
                 const unsigned long long* srcStart, const uint8_t* srcChar, unsigned long long* runStart,
                 uint8_t* runChar, hipStream_t st) {
  if (U)
    hipLaunchKernelGGL(k_dm_place, g1d(U), dim3(256), 0, st, runs, runOff, srcOff, U, sa, E, n, P0, P1, srcStart,
                       srcChar, runStart, runChar);
}

}  // namespace cmsbwt
