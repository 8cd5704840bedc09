// elem_writer.h — the element writer's per-element segments (FN:1631-1777)
// and the fused run scan of the one-GPU writer.
//
// Writer elements in output order: the E end phrases, then per SA rank r >= 1
// its heads in head-rank order, or one element when it has none.  Each
// element emits <= 3 segments (counter refchars, head character, remainder
// quirk of FN:1761-1770 / the single remainder of FN:1678-1686); runs merge
// across elements when the character repeats.  Shared by merge.hip (kernels)
// and engine.h (the fused scan is a rocPRIM lookback scan whose input
// computes each element's run summary and whose output emits its runs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstddef>
#include <iterator>

#include "merge_kernels.h"

namespace cmsbwt {

struct ElemArgs {
  const int32_t* sa;
  const uint8_t* bwt;
  const int64_t* bucket;
  const uint32_t* posBegin;
  const uint32_t* slot;
  const uint32_t* itemOfSlot;
  const uint32_t* headBase;            // per SA rank (n), exclusive head counts
  const uint32_t* elemBase;            // per SA rank (n), exclusive element counts
  const uint32_t* rOf;                 // per element: its SA rank
  const uint8_t* bwtHeads;
  const unsigned long long* counter;   // by slot
  const unsigned long long* cum;       // by slot: inclusive sum of counter + 1
  const uint4* info1;                  // per SA rank: element base, heads, slot base, head base
  const unsigned long long* info2;     // per SA rank: bucket (56-bit two's complement) | BWT char << 56
  uint32_t n, E, H;
  int rle;
  // position-sharded merge: head characters by local slot (one GPU: null,
  // characters by head rank from bwtHeads)
  const uint8_t* bwtSlot;
};

template <class F>
__device__ __forceinline__ void d_elem_segments(const ElemArgs& A, uint32_t e, F&& f) {
  const uint32_t r = A.rOf[e];
  const uint4 I = A.info1[r];  // the rank's fields, read once per element (k_el_info)
  const uint32_t k = e - I.x;
  if (r == 0) { f(A.bwtSlot ? A.bwtSlot[I.z + k] : A.bwtHeads[k], 1ull); return; }  // end phrases (units u < E)
  const unsigned long long J = A.info2[r];
  const uint8_t c = (uint8_t)(J >> 56);
  const int64_t b = ((int64_t)(J << 8)) >> 8;
  if (b > 0) { if (k == 0) f(c, (unsigned long long)b); return; }
  if (b == 0) return;
  const uint32_t nh = I.y;
  if (nh == 0) {  // no items: the item loop is empty (FN:1761-1770 / 1678-1686)
    if (!A.rle) f(c, (unsigned long long)(-b));
    return;
  }
  const uint32_t s0 = I.z, s = s0 + k;
  const unsigned long long cs = A.counter[s];
  if (cs) f(c, cs);
  f(A.bwtSlot ? A.bwtSlot[s] : A.bwtHeads[I.w + k], 1ull);
  const bool last = A.rle ? (s + 1 >= A.H || A.itemOfSlot[s + 1] != A.itemOfSlot[s]) : k + 1 == nh;
  if (last) {
    const int64_t acc = b + (int64_t)(A.cum[s] - (s0 ? A.cum[s0 - 1] : 0ull));
    if (A.rle ? acc != 0 : acc < 0) f(c, (unsigned long long)(-acc));
  }
}


inline ElemArgs elem_args(const ElemIn& w) {
  return ElemArgs{w.sa, w.bwt, w.bucket, w.posBegin, w.slot, w.itemOfSlot, w.headBase, w.elemBase, w.rOf,
                  w.bwtHeads, w.counter, w.cum, w.info1, w.info2, w.n, w.E, w.H, w.rle, w.bwtSlot};
}

// Run summary of a range of elements: runs, symbols, where its last (open)
// run starts, and (non-empty, last char, first char).  Combining two ranges
// merges the run at their seam when the characters agree -- an associative
// operation with identity {0, 0, 0, 0}.
struct WrState {
  unsigned long long runs, sym;
  unsigned long long lastStart;  // symbol offset of the last run's start in the range
  uint32_t hl;                   // 1 << 16 | last << 8 | first, 0 when empty
  uint32_t pad;
};
struct WrOp {
  __host__ __device__ WrState operator()(const WrState& a, const WrState& b) const {
    const bool an = (a.hl >> 16) != 0, bn = (b.hl >> 16) != 0;
    if (!bn) return a;
    if (!an) return b;
    const bool seam = ((a.hl >> 8) & 0xffu) == (b.hl & 0xffu);
    WrState r;
    r.runs = a.runs + b.runs - (seam ? 1ull : 0ull);
    r.sym = a.sym + b.sym;
    r.lastStart = (seam && b.runs == 1) ? a.lastStart : a.sym + b.lastStart;
    r.hl = (1u << 16) | (b.hl & 0xff00u) | (a.hl & 0xffu);
    r.pad = 0;
    return r;
  }
};
// the segments of element e, kept in registers (<= 3: counter refchars, head
// character, remainder); fixed fields, never indexed at run time (an array
// indexed by the segment count went to scratch memory)
struct ElemSegs {
  uint32_t n;
  uint32_t c0, c1, c2;
  unsigned long long n0, n1, n2;
  __device__ __forceinline__ uint32_t ch(uint32_t k) const { return k == 0 ? c0 : (k == 1 ? c1 : c2); }
  __device__ __forceinline__ unsigned long long cnt(uint32_t k) const { return k == 0 ? n0 : (k == 1 ? n1 : n2); }
  __device__ WrState state() const {
    WrState s{0ull, 0ull, 0ull, 0u, 0u};
    int prev = -1;
#pragma unroll
    for (uint32_t k = 0; k < 3; k++)
      if (k < n) {
        if ((int)ch(k) != prev) {
          s.runs++;
          s.lastStart = s.sym;
        }
        prev = (int)ch(k);
        s.sym += cnt(k);
      }
    if (n) s.hl = (1u << 16) | (ch(n - 1) << 8) | c0;
    return s;
  }
};
// an element's segments in 16 bytes (k_el_wr_tiles stores them in element
// order, k_el_wr_emit_tiles reads them back sequentially instead of
// re-gathering the per-slot inputs): x = n | c0 << 8 | c1 << 16 | c2 << 24,
// the first and the last segment's counts in 48 bits each (<= the collection
// length); a middle segment (n == 3: the head character between the counter
// refchars and the remainder, d_elem_segments) always counts 1
__device__ __forceinline__ uint4 segs_pack(const ElemSegs& g) {
  const unsigned long long a = g.n0, b = g.n == 3 ? g.n2 : (g.n == 2 ? g.n1 : 0ull);
  return make_uint4(g.n | (g.c0 << 8) | (g.c1 << 16) | (g.c2 << 24), (uint32_t)a,
                    ((uint32_t)(a >> 32) & 0xffffu) | (((uint32_t)b & 0xffffu) << 16), (uint32_t)(b >> 16));
}
__device__ __forceinline__ ElemSegs segs_unpack(const uint4 v) {
  ElemSegs g{v.x & 3u, (v.x >> 8) & 0xffu, (v.x >> 16) & 0xffu, (v.x >> 24) & 0xffu, 0ull, 0ull, 0ull};
  const unsigned long long a = v.y | ((unsigned long long)(v.z & 0xffffu) << 32);
  const unsigned long long b = (v.z >> 16) | ((unsigned long long)v.w << 16);
  g.n0 = a;
  g.n1 = g.n == 3 ? 1ull : b;
  g.n2 = b;
  return g;
}
__device__ __forceinline__ ElemSegs d_elem_collect(const ElemArgs& A, uint32_t e) {
  ElemSegs g{0u, 0u, 0u, 0u, 0ull, 0ull, 0ull};
  d_elem_segments(A, e, [&](uint8_t c, unsigned long long cnt) {
    if (g.n == 0) { g.c0 = c; g.n0 = cnt; }
    else if (g.n == 1) { g.c1 = c; g.n1 = cnt; }
    else { g.c2 = c; g.n2 = cnt; }
    g.n++;
  });
  return g;
}

}  // namespace cmsbwt
