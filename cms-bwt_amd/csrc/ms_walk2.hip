// ms_walk2.hip — uniform-step MS walk (the default walk kernel).
//
// Same semantics as k_ms_walk (FN:45-149, FN:1151-1212, rmq_tree.h:184-225),
// restructured for SIMT.  In the per-lane walk the nested loops (binary
// searches, LCE, PLCP skip, PSV/NSV scans) make the 64 lanes of a wave issue
// their dependent loads in separate, mostly-inactive instructions.  Here each
// iteration issues one round of loads for all lanes (a lane loads up to two
// addresses A and B, as a byte, a dword or 16/32 bytes) and every lane advances
// its own state machine by exactly one memory step; the work between two
// loads (head record, contraction set-up, next character) runs as "compute
// phases", each emitted once.  Lanes pull restart chunks from per-band queues.
//
//   load phase  loads                          next
//   BS_TEXT     t[j], SA[first probe]          BS_X          (FN:94-149)
//   BS_SA       SA[m]                          BS_X
//   BS_X        x[SA[m]+off]                   BS_SA / FAIL_SA / CHAR
//   FAIL_SA     SA[insertion point]            POST          (FN:65-76)
//   LCE_SA      SA[lb]                         LCE           (FN:52-62)
//   LCE         16 B of x and of the text      POST / LCE_COOP
//   LCE_COOP    (none) the whole wave compares 1 KiB per step of one lane's
//               long extension with coalesced loads, lane by lane -> POST
//   SKIP1       min(PLCP, 255)[T-16..T-1], bytes  ISA1 / SKIP0 (FN:1176-1185)
//   SKIP0       PLCP[pos+1]                    ISA1 / GALLOP
//   GALLOP/SKIPBS  one PLCP probe              ISA1
//   ISA1        record of ISA[pos+1]           ADV / ADJ0    (FN:1187, FN:11-25)
//   CONP        records of psi(lb), psi(rb)    ADV / ADJ0    (FN:34-43, FN:11-25)
//               (a record carries the 6 LCP entries on either side of r, so
//               adjustInterval usually ends in the same load)
//   ADJ         8 LCP entries for PSV + 8 for NSV  ADJ / ADV (FN:11-25)
//   PFX_TEXT    K text bytes: codes of t[i..i+l) for l <= K   PFX_PROBE / BS
//   PFX_PROBE   prefix-rank table entries of length-l codes: the SA interval
//               of t[i..i+l) or, when it does not occur, its insertion point;
//               a binary search over l finds the longest match (restarts from
//               the root and extensions at depth < K over large intervals)
//   EXT1        one character over an interval of <= 16 suffixes without a
//               binary search: its children at depth off start where LCP ==
//               off; child characters D[start] and, for the first, U[end]
//   EXT_A/EXT_B the same when the interval has one child at depth off (its
//               character is x[SA[lb]+off]: SA[lb], then the byte)
//   compute phases (no load): ADJ0 (start adjustInterval), ADV (next
//   position, FN:1195-1196), POST (head record FN:1154-1171 and the
//   contraction choice FN:1175-1194), CHAR (next character, FN:45-62).
//
// Cost model (measured on the benchmark): neither latency (2..6 waves per
// SIMD time the same) nor L2 locality (per-XCD offset bands change nothing)
// bounds the walk; the issued instructions per step do.  Hence few, narrow
// loads, compute written once, and long extensions moved to coalesced
// wave-wide compares.
#include <type_traits>

#include "device_common.h"
#include "kernels.h"

namespace cmsbwt {

namespace {

enum : uint32_t {
  PH_DONE = 0,
  PH_NEXT,  // needs a new chunk (no load)
  // load phases
  PH_BS_TEXT,
  PH_BS_SA,
  PH_BS_X,
  PH_FAIL_SA,
  PH_LCE_SA,
  PH_LCE,
  PH_SKIP1,
  PH_SKIP0,
  PH_GALLOP,
  PH_SKIPBS,
  PH_ISA1,
  PH_CONP,
  PH_EXT1,
  PH_ADJ,
  PH_PFX_TEXT,
  PH_PFX_PROBE,
  PH_EXT_A,
  PH_EXT_B,
  PH_SKTXT,
  PH_IVL,
  PH_LCE_COOP,  // served by the whole wave (no lane load)
  // compute phases
  PC_ADJ0,
  PC_PFX,   // (prefetch) a position whose probe entry is in registers
  PC_ADV,
  PC_POST,
  PC_CHAR,
  PH_COUNT
};

// Loads through global-address-space pointers (global_load_*, not flat), each
// as narrow as the step needs.
#define GPTR(T, a) ((const __attribute__((address_space(1))) T*)(a))
__device__ __forceinline__ uint32_t ld1(uintptr_t a) { return *GPTR(uint8_t, a); }
__device__ __forceinline__ uint32_t ld4(uintptr_t a) { return *GPTR(uint32_t, a); }
// 8 bytes at a 4-byte aligned address
__device__ __forceinline__ uint2 ld8(uintptr_t a) {
  typedef uint32_t u2u __attribute__((ext_vector_type(2), aligned(4)));
  const u2u v = *GPTR(u2u, a);
  return make_uint2(v.x, v.y);
}
// 16 bytes at any address (gfx950 global loads allow unaligned dwordx4)
__device__ __forceinline__ uint4 ldu16(uintptr_t a) {
  typedef uint32_t u4u __attribute__((ext_vector_type(4), aligned(1)));
  const u4u v = *GPTR(u4u, a);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// non-temporal forms for bytes read once (the text of long extensions, the
// prefix-table probes): measured 15.12 -> 14.96 ms with both (r03 A/B)
__device__ __forceinline__ uint4 ldu16_nt(uintptr_t a) {
  typedef uint32_t u4u __attribute__((ext_vector_type(4), aligned(1)));
  const u4u v = __builtin_nontemporal_load(GPTR(u4u, a));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld8_nt(uintptr_t a) {
  typedef uint32_t u2u __attribute__((ext_vector_type(2), aligned(4)));
  const u2u v = __builtin_nontemporal_load(GPTR(u2u, a));
  return make_uint2(v.x, v.y);
}
// slot loads of one step (`use` bits)
enum : uint32_t {
  U0B = 1,    // byte at A
  U0D = 2,    // dword at A
  U0Q = 4,    // 16 B at A
  U1Q = 8,    // 16 B at A + 16
  U2D = 16,   // dword at B
  U2Q = 32,   // 16 B at B
  U3Q = 64,   // 16 B at B + 16
  U2B = 128,  // byte at B
  U4Q = 256,  // 16 B at A + 32
  U5Q = 512,  // 16 B at A + 48
  U0E = 1024, // 8 B at A
  U2E = 2048, // 8 B at B
  UREG = 4096, // (no load) the probe's next window comes from the skip's 32 text bytes
  U3E = 8192,  // 8 B of the prefix tables at entry u8 (the prefetched probe of i + 1)
};
// First differing byte of two 16-byte strings: 16 if equal.
__device__ __forceinline__ uint32_t diff16(const uint4& x, const uint4& t, uint8_t& xc, uint8_t& tc) {
  const uint64_t x0 = x.x | ((uint64_t)x.y << 32), x1 = x.z | ((uint64_t)x.w << 32);
  const uint64_t t0 = t.x | ((uint64_t)t.y << 32), t1 = t.z | ((uint64_t)t.w << 32);
  const uint64_t d0 = x0 ^ t0, d1 = x1 ^ t1;
  if (!(d0 | d1)) return 16;
  const uint64_t d = d0 ? d0 : d1;
  const uint32_t bit = (uint32_t)__builtin_ctzll(d) & ~7u;
  xc = (uint8_t)((d0 ? x0 : x1) >> bit);
  tc = (uint8_t)((d0 ? t0 : t1) >> bit);
  return (d0 ? 0 : 8) + bit / 8;
}

// First and second differing bytes of two 16-byte strings (16 when none).
__device__ __forceinline__ void diff16x2(const uint4& x, const uint4& t, uint32_t& m1, uint32_t& c1, uint32_t& m2,
                                         uint32_t& c2) {
  const uint64_t x0 = x.x | ((uint64_t)x.y << 32), x1 = x.z | ((uint64_t)x.w << 32);
  const uint64_t t0 = t.x | ((uint64_t)t.y << 32), t1 = t.z | ((uint64_t)t.w << 32);
  uint64_t d0 = x0 ^ t0, d1 = x1 ^ t1;
  m1 = m2 = 16;
  c1 = c2 = 0;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    if (!(d0 | d1)) break;
    const bool lo = d0 != 0;
    const uint32_t bit = (uint32_t)__builtin_ctzll(lo ? d0 : d1) & ~7u;
    const uint32_t m = (lo ? 0u : 8u) + bit / 8;
    const uint32_t c = (uint32_t)(uint8_t)((lo ? x0 : x1) >> bit) | ((uint32_t)(uint8_t)((lo ? t0 : t1) >> bit) << 8);
    if (r == 0) { m1 = m; c1 = c; } else { m2 = m; c2 = c; }
    if (lo) d0 &= ~(0xffull << bit); else d1 &= ~(0xffull << bit);
  }
}

// Cooperative LCE, per thread: the pieces with a mismatch (pm), and in the
// first of them (mj) the first mismatch (mine, its chars cc) and, with
// `two`, the second (mine2, cc2).  The pieces are tested with xors first and
// only that piece is decoded (one diff instead of one per piece).
template <uint32_t J>
__device__ __forceinline__ void first_piece_diff(const uint4 (&xv)[J], const uint4 (&tv)[J], bool two,
                                                 uint32_t& mine, uint32_t& mj, uint32_t& cc, uint32_t& pm,
                                                 uint32_t& mine2, uint32_t& cc2) {
  uint32_t p = 0;
#pragma unroll
  for (uint32_t j = 0; j < J; j++) {
    const uint32_t d = (xv[j].x ^ tv[j].x) | (xv[j].y ^ tv[j].y) | (xv[j].z ^ tv[j].z) | (xv[j].w ^ tv[j].w);
    p |= (d != 0 ? 1u : 0u) << j;
  }
  pm = p;
  if (p) {
    // the lowest piece with a mismatch, by priority (a select per piece, so
    // that no indexed copy of the arrays goes to scratch)
    uint32_t x0 = xv[J - 1].x, x1 = xv[J - 1].y, x2 = xv[J - 1].z, x3 = xv[J - 1].w;
    uint32_t t0 = tv[J - 1].x, t1 = tv[J - 1].y, t2 = tv[J - 1].z, t3 = tv[J - 1].w;
#pragma unroll
    for (int j = (int)J - 2; j >= 0; j--) {
      const bool s = (p >> j) & 1u;
      x0 = s ? xv[j].x : x0; x1 = s ? xv[j].y : x1; x2 = s ? xv[j].z : x2; x3 = s ? xv[j].w : x3;
      t0 = s ? tv[j].x : t0; t1 = s ? tv[j].y : t1; t2 = s ? tv[j].z : t2; t3 = s ? tv[j].w : t3;
    }
    const uint4 x = make_uint4(x0, x1, x2, x3), t = make_uint4(t0, t1, t2, t3);
    mj = (uint32_t)__builtin_ctz(p);
    if (two) {
      diff16x2(x, t, mine, cc, mine2, cc2);
    } else {
      uint8_t xc = 0, tc = 0;
      mine = diff16(x, t, xc, tc);
      cc = (uint32_t)xc | ((uint32_t)tc << 8);
    }
  }
}

// Level geometry of the LCP block minima, staged in LDS.
struct Lv {
  const uint32_t* len;  // lvlLen
  const uint32_t* off;  // lvlOff (entries from lcp)
  int nlvl;
  int32_t n;
  const int32_t* lcp;
};

// ---- PSV (UP=false) / NSV (UP=true) as a state machine over 8-entry windows
// (rmq_tree.h:184-225).  State: cur/lim = remaining range of the current
// array (down: cur..lim, up: cur..lim), res = answer, idx = climbing index,
// ls = level | stage << 4.  Stages: 0 = LCP block of the start, 1 = climb
// level L, 2 = descend level L, 3 = final LCP block, 4 = done.
constexpr uint32_t kScanDone = 4u << 4;

template <bool UP>
__device__ __forceinline__ int32_t window_base(int32_t cur) {
  const int32_t b = UP ? (cur & ~3) : (cur & ~3) - 4;
  return b < 0 ? 0 : b;
}

template <bool UP>
__device__ __forceinline__ uintptr_t scan_addr(const Lv& V, int32_t cur, uint32_t ls) {
  const uint32_t stg = ls >> 4;
  const uint32_t off = (stg == 0 || stg == 3) ? 0u : V.off[ls & 15];
  return (uintptr_t)(V.lcp + off + (uint32_t)window_base<UP>(cur));
}

// Stage transitions that need no memory access.  At most two per call (the
// usual case needs one); a range left empty is seen as exhausted by the next
// scan_step, which settles again, so the walk stays correct with fewer
// unrolled copies of this code.
template <bool UP>
__device__ __forceinline__ void scan_settle(const Lv& V, int32_t& cur, int32_t& lim, int32_t& res, int32_t& idx,
                                            uint32_t& ls) {
  for (int guard = 0; guard < 2; guard++) {
    uint32_t stg = ls >> 4, L = ls & 15;
    if (stg == 4) return;
    if (UP ? (cur <= lim) : (cur >= lim)) return;  // range left: needs a load
    if (stg == 0) {
      stg = 1;
      L = 0;
    } else if (stg == 1) {
      const int32_t len = (int32_t)V.len[L];
      const bool top = UP ? (min(idx | 63, len - 1) >= len - 1) : ((idx & ~63) == 0);
      idx >>= 6;
      L++;
      if (top || (int)L >= V.nlvl) { res = -1; ls = kScanDone; return; }
    } else {  // a descent always finds (block minimum < ub); defensive
      res = -1;
      ls = kScanDone;
      return;
    }
    const int32_t len = (int32_t)V.len[L];
    if (!UP) { cur = idx - 1; lim = idx & ~63; }
    else { cur = idx + 1; lim = min(idx | 63, len - 1); }
    ls = L | (stg << 4);
  }
}

template <bool UP>
__device__ __forceinline__ void scan_start(const Lv& V, int32_t i, int32_t& cur, int32_t& lim, int32_t& res,
                                           int32_t& idx, uint32_t& ls) {
  res = -1;
  if (UP && i >= V.n) { ls = kScanDone; return; }
  ls = 0;
  idx = i >> 6;
  cur = i;
  lim = UP ? min(i | 63, V.n - 1) : (i & ~63);
  scan_settle<UP>(V, cur, lim, res, idx, ls);
}

template <bool UP>
__device__ __forceinline__ void scan_step(const Lv& V, const uint4& v0, const uint4& v1, int32_t ub, int32_t& cur,
                                          int32_t& lim, int32_t& res, int32_t& idx, uint32_t& ls) {
  const int32_t base = window_base<UP>(cur);
  const int32_t e[8] = {(int32_t)v0.x, (int32_t)v0.y, (int32_t)v0.z, (int32_t)v0.w,
                        (int32_t)v1.x, (int32_t)v1.y, (int32_t)v1.z, (int32_t)v1.w};
  const int32_t klo = (UP ? max(cur, base) : max(lim, base)) - base;
  const int32_t khi = (UP ? min(lim, base + 7) : min(cur, base + 7)) - base;
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 8; k++)
    if (k >= klo && k <= khi && e[k] < ub) m |= 1u << k;
  if (m) {
    const int32_t k = UP ? base + __builtin_ctz(m) : base + 31 - __builtin_clz(m);
    const uint32_t stg = ls >> 4, L = ls & 15;
    if (stg == 0 || stg == 3) { res = k; ls = kScanDone; return; }
    // hit in a level array: descend into block k of the level below
    int32_t top;
    uint32_t nls;
    if (L == 0) { top = V.n - 1; nls = 3u << 4; }
    else { top = (int32_t)V.len[L - 1] - 1; nls = (L - 1) | (2u << 4); }
    const int32_t lo = k * 64, hi = min(k * 64 + 63, top);
    if (UP) { cur = lo; lim = hi; } else { cur = hi; lim = lo; }
    ls = nls;
    return;
  }
  cur = UP ? base + 8 : base - 1;
  scan_settle<UP>(V, cur, lim, res, idx, ls);
}

}  // namespace

struct Walk2Args {
  DevRef R;
  const uint8_t* text;
  const uint64_t* docOff;
  const Chunk* chunks;
  uint32_t nchunks;
  const uint32_t* order;      // chunk ids grouped by band
  const uint32_t* bandStart;  // nbands + 1
  uint32_t nbands;
  uint32_t* nextChunk;        // one counter per band, 64 B apart (zeroed)
  Pool pool;
  uint32_t* chunkCount;
  unsigned long long* stats;  // STATS builds: per-phase lane-steps, wave-steps, ...
};

#ifndef CMSBWT_COOP_J
#define CMSBWT_COOP_J 4
#endif
constexpr uint32_t kCoopJ = CMSBWT_COOP_J;  // 16-B pieces per thread per cooperative round
// pending long extensions served together (r03 A/B, walk kernel: 1 -> 15.12 ms,
// 4 -> 14.74 ms: a round trip of the wave serves four slots instead of ~2)
// Round 6, re-measured on the current kernel (slot refill, memo; A/B on one
// box each, bit-exact, walk kernel): 3 -> 11.25-11.36 ms, 4 -> 10.78-10.90,
// 5 -> 10.69, 6 -> 10.62-10.67, 8 -> 10.39-10.42, 12 -> 10.35-10.48, 16 ->
// 10.28-10.43; with 32-record pool blocks 8 -> 10.16-10.30, 12 -> 9.92-10.01.
// A session of the four refilled slots then serves at least twelve
// extensions, so the wave enters the cooperative loop a third as often.
// (Round 3, before the refill: 3: 14.58 ms, 4: 14.74, 5: 15.6, 8: 17.1.)
#ifndef CMSBWT_COOP_MIN
#define CMSBWT_COOP_MIN 12
#endif
constexpr uint32_t kCoopMin = CMSBWT_COOP_MIN;
// slots of the refilled session (CMSBWT_COOP_SLOTS: 4 slots of 16 threads,
// 1 KiB per slot per round with kCoopJ = 4; 8 slots of 8 threads, 512 B)
#ifndef CMSBWT_COOP_SLOTS
#define CMSBWT_COOP_SLOTS 4
#endif
constexpr uint32_t kSlots = CMSBWT_COOP_SLOTS;
constexpr uint32_t kSlotW = 64 / kSlots;
static_assert(kSlots == 4 || kSlots == 8 || kSlots == 16, "slots of 16, 8 or 4 threads");
// a cooperative round tests its pieces with xors and decodes only the first
// mismatching one (CMSBWT_PIECE_XOR=0: every piece decoded, for A/B)
#ifndef CMSBWT_PIECE_XOR
#define CMSBWT_PIECE_XOR 1
#endif
constexpr bool kPieceXor = CMSBWT_PIECE_XOR != 0;
// fused cooperative LCE (CMSBWT_COOP_FUSED=1): the four slots' loads ride
// in the wave's memory step beside the lanes' own loads, so an extension is
// compared while the other lanes keep walking, instead of in a session that
// stops the wave (pending lanes join a free slot at the end of the step)
#ifndef CMSBWT_COOP_FUSED
#define CMSBWT_COOP_FUSED 0
#endif
constexpr bool kFused = CMSBWT_COOP_FUSED != 0;
static_assert(!kFused || kSlots == 4, "the fused slots are four of 16 threads");
// four slots whose ended extensions are replaced by pending lanes within the
// round loop (CMSBWT_COOP_REFILL=0 builds the fixed groups of four for A/B)
#ifndef CMSBWT_COOP_REFILL
#define CMSBWT_COOP_REFILL 1
#endif
constexpr bool kCoopRefill = CMSBWT_COOP_REFILL != 0;
// short unique matches go straight to the next position's probe instead of
// the PLCP skip (CMSBWT_PROBE_NOSKIP=0 keeps the skip, for A/B)
#ifndef CMSBWT_PROBE_NOSKIP
#define CMSBWT_PROBE_NOSKIP 1
#endif
constexpr bool kProbeNoSkip = CMSBWT_PROBE_NOSKIP != 0;
// the text side of cooperative extensions read non-temporally (r03: 15.12 ->
// 14.96 ms); CMSBWT_COOP_TEXT_NT=0 reads it through L2 (the bytes past the
// mismatch are read again by the next extension and the skip)
#ifndef CMSBWT_COOP_TEXT_NT
#define CMSBWT_COOP_TEXT_NT 1
#endif
// alignment memo: a cooperative extension that ends at a mismatch (a SNP of a
// copy) also reports the next mismatch at the same text-to-reference offset in
// the bytes its round read, or how far they are clean; the extension at that
// offset after the SNP (the copy's next long match) starts there instead of
// reading those bytes again (CMSBWT_ALIGN_MEMO=1)
#ifndef CMSBWT_ALIGN_MEMO
#define CMSBWT_ALIGN_MEMO 1
#endif
constexpr bool kAlignMemo = CMSBWT_ALIGN_MEMO != 0;
// the memo's four words per lane in LDS instead of registers: read when an
// extension starts, written when a cooperative extension ends; four VGPRs
// fewer across the step loop.  With the paired probes' prefetch the
// specialised instance spilled five VGPRs to scratch (writes of the launch
// 1.85 -> 2.41 GB); without the spills (A/B one box, two runs each,
// bit-exact): walk kernel 10.01-10.02 -> 9.18-9.22 ms.  LDS per block
// 33.1 -> 37.2 KB (four blocks per CU still fit).  CMSBWT_MEMO_LDS=0 keeps
// them in registers
#ifndef CMSBWT_MEMO_LDS
#define CMSBWT_MEMO_LDS 1
#endif
constexpr bool kMemoLds = CMSBWT_MEMO_LDS != 0;
// the chunk id and pool-block sequence of each lane in LDS (used when a pool
// block starts and when the chunk ends): two VGPRs fewer (CMSBWT_CHUNK_LDS;
// A/B one box, bit-exact: walk kernel 9.20-9.25 vs 9.02-9.28 ms, no change
// once nothing spills, so it stays off)
#ifndef CMSBWT_CHUNK_LDS
#define CMSBWT_CHUNK_LDS 0
#endif
constexpr bool kChunkLds = CMSBWT_CHUNK_LDS != 0;
// diagnostic builds (CMSBWT_MEMO_CHECK=1): a memo hit only predicts; the LCE
// runs as without the memo and the result is compared with the prediction
// (and the predicted match end with the reference and text bounds); the
// first disagreements are printed
#ifndef CMSBWT_MEMO_CHECK
#define CMSBWT_MEMO_CHECK 0
#endif
constexpr bool kMemoCheck = CMSBWT_MEMO_CHECK != 0;
// probe prefetch (specialised instance): a probe step at position i whose
// window holds K + 1 symbols also loads the table entry of position i + 1
// (its code is known from the same window); when the walk reaches i + 1 by
// the next-position route, that entry is used in a second pass of the compute
// phases of the same iteration (PC_PFX), so a mismatch region's heads (one
// probe each) take one load step per two positions.  Measured (round 5,
// config 3): probe lane-steps 131.9 M -> 69.3 M, wave steps 4.04 M -> 2.45 M,
// walk kernel unchanged (12.0 ms either way, 5 VGPRs spilled with it): the
// walk is bound by its random-line traffic, not by its dependent round
// trips.  Off by default; CMSBWT_PFX_PREFETCH=1 builds it (bit-exact).
#ifndef CMSBWT_PFX_PREFETCH
#define CMSBWT_PFX_PREFETCH 0
#endif
// paired probe lines (round 6): with the paired level-K table (DevRef::pfk)
// the probe of i and the prefetched probe of i + 1 read the same 64-byte line
// (their K-mers share K - 1 symbols), so a mismatch region's heads take one
// random line per two positions instead of one each.  Turns the prefetch on.
// Measured (config 3, one box, bit-exact): L2 -> fabric read requests 286 M
// -> 250 M per launch, walk kernel 10.73-10.86 -> 10.65-10.82 ms (within the
// box's spread), with non-temporal probe loads 10.95-11.03 ms: the walk is
// not bound by its random lines.  Re-measured on
// the final configuration (cooperative sessions from 12 lanes, 32-record
// blocks; one box, two runs each, bit-exact): walk kernel 9.97-10.06 ->
// 9.83-9.93 ms (the prefetch alone, without the pairs: 10.42-10.54), so it
// is on: the table costs 4.3 GB of HBM at K = 14.  The environment switch
// CMSBWT_PFX_PAIR=0 skips the table (the walk then prefetches unpaired);
// -DCMSBWT_PFX_PAIR=0 builds the walk without either.
#ifndef CMSBWT_PFX_PAIR
#define CMSBWT_PFX_PAIR 1
#endif
// the paired probes as cached loads (non-temporal loads of one line do not
// share a fabric request)
#ifndef CMSBWT_PAIR_CACHED
#define CMSBWT_PAIR_CACHED 1
#endif
constexpr bool kPairCached = CMSBWT_PAIR_CACHED != 0;
// the register barrier after a memo hit in the specialised instance too (the
// generic instance has it unless CMSBWT_MEMO_GENERIC_BARRIER=0).  Round 6:
// the fault it guarded against is the backend pass SIOptimizeVGPRLiveRange,
// now disabled for this file (Makefile W2FLAGS); the barrier
// stays in both instances as a second guard (A/B on one box: walk kernel
// 10.83-10.87 ms without, 10.80-10.87 ms with it)
#ifndef CMSBWT_MEMO_BARRIER
#define CMSBWT_MEMO_BARRIER 1
#endif
constexpr bool kMemoBarrier = CMSBWT_MEMO_BARRIER != 0;
// (tools/memo_isa.sh) CMSBWT_MEMO_GENERIC_BARRIER=0 drops the barrier from the
// generic instance too: the build that reproduces the code-generation fault
#ifndef CMSBWT_MEMO_GENERIC_BARRIER
#define CMSBWT_MEMO_GENERIC_BARRIER 1
#endif
constexpr bool kMemoGenBarrier = CMSBWT_MEMO_GENERIC_BARRIER != 0;
__device__ uint32_t g_memo_bad = 0;
// waves per SIMD of the walk (Makefile W2WAVES; measured 3 -> 16.50 ms,
// 4 -> 16.44-16.68, 5 -> 16.9, 6 -> 31.3 with register spills)
#ifndef CMSBWT_W2_WAVES
#define CMSBWT_W2_WAVES 4
#endif
// head records staged per lane in LDS and stored kHeadBufN at a time (one
// 64- or 128-byte piece of the lane's pool block) instead of one 16-byte
// store per head, which left every record a partial line of its own on the
// fabric (A/B: walk kernel 11.24-11.38 -> 10.73-10.79 ms with 4 records;
// 8, a whole line: 10.96-11.02 -> 10.74-10.87 ms on another box)
#ifndef CMSBWT_HEAD_BUF
#define CMSBWT_HEAD_BUF 8
#endif
constexpr uint32_t kHeadBufN = CMSBWT_HEAD_BUF;  // records per store (0: none; 4: 64 B; 8: a 128-byte line)
constexpr bool kHeadBuf = kHeadBufN != 0;
static_assert(kHeadBufN == 0 || (kHeadBufN <= kPoolB && kPoolB % kHeadBufN == 0), "pieces tile the pool block");
static_assert(sizeof(HeadRec) == sizeof(uint4), "head records are stored as uint4");
template <bool STATS, bool FAST>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CMSBWT_W2_WAVES, 8)))
k_ms_walk2(Walk2Args A) {
  // four blocks of 256 lanes per CU (four waves per SIMD) need <= 40 KB of
  // LDS per block: the per-lane arrays below must fit beside each other
  static_assert((kHeadBuf ? kHeadBufN : 1) * 256 * 16 + (kMemoLds ? 256 : 1) * 16 + (kChunkLds ? 256 : 1) * 8 +
                        (kWalkLchar ? 256 : 1) * 8 + 32 * 8 + 256 + 2 * kMaxLevels * 4 + 17 * 4 <=
                    160 * 1024 / 4,
                "walk LDS per block exceeds a quarter of the CU's 160 KB");
  __shared__ unsigned long long sc[STATS ? 32 : 1];
  __shared__ uint8_t kmapL[256];
  __shared__ uint32_t lvlL[2 * kMaxLevels];
  __shared__ uint32_t pfxL[17];
  __shared__ uint4 hbuf[kHeadBuf ? kHeadBufN : 1][256];  // 16 B x kHeadBufN per lane (slot-major: no bank conflicts)
  __shared__ uint4 memoL[kMemoLds ? 256 : 1];  // (CMSBWT_MEMO_LDS) amAlign, amLo, amFront, amC per lane
  if (kMemoLds) memoL[threadIdx.x] = make_uint4(0u, 0xffffffffu, 0u, 0u);
  __shared__ uint2 chunkL[kChunkLds ? 256 : 1];  // (CMSBWT_CHUNK_LDS) cid, seq per lane
  // (CMSBWT_WALK_LCHAR) per lane: a text index and its byte, the first byte of
  // the last window that a window one position further replaced
  __shared__ uint2 prevL[kWalkLchar ? 256 : 1];
  if (kWalkLchar) prevL[threadIdx.x] = make_uint2(0xffffffffu, 0u);
  if (STATS && threadIdx.x < 32) sc[threadIdx.x] = 0;
  if (A.R.pfx) kmapL[threadIdx.x] = A.R.kmap[threadIdx.x];  // blockDim == 256
  if (threadIdx.x < 17) pfxL[threadIdx.x] = A.R.pfxOff[threadIdx.x];
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < kMaxLevels; k++) {
      lvlL[k] = A.R.lvlLen[k];
      lvlL[kMaxLevels + k] = A.R.lvlOff[k];
    }
  }
  __syncthreads();
  const DevRef& R = A.R;
  // table configuration; FAST instances (DNA alphabet, exact carried
  // intervals, every walk table present: the benchmark's case) fold these to
  // constants, so the code of the other configurations is not emitted
  const bool hasPfx = FAST || R.pfx != nullptr;
  const bool pfxDna = FAST || R.pfxDna != 0;
  const bool pfxExact = FAST || R.pfxExact != 0;
  const bool hasLd = FAST || R.ld != nullptr;
  const bool hasIr = FAST || R.ir != nullptr;
  // the alignment memo runs in both instances (the generic one with the
  // register barrier at a hit, see start_lce)
  const bool memo = kAlignMemo;
  const Lv V{lvlL, lvlL + kMaxLevels, R.nlvl, (int32_t)R.n, R.lcp};
  const uint32_t n = R.n;
  const uintptr_t X = (uintptr_t)R.x;
  const uintptr_t SA = (uintptr_t)R.sa;
  const uintptr_t P = (uintptr_t)R.plcp;
  const uintptr_t P8 = (uintptr_t)R.plcp8;
  const uint32_t lane = threadIdx.x & 63;

  // chunk
  uint32_t cid = 0, a = 0, b = 0;
  uintptr_t T = 0;
  // walk state (FN:1151-1196)
  uint32_t i = 0, len = 0, pos = 0, prevPos = 0;
  int32_t lb = 0, rb = 0;
  bool smaller = false;
  // text window of the prefix-table path: tw = t[twAt .. twAt+16), with the
  // code of its first wm <= K symbols in wcode
  uint4 tw = make_uint4(0, 0, 0, 0);
  uint32_t twAt = 0xffffffffu, wcode = 0, wm = 0;
  // (prefetch) the window's 2-bit codes of all 16 bytes and its first
  // non-symbol index; the prefetched entry (pfE) is that of position pfAt
  constexpr bool kPrefetch = FAST && (CMSBWT_PFX_PREFETCH != 0 || CMSBWT_PFX_PAIR != 0);
  // paired lines when the table is there (a runtime choice: CMSBWT_PFX_PAIR=0)
  const bool pairOn = kPrefetch && CMSBWT_PFX_PAIR != 0 && R.pfk != nullptr;
  const uint32_t* const pfxK = pairOn ? R.pfk : R.pfx;  // where the prefetched entries live
  uint32_t wfull = 0, wbad = 0, pfAt = 0xffffffffu;
  uint2 pfE = make_uint2(0u, 0u);
  // the 32 text bytes t[t32At ..) the last skip step loaded around the match
  // end: the probes of the next positions (a mismatch region) take their
  // windows from them instead of loading the text again
  uint4 t32a = make_uint4(0, 0, 0, 0), t32b = t32a;
  uint32_t t32At = 0xfffffff0u;
  // alignment memo (kAlignMemo): at offset amAlign = pos - i the text
  // positions [amLo, amFront) match the reference; amC bit 16: the bytes at
  // amFront differ (x byte | text byte << 8)
  uint32_t amAlign = 0, amLo = 0xffffffffu, amFront = 0, amC = 0;
  // CMSBWT_MEMO_CHECK builds: the memo's prediction, checked against the LCE
  uint32_t chkOn = 0, chkLen = 0, chkC = 0, chkLo = 0, chkLen0 = 0;
  // emission
  // pool blocks are reserved kPoolBatch at a time (blk .. blkEnd) and kept
  // across this lane's chunks; blocks never started keep blkMeta.x = ~0
  uint32_t count = 0, blk = 0xffffffffu, blkEnd = 0, fill = kPoolB, seq = 0;
  uint32_t phase = PH_NEXT, use = 0;
  uintptr_t ad0 = X, ad2 = X;
  // fused cooperative LCE: the slots' lanes (6 bits each), open slots, lanes
  // held by a slot; per thread: its slot's offset and x / text addresses
  uint64_t fLs = 0, fSlotted = 0;
  uint32_t fOpen = 0, fRun = 0;
  uintptr_t fXa = X, fTa = X;
  // phase-local slots
  int32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0, u4 = 0, u5 = 0, u6 = 0, u7 = 0, u8 = 0;
  uint32_t u9 = 0;
  // binary search (BS_*): u0 = c | ansVal << 8 | ansSet << 16 | ubMode << 17,
  //   u1 = lo, u2 = hi (exclusive), u3 = probe, u5 = new lb while searching the right end
  // EXT_*: u0 = the text character
  // skip (SKIP1/GALLOP/SKIPBS): u1 = lo, u2 = hi, u3 = probe, u4 = gallop step
  // ADJ0: u0 / u5 = the two ISA values;  ADJ: PSV = (u0 cur, u1 lim, u2 res,
  //   u3 idx, u4 ls), NSV = (u5, u6, u7, u8, u9)
  // `len` doubles as `off` during an extension (FN:48: off starts at len).

  auto begin_bs = [&]() {  // binary searches for the character at j = i + len
    phase = PH_BS_TEXT;
    u1 = lb;
    u2 = rb + 1;
    u3 = (u1 + u2) >> 1;
    u0 = 0;
    ad0 = T + i + len;
    ad2 = SA + 4ull * (uint32_t)u3;
    use = U0B | U2D;
  };
  // a new text window at `at`: codes of its leading symbols (at most K)
  auto set_window = [&](const uint4 v, uint32_t at) {
    if (kWalkLchar && twAt != 0xffffffffu && twAt + 1 == at) prevL[threadIdx.x] = make_uint2(twAt, tw.x & 0xffu);
    tw = v;
    twAt = at;
    const uint32_t K = R.kmerK, Bb = R.kmerB;
    if (pfxDna) {  // alphabet ACGT: 2-bit codes of 4 bytes at a time
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      uint32_t full = 0, bad = 16;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        // A C G T (0x41 43 47 54) -> 0 1 2 3 in bits 1..2 xor 2..3 of each byte
        const uint32_t c = ((w4[q] >> 1) ^ (w4[q] >> 2)) & 0x03030303u;
        const uint32_t x = __builtin_amdgcn_perm(0u, 0x54474341u, c) ^ w4[q];  // zero byte: a symbol
        if (bad == 16 && x) bad = 4 * q + ((uint32_t)__builtin_ctz(x) >> 3);
        full |= (((c & 3u) << 6) | ((c >> 4) & 0x30u) | ((c >> 14) & 0xcu) | ((c >> 24) & 3u)) << (24 - 8 * q);
      }
      wm = bad < K ? bad : K;
      wcode = wm ? full >> (32 - 2 * wm) : 0u;
      if (kPrefetch) {
        wfull = full;
        wbad = bad;
      }
      return;
    }
    uint32_t code = 0, m = 0;
    bool run = true;
#pragma unroll
    for (uint32_t d = 0; d < 16; d++) {
      if (d < K && run) {
        const uint32_t w = d < 4 ? v.x : d < 8 ? v.y : d < 12 ? v.z : v.w;
        const uint32_t mp = kmapL[(w >> (8 * (d & 3))) & 0xff];
        if (mp == 0xff) run = false;
        else { code = (code << Bb) | mp; m = d + 1; }
      }
    }
    wcode = code;
    wm = m;
  };
  // probe of the prefix tables for t[i..i+m) (window at i): its interval, or
  // the answer entry; without pfxExact also the carried prefix's entry (the
  // interval must be exactly t[i..i+len)'s, not the root of FN:37-39); with
  // it the window at i + 1 for the next position
  auto pfx_probe = [&]() {
    const uint32_t m = wm, code = wcode, Bb = R.kmerB;
    // the next byte is no symbol (document end), or len = 0 away from the
    // root: character by character
    if (m <= len || (len == 0 && !(lb == 0 && rb == (int32_t)n - 1))) {
      begin_bs();
      return;
    }
    phase = PH_PFX_PROBE;
    u6 = (int32_t)code;  // kept: the probe step replaces the window
    u7 = (int32_t)m;
    const bool pairK = pairOn && m == R.kmerK;
    if (pairK) {  // slot t[i] of line t[i+1 .. i+K) (its K-1 symbol suffix)
      const uint32_t K1 = 2 * (R.kmerK - 1);
      ad0 = (uintptr_t)(R.pfk + 2 * (8ull * (code & ((1u << K1) - 1u)) + (code >> K1)));
    } else {
      ad0 = (uintptr_t)(R.pfx + pfxL[m] + 2 * code);
    }
    use = U0E;
    if (kPrefetch && m == R.kmerK && R.kmerK <= 15 && wbad > R.kmerK) {
      // the entry of i + 1: symbols 1 .. K of this window (paired: slot
      // 4 + t[i+K] of the same line t[i+1 .. i+K))
      const uint32_t K = R.kmerK;
      const uint32_t code1 = (wfull >> (32 - 2 * (K + 1))) & ((1u << (2 * K)) - 1u);
      u8 = pairK ? (int32_t)(2 * (8 * (code1 >> 2) + 4 + (code1 & 3))) : (int32_t)(pfxL[K] + 2 * code1);
      use |= U3E;
    }
    if (pfxExact) {
      if (i + 1 - t32At <= 16u) {
        use |= UREG;
      } else {
        ad2 = T + i + 1;
        use |= U2Q;
      }
    } else if (len > 0) {
      ad2 = (uintptr_t)(R.pfx + pfxL[len] + 2 * (code >> (Bb * (m - len))));
      use |= U2E;
    }
  };
  auto begin_pfx = [&]() {
    if (twAt == i) {
      if (kPrefetch && pfAt == i && wm == R.kmerK && wm > len && !(len == 0 && !(lb == 0 && rb == (int32_t)n - 1))) {
        phase = PC_PFX;  // (pfx_probe's load, served by the prefetched entry)
        use = 0;
        pfAt = 0xffffffffu;
        return;
      }
      pfx_probe();
    } else {
      phase = PH_PFX_TEXT;
      ad0 = T + i;
      use = U0Q;
    }
  };
  // next character(s) over a large interval: prefix-rank tables below depth K
  auto begin_search = [&]() {
    if (hasPfx && len < R.kmerK) begin_pfx();
    else begin_bs();
  };
  auto isa1 = [&]() {
    phase = PH_ISA1;
    if (hasIr) { ad0 = (uintptr_t)(R.ir + pos + 1); use = U0Q; }
    else { ad0 = (uintptr_t)(R.isa + pos + 1); use = U0D; }
  };
  // the carried interval after a skip or a mismatch is not needed when the
  // next position resolves by a table probe (pfxExact, len < K, K symbols
  // ahead): it is marked unknown (lb < 0), the root when len = 0
  auto virtual_interval = [&]() {
    if (len == 0) { lb = 0; rb = (int32_t)n - 1; }
    else { lb = -1; rb = -2; }
  };
  // text index of the 32 bytes a skip step loads: the next position after an
  // exit inside the PLCP window lies at offset 0..16 of them
  auto skip_text_base = [&]() -> uint32_t { return i + len + 1 >= 16 ? i + len - 15 : 0u; };
  auto skip_done = [&](uint32_t s) {
    i += s;
    len -= s;
    pos += s;
    if (pfxExact && len < R.kmerK) {  // the window at i + 1 decides
      phase = PH_SKTXT;
      ad0 = T + i + 1;
      use = U0Q;
    } else {
      isa1();
    }
  };
  // adjustInterval(lo, hi, len) from the records of lo (PSV side: LCP[lo],
  // LCP[lo-1], ..) and of hi (NSV side: LCP[hi+1], ..); the general scan
  // (ADJ0/ADJ) when the answer is not inside them
  auto adj_records = [&](uint32_t lo, uint32_t hi, const uint4& rl, const uint4& rh) {
    if (len - 1u < 254u) {
      // bytes 0..5 of the PSV side (rl.y, rl.z) and of the NSV side (rh.z
      // from byte 2, rh.w), compared in 32-bit registers
      int jp = -1, jn = -1;
#pragma unroll
      for (int j = 5; j >= 0; j--) {
        const uint32_t pb = (j < 4 ? rl.y >> (8 * j) : rl.z >> (8 * (j - 4))) & 0xffu;
        const uint32_t nb = (j < 2 ? rh.z >> (16 + 8 * j) : rh.w >> (8 * (j - 2))) & 0xffu;
        if (pb < len) jp = j;
        if (nb < len) jn = j;
      }
      if (jp >= 0 && jn >= 0) {
        lb = (int32_t)lo - jp;
        rb = (int32_t)hi + jn;
        phase = PC_ADV;
        use = 0;
        return;
      }
    }
    u0 = (int32_t)lo;
    u5 = (int32_t)hi;
    phase = PC_ADJ0;
    use = 0;
  };
  // gallop (u4 = step, u1 = lo, below the cap u2 where the predicate holds)
  // then binary search on (u1, u2]
  auto skip_probe = [&](bool galloping) {
    if (galloping) {
      const uint64_t t = (uint64_t)(uint32_t)u1 + (uint32_t)u4;
      if (t < (uint32_t)u2) {
        u3 = (int32_t)t;
        phase = PH_GALLOP;
        ad0 = P + 4ull * (pos + 1 + (uint32_t)u3);
        use = U0D;
        return;
      }
    }
    if ((uint32_t)u2 - (uint32_t)u1 > 1) {
      u3 = (int32_t)((uint32_t)u1 + (((uint32_t)u2 - (uint32_t)u1) >> 1));
      phase = PH_SKIPBS;
      ad0 = P + 4ull * (pos + 1 + (uint32_t)u3);
      use = U0D;
    } else {
      skip_done((uint32_t)u2);
    }
  };
  // FN:52-62 from (pos, len): 16 bytes of x and of the text, unless the
  // alignment memo already knows where this offset's match ends
  auto start_lce = [&]() {
    if (kMemoLds && memo) {
      const uint4 m = memoL[threadIdx.x];
      amAlign = m.x;
      amLo = m.y;
      amFront = m.z;
      amC = m.w;
    }
    if (memo && pos - i == amAlign && i + len >= amLo && i + len <= amFront) {
      if (kMemoCheck) {  // predict only; the LCE below runs and PC_POST compares
        chkOn = 1;
        chkLen = amFront - i;
        chkC = amC;
        chkLo = amLo;
        chkLen0 = len;
      } else {
      len = amFront - i;
      // with the backend's SIOptimizeVGPRLiveRange pass on, the generic
      // instance was miscompiled here without this register barrier: the
      // head recorded after a hit carried pos = i + K + 1 (the pass gave
      // `pos` an undefined value on the path of the lanes that took the
      // branch before; DESIGN.md §3.1, tools/memo_isa.sh).  The pass is off
      // for this file; the barrier stays as a second guard
      if ((!FAST && kMemoGenBarrier) || kMemoBarrier) asm volatile("" : "+v"(pos));
      if (amC & 0x10000u) {  // the mismatch at amFront (FN:55)
        smaller = (int8_t)(uint8_t)amC > (int8_t)(uint8_t)(amC >> 8);
        phase = PC_POST;
        use = 0;
        return;
      }
      }
    }
    phase = PH_LCE;
    ad0 = X + pos + len;
    ad2 = T + i + len;
    use = U0Q | U2Q;
  };
  auto set_adj_addr = [&]() {
    use = 0;
    if ((uint32_t)u4 != kScanDone) { ad0 = scan_addr<false>(V, u0, (uint32_t)u4); use |= U0Q | U1Q; }
    if (u9 != kScanDone) { ad2 = scan_addr<true>(V, u5, u9); use |= U2Q | U3Q; }
  };
  auto adj_or_finish = [&]() {
    if ((uint32_t)u4 == kScanDone && u9 == kScanDone) {
      lb = u2 == -1 ? 0 : u2;
      rb = u7 == -1 ? (int32_t)n - 1 : u7 - 1;
      phase = PC_ADV;
      use = 0;
    } else {
      phase = PH_ADJ;
      set_adj_addr();
    }
  };

  // the probe entry (ex, ey) of t[i..i+m) (m = u7, code = u6): FN:45-88's
  // outcome as the binary searches would find it (PH_PFX_PROBE, and PC_PFX for
  // a prefetched entry)
  auto pfx_entry = [&](uint32_t ex, uint32_t ey) {
    const uint32_t m = (uint32_t)u7, code = (uint32_t)u6, Bb = R.kmerB;
    if (ey == (kPfxOne | 1u)) {  // t[i..i+m) occurs once, at ex: extend there (FN:52-62)
      lb = rb = 0;
      len = m;
      pos = ex;
      start_lce();
      return;
    }
    if (!(ey & kPfxAns)) {  // t[i..i+m) occurs: its interval, depth m
      lb = (int32_t)ex;
      rb = (int32_t)(ex + ey) - 1;
      len = m;
      phase = PC_CHAR;
      use = 0;
      return;
    }
    // answer entry: the longest occurring prefix t[i..i+l), the insertion
    // point's SA value and `smaller` of FN:65-76, as the binary searches
    // from the (exact) carried interval would find them
    len = ey & 0xffu;
    pos = ex;
    smaller = (ey & kPfxSmaller) != 0;
    use = 0;
    phase = PC_POST;
    if (ey & kPfxSingle) {
      lb = rb = 0;  // a one-suffix interval: the skip of FN:1175-1189 follows
    } else if (pfxExact && wm == R.kmerK) {
      lb = -1;  // the next position resolves by its own probe
      rb = -2;
    } else if (len == 0) {
      lb = 0;
      rb = (int32_t)n - 1;
    } else {  // contractLeft needs the interval of t[i..i+l)
      phase = PH_IVL;
      ad0 = (uintptr_t)(R.pfx + pfxL[len] + 2 * (code >> (Bb * (m - len))));
      use = U0E;
    }
  };

  while (true) {
    // ---- refill lanes from the chunk queues (one atomic per wave and band).
    // Chunks are banded by their offset inside the document; blocks that
    // share an XCD (equal blockIdx % 8 under round-robin placement) start on
    // the same band.  Exhausted bands are stolen from in turn.
    uint64_t need = __ballot(phase == PH_NEXT);
    for (uint32_t s2 = 0; need && s2 < A.nbands; s2++) {
      const uint32_t band = (blockIdx.x + s2) % A.nbands;
      const uint32_t first = (uint32_t)__builtin_ctzll(need);
      const uint32_t bs0 = A.bandStart[band], bsz = A.bandStart[band + 1] - bs0;
      uint32_t base = 0;
      if (lane == first) base = atomicAdd(&A.nextChunk[16 * band], (uint32_t)__popcll(need));
      base = __shfl(base, first);
      const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1));
      const bool mine = phase == PH_NEXT && base < bsz && rank < bsz - base;
      need &= ~__ballot(mine);
      if (mine) {
        cid = A.order[bs0 + base + rank];
        const Chunk ch = A.chunks[cid];
        T = (uintptr_t)(A.text + A.docOff[ch.doc]);
        a = ch.a;
        b = ch.b;
        count = 0;
        fill = kPoolB;
        seq = 0;
        if (kChunkLds) chunkL[threadIdx.x] = make_uint2(cid, 0u);
        i = a > 0 ? a - 1 : 0;
        if (i >= b) {
          A.chunkCount[cid] = 0;  // empty document: refills next iteration
        } else {
          len = 0;
          pos = n - 1;
          lb = 0;
          rb = (int32_t)n - 1;
          prevPos = 0xfffffffeu;  // prevPos + 1 never equals a position
          smaller = false;
          twAt = 0xffffffffu;
          t32At = 0xfffffff0u;  // (another document's bytes)
          if (kWalkLchar) prevL[threadIdx.x].x = 0xffffffffu;
          amLo = 0xffffffffu;
          if (kMemoLds) memoL[threadIdx.x].y = 0xffffffffu;
          pfAt = 0xffffffffu;
          if (hasPfx) {
            phase = PH_PFX_TEXT;
            ad0 = T + i;
            use = U0Q;
          } else {
            phase = PC_CHAR;
          }
        }
      }
    }
    if (need && phase == PH_NEXT && ((need >> lane) & 1)) {  // every band is empty
      phase = PH_DONE;
      use = 0;
    }

    // ---- compute phases, in chain order (ADJ0 -> PFX -> POST -> ADV -> CHAR;
    // POST reaches ADV when the contraction is dropped).  A second pass runs
    // when a lane's CHAR found its probe entry prefetched (PC_PFX), so that
    // position is settled in this iteration too.
    for (uint32_t pass = 0;; pass++) {
    if (phase == PC_ADJ0) {  // adjustInterval(lo = u0, hi = u5, len) (FN:11-25)
      const int32_t lo = u0, hi = u5;
      uint32_t ls0;
      scan_start<false>(V, lo, u0, u1, u2, u3, ls0);
      scan_start<true>(V, hi + 1, u5, u6, u7, u8, u9);
      u4 = (int32_t)ls0;
      adj_or_finish();
    }
    if (kPrefetch && phase == PC_PFX) {  // pfx_probe at i with the prefetched entry
      // the window at i + 1 from this one (15 bytes: K <= 14 symbols and the
      // prefetch's symbol K, as the text load at i + 1 would give them)
      const uint32_t K = R.kmerK;
      u6 = (int32_t)wcode;
      u7 = (int32_t)K;
      const uint4 sh = make_uint4(__builtin_amdgcn_alignbyte(tw.y, tw.x, 1), __builtin_amdgcn_alignbyte(tw.z, tw.y, 1),
                                  __builtin_amdgcn_alignbyte(tw.w, tw.z, 1), tw.w >> 8);
      set_window(sh, i + 1);
      pfx_entry(pfE.x, pfE.y);
    }
    if (phase == PC_POST) {  // head test and record (FN:1154-1171), then contraction
      if (kMemoCheck && chkOn) {  // the LCE's result against the memo's prediction
        chkOn = 0;
        const bool mm = (chkC & 0x10000u) != 0;
        const bool sm = (int8_t)(uint8_t)chkC > (int8_t)(uint8_t)(chkC >> 8);
        const uint32_t got = i + len;  // text index of the LCE's mismatch
        const bool bad = mm ? (len != chkLen || smaller != sm) : (len < chkLen);
        if (bad || chkLen + amAlign + i >= n || got + amAlign >= n + (uint32_t)kTextPad) {
          const uint32_t k = atomicAdd(&g_memo_bad, 1u);
          if (k < 16)
            printf("[memo] chunk %u i %u pos %u len0 %u -> lce len %u smaller %d | memo align %u lo %u front %u "
                   "c %05x predicted len %u smaller %d\n",
                   cid, i, pos, chkLen0, len, (int)smaller, amAlign, chkLo, chkLen + i, chkC, chkLen, (int)sm);
        }
      }
      const bool head = i >= a && pos != prevPos + 1;
      // new pool blocks: one atomic per wave for every lane whose reserved
      // blocks ran out (a single counter takes every reservation of the grid)
      const bool refill = head && fill == kPoolB && blk + 1 >= blkEnd;
      const uint64_t rq = __ballot(refill);
      if (rq) {
        const uint32_t leader = (uint32_t)__builtin_ctzll(rq);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(A.pool.used, kPoolBatch * (uint32_t)__popcll(rq));
        base = __shfl(base, (int)leader);
        if (refill) {
          blk = base + kPoolBatch * (uint32_t)__popcll(rq & ((1ull << lane) - 1)) - 1;  // blk++ below
          blkEnd = blk + 1 + kPoolBatch;
        }
      }
      if (head) {
        // flags: smaller, and the byte before the head when the window gave it
        uint32_t hflags = smaller ? 1u : 0u;
        if (kWalkLchar) {
          const uint2 pv = prevL[threadIdx.x];
          if (i > 0 && pv.x == i - 1) hflags |= (0x100u | pv.y) << 8;
        }
        if (fill == kPoolB) {
          blk++;
          fill = 0;
          if (kChunkLds) {
            const uint2 cs = chunkL[threadIdx.x];
            cid = cs.x;
            seq = cs.y;
          }
          if (blk < A.pool.capBlocks) A.pool.blkMeta[blk] = make_uint2(cid, seq);  // (one 8-byte store)
          seq++;
          if (kChunkLds) chunkL[threadIdx.x].y = seq;
        }
        if (kHeadBuf) {
          constexpr uint32_t M = kHeadBufN - 1;
          hbuf[fill & M][threadIdx.x] = make_uint4(i, pos, len, hflags);
          if ((fill & M) == M && blk < A.pool.capBlocks) {  // a full piece of the block
            uint4* dst = (uint4*)(A.pool.rec + (uint64_t)blk * kPoolB + (fill - M));
#pragma unroll
            for (uint32_t k = 0; k < kHeadBufN; k++) dst[k] = hbuf[k][threadIdx.x];
          }
        } else if (blk < A.pool.capBlocks) {
          HeadRec r;
          r.start = i;
          r.pos = pos;
          r.len = len;
          r.flags = hflags;
          A.pool.rec[(uint64_t)blk * kPoolB + fill] = r;
        }
        fill++;
        count++;
      }
      len--;
      if (kProbeNoSkip && pfxExact && hasPfx && lb == rb && len < R.kmerK && twAt == i + 1 && wm == R.kmerK) {
        // a short unique match (the mismatch region around a SNP): the
        // next position's K symbols are decoded, and its probe gives its MS
        // triple, which depends on the text alone -- a
        // continuation shows as pos == prevPos + 1 (no head) -- so the skip
        // (FN:1175-1189, one PLCP and one text load that usually skip
        // nothing here) is not taken
        virtual_interval();
        phase = PC_ADV;
        use = 0;
      } else if (lb == rb) {  // FN:1175-1189: skip, then adjustInterval(ISA[pos+1])
        // the exit is the first q >= pos+1 with PLCP[q] + q >= T = pos+1+len;
        // PLCP of a random-like text is ~log4 n, so it lies ~12 below T:
        // probe the 16 entries below T first
        phase = PH_SKIP1;
        const uint64_t TT = (uint64_t)pos + 1 + len;
        ad0 = P8 + (TT >= 16 ? TT - 16 : 0);  // min(PLCP, 255) bytes: one 16-B load
        use = U0Q;
        if (pfxExact && hasPfx) {  // and the 32 text bytes around the match end: the next window
          ad2 = T + skip_text_base();
          use |= U2Q | U3Q;
        }
      } else if (lb < 0) {  // unknown interval: the next position's probe supersedes contractLeft
        if (len == 0) { lb = 0; rb = (int32_t)n - 1; }
        phase = PC_ADV;
        use = 0;
      } else {  // FN:1190-1194: contractLeft from the psi records of lb and rb
        phase = PH_CONP;
        ad0 = (uintptr_t)(R.pr + (uint32_t)lb);
        ad2 = (uintptr_t)(R.pr + (uint32_t)rb);
        use = U0Q | U2Q;
      }
    }
    if (phase == PC_ADV) {  // FN:1195-1196
      i++;
      prevPos = pos;
      if (i >= b) {
        if (kChunkLds) cid = chunkL[threadIdx.x].x;
        A.chunkCount[cid] = count;
        phase = PH_NEXT;
        use = 0;
        constexpr uint32_t M = kHeadBuf ? kHeadBufN - 1 : 0;
        if (kHeadBuf && fill != kPoolB && (fill & M) && blk < A.pool.capBlocks) {  // the chunk's last records
          uint4* dst = (uint4*)(A.pool.rec + (uint64_t)blk * kPoolB + (fill & ~M));
          for (uint32_t k = 0; k < (fill & M); k++) dst[k] = hbuf[k][threadIdx.x];
        }
      } else {
        phase = PC_CHAR;
      }
    }
    if (phase == PC_CHAR) {  // next character of computeMSFactorAt at j = i + len
      if (lb == rb) {
        phase = PH_LCE_SA;
        ad0 = SA + 4ull * (uint32_t)lb;
        use = U0D;
      } else if (pfxExact && len < R.kmerK) {  // (the only way on an unknown interval)
        begin_pfx();
      } else if (hasLd && rb - lb < 16 && len < 0xffffu) {
        phase = PH_EXT1;
        ad0 = (uintptr_t)(R.ld + lb);
        ad2 = T + i + len;
        use = U0Q | U1Q | U4Q | U5Q | U2B;
      } else {
        begin_search();
      }
    }
    if (!kPrefetch || pass == 1 || !__ballot(phase == PC_PFX)) break;
    }

    if (!__ballot(phase != PH_DONE)) break;
    if (STATS) {
      if (phase != PH_DONE) atomicAdd(&sc[phase], 1ull);
      if (phase == PH_ADJ) {
        if ((uint32_t)u4 != kScanDone) atomicAdd(&sc[26 + ((uint32_t)u4 >> 4)], 1ull);
        if (u9 != kScanDone) atomicAdd(&sc[26 + (u9 >> 4)], 1ull);
      }
      if (lane == 0) atomicAdd(&sc[30], 1ull);
    }
    // ---- one memory step
    uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0, v2 = v0, v3 = v0, v4 = v0, v5 = v0;
    if (use & U0B) v0.x = ld1(ad0);
    if (use & U0D) v0.x = ld4(ad0);
    if (use & U0Q) v0 = ldu16(ad0);
    if (use & U1Q) v1 = ldu16(ad0 + 16);
    if (use & U2D) v2.x = ld4(ad2);
    if (use & U2B) v2.x = ld1(ad2);
    if (use & U2Q) v2 = ldu16(ad2);
    if (use & U3Q) v3 = ldu16(ad2 + 16);
    if (use & U4Q) v4 = ldu16(ad0 + 32);
    if (use & U5Q) v5 = ldu16(ad0 + 48);
    if (use & U0E) { const uint2 w = kPairCached && pairOn ? ld8(ad0) : ld8_nt(ad0); v0.x = w.x; v0.y = w.y; }
    if (use & U2E) { const uint2 w = ld8(ad2); v2.x = w.x; v2.y = w.y; }
    if (kPrefetch && (use & U3E)) {
      const uintptr_t a3 = (uintptr_t)(pfxK + (uint32_t)u8);
      const uint2 w = kPairCached && pairOn ? ld8(a3) : ld8_nt(a3);
      v3.x = w.x;
      v3.y = w.y;
    }
    if (kFused && fOpen) {  // the open slots' pieces, compared in this same memory step
      const uint32_t g = lane >> 4, k = lane & 15;
      uint32_t mine = 16, mj = 0, cc = 0, pm = 0, mine2 = 16, cc2 = 0;
      if ((fOpen >> g) & 1) {
        uint4 xv[kCoopJ], tv[kCoopJ];
#pragma unroll
        for (uint32_t j = 0; j < kCoopJ; j++) {
          const uint32_t o = fRun + 16 * (k + 16 * j);
          xv[j] = ldu16(fXa + o);
          tv[j] = CMSBWT_COOP_TEXT_NT ? ldu16_nt(fTa + o) : ldu16(fTa + o);
        }
        first_piece_diff<kCoopJ>(xv, tv, memo, mine, mj, cc, pm, mine2, cc2);
      }
      if (STATS && lane == 0) atomicAdd(&sc[31], 1ull);
      uint64_t mask[kCoopJ], anyM[kCoopJ];
#pragma unroll
      for (uint32_t j = 0; j < kCoopJ; j++) {
        mask[j] = __ballot(mine < 16 && mj == j);
        anyM[j] = memo ? __ballot((pm >> j) & 1) : 0ull;
      }
      uint32_t closed = 0;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        if (!((fOpen >> q) & 1)) continue;
        const uint64_t sm = 0xffffull << (16 * q);
        const uint32_t Lq = (uint32_t)(fLs >> (6 * q)) & 63u;
#pragma unroll
        for (uint32_t j = 0; j < kCoopJ; j++) {
          const uint64_t hit = mask[j] & sm;
          if (hit) {  // first mismatching byte of slot q: piece j, thread f (as in the session below)
            const uint32_t f = (uint32_t)__builtin_ctzll(hit);
            const uint32_t mm = (uint32_t)__shfl((int)mine, (int)f);
            const uint32_t c2 = (uint32_t)__shfl((int)cc, (int)f);
            const uint32_t rq = (uint32_t)__shfl((int)fRun, (int)f);
            uint32_t off2 = rq + 16u * 16u * kCoopJ, c2b = 0;
            if (memo) {
              const uint32_t m2f = (uint32_t)__shfl((int)mine2, (int)f);
              const uint32_t c2f = (uint32_t)__shfl((int)cc2, (int)f);
              if (m2f < 16) {
                off2 = rq + 16 * ((f - 16 * q) + 16 * j) + m2f;
                c2b = c2f | 0x10000u;
              } else {
                uint32_t j2 = j, f2 = 64;
                const uint64_t later = anyM[j] & sm & ~((2ull << f) - 1);
                if (later) {
                  f2 = (uint32_t)__builtin_ctzll(later);
                } else {
#pragma unroll
                  for (uint32_t jj = 0; jj < kCoopJ; jj++)
                    if (jj > j && f2 == 64 && (anyM[jj] & sm)) { j2 = jj; f2 = (uint32_t)__builtin_ctzll(anyM[jj] & sm); }
                }
                if (f2 == f) {
                  off2 = rq + 16 * ((f - 16 * q) + 16 * j2);
                } else if (f2 < 64) {
                  off2 = rq + 16 * ((f2 - 16 * q) + 16 * j2) + (uint32_t)__shfl((int)mine, (int)f2);
                  c2b = (uint32_t)__shfl((int)cc, (int)f2) | 0x10000u;
                }
              }
            }
            if (lane == Lq) {
              if (memo) {
                const uint32_t base = i + len;  // text index of this slot's byte 0
                amAlign = pos - i;
                amLo = base + rq + 16 * ((f - 16 * q) + 16 * j) + mm + 1;
                amFront = base + off2;
                amC = c2b;
                if (kMemoLds) memoL[threadIdx.x] = make_uint4(amAlign, amLo, amFront, amC);
              }
              len += rq + 16 * ((f - 16 * q) + 16 * j) + mm;
              smaller = (int8_t)(uint8_t)c2 > (int8_t)(uint8_t)(c2 >> 8);  // FN:55
              phase = PC_POST;
            }
            closed |= 1u << q;
            fSlotted &= ~(1ull << Lq);
            break;
          }
        }
      }
      fOpen &= ~closed;
      fRun += 16u * 16u * kCoopJ;
    }
    // PLCP skip (FN:1176-1185): the exit inside the 16-entry window below
    // the match end, if it is there (skS = the skip, or ~0u)
    uint32_t skS = 0xffffffffu;
    if (phase == PH_SKIP1) {
      // entries Wb..Wb+15 below TT; PLCP[q] + q is non-decreasing, so the
      // window decides when it starts at or below pos+1 or below the exit.
      // 32-bit arithmetic: positions and PLCP values are below n < 2^31, so
      // no sum wraps (a negative tail entry wraps to a value below TT, as the
      // signed sum would be)
      // Entry k (q = Wb + k < TT) crosses when e[k] + k >= D = TT - Wb; the
      // crossings are a suffix of the window (monotone), so the first one is
      // the number c of entries that do not cross: one add, compare and
      // carry-add per entry.  The exit is the first crossing at or above
      // pos+1 (kmin = q0 - Wb when the window starts below it).
      const uint32_t TT = pos + 1 + len, q0 = pos + 1;
      const uint32_t Wb = TT >= 16 ? TT - 16 : 0, D = TT - Wb;
      // entries as bytes min(PLCP, 255): exact for the test e + k >= D <= 16
      const uint32_t w4[4] = {v0.x, v0.y, v0.z, v0.w};
      uint32_t c = 0;
#pragma unroll
      for (uint32_t k = 0; k < 16; k++) c += ((w4[k >> 2] >> (8 * (k & 3))) & 0xffu) + k < D ? 1u : 0u;
      if (Wb <= q0 || c > 0) {
        const uint32_t kmin = Wb <= q0 ? q0 - Wb : 0u;
        skS = Wb + (c > kmin ? c : kmin) - q0;
      }
    }
    // the text window this step loaded (one call site: the code is emitted once)
    {
      const bool wa = phase == PH_PFX_TEXT || phase == PH_SKTXT;
      const bool sk = phase == PH_SKIP1 && pfxExact && hasPfx;  // the skip loaded 32 text bytes
      const bool ws = sk && skS != 0xffffffffu && len - skS < R.kmerK;
      const bool wr = (use & UREG) != 0;
      if (sk) {
        t32a = v2;
        t32b = v3;
        t32At = skip_text_base();
      }
      if (wa || ws || (phase == PH_PFX_PROBE && pfxExact)) {
        uint4 vv = make_uint4(wa ? v0.x : v2.x, wa ? v0.y : v2.y, wa ? v0.z : v2.z, wa ? v0.w : v2.w);
        uint32_t at = phase == PH_PFX_TEXT ? i : i + 1;
        if (ws || wr) {  // bytes o..o+15 of the 32 skip bytes, o = next position - their base
          if (ws) at = i + skS + 1;
          const uint32_t o = at - t32At;
          uint32_t d[8] = {t32a.x, t32a.y, t32a.z, t32a.w, t32b.x, t32b.y, t32b.z, t32b.w};
          if (o & 16) { d[0] = d[4]; d[1] = d[5]; d[2] = d[6]; d[3] = d[7]; d[4] = d[5] = d[6] = d[7] = 0; }
          if (o & 8) { d[0] = d[2]; d[1] = d[3]; d[2] = d[4]; d[3] = d[5]; d[4] = d[6]; d[5] = d[7]; }
          if (o & 4) { d[0] = d[1]; d[1] = d[2]; d[2] = d[3]; d[3] = d[4]; d[4] = d[5]; }
          const uint32_t sh = o & 3;
          vv = make_uint4(__builtin_amdgcn_alignbyte(d[1], d[0], sh), __builtin_amdgcn_alignbyte(d[2], d[1], sh),
                          __builtin_amdgcn_alignbyte(d[3], d[2], sh), __builtin_amdgcn_alignbyte(d[4], d[3], sh));
        }
        set_window(vv, at);
      }
    }
    // ---- one state-machine step (load phases)
    switch (phase) {
      case PH_BS_TEXT: {  // c = t[j]; the first probe's SA value is in slot 2
        u0 = (int32_t)v0.x;
        ad0 = X + v2.x + len;
        phase = PH_BS_X;
        use = U0B;
        break;
      }
      case PH_BS_SA: {
        ad0 = X + v0.x + len;
        phase = PH_BS_X;
        use = U0B;
        break;
      }
      case PH_BS_X: {
        const uint32_t v = v0.x;
        const uint32_t f = (uint32_t)u0, c = f & 0xff;
        if (!(f & (1u << 17))) {
          if (v < c) u1 = u3 + 1;
          else { u2 = u3; u0 = (int32_t)(c | (v << 8) | (1u << 16)); }
        } else {
          if (v <= c) u1 = u3 + 1;
          else u2 = u3;
        }
        // lower_bound / upper_bound driver: next probe or result
        for (int g = 0; g < 2; g++) {
          if (u1 < u2) {
            u3 = (u1 + u2) >> 1;
            phase = PH_BS_SA;
            ad0 = SA + 4ull * (uint32_t)u3;
            use = U0D;
            break;
          }
          const uint32_t f2 = (uint32_t)u0;
          if (!(f2 & (1u << 17))) {  // lower bound done
            if ((f2 & (1u << 16)) && ((f2 >> 8) & 0xff) == (f2 & 0xff)) {
              u5 = u1;  // new lb; now the right end in [lb'+1, rb+1)
              u0 = (int32_t)(f2 | (1u << 17));
              u1 = u5 + 1;
              u2 = rb + 1;
              continue;
            }
            int32_t mm = u1;  // mismatch: insertion point (FN:65-76)
            smaller = true;
            if (mm == rb + 1) { mm = rb; smaller = false; }
            phase = PH_FAIL_SA;
            ad0 = SA + 4ull * (uint32_t)mm;
            use = U0D;
            break;
          }
          // upper bound done: interval [u5, u1 - 1], one more matched character
          lb = u5;
          rb = u1 - 1;
          len++;
          phase = PC_CHAR;
          use = 0;
          break;
        }
        break;
      }
      case PH_FAIL_SA: {
        pos = v0.x;
        phase = PC_POST;
        break;
      }
      case PH_LCE_SA: {
        pos = v0.x;
        start_lce();
        break;
      }
      case PH_LCE: {
        uint8_t xc = 0, tc = 0;
        const uint32_t m = diff16(v0, v2, xc, tc);
        if (m < 16) {
          len += m;
          smaller = (int8_t)xc > (int8_t)tc;  // FN:55, char compare
          phase = PC_POST;
        } else {  // long extension: hand it to the wave
          len += 16;
          ad0 += 16;
          ad2 += 16;
          phase = PH_LCE_COOP;
        }
        use = 0;
        break;
      }
      case PH_SKIP1: {
        const uint32_t TT = pos + 1 + len, q0 = pos + 1;
        const uint32_t Wb = TT >= 16 ? TT - 16 : 0;
        if (skS != 0xffffffffu) {  // exit inside the window (scanned above)
          if (pfxExact && hasPfx && len - skS < R.kmerK) {  // the window of the next position is decoded
            i += skS;
            len -= skS;
            pos += skS;
            if (wm == R.kmerK) {
              virtual_interval();
              phase = PC_ADV;
              use = 0;
            } else {
              isa1();
            }
          } else {
            skip_done(skS);
          }
        } else {  // exit at or below Wb: PLCP[pos+1] first, then gallop
          phase = PH_SKIP0;
          ad0 = P + 4ull * (pos + 1);
          use = U0D;
          u2 = (int32_t)(Wb - q0);  // the predicate holds at s = Wb - (pos+1)
        }
        break;
      }
      case PH_SKIP0: {
        if ((int64_t)len <= (int64_t)(int32_t)v0.x) { skip_done(0); break; }
        u1 = 0;
        u4 = 1;
        skip_probe(true);
        break;
      }
      case PH_GALLOP: {
        const int64_t v = (int32_t)v0.x;
        if ((int64_t)len - (int64_t)(uint32_t)u3 <= v) {
          u2 = u3;
          skip_probe(false);
        } else {
          u1 = u3;
          u4 <<= 1;
          skip_probe(true);
        }
        break;
      }
      case PH_SKIPBS: {
        const int64_t v = (int32_t)v0.x;
        if ((int64_t)len - (int64_t)(uint32_t)u3 <= v) u2 = u3; else u1 = u3;
        skip_probe(false);
        break;
      }
      case PH_ISA1: {
        if (hasIr) adj_records(v0.x, v0.x, v0, v0);
        else { u0 = u5 = (int32_t)v0.x; phase = PC_ADJ0; use = 0; }
        break;
      }
      case PH_CONP: {
        if (v0.x == 0xffffffffu || v2.x == 0xffffffffu) {  // SA[lb] or SA[rb] = n-1: root (FN:37-39)
          lb = 0;
          rb = (int32_t)n - 1;
          phase = PC_ADV;
          use = 0;
        } else {
          adj_records(v0.x, v2.x, v0, v2);
        }
        break;
      }
      case PH_ADJ: {
        uint32_t ls0 = (uint32_t)u4;
        if (ls0 != kScanDone) scan_step<false>(V, v0, v1, (int32_t)len, u0, u1, u2, u3, ls0);
        u4 = (int32_t)ls0;
        if (u9 != kScanDone) scan_step<true>(V, v2, v3, (int32_t)len, u5, u6, u7, u8, u9);
        adj_or_finish();
        break;
      }
      case PH_EXT_A: {
        u0 = (int32_t)v2.x;  // the text character
        phase = PH_EXT_B;
        ad0 = (uintptr_t)(R.ld + lb);
        ad2 = X + v0.x + len;
        use = U0Q | U1Q | U4Q | U5Q | U2B;
        break;
      }
      case PH_EXT1:
      case PH_EXT_B: {
        // children of [lb, rb] at depth off = len, in character order: they
        // start at lb and at each k in (lb, rb] with LCP[k] == off; child j > 0
        // has character D[k], the first x[SA[lb]+off] (EXT_B: loaded) =
        // U[(start of the second child) - 1] (EXT1)
        const bool one = phase == PH_EXT1;
        const uint32_t c = one ? (v2.x & 0xff) : (uint32_t)u0;
        const uint32_t e[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                                v4.x, v4.y, v4.z, v4.w, v5.x, v5.y, v5.z, v5.w};
        const int32_t S1 = rb - lb;
        bool valid = true;
        int32_t lo = -1, hi = -1, mm = rb + 1, k1 = 0;
        uint32_t curChar = one ? 0x100u : (v2.x & 0xff);
        int32_t curStart = lb;
#pragma unroll
        for (int k = 1; k < 16; k++) {
          if (k <= S1) {
            const uint32_t l = e[k] >> 16;
            if (l < len) valid = false;
            if (l == len) {
              if (!k1) {
                k1 = k;
                if (one) curChar = e[k - 1] & 0xff;
              }
              if (curChar == c) { lo = curStart; hi = lb + k - 1; }
              if (curChar > c && mm == rb + 1) mm = curStart;
              curChar = (e[k] >> 8) & 0xff;
              curStart = lb + k;
            }
          }
        }
        if (curChar == c) { lo = curStart; hi = rb; }
        if (curChar > c && curChar < 0x100u && mm == rb + 1) mm = curStart;
        if (!valid) {  // not an lcp-interval of depth off (root after contraction)
          begin_bs();
        } else if (one && !k1) {  // a single child: its character needs SA[lb]
          phase = PH_EXT_A;
          ad0 = SA + 4ull * (uint32_t)lb;
          ad2 = T + i + len;
          use = U0D | U2B;
        } else if (lo >= 0) {  // FN:79-84: one more matched character
          lb = lo;
          rb = hi;
          len++;
          phase = PC_CHAR;
          use = 0;
        } else {  // FN:65-76: insertion point of c
          smaller = true;
          if (mm == rb + 1) { mm = rb; smaller = false; }
          phase = PH_FAIL_SA;
          ad0 = SA + 4ull * (uint32_t)mm;
          use = U0D;
        }
        break;
      }
      case PH_PFX_TEXT: {  // window at i (set above), then the probe
        pfx_probe();
        break;
      }
      case PH_PFX_PROBE: {  // (wm/wcode already describe the window at i + 1)
        if (kPrefetch && (use & U3E)) {  // the entry of i + 1 rode along
          pfE = make_uint2(v3.x, v3.y);
          pfAt = i + 1;
        }
        if (!pfxExact && len > 0 && (v2.x != (uint32_t)lb || v2.y != (uint32_t)(rb - lb) + 1)) {
          begin_bs();
          break;
        }
        pfx_entry(v0.x, v0.y);
        break;
      }
      case PH_IVL: {
        lb = (int32_t)v0.x;
        rb = (int32_t)(v0.x + v0.y) - 1;
        phase = PC_POST;
        break;
      }
      case PH_SKTXT: {  // after a skip: K symbols at i + 1 (window set above) make the interval unnecessary
        if (wm == R.kmerK) {
          virtual_interval();
          phase = PC_ADV;
          use = 0;
        } else {
          isa1();
        }
        break;
      }
      default:
        break;
    }
    // ---- long extensions, compared by the whole wave with coalesced loads.
    // The pending lanes are served S = 1, 2 or 4 at a time (as many as are
    // pending), each by a slot of W = 64 / S threads; a thread compares
    // kCoopJ 16-byte pieces per round, piece j of thread k at byte
    // 16 (k + W j), so a slot covers 16 W kCoopJ contiguous bytes per round
    // (4 KiB for a single lane).  A slot ends at its first mismatch.
    // Pending lanes wait (idle, no load) until kCoopMin of them can share the
    // wave's round trips, unless no other lane of the wave is still walking.
    if (kFused) {  // pending lanes take the free slots; their pieces load in the next memory step
      uint64_t pend = __ballot(phase == PH_LCE_COOP) & ~fSlotted;
      uint32_t fresh = 0;
      while (pend && fOpen != 15u) {
        const uint32_t q = (uint32_t)__builtin_ctz(~fOpen & 15u);
        const uint32_t L = (uint32_t)__builtin_ctzll(pend);
        pend &= pend - 1;
        fLs = (fLs & ~(63ull << (6 * q))) | ((uint64_t)L << (6 * q));
        fSlotted |= 1ull << L;
        fOpen |= 1u << q;
        fresh |= 1u << q;
      }
      if (fresh) {
        const uint32_t g = lane >> 4;
        const uint32_t myL = (uint32_t)(fLs >> (6 * g)) & 63u;
        const uintptr_t nx = ((uintptr_t)__shfl((uint32_t)(ad0 >> 32), (int)myL) << 32) | __shfl((uint32_t)ad0, (int)myL);
        const uintptr_t nt = ((uintptr_t)__shfl((uint32_t)(ad2 >> 32), (int)myL) << 32) | __shfl((uint32_t)ad2, (int)myL);
        if ((fresh >> g) & 1) { fXa = nx; fTa = nt; fRun = 0; }
      }
      continue;
    }
    uint64_t coop = __ballot(phase == PH_LCE_COOP);
    const bool drain = coop == __ballot(phase != PH_DONE);
    if (kCoopRefill && (uint32_t)__popcll(coop) >= kSlots && (drain || (uint32_t)__popcll(coop) >= kCoopMin)) {
      // kSlots slots of kSlotW threads, each with its own offset: a slot whose
      // extension ends takes the next pending lane in the same round trip, so
      // the wave's rounds follow the total length of the extensions instead
      // of the longest of each group of four (r04).
      // the slots' lanes, 6 bits each (wave-uniform; packed so that a slot
      // index that is not a constant does not put an array in scratch)
      uint64_t LsP0 = 0, LsP1 = 0;
      auto ls_get = [&](uint32_t q) -> uint32_t {
        return (uint32_t)(((q < 8 ? LsP0 : LsP1) >> (6 * (q & 7))) & 63u);
      };
      auto ls_set = [&](uint32_t q, uint32_t v) {
        const uint32_t sh = 6 * (q & 7);
        if (q < 8) LsP0 = (LsP0 & ~(63ull << sh)) | ((uint64_t)v << sh);
        else LsP1 = (LsP1 & ~(63ull << sh)) | ((uint64_t)v << sh);
      };
#pragma unroll
      for (uint32_t q = 0; q < kSlots; q++) {
        ls_set(q, (uint32_t)__builtin_ctzll(coop));
        coop &= coop - 1;
      }
      const uint32_t g = lane / kSlotW, k = lane % kSlotW;
      auto slot_lane = [&]() { return ls_get(g); };
      uint32_t myL = slot_lane();
      uintptr_t xa = ((uintptr_t)__shfl((uint32_t)(ad0 >> 32), (int)myL) << 32) | __shfl((uint32_t)ad0, (int)myL);
      uintptr_t ta = ((uintptr_t)__shfl((uint32_t)(ad2 >> 32), (int)myL) << 32) | __shfl((uint32_t)ad2, (int)myL);
      uint32_t runT = 0, open = (1u << kSlots) - 1u;
      while (open) {
        uint32_t mine = 16, mj = 0, cc = 0;
        uint32_t pm = 0, mine2 = 16, cc2 = 0;  // (memo) pieces with a mismatch; 2nd mismatch of piece mj
        if ((open >> g) & 1) {
          uint4 xv[kCoopJ], tv[kCoopJ];
#pragma unroll
          for (uint32_t j = 0; j < kCoopJ; j++) {
            const uint32_t o = runT + 16 * (k + j * kSlotW);
            xv[j] = ldu16(xa + o);
            tv[j] = CMSBWT_COOP_TEXT_NT ? ldu16_nt(ta + o) : ldu16(ta + o);
          }
          if (kPieceXor) {
            first_piece_diff<kCoopJ>(xv, tv, memo, mine, mj, cc, pm, mine2, cc2);
          } else {
#pragma unroll
          for (int j = (int)kCoopJ - 1; j >= 0; j--) {
            if (memo) {
              uint32_t m1, c1, m2, c2;
              diff16x2(xv[j], tv[j], m1, c1, m2, c2);
              if (m1 < 16) { mine = m1; mj = (uint32_t)j; cc = c1; mine2 = m2; cc2 = c2; pm |= 1u << j; }
            } else {
              uint8_t xc = 0, tc = 0;
              const uint32_t m = diff16(xv[j], tv[j], xc, tc);
              if (m < 16) { mine = m; mj = (uint32_t)j; cc = (uint32_t)xc | ((uint32_t)tc << 8); }
            }
          }
          }
        }
        if (STATS && lane == 0) atomicAdd(&sc[31], 1ull);
        uint64_t mask[kCoopJ], anyM[kCoopJ];
#pragma unroll
        for (uint32_t j = 0; j < kCoopJ; j++) {
          mask[j] = __ballot(mine < 16 && mj == j);
          anyM[j] = memo ? __ballot((pm >> j) & 1) : 0ull;
        }
        uint32_t fresh = 0;  // slots given a new lane this round
#pragma unroll
        for (uint32_t q = 0; q < kSlots; q++) {
          if (!((open >> q) & 1)) continue;
          const uint64_t sm = (~0ull >> (64 - kSlotW)) << (q * kSlotW);
#pragma unroll
          for (uint32_t j = 0; j < kCoopJ; j++) {
            const uint64_t hit = mask[j] & sm;
            if (hit) {  // first mismatching byte of slot q: piece j, thread f
              const uint32_t f = (uint32_t)__builtin_ctzll(hit);
              const uint32_t mm = (uint32_t)__shfl((int)mine, (int)f);
              const uint32_t c2 = (uint32_t)__shfl((int)cc, (int)f);
              const uint32_t rq = (uint32_t)__shfl((int)runT, (int)f);
              // memo: the next mismatch after (piece j, thread f) in byte
              // order (the same piece of f, a later thread's piece j, then
              // a later piece), else the round's end, clean
              uint32_t off2 = rq + 16u * kSlotW * kCoopJ, c2b = 0;
              if (memo) {
                const uint32_t m2f = (uint32_t)__shfl((int)mine2, (int)f);
                const uint32_t c2f = (uint32_t)__shfl((int)cc2, (int)f);
                if (m2f < 16) {
                  off2 = rq + 16 * ((f - q * kSlotW) + j * kSlotW) + m2f;
                  c2b = c2f | 0x10000u;
                } else {
                  uint32_t j2 = j, f2 = 64;
                  const uint64_t later = anyM[j] & sm & ~((2ull << f) - 1);
                  if (later) {
                    f2 = (uint32_t)__builtin_ctzll(later);
                  } else {
#pragma unroll
                    for (uint32_t jj = 0; jj < kCoopJ; jj++)
                      if (jj > j && f2 == 64 && (anyM[jj] & sm)) { j2 = jj; f2 = (uint32_t)__builtin_ctzll(anyM[jj] & sm); }
                  }
                  if (f2 == f) {  // f's own later piece: its first mismatch there is not kept; clean up to it
                    off2 = rq + 16 * ((f - q * kSlotW) + j2 * kSlotW);
                  } else if (f2 < 64) {  // (f2 != f: its first mismatch is in piece j2, an earlier one would precede (j, f))
                    off2 = rq + 16 * ((f2 - q * kSlotW) + j2 * kSlotW) + (uint32_t)__shfl((int)mine, (int)f2);
                    c2b = (uint32_t)__shfl((int)cc, (int)f2) | 0x10000u;
                  }
                }
              }
              if (lane == ls_get(q)) {
                if (memo) {
                  const uint32_t base = i + len;  // text index of this slot's byte 0
                  amAlign = pos - i;
                  amLo = base + rq + 16 * ((f - q * kSlotW) + j * kSlotW) + mm + 1;
                  amFront = base + off2;
                  amC = c2b;
                  if (kMemoLds) memoL[threadIdx.x] = make_uint4(amAlign, amLo, amFront, amC);
                }
                len += rq + 16 * ((f - q * kSlotW) + j * kSlotW) + mm;
                smaller = (int8_t)(uint8_t)c2 > (int8_t)(uint8_t)(c2 >> 8);  // FN:55
                phase = PC_POST;
              }
              if (coop) {
                ls_set(q, (uint32_t)__builtin_ctzll(coop));
                coop &= coop - 1;
                fresh |= 1u << q;
              } else {
                open &= ~(1u << q);
              }
              break;
            }
          }
        }
        runT = ((fresh >> g) & 1) ? 0u : runT + 16u * kSlotW * kCoopJ;
        if (fresh) {
          myL = slot_lane();
          const uintptr_t nx = ((uintptr_t)__shfl((uint32_t)(ad0 >> 32), (int)myL) << 32) |
                               __shfl((uint32_t)ad0, (int)myL);
          const uintptr_t nt = ((uintptr_t)__shfl((uint32_t)(ad2 >> 32), (int)myL) << 32) |
                               __shfl((uint32_t)ad2, (int)myL);
          if ((fresh >> g) & 1) { xa = nx; ta = nt; }
        }
      }
    }
    while (coop && (drain || (uint32_t)__popcll(coop) >= kCoopMin)) {
      const uint32_t P = (uint32_t)__popcll(coop);
      const uint32_t S = P >= 4 ? 4u : P >= 2 ? 2u : 1u;
      const uint32_t lgW = S == 4 ? 4u : S == 2 ? 5u : 6u;
      const uint32_t W = 1u << lgW;
      uint32_t Ls[4] = {0, 0, 0, 0};
#pragma unroll
      for (uint32_t q = 0; q < 4; q++)
        if (q < S) {
          Ls[q] = (uint32_t)__builtin_ctzll(coop);
          coop &= coop - 1;
        }
      const uint32_t g = lane >> lgW, k = lane & (W - 1);
      const uint32_t myL = g == 0 ? Ls[0] : g == 1 ? Ls[1] : g == 2 ? Ls[2] : Ls[3];
      const uintptr_t xa = ((uintptr_t)__shfl((uint32_t)(ad0 >> 32), (int)myL) << 32) | __shfl((uint32_t)ad0, (int)myL);
      const uintptr_t ta = ((uintptr_t)__shfl((uint32_t)(ad2 >> 32), (int)myL) << 32) | __shfl((uint32_t)ad2, (int)myL);
      // pieces per thread: the first round reads 1 KiB per slot, later
      // rounds double up to kCoopJ pieces (a lane's remaining match is
      // usually shorter than 1 KiB: no over-read on the common case)
      uint32_t run = 0, open = (1u << S) - 1;  // open: slots still comparing
      uint32_t jr = S < kCoopJ ? S : kCoopJ;
      while (open) {
        uint32_t mine = 16, mj = 0, cc = 0;  // this thread's first mismatch: piece, offset, chars
        uint32_t pm = 0, mine2 = 16, cc2 = 0;  // (memo) pieces with a mismatch; 2nd mismatch of piece mj
        // one round of JR pieces (fixed-size arrays: no register spills)
        auto cmp_round = [&](auto jrc) {
          constexpr uint32_t JR = decltype(jrc)::value;
          uint4 xv[JR], tv[JR];
#pragma unroll
          for (uint32_t j = 0; j < JR; j++) {
            const uint32_t o = run + 16 * (k + (j << lgW));
            xv[j] = ldu16(xa + o);
            tv[j] = CMSBWT_COOP_TEXT_NT ? ldu16_nt(ta + o) : ldu16(ta + o);
          }
          if (kPieceXor) {
            first_piece_diff<JR>(xv, tv, memo, mine, mj, cc, pm, mine2, cc2);
            return;
          }
#pragma unroll
          for (int j = (int)JR - 1; j >= 0; j--) {
            if (memo) {
              uint32_t m1, c1, m2, c2;
              diff16x2(xv[j], tv[j], m1, c1, m2, c2);
              if (m1 < 16) { mine = m1; mj = (uint32_t)j; cc = c1; mine2 = m2; cc2 = c2; pm |= 1u << j; }
            } else {
              uint8_t xc = 0, tc = 0;
              const uint32_t m = diff16(xv[j], tv[j], xc, tc);
              if (m < 16) { mine = m; mj = (uint32_t)j; cc = (uint32_t)xc | ((uint32_t)tc << 8); }
            }
          }
        };
        if ((open >> g) & 1) {
          if (jr == 4) cmp_round(std::integral_constant<uint32_t, 4u>{});
          else if (jr == 2) cmp_round(std::integral_constant<uint32_t, 2u>{});
          else cmp_round(std::integral_constant<uint32_t, 1u>{});
        }
        if (STATS && lane == 0) atomicAdd(&sc[31], 1ull);
        // per piece index j: threads whose first mismatch lies in piece j
        uint64_t mask[kCoopJ], anyM[kCoopJ];
#pragma unroll
        for (uint32_t j = 0; j < kCoopJ; j++) {
          mask[j] = __ballot(mine < 16 && mj == j);
          anyM[j] = memo ? __ballot((pm >> j) & 1) : 0ull;
        }
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
          if (q >= S || !((open >> q) & 1)) continue;
          const uint64_t sm = (W == 64 ? ~0ull : ((1ull << W) - 1)) << (q << lgW);
#pragma unroll
          for (uint32_t j = 0; j < kCoopJ; j++) {
            const uint64_t hit = mask[j] & sm;
            if (hit) {  // first mismatching byte of slot q: piece j, thread f
              const uint32_t f = (uint32_t)__builtin_ctzll(hit);
              const uint32_t mm = (uint32_t)__shfl((int)mine, (int)f);
              const uint32_t c2 = (uint32_t)__shfl((int)cc, (int)f);
              // memo (as in the refill loop): the next mismatch in byte order,
              // else the round's end
              uint32_t off2 = run + 16u * W * jr, c2b = 0;
              if (memo) {
                const uint32_t m2f = (uint32_t)__shfl((int)mine2, (int)f);
                const uint32_t c2f = (uint32_t)__shfl((int)cc2, (int)f);
                if (m2f < 16) {
                  off2 = run + 16 * ((f - (q << lgW)) + (j << lgW)) + m2f;
                  c2b = c2f | 0x10000u;
                } else {
                  uint32_t j2 = j, f2 = 64;
                  const uint64_t later = anyM[j] & sm & ~((2ull << f) - 1);
                  if (later) {
                    f2 = (uint32_t)__builtin_ctzll(later);
                  } else {
#pragma unroll
                    for (uint32_t jj = 0; jj < kCoopJ; jj++)
                      if (jj > j && f2 == 64 && (anyM[jj] & sm)) { j2 = jj; f2 = (uint32_t)__builtin_ctzll(anyM[jj] & sm); }
                  }
                  if (f2 == f) {
                    off2 = run + 16 * ((f - (q << lgW)) + (j2 << lgW));
                  } else if (f2 < 64) {
                    off2 = run + 16 * ((f2 - (q << lgW)) + (j2 << lgW)) + (uint32_t)__shfl((int)mine, (int)f2);
                    c2b = (uint32_t)__shfl((int)cc, (int)f2) | 0x10000u;
                  }
                }
              }
              if (lane == Ls[q]) {
                if (memo) {
                  const uint32_t base = i + len;
                  amAlign = pos - i;
                  amLo = base + run + 16 * ((f - (q << lgW)) + (j << lgW)) + mm + 1;
                  amFront = base + off2;
                  amC = c2b;
                  if (kMemoLds) memoL[threadIdx.x] = make_uint4(amAlign, amLo, amFront, amC);
                }
                len += run + 16 * ((f - (q << lgW)) + (j << lgW)) + mm;
                smaller = (int8_t)(uint8_t)c2 > (int8_t)(uint8_t)(c2 >> 8);  // FN:55
                phase = PC_POST;
              }
              open &= ~(1u << q);
              break;
            }
          }
        }
        run += 16u * W * jr;
        jr = 2 * jr < kCoopJ ? 2 * jr : kCoopJ;
      }
    }
  }
  if (STATS) {
    __syncthreads();
    if (threadIdx.x < 32) atomicAdd(&A.stats[threadIdx.x], sc[threadIdx.x]);
  }
}

void launch_ms_walk2(const DevRef& R, const uint8_t* text, const uint64_t* docOff, const Chunk* chunks,
                     uint32_t nchunks, const uint32_t* order, const uint32_t* bandStart, uint32_t nbands,
                     uint32_t* nextChunk, const Pool& pool, uint32_t* chunkCount, uint32_t lanes,
                     unsigned long long* stats, hipStream_t st) {
  if (!nchunks) return;
  Walk2Args A{R, text, docOff, chunks, nchunks, order, bandStart, nbands, nextChunk, pool, chunkCount, stats};
  const uint32_t blocks = (std::min<uint32_t>(lanes, nchunks) + 255) / 256;
  const bool fast = R.pfx && R.pfxDna && R.pfxExact && R.ld && R.ir;
  if (stats) {
    if (fast) hipLaunchKernelGGL((k_ms_walk2<true, true>), dim3(blocks), dim3(256), 0, st, A);
    else hipLaunchKernelGGL((k_ms_walk2<true, false>), dim3(blocks), dim3(256), 0, st, A);
  } else {
    if (fast) hipLaunchKernelGGL((k_ms_walk2<false, true>), dim3(blocks), dim3(256), 0, st, A);
    else hipLaunchKernelGGL((k_ms_walk2<false, false>), dim3(blocks), dim3(256), 0, st, A);
  }
}

}  // namespace cmsbwt
