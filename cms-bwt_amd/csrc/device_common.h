// device_common.h — shared device-side definitions for the CMS-BWT engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmsbwt {

constexpr int kMaxLevels = 6;   // block-minima levels over LCP (64^6 > 2^32)
// head records per pool block: 32 (round 6) = a whole 128-byte line of every
// u32 array the head scatter writes per block, and half the block
// transitions of the walk (A/B one box, walk kernel 10.78-10.90 ->
// 10.51-10.54 ms with 16 -> 32; 64 was no better and costs more step time)
#ifndef CMSBWT_POOL_B
#define CMSBWT_POOL_B 32
#endif
constexpr uint32_t kPoolB = CMSBWT_POOL_B;
// the walk records each head's BWT character (the text byte before it) in
// its record when the lane's sliding window just held it (HeadRec.flags bits
// 8..15, bit 16 = known); k_finalize then reads the text only for the others
// (CMSBWT_WALK_LCHAR, one setting for every translation unit).  Measured
// (round 6, A/B one box, bit-exact, 356 parity tests green): walk stage
// 12.32-12.47 -> 12.64-12.70 ms, the walk's LDS writes cost more than the
// text lines k_finalize no longer streams; off
#ifndef CMSBWT_WALK_LCHAR
#define CMSBWT_WALK_LCHAR 0
#endif
constexpr bool kWalkLchar = CMSBWT_WALK_LCHAR != 0;
// pool blocks a lane of the uniform-step walk reserves per atomic (it keeps
// unused ones for its next chunk; blocks never started keep blkMeta.x = ~0)
constexpr uint32_t kPoolBatch = 16;
constexpr uint8_t kSep = 2;     // CMS-BWT.h:28
// Readable tail after x and after the collection text: the cooperative LCE
// of the walk reads up to 4 KiB past its current position.
constexpr uint64_t kTextPad = 8192;

// Reference index staged in HBM; int32/uint32 arrays,
// x as bytes with 64 bytes of padding so the LCE loop can read 16 B past n.
struct DevRef {
  const uint8_t* x;
  const int32_t* sa;
  const uint32_t* isa;
  const int32_t* lcp;     // n+1 entries
  const int32_t* plcp;    // max-neighbour PLCP (FN:272-274)
  // min(PLCP, 255) as bytes (n + 32): the PLCP skip's first window (16 entries
  // below the match end) only asks PLCP[q] >= T - q <= 16, so one 16-B load
  // decides it, from a 1/4-size array that stays in the XCDs' L2
  const uint8_t* plcp8;
  const uint8_t* bwt;
  const int32_t* lvl[kMaxLevels];  // lvl[0][b] = min lcp[64b..64b+63], lvl[k] = min of 64 lvl[k-1]
  uint32_t lvlLen[kMaxLevels];
  uint32_t lvlOff[kMaxLevels];     // lvl[k] == lcp + lvlOff[k] (one buffer, 16-B aligned levels)
  int nlvl;
  uint32_t n;
  // Prefix-rank tables (walk only): over the reference's own alphabet (kmap:
  // byte -> symbol, 0xff = absent; B bits per symbol), for every length
  // l = 1..kmerK and every l-symbol string P (code c = sum P[d] << B(l-1-d)),
  // pfx[pfxOff[l] + 2c] = the number of suffixes of x smaller than P in their
  // first l bytes (where P's SA interval starts, or P's insertion point when
  // it does not occur) and pfx[pfxOff[l] + 2c + 1] = the number of suffixes
  // starting with P.  pfx == nullptr disables them.
  // A P that does not occur holds instead the walk's answer for any text
  // starting with P (an "answer entry", word 1 has kPfxAns): the longest
  // occurring prefix length l (< |P|) in the low byte, pos = SA[mm] in word 0
  // with mm the insertion point of P[0..l] inside the interval of P[0..l)
  // (FN:65-76: the interval's last index and smaller = false when P[0..l]
  // sorts after all of it), kPfxSmaller = smaller, kPfxSingle = that
  // interval holds one suffix.  Occurring entries keep (Start, Count).
  const uint32_t* pfx;
  // Paired level-K table (DNA only, B = 2; nullptr: absent): line Z, one per
  // (K-1)-symbol string, holds 8 entries of pfx's level K -- slot j < 4 the
  // K-mer j.Z (Z its suffix), slot 4 + j the K-mer Z.j (Z its prefix).  The
  // K-mers of text positions i and i + 1 share their middle K - 1 symbols, so
  // the walk's probe of i (slot t[i]) and the prefetched probe of i + 1 (slot
  // 4 + t[i+K]) read one 64-byte line instead of two random lines.
  const uint32_t* pfk;
  uint32_t pfxOff[17];
  const uint8_t* kmap;  // 256 entries
  uint32_t kmerK, kmerB;
  // 1 when no carried SA interval can be inexact: the reference holds no byte
  // 0 or 1, so no text prefix can reach rank 0 and contractLeft never returns
  // the root with len > 0 (FN:37-39).  The walk then trusts answer entries
  // without re-reading the carried prefix's interval, and may drop a
  // contraction whose result the next position's table probe supersedes.
  uint32_t pfxExact;
  uint32_t pfxDna;  // the symbols are exactly A, C, G, T (codes 0..3)
  // Child table (walk only): ld[k] = min(LCP[k], 2^16-1) << 16 | D[k] << 8 | U[k]
  // with D[k] = x[SA[k]+LCP[k]] (where suffix k leaves suffix k-1) and
  // U[k] = x[SA[k]+LCP[k+1]] (where it leaves suffix k+1); nullptr disables
  // the small-interval extension.
  const uint32_t* ld;
  // Adjacency records (walk only), 4 words each: r, then LCP[r], LCP[r-1] ..
  // LCP[r-5] and LCP[r+1] .. LCP[r+6] as bytes clipped to 255.  pr[k] is the
  // record of r = psi(k) = ISA[SA[k]+1] (r = 0xffffffff when SA[k] = n-1),
  // ir[q] the record of r = ISA[q].  nullptr disables them.
  const uint4* pr;
  const uint4* ir;
};

constexpr uint32_t kPfxAns = 0x80000000u;
constexpr uint32_t kPfxSingle = 0x40000000u;
constexpr uint32_t kPfxSmaller = 0x20000000u;
// an occurring P with one suffix holds (SA of it, kPfxOne | 1) instead of
// (Start, 1): the walk's singleton extension starts at the reference position
constexpr uint32_t kPfxOne = 0x40000000u;

// One restart chunk of the MS walk: positions [a, b) of document `doc`.
struct Chunk {
  uint32_t doc;
  uint32_t a;
  uint32_t b;
  uint32_t last;  // 1 if this is the last chunk of its document
};

// 16-byte head record as written by the MS walk (MatchInVectorBigger, match.h:5-16,
// minus toNext/idx which are assigned later).
struct HeadRec {
  uint32_t start;   // doc-local position
  uint32_t pos;     // reference position of the match
  uint32_t len;     // match length
  uint32_t flags;   // bit 0 smaller (the head's BWT character is read by k_finalize)
};

struct Pool {
  HeadRec* rec;
  uint2* blkMeta;      // (chunk, block sequence in the chunk) per block; chunk ~0: reserved, never started
  uint32_t* used;      // atomic block counter
  uint32_t capBlocks;
};

}  // namespace cmsbwt
