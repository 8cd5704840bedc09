// kernels.h — host-side launchers of the engine's HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "device_common.h"

namespace cmsbwt {

// Heads in document (idx) order, SoA.
struct HeadsSoA {
  uint32_t* start;
  uint32_t* pos;
  uint32_t* len;
  uint8_t* smaller;
  uint8_t* lchar;
  uint32_t* isa;       // isaNext after k_finalize
  uint32_t* tonext;
  uint16_t* nexthead;
};

// A head's grouping fields carried through the position radix sort (16 B).
struct HeadKV {
  uint32_t idx, len, isa, tonext;  // len: bit 31 = smaller
};

// Items (distinct (pos, len, isaNext) keys) in map order: pos ascending, then
// the MatchInSet order of match.h:27-33 — the order of the reference's slots.
struct ItemsSoA {
  uint32_t* pos;
  uint32_t* len;
  uint32_t* isa;
  uint8_t* smaller;
  uint32_t* until;     // untilNext of the first-inserted head
  uint32_t* count;     // heads in the item
  uint32_t* first;     // offset of its members in `perm`
  uint32_t* slot;      // exclusive prefix of count (prefixSumForPositions)
  uint32_t* fbegin;    // unused
  unsigned long long* sk;  // per item search key: smaller ? len<<32|isa : ~len<<32|isa
};

// ms_walk.hip
void launch_chunk_with_end(const Chunk* chunks, const uint32_t* chunkCount, uint32_t nch, unsigned long long* out,
                           hipStream_t st);
void launch_scatter_heads(const Pool& pool, uint32_t blocksUsed, const uint32_t* chunkCount,
                          const unsigned long long* chunkBase, const HeadsSoA& h, const Chunk* chunks,
                          const uint8_t* text, const uint64_t* docOff, uint32_t* hdoc, hipStream_t st);
// ms_walk2.hip: uniform-step walk; `lanes` resident lanes pull chunks from
// per-band queues: order[bandStart[k] ..) are band k's chunk ids, nextChunk[16k]
// its (zeroed) counter
void launch_ms_walk2(const DevRef& R, const uint8_t* text, const uint64_t* docOff, const Chunk* chunks,
                     uint32_t nchunks, const uint32_t* order, const uint32_t* bandStart, uint32_t nbands,
                     uint32_t* nextChunk, const Pool& pool, uint32_t* chunkCount, uint32_t lanes,
                     unsigned long long* stats, hipStream_t st);
void launch_end_phrases(const uint8_t* text, const uint64_t* docOff, uint32_t ndocs,
                        const uint32_t* docLastChunk, const uint32_t* chunkCount,
                        const unsigned long long* chunkBase, uint32_t n, const HeadsSoA& h, uint32_t* docEndIdx,
                        uint32_t* hdoc, hipStream_t st);
// ISA[p] | x[p] << 24 (references shorter than 2^24): k_finalize's isaNext
// and order-check reads in one random line
void launch_isax(const uint32_t* isa, const uint8_t* x, uint32_t n, uint32_t* out, hipStream_t st);
void launch_finalize(const DevRef& R, const HeadsSoA& h, uint32_t H, const uint32_t* docEndIdx,
                     uint32_t ndocs, const uint8_t* text, const uint64_t* docOff, uint32_t* errFlags,
                     const uint32_t* hdoc, hipStream_t st,
                     const uint32_t* isax = nullptr);
// run buckets: diff[0..n] and hasHead[0..n) from the heads' runs, through
// nb = (n >> sh) + 1 bins of 2^sh positions, sh <= kRunBinShift (count into
// zeroed binCnt[nb+1]; scatter with binCur = exclusive prefix of the counts;
// emit with binOff = that prefix).  Bin counters live in LDS up to
// kRunBinLdsMax bins, in global memory beyond (or when `global`).
constexpr uint32_t kRunBinShift = 13;
constexpr uint32_t kRunBinLdsMax = 16384;
void launch_run_bin_count(const HeadsSoA& h, uint32_t H, uint32_t n, uint32_t nb, uint32_t sh, bool global,
                          uint32_t* binCnt, hipStream_t st);
void launch_run_bin_scatter(const HeadsSoA& h, uint32_t H, uint32_t n, uint32_t nb, uint32_t sh, bool global,
                            uint32_t* binCur, uint32_t* vals, hipStream_t st);
void launch_run_bin_emit(const uint32_t* vals, const uint32_t* binOff, uint32_t n, uint32_t nb, uint32_t sh,
                         int32_t* diff, uint8_t* hasHead, hipStream_t st);

// coll_read.hip: the collection reader on the device (getline semantics of
// FN:1138-1275 without -p) over raw file bytes in HBM, tiles of kRdTile bytes.
constexpr uint32_t kRdTile = 16384;
void launch_rd_lastnl(const uint8_t* raw, uint64_t len, uint64_t ntiles, uint64_t* lastNl1, hipStream_t st);
void launch_rd_count(const uint8_t* raw, uint64_t len, uint64_t ntiles, const uint64_t* carry, uint32_t* cnt,
                     uint32_t* seps, hipStream_t st);
void launch_rd_emit(const uint8_t* raw, uint64_t len, uint64_t ntiles, const uint64_t* carry,
                    const uint64_t* outBase, const uint64_t* sepBase, const uint8_t* present, uint8_t* out,
                    uint64_t* docOff, unsigned long long* badByte, hipStream_t st);

// coll_read.hip: plain .bwt expansion of the packed runs, bytes [o0, o0+len)
// of the output into out (16-B aligned); start = exclusive scan of lengths
void launch_out_split(const uint8_t* rec, uint64_t R, unsigned long long* len, uint8_t* chr, hipStream_t st);
void launch_out_expand(const unsigned long long* start, const uint8_t* chr, uint64_t R, uint64_t o0, uint64_t len,
                       uint8_t* out, hipStream_t st);

// ref_index.hip: reference index on the device (prefix-doubling SA, Φ-PLCP)
constexpr uint32_t kIdxH0 = 7;      // initial key: 7 symbols of 9 bits
constexpr uint32_t kIdxChunk = 64;  // positions per thread in the Φ-PLCP pass
void launch_ix_init(const uint8_t* x, uint32_t n, unsigned long long* key, uint32_t* idx, hipStream_t st);
void launch_ix_heads(const unsigned long long* key, const uint32_t* slot, uint32_t m, uint32_t* headIn, uint32_t* tie,
                     hipStream_t st);
void launch_ix_place(const uint32_t* val, const uint32_t* slot, const uint32_t* head, uint32_t m, int32_t* sa,
                     uint32_t* rank, hipStream_t st);
void launch_ix_keys(const uint32_t* act, uint32_t U, const int32_t* sa, const uint32_t* rank, uint32_t n, uint32_t h,
                    unsigned long long* key, uint32_t* val, hipStream_t st);
void launch_ix_isa(const int32_t* sa, uint32_t n, uint32_t* isa, int32_t* phi, hipStream_t st);
void launch_ix_lcp(const uint8_t* x, const int32_t* sa, uint32_t n, const uint32_t* isa, const int32_t* phi,
                   int32_t* plcpRaw, int32_t* lcp, int32_t* plcp, hipStream_t st);
void launch_ix_bwt(const uint8_t* x, const int32_t* sa, uint32_t n, uint8_t* bwt, hipStream_t st);
void launch_ix_plcp_check(const int32_t* plcp, uint32_t n, uint32_t* err, hipStream_t st);
// min(PLCP, 255) bytes for the walk's first skip window (DevRef::plcp8)
void launch_ix_plcp8(const int32_t* plcp, uint32_t n, uint8_t* out, hipStream_t st);
void launch_ix_level(const int32_t* prev, uint32_t prevLen, int32_t* cur, uint32_t curLen, hipStream_t st);
void launch_ix_child(const uint8_t* x, const int32_t* sa, const int32_t* lcp, uint32_t n, uint32_t* ld,
                     hipStream_t st);
void launch_ix_adjacency(const int32_t* sa, const uint32_t* isa, const int32_t* lcp, uint32_t n, uint32_t* pr,
                         uint32_t* ir, hipStream_t st);
void launch_ix_pfx_count(const uint8_t* x, uint32_t n, uint32_t l, uint32_t B, const uint8_t* map,
                         const uint32_t* below, uint32_t* cur, uint8_t* term, uint32_t* cf, uint32_t* ct,
                         hipStream_t st);
void launch_ix_pfx_write(const uint32_t* cfEx, const uint32_t* ctIn, const uint32_t* cf, uint64_t E1, uint32_t* o,
                         hipStream_t st);
void launch_ix_pfx_one(uint32_t* tab, uint64_t E, const int32_t* sa, hipStream_t st);
// paired level-K table (DevRef::pfk), 16 words per line of 4^(K-1)
void launch_ix_pfx_pair(const uint32_t* tabK, uint32_t K, uint32_t* out, hipStream_t st);
void launch_ix_pfx_answer(uint32_t* tab, const uint32_t* par, uint64_t E, uint32_t B, const int32_t* sa, uint32_t n,
                          uint32_t l, hipStream_t st);

// synth.hip
void launch_synth_collection(uint8_t* text, uint64_t L, uint64_t seed, uint64_t copy_begin, uint64_t ncopies,
                             uint64_t pthr, uint64_t base, hipStream_t st);

}  // namespace cmsbwt
