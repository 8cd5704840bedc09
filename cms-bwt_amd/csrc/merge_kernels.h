// merge_kernels.h — launchers for merge.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

namespace cmsbwt {


void mk_iota(uint32_t* p, uint64_t n, hipStream_t st);
void mk_gather(const uint32_t* src, const uint32_t* perm, uint32_t* dst, uint64_t n, hipStream_t st);
void mk_item_flags(const uint32_t* perm, const HeadsSoA& h, uint32_t* flag, uint64_t H, hipStream_t st);
void mk_group_key(const HeadsSoA& h, uint64_t H, int bN, int bL, unsigned long long* key, hipStream_t st);
// grouping, position first (radix by pos, then per-position segments)
// members of the big segments (bpos, offsets off in the big list) reordered
// into map order; t* are temporaries of the big list's size
void mk_grp_big_maporder(const uint32_t* bpos, uint32_t nb, const uint32_t* hb, const uint32_t* off,
                         unsigned long long* key, uint32_t* perm, uint32_t* ts, uint8_t* sm, unsigned long long* tKey,
                         uint32_t* tPerm, uint32_t* tTs, uint8_t* tSm, uint32_t* tF, int bN, hipStream_t st);
void mk_grp_seg(const uint32_t* posS, const uint32_t* hb, const HeadKV* kv, uint32_t H, int bN, int bL,
                unsigned long long* key, uint32_t* perm, uint32_t* tsOut, uint8_t* smOut, uint32_t* bigList,
                uint32_t maxSmall, int32_t* diffEnds, uint32_t n, hipStream_t st);
void mk_run_starts(const uint32_t* hb, uint32_t n, int32_t* diff, uint8_t* hasHead, hipStream_t st);
void mk_grp_big_fields(const uint32_t* idx, uint32_t B, const uint32_t* perm, const HeadsSoA& h, uint32_t* tsOut,
                       uint8_t* smOut, hipStream_t st);
void mk_grp_big_sizes(const uint32_t* pos, uint32_t nb, const uint32_t* hb, uint32_t* sz, hipStream_t st);
void mk_grp_big_expand(const uint32_t* pos, uint32_t nb, const uint32_t* hb, const uint32_t* off, uint32_t* idx,
                       hipStream_t st);
void mk_gather_kp(const uint32_t* idx, uint32_t B, const unsigned long long* key, const uint32_t* perm,
                  unsigned long long* keyB, uint32_t* permB, hipStream_t st);
void mk_scatter_kp(const uint32_t* idx, uint32_t B, const unsigned long long* keyB, const uint32_t* permB,
                   unsigned long long* key, uint32_t* perm, hipStream_t st);
void mk_item_flags64(const unsigned long long* key, uint32_t* flag, uint64_t H, hipStream_t st);
void mk_item_fill64(const unsigned long long* key, const uint32_t* perm, const uint32_t* flag, const uint32_t* incl,
                    const HeadsSoA& h, const uint32_t* tsS, const uint8_t* smS, uint64_t H, int bN, int bL,
                    const ItemsSoA& it, hipStream_t st);
void mk_item_fill(const uint32_t* perm, const uint32_t* flag, const uint32_t* incl, const HeadsSoA& h,
                  uint64_t H, const ItemsSoA& it, hipStream_t st);
void mk_item_count(const uint32_t* first, uint32_t* count, uint32_t K, uint32_t H, hipStream_t st);
// slot-major members: item of each slot, member idx of each slot, ranks and
// unresolved sa positions (0xffffffff = resolved), next-head ranks
void mk_slot_mark(const uint32_t* slot, uint32_t K, uint32_t* mark, hipStream_t st);
void mk_slot_members(const ItemsSoA& it, const uint32_t* itemOfSlot, const uint32_t* perm, uint32_t H, uint32_t* Pm,
                     hipStream_t st);
void mk_pos_rank_base(const uint32_t* posBegin, const uint32_t* slot, const uint32_t* isaRef,
                      const uint32_t* itemRankBase, const uint32_t* headBase, uint32_t n, uint32_t E,
                      uint32_t* rankBase, uint32_t* gBase, hipStream_t st);
// gItem (optional, K): the first sa position (= 1 + first head rank) of each
// item; unres (optional, H + 1): per sa position, 1 when its item has >= 2 heads
void mk_ranks_slot(const ItemsSoA& it, const uint32_t* itemOfSlot, const uint32_t* Pm, uint32_t H,
                   const uint32_t* rankBase, const uint32_t* gBase, uint32_t n, int32_t* T, uint32_t* sa,
                   uint32_t* grp, uint32_t* actv, hipStream_t st, uint32_t* gItem = nullptr,
                   uint8_t* unres = nullptr, uint32_t saFlag = 0u);
// byte-flag compaction into the kept indices (k_sel_count / k_sel_write)
void mk_sel_count8(const uint8_t* flags, uint32_t n, uint32_t* tileCnt, hipStream_t st);
// the same over bit 31 of u32 words; p[i] &= m
void mk_sel_count31(const uint32_t* words, uint32_t n, uint32_t* tileCnt, hipStream_t st);
void mk_sel_write_idx31(const uint32_t* words, uint32_t n, const uint32_t* tileOff, uint32_t* out, hipStream_t st);
void mk_and_u32(uint32_t* p, uint64_t n, uint32_t m, hipStream_t st);
void mk_sel_write_idx8(const uint8_t* flags, uint32_t n, const uint32_t* tileOff, uint32_t* out, hipStream_t st);
// the character before each head at slot[q] + rank - (gItem[q] - 1)
void mk_head_chars_slot(const uint32_t* Pm, const uint32_t* grp, const uint8_t* lchar, const ItemsSoA& it,
                        const uint32_t* itemOfSlot, const uint32_t* gItem, uint32_t H, uint8_t* bwtSlot,
                        hipStream_t st);
// fixed counter windows of winPos targets over [P0, P1): inclusive window
// count per position and the nw + 1 window starts
void mk_win_fixed(uint32_t n, uint32_t P0, uint32_t P1, uint32_t winPos, uint32_t nw, uint32_t* wincl,
                  uint32_t* winStart, hipStream_t st);
// *p = v, stream-ordered (no host staging of a stack value)
void mk_set_u32(uint32_t* p, uint32_t v, hipStream_t st);
// statistics of the counter's (item, target) pairs (CMSBWT_COUNTER_STATS=2)
void mk_counter_shape(const ItemsSoA& it, uint32_t K, uint32_t n, unsigned long long* out, hipStream_t st);
// per head in document order: (next-head rank, head rank, BWT character)
void mk_nhr_rec(const uint32_t* grp, const uint16_t* nexthead, const uint8_t* lchar, uint32_t H, uint4* rec,
                hipStream_t st);
// nbi: H scratch words (next-head rank per head in document order)
// headRank - sub = rank of each head (sub 1 with the final group labels)
void mk_nhr_slot(const uint32_t* Pm, const uint32_t* headRank, uint32_t sub, const uint16_t* nexthead, uint32_t H,
                 uint32_t* nbi, uint32_t* nhr, hipStream_t st);
void mk_head_chars(const uint32_t* sa, const uint8_t* lchar, uint32_t H, uint8_t* bwtHeads, hipStream_t st);
void mk_nhr_idx(const uint32_t* headRank, uint32_t sub, const uint16_t* nexthead, uint32_t H, uint32_t* nbi,
                hipStream_t st);
void mk_nhr_sort_small(const ItemsSoA& it, uint32_t K, uint32_t* nhr, uint32_t* bigList, hipStream_t st);
// next-head rank of each slot's member ranked inside its item (items <= kSmallSeg);
// nbi in document order read through Pm, or already in slot order (Pm null)
// rec (with Pm): records of mk_nhr_rec instead of nbi; each slot also writes
// its head's character at slot[q] + rank - (gItem[q] - 1) of bwtSlot
void mk_nhr_rank(const uint32_t* Pm, const uint32_t* nbi, const uint32_t* itemOfSlot, uint32_t H, uint32_t* nhr,
                 hipStream_t st, const uint4* rec = nullptr, const uint32_t* slot = nullptr,
                 const uint32_t* gItem = nullptr, uint8_t* bwtSlot = nullptr);
void mk_nhr_big_list(const ItemsSoA& it, uint32_t K, uint32_t* bigList, hipStream_t st);
void mk_nhr_big_fill(const uint32_t* items, const uint32_t* off, uint32_t nb, const ItemsSoA& it, const uint32_t* nhr,
                     unsigned long long* key, uint32_t* slots, hipStream_t st);
void mk_item_counts_of(const uint32_t* items, uint32_t nb, const uint32_t* count, uint32_t* out, hipStream_t st);
void mk_nhr_big_back(const unsigned long long* sorted, const uint32_t* slots, uint32_t B, uint32_t* nhr,
                     hipStream_t st);
void mk_item_permute(const ItemsSoA& in, const uint32_t* order, const ItemsSoA& out, uint32_t K, hipStream_t st);
void mk_pos_begin(const uint32_t* ipos, uint32_t K, uint32_t n, uint32_t* posBegin, hipStream_t st);
void mk_pos_f(const uint32_t* ipos, const uint8_t* ism, const uint32_t* posBegin, uint32_t K, uint32_t n,
              uint32_t* posF, hipStream_t st);
// positions whose items break the map-order invariant: counted into *viol and,
// when amb is given, marked amb[pos] = 1
void mk_check_items(const ItemsSoA& it, const uint32_t* posBegin, const uint32_t* posF, uint32_t K,
                    unsigned long long* viol, uint8_t* amb, hipStream_t st);
void mk_sa_counts(const int32_t* sa, const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t E,
                  uint32_t* itemsSA, uint32_t* headsSA, hipStream_t st);
void mk_dbl_keys(const uint32_t* act, const uint32_t* sa, const uint32_t* grp, uint32_t h, uint32_t U,
                 uint64_t* key, uint32_t* val, hipStream_t st, uint32_t saMask = 0xffffffffu);
void mk_dbl_apply(const uint32_t* act, const uint64_t* key, const uint32_t* val, uint32_t U, uint32_t* sa,
                  uint32_t* lab, hipStream_t st);
void mk_dbl_groups(const uint32_t* act, const uint64_t* key, const uint32_t* val, const uint32_t* labMax,
                   uint32_t U, uint32_t* grp, uint32_t* keep, hipStream_t st);
// u32 plus scans over tiles of 2048 (tile sums, their scan, the tiles)
uint64_t scan_tiles(uint64_t n);
void mk_scan_sums(const uint32_t* in, uint64_t n, uint32_t* sums, hipStream_t st);
void mk_scan_tiles(const uint32_t* in, uint32_t* out, uint64_t n, const uint32_t* tileOff, uint32_t init,
                   bool inclusive, hipStream_t st);
// the same over u64 values plus a constant
void mk_scan64_sums(const unsigned long long* in, uint64_t n, uint32_t add, unsigned long long* sums, hipStream_t st);
void mk_scan64_tiles(const unsigned long long* in, unsigned long long* out, uint64_t n, const unsigned long long* tileOff,
                     uint32_t add, bool inclusive, hipStream_t st);
// order-preserving compaction of flagged u32 values (tiles of 2048); `out`
// must not alias `in` (k_sel_write reads in[] after other blocks may have
// written their compacted values)
uint32_t sel_tiles(uint32_t n);
void mk_sel_count(const uint32_t* flags, uint32_t n, uint32_t* tileCnt, hipStream_t st);
void mk_sel_write(const uint32_t* in, const uint32_t* flags, uint32_t n, const uint32_t* tileOff, uint32_t* out,
                  hipStream_t st);
// map order of each position's items, one thread per position (the composite-key
// grouping paths; the position-first grouping emits map order itself)
void mk_map_order(const uint32_t* posBegin, const uint32_t* len, const uint8_t* sm, uint32_t n, uint32_t* order,
                  hipStream_t st);
// per-group doubling round (small groups sorted by one thread each)
void mk_dbl_small2(const uint32_t* gflag, uint32_t U, const uint32_t* act, uint64_t* key, uint32_t* val, uint32_t* sa,
                   uint32_t* grp, uint32_t* keep, uint32_t* bigList, uint32_t maxSmall, hipStream_t st);
void mk_dbl_rank(uint32_t U, const uint32_t* act, const uint64_t* key, const uint32_t* val, uint32_t* sa,
                 uint32_t* grp, uint32_t* keep, uint32_t* bigList, uint32_t maxSmall, hipStream_t st);
void mk_dbl_gstart(const uint64_t* key, uint32_t U, uint32_t* flag, hipStream_t st);
void mk_dbl_gather_big(const uint32_t* orig, uint32_t B, const uint32_t* act, const uint64_t* key, const uint32_t* val,
                       uint32_t* actB, uint64_t* keyB, uint32_t* valB, hipStream_t st);
void mk_scatter_u32(const uint32_t* src, const uint32_t* idx, uint32_t n, uint32_t* dst, hipStream_t st);
void mk_win_flags(const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t P0, uint32_t P1,
                  uint32_t winPos, uint32_t slotCap, uint32_t* flag, hipStream_t st);
void mk_win_starts(const uint32_t* flag, const uint32_t* winIncl, uint32_t n, uint32_t* winStart, hipStream_t st);
void mk_win_cross(const ItemsSoA& it, uint32_t K, const uint32_t* winIncl, uint32_t n, uint32_t* cnt,
                  const uint32_t* off, uint32_t* keyW, uint32_t* valQ, unsigned long long* errs, int fill,
                  hipStream_t st);
void mk_win_cross_off(const uint32_t* keyW, uint32_t ncross, uint32_t nw, uint32_t* crossOff, hipStream_t st);
// crossing lists without a sort (merge.hip k_xw_*): sources sv = 0 .. nw
// (0: items before P0, sv: window sv - 1); kXwMaxDepth bounds the depth
constexpr uint32_t kXwMaxDepth = 1024;
void mk_xw_depth(const uint32_t* posBegin, const uint32_t* winStart, uint32_t P0, uint32_t nsv, const uint32_t* cnt,
                 uint32_t* depth, hipStream_t st);
void mk_xw_hist(const uint32_t* posBegin, const uint32_t* winStart, uint32_t P0, uint32_t nsv, const uint32_t* cnt,
                const uint32_t* depth, const uint32_t* toff, uint32_t* T, hipStream_t st);
void mk_xw_count(const uint32_t* depth, const uint32_t* toff, const uint32_t* T, uint32_t nw, uint32_t maxDepth,
                 uint32_t* segOff, uint32_t* count, hipStream_t st);
void mk_xw_place(const uint32_t* posBegin, const uint32_t* winStart, uint32_t P0, uint32_t nsv, const uint32_t* cnt,
                 const uint32_t* depth, const uint32_t* toff, const uint32_t* segOff, const uint32_t* crossOff,
                 uint32_t* crossList, hipStream_t st);
void mk_item_sk(const ItemsSoA& it, uint32_t K, hipStream_t st);
// Queries of the checked counter (hr != nullptr) whose target t has mask[t]
// are not answered on the device: (source slot, t) pairs go to list (cnt
// counts them, the first cap are stored) for the host's std::map replay; a
// query at an unmasked target that could land differently in a std::map
// (match.h:27-33 not a strict weak order there) sets amb[t] and counts in
// stats[3].
struct HostRoute {
  const uint8_t* mask = nullptr;
  uint8_t* amb = nullptr;
  uint32_t* list = nullptr;
  unsigned long long* cnt = nullptr;
  unsigned long long cap = 0;
};
// Equal-key counter queries (FN:1537-1589: the answer compares next-head
// ranks) listed by a counter pass that runs before the next-head ranks exist:
// 16-byte records (query slot, query count, item slot, item count | hasNext
// << 31).  cnt[0] counts every listing, so cnt[0] > cap means overflow (the
// counter is then run again with the ranks).
struct EqList {
  uint4* rec = nullptr;
  unsigned long long* cnt = nullptr;
  unsigned long long cap = 0;
};
// the listed equal-key queries against the next-head ranks (adds and the
// good / bad statistics of FN:1537-1589)
void mk_counter_eq(const uint4* rec, uint32_t m, const uint32_t* nhr, unsigned long long* counter,
                   unsigned long long* stats, hipStream_t st);
void mk_counter_win(const ItemsSoA& it, const uint32_t* posBegin, const uint32_t* posF, const uint32_t* nhr,
                    const uint32_t* winStart, uint32_t nw, const uint32_t* crossOff, const uint32_t* crossList,
                    unsigned long long* counter, unsigned long long* stats, uint32_t n, uint32_t slotCap,
                    const HostRoute* hr, hipStream_t st);
// counter[slot[i]] += add[i]
void mk_counter_adds(const uint32_t* slot, const unsigned long long* add, uint32_t m, unsigned long long* counter,
                     hipStream_t st);
// mask[i] |= other[i]
void mk_or_mask(uint8_t* mask, const uint8_t* other, uint32_t n, hipStream_t st);
// target-major counter: windows of <= 256 targets (winStart), register accumulators
// eq.rec != nullptr (nhr unused): equal-key queries are listed in eq
void mk_counter_tgt(const ItemsSoA& it, const uint32_t* posBegin, const uint32_t* posF, const uint32_t* nhr,
                    const uint32_t* winStart, uint32_t nw, const uint32_t* crossOff, const uint32_t* crossList,
                    unsigned long long* counter, unsigned long long* stats, uint32_t n, hipStream_t st,
                    EqList eq = EqList{}, const uint4* irec = nullptr);
// per item (pos, until, len, count | smaller << 31): the counter's staging
// loads of an item in one 16-byte read
void mk_item_rec(const ItemsSoA& it, uint32_t K, uint4* out, hipStream_t st);
void mk_count_distinct(const uint32_t* v, uint32_t K, unsigned long long* out, hipStream_t st);
void mk_bucket(const int32_t* countIncl, const uint8_t* hasHead, uint32_t n, int64_t* bucket, hipStream_t st);
// run writer: units = E end phrases + SA ranks 1..n-1 (sharded merge), or
// elements (one GPU); a unit's / element's first run joins the previous one
void mk_wr_adjust(const uint32_t* hl, const uint32_t* prevHL, uint32_t U, uint32_t* runs, hipStream_t st);
void mk_wr_records(const unsigned long long* runStart, const uint8_t* runChar, uint64_t R, unsigned long long total,
                   uint8_t* out, hipStream_t st);
// element writer (one GPU): one thread per end phrase / head / head-less SA rank
struct ElemIn {
  const int32_t* sa;
  const uint8_t* bwt;
  const int64_t* bucket;
  const uint32_t* posBegin;
  const uint32_t* slot;
  const uint32_t* itemOfSlot;
  const uint32_t* headBase;
  const uint32_t* elemBase;
  const uint32_t* rOf;
  const uint8_t* bwtHeads;
  const unsigned long long* counter;
  const unsigned long long* cum;  // inclusive scan of counter + 1 over slots
  uint4* info1;                   // per SA rank (filled by mk_el_info)
  unsigned long long* info2;
  uint32_t n, E, H;
  int rle;
  const uint8_t* bwtSlot = nullptr;  // sharded merge: head characters by local slot
};
void mk_el_info(const ElemIn& w, hipStream_t st);
void mk_el_count(const uint32_t* headBase, uint32_t n, uint32_t E, uint32_t H, uint32_t* m, hipStream_t st);
void mk_el_rof(const uint32_t* elemBase, const uint32_t* m, uint32_t n, uint32_t* rOf, hipStream_t st);
// segs != null: each element's segments also stored (16 B, segs_pack) for
// mk_dm_el_emit to read back
void mk_el_wr_count(const ElemIn& w, uint32_t V, uint32_t* runs, unsigned long long* sym, uint32_t* hl,
                    hipStream_t st, uint4* segs = nullptr);
// run and symbol offsets packed into one 64-bit scan (symbol totals < 2^34,
// run totals < 2^30): k_el_wr_emit takes the packed offsets with symOff == nullptr
constexpr uint32_t kPackSymBits = 34;
void mk_el_wr_emit(const ElemIn& w, uint32_t V, const unsigned long long* runOff, const unsigned long long* symOff,
                   const uint32_t* prevHL, unsigned long long* runStart, uint8_t* runChar, hipStream_t st);
// the writer's run scan in tiles (elem_writer.h WrState / WrOp): per-tile
// summaries, then emission at each element's prefix; total = {runs, symbols}
struct WrState;
// segOut / segIn (optional, V x 16 B): the elements' segments stored by the
// first pass and read back by the second (elem_writer.h segs_pack)
void mk_el_wr_tiles(const ElemIn& w, uint32_t V, WrState* tileSum, hipStream_t st, uint4* segOut = nullptr);
// (rec: the 9-byte run records, FN:1708-1709, written directly)
void mk_el_wr_emit_tiles(const ElemIn& w, uint32_t V, const WrState* tilePre, uint8_t* rec,
                         unsigned long long* total, hipStream_t st, const uint4* segIn = nullptr);
// element writer of the position-sharded merge (elements of the owned SA
// ranks, units summarised for the all-reduce, emission per element)
void mk_dm_el_count(const int32_t* sa, const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t E,
                    uint32_t P0, uint32_t P1, uint32_t* m, hipStream_t st);
void mk_dm_el_info(const ElemIn& w, uint32_t P0, uint32_t P1, hipStream_t st);
void mk_dm_el_adj(const uint32_t* rOf, const uint32_t* hl, const uint32_t* runs, uint32_t V, uint32_t* adj,
                  hipStream_t st);
void mk_dm_el_units(const uint32_t* elemBase, const uint32_t* m, const unsigned long long* runIn,
                    const unsigned long long* symIn, const uint32_t* hl, uint32_t n, uint32_t E, uint32_t U,
                    int64_t* out, hipStream_t st);
void mk_dm_el_emit(const ElemIn& w, uint32_t V, const unsigned long long* runIn, const unsigned long long* symIn,
                   const unsigned long long* unitRunOff, const unsigned long long* unitSymOff, const uint32_t* prevHL,
                   const uint32_t* unitHL, const uint32_t* hl, unsigned long long* runStart, uint8_t* runChar,
                   hipStream_t st, const uint4* segs = nullptr);

// dist_kernels.hip: position-sharded merge (multi-GPU)
void mk_dm_owner(const uint32_t* vals, const uint32_t* idx, uint64_t n, const uint32_t* split, uint32_t world,
                 uint32_t* dest, hipStream_t st);
void mk_dm_bounds(const uint32_t* sorted, uint64_t n, uint32_t world, uint32_t* bounds, hipStream_t st);
void mk_dm_pack_heads(const uint32_t* perm, const HeadsSoA& h, uint64_t n, int32_t* out, hipStream_t st);
void mk_dm_unpack_heads(const int32_t* in, uint64_t n, const HeadsSoA& h, hipStream_t st);
void mk_dm_runs(const uint32_t* pos, const uint32_t* tonext, uint64_t H, uint32_t n, int32_t* diff, uint8_t* hasHead,
                hipStream_t st);
void mk_dm_sa_counts(const int32_t* sa, const uint32_t* posBegin, const uint32_t* slot, uint32_t n, uint32_t Eown,
                     uint32_t* out, hipStream_t st);
void mk_dm_group_labels(const ItemsSoA& it, const uint32_t* itemOfSlot, const uint32_t* Pm, uint32_t H,
                        const uint32_t* gBase, uint32_t n, uint32_t bias, unsigned long long* back, uint32_t* gItem,
                        hipStream_t st);
void mk_dm_grp_init(const uint32_t* perm, const unsigned long long* in, uint64_t n, uint32_t* grp, uint32_t* actFlag,
                    hipStream_t st);
void mk_dm_dbl_pack(const uint32_t* aPerm, const uint32_t* act, const uint32_t* grp, uint32_t h, uint64_t n,
                    uint32_t H, int32_t* out, uint32_t* err, hipStream_t st);
// label owner: sort by label offset, rank small groups in LDS, list big ones
void mk_dm_dbl_lkeys(const int32_t* in, uint64_t n, uint32_t G0, uint32_t* key, unsigned long long* val,
                     hipStream_t st);
void mk_dm_dbl_rank(const uint32_t* key, const unsigned long long* val, uint64_t n, uint32_t G0,
                    unsigned long long* res, uint32_t* bigList, hipStream_t st);
void mk_dm_dbl_bigkeys(const uint32_t* list, uint32_t B, const uint32_t* key, const unsigned long long* val,
                       uint32_t G0, unsigned long long* k64, uint32_t* v2, hipStream_t st);
void mk_dm_dbl_marks(const unsigned long long* key, uint64_t n, uint32_t* gs, uint32_t* ks, hipStream_t st);
void mk_dm_dbl_result(const unsigned long long* key, const uint32_t* val, const uint32_t* gsMax,
                      const uint32_t* ksMax, uint64_t n, unsigned long long* res, hipStream_t st);
void mk_dm_dbl_apply(const uint32_t* aPerm, const uint32_t* act, const unsigned long long* back, uint64_t n, uint32_t* grp,
                     uint32_t* keep, hipStream_t st);
// (head rank, next-head rank, BWT character): 3 words per head in send order
void mk_dm_pack_ranks(const uint32_t* perm, const uint32_t* grp, const uint16_t* nexthead, const uint8_t* lchar,
                      uint64_t n, uint32_t H, uint32_t bias, int32_t* out, uint32_t* err, hipStream_t st);
// head characters by slot (bwtSlot) and the next-head ranks in slot order (nbiS)
void mk_dm_load_ranks(const int32_t* in, const uint32_t* Pm, const uint32_t* itemOfSlot, const ItemsSoA& it,
                      const uint32_t* gItem, uint32_t H, uint32_t* nbiS, uint8_t* bwtSlot, uint32_t* err,
                      hipStream_t st);
void mk_dm_halo_count(const ItemsSoA& it, uint32_t K, const uint32_t* split, uint32_t world, uint32_t rank,
                      uint32_t n, uint32_t* c, hipStream_t st);
void mk_dm_halo_fill(const uint32_t* c, const uint32_t* off, uint32_t K, uint32_t rank, uint32_t* dest,
                     uint32_t* item, hipStream_t st);
void mk_dm_pair_words(const uint32_t* item, uint32_t np, const uint32_t* count, uint32_t* w, hipStream_t st);
void mk_dm_halo_pack(const uint32_t* item, uint32_t np, const ItemsSoA& it, const uint32_t* nhr, const uint32_t* wOff,
                     int32_t* hdr, int32_t* words, hipStream_t st);
void mk_dm_halo_unpack(const int32_t* hdr, uint32_t nh, const ItemsSoA& c, hipStream_t st);
void mk_dm_units_pack(const uint32_t* runs, const uint32_t* hl, const unsigned long long* sym, uint32_t U,
                      int64_t* out, hipStream_t st);
void mk_dm_units_unpack(const int64_t* in, uint32_t U, uint32_t* runs, uint32_t* hl, unsigned long long* sym,
                        hipStream_t st);
void mk_dm_own_runs(const uint32_t* runs, uint32_t U, const int32_t* sa, uint32_t E, uint32_t n, uint32_t P0,
                    uint32_t P1, unsigned long long* out, hipStream_t st);
void mk_dm_place(const uint32_t* runs, const unsigned long long* runOff, const unsigned long long* srcOff, uint32_t U,
                 const int32_t* sa, uint32_t E, uint32_t n, uint32_t P0, uint32_t P1,
                 const unsigned long long* srcStart, const uint8_t* srcChar, unsigned long long* runStart,
                 uint8_t* runChar, hipStream_t st);

}  // namespace cmsbwt
