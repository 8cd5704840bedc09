// dist_merge.hip — the MS-factor -> BWT-run merge sharded over ranks by
// reference position (SURVEY.md §8e "later": partition counterSmallerThanHead
// and emission by reference position / SA range).
//
// One process per GPU.  After each rank's document-local walk and j-scan
// (FN:1151-1385) the merge runs as:
//   1. heads -> owner of their position (all-to-all); per-position arrays
//      (bucket difference array, head flags) all-reduced;
//   2. position owner: grouping into items and map order (FN:1387-1416),
//      per-SA-rank item/head counts all-reduced -> every member's initial
//      group label in the head-string suffix array (FN:1432-1453), returned
//      to the head's document rank;
//   3. libsais_int (FN:1455-1459) as prefix doubling: document ranks build
//      (label, label of suffix + h) keys (lookups stay inside the document,
//      whose end phrase has a unique rank), owners of label ranges sort them
//      and relabel; repeated until every suffix is alone in its group;
//   4. head ranks / next-head ranks (FN:1468-1494) -> position owners;
//   5. counterSmallerThanHead (FN:1523-1603) per position range, with the
//      items of earlier ranks that reach into it (halo);
//   6. writer units (FN:1695-1777): per-unit run counts all-reduced, each rank
//      emits the runs of its units, rank 0 places them and packs records.
// The transport is the caller's (cmsbwt/dist.py: torch.distributed, RCCL
// over xGMI); every call here ends with the engine stream synchronised.
#include "engine.h"

namespace cmsbwt {

template <class T>
static void swap_buf(DBuf<T>& a, DBuf<T>& b) {
  std::swap(a.p, b.p);
  std::swap(a.n, b.n);
  std::swap(a.owner, b.owner);
}

void Engine::partition(const uint32_t* dest, uint64_t cnt, DBuf<uint32_t>& perm, std::vector<uint64_t>& counts) {
  const uint32_t world = dm.world;
  counts.assign(world, 0);
  perm.alloc(cnt);
  if (!cnt) return;
  if (cnt >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "partition larger than 2^32"};
  if (world == 1) {  // one destination: send order = input order
    mk_iota(perm.p, cnt, st);
    counts[0] = cnt;
    return;
  }
  DBuf<uint32_t> io, k2, bnd;
  io.alloc(cnt); k2.alloc(cnt); bnd.alloc((uint64_t)world + 1);
  mk_iota(io.p, cnt, st);
  sort_pairs(dest, k2.p, io.p, perm.p, cnt, bits_for(world - 1));  // stable
  mk_dm_bounds(k2.p, cnt, world, bnd.p, st);
  std::vector<uint32_t> b(world + 1);
  HIPCHK(hipMemcpyAsync(b.data(), bnd.p, (world + 1) * 4, hipMemcpyDeviceToHost, st));
  sync();
  for (uint32_t k = 0; k < world; k++) counts[k] = b[k + 1] - b[k];
}

void Engine::dm_check_err(const char* where) {
  const uint32_t e = read1(dm.err.p);
  if (e) throw InputError{CMSBWT_EINPUT, std::string("internal: sharded merge invariant broken in ") + where +
                                             " (flags " + std::to_string(e) + ")"};
}

void Engine::dm_begin(uint32_t world, uint32_t rank, uint64_t heads_total, uint64_t docs_total, uint32_t flags,
                      int rle) {
  if (!walked) throw InputError{CMSBWT_EARG, "run ms_walk first"};
  if (world < 1 || world > 64 || rank >= world) throw InputError{CMSBWT_EARG, "bad world/rank"};
  // head indices, group labels and ranks are uint32 (labels 1 .. H + 1): the
  // reference's int32 limit (FN:1436-1437, 1456) is lifted to 2^32 - 2
  if (heads_total >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "more than 2^32-2 heads (uint32 head indices)"};
  if (heads_total == 0)  // as Engine::merge: FN:1359-1385 is undefined without heads
    throw InputError{CMSBWT_EINPUT, "collection has no documents (reference behaviour undefined, FN:1359-1385)"};
  const uint32_t n = R.n;
  merged = false;
  dm.on = false;
  dm.world = world;
  dm.rank = rank;
  dm.Htot = (uint32_t)heads_total;
  dm.E = (uint32_t)docs_total;
  dm.rle = rle;
  dm.check = !(flags & 1u) || env_u32("CMSBWT_FORCE_CHECK", 0) != 0;
  // group labels are 1 .. Htot (+ bias: tests push them across 2^31 with
  // small inputs; the labels, the label-range owners and the doubling keys
  // carry it, the head ranks drop it)
  {
    const char* b = getenv("CMSBWT_DM_LABEL_BIAS");
    const uint64_t bias = b ? strtoull(b, nullptr, 10) : 0;
    if (bias + heads_total >= 0xffffffffull) throw InputError{CMSBWT_EARG, "label bias too large"};
    dm.labelBias = (uint32_t)bias;
  }
  dm.Psplit.assign(world + 1, 0);
  dm.Gsplit.assign(world + 1, 0);
  for (uint32_t k = 0; k <= world; k++) {
    dm.Psplit[k] = (uint32_t)((uint64_t)k * n / world);
    dm.Gsplit[k] = dm.labelBias + 1 + (uint32_t)((uint64_t)k * dm.Htot / world);
  }
  dm.Gsplit[world] = dm.labelBias + dm.Htot + 1;
  dm.P0 = dm.Psplit[rank];
  dm.P1 = dm.Psplit[rank + 1];
  dm.dPsplit.alloc(world + 1);
  dm.dGsplit.alloc(world + 1);
  HIPCHK(hipMemcpyAsync(dm.dPsplit.p, dm.Psplit.data(), (world + 1) * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dm.dGsplit.p, dm.Gsplit.data(), (world + 1) * 4, hipMemcpyHostToDevice, st));
  dm.err.alloc(1);
  dm.err.zero(st);
  sync();
}

// ---- 1. heads to the owners of their positions
void Engine::dm_route_heads(uint64_t* counts) {
  DBuf<uint32_t> dest;
  dest.alloc(H);
  mk_dm_owner(hPos.p, nullptr, H, dm.dPsplit.p, dm.world, dest.p, st);
  partition(dest.p, H, dm.hPerm, dm.hCnt);
  for (uint32_t k = 0; k < dm.world; k++) counts[k] = dm.hCnt[k];
}

void Engine::dm_pack_heads(int32_t* out) {
  mk_dm_pack_heads(dm.hPerm.p, heads(), H, out, st);
  HIPCHK(hipGetLastError());
  sync();
}

// ---- 2. items of the owned positions (received in global idx order:
// ranks in order, each in document order) and per-SA-rank counts
void Engine::dm_group(const int32_t* recv, uint64_t nrecv, uint32_t* saCounts) {
  if (nrecv >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "too many heads on one rank"};
  const uint32_t n = R.n;
  const uint32_t Hp = dm.Hp = (uint32_t)nrecv;
  dmt(nullptr);
  dm.rPos.alloc(Hp); dm.rLen.alloc(Hp); dm.rIsa.alloc(Hp); dm.rTon.alloc(Hp);
  dm.rSm.alloc(Hp); dm.rCh.alloc(Hp);
  HeadsSoA r{nullptr, dm.rPos.p, dm.rLen.p, dm.rSm.p, dm.rCh.p, dm.rIsa.p, dm.rTon.p, nullptr};
  mk_dm_unpack_heads(recv, Hp, r, st);
  dmt("unpack");
  // run buckets (FN:1162-1171) of the heads at the owned positions, from the
  // grouping's position sort: head flags of the owned positions are final,
  // the difference array is summed over ranks (a run may end in a later
  // range) with the per-SA-rank counts, in saCounts[2n .. 3n]
  runsValid = false;
  group_items(r, Hp, n, dm.IS);
  dmt("group_items");
  if (!runsValid) {  // grouped by the composite-key sorts (keys wider than 64 bits): count them here
    diff.alloc((uint64_t)n + 1);
    diff.zero(st);
    hasHead.alloc(n);
    hasHead.zero(st);
    mk_dm_runs(dm.rPos.p, dm.rTon.p, Hp, n, diff.p, hasHead.p, st);
    runsValid = true;
  }
  const uint32_t K = dm.IS.K;
  ItemsSoA S = dm.IS.soa();
  dm.viol = 0;
  if (dm.check && K) {
    DBuf<unsigned long long> v;
    v.alloc(1);
    v.zero(st);
    mk_check_items(S, dm.IS.posBegin.p, dm.IS.posF.p, K, v.p, nullptr, st);
    dm.viol = read1(v.p);
  }
  dmt("check");
  // slot-major members: item of each slot, received index of each slot
  dm.itemOfSlot.alloc(Hp);
  if (Hp) {
    DBuf<uint32_t> mark;
    mark.alloc(Hp);
    mark.zero(st);
    mk_slot_mark(S.slot, K, mark.p, st);
    inscan(mark.p, dm.itemOfSlot.p, Hp, rocprim::plus<uint32_t>());
  }
  if (dm.IS.slotIsFirst) {
    dm.Pm.swap_in(dm.IS.P);  // members already in slot order
  } else {
    dm.Pm.alloc(Hp);
    if (Hp) mk_slot_members(S, dm.itemOfSlot.p, dm.IS.P.p, Hp, dm.Pm.p, st);
  }
  const bool ownsEnd = dm.P0 <= n - 1 && n - 1 < dm.P1;
  mk_dm_sa_counts(dsa.p, dm.IS.posBegin.p, S.slot, n, ownsEnd ? dm.E : 0, saCounts, st);
  HIPCHK(hipMemcpyAsync(saCounts + 2ull * n, diff.p, ((uint64_t)n + 1) * 4, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipGetLastError());
  sync();
  dmt("slots+sa_counts");
  dmtFlush("dm_group");
}

void Engine::dm_labels(const uint32_t* saCounts, unsigned long long* back) {
  const uint32_t n = R.n;
  // the difference array summed over ranks (head flags stay this rank's)
  HIPCHK(hipMemcpyAsync(diff.p, saCounts + 2ull * n, ((uint64_t)n + 1) * 4, hipMemcpyDeviceToDevice, st));
  dm.headBase.alloc(n);
  exscan(saCounts + n, dm.headBase.p, 0u, n);
  dm.gItem.alloc(std::max<uint32_t>(dm.IS.K, 1));
  {
    DBuf<uint32_t> gBase;
    gBase.alloc(n);
    mk_pos_rank_base(dm.IS.posBegin.p, dm.IS.slot.p, disa.p, nullptr, dm.headBase.p, n, 0, nullptr, gBase.p, st);
    mk_dm_group_labels(dm.IS.soa(), dm.itemOfSlot.p, dm.Pm.p, dm.Hp, gBase.p, n, dm.labelBias, back, dm.gItem.p, st);
  }
  HIPCHK(hipGetLastError());
  sync();
}

// ---- 3. prefix doubling of the head string
uint64_t Engine::dm_dbl_init(const unsigned long long* labels) {
  dm.grp.alloc(H);
  dm.act.alloc(H);
  dm.U = 0;
  if (H) {
    // unresolved members listed in send order (the doubling does not depend
    // on the order of act): one scatter per head, the labels
    DBuf<uint32_t> flag;
    flag.alloc(H);
    mk_dm_grp_init(dm.hPerm.p, labels, H, dm.grp.p, flag.p, st);
    dm.U = select_flagged(dm.hPerm.p, flag.p, dm.act.p, H);
  }
  return dm.U;
}

void Engine::dm_dbl_route(uint64_t h, uint64_t* counts) {
  if (h >= 0x80000000ull) throw InputError{CMSBWT_EINPUT, "internal: head-string suffix sort did not converge"};
  dm.dblH = (uint32_t)h;
  DBuf<uint32_t> dest;
  dest.alloc(dm.U);
  mk_dm_owner(dm.grp.p, dm.act.p, dm.U, dm.dGsplit.p, dm.world, dest.p, st);
  std::vector<uint64_t> c;
  partition(dest.p, dm.U, dm.aPerm, c);
  for (uint32_t k = 0; k < dm.world; k++) counts[k] = c[k];
}

void Engine::dm_dbl_pack(int32_t* out) {
  mk_dm_dbl_pack(dm.aPerm.p, dm.act.p, dm.grp.p, dm.dblH, dm.U, H, out, dm.err.p, st);
  HIPCHK(hipGetLastError());
  sync();
  dm_check_err("doubling keys");
}

// label-range owner: new labels of the received (label, label2) pairs.  The
// members are sorted by label only (bits of the owned label range), groups of
// <= 32 members ranked by counting in LDS (k_dm_dbl_rank); the members of
// larger groups go through the full-key sort.
void Engine::dm_dbl_sort(const int32_t* recv, uint64_t nrecv, unsigned long long* res) {
  if (!nrecv) return;
  if (nrecv >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "doubling group larger than 2^32"};
  const uint32_t G0 = dm.Gsplit[dm.rank], G1 = dm.Gsplit[dm.rank + 1];
  DBuf<uint32_t> key, key2, big;
  DBuf<unsigned long long> val, val2;
  key.alloc(nrecv); key2.alloc(nrecv); val.alloc(nrecv); val2.alloc(nrecv); big.alloc(nrecv + 1);
  mk_dm_dbl_lkeys(recv, nrecv, G0, key.p, val.p, st);
  sort_pairs(key.p, key2.p, val.p, val2.p, nrecv, bits_for(G1 > G0 ? G1 - G0 - 1 : 0));
  key.release();
  val.release();
  HIPCHK(hipMemsetAsync(big.p, 0, 4, st));
  mk_dm_dbl_rank(key2.p, val2.p, nrecv, G0, res, big.p, st);
  const uint32_t B = read1(big.p);
  if (B) {
    DBuf<unsigned long long> k64, k64b;
    DBuf<uint32_t> v, vb, gs, ks, gsM, ksM;
    k64.alloc(B); k64b.alloc(B); v.alloc(B); vb.alloc(B);
    mk_dm_dbl_bigkeys(big.p + 1, B, key2.p, val2.p, G0, k64.p, v.p, st);
    sort_pairs(k64.p, k64b.p, v.p, vb.p, B, 32 + bits_for(G1 - 1));  // labels < G1
    gs.alloc(B); ks.alloc(B); gsM.alloc(B); ksM.alloc(B);
    mk_dm_dbl_marks(k64b.p, B, gs.p, ks.p, st);
    inscan(gs.p, gsM.p, B, rocprim::maximum<uint32_t>());
    inscan(ks.p, ksM.p, B, rocprim::maximum<uint32_t>());
    mk_dm_dbl_result(k64b.p, vb.p, gsM.p, ksM.p, B, res, st);
  }
  HIPCHK(hipGetLastError());
  sync();
}

uint64_t Engine::dm_dbl_apply(const unsigned long long* back) {
  if (!dm.U) return 0;
  DBuf<uint32_t> keep, act2;
  keep.alloc(dm.U);
  act2.alloc(dm.U);
  mk_dm_dbl_apply(dm.aPerm.p, dm.act.p, back, dm.U, dm.grp.p, keep.p, st);
  dm.U = select_flagged(dm.act.p, keep.p, act2.p, dm.U);
  swap_buf(dm.act, act2);
  return dm.U;
}

// ---- 4. head ranks and next-head ranks to the position owners
void Engine::dm_pack_ranks(int32_t* out) {
  mk_dm_pack_ranks(dm.hPerm.p, dm.grp.p, hNext.p, hChar.p, H, H, dm.labelBias, out, dm.err.p, st);
  HIPCHK(hipGetLastError());
  sync();
  dm_check_err("next-head ranks");
}

void Engine::dm_load_ranks(const int32_t* recv) {
  const uint32_t Hp = dm.Hp;
  dm.nhr.alloc(std::max<uint32_t>(Hp, 1));
  dm.bwtSlot.alloc(std::max<uint32_t>(Hp, 1));  // never null: selects the sharded writer
  ItemsSoA S = dm.IS.soa();
  {
    // FN:1480-1494: next-head ranks sorted per item, as on one GPU (ranked
    // inside small items through Pm, large items by one sort)
    DBuf<uint32_t> nbi;
    nbi.alloc(std::max<uint32_t>(Hp, 1));
    mk_dm_load_ranks(recv, dm.Pm.p, dm.itemOfSlot.p, S, dm.gItem.p, Hp, nbi.p, dm.bwtSlot.p, dm.err.p, st);
    if (Hp) {
      mk_nhr_rank(nullptr, nbi.p, dm.itemOfSlot.p, Hp, dm.nhr.p, st);  // nbi in slot order
      sort_nhr_items(S, dm.IS.K, dm.itemOfSlot.p, dm.nhr.p, Hp, true);
    }
  }
  HIPCHK(hipGetLastError());
  sync();
  dm_check_err("head characters");
}

// ---- 5. counters: items reaching into later ranks travel there first
void Engine::dm_route_halo(uint64_t* itemCounts, uint64_t* wordCounts) {
  const uint32_t K = dm.IS.K, world = dm.world;
  ItemsSoA S = dm.IS.soa();
  DBuf<uint32_t> c, off;
  c.alloc(K);
  off.alloc(K);
  mk_dm_halo_count(S, K, dm.dPsplit.p, world, dm.rank, R.n, c.p, st);
  exscan(c.p, off.p, 0u, K);
  const uint32_t np = K ? (uint32_t)sum2(off.p + (K - 1), c.p + (K - 1)) : 0;
  dm.npairs = np;
  DBuf<uint32_t> dest, item, perm, w;
  dest.alloc(np);
  item.alloc(np);
  mk_dm_halo_fill(c.p, off.p, K, dm.rank, dest.p, item.p, st);
  std::vector<uint64_t> cnt;
  partition(dest.p, np, perm, cnt);
  dm.pairItem.alloc(np);
  mk_gather(item.p, perm.p, dm.pairItem.p, np, st);
  w.alloc(np);
  dm.pairWordOff.alloc((uint64_t)np + 1);
  mk_dm_pair_words(dm.pairItem.p, np, S.count, w.p, st);
  exscan(w.p, dm.pairWordOff.p, 0u, np);
  uint64_t b = 0;
  for (uint32_t k = 0; k < world; k++) {
    itemCounts[k] = cnt[k];
    const uint64_t e = b + cnt[k];
    const uint32_t wb = b < np ? read1(dm.pairWordOff.p + b) : 0;
    const uint32_t we = e < np ? read1(dm.pairWordOff.p + e) : (np ? read1(dm.pairWordOff.p + (np - 1)) + read1(w.p + (np - 1)) : 0);
    wordCounts[k] = cnt[k] ? we - wb : 0;
    b = e;
  }
}

void Engine::dm_pack_halo(int32_t* hdr, int32_t* words) {
  mk_dm_halo_pack(dm.pairItem.p, dm.npairs, dm.IS.soa(), dm.nhr.p, dm.pairWordOff.p, hdr, words, st);
  HIPCHK(hipGetLastError());
  sync();
}

void Engine::dm_counter(const int32_t* hdr, uint64_t nh, const int32_t* words, uint64_t nw, uint64_t* out6) {
  const uint32_t n = R.n, K = dm.IS.K, Hp = dm.Hp;
  if (nh + K >= 0xffffffffull || nw + Hp >= 0x7fffffffull) throw InputError{CMSBWT_ELIMIT, "halo too large"};
  const uint32_t Kh = (uint32_t)nh, Kc = Kh + K, Hc = (uint32_t)nw + Hp;
  const ItemsSoA S = dm.IS.soa();
  dmt(nullptr);
  if (Kh == 0 && nw == 0) {  // no halo (rank 0, or one rank): the own items as they are
    DBuf<unsigned long long> cst;
    cst.alloc(8);
    cst.zero(st);
    dm.counter.alloc((uint64_t)Hp + 1);
    dm.counter.zero(st);
    counter_phase(S, K, dm.IS.posBegin.p, dm.IS.posF.p, dm.nhr.p, dm.counter.p, cst.p, n, dm.P0, dm.P1, dm.check);
    dmt("counter_phase");
    dmtFlush("dm_counter");
    unsigned long long cs[8];
    HIPCHK(hipMemcpyAsync(cs, cst.p, sizeof(cs), hipMemcpyDeviceToHost, st));
    sync();
    for (int k = 0; k < 5; k++) out6[k] = cs[k];
    out6[3] += dm.viol;
    out6[5] = K;
    stats.counter_kernel_ms = counter_kernel_ms;
    return;
  }
  // combined items: halo (positions before P0, ascending) then the own items
  DBuf<uint32_t> cPos, cLen, cIsa, cUntil, cCount, cSlot, cNhr, pb, pf;
  DBuf<uint8_t> cSmall;
  DBuf<unsigned long long> cSk, cst;
  cPos.alloc(Kc); cLen.alloc(Kc); cIsa.alloc(Kc); cUntil.alloc(Kc); cCount.alloc(Kc); cSmall.alloc(Kc);
  cSk.alloc(Kc); cSlot.alloc((uint64_t)Kc + 1); cNhr.alloc(std::max<uint32_t>(Hc, 1));
  ItemsSoA C{cPos.p, cLen.p, cIsa.p, cSmall.p, cUntil.p, cCount.p, nullptr, cSlot.p, nullptr, cSk.p};
  mk_dm_halo_unpack(hdr, Kh, C, st);
  dmt("halo_unpack");
  auto cp = [&](void* d, const void* s, uint64_t b) {
    if (b) HIPCHK(hipMemcpyAsync(d, s, b, hipMemcpyDeviceToDevice, st));
  };
  cp(cPos.p + Kh, S.pos, (uint64_t)K * 4);
  cp(cLen.p + Kh, S.len, (uint64_t)K * 4);
  cp(cIsa.p + Kh, S.isa, (uint64_t)K * 4);
  cp(cUntil.p + Kh, S.until, (uint64_t)K * 4);
  cp(cCount.p + Kh, S.count, (uint64_t)K * 4);
  cp(cSmall.p + Kh, S.smaller, K);
  cp(cNhr.p, words, nw * 4);
  cp(cNhr.p + nw, dm.nhr.p, (uint64_t)Hp * 4);
  exscan(cCount.p, cSlot.p, 0u, Kc);
  HIPCHK(hipMemcpyAsync(cSlot.p + Kc, &Hc, 4, hipMemcpyHostToDevice, st));
  mk_item_sk(C, Kc, st);
  pb.alloc((uint64_t)n + 1);
  pf.alloc(n);
  mk_pos_begin(cPos.p, Kc, n, pb.p, st);
  mk_pos_f(cPos.p, cSmall.p, pb.p, Kc, n, pf.p, st);
  sync();  // Hc is a stack variable
  dmt("combine");
  if (Kc && read1(cSlot.p + (Kc - 1)) + read1(cCount.p + (Kc - 1)) != Hc)
    throw InputError{CMSBWT_EINPUT, "internal: halo payload does not match its item counts"};
  DBuf<unsigned long long> cc;
  cc.alloc((uint64_t)Hc + 1);
  cc.zero(st);
  cst.alloc(8);
  cst.zero(st);
  counter_phase(C, Kc, pb.p, pf.p, cNhr.p, cc.p, cst.p, n, dm.P0, dm.P1, dm.check);
  dmt("counter_phase");
  dmtFlush("dm_counter");
  dm.counter.alloc((uint64_t)Hp + 1);
  dm.counter.zero(st);
  cp(dm.counter.p, cc.p + nw, (uint64_t)Hp * 8);
  unsigned long long cs[8];
  HIPCHK(hipMemcpyAsync(cs, cst.p, sizeof(cs), hipMemcpyDeviceToHost, st));
  sync();
  for (int k = 0; k < 5; k++) out6[k] = cs[k];
  out6[3] += dm.viol;
  out6[5] = K;  // items of the owned positions
  stats.counter_kernel_ms = counter_kernel_ms;
}

// ---- 6. writer: the element writer of one GPU over the SA ranks of the
// owned positions (one thread per end phrase / head / head-less rank);
// elements summarised per writer unit for the all-reduce
void Engine::dm_units(int64_t* out) {
  const uint32_t n = R.n;
  if ((uint64_t)dm.E + n - 1 >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "too many writer units"};
  const uint32_t Uw = dm.Uw = dm.E + n - 1;
  dmt(nullptr);
  dm.bucket.alloc(n);
  {
    DBuf<int32_t> cnt;
    cnt.alloc(n);
    inscan(diff.p, cnt.p, n, rocprim::plus<int32_t>());
    mk_bucket(cnt.p, hasHead.p, n, dm.bucket.p, st);
  }
  dmt("bucket");
  ItemSet& IS = dm.IS;
  DBuf<uint32_t> m;
  m.alloc(n);
  dm.eBase.alloc(n);
  mk_dm_el_count(dsa.p, IS.posBegin.p, IS.slot.p, n, dm.E, dm.P0, dm.P1, m.p, st);
  exscan(m.p, dm.eBase.p, 0u, n);
  const uint64_t V64 = sum2(dm.eBase.p + (n - 1), m.p + (n - 1));
  if (V64 >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "too many writer elements"};
  const uint32_t V = dm.V = (uint32_t)V64;
  dm.rOf.alloc(std::max<uint32_t>(V, 1));
  mk_el_rof(dm.eBase.p, m.p, n, dm.rOf.p, st);
  dmt("el_count+rof");
  const uint32_t Hp = dm.Hp;
  dm.cum.alloc(std::max<uint32_t>(Hp, 1));
  if (Hp)
    inscan_plus1_u64(dm.counter.p, dm.cum.p, Hp);
  dm.info1.alloc(n);
  dm.info2.alloc(n);
  const ElemIn ei = dm_elem_in();
  mk_dm_el_info(ei, dm.P0, dm.P1, st);
  dmt("cum+el_info");
  DBuf<uint32_t> runs, adj;
  DBuf<unsigned long long> sym;
  runs.alloc(std::max<uint32_t>(V, 1)); adj.alloc(std::max<uint32_t>(V, 1)); sym.alloc(std::max<uint32_t>(V, 1));
  dm.ehl.alloc(std::max<uint32_t>(V, 1));
  dm.runIn.alloc(std::max<uint32_t>(V, 1));
  dm.symPacked = false;
  if (V) {
    // the elements' segments kept for dm_emit (CMSBWT_WR_SEGBUF=0: recomputed
    // there, as the round-5 writer did)
    if (env_u32("CMSBWT_WR_SEGBUF", 1)) dm.segs.alloc(V);
    else dm.segs.release();
    mk_el_wr_count(ei, V, runs.p, sym.p, dm.ehl.p, st, dm.segs.p);
    mk_dm_el_adj(dm.rOf.p, dm.ehl.p, runs.p, V, adj.p, st);
    dmt("wr_count+adj");
    // runs and symbols in one packed inclusive scan when the totals fit (as
    // the one-GPU writer), else two
    uint64_t symTotal = 0;
    {
      DBuf<unsigned long long> tot;
      tot.alloc(1);
      size_t b = 0;
      HIPCHK(rocprim::reduce(nullptr, b, sym.p, tot.p, 0ull, (size_t)V, rocprim::plus<unsigned long long>(), st));
      HIPCHK(rocprim::reduce(scratch(b), b, sym.p, tot.p, 0ull, (size_t)V, rocprim::plus<unsigned long long>(), st));
      symTotal = read1(tot.p);
    }
    dm.symPacked = symTotal < (1ull << kPackSymBits) && 3ull * V < (1ull << (64 - kPackSymBits)) &&
                   !env_u32("CMSBWT_WR_TWO_SCANS", 0);
    if (dm.symPacked) {
      inscan(rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint32_t>(0u),
                                              PackAdjSym{adj.p, sym.p}),
             dm.runIn.p, V, rocprim::plus<unsigned long long>());
    } else {
      dm.symIn.alloc(V);
      inscan(rocprim::make_transform_iterator(adj.p, WidenU64()), dm.runIn.p, V, rocprim::plus<unsigned long long>());
      inscan(sym.p, dm.symIn.p, V, rocprim::plus<unsigned long long>());
    }
  }
  dmt("elem_scans");
  mk_dm_el_units(dm.eBase.p, m.p, dm.runIn.p, dm.symPacked ? nullptr : dm.symIn.p, dm.ehl.p, n, dm.E, Uw, out, st);
  HIPCHK(hipGetLastError());
  sync();
  dmt("el_units");
  dmtFlush("dm_units");
}

ElemIn Engine::dm_elem_in() {
  ElemIn ei{dsa.p, dbwt.p, dm.bucket.p, dm.IS.posBegin.p, dm.IS.slot.p, dm.itemOfSlot.p, nullptr, dm.eBase.p,
            dm.rOf.p, nullptr, dm.counter.p, dm.cum.p, dm.info1.p, dm.info2.p, R.n, dm.E, dm.Hp, dm.rle};
  ei.bwtSlot = dm.bwtSlot.p;
  return ei;
}

uint64_t Engine::dm_emit(const int64_t* unitsAll) {
  const uint32_t n = R.n, Uw = dm.Uw;
  dmt(nullptr);
  DBuf<unsigned long long> sym, own, srcOff;
  dm.uruns.alloc(Uw); dm.uhl.alloc(Uw); sym.alloc(Uw); dm.uprev.alloc(Uw);
  mk_dm_units_unpack(unitsAll, Uw, dm.uruns.p, dm.uhl.p, sym.p, st);
  // a unit's first segment continues the previous non-empty unit's run when
  // the characters match (global over all ranks' units)
  exscan(dm.uhl.p, dm.uprev.p, 0u, Uw, LastNonEmpty());
  mk_wr_adjust(dm.uhl.p, dm.uprev.p, Uw, dm.uruns.p, st);
  dm.runOff.alloc(Uw);
  dm.symOff.alloc(Uw);
  auto runs64 = rocprim::make_transform_iterator(dm.uruns.p, WidenU64());
  exscan(runs64, dm.runOff.p, 0ull, Uw);
  exscan(sym.p, dm.symOff.p, 0ull, Uw);
  dm.Rn = sum2(dm.runOff.p + (Uw - 1), dm.uruns.p + (Uw - 1));
  dm.symbols = sum2(dm.symOff.p + (Uw - 1), sym.p + (Uw - 1));
  dmt("unit_scans");
  const ElemIn ei = dm_elem_in();
  if (dm.rank == 0) {
    // rank 0 holds the output: its own runs go straight to their global indices
    dm.gStart.alloc(std::max<uint64_t>(dm.Rn, 1));
    dm.gChar.alloc(std::max<uint64_t>(dm.Rn, 1));
    mk_dm_el_emit(ei, dm.V, dm.runIn.p, dm.symPacked ? nullptr : dm.symIn.p, dm.runOff.p, dm.symOff.p, dm.uprev.p, dm.uhl.p, dm.ehl.p,
                  dm.gStart.p, dm.gChar.p, st, dm.segs.p);
    dm.Rloc = 0;
  } else {
    // this rank's runs, its units in unit order (rank 0 places them)
    own.alloc(Uw);
    srcOff.alloc(Uw);
    mk_dm_own_runs(dm.uruns.p, Uw, dsa.p, dm.E, n, dm.P0, dm.P1, own.p, st);
    exscan(own.p, srcOff.p, 0ull, Uw);
    dm.Rloc = sum2(srcOff.p + (Uw - 1), own.p + (Uw - 1));
    dm.locStart.alloc(std::max<uint64_t>(dm.Rloc, 1));
    dm.locChar.alloc(std::max<uint64_t>(dm.Rloc, 1));
    mk_dm_el_emit(ei, dm.V, dm.runIn.p, dm.symPacked ? nullptr : dm.symIn.p, srcOff.p, dm.symOff.p, dm.uprev.p, dm.uhl.p, dm.ehl.p,
                  dm.locStart.p, dm.locChar.p, st, dm.segs.p);
  }
  HIPCHK(hipGetLastError());
  sync();
  dm.segs.release();
  dmt("emit");
  dmtFlush("dm_emit");
  return dm.Rloc;
}

void Engine::dm_copy_stream(unsigned long long* start, uint8_t* chars) {
  if (dm.Rloc) {
    HIPCHK(hipMemcpyAsync(start, dm.locStart.p, dm.Rloc * 8, hipMemcpyDefault, st));
    HIPCHK(hipMemcpyAsync(chars, dm.locChar.p, dm.Rloc, hipMemcpyDefault, st));
  }
  sync();
}

// rank 0: the other ranks' runs at their global run indices (its own are
// there already), then the records
void Engine::dm_finish(const unsigned long long* const* starts, const uint8_t* const* chars, const uint64_t* counts,
                       const uint64_t* gstats) {
  if (dm.rank != 0) throw InputError{CMSBWT_EARG, "dm_finish runs on rank 0"};
  const uint32_t n = R.n, Uw = dm.Uw, world = dm.world;
  const uint64_t Rn = dm.Rn;
  DBuf<unsigned long long> own, srcOff;
  own.alloc(Uw);
  srcOff.alloc(Uw);
  for (uint32_t k = 0; k < world; k++) {
    if (k == dm.rank) continue;
    mk_dm_own_runs(dm.uruns.p, Uw, dsa.p, dm.E, n, dm.Psplit[k], dm.Psplit[k + 1], own.p, st);
    exscan(own.p, srcOff.p, 0ull, Uw);
    const uint64_t rk = sum2(srcOff.p + (Uw - 1), own.p + (Uw - 1));
    if (rk != counts[k]) throw InputError{CMSBWT_EINPUT, "internal: rank " + std::to_string(k) + " sent " +
                                                             std::to_string(counts[k]) + " runs, expected " +
                                                             std::to_string(rk)};
    if (rk)
      mk_dm_place(dm.uruns.p, dm.runOff.p, srcOff.p, Uw, dsa.p, dm.E, n, dm.Psplit[k], dm.Psplit[k + 1], starts[k],
                  chars[k], dm.gStart.p, dm.gChar.p, st);
  }
  DBuf<unsigned long long>& runStart = dm.gStart;
  DBuf<uint8_t>& runChar = dm.gChar;
  runs.alloc(Rn * 9);
  mk_wr_records(runStart.p, runChar.p, Rn, dm.symbols, runs.p, st);
  HIPCHK(hipGetLastError());
  sync();
  nruns = Rn;
  lastRle = dm.rle;
  merged = true;
  dm.on = true;
  stats.first_rank_to_head = stats.last_rank_to_head = -1;  // head ranks stay on the document ranks
  // gstats: heads, keys, ndocs, chars, bad, good, nothing, violations
  stats.heads = gstats[0];
  stats.keys = gstats[1];
  stats.ndocs = gstats[2];
  stats.chars = gstats[3];
  stats.counter_bad = gstats[4];
  stats.counter_good = gstats[5];
  stats.counter_nothing = gstats[6];
  stats.order_violations = gstats[7];
  stats.current_sum = gstats[0];
  stats.rank = gstats[2] + 2 + (gstats[1] ? gstats[1] - 1 : 0);
  stats.runs = Rn;
  stats.symbols = dm.symbols;
}

}  // namespace cmsbwt
