// map_replay.h — exact std::map layouts where match.h's comparator is not a
// strict weak order.
//
// MatchInSet::operator< (match.h:27-33) orders smaller=true keys before
// smaller=false keys of another length, but keys of equal length by isaNext
// alone.  When a position holds a smaller=true key of length L whose isaNext
// is not below that of a smaller=false key of length L (possible with bytes
// >= 0x80: FN:55 compares signed chars, the suffix array unsigned ones), the
// relation has cycles and the reference's std::map layout — the order of its
// entries, whether an insertion finds an equal key, where lower_bound lands —
// depends on the insertion history.  The device flags such positions
// (k_check_items) and such queries (k_counter_win<true>); this file replays
// exactly what the reference does there, on the host, with std::map itself:
// the heads of a position inserted in index order (FN:1401-1414: phrases
// sorted by (pos, idx), one insert each), and the lower_bound queries of
// FN:1529-1597 against the replayed maps.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <map>
#include <utility>
#include <vector>

namespace cmsbwt {

// match.h:18-38
struct RefKey {
  uint32_t len;
  bool smaller;
  uint32_t isaNext;
  bool operator==(const RefKey& o) const { return len == o.len && isaNext == o.isaNext; }
  bool operator<(const RefKey& o) const {
    if (len != o.len) return smaller * (len < o.len) + !o.smaller * (len > o.len);
    return isaNext < o.isaNext;
  }
};

// Items of all positions on the host, in the device layout (engine.h ItemSet):
// items in map order, members of item k at P[first[k] .. first[k] + count[k]).
struct HostItems {
  std::vector<uint32_t> pos, len, isa, until, count, first, P;
  std::vector<uint8_t> small;
  std::vector<uint32_t> posBegin;  // n + 1
};

// The members of position p's items as (idx, key, toNext) in insertion order.
struct ReplayHead {
  uint32_t idx;
  RefKey key;
  uint32_t toNext;
};
inline std::vector<ReplayHead> heads_at(const HostItems& I, uint32_t p, const std::vector<uint8_t>& hsmall,
                                        const std::vector<uint32_t>* htonext) {
  std::vector<ReplayHead> v;
  for (uint32_t k = I.posBegin[p]; k < I.posBegin[p + 1]; k++)
    for (uint32_t m = 0; m < I.count[k]; m++) {
      const uint32_t idx = I.P[I.first[k] + m];
      v.push_back(ReplayHead{idx, RefKey{I.len[k], hsmall[idx] != 0, I.isa[k]}, htonext ? (*htonext)[idx] : 0u});
    }
  std::sort(v.begin(), v.end(), [](const ReplayHead& a, const ReplayHead& b) { return a.idx < b.idx; });
  return v;
}

// Rebuild the items of the flagged positions by replaying their insertions
// (FN:1406-1413: the first insertion of a key makes the entry with its
// smaller flag and toNext; a later insertion that finds an equal key only
// appends its idx).  Members of a position occupy one contiguous range of P;
// the rebuilt items reuse it.  K may change (an insertion whose search path
// misses an equal key adds a second entry, as std::map does).
inline void replay_items(HostItems& I, const std::vector<uint8_t>& flagged, const std::vector<uint8_t>& hsmall,
                         const std::vector<uint32_t>& htonext) {
  const uint32_t n = (uint32_t)flagged.size();
  HostItems O;
  O.P = I.P;
  O.posBegin.assign((size_t)n + 1, 0);
  const size_t K0 = I.pos.size();
  for (auto* v : {&O.pos, &O.len, &O.isa, &O.until, &O.count, &O.first}) v->reserve(K0);
  O.small.reserve(K0);
  for (uint32_t p = 0; p < n; p++) {
    O.posBegin[p] = (uint32_t)O.pos.size();
    const uint32_t b = I.posBegin[p], e = I.posBegin[p + 1];
    if (!flagged[p] || b == e) {
      for (uint32_t k = b; k < e; k++) {
        O.pos.push_back(I.pos[k]); O.len.push_back(I.len[k]); O.isa.push_back(I.isa[k]);
        O.until.push_back(I.until[k]); O.count.push_back(I.count[k]); O.first.push_back(I.first[k]);
        O.small.push_back(I.small[k]);
      }
      continue;
    }
    uint32_t base = UINT32_MAX;
    for (uint32_t k = b; k < e; k++) base = std::min(base, I.first[k]);
    const std::vector<ReplayHead> hs = heads_at(I, p, hsmall, &htonext);
    std::map<RefKey, std::pair<uint32_t, std::vector<uint32_t>>> m;  // key -> (toNext, idxs)
    for (const ReplayHead& h : hs) {
      auto ins = m.insert({h.key, {h.toNext, {h.idx}}});
      if (!ins.second) ins.first->second.second.push_back(h.idx);
    }
    uint32_t off = base;
    for (const auto& kv : m) {
      O.pos.push_back(p); O.len.push_back(kv.first.len); O.isa.push_back(kv.first.isaNext);
      O.until.push_back(kv.second.first); O.count.push_back((uint32_t)kv.second.second.size());
      O.first.push_back(off); O.small.push_back(kv.first.smaller ? 1 : 0);
      for (uint32_t idx : kv.second.second) O.P[off++] = idx;
    }
  }
  O.posBegin[n] = (uint32_t)O.pos.size();
  I = std::move(O);
}

// Host answers of counter queries routed off the device: (source slot, target)
// pairs, FN:1529-1597 with std::map::lower_bound on the replayed map of the
// target.  slot: K + 1 entries (prefixSumForPositions), nhr: sorted next-head
// ranks in slot order.  Adds go to (slot, value) pairs.
struct HostQueryOut {
  std::vector<std::pair<uint32_t, uint64_t>> adds;
  uint64_t bad = 0, good = 0;
};
inline HostQueryOut host_queries(const HostItems& I, const std::vector<uint32_t>& slot, const std::vector<uint32_t>& nhr,
                                 const std::vector<uint8_t>& hsmall, std::vector<std::pair<uint32_t, uint32_t>> q,
                                 bool* layoutMismatch) {
  HostQueryOut o;
  *layoutMismatch = false;
  std::sort(q.begin(), q.end(), [](const auto& a, const auto& b) { return a.second < b.second; });
  std::map<RefKey, std::pair<uint32_t, uint32_t>> m;  // key -> (rank within the map (FN:1448), members)
  uint32_t cur = UINT32_MAX;
  for (const auto& pr : q) {
    const uint32_t sq = pr.first, t = pr.second;
    if (t != cur) {  // replay the map of t: heads in index order, as FN:1401-1414
      cur = t;
      m.clear();
      for (const ReplayHead& h : heads_at(I, t, hsmall, nullptr)) m.insert({h.key, {0u, 0u}}).first->second.second++;
      uint32_t r = 0, k = I.posBegin[t];
      for (auto& kv : m) {  // the device items of t must be the map's entries in order
        if (k >= I.posBegin[t + 1] || I.len[k] != kv.first.len || I.isa[k] != kv.first.isaNext ||
            (I.small[k] != 0) != kv.first.smaller || I.count[k] != kv.second.second)
          *layoutMismatch = true;
        kv.second.first = r++;
        k++;
      }
      if (k != I.posBegin[t + 1]) *layoutMismatch = true;
      if (*layoutMismatch) return o;
    }
    const uint32_t qi = (uint32_t)(std::upper_bound(slot.begin(), slot.end() - 1, sq) - slot.begin()) - 1;
    const uint32_t cq = I.count[qi];
    const RefKey toFind{I.len[qi] - 1 - (t - I.pos[qi] - 1), I.small[qi] != 0, I.isa[qi]};  // uint32 wrap, FN:1532
    auto ptr = m.lower_bound(toFind);
    if (ptr == m.end()) continue;  // FN:1535-1536
    const uint32_t tq = I.posBegin[t] + ptr->second.first;
    const uint32_t so = slot[tq], co = I.count[tq];
    const bool hasNext = std::next(ptr) != m.end();
    const uint32_t* me = nhr.data() + sq;
    const uint32_t* ot = nhr.data() + so;
    if (ptr->first == toFind) {  // FN:1537-1589
      if (me[cq - 1] < ot[0]) {
        o.adds.push_back({so, cq});
        o.good++;
      } else if (me[0] > ot[co - 1]) {
        if (hasNext) o.adds.push_back({so + co, cq});
        o.good++;
      } else {
        o.bad++;
        uint32_t a = 0, b = 0;
        while (a < cq && b < co) {
          if (me[a] < ot[b]) {
            o.adds.push_back({so + b, 1});
            a++;
          } else {
            b++;
          }
        }
        if (a < cq && hasNext) o.adds.push_back({so + co, cq - a});
      }
    } else {  // FN:1590-1596
      o.good++;
      o.adds.push_back({so, cq});
    }
  }
  return o;
}

}  // namespace cmsbwt
