// cmsbwt_oracle.cpp — CPU restatement of the reference CMS-BWT pipeline.
//
// *** TEST INFRASTRUCTURE ONLY. ***  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this.  The product (cms-bwt_amd/,
// libcmsbwt.so, the cmsbwt CLI) never links, calls or executes it.
//
// It restates fmasillo/CMS-BWT (reference @ /root/reference) single-threaded,
// quirks included.  "FN" = CMS-BWT-functions.cpp.
//
//   reference index ........ FN:151-310   (initialize_reference)
//   PSV / NSV on LCP ........ rmq_tree.h:184-225 (exact semantics, own blocks)
//   MS factor + bin. search . FN:11-149
//   collection walk ......... FN:1093-1352 (large ref) / FN:312-559 (small ref)
//   j-scan .................. FN:1359-1385
//   (pos, idx) sort + maps .. FN:1387-1416, match.h:18-55
//   ranks + libsais_int ..... FN:1432-1494
//   prefix sums ............. FN:1504-1515
//   counterSmallerThanHead .. FN:1523-1603 (the small path's -b buffering,
//                             FN:711-906, only reorders commutative += and is
//                             not restated separately)
//   inversion ............... FN:1618-1628
//   .bwt writer ............. FN:1631-1694
//   .rl_bwt writer .......... FN:1695-1777 (remainder quirk at 1761-1770)
//
// libsais is an empty submodule in the reference tree (.gitmodules:1-3,
// SURVEY.md §8c), so the four libsais entry points are replaced by textbook
// algorithms: prefix-doubling suffix sorting (libsais, libsais_int) and the
// Phi method (libsais_plcp, libsais_lcp).  Both inputs end in a unique
// smallest symbol (FN:236-237, FN:1453), so SA/PLCP/LCP are unique and any
// correct algorithm reproduces libsais exactly.
//
// The .phrases spill of the large path (FN:1214-1256) is not restated: every
// spill batch ends at a document end, so the batch j-scan yields the same
// values, and per reference position the map insertion order stays ascending
// idx (the batches are idx-contiguous).
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#include <algorithm>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

namespace orc {

typedef std::chrono::steady_clock clk;
static double secs(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}
static long long msecs(clk::time_point a, clk::time_point b) {
  return (long long)std::chrono::duration_cast<std::chrono::milliseconds>(b - a).count();
}

static const char kSep = (char)2;  // CMS-BWT.h:28 sequenceSeparator

struct Args {  // utils.h:8-14
  std::string filename, outname;
  bool rle = false;
  unsigned buffer = 2;
  uint64_t prefix = UINT64_MAX;
};

// ---------------------------------------------------------------- suffix sort
// Prefix doubling with two stable counting sorts per round.  `rk` holds the
// initial symbol ranks in [0, sigma); on return `sa` is the suffix array.
static void suffix_sort(std::vector<int32_t>& rk, int64_t sigma, std::vector<int32_t>& sa) {
  const int64_t n = (int64_t)rk.size();
  sa.assign(n, 0);
  if (n == 0) return;
  std::vector<int32_t> tmp(n), key2(n);
  std::vector<int64_t> cnt(std::max<int64_t>(sigma, n) + 1);
  // initial sort by symbol
  std::fill(cnt.begin(), cnt.end(), 0);
  for (int64_t i = 0; i < n; i++) cnt[rk[i] + 1]++;
  for (size_t c = 1; c < cnt.size(); c++) cnt[c] += cnt[c - 1];
  for (int64_t i = 0; i < n; i++) sa[cnt[rk[i]]++] = (int32_t)i;
  // dense ranks
  tmp[sa[0]] = 0;
  for (int64_t k = 1; k < n; k++) tmp[sa[k]] = tmp[sa[k - 1]] + (rk[sa[k]] != rk[sa[k - 1]]);
  rk.swap(tmp);
  if (rk[sa[n - 1]] == n - 1) return;
  for (int64_t h = 1;; h <<= 1) {
    // order by second key rk[i+h] (missing = smallest), stable in sa order
    int64_t p = 0;
    for (int64_t i = n - h; i < n; i++) if (i >= 0) tmp[p++] = (int32_t)i;
    for (int64_t k = 0; k < n; k++) if (sa[k] >= h) tmp[p++] = (int32_t)(sa[k] - h);
    // stable counting sort by first key
    std::fill(cnt.begin(), cnt.begin() + n + 1, 0);
    for (int64_t i = 0; i < n; i++) cnt[rk[i] + 1]++;
    for (int64_t c = 1; c <= n; c++) cnt[c] += cnt[c - 1];
    for (int64_t k = 0; k < n; k++) sa[cnt[rk[tmp[k]]]++] = tmp[k];
    for (int64_t i = 0; i < n; i++) key2[i] = i + h < n ? rk[i + h] : -1;
    tmp[sa[0]] = 0;
    for (int64_t k = 1; k < n; k++)
      tmp[sa[k]] = tmp[sa[k - 1]] +
                   (rk[sa[k]] != rk[sa[k - 1]] || key2[sa[k]] != key2[sa[k - 1]]);
    rk.swap(tmp);
    if (rk[sa[n - 1]] == n - 1) break;
  }
}

// ------------------------------------------------------------ PSV / NSV tree
// rmq_tree.h:184-225: psv(i,ub) = max{j <= i : a[j] < ub} or -1,
// nsv(i,ub) = min{j >= i, j < n : a[j] < ub} or -1.  Two levels of block minima.
struct Smaller {
  const int32_t* a = nullptr;
  int64_t n = 0;
  static const int B = 128;
  std::vector<int32_t> m1, m2;  // min per block of B, per block of B*B
  void build(const int32_t* arr, int64_t len) {
    a = arr; n = len;
    m1.assign((n + B - 1) / B, INT32_MAX);
    for (int64_t i = 0; i < n; i++) m1[i / B] = std::min(m1[i / B], a[i]);
    m2.assign((m1.size() + B - 1) / B, INT32_MAX);
    for (size_t i = 0; i < m1.size(); i++) m2[i / B] = std::min(m2[i / B], m1[i]);
  }
  int64_t psv(int64_t i, int32_t ub) const {
    if (i >= n) i = n - 1;
    if (i < 0) return -1;
    int64_t b = i / B;
    for (int64_t j = i; j >= b * B; j--) if (a[j] < ub) return j;
    int64_t c = b - 1;
    // blocks in the same super-block
    for (; c >= 0 && (c + 1) % B != 0; c--) if (m1[c] < ub) goto found;
    for (int64_t s = (c + 1) / B - 1; s >= 0; s--) {
      if (m2[s] < ub) {
        for (c = s * B + B - 1; c >= s * B; c--) if (m1[c] < ub) goto found;
      }
    }
    return -1;
  found:
    for (int64_t j = std::min(n, (c + 1) * B) - 1; j >= c * B; j--) if (a[j] < ub) return j;
    return -1;
  }
  int64_t nsv(int64_t i, int32_t ub) const {
    if (i < 0) i = 0;
    if (i >= n) return -1;
    int64_t b = i / B;
    for (int64_t j = i; j < std::min(n, (b + 1) * B); j++) if (a[j] < ub) return j;
    int64_t c = b + 1;
    int64_t nb = (int64_t)m1.size();
    for (; c < nb && c % B != 0; c++) if (m1[c] < ub) goto found;
    for (int64_t s = c / B; s < (int64_t)m2.size(); s++) {
      if (m2[s] < ub) {
        for (c = s * B; c < std::min(nb, (s + 1) * B); c++) if (m1[c] < ub) goto found;
      }
    }
    return -1;
  found:
    for (int64_t j = c * B; j < std::min(n, (c + 1) * B); j++) if (a[j] < ub) return j;
    return -1;
  }
};

// ------------------------------------------------------------- match records
struct Head {  // match.h:5-16 MatchInVectorBigger
  uint32_t start, pos, len;
  bool smaller;
  uint32_t toNext, idx;
};
struct Key {  // match.h:18-38 MatchInSet
  uint32_t len;
  bool smaller;
  uint32_t isaNext;
  bool operator==(const Key& o) const { return len == o.len && isaNext == o.isaNext; }
  bool operator<(const Key& o) const {  // match.h:27-33, non-strict-weak in general
    if (len != o.len) return (smaller && len < o.len) || (!o.smaller && len > o.len);
    return isaNext < o.isaNext;
  }
};
struct Item {  // match.h:40-55 ItemMatchInSet
  uint32_t untilNext = 0, rank = 0;
  std::vector<uint32_t> idxs;
};
typedef std::map<Key, Item> KeyMap;

// ------------------------------------------------------------------ engine
struct Engine {
  Args arg;
  std::ostream* log = &std::cerr;
  std::string dumpdir;
  // reference globals, CMS-BWT.h:34-53
  std::string x;
  std::vector<int32_t> SA, LCP, PLCP;
  std::vector<uint32_t> ISA;
  std::vector<uint8_t> BWT;
  Smaller rmq;
  uint32_t n = 0;
  uint64_t sn = 0;
  uint64_t D = 1;  // CMS-BWT.h:53
  bool present[256];
  double t_index = 0, t_collection = 0;
  std::string error;

  // ---- FN:151-310
  bool init_reference(const std::string& refFile, const std::string& collFile) {
    auto t1 = clk::now();
    FILE* f = fopen(refFile.c_str(), "r");
    if (!f) { error = "Error opening file of base sequence " + refFile; *log << error << "\n"; return false; }
    *log << "About to read ref\n";
    fseek(f, 0, SEEK_END);
    unsigned int fsz = (unsigned int)ftell(f);
    *log << "n = " << fsz << '\n';
    fseek(f, 0, SEEK_SET);
    if (!fsz) { fclose(f); error = "Reference file is empty!"; *log << error << "\n"; return false; }
    char first = 0;
    if (fread(&first, 1, 1, f) != 1) first = 0;
    if (first == '>') {  // FASTA: FN:171-189
      std::ifstream in(refFile);
      std::string line, content;
      while (std::getline(in, line).good()) {
        if (line.empty() || line[0] == '>') { x += content; content.clear(); }
        else content += line;
      }
      x += content;
    } else {  // raw: FN:190-199
      x.resize(fsz);
      fseek(f, 0, SEEK_SET);
      if (fread(&x[0], 1, fsz, f) != fsz) { fclose(f); error = "Error reading reference"; return false; }
    }
    fclose(f);
    *log << "Reference (size = " << x.size() << "):\n\t";
    auto t01 = clk::now();
    // FN:208-213: strip one trailing \n, \r or \0, then one '$'
    if (!x.empty() && (x.back() == '\n' || x.back() == '\r' || x.back() == 0)) x.pop_back();
    if (!x.empty() && x.back() == '$') x.pop_back();
    // FN:215-226: _sn from the collection file size and -p
    FILE* c = fopen(collFile.c_str(), "r");
    if (!c) { error = "Error opening file of sequence (" + collFile + ")"; *log << error << "\n"; return false; }
    fseek(c, 0, SEEK_END);
    uint64_t csz = (uint64_t)ftello(c);
    *log << "ftello(infile): " << csz << '\n';
    sn = std::min<uint64_t>(csz, arg.prefix);
    *log << "sn: " << sn << '\n';
    fclose(c);
    // FN:231-237: append every absent byte 3..127, then \1 \0
    bool seen[256] = {false};
    for (unsigned char ch : x) seen[ch] = true;
    for (int ch = 3; ch < 128; ch++) if (!seen[ch]) x.push_back((char)ch);
    x.push_back((char)1);
    x.push_back((char)0);
    auto t02 = clk::now();
    *log << "Augmenting reference done in " << msecs(t01, t02) << " ms\n";
    // FN:246-252: suffix array (libsais)
    t01 = clk::now();
    n = (uint32_t)x.size();
    {
      std::vector<int32_t> rk(n);
      for (uint32_t i = 0; i < n; i++) rk[i] = (uint8_t)x[i];
      suffix_sort(rk, 256, SA);
    }
    t02 = clk::now();
    *log << "Computing SA done in " << msecs(t01, t02) << " ms\n";
    // FN:258-268: ISA
    t01 = clk::now();
    ISA.assign(n, 0);
    for (uint32_t r = 0; r < n; r++) ISA[SA[r]] = r;
    t02 = clk::now();
    *log << "\tComputing ISA...\n";
    *log << "Computing ISA done in " << msecs(t01, t02) << " ms\n";
    // FN:270-274: PLCP/LCP (Phi method), LCP[n] = -1, then PLCP := max of neighbour LCPs
    t01 = clk::now();
    PLCP.assign(n, 0);
    LCP.assign((size_t)n + 1, 0);
    {
      std::vector<int32_t> phi(n, -1);
      for (uint32_t r = 1; r < n; r++) phi[SA[r]] = SA[r - 1];
      int64_t l = 0;
      for (int64_t i = 0; i < n; i++) {
        if (phi[i] < 0) { PLCP[i] = 0; l = 0; continue; }
        int64_t j = phi[i];
        while (i + l < n && j + l < n && x[i + l] == x[j + l]) l++;
        PLCP[i] = (int32_t)l;
        if (l > 0) l--;
      }
    }
    for (uint32_t r = 0; r < n; r++) LCP[r] = PLCP[SA[r]];
    LCP[n] = -1;
    for (uint32_t i = 0; i < n; i++) PLCP[i] = std::max(LCP[ISA[i]], LCP[(size_t)ISA[i] + 1]);
    t02 = clk::now();
    *log << "Computing LCP and PLCP done in " << msecs(t01, t02) << " ms\n";
    // FN:281-289: PSV/NSV structure over LCP[0..n-1]
    t01 = clk::now();
    *log << "Computing RMQ...\n";
    rmq.build(LCP.data(), n);
    t02 = clk::now();
    *log << "Computing RMQ done in " << msecs(t01, t02) << " ms\n";
    // FN:291-302: reference BWT
    t01 = clk::now();
    *log << "Computing BWT...\n";
    BWT.assign(n, 0);
    for (uint32_t r = 0; r < n; r++) BWT[r] = SA[r] > 0 ? (uint8_t)x[SA[r] - 1] : 0;
    t02 = clk::now();
    *log << "Computing BWT done in " << msecs(t01, t02) << " ms\n";
    *log << "Finished pre-processing\n";
    *log << "Preprocessing done in " << msecs(t1, clk::now()) << " ms\n";
    for (int ch = 0; ch < 256; ch++) present[ch] = false;
    for (uint32_t i = 0; i + 2 < n; i++) present[(uint8_t)x[i]] = true;
    t_index = secs(t1, clk::now());
    return true;
  }

  // ---- FN:11-25
  std::pair<int, int> adjust(int lo, int hi, int offset) const {
    int p = (int)rmq.psv(lo, offset);
    if (p == -1) p = 0;
    int q = (int)rmq.nsv((int64_t)hi + 1, offset);
    if (q == -1) q = (int)n - 1; else q--;
    return {p, q};
  }
  // ---- FN:34-43
  std::pair<int, int> contract_left(int lo, int hi, int offset) const {
    uint32_t sl = (uint32_t)SA[lo], sh = (uint32_t)SA[hi];
    if (sl == n - 1 || sh == n - 1) return {0, (int)n - 1};
    return adjust((int)ISA[sl + 1], (int)ISA[sh + 1], offset);
  }
  // ---- FN:94-120 (leftmost index in [lo,hi] with x[SA[m]+off]==c, else -(ins+1))
  int32_t bs_left(int32_t lo, int32_t hi, uint32_t off, uint8_t c) const {
    int32_t a = lo, b = hi;
    while (a <= b) {
      int32_t m = (a + b) >> 1;
      uint8_t v = (uint8_t)x[(uint32_t)SA[m] + off];
      if (v < c) a = m + 1;
      else if (v > c) b = m - 1;
      else {
        if (m == lo) return m;
        if ((uint8_t)x[(uint32_t)SA[m - 1] + off] == v) b = m - 1;
        else return m;
      }
    }
    return -(a + 1);
  }
  // ---- FN:123-149
  int32_t bs_right(int32_t lo, int32_t hi, uint32_t off, uint8_t c) const {
    int32_t a = lo, b = hi;
    while (a <= b) {
      int32_t m = (a + b) >> 1;
      uint8_t v = (uint8_t)x[(uint32_t)SA[m] + off];
      if (v < c) a = m + 1;
      else if (v > c) b = m - 1;
      else {
        if (m == hi) return m;
        if ((uint8_t)x[(uint32_t)SA[m + 1] + off] == v) a = m + 1;
        else return m;
      }
    }
    return -(a + 1);
  }
  // ---- FN:45-88
  void ms_factor(const std::string& t, uint64_t i, uint32_t* pos, uint32_t* len,
                 int32_t& lb, int32_t& rb, bool& smaller) const {
    uint32_t off = *len;
    uint64_t j = i + off;
    int32_t nlb = lb, nrb = rb;
    uint32_t match = (uint32_t)SA[nlb];
    while (j < sn) {
      if (nlb == nrb) {
        char r = x[(uint32_t)SA[nlb] + off];
        if (r != t[j]) { smaller = r > t[j]; break; }  // char (signed) compare
        lb = nlb; rb = nrb;
      } else {
        nlb = bs_left(nlb, nrb, off, (uint8_t)t[j]);
        if (nlb < 0) {
          int32_t mm = -nlb - 1;
          smaller = true;
          if (mm == nrb + 1) { mm--; smaller = false; }
          match = (uint32_t)SA[mm];
          break;
        }
        nrb = bs_right(nlb, nrb, off, (uint8_t)t[j]);
        lb = nlb; rb = nrb;
      }
      match = (uint32_t)SA[nlb];
      j++;
      off++;
    }
    *pos = match;
    *len = off;
  }

  // ---- collection state
  std::vector<int64_t> bucket;
  std::vector<uint8_t> listOfChars;
  std::vector<Head> V;
  uint32_t headNumber = 0;
  uint32_t ndoc = 1;

  void bump(uint32_t p, bool head) {  // FN:1162-1171
    int64_t& b = bucket[p];
    if (head) { if (b > 0) b = -b - 1; else b--; }
    else { if (b >= 0) b++; else b--; }
  }
  void end_phrase(uint32_t iCur, char lastChar) {  // FN:1198-1212
    V.push_back(Head{iCur, n - 1, 0, false, 0, headNumber++});
    bucket[n - 1]--;
    ndoc++;
    listOfChars.push_back((uint8_t)lastChar);
  }
  // FN:1139-1212: one document (content already has the separator appended)
  bool walk_document(const std::string& content) {
    D++;
    int64_t i = 0;
    int32_t lb = 0, rb = (int32_t)n - 1;
    bool smaller = false;  // uninitialised in the reference; only read after a write
    uint64_t prevPos = (uint64_t)-2;
    uint32_t pos = n - 1, len = 0, iCur = 0;
    for (int64_t k = 0; k + 1 < (int64_t)content.size(); k++) {
      if (!present[(uint8_t)content[k]]) {
        error = "collection byte " + std::to_string((int)(uint8_t)content[k]) +
                " does not occur in the reference (reference behaviour undefined)";
        return false;
      }
    }
    while (i < (int64_t)content.size() - 1) {
      ms_factor(content, (uint64_t)i, &pos, &len, lb, rb, smaller);
      if ((uint64_t)pos != prevPos + 1) {
        V.push_back(Head{iCur, pos, len, smaller, 0, headNumber++});
        listOfChars.push_back(i == 0 ? (uint8_t)kSep : (uint8_t)content[i - 1]);
        bump(pos, true);
      } else {
        bump(pos, false);
      }
      iCur++;
      len--;
      if (lb == rb) {
        while (len > (uint32_t)PLCP[(size_t)pos + 1]) {  // FN:1176-1185
          i++; iCur++; len--; pos++;
          bump(pos, false);
        }
        auto iv = adjust((int)ISA[(size_t)pos + 1], (int)ISA[(size_t)pos + 1], (int)len);
        lb = iv.first; rb = iv.second;
      } else {
        auto iv = contract_left(lb, rb, (int)len);
        lb = iv.first; rb = iv.second;
      }
      i++;
      prevPos = pos;
    }
    end_phrase(iCur, i == 0 ? kSep : content[content.size() - 2]);
    return true;
  }

  // FN:1093-1352 (+ small path FN:312-559): read and walk the collection.
  bool parse_collection(const std::string& collFile) {
    bucket.assign(n, 0);
    std::ifstream in(collFile, std::ios::in);
    std::string line, content;
    uint64_t charactersRead = 0;
    while (std::getline(in, line).good()) {
      if (line.empty() || line[0] == '>') {
        content += kSep;
        charactersRead++;
        if (!walk_document(content)) return false;
        content.clear();
      } else {
        charactersRead += line.size();
        if (charactersRead >= sn - 1) {  // FN:1259-1262 (-p cut, uint64 wrap kept)
          content += line.substr(0, line.size() - (charactersRead - sn) - 1);
          break;
        }
        content += line;
      }
    }
    if (!content.empty()) {  // FN:1269-1350 tail document
      content += kSep;
      charactersRead++;
      if (charactersRead < sn - 1) sn = charactersRead;
      // The tail loop (FN:1284-1350) restarts at every separator byte inside
      // `content`; the collection bytes are checked to exclude \x02, so the
      // only separator is the final one and the tail walk equals walk_document.
      if (!walk_document(content)) return false;
    }
    return true;
  }

  void dump(const std::string& name, const void* p, size_t bytes) {
    if (dumpdir.empty()) return;
    FILE* f = fopen((dumpdir + "/" + name).c_str(), "wb");
    if (!f) return;
    if (bytes) fwrite(p, 1, bytes, f);
    fclose(f);
  }

  bool process_collection(const std::string& collFile) {
    const bool small = n < 1000000;  // FN:1792
    *log << "File is in memory\n";
    *log << "_x.len: " << n << '\n';
    *log << "_sx.len: " << sn << '\n';
    auto t1 = clk::now();
    *log << "About to start main parsing loop...\n";
    if (!parse_collection(collFile)) { *log << error << "\n"; return false; }
    *log << "Finished parsing file of length: " << sn << "\n";
    const uint64_t H = V.size();
    if (H == 0) {  // FN:1359 `size() - 1` wraps and FN:1385 writes V[-1]: undefined
      error = "collection has no documents (reference behaviour undefined, FN:1359-1385)";
      *log << error << "\n";
      return false;
    }
    if (!dumpdir.empty()) {
      std::vector<uint32_t> st(H);
      for (uint64_t i = 0; i < H; i++) st[i] = V[i].start;
      dump("h_start.u32", st.data(), H * 4);
    }
    // ---- j-scan FN:1359-1385
    std::unordered_map<uint32_t, KeyMap> maps;
    std::vector<uint32_t> keys;
    maps[n - 1];
    keys.push_back(n - 1);
    std::vector<uint16_t> nextHead;
    nextHead.reserve(H);
    uint64_t j = 0;
    for (uint64_t i = 0; i + 1 < H; i++) {
      if (maps.try_emplace(V[i].pos).second) keys.push_back(V[i].pos);
      while (((V[j].start + V[j].len <= V[i].start + V[i].len) & (V[j].len != 0))) j++;
      V[i].toNext = V[i].len > 0 ? V[i + 1].start - V[i].start - 1 : 0;
      uint32_t q = V[j].pos + (V[i].start + V[i].len - V[j].start);
      if (q >= n) { error = "isaNext index out of range (reference UB)"; *log << error << "\n"; return false; }
      V[i].start = ISA[q];
      nextHead.push_back((uint16_t)(j - i));
      if (V[i].len == 0) j++;
    }
    nextHead.push_back(0);
    V[H - 1].start = 0;
    if (!dumpdir.empty()) {
      std::vector<uint32_t> a(H), b(H), c(H), d(H);
      std::vector<uint8_t> s(H);
      for (uint64_t i = 0; i < H; i++) {
        a[i] = V[i].start; b[i] = V[i].pos; c[i] = V[i].len; d[i] = V[i].toNext; s[i] = V[i].smaller;
      }
      dump("h_isa.u32", a.data(), H * 4);
      dump("h_pos.u32", b.data(), H * 4);
      dump("h_len.u32", c.data(), H * 4);
      dump("h_tonext.u32", d.data(), H * 4);
      dump("h_smaller.u8", s.data(), H);
      dump("h_nexthead.u16", nextHead.data(), H * 2);
      dump("h_lchar.u8", listOfChars.data(), H);
      dump("bucket.i64", bucket.data(), (size_t)n * 8);
    }
    // ---- sort by (pos, idx) and insert FN:1387-1416
    std::sort(V.begin(), V.end(), [](const Head& a, const Head& b) {
      return a.pos != b.pos ? a.pos < b.pos : a.idx < b.idx;
    });
    for (const Head& h : V) {
      auto ins = maps[h.pos].insert({Key{h.len, h.smaller, h.start}, Item{}});
      if (ins.second) { ins.first->second.untilNext = h.toNext; ins.first->second.idxs.push_back(h.idx); }
      else ins.first->second.idxs.push_back(h.idx);
    }
    std::vector<Head>().swap(V);
    uint64_t nkeys = 0;
    for (auto& kv : maps) nkeys += kv.second.size();
    *log << "phrasesSet.size(): " << maps.size() << "\n";
    *log << "headNumber: " << headNumber << "\n";
    if (small) *log << "uniqueHeadNumber: " << nkeys << "\n";
    *log << "ndoc: " << ndoc << "\n";
    *log << "docBoundaries.size(): " << D << "\n";
    *log << "Time to compute matching statistics: " << msecs(t1, clk::now()) << " milliseconds\n";
    stat_heads = headNumber; stat_positions = maps.size(); stat_keys = nkeys;

    // ---- ranks FN:1432-1453
    *log << "Going to compute ranks for positions\n";
    auto tr = clk::now();
    std::sort(keys.begin(), keys.end(), [this](uint32_t a, uint32_t b) { return ISA[a] < ISA[b]; });
    int64_t rank = 1;
    std::vector<int32_t> T((size_t)H + 1, 0);
    for (uint32_t p : keys) {
      uint32_t within = 0;
      for (auto& kv : maps[p]) {
        for (uint32_t idx : kv.second.idxs) {
          T[idx] = (int32_t)rank;
          if (p == n - 1) rank++;
        }
        kv.second.rank = within++;
        rank++;
      }
    }
    *log << "Rank: " << rank << "\n";
    stat_rank = rank;
    T[H] = 0;
    dump("rank2head.i32", T.data(), (H + 1) * 4);
    // ---- libsais_int FN:1455-1472
    auto ts = clk::now();
    std::vector<int32_t> SAT;
    {
      std::vector<int32_t> rk(T);
      suffix_sort(rk, rank, SAT);
    }
    *log << "libsais_int ran in " << msecs(ts, clk::now()) << " milliseconds\n";
    dump("head2rank.i32", SAT.data(), (H + 1) * 4);
    std::vector<uint8_t> BWTheads((size_t)H + 1, 0);
    for (uint64_t r = 0; r < H; r++) {
      T[SAT[r + 1]] = (int32_t)r;
      BWTheads[r] = listOfChars[SAT[r + 1]];
    }
    std::vector<uint8_t>().swap(listOfChars);
    std::vector<int32_t>().swap(SAT);
    *log << "First rankToHead: " << T[0] << "\n";
    *log << "Last rankToHead: " << T[H - 1] << "\n";
    dump("bwtheads.u8", BWTheads.data(), H);
    // ---- next-head ranks FN:1480-1494
    for (uint32_t p : keys) {
      for (auto& kv : maps[p]) {
        for (auto& v : kv.second.idxs) v = (uint32_t)T[v + nextHead[v]];
        std::sort(kv.second.idxs.begin(), kv.second.idxs.end());
      }
    }
    std::vector<int32_t>().swap(T);
    std::vector<uint16_t>().swap(nextHead);
    *log << "Done computing ranks for positions in " << msecs(tr, clk::now()) << " milliseconds\n";
    // ---- prefix sums FN:1504-1515
    std::sort(keys.begin(), keys.end());
    std::unordered_map<uint32_t, std::vector<uint64_t>> psum;
    uint64_t cur = 0;
    for (uint32_t p : keys) {
      auto& v = psum[p];
      for (auto& kv : maps[p]) { v.push_back(cur); cur += kv.second.idxs.size(); }
      v.push_back(cur);
    }
    *log << "currentSum: " << cur << "\n";
    // ---- counterSmallerThanHead FN:1523-1603
    *log << "Going to compute counterSmallerThanHead for positions\n";
    auto tc = clk::now();
    uint64_t bad = 0, good = 0, nothing = 0;
    std::vector<uint64_t> counter((size_t)H + 1, 0);
    for (uint32_t p : keys) {
      for (auto it = maps[p].begin(); it != maps[p].end(); ++it) {
        const Item& me = it->second;
        for (uint32_t k = 0; k < me.untilNext; k++) {
          uint32_t t = p + 1 + k;
          if (bucket[t] >= 0) { nothing++; continue; }
          Key want{it->first.len - 1 - k, it->first.smaller, it->first.isaNext};
          KeyMap& there = maps[t];
          auto q = there.lower_bound(want);
          if (q == there.end()) continue;
          const std::vector<uint64_t>& ps = psum[t];
          if (q->first == want) {
            bad++;
            const Item& ot = q->second;
            bool hasNext = std::next(q) != there.end();
            if (me.idxs.back() < ot.idxs.front()) {
              counter[ps[ot.rank]] += me.idxs.size();
              bad--; good++;
              continue;
            }
            if (me.idxs.front() > ot.idxs.back()) {
              if (hasNext) counter[ps[ot.rank + 1]] += me.idxs.size();
              bad--; good++;
              continue;
            }
            uint32_t a = 0, b = 0;
            while (a < me.idxs.size() && b < ot.idxs.size()) {
              if (me.idxs[a] < ot.idxs[b]) { counter[ps[ot.rank] + b]++; a++; }
              else b++;
            }
            if (a < me.idxs.size() && hasNext) counter[ps[ot.rank + 1]] += me.idxs.size() - a;
          } else {
            good++;
            counter[ps[q->second.rank]] += me.idxs.size();
          }
        }
      }
    }
    *log << "counterBad: " << bad << "\n";
    *log << "counterGood: " << good << "\n";
    *log << "counterDoNothing: " << nothing << "\n";
    *log << "Done computing counterSmallerThanHead for positions in " << msecs(tc, clk::now())
         << " milliseconds\n";
    stat_bad = bad; stat_good = good; stat_nothing = nothing; stat_currentSum = cur;
    dump("counters.u64", counter.data(), (H + 1) * 8);
    if (small) {  // FN:919-924
      std::ofstream o(arg.outname + ".counterSmallerThanHead_true", std::ios::out | std::ios::binary);
      o.write((const char*)counter.data(), (std::streamsize)((H + 1) * 8));
    }
    // per-position item list sizes (for the writers)
    std::unordered_map<uint32_t, std::vector<uint64_t>>& PS = psum;
    maps.clear();
    // ---- inversion FN:1618-1628
    {
      std::vector<int64_t> cp(bucket);
      for (uint32_t i = 0; i < n; i++) bucket[ISA[i]] = cp[i];
    }
    *log << "Inverted data in bucketsForExpandedBWT\n";
    if (!arg.rle) write_plain(BWTheads, counter, PS);
    else write_rle(BWTheads, counter, PS);
    t_collection = secs(t1, clk::now());
    return true;
  }

  // ---- FN:1631-1694
  void write_plain(const std::vector<uint8_t>& BWTheads, const std::vector<uint64_t>& counter,
                   std::unordered_map<uint32_t, std::vector<uint64_t>>& PS) {
    std::ofstream o(arg.outname + ".bwt", std::ios::out | std::ios::binary);
    std::string buf;
    buf.reserve(1 << 20);
    auto put = [&](uint8_t c) {
      buf.push_back((char)c);
      if (buf.size() == (1 << 20)) { o.write(buf.data(), buf.size()); buf.clear(); }
    };
    for (uint64_t d = 0; d + 1 < D; d++) put(BWTheads[d]);
    uint64_t hc = D - 1;
    for (uint32_t r = 1; r < n; r++) {
      uint8_t c = BWT[r];
      int64_t& b = bucket[r];
      if (b >= 0) {
        for (int64_t k = 0; k < b; k++) put(c);
      } else {
        const std::vector<uint64_t>& ps = PS[(uint32_t)SA[r]];
        for (size_t s = 0; s + 1 < ps.size(); s++) {
          for (uint64_t slot = ps[s]; slot < ps[s + 1]; slot++) {
            for (uint64_t k = 0; k < counter[slot]; k++) { put(c); b++; }
            put(BWTheads[hc++]);
            b++;
          }
        }
        for (int64_t k = b; k < 0; k++) put(c);
      }
    }
    if (!buf.empty()) o.write(buf.data(), buf.size());
  }

  // ---- FN:1695-1777 (including the per-item remainder quirk, FN:1761-1770)
  void write_rle(const std::vector<uint8_t>& BWTheads, const std::vector<uint64_t>& counter,
                 std::unordered_map<uint32_t, std::vector<uint64_t>>& PS) {
    std::ofstream o(arg.outname + ".rl_bwt", std::ios::out | std::ios::binary);
    uint8_t prev = 0;
    uint64_t run = 0;
    auto emit = [&]() {
      o.write((const char*)&run, 8);
      o.write((const char*)&prev, 1);
      stat_runs++;
    };
    for (uint64_t d = 0; d + 1 < D; d++) {
      if (prev != BWTheads[d]) {
        if (run > 0) emit();
        run = 1;
        prev = BWTheads[d];
      } else {
        run++;
      }
    }
    uint64_t hc = D - 1;
    auto add = [&](uint8_t c, uint64_t k) {
      if (prev != c) { emit(); run = k; prev = c; }
      else run += k;
    };
    for (uint32_t r = 1; r < n; r++) {
      uint8_t c = BWT[r];
      int64_t& b = bucket[r];
      if (b > 0) {
        add(c, (uint64_t)b);
      } else if (b < 0) {
        const std::vector<uint64_t>& ps = PS[(uint32_t)SA[r]];
        for (size_t s = 0; s + 1 < ps.size(); s++) {
          for (uint64_t slot = ps[s]; slot < ps[s + 1]; slot++) {
            if (counter[slot]) { add(c, counter[slot]); b += (int64_t)counter[slot]; }
            add(BWTheads[hc++], 1);
            b++;
          }
          if (b != 0) add(c, (uint64_t)(-b));  // quirk: inside the per-item loop
        }
      }
    }
    emit();
  }

  uint64_t stat_heads = 0, stat_positions = 0, stat_keys = 0, stat_bad = 0, stat_good = 0,
           stat_nothing = 0, stat_currentSum = 0, stat_runs = 0;
  int64_t stat_rank = 0;
};

}  // namespace orc

extern "C" {

// Full run on files.  Returns 0 on success, 1 on an error the reference would
// exit(1) on, 3 on reference-undefined input.  times[0] = reference index
// seconds, times[1] = collection seconds (parse .. output closed).
// stats (may be null) receives {H, positions, keys, rank, currentSum, bad,
// good, nothing, runs, D}.
int oracle_run(const char* ref_path, const char* coll_path, const char* outname, int rle,
               unsigned long long prefix, const char* dump_dir, double* times,
               unsigned long long* stats) {
  orc::Engine e;
  e.arg.outname = outname;
  e.arg.rle = rle != 0;
  e.arg.prefix = prefix;
  if (dump_dir) e.dumpdir = dump_dir;
  std::ofstream logf(std::string(outname) + ".log");
  e.log = &logf;
  if (!e.init_reference(ref_path, coll_path)) return 1;
  if (!e.process_collection(coll_path)) return e.error.rfind("Error", 0) == 0 ? 1 : 3;
  if (times) { times[0] = e.t_index; times[1] = e.t_collection; }
  if (stats) {
    unsigned long long s[10] = {e.stat_heads, e.stat_positions, e.stat_keys,
                                (unsigned long long)e.stat_rank, e.stat_currentSum, e.stat_bad,
                                e.stat_good, e.stat_nothing, e.stat_runs, e.D};
    memcpy(stats, s, sizeof(s));
  }
  return 0;
}

}  // extern "C"
