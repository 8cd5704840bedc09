// host_index.cpp — reference index on the host.
//
// north_star keeps the suffix sort of the single reference string on the host;
// libsais is an empty submodule in the reference tree (.gitmodules:1-3), so the
// SA is built here by induced sorting (SA-IS, Nong/Zhang/Chan 2009) written
// from scratch, then ISA, PLCP (Phi method), LCP, the max-neighbour PLCP of
// FN:272-274 and the reference BWT of FN:294-297.  The SA is unique (x ends in
// a unique \0, FN:236-237), so the result equals what libsais produces.
#include "host_index.h"

#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <fstream>

namespace cmsbwt {

namespace {

// Core SA-IS on T[0..n) with T[n-1] the unique smallest symbol 0.
void sais_core(const int32_t* T, int32_t* SA, int32_t n, int32_t K) {
  if (n == 1) { SA[0] = 0; return; }
  std::vector<uint8_t> stype(n);  // 1 = S-type, 0 = L-type
  stype[n - 1] = 1;
  for (int32_t i = n - 2; i >= 0; i--)
    stype[i] = (T[i] < T[i + 1] || (T[i] == T[i + 1] && stype[i + 1])) ? 1 : 0;
  auto lms = [&](int32_t i) { return i > 0 && stype[i] && !stype[i - 1]; };
  std::vector<int32_t> cnt(K, 0), bkt(K);
  for (int32_t i = 0; i < n; i++) cnt[T[i]]++;
  auto ends = [&]() { int32_t s = 0; for (int32_t c = 0; c < K; c++) { s += cnt[c]; bkt[c] = s; } };
  auto starts = [&]() { int32_t s = 0; for (int32_t c = 0; c < K; c++) { bkt[c] = s; s += cnt[c]; } };
  auto induce = [&]() {
    starts();
    for (int32_t i = 0; i < n; i++) {
      int32_t j = SA[i] - 1;
      if (SA[i] > 0 && !stype[j]) SA[bkt[T[j]]++] = j;
    }
    ends();
    for (int32_t i = n - 1; i >= 0; i--) {
      int32_t j = SA[i] - 1;
      if (SA[i] > 0 && stype[j]) SA[--bkt[T[j]]] = j;
    }
  };
  // 1. sort LMS substrings by induction
  std::fill(SA, SA + n, -1);
  ends();
  for (int32_t i = 1; i < n; i++) if (lms(i)) SA[--bkt[T[i]]] = i;
  induce();
  int32_t n1 = 0;
  for (int32_t i = 0; i < n; i++) if (lms(SA[i])) SA[n1++] = SA[i];
  // 2. name LMS substrings, recurse if names are not unique
  std::fill(SA + n1, SA + n, -1);
  int32_t name = 0, prev = -1;
  for (int32_t i = 0; i < n1; i++) {
    int32_t p = SA[i];
    bool diff = prev < 0;
    for (int32_t d = 0; !diff; d++) {
      if (T[p + d] != T[prev + d] || stype[p + d] != stype[prev + d]) diff = true;
      else if (d > 0 && lms(p + d)) break;
    }
    if (diff) { name++; prev = p; }
    SA[n1 + p / 2] = name - 1;
  }
  for (int32_t i = n - 1, j = n - 1; i >= n1; i--) if (SA[i] >= 0) SA[j--] = SA[i];
  int32_t* s1 = SA + n - n1;
  if (name < n1) sais_core(s1, SA, n1, name);
  else for (int32_t i = 0; i < n1; i++) SA[s1[i]] = i;
  // 3. induce the full SA from the sorted LMS suffixes
  ends();
  for (int32_t i = 1, j = 0; i < n; i++) if (lms(i)) s1[j++] = i;
  for (int32_t i = 0; i < n1; i++) SA[i] = s1[SA[i]];
  std::fill(SA + n1, SA + n, -1);
  for (int32_t i = n1 - 1; i >= 0; i--) {
    int32_t j = SA[i];
    SA[i] = -1;
    SA[--bkt[T[j]]] = j;
  }
  induce();
}

}  // namespace

void suffix_array_sais(const int32_t* s, int32_t* sa, int64_t n, int64_t k) {
  if (n <= 0) return;
  std::vector<int32_t> t(n + 1), w(n + 1);
  for (int64_t i = 0; i < n; i++) t[i] = s[i] + 1;
  t[n] = 0;
  sais_core(t.data(), w.data(), (int32_t)(n + 1), (int32_t)(k + 1));
  for (int64_t i = 0; i < n; i++) sa[i] = w[i + 1];
}

bool read_reference(const std::string& path, std::string& x, std::string& err, uint64_t* file_bytes,
                    uint64_t* read_size) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) { err = "Error opening file of base sequence " + path; return false; }
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (file_bytes) *file_bytes = sz > 0 ? (uint64_t)sz : 0;
  if (sz <= 0) { fclose(f); err = "Reference file is empty!"; return false; }
  std::string raw((size_t)sz, '\0');
  size_t got = fread(&raw[0], 1, (size_t)sz, f);
  fclose(f);
  if (got != (size_t)sz) { err = "Error reading " + std::to_string(sz) + " bytes from file " + path; return false; }
  x.clear();
  if (raw[0] == '>') {
    // FN:171-189: getline(...).good() loop; an unterminated last line is
    // dropped, header/blank lines flush the pending sequence.
    x.reserve(raw.size());
    size_t b = 0;
    std::string content;
    while (true) {
      size_t e = raw.find('\n', b);
      if (e == std::string::npos) break;  // good() false: last partial line dropped
      if (e == b || raw[b] == '>') { x += content; content.clear(); }
      else content.append(raw, b, e - b);
      b = e + 1;
    }
    x += content;
  } else {
    x.swap(raw);  // FN:190-199
  }
  if (read_size) *read_size = x.size();
  // FN:208-213
  if (!x.empty() && (x.back() == '\n' || x.back() == '\r' || x.back() == 0)) x.pop_back();
  if (!x.empty() && x.back() == '$') x.pop_back();
  return true;
}

void augment_reference(const std::string& trimmed, HostIndex& ix) {
  std::string& x = ix.x;
  x = trimmed;
  ix.ref_len = trimmed.size();
  // FN:231-237: append absent bytes 3..127, then \1 \0
  // one histogram pass (4 interleaved counters) gives seen[], present[] and
  // the symbol counts of the prefix-rank tables
  uint64_t h4[4][256] = {{0}};
  const unsigned char* p = (const unsigned char*)trimmed.data();
  const size_t L = trimmed.size();
  size_t i = 0;
  for (; i + 4 <= L; i += 4) {
    h4[0][p[i]]++;
    h4[1][p[i + 1]]++;
    h4[2][p[i + 2]]++;
    h4[3][p[i + 3]]++;
  }
  for (; i < L; i++) h4[0][p[i]]++;
  for (int c = 0; c < 256; c++) ix.hist[c] = h4[0][c] + h4[1][c] + h4[2][c] + h4[3][c];
  for (int c = 3; c < 128; c++) if (!ix.hist[c]) x.push_back((char)c);
  x.push_back((char)1);
  x.push_back((char)0);
  ix.n = (uint32_t)x.size();
  for (int c = 0; c < 256; c++) ix.present[c] = ix.hist[c] != 0 || (c >= 3 && c < 128);
}

void build_index(const std::string& trimmed, HostIndex& ix) {
  auto now = [] { return std::chrono::steady_clock::now(); };
  augment_reference(trimmed, ix);
  const std::string& x = ix.x;
  const uint32_t n = ix.n;
  auto t0 = now();
  {
    std::vector<int32_t> s(n);
    for (uint32_t i = 0; i < n; i++) s[i] = (uint8_t)x[i];
    ix.sa.resize(n);
    suffix_array_sais(s.data(), ix.sa.data(), n, 256);
  }
  auto t1 = now();
  ix.isa.resize(n);
  for (uint32_t r = 0; r < n; r++) ix.isa[ix.sa[r]] = r;
  // Phi-method PLCP, then LCP[r] = PLCP[SA[r]] with LCP[0] = 0, LCP[n] = -1
  std::vector<int32_t> plcp(n);
  {
    std::vector<int32_t> phi(n);
    phi[ix.sa[0]] = -1;
    for (uint32_t r = 1; r < n; r++) phi[ix.sa[r]] = ix.sa[r - 1];
    int64_t l = 0;
    const char* s = x.data();
    for (int64_t i = 0; i < (int64_t)n; i++) {
      int64_t j = phi[i];
      if (j < 0) { plcp[i] = 0; l = 0; continue; }
      while (i + l < (int64_t)n && j + l < (int64_t)n && s[i + l] == s[j + l]) l++;
      plcp[i] = (int32_t)l;
      if (l > 0) l--;
    }
  }
  ix.lcp.resize((size_t)n + 1);
  for (uint32_t r = 0; r < n; r++) ix.lcp[r] = plcp[ix.sa[r]];
  ix.lcp[n] = -1;
  ix.plcp.resize(n);
  for (uint32_t i = 0; i < n; i++)
    ix.plcp[i] = std::max(ix.lcp[ix.isa[i]], ix.lcp[(size_t)ix.isa[i] + 1]);
  ix.bwt.resize(n);
  for (uint32_t r = 0; r < n; r++) ix.bwt[r] = ix.sa[r] > 0 ? (uint8_t)x[ix.sa[r] - 1] : 0;
  auto t2 = now();
  ix.t_sa = std::chrono::duration<double>(t1 - t0).count();
  ix.t_lcp = std::chrono::duration<double>(t2 - t1).count();
}

}  // namespace cmsbwt
