// memo_check.cpp -- host replica of the walk's alignment-memo search
// (ms_walk2.hip, cooperative refill loop): for one slot of 16 threads x 4
// pieces of 16 bytes (piece j of thread k at byte 16 (k + 16 j)), the first
// mismatch and the NEXT one (or the clean end of the round) from per-thread
// first / second differences and per-piece ballots, against brute force on
// random byte strings.  Built and run by tests/test_host.py.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
struct u4 { uint32_t x, y, z, w; };
static void diff16x2(const u4& x, const u4& t, uint32_t& m1, uint32_t& c1, uint32_t& m2, uint32_t& c2) {
  const uint64_t x0 = x.x | ((uint64_t)x.y << 32), x1 = x.z | ((uint64_t)x.w << 32);
  const uint64_t t0 = t.x | ((uint64_t)t.y << 32), t1 = t.z | ((uint64_t)t.w << 32);
  uint64_t d0 = x0 ^ t0, d1 = x1 ^ t1;
  m1 = m2 = 16; c1 = c2 = 0;
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
int main() {
  std::mt19937 rng(1);
  int bad = 0;
  for (int it = 0; it < 200000; it++) {
    uint8_t X[1024], T[1024];
    for (int b = 0; b < 1024; b++) X[b] = T[b] = rng() & 3;
    int nm = rng() % 5;
    for (int k = 0; k < nm; k++) { int p = rng() % 1024; T[p] = (X[p] + 1 + rng() % 3) & 3; }
    // threads k=0..15, pieces j=0..3 at byte 16*(k + 16j)
    uint32_t mine[64], mj[64], cc[64], pm[64], mine2[64], cc2[64];
    for (int k = 0; k < 16; k++) {
      mine[k] = 16; mj[k] = 0; cc[k] = 0; pm[k] = 0; mine2[k] = 16; cc2[k] = 0;
      for (int j = 3; j >= 0; j--) {
        u4 xv, tv; memcpy(&xv, X + 16 * (k + 16 * j), 16); memcpy(&tv, T + 16 * (k + 16 * j), 16);
        uint32_t m1, c1, m2, c2; diff16x2(xv, tv, m1, c1, m2, c2);
        if (m1 < 16) { mine[k] = m1; mj[k] = j; cc[k] = c1; mine2[k] = m2; cc2[k] = c2; pm[k] |= 1u << j; }
      }
    }
    uint64_t mask[4], anyM[4];
    for (int j = 0; j < 4; j++) { mask[j] = anyM[j] = 0; for (int k = 0; k < 16; k++) { if (mine[k] < 16 && mj[k] == (uint32_t)j) mask[j] |= 1ull << k; if ((pm[k] >> j) & 1) anyM[j] |= 1ull << k; } }
    const uint64_t sm = 0xffff; const uint32_t q = 0, rq = 0;
    // true mismatches
    int tm1 = -1, tm2 = -1;
    for (int b = 0; b < 1024; b++) if (X[b] != T[b]) { if (tm1 < 0) tm1 = b; else if (tm2 < 0) { tm2 = b; } }
    bool found = false;
    for (uint32_t j = 0; j < 4 && !found; j++) {
      const uint64_t hit = mask[j] & sm;
      if (!hit) continue;
      found = true;
      const uint32_t f = __builtin_ctzll(hit);
      const uint32_t off1 = rq + 16 * ((f - (q << 4)) + (j << 4)) + mine[f];
      uint32_t off2 = rq + 1024, c2b = 0;
      const uint32_t m2f = mine2[f], c2f = cc2[f];
      if (m2f < 16) { off2 = rq + 16 * ((f - (q << 4)) + (j << 4)) + m2f; c2b = c2f | 0x10000; }
      else {
        uint32_t j2 = j, f2 = 64;
        const uint64_t later = anyM[j] & sm & ~((2ull << f) - 1);
        if (later) f2 = __builtin_ctzll(later);
        else for (uint32_t jj = 0; jj < 4; jj++) if (jj > j && f2 == 64 && (anyM[jj] & sm)) { j2 = jj; f2 = __builtin_ctzll(anyM[jj] & sm); }
        if (f2 == f) off2 = rq + 16 * ((f - (q << 4)) + (j2 << 4));
        else if (f2 < 64) { off2 = rq + 16 * ((f2 - (q << 4)) + (j2 << 4)) + mine[f2]; c2b = cc[f2] | 0x10000; }
      }
      if ((int)off1 != tm1) { bad++; if (bad < 5) printf("off1 %u vs %d\n", off1, tm1); }
      if (c2b & 0x10000) {
        if ((int)off2 != tm2) { bad++; if (bad < 10) printf("it %d off2 %u vs true %d\n", it, off2, tm2); }
        else if ((c2b & 0xff) != X[off2] || ((c2b >> 8) & 0xff) != T[off2]) { bad++; if (bad < 10) printf("chars\n"); }
      } else {
        if (tm2 >= 0 && tm2 < (int)off2) { bad++; if (bad < 10) printf("it %d clean to %u but mismatch at %d\n", it, off2, tm2); }
      }
    }
    if (!found && tm1 >= 0) { bad++; printf("missed\n"); }
  }
  printf("bad %d\n", bad);
  return bad != 0;
}
