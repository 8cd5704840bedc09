// gen_synth — write the SURVEY.md §8(d) synthetic workload as FASTA files.
//
//   gen_synth L C p seed outprefix [width [threads]]
//
// Produces <outprefix>.ref.fa, <outprefix>.coll.fa and <outprefix>.list (the
// two-line list file the cmsbwt CLI takes, main.cpp:97-115 of the reference).
// Bytes are a pure function of (L, C, p, seed, width): see synth.h.  Copies
// are independent, so threads (default: hardware threads, at most 16) each
// format whole copies and pwrite them at their precomputed file offsets; the
// file is the same for any thread count.
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../cms-bwt_amd/csrc/synth.h"

// bytes of one sequence as written: width 0 = one line, otherwise lines of
// `width` symbols, each ended by '\n' (no line at all for an empty sequence)
static uint64_t seq_bytes(uint64_t L, uint64_t width) {
  return width == 0 ? L + 1 : L + (L + width - 1) / width;
}

static void format_seq(char* o, const char* s, uint64_t L, uint64_t width) {
  if (width == 0) {
    memcpy(o, s, L);
    o[L] = '\n';
    return;
  }
  for (uint64_t k = 0; k < L; k += width) {
    const uint64_t m = std::min(width, L - k);
    memcpy(o, s + k, m);
    o[m] = '\n';
    o += m + 1;
  }
}

static bool pwrite_all(int fd, const char* p, uint64_t len, uint64_t off) {
  while (len) {
    ssize_t w = pwrite(fd, p, len, (off_t)off);
    if (w <= 0) return false;
    p += w;
    len -= (uint64_t)w;
    off += (uint64_t)w;
  }
  return true;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s L C p seed outprefix [width [threads]]\n", argv[0]);
    return 2;
  }
  const uint64_t L = strtoull(argv[1], 0, 10);
  const uint64_t C = strtoull(argv[2], 0, 10);
  const double p = atof(argv[3]);
  const uint64_t seed = strtoull(argv[4], 0, 10);
  const std::string pre = argv[5];
  const uint64_t width = argc > 6 ? strtoull(argv[6], 0, 10) : 0;
  unsigned nt = argc > 7 ? (unsigned)atoi(argv[7]) : std::thread::hardware_concurrency();
  nt = std::max(1u, std::min(16u, nt));
  const uint64_t thr = synth_threshold(p);
  const uint64_t sb = seq_bytes(L, width);

  std::vector<char> ref(L), buf(sb + 8);
  for (uint64_t k = 0; k < L; k++) ref[k] = synth_acgt(synth_base_code(seed, k));
  {
    FILE* fr = fopen((pre + ".ref.fa").c_str(), "wb");
    if (!fr) { perror("ref"); return 1; }
    format_seq(buf.data(), ref.data(), L, width);
    fputs(">ref\n", fr);
    fwrite(buf.data(), 1, sb, fr);
    if (fclose(fr) != 0) { perror("ref"); return 1; }
  }

  // copy c starts at sum_{c' < c} (header(c') + sb)
  std::vector<uint64_t> off(C + 2, 0);
  for (uint64_t c = 1; c <= C; c++) off[c + 1] = off[c] + std::to_string(c).size() + 7 + sb;
  int fd = open((pre + ".coll.fa").c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) { perror("coll"); return 1; }
  std::atomic<uint64_t> next{1};
  std::atomic<int> err{0};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++)
    th.emplace_back([&] {
      std::vector<char> s(L), o(sb + 32);
      for (uint64_t c; !err && (c = next++) <= C;) {
        for (uint64_t k = 0; k < L; k++) s[k] = synth_acgt(synth_copy_code(seed, c, k, thr));
        const int h = snprintf(o.data(), 32, ">copy_%llu\n", (unsigned long long)c);
        format_seq(o.data() + h, s.data(), L, width);
        if (!pwrite_all(fd, o.data(), (uint64_t)h + sb, off[c])) err = 1;
      }
    });
  for (auto& t : th) t.join();
  if (err || close(fd) != 0) { perror("coll"); return 1; }

  FILE* fl = fopen((pre + ".list").c_str(), "wb");
  if (!fl) { perror("list"); return 1; }
  fprintf(fl, "%s.ref.fa\n%s.coll.fa\n", pre.c_str(), pre.c_str());
  fclose(fl);
  return 0;
}
