// gen_synth — write the SURVEY.md §8(d) synthetic workload as FASTA files.
//
//   gen_synth L C p seed outprefix [width]
//
// Produces <outprefix>.ref.fa, <outprefix>.coll.fa and <outprefix>.list (the
// two-line list file the cmsbwt CLI takes, main.cpp:97-115 of the reference).
// Bytes are a pure function of (L, C, p, seed, width): see synth.h.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "../cms-bwt_amd/csrc/synth.h"

static void write_seq(FILE* f, const std::vector<char>& s, uint64_t width) {
  if (width == 0) {
    fwrite(s.data(), 1, s.size(), f);
    fputc('\n', f);
    return;
  }
  for (uint64_t k = 0; k < s.size(); k += width) {
    uint64_t m = s.size() - k < width ? s.size() - k : width;
    fwrite(s.data() + k, 1, m, f);
    fputc('\n', f);
  }
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s L C p seed outprefix [width]\n", argv[0]);
    return 2;
  }
  uint64_t L = strtoull(argv[1], 0, 10);
  uint64_t C = strtoull(argv[2], 0, 10);
  double p = atof(argv[3]);
  uint64_t seed = strtoull(argv[4], 0, 10);
  std::string pre = argv[5];
  uint64_t width = argc > 6 ? strtoull(argv[6], 0, 10) : 0;
  uint64_t thr = synth_threshold(p);

  std::vector<char> s(L);
  for (uint64_t k = 0; k < L; k++) s[k] = synth_acgt(synth_base_code(seed, k));
  FILE* fr = fopen((pre + ".ref.fa").c_str(), "wb");
  if (!fr) { perror("ref"); return 1; }
  fputs(">ref\n", fr);
  write_seq(fr, s, width);
  fclose(fr);

  FILE* fc = fopen((pre + ".coll.fa").c_str(), "wb");
  if (!fc) { perror("coll"); return 1; }
  std::vector<char> buf(1 << 20);
  setvbuf(fc, buf.data(), _IOFBF, buf.size());
  for (uint64_t c = 1; c <= C; c++) {
    for (uint64_t k = 0; k < L; k++) s[k] = synth_acgt(synth_copy_code(seed, c, k, thr));
    fprintf(fc, ">copy_%llu\n", (unsigned long long)c);
    write_seq(fc, s, width);
  }
  fclose(fc);

  FILE* fl = fopen((pre + ".list").c_str(), "wb");
  if (!fl) { perror("list"); return 1; }
  fprintf(fl, "%s.ref.fa\n%s.coll.fa\n", pre.c_str(), pre.c_str());
  fclose(fl);
  return 0;
}
