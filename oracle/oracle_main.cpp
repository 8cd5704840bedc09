// oracle_main.cpp — CLI wrapper around the oracle (TEST INFRASTRUCTURE ONLY).
// Same surface as the reference main.cpp:14-132 ("p:b:o:rh", two-line list
// file) plus "-d <dir>" to dump intermediate arrays for stage parity tests.
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <fstream>

extern "C" int oracle_run(const char*, const char*, const char*, int, unsigned long long,
                          const char*, double*, unsigned long long*);

int main(int argc, char** argv) {
  std::string out, dump;
  int rle = 0;
  unsigned long long prefix = ~0ull;
  int c;
  while ((c = getopt(argc, argv, "p:b:o:rhd:")) != -1) {
    switch (c) {
      case 'p': prefix = strtoull(optarg, 0, 10); break;
      case 'b': break;
      case 'r': rle = 1; break;
      case 'o': out = optarg; break;
      case 'd': dump = optarg; break;
      default: fprintf(stderr, "usage: %s [-p N] [-b GB] [-r] [-o base] [-d dumpdir] list\n", argv[0]); return 255;
    }
  }
  if (optind + 1 != argc) { fprintf(stderr, "Invalid number of arguments\n"); return 255; }
  std::string list = argv[optind];
  if (out.empty()) out = list;
  std::ifstream in(list);
  if (!in) { fprintf(stderr, "Error opening file %s\n", list.c_str()); return 1; }
  std::string ref, coll;
  std::getline(in, ref);
  std::getline(in, coll);
  coll.erase(coll.find_last_not_of(" \n\r\t") + 1);
  if (ref.empty() || coll.empty()) { fprintf(stderr, "Error: empty line in %s\n", list.c_str()); return 1; }
  double t[2] = {0, 0};
  unsigned long long s[10];
  int rc = oracle_run(ref.c_str(), coll.c_str(), out.c_str(), rle, prefix,
                      dump.empty() ? nullptr : dump.c_str(), t, s);
  if (rc == 0)
    printf("oracle: index %.3f s, collection %.3f s, heads %llu, keys %llu, runs %llu\n", t[0], t[1],
           s[0], s[2], s[8]);
  return rc;
}
