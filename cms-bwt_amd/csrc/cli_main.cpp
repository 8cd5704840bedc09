// cli_main.cpp — the `cmsbwt` command, a drop-in for the reference's
// main.cpp:14-132: same getopt surface ("p:b:o:rh"), same two-line list file,
// same outputs (<base>.rl_bwt | <base>.bwt, <base>.log, and
// <base>.counterSmallerThanHead_true for references below 1e6 symbols).
// Extra flags: -g <device> selects the HIP device (rank 0's with -n),
// -n <gpus> runs on that many GPUs in this process (SURVEY.md §8(b) n_gpus;
// ranks wrap over the devices, so -n 4 on one GPU runs four ranks on it),
// -t peer|rccl picks the multi-GPU transport, -v prints stage times.
#include <getopt.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>
#include <fstream>
#include <iostream>
#include <string>

#include "../../include/cmsbwt.h"

static void print_help(char** argv) {  // main.cpp:14-24
  std::cout << "Usage: " << argv[0] << " [options] <input filename>" << std::endl;
  std::cout << "<input filename> is the name of the file containing paths to the reference sequence (in the "
               "first line) and to the collection file (in the second line)."
            << std::endl;
  std::cout << "  Options: " << std::endl
            << "\t-p \tread only a prefix of the file expressed in number of characters, def. whole file"
            << std::endl
            << "\t-b \tsize for the additional memory buffer in GB, def. 2 " << std::endl
            << "\t-r \toutputs the run-length encoded BWT, def. false " << std::endl
            << "\t-o \tbasename for the output files, def. <input filename>" << std::endl
            << "\t-g \tHIP device ordinal, def. 0" << std::endl
            << "\t-n \tnumber of GPUs (ranks in this process), def. 1" << std::endl
            << "\t-t \tmulti-GPU transport: peer (HBM pulls over xGMI) or rccl, def. peer" << std::endl
            << "\t-v \tprint stage timings" << std::endl
            << "\t-h \tprints this help" << std::endl;
  exit(-1);
}

int main(int argc, char** argv) {
  const auto t0 = std::chrono::steady_clock::now();
  std::string filename, outname;
  unsigned long long prefix = UINT64_MAX;
  unsigned buffer = 2;
  int rle = 0, device = 0, verbose = 0, ngpus = 1, backend = CMSBWT_BACKEND_PEER;
  puts("==== Command line:");
  for (int i = 0; i < argc; i++) printf(" %s", argv[i]);
  puts("");
  int c;
  while ((c = getopt(argc, argv, "p:b:o:rhg:vn:t:")) != -1) {
    switch (c) {
      case 'p': prefix = strtoull(optarg, nullptr, 10); break;
      case 'b': buffer = (unsigned)atoi(optarg); break;
      case 'r': rle = 1; break;
      case 'o': outname = optarg; break;
      case 'g': device = atoi(optarg); break;
      case 'v': verbose = 1; break;
      case 'n': ngpus = atoi(optarg); break;
      case 't':
        if (std::string(optarg) == "rccl") backend = CMSBWT_BACKEND_RCCL;
        else if (std::string(optarg) == "peer") backend = CMSBWT_BACKEND_PEER;
        else { std::cout << "Unknown transport " << optarg << ". Use -h for help." << std::endl; exit(-1); }
        break;
      case 'h': print_help(argv); break;
      default: std::cout << "Unknown option. Use -h for help." << std::endl; exit(-1);
    }
  }
  if (argc == optind + 1) filename = argv[optind];
  else { std::cout << "Invalid number of arguments" << std::endl; print_help(argv); }
  if (outname.empty()) outname = filename;
  if (ngpus < 1 || ngpus > 64) { std::cout << "Invalid number of GPUs " << ngpus << std::endl; exit(-1); }
  std::cout << "==== Parameters:" << std::endl;
  std::cout << "Input file: " << filename << std::endl;
  std::cout << "Output basename: " << outname << std::endl;
  std::cout << "Prefix length: " << prefix << std::endl;
  std::cout << "Buffer size: " << buffer << " GB" << std::endl;
  std::cout << "Output format: " << (rle ? "RLE" : "FULL") << std::endl;
  std::cout << std::endl;

  std::ifstream in(filename);  // main.cpp:90-115
  if (!in) { fprintf(stderr, "Error opening file %s\n", filename.c_str()); exit(1); }
  std::string line;
  std::getline(in, line);
  if (line.empty()) { fprintf(stderr, "Error: first line of file %s is empty\n", filename.c_str()); exit(1); }
  std::string ref = line;
  std::getline(in, line);
  if (line.empty()) { fprintf(stderr, "Error: second line of file %s is empty\n", filename.c_str()); exit(1); }
  std::string coll = line;
  coll.erase(coll.find_last_not_of(" \n\r\t") + 1);
  if (coll.empty()) { fprintf(stderr, "Error: second line of file %s is empty\n", filename.c_str()); exit(1); }

  auto t1 = std::chrono::steady_clock::now();
  std::cout << "==== CMS-BWT" << std::endl;
  std::cout << "==== For more information about the execution, please check the log file: " << outname + ".log"
            << std::endl;
  std::cout << "==== Processing reference sequence" << std::endl;
  cmsbwt_args a{prefix, buffer, rle, outname.c_str(), device, verbose, ngpus, backend};
  cmsbwt_stats s{};
  int rc = cmsbwt_run_sized(&a, sizeof a, ref.c_str(), coll.c_str(), &s, sizeof s);
  if (rc != CMSBWT_OK) {
    fprintf(stderr, "cmsbwt: failed with code %d (see %s.log)\n", rc, outname.c_str());
    return rc == CMSBWT_EIO ? 1 : 2 + rc;
  }
  std::cout << "==== Processing collection" << std::endl;
  auto t2 = std::chrono::steady_clock::now();
  std::cout << "==== Time elapsed: " << std::chrono::duration_cast<std::chrono::milliseconds>(t2 - t1).count()
            << " ms" << std::endl;
  if (verbose)
    fprintf(stderr, "cli: main to run %.3fs, run %.3fs\n", std::chrono::duration<double>(t1 - t0).count(),
            std::chrono::duration<double>(t2 - t1).count());
  return 0;
}
