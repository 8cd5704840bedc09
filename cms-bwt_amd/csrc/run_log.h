// run_log.h — the reference's .log of one run, shared by
// the one-GPU cmsbwt_run (engine.hip) and the in-process multi-GPU run
// (multi.hip).  Keys and their order follow initialize_reference
// (FN:161-309) and the large / small collection pass (FN:1094-1627,
// FN:312-936).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <ostream>

#include "../../include/cmsbwt.h"

namespace cmsbwt {

// FN:161-309, from `n = ` to `Preprocessing done in`.  sn0 = collection file
// size (~0 when it cannot be opened: the reference's error line is written
// and true returned, the caller exits with EIO, FN:216-219).
inline bool log_reference(std::ostream& log, const cmsbwt_stats& s, uint64_t sn0, uint64_t prefix,
                          const char* coll_path, long long preprocMs) {
  log << "n = " << s.ref_file_bytes << '\n';
  log << "Reference (size = " << s.ref_read_size << "):\n\t";
  if (sn0 == ~0ull) {
    log << "Error opening file of sequence (" << coll_path << ")\n";
    return true;
  }
  log << "ftello(infile): " << sn0 << '\n';
  log << "sn: " << std::min<uint64_t>(sn0, prefix) << '\n';
  log << "Augmenting reference done in " << (long long)s.t_augment_ms << " ms\n";
  log << "Computing SA done in " << (long long)s.t_sa_ms << " ms\n";
  log << "\tComputing ISA..." << '\n';
  log << "Computing ISA done in " << (long long)s.t_isa_ms << " ms\n";
  log << "Computing LCP and PLCP done in " << (long long)s.t_lcp_ms << " ms\n";
  log << "Computing RMQ...\n";
  log << "Computing RMQ done in " << (long long)s.t_rmq_ms << " ms\n";
  log << "Computing BWT...\n";
  log << "Computing BWT done in " << (long long)s.t_bwt_ms << " ms\n";
  log << "Finished pre-processing\n";
  log << "Preprocessing done in " << preprocMs << " ms\n";
  return false;
}

// FN:1094-1097 (before the document loop)
inline void log_collection_start(std::ostream& log, const cmsbwt_stats& s, uint64_t xlen) {
  log << "File is in memory\n";
  log << "_x.len: " << xlen << '\n';
  log << "_sx.len: " << s.sn_initial << '\n';
  log << "About to start main parsing loop...\n";
}

// The in-process multi-GPU run of cmsbwt_run (multi.hip).
int run_multi(const cmsbwt_args* a, const char* ref_path, const char* coll_path, cmsbwt_stats* stats_out);

// FN:1417-1627 (after the merge): small = the small-reference path
// (FN:1792, _n < 1e6), sn = the final _sn, buffer_gb = -b.
inline void log_collection_end(std::ostream& log, const cmsbwt_stats& s, bool small, uint64_t sn,
                               uint32_t buffer_gb) {
  if (!small) log << "phrasesSet.size(): " << s.positions << "\n";
  log << "headNumber: " << s.heads << "\n";
  if (small) log << "uniqueHeadNumber: " << s.keys << "\n";
  log << "ndoc: " << s.ndocs + 1 << "\n";
  log << "docBoundaries.size(): " << s.ndocs + 1 << "\n";
  log << "Time to compute matching statistics: " << (long long)(s.t_ms_walk_s * 1000) << " milliseconds\n";
  log << "Going to compute ranks for positions\n";
  if (!small) log << "Rank: " << s.rank << "\n";
  log << "libsais_int ran in " << (long long)s.t_libsais_int_ms << " milliseconds\n";
  log << "First rankToHead: " << s.first_rank_to_head << "\n";
  log << "Last rankToHead: " << s.last_rank_to_head << "\n";
  log << "Done computing ranks for positions in " << (long long)s.t_ranks_ms << " milliseconds\n";
  log << "currentSum: " << s.current_sum << "\n";
  log << "Going to compute counterSmallerThanHead for positions\n";
  if (small) {  // FN:713-727: the -b buffer of the small path (unsigned int GB * 2^30, wrapping)
    const uint32_t cap32 = buffer_gb * 1073741824u;
    const double ram = sn < (uint64_t)cap32 ? (double)sn : (double)cap32;
    log << "capOfBufferSuffixes = " << (uint64_t)(ram / 20.0 + 1) << "\n";
  }
  log << "counterBad: " << s.counter_bad << "\n";
  log << "counterGood: " << s.counter_good << "\n";
  log << "counterDoNothing: " << s.counter_nothing << "\n";
  log << "Done computing counterSmallerThanHead for positions in " << (long long)s.t_counter_ms
      << " milliseconds\n";
  log << "Inverted data in bucketsForExpandedBWT\n";
}

}  // namespace cmsbwt
