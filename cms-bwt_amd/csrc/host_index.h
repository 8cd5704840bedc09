// host_index.h — reference index built on the host.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace cmsbwt {

struct HostIndex {
  std::string x;               // augmented reference, FN:231-237
  uint32_t n = 0;              // _n
  uint64_t ref_len = 0;        // trimmed reference length before augmentation
  std::vector<int32_t> sa;     // _SA
  std::vector<uint32_t> isa;   // _ISA
  std::vector<int32_t> lcp;    // _LCP, n+1 entries, lcp[0]=0, lcp[n]=-1
  std::vector<int32_t> plcp;   // _PLCP after the max-neighbour redefinition (FN:272-274)
  std::vector<uint8_t> bwt;    // _BWT
  bool present[256];           // bytes occurring in x[0..n-3] (collection check)
  uint64_t hist[256];          // byte counts of the trimmed reference
  double t_sa = 0, t_lcp = 0;  // SA; everything after it (walk tables included)
  // stages of the reference's log (FN:240-299); device build only
  double t_augment = 0, t_isa = 0, t_lcp_only = 0, t_rmq = 0, t_bwt = 0;
  uint64_t file_bytes = 0, read_size = 0;  // FN:166 `n = `, FN:205 `Reference (size = `
};

// Suffix array of s[0..n) over alphabet [0, k) with the "end of string is
// smallest" convention (same as libsais).  Induced sorting (SA-IS).
void suffix_array_sais(const int32_t* s, int32_t* sa, int64_t n, int64_t k);

// FN:155-213: read FASTA (first byte '>') or raw reference, trim.
bool read_reference(const std::string& path, std::string& x, std::string& err, uint64_t* file_bytes = nullptr,
                    uint64_t* read_size = nullptr);
// FN:231-237: x = trimmed + absent bytes 3..127 + \1 \0; n, ref_len, present.
void augment_reference(const std::string& trimmed, HostIndex& ix);
// FN:231-297 on an already-read+trimmed sequence.
void build_index(const std::string& trimmed, HostIndex& ix);

}  // namespace cmsbwt
