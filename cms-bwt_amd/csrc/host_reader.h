// host_reader.h — collection reader with the reference's document semantics.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace cmsbwt {

// Documents as walked by FN:1138-1352: doc k = text[off[k] .. off[k+1]-1),
// every document followed in `text` by the separator byte 0x02.  `sn` is the
// reference's _sn after the pass (FN:223, FN:1272-1274).
struct Collection {
  std::vector<uint8_t> text;    // docs, each + '\x02'
  std::vector<uint64_t> off;    // ndocs+1 entries; off[k+1] = off[k] + len_k + 1
  uint64_t sn = 0;
  uint64_t chars = 0;           // sequence bytes (separators excluded)
  uint64_t ndocs() const { return off.empty() ? 0 : off.size() - 1; }
};

// file_size: ftello of the collection (FN:221-223); prefix = -p.
bool read_collection(const std::string& path, uint64_t prefix, Collection& c, std::string& err);

}  // namespace cmsbwt
