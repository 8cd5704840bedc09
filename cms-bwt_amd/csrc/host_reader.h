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

// Byte-range shards of the collection for `world` ranks: rank k reads
// [bounds[k], bounds[k+1]) and walks the documents closed inside it (plus the
// tail document for the last rank).  bounds[k] is the first byte after the
// last document-ending line (empty or '>', newline-terminated; FN:1138-1139)
// that starts before k * size / world, so every slice begins at a document
// start and reading the slices in rank order gives the documents of the
// whole file, in order (no -p: its cut depends on the bytes before it).
bool shard_bounds(const std::string& path, uint32_t world, std::vector<uint64_t>& bounds, uint64_t& fsz,
                  std::string& err);
// bounds[k] for B = k * size / world (~0 on a read error)
uint64_t shard_start(int fd, uint64_t fsz, uint64_t B);

}  // namespace cmsbwt
