// host_reader.cpp — collection reader.
//
// Same document boundaries as the reference's std::getline(...).good() loop
// (FN:1138-1267) and its tail document (FN:1269-1275), on one buffered pass:
//   * a line is used only if '\n'-terminated (an unterminated last line makes
//     good() false and is dropped);
//   * an empty line or a line starting with '>' ends the current document
//     (possibly empty: a leading '>' yields an empty first document);
//   * -p: once charactersRead >= _sn-1 the line is cut to
//     size - (charactersRead - _sn) - 1 bytes (uint64 wrap kept) and reading
//     stops; the pending content becomes the tail document.
#include "host_reader.h"

#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>

namespace cmsbwt {

bool read_collection(const std::string& path, uint64_t prefix, Collection& c, std::string& err) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) { err = "Error opening file of sequence (" + path + ")"; return false; }
  fseeko(f, 0, SEEK_END);
  uint64_t fsz = (uint64_t)ftello(f);
  fseeko(f, 0, SEEK_SET);
  uint64_t sn = std::min<uint64_t>(fsz, prefix);
  c.text.clear();
  c.off.assign(1, 0);
  c.text.reserve(fsz + 64);
  const char sep = 2;
  uint64_t charactersRead = 0;
  uint64_t docBegin = 0;  // offset in c.text of the pending document
  bool stop = false;

  const size_t CH = 1 << 24;
  std::vector<char> buf(CH);
  std::string partial;  // carried line fragment across buffer refills
  auto handle_line = [&](const char* s, size_t len) {
    if (len == 0 || s[0] == '>') {
      c.text.push_back(sep);
      charactersRead++;
      c.off.push_back(c.text.size());
      docBegin = c.text.size();
      return;
    }
    charactersRead += len;
    if (charactersRead >= sn - 1) {
      uint64_t take = (uint64_t)len - (charactersRead - sn) - 1;
      if (take > len) take = len;
      c.text.insert(c.text.end(), s, s + take);
      stop = true;
      return;
    }
    c.text.insert(c.text.end(), s, s + len);
  };
  while (!stop) {
    size_t got = fread(buf.data(), 1, CH, f);
    if (got == 0) break;
    size_t b = 0;
    while (b < got && !stop) {
      const char* nl = (const char*)memchr(buf.data() + b, '\n', got - b);
      if (!nl) { partial.append(buf.data() + b, got - b); b = got; break; }
      size_t e = (size_t)(nl - buf.data());
      if (!partial.empty()) {
        partial.append(buf.data() + b, e - b);
        handle_line(partial.data(), partial.size());
        partial.clear();
      } else {
        handle_line(buf.data() + b, e - b);
      }
      b = e + 1;
    }
  }
  fclose(f);
  // trailing fragment without '\n' is dropped (getline(...).good() == false)
  if (c.text.size() > docBegin) {  // tail document, FN:1269-1275
    c.text.push_back(sep);
    charactersRead++;
    if (charactersRead < sn - 1) sn = charactersRead;
    c.off.push_back(c.text.size());
  }
  c.sn = sn;
  c.chars = c.text.size() - c.ndocs();
  return true;
}

}  // namespace cmsbwt

// ---- byte-range sharding of the collection file (one rank per GPU)
namespace cmsbwt {

static bool pread_all(int fd, uint8_t* buf, uint64_t len, uint64_t off) {
  while (len) {
    const ssize_t r = pread(fd, buf, len, (off_t)off);
    if (r <= 0) return false;
    buf += r;
    len -= (uint64_t)r;
    off += (uint64_t)r;
  }
  return true;
}

// First byte after the '\n' that ends the line starting at s, or ~0 when the
// line is not terminated (getline().good() drops it, FN:1138).
static uint64_t line_end(int fd, uint64_t fsz, uint64_t s) {
  std::vector<uint8_t> buf(1 << 20);
  for (uint64_t at = s; at < fsz;) {
    const uint64_t len = std::min<uint64_t>(buf.size(), fsz - at);
    if (!pread_all(fd, buf.data(), len, at)) return ~0ull;
    const void* nl = memchr(buf.data(), '\n', len);
    if (nl) return at + (uint64_t)((const uint8_t*)nl - buf.data()) + 1;
    at += len;
  }
  return ~0ull;
}

uint64_t shard_start(int fd, uint64_t fsz, uint64_t B) {
  if (B == 0) return 0;
  if (B >= fsz) return fsz;
  // backwards from B in windows: the last line start s < B whose line ends a
  // document (empty or '>', FN:1139) and is '\n'-terminated
  const uint64_t W = 4ull << 20;
  std::vector<uint8_t> buf(W + 1);
  uint64_t hi = B;  // candidates s in [lo, hi)
  while (hi > 0) {
    const uint64_t lo = hi > W ? hi - W : 0;
    const uint64_t rd = lo ? lo - 1 : 0;  // one byte before lo: is lo a line start?
    if (!pread_all(fd, buf.data(), hi - rd, rd)) return ~0ull;
    const uint8_t* b = buf.data() + (lo - rd);  // b[i] = x[lo + i]
    for (uint64_t s = hi; s-- > lo;) {
      const bool start = s == 0 || b[(int64_t)(s - lo) - 1] == '\n';
      if (!start) continue;
      const uint8_t c = b[s - lo];
      if (c == '\n') return s + 1;
      if (c == '>') {
        const uint64_t e = line_end(fd, fsz, s);
        if (e != ~0ull) return e;
      }
    }
    hi = lo;
  }
  return 0;
}

bool shard_bounds(const std::string& path, uint32_t world, std::vector<uint64_t>& bounds, uint64_t& fsz,
                  std::string& err) {
  int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) { err = "Error opening file of sequence (" + path + ")"; return false; }
  struct stat sb;
  if (fstat(fd, &sb) != 0) { close(fd); err = "cannot stat " + path; return false; }
  fsz = (uint64_t)sb.st_size;
  bounds.assign(world + 1, 0);
  bounds[world] = fsz;
  for (uint32_t k = 1; k < world; k++) {
    bounds[k] = shard_start(fd, fsz, (uint64_t)((unsigned __int128)k * fsz / world));
    if (bounds[k] == ~0ull) { close(fd); err = "read error on " + path; return false; }
  }
  close(fd);
  return true;
}

}  // namespace cmsbwt
