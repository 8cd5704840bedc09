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

#include <stdio.h>
#include <string.h>
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
