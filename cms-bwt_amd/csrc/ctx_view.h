// ctx_view.h — what the in-process multi-GPU driver (multi.hip) reads of a
// rank's engine, without including engine.h (whose rocPRIM instantiations
// would otherwise be compiled into that translation unit a second time).
// Defined in engine.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/cmsbwt.h"

namespace cmsbwt {

struct CtxView {
  int device = 0;
  hipStream_t st = nullptr;
  uint32_t n = 0;            // augmented reference length
  uint32_t H = 0;            // heads of this rank's walk
  uint64_t ndocs = 0, chars = 0, sn = 0;
  bool collTail = false;     // the device reader closed a tail document
  bool orderInvariant = false;
  // walk outputs: h_start h_pos h_len h_smaller h_lchar h_isa h_tonext h_nexthead
  const void* heads[8] = {};
  const int32_t* diff = nullptr;     // run difference array, n + 1
  const uint8_t* hasHead = nullptr;  // head flags, n
  // sharded merge state
  uint32_t dmItems = 0;              // items of the owned positions
  const uint32_t* dmItemPos = nullptr;
  const uint32_t* dmGrp = nullptr;   // group label (1 + head rank) per head
  uint64_t dmU = 0;                  // unresolved members after dm_dbl_init
  uint32_t dmLabelBias = 0;          // added to every label in dmGrp
  cmsbwt_stats stats{};
  uint64_t devicePeak = 0;
};

CtxView ctx_view(const cmsbwt_ctx* c);
// device buffers from the rank's caching allocator (same stream order)
void* ctx_alloc(cmsbwt_ctx* c, uint64_t bytes);
void ctx_free(cmsbwt_ctx* c, void* p);
// distinct values of a sorted array (phrasesSet.size() of the owned items)
uint64_t ctx_count_distinct(cmsbwt_ctx* c, const uint32_t* v, uint32_t k);

struct CtxError {
  int code;
  std::string msg;
};

}  // namespace cmsbwt
