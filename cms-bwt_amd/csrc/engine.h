#pragma once
// engine.h — host orchestration of the CMS-BWT hot path on one MI355X; the
// Engine shared by engine.hip (C ABI) and dist_merge.hip (multi-GPU merge).
//
// Stage map (reference = CMS-BWT-functions.cpp, "FN"):
//   load_reference ... FN:151-310  (host SA-IS + LCP, staged into HBM)
//   load_collection .. FN:1138-1275 (reader) -> text + doc offsets in HBM
//   ms_walk .......... FN:1151-1212 walk (k_ms_walk), FN:1359-1385 j-scan
//   merge ............ FN:1387-1416 grouping (radix sorts), FN:1432-1494 ranks
//                      + suffix sort of the head string (prefix doubling),
//                      FN:1504-1603 counters, FN:1618-1777 inversion + runs
#ifndef CMSBWT_POS_SORT_BITS
#define CMSBWT_POS_SORT_BITS 0  // 0: rocPRIM's default digits for the position sort
#endif
#ifndef CMSBWT_POS_SORT_IPT
#define CMSBWT_POS_SORT_IPT 12
#endif
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <cstring>

#include <hip/hip_runtime.h>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

// rocPRIM's radix sort assumes any non-pointer input may alias its output and,
// with an odd number of digit passes, first copies keys and values into its
// temporary buffers (a 16-B HeadKV per head for the position sort: ~0.5 ms
// at 1e8 heads).  The grouping's value input is computed from the head SoA
// (MakeHeadKV over a counting iterator) and never aliases a sort buffer, so
// tell it so; the first pass then reads the input directly.  Declared before
// the rocPRIM device headers: their qualified call is looked up there.
// The hook depends on a private rocPRIM detail: it is declared only for the
// rocPRIM major version it was written against (4.x, ROCm 7.2), and it
// returns its own type so that a static_assert below proves the overload is
// the one selected (a rocPRIM change that stops it matching fails the build
// instead of silently bringing the copy back).
#include <rocprim/rocprim_version.hpp>
#if ROCPRIM_VERSION >= 400000 && ROCPRIM_VERSION < 500000
#define CMSBWT_NOALIAS_HOOK 1
namespace cmsbwt {
struct MakeHeadKV;
struct NoAlias {  // "cannot alias", as the bool rocPRIM stores
  __host__ __device__ constexpr operator bool() const { return false; }
};
}  // namespace cmsbwt
BEGIN_ROCPRIM_NAMESPACE
namespace detail {
template <class V, class D, class O>
inline cmsbwt::NoAlias can_iterators_alias(transform_iterator<counting_iterator<unsigned int, D>, cmsbwt::MakeHeadKV, V>,
                                           O*, const size_t) {
  return {};
}
}  // namespace detail
END_ROCPRIM_NAMESPACE
#else
#define CMSBWT_NOALIAS_HOOK 0
#endif
#include <rocprim/rocprim.hpp>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <exception>
#include <thread>
#include <fstream>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cmsbwt.h"
#include "device_common.h"
#include "host_index.h"
#include "host_reader.h"
#include "kernels.h"
#include "map_replay.h"
#include "merge_kernels.h"
#include "elem_writer.h"
#include "synth.h"

namespace cmsbwt {

struct IsActive {  // an unresolved member's sa position (0xffffffff = resolved)
  __host__ __device__ bool operator()(uint32_t v) const { return v != 0xffffffffu; }
};
struct LastNonEmpty {  // scan operator: the later non-empty unit's (has, last, first) wins
  __host__ __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return (b >> 16) ? b : a; }
};
struct WidenU64 {
  __host__ __device__ uint64_t operator()(uint32_t v) const { return (uint64_t)v; }
};
struct MakeHeadKV {  // head idx -> its grouping fields
  const uint32_t* len;
  const uint32_t* isa;
  const uint8_t* smaller;
  const uint32_t* tonext;
  __host__ __device__ HeadKV operator()(uint32_t i) const {
    return HeadKV{i, len[i] | (smaller[i] ? 0x80000000u : 0u), isa[i], tonext[i]};
  }
};
#if CMSBWT_NOALIAS_HOOK
// the position sort's computed input must select the hook above (else rocPRIM
// copies it into its buffers first, ~0.5 ms per step at 1e8 heads)
static_assert(std::is_same<decltype(::rocprim::detail::can_iterators_alias(
                               rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint32_t>(0u),
                                                                MakeHeadKV{}),
                               (HeadKV*)nullptr, size_t{0})),
                           NoAlias>::value,
              "rocPRIM no longer selects the no-alias hook for the position sort's input");
#endif
struct AdjustedRuns {  // k_wr_adjust's rule, as a scan input
  const uint32_t* runs;
  const uint32_t* hl;
  const uint32_t* prev;
  __host__ __device__ unsigned long long operator()(uint32_t u) const {
    const uint32_t a = hl[u], pv = prev[u];
    return (unsigned long long)runs[u] - (((a >> 16) && (pv >> 16) && (a & 0xff) == ((pv >> 8) & 0xff)) ? 1u : 0u);
  }
  template <class Eng>
  unsigned long long host(uint32_t u, Eng* e) const {  // the last element's value, read back to the host
    const uint32_t a = e->read1(hl + u), pv = e->read1(prev + u), r = e->read1(runs + u);
    return (unsigned long long)r - (((a >> 16) && (pv >> 16) && (a & 0xff) == ((pv >> 8) & 0xff)) ? 1u : 0u);
  }
};
// (adjusted runs << kPackSymBits) | symbols of a writer element: both
// exclusive scans of the writer in one pass
struct PackedRunsSym {
  AdjustedRuns runs;
  const unsigned long long* sym;
  __host__ __device__ unsigned long long operator()(uint32_t u) const {
    return (runs(u) << kPackSymBits) | sym[u];
  }
};
// (adjusted runs << kPackSymBits) | symbols of a sharded-writer element
struct PackAdjSym {
  const uint32_t* adj;
  const unsigned long long* sym;
  __host__ __device__ unsigned long long operator()(uint32_t u) const {
    return ((unsigned long long)adj[u] << kPackSymBits) | sym[u];
  }
};
struct PlusOneU64 {
  __host__ __device__ unsigned long long operator()(unsigned long long v) const { return v + 1; }
};

struct HipError {
  std::string msg;
};

#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess)                                                                      \
      throw HipError{std::string(#x) + " -> " + hipGetErrorString(e_) + " @" + std::to_string(__LINE__)}; \
  } while (0)

struct InputError {
  int code;
  std::string msg;
};

// Caching device allocator: the step allocates the same sequence of buffers
// every time, so blocks are kept after release and handed back on the next
// request of a similar size (all work runs on one stream, so stream order
// makes reuse safe).  hipMalloc/hipFree of multi-GB buffers otherwise cost
// tens of milliseconds per step.
struct DevAlloc {
  std::multimap<uint64_t, void*> freeBlocks;
  std::unordered_map<void*, uint64_t> sizes;
  uint64_t cached = 0;
  uint64_t limit = 96ull << 30;
  void* get(uint64_t bytes) {
    bytes = (std::max<uint64_t>(bytes, 64) + 255) & ~255ull;
    auto it = freeBlocks.lower_bound(bytes);
    if (it != freeBlocks.end() && it->first <= bytes + bytes / 4 + (4u << 20)) {
      void* p = it->second;
      cached -= it->first;
      live += it->first;
      peak = std::max(peak, live);
      freeBlocks.erase(it);
      return p;
    }
    void* p = nullptr;
    mallocs++;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      trim();
      if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        throw HipError{"device out of memory: request " + std::to_string(bytes >> 20) + " MiB with " +
                       std::to_string(live >> 20) + " MiB live (peak " + std::to_string(peak >> 20) + " MiB)"};
      }
    }
    sizes[p] = bytes;
    live += bytes;
    peak = std::max(peak, live);
    return p;
  }
  uint64_t live = 0, peak = 0;  // bytes handed out by get() and not yet put() back
  uint64_t mallocs = 0, trims = 0;  // hipMalloc calls (cache misses) and full trims
  void put(void* p) {
    auto s = sizes.find(p);
    if (s == sizes.end()) { (void)hipFree(p); return; }
    live -= s->second;
    freeBlocks.emplace(s->second, p);
    cached += s->second;
    if (cached > limit) trim();
  }
  void trim() {
    trims++;
    (void)hipDeviceSynchronize();
    for (auto& kv : freeBlocks) {
      sizes.erase(kv.second);
      (void)hipFree(kv.second);
    }
    freeBlocks.clear();
    cached = 0;
  }
  ~DevAlloc() {
    trim();
    for (auto& kv : sizes) (void)hipFree(kv.first);
  }
};
inline thread_local DevAlloc* g_alloc = nullptr;

template <class T>
struct DBuf {
  T* p = nullptr;
  uint64_t n = 0;
  DevAlloc* owner = nullptr;
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  ~DBuf() { release(); }
  void alloc(uint64_t k) {
    release();
    n = k;
    if (!k) return;
    owner = g_alloc;
    if (owner) p = (T*)owner->get(k * sizeof(T));
    else HIPCHK(hipMalloc((void**)&p, std::max<uint64_t>(k * sizeof(T), 64)));
  }
  void zero(hipStream_t st) { if (n) HIPCHK(hipMemsetAsync(p, 0, n * sizeof(T), st)); }
  void release() {
    if (p) {
      if (owner) owner->put(p);
      else (void)hipFree(p);
    }
    p = nullptr;
    n = 0;
    owner = nullptr;
  }
  uint64_t bytes() const { return n * sizeof(T); }
  void swap_in(DBuf& o) {  // take o's buffer (ours goes to o)
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(owner, o.owner);
  }
};

static uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = getenv(name);
  return v ? (uint32_t)strtoul(v, nullptr, 10) : dflt;
}

static int bits_for(uint64_t v) {  // bits to represent values in [0, v]
  int b = 1;
  while (b < 64 && (v >> b)) b++;
  return b;
}

struct Engine {
  DevAlloc alloc;  // first member: destroyed last
  // side-stream buffers (merge): a pool of their own, so a block the main
  // stream may still read is never handed to side work inside one fork epoch
  DevAlloc sideAlloc;
  int device = 0;
  hipStream_t st = nullptr;
  std::string err;
  cmsbwt_stats stats{};

  // ---- reference
  bool refLoaded = false;
  HostIndex hix;
  DBuf<uint8_t> dx, dbwt;
  DBuf<int32_t> dsa, dlcp, dplcp;
  DBuf<uint8_t> dplcp8;  // min(PLCP, 255), the walk's first skip window
  DBuf<uint32_t> disa;
  DBuf<uint32_t> dpfx, dpfk;
  DBuf<uint32_t> dld;
  DBuf<uint4> dpr, dir;
  DBuf<uint8_t> dkmap;
  DevRef R{};

  // ---- collection
  bool collLoaded = false;
  DBuf<uint8_t> dtext;
  DBuf<uint64_t> ddoc;
  std::vector<uint64_t> hdoc;  // doc offsets (ndocs+1), doc k = [hdoc[k], hdoc[k+1]-1)
  uint64_t ndocs = 0, chars = 0, sn = 0;
  uint64_t collChars = 0;  // chars of the loaded collection (ms_walk input)
  bool collTail = false;   // the device reader closed a tail document (FN:1269-1275)

  // ---- walk outputs
  bool walked = false;
  uint32_t H = 0;
  DBuf<uint32_t> hStart, hPos, hLen, hIsa, hTonext;
  DBuf<uint8_t> hSmall, hChar;
  DBuf<uint16_t> hNext;
  DBuf<int32_t> diff;
  DBuf<uint8_t> hasHead;

  // ---- merge outputs (kept for parity copies)
  bool merged = false;
  uint32_t K = 0;
  DBuf<int32_t> T;
  DBuf<uint32_t> saT;
  DBuf<uint8_t> bwtHeads;  // parity copies only (CMSBWT_KEEP_STAGES)
  DBuf<uint8_t> bwtSlot;   // the character before each head, by slot in head-rank order
  DBuf<unsigned long long> counter;
  DBuf<int64_t> bucket;
  DBuf<uint8_t> runs;
  uint64_t nruns = 0;
  int lastRle = 1;
  DBuf<uint8_t> tmp;  // rocPRIM scratch
  // Side stream of the merge: work off the main chain (the counter's windows
  // beside the ranks and the suffix sort, the writer's inputs beside the
  // counter) runs there concurrently.  Inside a Side scope every helper
  // (scans, sorts, read-backs, scratch) follows st / tmp, which it swaps, and
  // new buffers come from sideAlloc.  Buffers a side epoch hands to the main
  // stream live until the merge's final synchronisation.
  hipStream_t st2 = nullptr;
  DBuf<uint8_t> tmp2;
  hipEvent_t evFork[2] = {}, evJoin = nullptr;
  struct Side {
    Engine& e;
    DevAlloc* prev;
    Side(Engine& en, hipEvent_t fork) : e(en), prev(g_alloc) {
      HIPCHK(hipStreamWaitEvent(e.st2, fork, 0));
      std::swap(e.st, e.st2);
      e.tmp.swap_in(e.tmp2);
      g_alloc = &e.sideAlloc;
    }
    ~Side() {
      std::swap(e.st, e.st2);
      e.tmp.swap_in(e.tmp2);
      g_alloc = prev;
    }
  };
  // the main stream waits for everything enqueued on the side stream so far
  void join_side() {
    HIPCHK(hipEventRecord(evJoin, st2));
    HIPCHK(hipStreamWaitEvent(st, evJoin, 0));
  }

  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // merge phase marks for the reference's log timers: ranks start, doubling
  // start / end, ranks end, counter start / end
  hipEvent_t evm[6] = {};
  DBuf<uint32_t> rthFL;  // grp[0], grp[H-1] of the last merge (First/Last rankToHead + 1)

  explicit Engine(int dev) : device(dev) {
    g_alloc = &alloc;
    HIPCHK(hipSetDevice(dev));
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
    for (auto& e : evFork) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&evJoin, hipEventDisableTiming));
    HIPCHK(hipEventCreate(&ev0));
    HIPCHK(hipEventCreate(&ev1));
    for (auto& e : evm) HIPCHK(hipEventCreate(&e));
  }
  ~Engine() {
    g_alloc = &alloc;
    if (pend.on) {  // a collection upload still streaming into HBM: stop it
      pend.cancel = true;
      pend.th.join();
      pend.on = false;
    }
    for (void* b : pinned) (void)hipHostFree(b);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    for (auto e : evm) if (e) (void)hipEventDestroy(e);
    for (auto e : evFork) if (e) (void)hipEventDestroy(e);
    if (evJoin) (void)hipEventDestroy(evJoin);
    if (st2) { (void)hipStreamSynchronize(st2); (void)hipStreamDestroy(st2); }
    if (st) (void)hipStreamDestroy(st);
  }

  void* scratch(size_t bytes) {
    if (tmp.n < bytes) tmp.alloc(bytes + (bytes >> 3) + 256);
    return tmp.p;
  }
  void sync() { HIPCHK(hipStreamSynchronize(st)); }
  // CMSBWT_DM_TIMING=1: host-timed sub-stages of the sharded merge's calls
  // (synchronising the stream at every mark; attribution runs only)
  int dmtOn = -1;
  std::chrono::steady_clock::time_point dmtT;
  std::string dmtLine;
  uint64_t dmtMallocs = 0, dmtTrims = 0;
  void dmt(const char* what) {
    if (dmtOn < 0) dmtOn = env_u32("CMSBWT_DM_TIMING", 0) ? 1 : 0;
    if (!dmtOn) return;
    sync();
    const auto t = std::chrono::steady_clock::now();
    if (what) {
      char b[96];
      const uint64_t m = alloc.mallocs + sideAlloc.mallocs, tr = alloc.trims + sideAlloc.trims;
      if (m != dmtMallocs || tr != dmtTrims)
        snprintf(b, sizeof b, " %s %.2f (+%llu malloc, +%llu trim)", what,
                 std::chrono::duration<double, std::milli>(t - dmtT).count(), (unsigned long long)(m - dmtMallocs),
                 (unsigned long long)(tr - dmtTrims));
      else
        snprintf(b, sizeof b, " %s %.2f", what, std::chrono::duration<double, std::milli>(t - dmtT).count());
      dmtLine += b;
      dmtMallocs = m;
      dmtTrims = tr;
    }
    dmtT = t;
  }
  void dmtFlush(const char* call) {
    if (dmtOn != 1) return;
    fprintf(stderr, "[dm-timing] rank %u %s:%s\n", dm.rank, call, dmtLine.c_str());
    dmtLine.clear();
  }

  template <class T_>
  T_ read1(const T_* d) {
    T_ v;
    HIPCHK(hipMemcpyAsync(&v, d, sizeof(T_), hipMemcpyDeviceToHost, st));
    sync();
    return v;
  }
  // *a + *b read back with one synchronisation (the sizes after a scan: last
  // exclusive offset + last count)
  template <class A_, class B_>
  uint64_t sum2(const A_* a, const B_* b) {
    A_ va;
    B_ vb;
    HIPCHK(hipMemcpyAsync(&va, a, sizeof(A_), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&vb, b, sizeof(B_), hipMemcpyDeviceToHost, st));
    sync();
    return (uint64_t)va + (uint64_t)vb;
  }

  // ---- rocPRIM helpers
  template <class In, class Out, class Init, class Op>
  void exscan(In in, Out out, Init init, uint64_t n, Op op) {
    if (!n) return;
    size_t b = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, b, in, out, init, (size_t)n, op, st));
    HIPCHK(rocprim::exclusive_scan(scratch(b), b, in, out, init, (size_t)n, op, st));
  }
  // u32 plus scans of plain arrays: the tile scan of merge.hip (tile sums,
  // their rocPRIM scan, the tiles); anything else: rocPRIM
  template <class In, class Out>
  static constexpr bool kTileScan =
      (std::is_same_v<In, uint32_t*> || std::is_same_v<In, const uint32_t*>) && std::is_same_v<Out, uint32_t*>;
  void tile_scan(const uint32_t* in, uint32_t* out, uint32_t init, uint64_t n, bool inclusive) {
    const uint64_t nt = scan_tiles(n);
    DBuf<uint32_t> sums, off;
    sums.alloc(nt);
    off.alloc(nt);
    mk_scan_sums(in, n, sums.p, st);
    size_t b = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, b, sums.p, off.p, 0u, (size_t)nt, rocprim::plus<uint32_t>(), st));
    HIPCHK(rocprim::exclusive_scan(scratch(b), b, sums.p, off.p, 0u, (size_t)nt, rocprim::plus<uint32_t>(), st));
    mk_scan_tiles(in, out, n, off.p, init, inclusive, st);
  }
  static bool rocprim_scan() { return env_u32("CMSBWT_ROCPRIM_SCAN", 0) != 0; }
  // inclusive u64 scan of (in[i] + 1): the writer's cumulative counters
  void inscan_plus1_u64(const unsigned long long* in, unsigned long long* out, uint64_t n) {
    if (!n) return;
    if (rocprim_scan()) {
      inscan(rocprim::make_transform_iterator(in, PlusOneU64()), out, n, rocprim::plus<unsigned long long>());
      return;
    }
    const uint64_t nt = scan_tiles(n);
    DBuf<unsigned long long> sums, off;
    sums.alloc(nt);
    off.alloc(nt);
    mk_scan64_sums(in, n, 1u, sums.p, st);
    size_t b = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, b, sums.p, off.p, 0ull, (size_t)nt, rocprim::plus<unsigned long long>(),
                                   st));
    HIPCHK(rocprim::exclusive_scan(scratch(b), b, sums.p, off.p, 0ull, (size_t)nt,
                                   rocprim::plus<unsigned long long>(), st));
    mk_scan64_tiles(in, out, n, off.p, 1u, true, st);
  }
  template <class In, class Out, class Init>
  void exscan(In in, Out out, Init init, uint64_t n) {
    if (!n) return;
    if constexpr (kTileScan<In, Out> && std::is_same_v<Init, uint32_t>) {
      if (!rocprim_scan()) { tile_scan(in, out, init, n, false); return; }
    }
    size_t b = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, b, in, out, init, (size_t)n, rocprim::plus<Init>(), st));
    HIPCHK(rocprim::exclusive_scan(scratch(b), b, in, out, init, (size_t)n, rocprim::plus<Init>(), st));
  }
  template <class In, class Out, class Op>
  void inscan(In in, Out out, uint64_t n, Op op) {
    if (!n) return;
    if constexpr (kTileScan<In, Out> && std::is_same_v<Op, rocprim::plus<uint32_t>>) {
      if (!rocprim_scan()) { tile_scan(in, out, 0u, n, true); return; }
    }
    size_t b = 0;
    HIPCHK(rocprim::inclusive_scan(nullptr, b, in, out, (size_t)n, op, st));
    HIPCHK(rocprim::inclusive_scan(scratch(b), b, in, out, (size_t)n, op, st));
  }
  template <class Kt, class Vt>
  void sort_pairs(const Kt* kin, Kt* kout, const Vt* vin, Vt* vout, uint64_t n, int bits) {
    if (!n) return;
    size_t b = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, b, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, st));
    HIPCHK(rocprim::radix_sort_pairs(scratch(b), b, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, st));
  }
  template <class Kt>
  void sort_keys(const Kt* kin, Kt* kout, uint64_t n, int bits) {
    if (!n) return;
    size_t b = 0;
    HIPCHK(rocprim::radix_sort_keys(nullptr, b, kin, kout, (size_t)n, 0u, (unsigned)bits, st));
    HIPCHK(rocprim::radix_sort_keys(scratch(b), b, kin, kout, (size_t)n, 0u, (unsigned)bits, st));
  }
  uint32_t select_flagged_u64(const unsigned long long* in, const uint32_t* flags, unsigned long long* out,
                              uint32_t n) {
    if (!n) return 0;
    DBuf<uint32_t> cnt;
    cnt.alloc(1);
    size_t b = 0;
    HIPCHK(rocprim::select(nullptr, b, in, flags, out, cnt.p, (size_t)n, st));
    HIPCHK(rocprim::select(scratch(b), b, in, flags, out, cnt.p, (size_t)n, st));
    return read1(cnt.p);
  }
  uint32_t max_u32(const uint32_t* in, uint64_t n) {
    if (!n) return 0;
    DBuf<uint32_t> out;
    out.alloc(1);
    size_t b = 0;
    HIPCHK(rocprim::reduce(nullptr, b, in, out.p, 0u, (size_t)n, rocprim::maximum<uint32_t>(), st));
    HIPCHK(rocprim::reduce(scratch(b), b, in, out.p, 0u, (size_t)n, rocprim::maximum<uint32_t>(), st));
    return read1(out.p);
  }
  // order-preserving compaction; `out` must not alias `in` (both paths)
  uint32_t select_flagged(const uint32_t* in, const uint32_t* flags, uint32_t* out, uint32_t n) {
    if (!n) return 0;
    if ((const void*)in == (const void*)out) throw InputError{CMSBWT_EINTERNAL, "internal: select_flagged in place"};
    if (!env_u32("CMSBWT_ROCPRIM_SELECT", 0)) {  // two-pass tile compaction (merge.hip)
      const uint32_t nt = sel_tiles(n);
      DBuf<uint32_t> tc, to;
      tc.alloc(nt);
      to.alloc(nt);
      mk_sel_count(flags, n, tc.p, st);
      exscan(tc.p, to.p, 0u, nt);
      mk_sel_write(in, flags, n, to.p, out, st);
      return (uint32_t)sum2(to.p + (nt - 1), tc.p + (nt - 1));
    }
    DBuf<uint32_t> cnt;
    cnt.alloc(1);
    size_t b = 0;
    HIPCHK(rocprim::select(nullptr, b, in, flags, out, cnt.p, (size_t)n, st));
    HIPCHK(rocprim::select(scratch(b), b, in, flags, out, cnt.p, (size_t)n, st));
    return read1(cnt.p);
  }

  // =====================================================================
  // Reference index and walk tables built on the device (ref_index.hip):
  // the same arrays, layouts and tables as build_index() + stage_host(),
  // without a host round trip (tests/test_gpu_index.py compares them).
  void stage_device() {
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t0 = now();
    const uint32_t n = hix.n;
    if (env_u32("CMSBWT_TIMING", 0)) {  // the first kernel of the process loads the code object
      DBuf<uint32_t> one;
      one.alloc(1);
      mk_iota(one.p, 1, st);
      sync();
      fprintf(stderr, "[index] first launch %.3f s\n", std::chrono::duration<double>(now() - t0).count());
      t0 = now();
    }
    dx.alloc((uint64_t)n + kTextPad);
    HIPCHK(hipMemsetAsync(dx.p, 0, n + kTextPad, st));
    HIPCHK(hipMemcpyAsync(dx.p, hix.x.data(), n, hipMemcpyHostToDevice, st));
    dsa.alloc((uint64_t)n + 16);
    disa.alloc((uint64_t)n + 16);
    dplcp.alloc((uint64_t)n + 17);
    dbwt.alloc(n);
    dsa.zero(st);
    disa.zero(st);
    dplcp.zero(st);
    // LCP + block-minima levels in one buffer (layout of stage_host)
    memset(&R, 0, sizeof(R));
    std::vector<uint32_t> lvlLen;
    {
      uint64_t prev = n;
      do {
        prev = (prev + 63) / 64;
        lvlLen.push_back((uint32_t)prev);
      } while (prev > 64 && (int)lvlLen.size() < kMaxLevels);
    }
    auto pad = [](uint64_t k) { return (k + 16 + 3) & ~3ull; };
    uint64_t total = pad((uint64_t)n + 1);
    for (auto v : lvlLen) total += pad(v);
    dlcp.alloc(total);
    dlcp.zero(st);
    const bool saTm = env_u32("CMSBWT_TIMING", 0) != 0;
    auto saMark = [&](const char* what, uint64_t v) {
      if (!saTm) return;
      sync();
      fprintf(stderr, "[index]   %-12s %.3f s  (%llu)\n", what, std::chrono::duration<double>(now() - t0).count(),
              (unsigned long long)v);
    };
    {  // SA by prefix doubling
      DBuf<unsigned long long> k0, k1;
      DBuf<uint32_t> v0, v1, rank, headIn, head, tie, act, act2;
      k0.alloc(n); k1.alloc(n); v0.alloc(n); v1.alloc(n);
      rank.alloc(n); headIn.alloc(n); head.alloc(n); tie.alloc(n); act.alloc(n); act2.alloc(n);
      saMark("alloc", n);
      int32_t* sa = dsa.p;
      launch_ix_init(dx.p, n, k0.p, v0.p, st);
      saMark("keys", n);
      sort_pairs(k0.p, k1.p, v0.p, v1.p, n, 9 * kIdxH0);
      saMark("sort", n);
      launch_ix_heads(k1.p, nullptr, n, headIn.p, tie.p, st);
      inscan(headIn.p, head.p, n, rocprim::maximum<uint32_t>());
      launch_ix_place(v1.p, nullptr, head.p, n, sa, rank.p, st);
      mk_iota(act2.p, n, st);
      uint32_t U = select_flagged(act2.p, tie.p, act.p, n);
      saMark("first sort", U);
      const int bits = 32 + bits_for(n);
      uint64_t h = kIdxH0;
      int rounds = 0;
      while (U) {
        if (++rounds > 40 || h >= 2ull * n) throw InputError{CMSBWT_EDEVICE, "internal: prefix doubling did not converge"};
        launch_ix_keys(act.p, U, sa, rank.p, n, (uint32_t)std::min<uint64_t>(h, n), k0.p, v0.p, st);
        sort_pairs(k0.p, k1.p, v0.p, v1.p, U, bits);
        launch_ix_heads(k1.p, act.p, U, headIn.p, tie.p, st);
        inscan(headIn.p, head.p, U, rocprim::maximum<uint32_t>());
        launch_ix_place(v1.p, act.p, head.p, U, sa, rank.p, st);
        U = select_flagged(act.p, tie.p, act2.p, U);
        act.swap_in(act2);
        h <<= 1;
        saMark("round", U);
      }
    }
    sync();
    auto t1 = now();
    DBuf<uint32_t> err;
    err.alloc(1);
    err.zero(st);
    if (env_u32("CMSBWT_TIMING", 0)) fprintf(stderr, "[index] sa         %.3f s\n", std::chrono::duration<double>(t1 - t0).count());
    // stage times of the reference's log (FN:258-299): ISA, LCP + PLCP, RMQ
    // (the LCP block minima the PSV/NSV scans climb), BWT, by HIP events
    hipEvent_t ix[5];
    for (auto& e : ix) HIPCHK(hipEventCreate(&e));
    HIPCHK(hipEventRecord(ix[0], st));
    {
      DBuf<int32_t> phi, plcpRaw;
      phi.alloc(n);
      plcpRaw.alloc(n);
      launch_ix_isa(dsa.p, n, disa.p, phi.p, st);
      HIPCHK(hipEventRecord(ix[1], st));
      launch_ix_lcp(dx.p, dsa.p, n, disa.p, phi.p, plcpRaw.p, dlcp.p, dplcp.p, st);
      HIPCHK(hipEventRecord(ix[2], st));
    }
    launch_ix_plcp_check(dplcp.p, n, err.p, st);
    uint64_t off = pad((uint64_t)n + 1);
    const int32_t* prev = dlcp.p;
    uint32_t prevLen = n;
    int L = 0;
    for (auto v : lvlLen) {
      launch_ix_level(prev, prevLen, dlcp.p + off, v, st);
      R.lvl[L] = dlcp.p + off;
      R.lvlOff[L] = (uint32_t)off;
      R.lvlLen[L] = v;
      prev = dlcp.p + off;
      prevLen = v;
      off += pad(v);
      L++;
    }
    R.nlvl = L;
    HIPCHK(hipEventRecord(ix[3], st));
    launch_ix_bwt(dx.p, dsa.p, n, dbwt.p, st);
    HIPCHK(hipEventRecord(ix[4], st));
    HIPCHK(hipEventSynchronize(ix[4]));
    {
      float v = 0;
      double* dst[4] = {&hix.t_isa, &hix.t_lcp_only, &hix.t_rmq, &hix.t_bwt};
      for (int k = 0; k < 4; k++) {
        HIPCHK(hipEventElapsedTime(&v, ix[k], ix[k + 1]));
        *dst[k] = v / 1e3;
      }
    }
    for (auto e : ix) (void)hipEventDestroy(e);
    R.x = dx.p;
    R.sa = dsa.p;
    R.isa = disa.p;
    R.lcp = dlcp.p;
    R.plcp = dplcp.p;
    stage_plcp8(n);
    R.bwt = dbwt.p;
    R.n = n;
    if (read1(err.p)) throw InputError{CMSBWT_EINPUT, "internal: PLCP monotonicity violated"};
    const bool tm = env_u32("CMSBWT_TIMING", 0) != 0;
    auto mark = [&](const char* what) {
      if (!tm) return;
      sync();
      static auto last = now();
      auto t = now();
      fprintf(stderr, "[index] %-10s %.3f s\n", what, std::chrono::duration<double>(t - last).count());
      last = t;
    };
    mark("lcp+levels");
    build_prefix_tables(true);
    mark("pfx");
    dld.alloc((uint64_t)n + 16);
    dld.zero(st);
    launch_ix_child(dx.p, dsa.p, dlcp.p, n, dld.p, st);
    R.ld = dld.p;
    mark("child");
    dpr.alloc((uint64_t)n + 16);
    dir.alloc((uint64_t)n + 16);
    dpr.zero(st);
    dir.zero(st);
    launch_ix_adjacency(dsa.p, disa.p, dlcp.p, n, (uint32_t*)dpr.p, (uint32_t*)dir.p, st);
    R.pr = dpr.p;
    R.ir = dir.p;
    HIPCHK(hipGetLastError());
    sync();
    mark("adjacency");
    hix.t_sa = std::chrono::duration<double>(t1 - t0).count();
    hix.t_lcp = std::chrono::duration<double>(now() - t1).count();
  }

  void stage_plcp8(uint32_t n) {
    dplcp8.alloc((uint64_t)n + 32);
    HIPCHK(hipMemsetAsync(dplcp8.p + n, 0, 32, st));
    launch_ix_plcp8(dplcp.p, n, dplcp8.p, st);
    R.plcp8 = dplcp8.p;
  }

  // =====================================================================
  // reference (FN:151-310)
  void load_reference_bytes(const std::string& trimmed) {
    auto t0 = std::chrono::steady_clock::now();
    if (memchr(trimmed.data(), 2, trimmed.size()))
      throw InputError{CMSBWT_EINPUT, "reference contains byte 0x02 (the document separator)"};
    if (trimmed.size() + 130 >= (1ull << 31)) throw InputError{CMSBWT_ELIMIT, "reference longer than 2^31 (int32 SA)"};
    const char* hi = getenv("CMSBWT_HOST_INDEX");
    hix.t_isa = hix.t_lcp_only = hix.t_rmq = hix.t_bwt = 0;
    if (hi && *hi && *hi != '0') {
      build_index(trimmed, hix);
      hix.t_augment = 0;
      stage_host();
    } else {
      auto ta = std::chrono::steady_clock::now();
      augment_reference(trimmed, hix);
      hix.t_augment = std::chrono::duration<double>(std::chrono::steady_clock::now() - ta).count();
      stage_device();
    }
    refLoaded = true;
    stats.n = hix.n;
    stats.t_augment_ms = hix.t_augment * 1e3;
    stats.t_sa_ms = hix.t_sa * 1e3;
    stats.t_isa_ms = hix.t_isa * 1e3;
    stats.t_lcp_ms = hix.t_lcp_only * 1e3;
    stats.t_rmq_ms = hix.t_rmq * 1e3;
    stats.t_bwt_ms = hix.t_bwt * 1e3;
    stats.ref_file_bytes = hix.file_bytes;
    stats.ref_read_size = hix.read_size;
    stats.t_index_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  // host SA-IS index (build_index) staged into HBM with the walk tables
  // built on the host (CMSBWT_HOST_INDEX=1; the device build's reference)
  void stage_host() {
    const uint32_t n = hix.n;
    // Skip-search precondition: PLCP[q] + q non-decreasing.
    for (uint32_t q = 0; q + 1 < n; q++)
      if ((int64_t)hix.plcp[q + 1] + 1 < (int64_t)hix.plcp[q])
        throw InputError{CMSBWT_EINPUT, "internal: PLCP monotonicity violated"};
    dx.alloc((uint64_t)n + kTextPad);
    HIPCHK(hipMemsetAsync(dx.p, 0, n + kTextPad, st));
    HIPCHK(hipMemcpyAsync(dx.p, hix.x.data(), n, hipMemcpyHostToDevice, st));
    // +16 entries: the uniform-step walk loads whole aligned 16-B blocks (and
    // 8-entry windows) around an index, so arrays carry a readable tail
    dsa.alloc((uint64_t)n + 16);
    HIPCHK(hipMemcpyAsync(dsa.p, hix.sa.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    disa.alloc((uint64_t)n + 16);
    HIPCHK(hipMemcpyAsync(disa.p, hix.isa.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    dplcp.alloc((uint64_t)n + 17);
    HIPCHK(hipMemcpyAsync(dplcp.p, hix.plcp.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    dbwt.alloc(n);
    HIPCHK(hipMemcpyAsync(dbwt.p, hix.bwt.data(), n, hipMemcpyHostToDevice, st));
    // LCP and its block-minima levels in one buffer: [lcp | lvl0 | lvl1 ...],
    // each part 16-B aligned with >= 16 readable entries of tail
    memset(&R, 0, sizeof(R));
    std::vector<std::vector<int32_t>> levels;
    {
      std::vector<int32_t> prev(hix.lcp.begin(), hix.lcp.begin() + n), cur;
      do {
        cur.assign((prev.size() + 63) / 64, INT32_MAX);
        for (size_t i = 0; i < prev.size(); i++) cur[i / 64] = std::min(cur[i / 64], prev[i]);
        levels.push_back(cur);
        prev.swap(cur);
      } while (prev.size() > 64 && (int)levels.size() < kMaxLevels);
    }
    auto pad = [](uint64_t k) { return (k + 16 + 3) & ~3ull; };
    uint64_t total = pad((uint64_t)n + 1);
    for (auto& v : levels) total += pad(v.size());
    dlcp.alloc(total);
    HIPCHK(hipMemcpyAsync(dlcp.p, hix.lcp.data(), ((size_t)n + 1) * 4, hipMemcpyHostToDevice, st));
    uint64_t off = pad((uint64_t)n + 1);
    int L = 0;
    for (auto& v : levels) {
      HIPCHK(hipMemcpyAsync(dlcp.p + off, v.data(), v.size() * 4, hipMemcpyHostToDevice, st));
      R.lvl[L] = dlcp.p + off;
      R.lvlOff[L] = (uint32_t)off;
      R.lvlLen[L] = (uint32_t)v.size();
      off += pad(v.size());
      L++;
    }
    sync();  // `levels` is pageable host memory
    R.nlvl = L;
    R.x = dx.p;
    R.sa = dsa.p;
    R.isa = disa.p;
    R.lcp = dlcp.p;
    R.plcp = dplcp.p;
    stage_plcp8(n);
    R.bwt = dbwt.p;
    R.n = n;
    build_prefix_tables(false);
    build_child_table();
    build_adjacency_records();
    sync();
  }

  // Prefix-rank tables of the uniform-step walk (device_common.h).  With P's
  // interval known for every l <= K, an extension of computeMSFactorAt
  // (FN:45-88) at depth < K over a large interval jumps to the longest
  // matching depth by a few table probes, and a mismatch there has its
  // insertion point (FN:65-76) in the table too, instead of two binary
  // searches (FN:94-149) per character.  Start_l[c] counts the suffixes s
  // smaller than the l-string P of code c: those whose first l bytes are all
  // symbols with code < c, and those whose first non-symbol byte b (or end of
  // x) is at t < l with threshold code(s[0..t)) << B(l-t) + r(b) << B(l-1-t)
  // <= c, r(b) = the number of symbols below b (the augmentation bytes of
  // FN:231-237 are non-symbols anywhere in the byte order).  Stored with it:
  // Count_l[c], the suffixes starting with P (a non-symbol may sort between P
  // and its successor code, so the interval end is Start + Count, not the
  // next Start).  Only ASCII references: there the walk's signed (FN:55) and
  // unsigned orders agree.
  // the paired level-K table (DevRef::pfk) of a DNA reference, from pfx's
  // level K, unless CMSBWT_PFX_PAIR=0 (the walk, built with CMSBWT_PFX_PAIR=1
  // by default, probes it; ms_walk2.hip has the measurement)
  void build_pfx_pair() {
    R.pfk = nullptr;
    dpfk.release();
    if (!R.pfx || !R.pfxDna || R.kmerB != 2 || R.kmerK < 2 || R.kmerK > 14 || !env_u32("CMSBWT_PFX_PAIR", 1)) return;
    dpfk.alloc(16ull << (2 * (R.kmerK - 1)));
    launch_ix_pfx_pair(R.pfx + R.pfxOff[R.kmerK], R.kmerK, dpfk.p, st);
    HIPCHK(hipGetLastError());
    R.pfk = dpfk.p;
  }
  void build_prefix_tables(bool device) {
    R.pfk = nullptr;
    R.pfx = nullptr;
    R.kmap = nullptr;
    R.kmerK = R.kmerB = 0;
    R.pfxExact = R.pfxDna = 0;
    memset(R.pfxOff, 0, sizeof(R.pfxOff));
    if (!env_u32("CMSBWT_PFX", 1)) return;
    const uint32_t n = hix.n;
    const uint64_t* cnt = hix.hist;  // byte counts of the trimmed reference (augment_reference)
    std::vector<uint8_t> map(256, 0xff);
    std::vector<uint32_t> below(256, 0);  // r(b): symbols smaller than byte b
    uint32_t sigma = 0;
    for (int c = 0; c < 256; c++) {
      below[c] = sigma;
      if (cnt[c]) map[c] = (uint8_t)sigma++;
    }
    if (sigma < 2 || sigma > 64) return;
    for (int c = 128; c < 256; c++)
      if (cnt[c]) return;  // ASCII references only
    uint32_t B = 1;
    while ((1u << B) < sigma) B++;
    uint32_t lg = 1;
    while ((1ull << lg) < n) lg++;
    // 2^(B K) ~ 16 n: a K-mer of the text that straddles a mutation then
    // rarely occurs in the reference, and its answer entry ends the walk's
    // search in one probe (10 MB DNA: K = 14, 2.9 GB of tables)
    const uint32_t maxBits = std::min<uint32_t>(env_u32("CMSBWT_KMER_BITS", 28), std::max<uint32_t>(lg + 4, 12));
    const uint32_t K = std::min<uint32_t>(maxBits / B, 16);
    if (K < 3) return;
    uint64_t total = 0;
    for (uint32_t l = 1; l <= K; l++) {
      R.pfxOff[l] = (uint32_t)total;
      total += 2 * ((1ull << (B * l)) + 1);
    }
    if (device) {
      dpfx.alloc(total + 4);
      dpfx.zero(st);
      dkmap.alloc(256);
      HIPCHK(hipMemcpyAsync(dkmap.p, map.data(), 256, hipMemcpyHostToDevice, st));
      DBuf<uint32_t> dbelow, cur, cf, ct, cfEx, ctIn;
      DBuf<uint8_t> term;
      dbelow.alloc(256);
      HIPCHK(hipMemcpyAsync(dbelow.p, below.data(), 256 * 4, hipMemcpyHostToDevice, st));
      cur.alloc(n);
      term.alloc(n);
      cur.zero(st);
      term.zero(st);
      const uint64_t Emax1 = (1ull << (B * K)) + 1;
      cf.alloc(Emax1);
      ct.alloc(Emax1);
      cfEx.alloc(Emax1);
      ctIn.alloc(Emax1);
      for (uint32_t l = 1; l <= K; l++) {
        const uint64_t E1 = (1ull << (B * l)) + 1;
        HIPCHK(hipMemsetAsync(cf.p, 0, E1 * 4, st));
        HIPCHK(hipMemsetAsync(ct.p, 0, E1 * 4, st));
        launch_ix_pfx_count(dx.p, n, l, B, dkmap.p, dbelow.p, cur.p, term.p, cf.p, ct.p, st);
        exscan(cf.p, cfEx.p, 0u, E1);
        inscan(ct.p, ctIn.p, E1, rocprim::plus<uint32_t>());
        launch_ix_pfx_write(cfEx.p, ctIn.p, cf.p, E1, dpfx.p + R.pfxOff[l], st);
      }
      for (uint32_t l = 1; l <= K; l++)  // answer entries, level by level (each reads the level below)
        launch_ix_pfx_answer(dpfx.p + R.pfxOff[l], l > 1 ? dpfx.p + R.pfxOff[l - 1] : nullptr, 1ull << (B * l), B,
                             dsa.p, n, l, st);
      for (uint32_t l = 1; l <= K; l++) launch_ix_pfx_one(dpfx.p + R.pfxOff[l], 1ull << (B * l), dsa.p, st);
      HIPCHK(hipGetLastError());
      sync();  // map/below are pageable
      R.pfx = dpfx.p;
      R.kmap = dkmap.p;
      R.kmerK = K;
      R.kmerB = B;
      R.pfxExact = (cnt[0] == 0 && cnt[1] == 0) ? 1u : 0u;
      R.pfxDna = (sigma == 4 && cnt['A'] && cnt['C'] && cnt['G'] && cnt['T'] && !env_u32("CMSBWT_PFX_GENERIC", 0)) ? 1u : 0u;
      build_pfx_pair();
      return;
    }
    std::vector<uint32_t> tab(total + 4, 0);
    std::vector<uint32_t> cur(n, 0);
    std::vector<uint8_t> term(n, 0);
    std::vector<uint32_t> cf, ct;
    for (uint32_t l = 1; l <= K; l++) {
      const uint64_t E = 1ull << (B * l);
      cf.assign(E + 1, 0);
      ct.assign(E + 1, 0);
      for (uint32_t p = 0; p < n; p++) {
        uint32_t sym = 0;  // past the first non-symbol: zero padding
        if (!term[p]) {
          const uint64_t at = (uint64_t)p + l - 1;
          if (at >= n) {  // end of x: below everything
            term[p] = 1;
          } else {
            const uint8_t b = (uint8_t)hix.x[at];
            if (map[b] == 0xff) { term[p] = 1; sym = below[b]; }  // may carry (r(b) = 2^B)
            else sym = map[b];
          }
        }
        cur[p] = (cur[p] << B) + sym;
        (term[p] ? ct : cf)[cur[p]]++;
      }
      // (Start_l[c], Count_l[c]): Start = sum_{k < c} cf[k] + sum_{k <= c} ct[k]
      uint32_t* o = tab.data() + R.pfxOff[l];
      uint64_t sf = 0, stt = 0;
      for (uint64_t c = 0; c <= E; c++) {
        stt += ct[c];
        o[2 * c] = (uint32_t)(sf + stt);
        o[2 * c + 1] = cf[c];
        sf += cf[c];
      }
      // answer entries (k_ix_pfx_answer)
      const uint32_t* par = l > 1 ? tab.data() + R.pfxOff[l - 1] : nullptr;
      for (uint64_t c = 0; c < E; c++) {
        if (o[2 * c + 1]) continue;
        uint32_t S = 0, C = n;
        if (par) {
          const uint32_t p0 = par[2 * (c >> B)], p1 = par[2 * (c >> B) + 1];
          if (p1 & kPfxAns) { o[2 * c] = p0; o[2 * c + 1] = p1; continue; }
          S = p0;
          C = p1;
        }
        uint32_t mm = o[2 * c], f = kPfxAns | kPfxSmaller;
        if (mm >= S + C) { mm = S + C - 1; f = kPfxAns; }
        if (C == 1) f |= kPfxSingle;
        o[2 * c] = (uint32_t)hix.sa[mm];
        o[2 * c + 1] = f | (l - 1);
      }
    }
    for (uint32_t l = 1; l <= K; l++) {  // k_ix_pfx_one
      uint32_t* o = tab.data() + R.pfxOff[l];
      for (uint64_t c = 0; c < (1ull << (B * l)); c++)
        if (o[2 * c + 1] == 1u) { o[2 * c] = (uint32_t)hix.sa[o[2 * c]]; o[2 * c + 1] = kPfxOne | 1u; }
    }
    dpfx.alloc(total + 4);
    HIPCHK(hipMemcpyAsync(dpfx.p, tab.data(), (total + 4) * 4, hipMemcpyHostToDevice, st));
    dkmap.alloc(256);
    HIPCHK(hipMemcpyAsync(dkmap.p, map.data(), 256, hipMemcpyHostToDevice, st));
    sync();  // `tab` and `map` are pageable
    R.pfx = dpfx.p;
    R.kmap = dkmap.p;
    R.kmerK = K;
    R.kmerB = B;
    R.pfxExact = (cnt[0] == 0 && cnt[1] == 0) ? 1u : 0u;
      R.pfxDna = (sigma == 4 && cnt['A'] && cnt['C'] && cnt['G'] && cnt['T'] && !env_u32("CMSBWT_PFX_GENERIC", 0)) ? 1u : 0u;
    build_pfx_pair();
  }

  // Child table of the uniform-step walk: ld[k] packs LCP[k] (clipped to 16
  // bits) with D[k] = x[SA[k] + LCP[k]], the first character in which suffix
  // SA[k] differs from SA[k-1], and U[k] = x[SA[k] + LCP[k+1]], the one in
  // which it differs from SA[k+1].  Inside an lcp-interval of depth off the
  // children start at lb and at every k with LCP[k] == off; child j > 0 has
  // character D[start], the first child U[(start of child 1) - 1], so one
  // character of computeMSFactorAt over a small interval needs one window of
  // ld instead of two binary searches (FN:94-149).
  void build_child_table() {
    const uint32_t n = hix.n;
    std::vector<uint32_t> ld((size_t)n + 16, 0);
    auto chr = [&](uint32_t k, int32_t l) -> uint32_t {
      const uint64_t at = (uint64_t)(uint32_t)hix.sa[k] + (uint32_t)std::max<int32_t>(l, 0);
      return at < n ? (uint8_t)hix.x[at] : 0u;
    };
    for (uint32_t k = 0; k < n; k++) {
      const int32_t l = std::max<int32_t>(hix.lcp[k], 0);
      const uint32_t d = k ? chr(k, l) : 0u;
      const uint32_t u = hix.lcp[k + 1] >= 0 ? chr(k, hix.lcp[k + 1]) : 0u;
      ld[k] = (std::min<uint32_t>((uint32_t)l, 0xffffu) << 16) | (d << 8) | u;
    }
    dld.alloc((uint64_t)n + 16);
    HIPCHK(hipMemcpyAsync(dld.p, ld.data(), ((size_t)n + 16) * 4, hipMemcpyHostToDevice, st));
    sync();  // `ld` is pageable
    R.ld = dld.p;
  }

  // Adjacency records of the uniform-step walk (device_common.h): after
  // contractLeft (FN:34-43) and after the skip loop (FN:1187) adjustInterval
  // (FN:11-25) starts at r = psi(lb), psi(rb) or ISA[pos+1]; the record loaded
  // with r holds the 6 LCP entries on either side, so for lengths 1..254 and
  // intervals ending within them the new interval is known in that same load.
  // Entries outside [0, n] are 0 and never decide: LCP[0] = 0 and LCP[n] = -1
  // (stored as 0) end both scans first.
  void build_adjacency_records() {
    R.pr = R.ir = nullptr;
    const uint32_t n = hix.n;
    auto lc = [&](int64_t k) -> uint32_t {
      if (k < 0 || k > (int64_t)n) return 0;
      const int32_t v = hix.lcp[k];
      return v < 0 ? 0u : (uint32_t)std::min<int32_t>(v, 255);
    };
    auto rec = [&](uint32_t r, uint32_t* o) {
      uint32_t w[3] = {0, 0, 0};
      for (int j = 0; j < 6; j++) w[j / 4] |= lc((int64_t)r - j) << (8 * (j % 4));
      for (int j = 0; j < 6; j++) w[(6 + j) / 4] |= lc((int64_t)r + 1 + j) << (8 * ((6 + j) % 4));
      o[0] = r;
      o[1] = w[0];
      o[2] = w[1];
      o[3] = w[2];
    };
    std::vector<uint32_t> pr(4 * ((size_t)n + 16), 0), ir(4 * ((size_t)n + 16), 0);
    for (uint32_t k = 0; k < n; k++) {
      const uint32_t s = (uint32_t)hix.sa[k];
      if (s == n - 1) pr[4 * (size_t)k] = 0xffffffffu;
      else rec(hix.isa[s + 1], &pr[4 * (size_t)k]);
      rec(hix.isa[k], &ir[4 * (size_t)k]);
    }
    dpr.alloc((uint64_t)n + 16);
    dir.alloc((uint64_t)n + 16);
    HIPCHK(hipMemcpyAsync(dpr.p, pr.data(), ((size_t)n + 16) * 16, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dir.p, ir.data(), ((size_t)n + 16) * 16, hipMemcpyHostToDevice, st));
    sync();  // pageable
    R.pr = dpr.p;
    R.ir = dir.p;
  }

  // =====================================================================
  // collection
  void check_bytes(const uint8_t* p, uint64_t len) {
    for (uint64_t i = 0; i < len; i++)
      if (!hix.present[p[i]])
        throw InputError{CMSBWT_EINPUT, "collection byte " + std::to_string((int)p[i]) +
                                            " does not occur in the reference (reference behaviour undefined)"};
  }
  void reset_collection() {
    collLoaded = walked = merged = false;
    plan.valid = false;
    H = K = 0;
  }
  void upload_collection(const Collection& c) {
    if (!refLoaded) throw InputError{CMSBWT_EARG, "load the reference first"};
    auto t0 = std::chrono::steady_clock::now();
    upload_file_end(false);
    reset_collection();
    for (uint64_t d = 0; d < c.ndocs(); d++) {
      uint64_t len = c.off[d + 1] - c.off[d] - 1;
      if (len >= (1ull << 32) - 1) throw InputError{CMSBWT_ELIMIT, "document longer than 2^32 (uint32 positions)"};
      check_bytes(c.text.data() + c.off[d], len);
    }
    dtext.alloc(c.text.size() + kTextPad);
    HIPCHK(hipMemsetAsync(dtext.p + c.text.size(), kSep, kTextPad, st));
    if (!c.text.empty()) HIPCHK(hipMemcpyAsync(dtext.p, c.text.data(), c.text.size(), hipMemcpyHostToDevice, st));
    hdoc = c.off;
    ddoc.alloc(hdoc.size());
    HIPCHK(hipMemcpyAsync(ddoc.p, hdoc.data(), hdoc.size() * 8, hipMemcpyHostToDevice, st));
    sync();
    ndocs = c.ndocs();
    chars = collChars = c.chars;
    sn = c.sn;
    collLoaded = true;
    stats.t_upload_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  // ---- collection file -> HBM, lines resolved on the device (coll_read.hip)
  std::vector<void*> pinned;  // 2 staging buffers per reader thread, kept across calls
  uint64_t pinnedBytes = 0;
  uint64_t collMeta[3] = {0, 0, 0};  // sn, chars, ndocs (parity copies)

  // 2 * nt pinned buffers of CH bytes (reallocated only when the request changes)
  void ensure_pinned(uint32_t nt, uint64_t CH) {
    if (pinned.size() == 2 * nt && pinnedBytes == CH) return;
    for (void* b : pinned) (void)hipHostFree(b);
    pinned.assign(2 * nt, nullptr);
    pinnedBytes = 0;
    for (auto& b : pinned) HIPCHK(hipHostMalloc(&b, CH, hipHostMallocDefault));
    pinnedBytes = CH;
  }

  // pread of the file into pinned buffers by `nt` threads, each DMAing its
  // chunks to dst on its own stream (double-buffered: reading chunk c+2T
  // overlaps the copy of chunk c).  `cancel` (optional) stops the readers
  // between chunks; the call then returns with dst partly written.
  void stream_file(int fd, uint64_t base, uint64_t fsz, uint8_t* dst, const std::atomic<bool>* cancel = nullptr) {
    const uint32_t nt = std::max(1u, std::min(64u, env_u32("CMSBWT_READ_THREADS", 8)));
    ensure_pinned(nt, (uint64_t)std::max(1u, env_u32("CMSBWT_READ_CHUNK_MB", 32)) << 20);
    const uint64_t CH = pinnedBytes;
    const uint64_t nch = (fsz + CH - 1) / CH;
    std::atomic<int> err{0};
    std::vector<std::thread> th;
    for (uint32_t k = 0; k < nt && k < nch; k++)
      th.emplace_back([&, k] {
        hipStream_t s = nullptr;
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool used[2] = {false, false};
        auto ok = [&](hipError_t e) { if (e != hipSuccess) err = 2; return e == hipSuccess; };
        if (ok(hipSetDevice(device)) && ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) &&
            ok(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming)) &&
            ok(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming))) {
          uint32_t it = 0;
          for (uint64_t c = k; c < nch && !err && !(cancel && cancel->load()); c += nt, it++) {
            const int j = it & 1;
            uint8_t* buf = (uint8_t*)pinned[2 * k + j];
            if (used[j] && !ok(hipEventSynchronize(ev[j]))) break;
            const uint64_t off = c * CH, want = std::min(CH, fsz - off);
            uint64_t got = 0;
            while (got < want) {
              ssize_t r = pread(fd, buf + got, want - got, (off_t)(base + off + got));
              if (r <= 0) { err = 1; break; }
              got += (uint64_t)r;
            }
            if (err) break;
            if (!ok(hipMemcpyAsync(dst + off, buf, want, hipMemcpyHostToDevice, s))) break;
            if (!ok(hipEventRecord(ev[j], s))) break;
            used[j] = true;
          }
        }
        if (s) { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); }
        for (auto e : ev) if (e) (void)hipEventDestroy(e);
      });
    for (auto& t : th) t.join();
    if (err == 1) throw InputError{CMSBWT_EIO, "read error on the collection file"};
    if (err) throw HipError{"HIP error while streaming the collection file"};
  }

  // Whole-file upload started ahead of the reference index (cmsbwt_run): the
  // raw bytes stream into HBM on the reader threads' own streams while the
  // index kernels run on the engine stream; load_collection_file_gpu of the
  // same path then only waits for it.  Buffers are allocated here, on the
  // calling thread (the caching allocator is not shared with the readers).
  struct PendingUpload {
    bool on = false;
    std::string path;
    uint64_t fsz = 0;
    DBuf<uint8_t> raw;
    std::thread th;
    std::exception_ptr err;
    std::atomic<bool> cancel{false};
  } pend;
  void upload_file_begin(const std::string& path) {
    upload_file_end(false);
    int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return;  // the load reports the error, after the reference's
    struct stat sbuf;
    if (fstat(fd, &sbuf) != 0) { close(fd); return; }
    const uint64_t fsz = (uint64_t)sbuf.st_size, ntiles = (fsz + kRdTile - 1) / kRdTile;
    pend.raw.alloc(ntiles * kRdTile + kRdTile);
    ensure_pinned(std::max(1u, std::min(64u, env_u32("CMSBWT_READ_THREADS", 8))),
                  (uint64_t)std::max(1u, env_u32("CMSBWT_READ_CHUNK_MB", 32)) << 20);
    pend.on = true;
    pend.path = path;
    pend.fsz = fsz;
    pend.err = nullptr;
    pend.cancel = false;
    uint8_t* dst = pend.raw.p;
    pend.th = std::thread([this, fd, fsz, dst] {
      try {
        stream_file(fd, 0, fsz, dst, &pend.cancel);
      } catch (...) {
        pend.err = std::current_exception();
      }
      close(fd);
    });
  }
  // Wait for a pending upload; with take, hand its buffer over (else stop the
  // readers between chunks and drop it).
  bool upload_file_end(bool take, const std::string& path = "", DBuf<uint8_t>* raw = nullptr, uint64_t* fsz = nullptr) {
    if (!pend.on) return false;
    if (!take || path != pend.path) pend.cancel = true;
    pend.th.join();
    pend.on = false;
    const bool match = take && path == pend.path;
    std::exception_ptr e = pend.err;
    pend.err = nullptr;
    if (match) {
      if (e) std::rethrow_exception(e);
      raw->swap_in(pend.raw);
      *fsz = pend.fsz;
    }
    pend.raw.release();
    return match;
  }

  // Same Collection as read_collection(path, UINT64_MAX) + upload_collection
  // (tests/test_gpu_parity.py::test_gpu_reader_*), produced in HBM.  With a
  // byte range: the documents of bytes [off, off + len) of the file, which
  // must start at a document start (shard_bounds).
  void load_collection_file_gpu(const std::string& path, uint64_t fileOff = 0, uint64_t sliceLen = ~0ull) {
    if (!refLoaded) throw InputError{CMSBWT_EARG, "load the reference first"};
    auto t0 = std::chrono::steady_clock::now();
    reset_collection();
    DBuf<uint8_t> raw;
    uint64_t fsz = 0;
    const bool whole = fileOff == 0 && sliceLen == ~0ull;
    // a pending whole-file upload of another path (or a byte range of this
    // one) must stop before this call's readers use the same pinned buffers
    if (!whole) upload_file_end(false);
    if (!(whole && upload_file_end(true, path, &raw, &fsz))) {
      int fd = open(path.c_str(), O_RDONLY);
      if (fd < 0) throw InputError{CMSBWT_EIO, "Error opening file of sequence (" + path + ")"};
      struct stat sbuf;
      if (fstat(fd, &sbuf) != 0) { close(fd); throw InputError{CMSBWT_EIO, "cannot stat " + path}; }
      fileOff = std::min<uint64_t>(fileOff, (uint64_t)sbuf.st_size);
      fsz = std::min<uint64_t>(sliceLen, (uint64_t)sbuf.st_size - fileOff);  // bytes of this slice
      const uint64_t ntiles0 = (fsz + kRdTile - 1) / kRdTile;
      raw.alloc(ntiles0 * kRdTile + kRdTile);  // tiles read whole; '\n'/'>' lookups one past len
      try {
        stream_file(fd, fileOff, fsz, raw.p);
      } catch (...) {
        close(fd);
        throw;
      }
      close(fd);
    }
    const uint64_t ntiles = (fsz + kRdTile - 1) / kRdTile;
    DBuf<uint64_t> lastNl, carry;
    lastNl.alloc(ntiles + 1);
    carry.alloc(ntiles + 1);
    HIPCHK(hipMemsetAsync(lastNl.p + ntiles, 0, 8, st));
    launch_rd_lastnl(raw.p, fsz, ntiles, lastNl.p, st);
    exscan(lastNl.p, carry.p, (uint64_t)0, ntiles + 1, rocprim::maximum<uint64_t>());
    const uint64_t len = read1(carry.p + ntiles);  // 1 + last '\n': the lines
    const uint64_t nt = (len + kRdTile - 1) / kRdTile;
    DBuf<uint32_t> cnt, seps;
    DBuf<uint64_t> ob, sb;
    cnt.alloc(nt + 1);
    seps.alloc(nt + 1);
    ob.alloc(nt + 1);
    sb.alloc(nt + 1);
    HIPCHK(hipMemsetAsync(cnt.p + nt, 0, 4, st));
    HIPCHK(hipMemsetAsync(seps.p + nt, 0, 4, st));
    launch_rd_count(raw.p, len, nt, carry.p, cnt.p, seps.p, st);
    exscan(cnt.p, ob.p, (uint64_t)0, nt + 1);
    exscan(seps.p, sb.p, (uint64_t)0, nt + 1);
    const uint64_t total = read1(ob.p + nt), nsep = read1(sb.p + nt);
    dtext.alloc(total + 1 + kTextPad);
    ddoc.alloc(nsep + 2);
    HIPCHK(hipMemsetAsync(ddoc.p, 0, 8, st));
    DBuf<uint8_t> pres;
    DBuf<unsigned long long> bad;
    pres.alloc(256);
    bad.alloc(1);
    uint8_t ph[256];
    for (int b = 0; b < 256; b++) ph[b] = hix.present[b] ? 1 : 0;
    HIPCHK(hipMemcpyAsync(pres.p, ph, 256, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(bad.p, 0xff, 8, st));
    launch_rd_emit(raw.p, len, nt, carry.p, ob.p, sb.p, pres.p, dtext.p, ddoc.p, bad.p, st);
    HIPCHK(hipGetLastError());
    std::vector<uint64_t> off(nsep + 1);
    HIPCHK(hipMemcpyAsync(off.data(), ddoc.p, (nsep + 1) * 8, hipMemcpyDeviceToHost, st));
    const unsigned long long badv = read1(bad.p);
    uint64_t size = total, sn = fsz;
    collTail = total > off[nsep];
    if (collTail) {  // tail document (FN:1269-1275)
      const uint64_t e = total + 1;
      HIPCHK(hipMemsetAsync(dtext.p + total, kSep, 1, st));
      off.push_back(e);
      HIPCHK(hipMemcpyAsync(ddoc.p + nsep + 1, &off.back(), 8, hipMemcpyHostToDevice, st));
      size = e;
      if (size < sn - 1) sn = size;
    }
    HIPCHK(hipMemsetAsync(dtext.p + size, kSep, kTextPad, st));
    sync();
    raw.release();
    for (uint64_t d = 0; d + 1 < off.size(); d++)
      if (off[d + 1] - off[d] - 1 >= (1ull << 32) - 1)
        throw InputError{CMSBWT_ELIMIT, "document longer than 2^32 (uint32 positions)"};
    if (badv != ~0ull)
      throw InputError{CMSBWT_EINPUT, "collection byte " + std::to_string((int)(badv & 0xff)) +
                                          " does not occur in the reference (reference behaviour undefined)"};
    hdoc = std::move(off);
    ndocs = hdoc.size() - 1;
    chars = collChars = size - ndocs;
    this->sn = sn;
    collLoaded = true;
    stats.t_upload_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  void load_synth(uint64_t seed, uint64_t copy_begin, uint64_t ncopies, double p, int leadingEmpty) {
    if (!refLoaded) throw InputError{CMSBWT_EARG, "load the reference first"};
    reset_collection();
    // the reference must be the synthetic reference of the same seed: its
    // trimmed length is n - (augmentation) ; recover L from the stored x.
    const uint64_t L = hix.ref_len;
    for (uint64_t k = 0; k < std::min<uint64_t>(L, 4096); k++)
      if ((uint8_t)hix.x[k] != (uint8_t)synth_acgt(synth_base_code(seed, k)))
        throw InputError{CMSBWT_EARG, "loaded reference is not the synthetic reference of this seed"};
    uint64_t base = leadingEmpty ? 1 : 0;
    uint64_t total = base + ncopies * (L + 1);
    dtext.alloc(total + kTextPad);
    HIPCHK(hipMemsetAsync(dtext.p, kSep, total + kTextPad, st));
    launch_synth_collection(dtext.p, L, seed, copy_begin, ncopies, synth_threshold(p), base, st);
    HIPCHK(hipGetLastError());
    hdoc.clear();
    hdoc.push_back(0);
    if (leadingEmpty) hdoc.push_back(1);
    for (uint64_t d = 0; d < ncopies; d++) hdoc.push_back(base + (d + 1) * (L + 1));
    ddoc.alloc(hdoc.size());
    HIPCHK(hipMemcpyAsync(ddoc.p, hdoc.data(), hdoc.size() * 8, hipMemcpyHostToDevice, st));
    sync();
    ndocs = hdoc.size() - 1;
    chars = collChars = ncopies * L;
    sn = total;
    collLoaded = true;
  }

  // =====================================================================
  // MS walk (k_ms_walk2, a uniform-step walk over a chunk queue) + head
  // finalisation
  // lanes of the walk launch: at most 2048 blocks of 256 (chunks are pulled
  // from queues, so lanes beyond the chunk count would idle)
  static constexpr uint32_t kWalkLanes = 256u * 32 * 64;
  // lanes resident at CMSBWT_W2_WAVES waves per SIMD (Makefile: 4)
  static uint64_t resident_lanes() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      int v = 0;
      if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
    }
    return (uint64_t)cus * 4 * 4 * 64;
  }

  uint32_t chunk_size() const {
    if (const char* e = getenv("CMSBWT_CHUNK")) return (uint32_t)std::max(64L, atol(e));
    // queue-fed: about 1.5 chunks per resident lane (CUs x 4 SIMDs x 4 waves
    // x 64; restarts cost, a long last round of chunks costs too).  Config 3
    // (10 GB, 256 CUs): 16 K 16.6 ms, 20 K 16.3, 22-26 K 15.6-15.8, 28 K
    // 16.2, 32 K 16.5, 48 K 18.5 (walk kernel).
    uint64_t c = chars * 2 / (3 * resident_lanes());
    return (uint32_t)std::max<uint64_t>(1024, std::min<uint64_t>(32768, c));
  }

  void ms_walk() {
    if (!collLoaded) throw InputError{CMSBWT_EARG, "load a collection first"};
    auto t0 = std::chrono::steady_clock::now();
    walked = merged = false;
    ndocs = hdoc.size() - 1;  // walk_import may have replaced these with merged totals
    chars = collChars;
    if (ndocs == 0) {
      // No document (an empty file, or one unterminated line that getline().good()
      // drops, FN:1138): no heads and no runs.  A rank of a sharded run may own
      // no documents; a merge over zero heads in total is rejected in merge().
      H = 0;
      hStart.alloc(0); hPos.alloc(0); hLen.alloc(0); hIsa.alloc(0); hTonext.alloc(0);
      hSmall.alloc(0); hChar.alloc(0); hNext.alloc(0);
      diff.alloc((uint64_t)R.n + 1);
      diff.zero(st);
      hasHead.alloc(R.n);
      hasHead.zero(st);
      sync();
      runsValid = true;
      orderInvariant = true;
      walked = true;
      stats.order_invariant = 1;
      stats.heads = 0;
      stats.ndocs = 0;
      stats.chars = chars;
      stats.sn = sn;
      stats.ms_walk_kernel_ms = 0;
      stats.t_ms_walk_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      return;
    }
    const uint32_t C = chunk_size();
    if (!plan.valid || plan.C != C) build_plan(C);
    const uint32_t nch = plan.nch;
    DBuf<uint32_t> chunkCount, used, nextChunk;
    chunkCount.alloc(nch);
    used.alloc(1);
    nextChunk.alloc(16 * 8);
    DBuf<unsigned long long> w2stats;  // CMSBWT_W2_STATS=1: step counts of the uniform-step walk
    if (env_u32("CMSBWT_W2_STATS", 0)) {
      w2stats.alloc(32);
      w2stats.zero(st);
    }
    // pool sized for the head density of the previous walk on this engine
    // (3 % at first) + one partial block per chunk; an overflow re-runs the
    // walk with the measured size, so only the first walk of a denser
    // workload pays twice (1 % SNP collections have ~10 % heads)
    if (!densityLearned && nch >= 4096) sample_density(nch);
    // lanes launched: the resident ones (chunks come from queues, so a lane
    // beyond them would only wait for a CU); each may end holding up to
    // kPoolBatch - 1 reserved blocks it never started (config 3: 262 K lanes
    // x 15 x 16 heads x 16 B = 1.0 GB of slack against 1.6 GB of heads)
    const uint32_t lanes = (uint32_t)std::min<uint64_t>({(uint64_t)kWalkLanes, resident_lanes(), (uint64_t)nch});
    const uint64_t slack = (uint64_t)lanes * (kPoolBatch - 1);
    uint64_t cap = (uint64_t)nch + slack + (uint64_t)((double)chars * poolDensity * 1.1) / kPoolB + 1024;
    DBuf<HeadRec> rec;
    DBuf<uint2> blkMeta;
    uint32_t usedBlocks = 0;
    while (true) {
      if (cap > 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "head pool exceeds 2^32 blocks"};
      rec.alloc(cap * kPoolB);
      blkMeta.alloc(cap);
      used.zero(st);
      nextChunk.zero(st);
      HIPCHK(hipMemsetAsync(blkMeta.p, 0xff, cap * 8, st));
      Pool pool{rec.p, blkMeta.p, used.p, (uint32_t)cap};
      HIPCHK(hipEventRecord(ev0, st));
      launch_ms_walk2(R, dtext.p, ddoc.p, plan.dch.p, nch, plan.bandOrder.p, plan.bandStart.p, plan.nbands,
                      nextChunk.p, pool, chunkCount.p, lanes, w2stats.p, st);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(ev1, st));
      usedBlocks = read1(used.p);
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, ev0, ev1));
      stats.ms_walk_kernel_ms = ms;
      if (usedBlocks <= cap) break;
      cap = (uint64_t)usedBlocks + (uint64_t)nch + slack + 1024;
    }
    if (w2stats.p) {
      static const char* names[32] = {"done", "next", "bs_text", "bs_sa", "bs_x", "fail_sa", "lce_sa", "lce",
                                       "skip1", "skip0", "gallop", "skipbs", "isa1", "conp", "ext1", "adj",
                                       "pfx_text", "pfx_probe", "ext_a", "ext_b", "sktxt", "ivl", "lce_coop",
                                       "c_adj0", "c_adv", "c_post", "scan0", "scan1", "scan2", "scan3", "wave_steps",
                                       "coop_steps"};
      std::vector<unsigned long long> h(32);
      HIPCHK(hipMemcpy(h.data(), w2stats.p, 32 * 8, hipMemcpyDeviceToHost));
      for (int k = 0; k < 32; k++)
        if (h[k]) fprintf(stderr, "[w2stats] %-10s %llu\n", names[k] ? names[k] : "?", h[k]);
    }
    // chunk bases (end phrase counted in the last chunk of each document)
    DBuf<unsigned long long> withEnd, chunkBase;
    withEnd.alloc(nch);
    chunkBase.alloc(nch);
    launch_chunk_with_end(plan.dch.p, chunkCount.p, nch, withEnd.p, st);
    exscan(withEnd.p, chunkBase.p, 0ull, nch);
    {
      const unsigned long long tot = sum2(chunkBase.p + (nch - 1), withEnd.p + (nch - 1));
      // uint32 head indices and labels (1 .. H + 1): the reference's int32
      // limit (FN:1436-1437, 1456) is lifted to 2^32 - 2 heads
      if (tot >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "more than 2^32-2 heads (uint32 head indices)"};
      H = (uint32_t)tot;
    }
    if (chars) {  // head density for the next walk's pool
      poolDensity = std::max(1.0 / 32, (double)H / (double)chars);
      densityLearned = true;
    }
    hStart.alloc(H); hPos.alloc(H); hLen.alloc(H); hIsa.alloc(H); hTonext.alloc(H);
    hSmall.alloc(H); hChar.alloc(H); hNext.alloc(H);
    HeadsSoA h = heads();
    Pool pool{rec.p, blkMeta.p, used.p, (uint32_t)cap};
    DBuf<uint32_t> hDoc;  // document of each head (finalize)
    hDoc.alloc(H);
    launch_scatter_heads(pool, usedBlocks, chunkCount.p, chunkBase.p, h, plan.dch.p, dtext.p, ddoc.p, hDoc.p, st);
    DBuf<uint32_t> docEnd;
    docEnd.alloc(ndocs);
    launch_end_phrases(dtext.p, ddoc.p, (uint32_t)ndocs, plan.dLast.p, chunkCount.p, chunkBase.p, R.n, h, docEnd.p,
                       hDoc.p, st);
    DBuf<uint32_t> errf;
    errf.alloc(1);
    errf.zero(st);
    DBuf<uint32_t> isax;
    const bool packIsax = R.n < (1u << 24) && !env_u32("CMSBWT_NO_ISAX", 0);
    if (packIsax) {
      isax.alloc(R.n);
      launch_isax(R.isa, R.x, R.n, isax.p, st);
    }
    launch_finalize(R, h, H, docEnd.p, (uint32_t)ndocs, dtext.p, ddoc.p, errf.p, hDoc.p, st,
                    packIsax ? isax.p : nullptr);
    HIPCHK(hipGetLastError());
    // run buckets (diff, hasHead): from the grouping's position sort in
    // merge(), or through position bins on demand (ensure_runs)
    runsValid = false;
    if (env_u32("CMSBWT_RUN_BIN_SHIFT", 0) || env_u32("CMSBWT_RUN_BIN_GLOBAL", 0)) ensure_runs();
    uint32_t ef = read1(errf.p);
    // The comparator is provably consistent when every isaNext suffix starts
    // with its head's mismatch byte (k_finalize) and `smaller` follows the
    // unsigned byte order the suffix array uses: FN:55 compares signed chars,
    // so a reference byte >= 0x80 can make a singleton mismatch's `smaller`
    // disagree with isaNext and forces the checked merge.
    bool highBytes = false;
    for (int c = 0x80; c < 256; c++) highBytes |= hix.present[c];
    orderInvariant = (ef & 8u) == 0 && !highBytes;
    if (ef & 1) throw InputError{CMSBWT_EINPUT, "internal: match ends not monotone inside a document"};
    if (ef & 6) throw InputError{CMSBWT_EINPUT, "isaNext/run index outside the reference (reference UB)"};
    walked = true;
    stats.order_invariant = orderInvariant ? 1 : 0;
    stats.heads = H;
    stats.ndocs = ndocs;
    stats.chars = chars;
    stats.sn = sn;
    stats.t_ms_walk_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  // Restart chunks of the loaded collection; rebuilt when the collection or
  // the chunk size changes.
  struct ChunkPlan {
    bool valid = false;
    uint32_t C = 0, nch = 0;
    DBuf<Chunk> dch;
    DBuf<uint32_t> dLast;
    DBuf<uint32_t> bandOrder, bandStart;  // uniform-step walk: chunks grouped by offset band
    uint32_t nbands = 1;
  } plan;

  void build_plan(uint32_t C) {
    std::vector<Chunk> chunks;
    std::vector<uint32_t> lastChunk(ndocs);
    for (uint64_t d = 0; d < ndocs; d++) {
      uint64_t L = hdoc[d + 1] - hdoc[d] - 1;
      uint64_t nc = std::max<uint64_t>(1, (L + C - 1) / C);
      for (uint64_t k = 0; k < nc; k++) {
        Chunk ch;
        ch.doc = (uint32_t)d;
        ch.a = (uint32_t)(k * C);
        ch.b = (uint32_t)std::min<uint64_t>(L, (k + 1) * C);
        ch.last = k + 1 == nc;
        chunks.push_back(ch);
      }
      lastChunk[d] = (uint32_t)chunks.size() - 1;
    }
    const uint32_t nch = (uint32_t)chunks.size();
    plan.dch.alloc(nch);
    HIPCHK(hipMemcpyAsync(plan.dch.p, chunks.data(), nch * sizeof(Chunk), hipMemcpyHostToDevice, st));
    plan.dLast.alloc(ndocs);
    HIPCHK(hipMemcpyAsync(plan.dLast.p, lastChunk.data(), ndocs * 4, hipMemcpyHostToDevice, st));
    // Offset bands for the uniform-step walk: band = 8 * a / docLen, chunks of
    // a band in document order.  Copies of the reference then keep an XCD's
    // x / ISA / PLCP accesses inside one eighth of the reference.
    const uint32_t nb = 8;
    std::vector<uint32_t> bandCnt(nb + 1, 0), bandOf(nch);
    for (uint32_t c = 0; c < nch; c++) {
      const uint64_t L = hdoc[chunks[c].doc + 1] - hdoc[chunks[c].doc] - 1;
      bandOf[c] = L ? (uint32_t)std::min<uint64_t>(nb - 1, (uint64_t)chunks[c].a * nb / L) : 0;
      bandCnt[bandOf[c] + 1]++;
    }
    for (uint32_t k = 0; k < nb; k++) bandCnt[k + 1] += bandCnt[k];
    std::vector<uint32_t> bandOrd(nch), fillp(bandCnt.begin(), bandCnt.end() - 1);
    for (uint32_t c = 0; c < nch; c++) bandOrd[fillp[bandOf[c]]++] = c;
    plan.bandOrder.alloc(nch);
    HIPCHK(hipMemcpyAsync(plan.bandOrder.p, bandOrd.data(), nch * 4, hipMemcpyHostToDevice, st));
    plan.bandStart.alloc(nb + 1);
    HIPCHK(hipMemcpyAsync(plan.bandStart.p, bandCnt.data(), (nb + 1) * 4, hipMemcpyHostToDevice, st));
    plan.nbands = nb;
    sync();
    plan.C = C;
    plan.nch = nch;
    plan.valid = true;
  }

  // Run buckets (FN:1162-1171, 1203) through position bins, no random
  // atomics: head i covers [pos_i, pos_i + start_{i+1} - start_i).
  bool runsValid = false;
  void ensure_runs() {
    if (runsValid) return;
    HeadsSoA h = heads();
    diff.alloc((uint64_t)R.n + 1);
    hasHead.alloc(R.n);
    {
      // CMSBWT_RUN_BIN_SHIFT / CMSBWT_RUN_BIN_GLOBAL: smaller bins and the
      // global-counter path, for the tests
      const uint32_t sh = std::max(1u, std::min(kRunBinShift, env_u32("CMSBWT_RUN_BIN_SHIFT", kRunBinShift)));
      const bool global = env_u32("CMSBWT_RUN_BIN_GLOBAL", 0) != 0;
      const uint32_t nb = (R.n >> sh) + 1;
      DBuf<uint32_t> binCnt, binOff, binCur, vals;
      binCnt.alloc((uint64_t)nb + 1);
      binCnt.zero(st);
      binOff.alloc((uint64_t)nb + 1);
      binCur.alloc(nb);
      vals.alloc(2ull * H + 1);
      launch_run_bin_count(h, H, R.n, nb, sh, global, binCnt.p, st);
      exscan(binCnt.p, binOff.p, 0u, (uint64_t)nb + 1);
      HIPCHK(hipMemcpyAsync(binCur.p, binOff.p, (uint64_t)nb * 4, hipMemcpyDeviceToDevice, st));
      launch_run_bin_scatter(h, H, R.n, nb, sh, global, binCur.p, vals.p, st);
      launch_run_bin_emit(vals.p, binOff.p, R.n, nb, sh, diff.p, hasHead.p, st);
      HIPCHK(hipGetLastError());
    }
    runsValid = true;
  }

  HeadsSoA heads() {
    return HeadsSoA{hStart.p, hPos.p, hLen.p, hSmall.p, hChar.p, hIsa.p, hTonext.p, hNext.p};
  }

  // =====================================================================
  // merge
  // Items of a set of heads (FN:1387-1416): the members sorted by (pos, len,
  // isaNext, idx), one item per distinct key in map order (match.h:27-33),
  // slots (prefixSumForPositions, FN:1504-1515), per-position item ranges.
  struct ItemSet {
    uint32_t K = 0;
    bool slotIsFirst = false;  // slot[q] == first[q]: P is already slot-major
    DBuf<uint32_t> P;  // member (head index) of each sorted head
    DBuf<uint32_t> pos, len, isa, until, count, first, slot;  // map order; slot has K+1 entries
    DBuf<uint8_t> small;
    DBuf<unsigned long long> sk;
    DBuf<uint32_t> posBegin, posF;  // n+1, n
    ItemsSoA soa() { return ItemsSoA{pos.p, len.p, isa.p, small.p, until.p, count.p, first.p, slot.p, nullptr, sk.p}; }
  };
  void group_items(const HeadsSoA& h, uint32_t H, uint32_t n, ItemSet& S) {
    const int bN = bits_for(n);
    // ---- grouping: perm sorted by (pos, len, isaNext, idx)   FN:1387-1416
    const int bL = bits_for(max_u32(h.len, H));
    const bool packed = 2 * bN + bL <= 64 && !env_u32("CMSBWT_GROUP3", 0);
    DBuf<uint32_t> perm, key, key2;
    DBuf<uint32_t>& perm2 = S.P;
    perm.alloc(H); perm2.alloc(H); key.alloc(H); key2.alloc(H);
    DBuf<unsigned long long> gk, gk2;
    DBuf<uint32_t> tsS;  // position-first path: tonext and smaller of each sorted head
    DBuf<uint8_t> smS;
    const bool posFirst = packed && !env_u32("CMSBWT_GROUP64", 0);
    if (!posFirst) mk_iota(perm.p, H, st);
    if (posFirst) {
      // position first: one stable radix sort by pos (3 passes of 8 bits at
      // n = 1e7) carrying (idx, len, isaNext), then each position's segment
      // (~10 heads) sorted by (len, isaNext); long segments by a radix sort
      gk2.alloc(H);
      {
        DBuf<uint32_t> posS, hb;
        DBuf<HeadKV> kv;
        posS.alloc(H); kv.alloc(H); hb.alloc((uint64_t)n + 1);
        auto kvIn = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint32_t>(0u),
                                                     MakeHeadKV{h.len, h.isa, h.smaller, h.tonext});
        size_t b = 0;
#if CMSBWT_POS_SORT_BITS
        // wider digits: ceil(bN / bits) onesweep passes instead of ceil(bN / 8)
        using PosCfg = rocprim::radix_sort_config<
            rocprim::default_config, rocprim::default_config,
            rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                                rocprim::kernel_config<256, CMSBWT_POS_SORT_IPT>,
                                                CMSBWT_POS_SORT_BITS>>;
        HIPCHK(rocprim::radix_sort_pairs<PosCfg>(nullptr, b, h.pos, posS.p, kvIn, kv.p, (size_t)H, 0u, (unsigned)bN,
                                                 st));
        HIPCHK(rocprim::radix_sort_pairs<PosCfg>(scratch(b), b, h.pos, posS.p, kvIn, kv.p, (size_t)H, 0u,
                                                 (unsigned)bN, st));
#else
        HIPCHK(rocprim::radix_sort_pairs(nullptr, b, h.pos, posS.p, kvIn, kv.p, (size_t)H, 0u, (unsigned)bN, st));
        HIPCHK(rocprim::radix_sort_pairs(scratch(b), b, h.pos, posS.p, kvIn, kv.p, (size_t)H, 0u, (unsigned)bN, st));
#endif
        dmt("g.pos_sort");
        mk_pos_begin(posS.p, H, n, hb.p, st);
        // run buckets from the sorted heads: starts per position from hb,
        // ends counted in k_grp_seg (LDS histogram near the block's positions)
        // (CMSBWT_GRP_RUNS=0: the position-bin path of ensure_runs instead)
        const bool runsHere = !runsValid && env_u32("CMSBWT_GRP_RUNS", 1) != 0;
        if (runsHere) {
          diff.alloc((uint64_t)n + 1);
          hasHead.alloc(n);
          mk_run_starts(hb.p, n, diff.p, hasHead.p, st);
        }
        DBuf<uint32_t> bigList;
        bigList.alloc((uint64_t)n + 1);
        HIPCHK(hipMemsetAsync(bigList.p, 0, 4, st));
        tsS.alloc(H); smS.alloc(H);
        mk_grp_seg(posS.p, hb.p, kv.p, H, bN, bL, gk2.p, perm2.p, tsS.p, smS.p, bigList.p,
                   env_u32("CMSBWT_GROUP_SMALL", 64), runsHere ? diff.p : nullptr, n, st);
        if (runsHere) runsValid = true;
        dmt("g.grp_seg");
        kv.release();
        posS.release();
        const uint32_t nb = read1(bigList.p);
        if (nb) {
          DBuf<uint32_t> bpos, sz, off;
          bpos.alloc(nb); sz.alloc(nb); off.alloc(nb);
          sort_keys(bigList.p + 1, bpos.p, nb, bN);
          mk_grp_big_sizes(bpos.p, nb, hb.p, sz.p, st);
          exscan(sz.p, off.p, 0u, nb);
          const uint32_t B = (uint32_t)sum2(off.p + (nb - 1), sz.p + (nb - 1));
          DBuf<uint32_t> bidx, pB, pB2;
          DBuf<unsigned long long> kB, kB2;
          bidx.alloc(B); pB.alloc(B); pB2.alloc(B); kB.alloc(B); kB2.alloc(B);
          mk_grp_big_expand(bpos.p, nb, hb.p, off.p, bidx.p, st);
          mk_gather_kp(bidx.p, B, gk2.p, perm2.p, kB.p, pB.p, st);
          sort_pairs(kB.p, kB2.p, pB.p, pB2.p, B, 2 * bN + bL);  // stable: idx order kept per key
          mk_scatter_kp(bidx.p, B, kB2.p, pB2.p, gk2.p, perm2.p, st);
          mk_grp_big_fields(bidx.p, B, perm2.p, h, tsS.p, smS.p, st);
          // their members in map order too (k_grp_seg ranks the others so)
          DBuf<uint8_t> tS;
          tS.alloc(B);
          mk_grp_big_maporder(bpos.p, nb, hb.p, off.p, gk2.p, perm2.p, tsS.p, smS.p, kB.p, pB.p, pB2.p, tS.p, bidx.p,
                              bN, st);
        }
      }
    } else if (packed) {  // one sort on the composite key
      gk.alloc(H); gk2.alloc(H);
      mk_group_key(h, H, bN, bL, gk.p, st);
      sort_pairs(gk.p, gk2.p, perm.p, perm2.p, H, 2 * bN + bL);
      gk.release();
    } else {       // LSD: isaNext, len, pos
      mk_gather(h.isa, perm.p, key.p, H, st);
      sort_pairs(key.p, key2.p, perm.p, perm2.p, H, bN);
      mk_gather(h.len, perm2.p, key.p, H, st);
      sort_pairs(key.p, key2.p, perm2.p, perm.p, H, bL);
      mk_gather(h.pos, perm.p, key.p, H, st);
      sort_pairs(key.p, key2.p, perm.p, perm2.p, H, bN);
    }
    perm.release();
    dmt("g.big");
    DBuf<uint32_t>& P = perm2;  // sorted members
    // items
    uint32_t K = 0;
    if (H) {
      if (packed) mk_item_flags64(gk2.p, key.p, H, st);
      else mk_item_flags(P.p, h, key.p, H, st);
      inscan(key.p, key2.p, H, rocprim::plus<uint32_t>());
      K = read1(key2.p + (H - 1));
    }
    S.K = K;
    DBuf<uint32_t> aPos, aLen, aIsa, aUntil, aCount, aFirst;
    DBuf<uint8_t> aSmall;
    aPos.alloc(K); aLen.alloc(K); aIsa.alloc(K); aUntil.alloc(K); aCount.alloc(K); aFirst.alloc(K);
    aSmall.alloc(K);
    ItemsSoA A0{aPos.p, aLen.p, aIsa.p, aSmall.p, aUntil.p, aCount.p, aFirst.p, nullptr, nullptr, nullptr};
    if (packed) mk_item_fill64(gk2.p, P.p, key.p, key2.p, h, posFirst ? tsS.p : nullptr, smS.p, H, bN, bL, A0, st);
    else mk_item_fill(P.p, key.p, key2.p, h, H, A0, st);
    gk2.release();
    tsS.release(); smS.release();
    mk_item_count(aFirst.p, aCount.p, K, H, st);
    key.release();
    key2.release();
    // map order inside each position (match.h:27-33): the position-first
    // grouping ranked the members in map order already; the composite-key
    // sorts give (len, isaNext) order and one thread per position reorders
    // its items
    DBuf<uint32_t> pbA, order;
    pbA.alloc((uint64_t)n + 1);
    mk_pos_begin(aPos.p, K, n, pbA.p, st);
    S.slotIsFirst = posFirst;  // items and their members share one order
    if (posFirst) {
      S.pos.swap_in(aPos); S.len.swap_in(aLen); S.isa.swap_in(aIsa); S.until.swap_in(aUntil);
      S.count.swap_in(aCount); S.first.swap_in(aFirst); S.small.swap_in(aSmall);
      S.slot.alloc((uint64_t)K + 1); S.sk.alloc(K);
    } else {
      order.alloc(K);
      mk_map_order(pbA.p, aLen.p, aSmall.p, n, order.p, st);
      S.pos.alloc(K); S.len.alloc(K); S.isa.alloc(K); S.until.alloc(K); S.count.alloc(K); S.first.alloc(K);
      S.slot.alloc((uint64_t)K + 1); S.small.alloc(K); S.sk.alloc(K);
      ItemsSoA SS0 = S.soa();
      mk_item_permute(A0, order.p, SS0, K, st);
    }
    ItemsSoA SS = S.soa();
    mk_item_sk(SS, K, st);
    dmt("g.items");
    order.release();
    aPos.release(); aLen.release(); aIsa.release(); aUntil.release(); aCount.release(); aFirst.release();
    aSmall.release();
    // slots = prefixSumForPositions (FN:1504-1515)
    exscan(S.count.p, S.slot.p, 0u, K);
    {
      uint32_t hh = H;
      HIPCHK(hipMemcpyAsync(S.slot.p + K, &hh, 4, hipMemcpyHostToDevice, st));
      sync();  // hh is a stack variable
    }
    S.posBegin.swap_in(pbA);  // positions are unchanged by the reordering
    S.posF.alloc(n);
    mk_pos_f(S.pos.p, S.small.p, S.posBegin.p, K, n, S.posF.p, st);
  }

  // FN:1480-1494 sort of each item's next-head ranks (slot order): small
  // items by an in-place insertion sort, large ones by one global (item, nhr) sort
  void sort_nhr_items(const ItemsSoA& S, uint32_t K, const uint32_t* itemOfSlotP, uint32_t* nhrP, uint32_t H,
                      bool smallDone = false) {
    (void)itemOfSlotP;
    (void)H;
    DBuf<uint32_t> bigList;
    bigList.alloc((uint64_t)K + 1);
    HIPCHK(hipMemsetAsync(bigList.p, 0, 4, st));
    if (smallDone) mk_nhr_big_list(S, K, bigList.p, st);  // items <= kSmallSeg ranked by k_nhr_rank
    else mk_nhr_sort_small(S, K, nhrP, bigList.p, st);
    const uint32_t nb = K ? read1(bigList.p) : 0;
    if (!nb) return;
    // the large items in item order, their members at exclusive offsets
    DBuf<uint32_t> items, cnt, off;
    items.alloc(nb); cnt.alloc(nb); off.alloc(nb);
    sort_keys(bigList.p + 1, items.p, nb, bits_for(K));
    mk_item_counts_of(items.p, nb, S.count, cnt.p, st);
    exscan(cnt.p, off.p, 0u, nb);
    const uint32_t B = (uint32_t)sum2(off.p + (nb - 1), cnt.p + (nb - 1));
    DBuf<unsigned long long> bk, bk2;
    DBuf<uint32_t> bslots;
    bk.alloc(B); bk2.alloc(B); bslots.alloc(B);
    mk_nhr_big_fill(items.p, off.p, nb, S, nhrP, bk.p, bslots.p, st);
    sort_keys(bk.p, bk2.p, B, 32 + bits_for(K));
    mk_nhr_big_back(bk2.p, bslots.p, B, nhrP, st);
  }

  // counterSmallerThanHead (FN:1523-1603) over the target positions [P0, P1):
  // windows of positions whose slots fit the LDS budget, items reaching into a
  // window from the left in its crossing list (items before P0 included).
  struct WinPlan {
    bool tgt = false;
    uint32_t nw = 0, ncross = 0, slotCap = 0;
    DBuf<uint32_t> winStart, crossOff, crossList, wflag, wincl, crossCnt, itemOff, keyW, keyW2, valQ;
    DBuf<uint4> irec;  // target-major kernel: packed item fields
  };
  void counter_phase(const ItemsSoA& S, uint32_t K, const uint32_t* posBegin, const uint32_t* posF,
                     const uint32_t* nhrP, unsigned long long* counterP, unsigned long long* cstatsP, uint32_t n,
                     uint32_t P0, uint32_t P1, bool check, const HostRoute* hr = nullptr) {
    // checked queries without a host route: nothing masked, ambiguity only counted
    HostRoute none;
    DBuf<uint8_t> noneMask, noneAmb;
    DBuf<unsigned long long> noneCnt;
    if (check && !hr) {
      noneMask.alloc(n); noneMask.zero(st);
      noneAmb.alloc(n);
      noneCnt.alloc(1); noneCnt.zero(st);
      none = HostRoute{noneMask.p, noneAmb.p, nullptr, noneCnt.p, 0};
      hr = &none;
    }
    WinPlan W;
    win_prep(S, K, posBegin, n, P0, P1, check, cstatsP, W);
    dmt("win_prep");
    counter_run(W, S, posBegin, posF, nhrP, counterP, cstatsP, n, check, hr);
    sync();
    counter_time();
  }
  // the windows and crossing lists (one read-back: the crossing count)
  void win_prep(const ItemsSoA& S, uint32_t K, const uint32_t* posBegin, uint32_t n, uint32_t P0, uint32_t P1,
                bool check, unsigned long long* cstatsP, WinPlan& W) {
    // target-major kernel (default): windows of 256 targets, slots unbounded;
    // k_counter_win (checked queries, or CMSBWT_COUNTER_WIN=1): windows cut
    // by the LDS slot budget
    W.tgt = !check && !env_u32("CMSBWT_COUNTER_WIN", 0);
    const uint32_t winPos = W.tgt ? std::max(1u, std::min(256u, env_u32("CMSBWT_TGTWIN", 256)))
                                  : std::min(1024u, env_u32("CMSBWT_WINPOS", 1024));
    W.slotCap = std::min(3584u, env_u32("CMSBWT_WINSLOTS", 3584));  // kWinSlots (merge.hip)
    W.wincl.alloc(n);
    if (W.tgt) {
      // fixed windows of winPos targets: their starts and the inclusive
      // window count of every position need no scan
      W.nw = P1 > P0 ? (P1 - P0 + winPos - 1) / winPos : 0;
      W.winStart.alloc((uint64_t)W.nw + 1);
      mk_win_fixed(n, P0, P1, winPos, W.nw, W.wincl.p, W.winStart.p, st);
    } else {
      W.wflag.alloc(n);
      mk_win_flags(posBegin, S.slot, n, P0, P1, std::max(1u, winPos), W.slotCap, W.wflag.p, st);
      inscan(W.wflag.p, W.wincl.p, n, rocprim::plus<uint32_t>());
      W.nw = P1 > P0 ? read1(W.wincl.p + (n - 1)) : 0;
      W.winStart.alloc((uint64_t)W.nw + 1);
      mk_win_starts(W.wflag.p, W.wincl.p, n, W.winStart.p, st);
      mk_set_u32(W.winStart.p + W.nw, P1, st);
    }
    dmt("w.windows");
    // crossing lists: (window, item) pairs sorted by window
    W.crossCnt.alloc(K);
    mk_win_cross(S, K, W.wincl.p, n, W.crossCnt.p, nullptr, nullptr, nullptr, cstatsP + 4, 0, st);
    // fixed windows: the lists placed by distance without a sort (merge.hip
    // k_xw_*; CMSBWT_XW_SORT=1 keeps the sort of the (window, item) pairs)
    if (W.tgt && K && W.nw && !env_u32("CMSBWT_XW_SORT", 0) && cross_place(S, K, posBegin, P0, W)) return;
    W.itemOff.alloc(K);
    exscan(W.crossCnt.p, W.itemOff.p, 0u, K);
    W.ncross = K ? (uint32_t)sum2(W.itemOff.p + (K - 1), W.crossCnt.p + (K - 1)) : 0;
    dmt("w.cross_count");
    W.keyW.alloc(std::max<uint32_t>(W.ncross, 1));
    W.keyW2.alloc(std::max<uint32_t>(W.ncross, 1));
    W.valQ.alloc(std::max<uint32_t>(W.ncross, 1));
    W.crossList.alloc(std::max<uint32_t>(W.ncross, 1));
    mk_win_cross(S, K, W.wincl.p, n, W.crossCnt.p, W.itemOff.p, W.keyW.p, W.valQ.p, cstatsP + 4, 1, st);
    dmt("w.cross_fill");
    sort_pairs(W.keyW.p, W.keyW2.p, W.valQ.p, W.crossList.p, W.ncross, bits_for(W.nw));
    dmt("w.cross_sort");
    W.crossOff.alloc((uint64_t)W.nw + 1);
    mk_win_cross_off(W.keyW2.p, W.ncross, W.nw, W.crossOff.p, st);
    if (W.tgt && !env_u32("CMSBWT_NO_IREC", 0)) {
      W.irec.alloc(std::max<uint32_t>(K, 1));
      mk_item_rec(S, K, W.irec.p, st);
    }
  }
  // crossing lists of the fixed windows by distance (merge.hip k_xw_*):
  // sources sv = 0 .. nw (0: items before P0, else window sv - 1); false when
  // a source is deeper than kXwMaxDepth windows (the sort path then runs)
  bool cross_place(const ItemsSoA& S, uint32_t K, const uint32_t* posBegin, uint32_t P0, WinPlan& W) {
    const uint32_t nw = W.nw, nsv = nw + 1;
    DBuf<uint32_t> depth, toff, mx;
    depth.alloc(nsv);
    toff.alloc(nsv);
    mk_xw_depth(posBegin, W.winStart.p, P0, nsv, W.crossCnt.p, depth.p, st);
    exscan(depth.p, toff.p, 0u, nsv);
    uint32_t maxDepth = 0;
    {
      mx.alloc(1);
      size_t b = 0;
      HIPCHK(rocprim::reduce(nullptr, b, depth.p, mx.p, 0u, (size_t)nsv, rocprim::maximum<uint32_t>(), st));
      HIPCHK(rocprim::reduce(scratch(b), b, depth.p, mx.p, 0u, (size_t)nsv, rocprim::maximum<uint32_t>(), st));
      maxDepth = read1(mx.p);
    }
    if (maxDepth > kXwMaxDepth) return false;
    const uint64_t nT = sum2(toff.p + (nsv - 1), depth.p + (nsv - 1));
    DBuf<uint32_t> T, segOff, count;
    T.alloc(std::max<uint64_t>(nT, 1));
    segOff.alloc(std::max<uint64_t>(nT, 1));
    count.alloc((uint64_t)nw + 1);
    mk_xw_hist(posBegin, W.winStart.p, P0, nsv, W.crossCnt.p, depth.p, toff.p, T.p, st);
    mk_xw_count(depth.p, toff.p, T.p, nw, maxDepth, segOff.p, count.p, st);
    HIPCHK(hipMemsetAsync(count.p + nw, 0, 4, st));
    W.crossOff.alloc((uint64_t)nw + 1);
    exscan(count.p, W.crossOff.p, 0u, (uint64_t)nw + 1);
    const uint64_t nc = read1(W.crossOff.p + nw);
    if (nc >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "crossing list longer than 2^32"};
    W.ncross = (uint32_t)nc;
    W.crossList.alloc(std::max<uint32_t>(W.ncross, 1));
    mk_xw_place(posBegin, W.winStart.p, P0, nsv, W.crossCnt.p, depth.p, toff.p, segOff.p, W.crossOff.p,
                W.crossList.p, st);
    dmt("w.cross_place");
    if (W.tgt && !env_u32("CMSBWT_NO_IREC", 0)) {
      W.irec.alloc(std::max<uint32_t>(K, 1));
      mk_item_rec(S, K, W.irec.p, st);
    }
    return true;
  }
  // the counter kernel between ev0 and ev1 (no synchronisation; counter_time
  // reads the duration once the stream has passed ev1)
  void counter_run(WinPlan& W, const ItemsSoA& S, const uint32_t* posBegin, const uint32_t* posF,
                   const uint32_t* nhrP, unsigned long long* counterP, unsigned long long* cstatsP, uint32_t n,
                   bool check, const HostRoute* hr, EqList eq = EqList{}) {
    HIPCHK(hipEventRecord(ev0, st));
    if (eq.rec && !W.tgt) throw InputError{CMSBWT_EINTERNAL, "internal: equal-key listing needs the target-major counter"};
    if (W.tgt)
      mk_counter_tgt(S, posBegin, posF, nhrP, W.winStart.p, W.nw, W.crossOff.p, W.crossList.p, counterP, cstatsP,
                     n, st, eq, W.irec.p);
    else
      mk_counter_win(S, posBegin, posF, nhrP, W.winStart.p, W.nw, W.crossOff.p, W.crossList.p, counterP, cstatsP,
                     n, W.slotCap, check ? hr : nullptr, st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev1, st));
    windows = W.nw;
    crossings = W.ncross;
  }
  void counter_time() {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev0, ev1));
    counter_kernel_ms = ms;
  }

  // ---- comparator-ambiguity fallback (map_replay.h)
  template <class T_>
  std::vector<T_> down(const T_* d, uint64_t k) {
    std::vector<T_> v(k);
    if (k) HIPCHK(hipMemcpyAsync(v.data(), d, k * sizeof(T_), hipMemcpyDeviceToHost, st));
    sync();
    return v;
  }
  template <class T_>
  void up(DBuf<T_>& b, const std::vector<T_>& v) {
    b.alloc(v.size());
    if (!v.empty()) HIPCHK(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T_), hipMemcpyHostToDevice, st));
    sync();
  }
  HostItems download_items(ItemSet& IS, uint32_t n) {
    HostItems I;
    const uint32_t k = IS.K;
    I.pos = down(IS.pos.p, k); I.len = down(IS.len.p, k); I.isa = down(IS.isa.p, k);
    I.until = down(IS.until.p, k); I.count = down(IS.count.p, k); I.first = down(IS.first.p, k);
    I.small = down(IS.small.p, k);
    I.P = down(IS.P.p, H);
    I.posBegin = down(IS.posBegin.p, (uint64_t)n + 1);
    return I;
  }
  // Rebuild the items of the flagged positions from a host std::map replay of
  // their insertions (FN:1401-1414); every array derived from the items is
  // recomputed (K may change).
  void replay_item_positions(ItemSet& IS, const HeadsSoA& h, const uint8_t* maskD, uint32_t n) {
    HostItems I = download_items(IS, n);
    replay_items(I, down(maskD, n), down(h.smaller, H), down(h.tonext, H));
    const uint32_t k = (uint32_t)I.pos.size();
    up(IS.pos, I.pos); up(IS.len, I.len); up(IS.isa, I.isa); up(IS.until, I.until);
    up(IS.count, I.count); up(IS.first, I.first); up(IS.small, I.small); up(IS.P, I.P);
    IS.K = k;
    IS.slotIsFirst = false;
    IS.slot.alloc((uint64_t)k + 1);
    IS.sk.alloc(k);
    ItemsSoA SS = IS.soa();
    mk_item_sk(SS, k, st);
    exscan(IS.count.p, IS.slot.p, 0u, k);
    uint32_t hh = H;
    HIPCHK(hipMemcpyAsync(IS.slot.p + k, &hh, 4, hipMemcpyHostToDevice, st));
    mk_pos_begin(IS.pos.p, k, n, IS.posBegin.p, st);
    mk_pos_f(IS.pos.p, IS.small.p, IS.posBegin.p, k, n, IS.posF.p, st);
    sync();  // hh is a stack variable
  }
  // Checked counter (FN:1523-1603): the device answers every query whose
  // target is unmasked and unambiguous; a pass that meets an ambiguous query
  // masks its target and the counters are recomputed, so every query into a
  // masked target is answered by the host replay (host_queries).  Returns the
  // ambiguous queries of the first pass; cs receives the final statistics.
  uint64_t hostQueries = 0;
  uint64_t counter_checked(ItemSet& IS, const HeadsSoA& h, DBuf<uint32_t>& nhr, DBuf<uint8_t>& hostMask,
                           DBuf<unsigned long long>& cstats, uint32_t n, unsigned long long* cs) {
    ItemsSoA S = IS.soa();
    const uint32_t k = IS.K;
    DBuf<uint8_t> amb;
    amb.alloc(n);
    amb.zero(st);
    DBuf<unsigned long long> hcnt;
    hcnt.alloc(1);
    uint64_t cap = 1ull << 16, nq = 0, firstViol = 0;
    DBuf<uint32_t> hlist;
    hlist.alloc(2 * cap);
    for (int pass = 0;; pass++) {
      if (pass > 3) throw InputError{CMSBWT_EINTERNAL, "internal: checked counter did not settle"};
      counter.zero(st);
      cstats.zero(st);
      hcnt.zero(st);
      HostRoute hr{hostMask.p, amb.p, hlist.p, hcnt.p, cap};
      counter_phase(S, k, IS.posBegin.p, IS.posF.p, nhr.p, counter.p, cstats.p, n, 0, n, true, &hr);
      HIPCHK(hipMemcpyAsync(cs, cstats.p, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
      nq = read1(hcnt.p);
      if (pass == 0) firstViol = cs[3];
      if (cs[3]) {  // targets with ambiguous queries join the host replay
        mk_or_mask(hostMask.p, amb.p, n, st);
        continue;
      }
      if (nq > cap) {
        cap = nq;
        hlist.alloc(2 * cap);
        continue;
      }
      break;
    }
    hostQueries = nq;
    if (nq) {
      HostItems I = download_items(IS, n);
      const std::vector<uint32_t> lst = down(hlist.p, 2 * nq);
      std::vector<std::pair<uint32_t, uint32_t>> q(nq);
      for (uint64_t i = 0; i < nq; i++) q[i] = {lst[2 * i], lst[2 * i + 1]};
      bool mismatch = false;
      HostQueryOut o = host_queries(I, down(IS.slot.p, (uint64_t)k + 1), down(nhr.p, H), down(h.smaller, H),
                                    std::move(q), &mismatch);
      if (mismatch) throw InputError{CMSBWT_EINTERNAL, "internal: replayed std::map differs from the device items"};
      std::vector<uint32_t> as(o.adds.size());
      std::vector<unsigned long long> av(o.adds.size());
      for (size_t i = 0; i < o.adds.size(); i++) { as[i] = o.adds[i].first; av[i] = o.adds[i].second; }
      DBuf<uint32_t> das;
      DBuf<unsigned long long> dav;
      up(das, as);
      up(dav, av);
      mk_counter_adds(das.p, dav.p, (uint32_t)as.size(), counter.p, st);
      sync();
      cs[0] += o.bad;
      cs[1] += o.good;
    }
    return firstViol;
  }

  void merge(int rle) {
    if (!walked) throw InputError{CMSBWT_EARG, "run ms_walk first"};
    // Zero heads: the j-scan's `phrasesVector.size() - 1` (FN:1359) wraps and
    // FN:1385 writes phrasesVector[-1]; the reference's behaviour is undefined.
    if (H == 0) throw InputError{CMSBWT_EINPUT, "collection has no documents (reference behaviour undefined, FN:1359-1385)"};
    auto t0 = std::chrono::steady_clock::now();
    dm.on = false;
    // an error thrown while side work is pending: drain the side stream
    // before this scope's buffers go back to the pools (no-op otherwise)
    struct SideDrain {
      hipStream_t s;
      ~SideDrain() { (void)hipStreamSynchronize(s); }
    } sideDrain{st2};
    const uint32_t n = R.n;
    const uint32_t E = (uint32_t)ndocs;
    HeadsSoA h = heads();
    ItemSet IS;
    group_items(h, H, n, IS);
    ensure_runs();  // (the position-first grouping already counted them)
    K = IS.K;
    DBuf<uint32_t>& P = IS.P;
    DBuf<uint32_t>& sPos = IS.pos;
    DBuf<uint32_t>& sSlot = IS.slot;
    DBuf<uint32_t>& sUntil = IS.until;
    DBuf<uint32_t>& sCount = IS.count;
    DBuf<uint32_t>& posBegin = IS.posBegin;
    DBuf<uint32_t>& posF = IS.posF;
    ItemsSoA S = IS.soa();
    DBuf<unsigned long long> cstats;
    cstats.alloc(8);
    cstats.zero(st);
    // Comparator ambiguity (match.h:27-33): positions whose
    // items break the map-order invariant get their std::map layout replayed
    // on the host, and every counter query into them is answered there.
    // CMSBWT_FORCE_REPLAY=1 routes every position through that path (tests).
    const bool forceReplay = env_u32("CMSBWT_FORCE_REPLAY", 0) != 0;
    const bool check = !orderInvariant || forceReplay || env_u32("CMSBWT_FORCE_CHECK", 0) != 0;
    DBuf<uint8_t> hostMask;  // positions answered by the host replay
    uint64_t itemViol = 0;
    if (check) {
      hostMask.alloc(n);
      HIPCHK(hipMemsetAsync(hostMask.p, forceReplay ? 1 : 0, n, st));
      mk_check_items(S, posBegin.p, posF.p, K, cstats.p + 3, hostMask.p, st);
      itemViol = read1(cstats.p + 3);
      if (itemViol || forceReplay) {
        replay_item_positions(IS, h, hostMask.p, n);
        K = IS.K;
        S = IS.soa();
      }
    }

    // ---- ranks (FN:1432-1453)
    HIPCHK(hipEventRecord(evm[0], st));
    DBuf<uint32_t> itemsSA, headsSA, itemRankBase, headBase;
    // rank2head (T) is only kept for parity copies (CMSBWT_KEEP_STAGES=1):
    // the suffix sort below needs the group labels, not the ranks themselves
    const bool keepT = env_u32("CMSBWT_KEEP_STAGES", 0) != 0;
    itemsSA.alloc(n); headsSA.alloc(n); itemRankBase.alloc(n); headBase.alloc(n);
    mk_sa_counts(dsa.p, posBegin.p, sSlot.p, n, E, itemsSA.p, headsSA.p, st);
    if (keepT) exscan(itemsSA.p, itemRankBase.p, 0u, n);
    exscan(headsSA.p, headBase.p, 0u, n);
    itemsSA.release(); headsSA.release();
    // The counter (FN:1523-1603) reads the items alone except for equal-key
    // queries, which compare next-head ranks: it runs on the side stream
    // beside the ranks and the head-string suffix sort, with those queries
    // listed and answered once the ranks exist (k_counter_eq).  The writer's
    // inputs that do not read the counters go there too.
    counter.alloc((uint64_t)H + 1);
    counter.zero(st);
    HIPCHK(hipEventRecord(evFork[0], st));
    T.alloc((uint64_t)H + 1);
    saT.alloc((uint64_t)H + 1);
    DBuf<uint32_t> grp;
    grp.alloc((uint64_t)H + 1);
    {
      int32_t z = 0;
      uint32_t hh = H, zz = 0;
      HIPCHK(hipMemcpyAsync(T.p + H, &z, 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(saT.p, &hh, 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(grp.p + H, &zz, 4, hipMemcpyHostToDevice, st));
    }
    // slot-major members: item of each slot and member idx of each slot
    DBuf<uint32_t> itemOfSlot, Pm;
    itemOfSlot.alloc(H);
    {
      DBuf<uint32_t> mark;
      mark.alloc(H);
      mark.zero(st);
      mk_slot_mark(sSlot.p, K, mark.p, st);
      inscan(mark.p, itemOfSlot.p, H, rocprim::plus<uint32_t>());
    }
    // members in slot order: P itself when the grouping emitted items and
    // members in one order (P stays: the host replay reads it)
    if (!IS.slotIsFirst) {
      Pm.alloc(H);
      mk_slot_members(S, itemOfSlot.p, P.p, H, Pm.p, st);
    }
    const uint32_t* const PmP = IS.slotIsFirst ? P.p : Pm.p;
    // first sa position of each item (the BWT characters' slot base)
    DBuf<uint32_t> gItem;
    gItem.alloc(K);
    // per sa position: member of an item with >= 2 heads, in bit 31 of the sa
    // entry when head indices fit 31 bits (one random store per head fewer
    // than a byte array; CMSBWT_UNRES_BYTES=1 keeps the byte array)
    const bool flag31 = H < 0x80000000u && !env_u32("CMSBWT_UNRES_BYTES", 0);
    DBuf<uint8_t> unres;
    if (!flag31) unres.alloc((uint64_t)H + 1);
    {
      DBuf<uint32_t> rankBase, gBase;
      rankBase.alloc(n);
      gBase.alloc(n);
      mk_pos_rank_base(posBegin.p, sSlot.p, disa.p, itemRankBase.p, headBase.p, n, E, keepT ? rankBase.p : nullptr,
                       gBase.p, st);
      mk_ranks_slot(S, itemOfSlot.p, PmP, H, rankBase.p, gBase.p, n, keepT ? T.p : nullptr, saT.p, grp.p, nullptr,
                    st, gItem.p, flag31 ? nullptr : unres.p, flag31 ? 0x80000000u : 0u);
    }
    // (enqueued after the ranks: the host waits for the side stream's
    // crossing count while the main stream ranks)
    // ---- buckets (FN:1162-1171) and inversion (FN:1618-1628, done as a
    // gather); writer elements: the E end phrases, then per SA rank its heads
    // (or one element)
    DBuf<int32_t> bcnt;
    DBuf<uint32_t> wm, eBase, rOf;
    DBuf<uint4> info1;
    DBuf<unsigned long long> info2;
    uint32_t V = 0;
    bool Vread = false;
    auto read_V = [&]() {  // writer elements (stream-ordered after writer_inputs' exscan)
      if (Vread) return;
      const uint64_t V64 = sum2(eBase.p + (n - 1), wm.p + (n - 1));
      if (V64 >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "too many writer elements"};
      V = (uint32_t)V64;
      Vread = true;
    };
    auto writer_inputs = [&]() {
      bucket.alloc(n);
      bcnt.alloc(n);
      inscan(diff.p, bcnt.p, n, rocprim::plus<int32_t>());
      mk_bucket(bcnt.p, hasHead.p, n, bucket.p, st);
      wm.alloc(n); eBase.alloc(n);
      mk_el_count(headBase.p, n, E, H, wm.p, st);
      exscan(wm.p, eBase.p, 0u, n);
      // the element count V is read when the writer needs it (read_V): a
      // host read here would hold the host until the side stream had sorted
      // the crossing lists, with the main stream's doubling not yet enqueued
      // (~1.2 ms idle).  rOf is sized by the bound E + sum over SA ranks of
      // max(1, heads) <= E + n + H.
      const uint64_t Vmax = (uint64_t)E + n + H;
      if (Vmax >= 0xffffffffull) read_V();
      rOf.alloc(Vread ? V : Vmax);
      mk_el_rof(eBase.p, wm.p, n, rOf.p, st);
      info1.alloc(n); info2.alloc(n);
      ElemIn ei{dsa.p, dbwt.p, bucket.p, posBegin.p, sSlot.p, itemOfSlot.p, headBase.p, eBase.p, rOf.p, nullptr,
                nullptr, nullptr, info1.p, info2.p, n, E, H, rle};
      mk_el_info(ei, st);
    };
    WinPlan wp;
    DBuf<uint4> eqRec;
    DBuf<unsigned long long> eqCnt;
    EqList eql;
    // phrasesSet.size() for the log (distinct positions holding items)
    DBuf<unsigned long long> posCnt;
    // work volume (statistics only): sum of untilNext, read back with the
    // counter statistics
    DBuf<uint64_t> wsum;
    auto work_sum = [&]() {
      wsum.alloc(1);
      auto u64in = rocprim::make_transform_iterator(sUntil.p, WidenU64());
      size_t b = 0;
      HIPCHK(rocprim::reduce(nullptr, b, u64in, wsum.p, (uint64_t)0, (size_t)K, rocprim::plus<uint64_t>(), st));
      HIPCHK(rocprim::reduce(scratch(b), b, u64in, wsum.p, (uint64_t)0, (size_t)K, rocprim::plus<uint64_t>(), st));
    };
    if (!check) {
      Side sd(*this, evFork[0]);
      win_prep(S, K, posBegin.p, n, 0, n, false, cstats.p, wp);
      writer_inputs();
      posCnt.alloc(1);
      posCnt.zero(st);  // (on the side stream, like the count)
      mk_count_distinct(sPos.p, K, posCnt.p, st);
      work_sum();
    }
    // CMSBWT_COUNTER_OVERLAP=1: the counter itself on the side stream, its
    // equal-key queries answered after the ranks (bit-exact, but slower:
    // DESIGN.md §3.6a); the slot-window kernel (CMSBWT_COUNTER_WIN=1) always
    // runs after the ranks.  CMSBWT_EQ_CAP: list capacity (tests: overflow)
    const bool listed = !check && wp.tgt && env_u32("CMSBWT_COUNTER_OVERLAP", 0) != 0;
    if (listed) {
      Side sd(*this, evFork[0]);
      eql.cap = std::max<uint64_t>(1, std::min<uint64_t>(H, env_u32("CMSBWT_EQ_CAP", 1u << 27)));
      eqRec.alloc(eql.cap);
      eqCnt.alloc(1);
      eqCnt.zero(st);
      eql.rec = eqRec.p;
      eql.cnt = eqCnt.p;
      HIPCHK(hipEventRecord(evm[4], st));
      counter_run(wp, S, posBegin.p, posF.p, nullptr, counter.p, cstats.p, n, false, nullptr, eql);
      HIPCHK(hipEventRecord(evm[5], st));
    }
    itemRankBase.release();
    keptT = keepT;
    stats.rank = (uint64_t)E + 2 + (uint64_t)(K - 1);

    // ---- suffix sort of the head string (libsais_int, FN:1455-1459)
    HIPCHK(hipEventRecord(evm[1], st));
    {
      const int bH = bits_for(H);
      const bool dstats = env_u32("CMSBWT_DBL_STATS", 0) != 0;
      // unresolved members' sa positions, ascending (= SA rank, then map
      // order): every group is a contiguous range of act
      DBuf<uint32_t> act, act2, val, val2, lab, labMax, keep;
      uint32_t U = 0;
      {
        // the flagged sa positions, ascending (k_ranks_slot's flags)
        const uint32_t nf = H + 1, nt = sel_tiles(nf);
        DBuf<uint32_t> tc, to;
        tc.alloc(nt);
        to.alloc(nt);
        if (flag31) mk_sel_count31(saT.p, nf, tc.p, st);
        else mk_sel_count8(unres.p, nf, tc.p, st);
        exscan(tc.p, to.p, 0u, nt);
        U = (uint32_t)sum2(to.p + (nt - 1), tc.p + (nt - 1));
        act.alloc(std::max<uint32_t>(U, 1)); act2.alloc(std::max<uint32_t>(U, 1));
        if (flag31) mk_sel_write_idx31(saT.p, nf, to.p, act.p, st);
        else mk_sel_write_idx8(unres.p, nf, to.p, act.p, st);
        unres.release();
      }
      DBuf<uint64_t> k64, k64b;
      val.alloc(U); val2.alloc(U); lab.alloc(U); labMax.alloc(U); keep.alloc(U);
      k64.alloc(U); k64b.alloc(U);
      // Group leaders sort groups of <= 32 members by one thread each; the
      // members of larger groups go to one radix sort.
      const uint32_t maxSmall = env_u32("CMSBWT_DBL_SMALL", 32);
      // one thread per member (default) or per group leader (CMSBWT_DBL_LEADERS=1)
      const bool rankPath = !env_u32("CMSBWT_DBL_LEADERS", 0);
      DBuf<uint32_t> gflag, bigList, origB, actB, valB, keepB;
      DBuf<uint64_t> keyB;
      gflag.alloc(U); bigList.alloc((uint64_t)U + 1);
      for (uint64_t hstep = 1; U > 0; hstep <<= 1) {
        if (hstep > H) throw InputError{CMSBWT_EINPUT, "internal: head-string suffix sort did not converge"};
        mk_dbl_keys(act.p, saT.p, grp.p, (uint32_t)hstep, U, k64.p, val.p, st, flag31 ? 0x7fffffffu : 0xffffffffu);
        HIPCHK(hipMemsetAsync(bigList.p, 0, 4, st));
        if (rankPath) {
          mk_dbl_rank(U, act.p, k64.p, val.p, saT.p, grp.p, keep.p, bigList.p, maxSmall, st);
        } else {
          mk_dbl_gstart(k64.p, U, gflag.p, st);
          mk_dbl_small2(gflag.p, U, act.p, k64.p, val.p, saT.p, grp.p, keep.p, bigList.p, maxSmall, st);
        }
        const uint32_t B = read1(bigList.p);
        if (dstats) fprintf(stderr, "[dbl] h %llu U %u big %u\n", (unsigned long long)hstep, U, B);
        if (B) {
          // big members were appended group by group in any group order: put
          // them back in act order (the radix path maps sorted members onto
          // ascending sa positions)
          origB.alloc(B); actB.alloc(B); valB.alloc(B); keyB.alloc(B); keepB.alloc(B);
          sort_keys(bigList.p + 1, origB.p, B, bits_for(U));
          mk_dbl_gather_big(origB.p, B, act.p, k64.p, val.p, actB.p, keyB.p, valB.p, st);
          sort_pairs(keyB.p, k64b.p, valB.p, val2.p, B, 32 + bH);
          mk_dbl_apply(actB.p, k64b.p, val2.p, B, saT.p, lab.p, st);
          inscan(lab.p, labMax.p, B, rocprim::maximum<uint32_t>());
          mk_dbl_groups(actB.p, k64b.p, val2.p, labMax.p, B, grp.p, keepB.p, st);
          mk_scatter_u32(keepB.p, origB.p, B, keep.p, st);
        }
        U = select_flagged(act.p, keep.p, act2.p, U);
        std::swap(act.p, act2.p);
      }
    }
    // Every group is a single head now, and a group's label is its first sa
    // position: grp[idx] = 1 + rank of head idx (FN:1468-1471's rankToHead),
    // so the inverse permutation needs no scatter.
    // (members never moved by the sort keep the flag: cleared for the
    // parity copies and the BWTheads gather, the only later readers of sa)
    if (flag31 && keepT) mk_and_u32(saT.p, (uint64_t)H + 1, 0x7fffffffu, st);
    saFlagged = flag31 && !keepT;
    HIPCHK(hipEventRecord(evm[2], st));
    rthFL.alloc(2);
    HIPCHK(hipMemcpyAsync(rthFL.p, grp.p, 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(rthFL.p + 1, grp.p + (H - 1), 4, hipMemcpyDeviceToDevice, st));
    // BWTheads in head-rank order only for the parity copies: the writer
    // reads the characters by slot, placed by k_nhr_rank below
    if (keepT) {
      bwtHeads.alloc(H);
      mk_head_chars(saT.p, hChar.p, H, bwtHeads.p, st);
    } else {
      bwtHeads.release();
    }
    bwtSlot.alloc(H);

    // ---- next-head ranks, sorted per item (FN:1480-1494): small items by an
    // in-place insertion sort, large ones by one global (item, nhr) sort
    DBuf<uint32_t> nhr;
    nhr.alloc(H);
    {
      const bool fused = !env_u32("CMSBWT_NHR_SORT", 0);  // 1: gather, then per-item insertion sorts
      {
        DBuf<uint32_t> nbi;
        if (fused) {  // gather + rank inside the item in one pass, placing the characters
          DBuf<uint4> rec;
          rec.alloc(H);
          mk_nhr_rec(grp.p, hNext.p, hChar.p, H, rec.p, st);
          mk_nhr_rank(PmP, nullptr, itemOfSlot.p, H, nhr.p, st, rec.p, S.slot, gItem.p, bwtSlot.p);
        } else {
          nbi.alloc(H);
          mk_head_chars_slot(PmP, grp.p, hChar.p, S, itemOfSlot.p, gItem.p, H, bwtSlot.p, st);
          mk_nhr_slot(PmP, grp.p, 1u, hNext.p, H, nbi.p, nhr.p, st);
        }
      }
      sort_nhr_items(S, K, itemOfSlot.p, nhr.p, H, fused);
    }
    grp.release();
    Pm.release();
    HIPCHK(hipEventRecord(evm[3], st));

    // ---- counterSmallerThanHead (FN:1523-1603)
    uint64_t W = 0;
    {
      if (check) work_sum();
      if (!check) {
        join_side();
        const uint64_t nEq = listed ? read1(eqCnt.p) : 0;
        if (!listed) {
          HIPCHK(hipEventRecord(evm[4], st));
          counter_run(wp, S, posBegin.p, posF.p, nhr.p, counter.p, cstats.p, n, false, nullptr);
          HIPCHK(hipEventRecord(evm[5], st));
        } else if (nEq > eql.cap) {  // list overflow: the counter again, with the ranks
          counter.zero(st);
          HIPCHK(hipMemsetAsync(cstats.p, 0, 4 * 8, st));                // bad, good, nothing, violations
          HIPCHK(hipMemsetAsync(cstats.p + 5, 0, 3 * 8, st));            // (errors stay)
          HIPCHK(hipEventRecord(evm[4], st));
          counter_run(wp, S, posBegin.p, posF.p, nhr.p, counter.p, cstats.p, n, false, nullptr);
          HIPCHK(hipEventRecord(evm[5], st));
        } else {
          mk_counter_eq(eqRec.p, (uint32_t)nEq, nhr.p, counter.p, cstats.p, st);
        }
        eqListed = nEq;
      } else {  // (checked counter below: timed on the host)
        HIPCHK(hipEventRecord(evm[4], st));
        HIPCHK(hipEventRecord(evm[5], st));
      }
    }

    unsigned long long cs[8];
    uint64_t queryViol = 0;
    HIPCHK(hipMemcpyAsync(&W, wsum.p, 8, hipMemcpyDeviceToHost, st));
    double tCheckedMs = -1;  // checked path: device passes + host replay queries, wall time
    if (check) {
      const auto tc = std::chrono::steady_clock::now();
      queryViol = counter_checked(IS, h, nhr, hostMask, cstats, n, cs);
      tCheckedMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc).count();
    } else {
      HIPCHK(hipMemcpyAsync(cs, cstats.p, sizeof(cs), hipMemcpyDeviceToHost, st));
      sync();
      counter_time();
    }
    if (env_u32("CMSBWT_COUNTER_STATS", 0))
      fprintf(stderr, "[counter] bad %llu good %llu nothing %llu windows %u crossings %u searched %llu equal-key %llu\n",
              cs[0], cs[1], cs[2], windows, crossings, cs[5], (unsigned long long)eqListed);
    if (env_u32("CMSBWT_COUNTER_STATS", 0) >= 2) {
      DBuf<unsigned long long> sh;
      sh.alloc(40);
      sh.zero(st);
      mk_counter_shape(S, K, n, sh.p, st);
      unsigned long long hs[40];
      HIPCHK(hipMemcpyAsync(hs, sh.p, sizeof(hs), hipMemcpyDeviceToHost, st));
      sync();
      fprintf(stderr, "[counter shape] records %llu full %llu pairs %llu pairs-in-full %llu\n", hs[0], hs[1], hs[2],
              hs[3]);
      for (int b = 0; b < 32; b++)
        if (hs[8 + b]) fprintf(stderr, "[counter shape] range 2^%d: pairs %llu\n", b, hs[8 + b]);
    }
    stats.counter_bad = cs[0];
    stats.counter_good = cs[1];
    stats.counter_nothing = cs[2];
    stats.order_violations = itemViol + queryViol;
    stats.host_queries = hostQueries;
    if (cs[4]) throw InputError{CMSBWT_EINPUT, "counter target beyond the reference (reference UB)"};
    W_work = W;
    stats.counter_kernel_ms = counter_kernel_ms;
    stats.counter_work = W;

    if (check) writer_inputs();
    read_V();

    // ---- writer (FN:1631-1777) as segments + run-length merge
    uint64_t Rn = 0, symbols = 0;
    DBuf<unsigned long long> runStart;
    DBuf<uint8_t> runChar;
    bool recordsWritten = false;
    {
      DBuf<unsigned long long> cum;
      cum.alloc(H);
      inscan_plus1_u64(counter.p, cum.p, H);
      ElemIn ei{dsa.p, dbwt.p, bucket.p, posBegin.p, sSlot.p, itemOfSlot.p, headBase.p, eBase.p, rOf.p, bwtHeads.p,
                counter.p, cum.p, info1.p, info2.p, n, E, H, rle};
      ei.bwtSlot = bwtSlot.p;
      if (!env_u32("CMSBWT_WR_UNFUSED", 0)) {
        // run scan in tiles of 256 elements (merge.hip k_el_wr_tiles /
        // k_el_wr_emit_tiles): per-tile run summaries, their scan, then each
        // tile emits at its elements' prefixes, straight into the 9-byte
        // records; at most 3 runs per element
        const uint64_t cap = 3ull * V;
        runs.alloc(cap * 9);
        const uint32_t nt = (V + 255) / 256;
        DBuf<WrState> tsum, tpre;
        DBuf<unsigned long long> tot;
        tsum.alloc(nt); tpre.alloc(nt); tot.alloc(2);
        // the elements' segments kept between the passes (16 B each, element
        // order): the second pass reads them sequentially instead of
        // gathering the per-slot counters, sums and characters again
        // (CMSBWT_WR_SEGBUF=0: recomputed)
        DBuf<uint4> segs;
        if (env_u32("CMSBWT_WR_SEGBUF", 1)) segs.alloc(V);
        mk_el_wr_tiles(ei, V, tsum.p, st, segs.p);
        const WrState zero{0ull, 0ull, 0ull, 0u, 0u};
        size_t b = 0;
        HIPCHK(rocprim::exclusive_scan(nullptr, b, tsum.p, tpre.p, zero, (size_t)nt, WrOp{}, st));
        HIPCHK(rocprim::exclusive_scan(scratch(b), b, tsum.p, tpre.p, zero, (size_t)nt, WrOp{}, st));
        mk_el_wr_emit_tiles(ei, V, tpre.p, runs.p, tot.p, st, segs.p);
        recordsWritten = true;
        unsigned long long tt[2];
        HIPCHK(hipMemcpyAsync(tt, tot.p, sizeof(tt), hipMemcpyDeviceToHost, st));
        sync();
        Rn = tt[0];
        symbols = tt[1];
        if (Rn > cap) throw InputError{CMSBWT_EINTERNAL, "internal: writer emitted more than 3 runs per element"};
        itemOfSlot.release();
      } else {
      DBuf<uint32_t> wruns, whl, wprev;
      DBuf<unsigned long long> wsym, wrunOff, wsymOff;
      wruns.alloc(V); whl.alloc(V); wprev.alloc(V); wsym.alloc(V); wrunOff.alloc(V); wsymOff.alloc(V);
      mk_el_wr_count(ei, V, wruns.p, wsym.p, whl.p, st);
      exscan(whl.p, wprev.p, 0u, V, LastNonEmpty());
      // runs of each element, less one when its first segment continues the
      // previous non-empty element's run (k_wr_adjust, fused into the scan)
      // one packed scan when the totals fit (at most 3 runs per element; the
      // symbol total, which the remainder quirk of FN:1761-1770 can lift above
      // the collection length, from one reduce), else two
      const AdjustedRuns adj{wruns.p, whl.p, wprev.p};
      uint64_t symTotal = 0;
      {
        DBuf<unsigned long long> tot;
        tot.alloc(1);
        size_t b = 0;
        HIPCHK(rocprim::reduce(nullptr, b, wsym.p, tot.p, 0ull, (size_t)V, rocprim::plus<unsigned long long>(), st));
        HIPCHK(rocprim::reduce(scratch(b), b, wsym.p, tot.p, 0ull, (size_t)V, rocprim::plus<unsigned long long>(), st));
        symTotal = read1(tot.p);
      }
      const bool packed = symTotal < (1ull << kPackSymBits) && 3ull * V < (1ull << (64 - kPackSymBits)) &&
                          !env_u32("CMSBWT_WR_TWO_SCANS", 0);
      if (packed) {
        auto rs = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint32_t>(0u),
                                                   PackedRunsSym{adj, wsym.p});
        exscan(rs, wrunOff.p, 0ull, V);
        const unsigned long long last = read1(wrunOff.p + (V - 1));
        Rn = (last >> kPackSymBits) + adj.host(V - 1, this);
        symbols = (last & ((1ull << kPackSymBits) - 1)) + read1(wsym.p + (V - 1));
      } else {
        auto runs64 = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint32_t>(0u), adj);
        exscan(runs64, wrunOff.p, 0ull, V);
        exscan(wsym.p, wsymOff.p, 0ull, V);
        Rn = read1(wrunOff.p + (V - 1)) + adj.host(V - 1, this);
        symbols = sum2(wsymOff.p + (V - 1), wsym.p + (V - 1));
      }
      runStart.alloc(std::max<uint64_t>(Rn, 1)); runChar.alloc(std::max<uint64_t>(Rn, 1));
      mk_el_wr_emit(ei, V, wrunOff.p, packed ? nullptr : wsymOff.p, wprev.p, runStart.p, runChar.p, st);
      itemOfSlot.release();
      }
    }
    if (!recordsWritten) {
      runs.alloc(Rn * 9);
      mk_wr_records(runStart.p, runChar.p, Rn, symbols, runs.p, st);
    }
    HIPCHK(hipGetLastError());
    sync();
    nruns = Rn;
    lastRle = rle;
    merged = true;
    stats.keys = K;
    stats.current_sum = H;
    stats.runs = Rn;
    stats.symbols = symbols;
    if (check) {
      posCnt.alloc(1);
      posCnt.zero(st);
      mk_count_distinct(sPos.p, K, posCnt.p, st);
    }
    stats.positions = read1(posCnt.p);  // (side work was joined before the counter)
    {
      uint32_t fl[2] = {0, 0};
      HIPCHK(hipMemcpy(fl, rthFL.p, 8, hipMemcpyDeviceToHost));
      stats.first_rank_to_head = (int64_t)fl[0] - 1;
      stats.last_rank_to_head = (int64_t)fl[1] - 1;
      float a = 0, b = 0, c = 0;
      HIPCHK(hipEventElapsedTime(&a, evm[0], evm[3]));
      HIPCHK(hipEventElapsedTime(&b, evm[1], evm[2]));
      HIPCHK(hipEventElapsedTime(&c, evm[4], evm[5]));
      stats.t_ranks_ms = a;
      stats.t_libsais_int_ms = b;
      stats.t_counter_ms = tCheckedMs >= 0 ? tCheckedMs : c;
    }
    stats.t_merge_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  double poolDensity = 1.0 / 32;  // head-pool records per collection char (learned per engine)
  bool densityLearned = false;
  // First walk on this engine: walk every 32nd chunk into a scratch pool to
  // estimate the head density, so a dense collection (1 % SNP: ~10 % heads)
  // does not overflow the pool and re-run the whole walk.
  void sample_density(uint32_t nch) {
    std::vector<uint32_t> ids;
    for (uint32_t c = 0; c < nch; c += 32) ids.push_back(c);
    const uint32_t ns = (uint32_t)ids.size();
    DBuf<uint32_t> order, bstart, cnt, used, next;
    order.alloc(ns);
    bstart.alloc(2);
    cnt.alloc(nch);
    used.alloc(1);
    next.alloc(16 * 8);
    const uint32_t bs[2] = {0, ns};
    HIPCHK(hipMemcpyAsync(order.p, ids.data(), ns * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(bstart.p, bs, 8, hipMemcpyHostToDevice, st));
    used.zero(st);
    next.zero(st);
    const uint64_t sampleChars = (uint64_t)ns * plan.C;
    const uint32_t sampleLanes = std::min<uint32_t>(kWalkLanes, ns);
    const uint64_t cap = ns + (uint64_t)sampleLanes * (kPoolBatch - 1) + sampleChars / 2 / kPoolB + 1024;  // up to 50 % heads
    DBuf<HeadRec> rec;
    DBuf<uint2> blkMeta;
    rec.alloc(cap * kPoolB);
    blkMeta.alloc(cap);
    HIPCHK(hipMemsetAsync(blkMeta.p, 0xff, cap * 8, st));
    Pool pool{rec.p, blkMeta.p, used.p, (uint32_t)cap};
    launch_ms_walk2(R, dtext.p, ddoc.p, plan.dch.p, nch, order.p, bstart.p, 1, next.p, pool, cnt.p,
                    sampleLanes, nullptr, st);
    HIPCHK(hipGetLastError());
    // heads of the sampled chunks (an overflowing sample still counts them all)
    std::vector<uint32_t> hc(nch);
    HIPCHK(hipMemcpyAsync(hc.data(), cnt.p, (uint64_t)nch * 4, hipMemcpyDeviceToHost, st));
    sync();
    uint64_t heads = 0;
    for (uint32_t c : ids) heads += hc[c];
    if (sampleChars) poolDensity = std::max(1.0 / 32, 1.15 * (double)heads / (double)sampleChars);
  }
  float counter_kernel_ms = 0;
  bool keptT = false;  // rank2head written by the last merge
  bool saFlagged = false;  // saT may hold k_ranks_slot's bit-31 flags (cleared before a copy)
  uint32_t windows = 0, crossings = 0;
  uint64_t eqListed = 0;  // equal-key counter queries answered after the ranks (last merge)
  bool orderInvariant = false;  // set by ms_walk (k_finalize), false for imported shards
  uint64_t W_work = 0;



  // =====================================================================
  void copy_runs(uint8_t* out, uint64_t cap) {
    if (!merged) throw InputError{CMSBWT_EARG, "run merge first"};
    if (cap < nruns * 9) throw InputError{CMSBWT_EARG, "output buffer too small"};
    if (nruns) HIPCHK(hipMemcpyAsync(out, runs.p, nruns * 9, hipMemcpyDeviceToHost, st));
    sync();
  }

  // Device -> file through the pinned pool: chunk c (bytes [c*CH, ...)) is
  // produced on `st` by produce(off, len) (a device pointer), copied into a
  // pinned buffer and written with pwrite by one of the writer threads while
  // the next chunks are produced and copied.
  void stream_out(int fd, uint64_t total, const std::function<const uint8_t*(uint64_t, uint64_t)>& produce) {
    const uint32_t nt = std::max(1u, std::min(64u, env_u32("CMSBWT_WRITE_THREADS", 8)));
    ensure_pinned(nt, (uint64_t)std::max(1u, env_u32("CMSBWT_READ_CHUNK_MB", 32)) << 20);
    const uint64_t CH = pinnedBytes;
    const uint32_t NB = (uint32_t)pinned.size();
    const uint64_t nch = (total + CH - 1) / CH;
    std::vector<hipEvent_t> ev(NB, nullptr);
    for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    std::mutex mu;
    std::condition_variable cv;
    std::deque<uint64_t> q;
    std::vector<char> busy(NB, 0);
    bool done = false;
    std::atomic<int> err{0};
    std::vector<std::thread> th;
    for (uint32_t k = 0; k < nt; k++)
      th.emplace_back([&] {
        while (true) {
          uint64_t c;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return done || !q.empty(); });
            if (q.empty()) return;
            c = q.front();
            q.pop_front();
          }
          const uint32_t b = (uint32_t)(c % NB);
          const uint64_t off = c * CH, len = std::min(CH, total - off);
          if (hipEventSynchronize(ev[b]) != hipSuccess) err = 2;
          uint64_t put = 0;
          while (!err && put < len) {
            ssize_t w = pwrite(fd, (const uint8_t*)pinned[b] + put, len - put, (off_t)(off + put));
            if (w <= 0) { err = 1; break; }
            put += (uint64_t)w;
          }
          std::lock_guard<std::mutex> lk(mu);
          busy[b] = 0;
          cv.notify_all();
        }
      });
    auto finish = [&] {
      {
        std::lock_guard<std::mutex> lk(mu);
        done = true;
      }
      cv.notify_all();
      for (auto& t : th) t.join();
      for (auto e : ev) (void)hipEventDestroy(e);
    };
    try {
      for (uint64_t c = 0; c < nch && !err; c++) {
        const uint32_t b = (uint32_t)(c % NB);
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return !busy[b]; });
          busy[b] = 1;
        }
        const uint64_t off = c * CH, len = std::min(CH, total - off);
        const uint8_t* src = produce(off, len);
        HIPCHK(hipMemcpyAsync(pinned[b], src, len, hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(ev[b], st));
        std::lock_guard<std::mutex> lk(mu);
        q.push_back(c);
        cv.notify_all();
      }
    } catch (...) {
      finish();
      throw;
    }
    finish();
    if (err == 1) throw InputError{CMSBWT_EIO, "write error"};
    if (err) throw HipError{"HIP error while writing the output"};
  }

  void write_output(const std::string& outname, int rle) {
    if (!merged) throw InputError{CMSBWT_EARG, "run merge first"};
    if (rle != lastRle) throw InputError{CMSBWT_EARG, "merge was run with a different output format"};
    auto t0 = std::chrono::steady_clock::now();
    const std::string path = outname + (rle ? ".rl_bwt" : ".bwt");
    // no O_TRUNC: rewriting an existing output in place and cutting it to
    // size afterwards avoids freeing and refaulting its page-cache pages
    int fd = open(path.c_str(), O_WRONLY | O_CREAT, 0644);
    if (fd < 0) throw InputError{CMSBWT_EIO, "cannot open " + path};
    uint64_t outBytes = 0;
    try {
      if (rle) {  // FN:1695-1777: the packed 9-byte records as they are in HBM
        outBytes = nruns * 9;
        stream_out(fd, nruns * 9, [&](uint64_t off, uint64_t) { return runs.p + off; });
      } else {    // FN:1631-1694: the runs expanded on the device, chunk by chunk
        DBuf<unsigned long long> rlen, rstart;
        DBuf<uint8_t> rchr, chunk;
        rlen.alloc(std::max<uint64_t>(nruns, 1));
        rstart.alloc(std::max<uint64_t>(nruns, 1));
        rchr.alloc(std::max<uint64_t>(nruns, 1));
        launch_out_split(runs.p, nruns, rlen.p, rchr.p, st);
        exscan(rlen.p, rstart.p, 0ull, nruns);
        const uint64_t total = nruns ? read1(rstart.p + nruns - 1) + read1(rlen.p + nruns - 1) : 0;
        outBytes = total;
        ensure_pinned(std::max(1u, std::min(64u, env_u32("CMSBWT_WRITE_THREADS", 8))),
                      (uint64_t)std::max(1u, env_u32("CMSBWT_READ_CHUNK_MB", 32)) << 20);
        const uint64_t CH = pinnedBytes;
        chunk.alloc(2 * CH);
        uint64_t c = 0;
        stream_out(fd, total, [&](uint64_t off, uint64_t len) {
          uint8_t* dst = chunk.p + (c++ & 1) * CH;  // stream order: D2H of chunk c-2 precedes this
          launch_out_expand(rstart.p, rchr.p, nruns, off, len, dst, st);
          return dst;
        });
      }
    } catch (...) {
      // never leave new bytes over a previous run's tail: the reference's
      // ofstream truncates, so a failed write leaves an empty file
      if (ftruncate(fd, 0) != 0) (void)unlink(path.c_str());
      close(fd);
      throw;
    }
    if (ftruncate(fd, (off_t)outBytes) != 0) {
      (void)unlink(path.c_str());
      close(fd);
      throw InputError{CMSBWT_EIO, "cannot size " + path};
    }
    if (close(fd) != 0) throw InputError{CMSBWT_EIO, "cannot close " + path};
    if (R.n < 1000000 && !dm.on) {  // FN:919-924 small-reference side output (single-GPU merge)
      std::vector<unsigned long long> c((uint64_t)H + 1);
      HIPCHK(hipMemcpyAsync(c.data(), counter.p, c.size() * 8, hipMemcpyDeviceToHost, st));
      sync();
      FILE* f = fopen((outname + ".counterSmallerThanHead_true").c_str(), "wb");
      if (!f) throw InputError{CMSBWT_EIO, "cannot open counter file"};
      fwrite(c.data(), 8, c.size(), f);
      fclose(f);
    }
    stats.t_write_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  void walk_import(uint64_t heads, uint64_t nd, uint64_t nchars, uint32_t flags, const void* const* a) {
    if (!refLoaded) throw InputError{CMSBWT_EARG, "load the reference first"};
    if (heads >= 0xffffffffull) throw InputError{CMSBWT_ELIMIT, "more than 2^32-2 heads (uint32 head indices)"};
    walked = merged = false;
    H = (uint32_t)heads;
    hStart.alloc(H); hPos.alloc(H); hLen.alloc(H); hIsa.alloc(H); hTonext.alloc(H);
    hSmall.alloc(H); hChar.alloc(H); hNext.alloc(H);
    diff.alloc((uint64_t)R.n + 1);
    hasHead.alloc(R.n);
    auto in = [&](void* d, const void* s, uint64_t b) {
      if (b) HIPCHK(hipMemcpyAsync(d, s, b, hipMemcpyDefault, st));
    };
    in(hStart.p, a[0], (uint64_t)H * 4); in(hPos.p, a[1], (uint64_t)H * 4); in(hLen.p, a[2], (uint64_t)H * 4);
    in(hSmall.p, a[3], H); in(hChar.p, a[4], H); in(hIsa.p, a[5], (uint64_t)H * 4);
    in(hTonext.p, a[6], (uint64_t)H * 4); in(hNext.p, a[7], (uint64_t)H * 2);
    in(diff.p, a[8], ((uint64_t)R.n + 1) * 4); in(hasHead.p, a[9], R.n);
    sync();
    runsValid = true;
    ndocs = nd;
    chars = nchars;
    collLoaded = walked = true;
    orderInvariant = (flags & 1u) != 0;
    stats.heads = H;
    stats.ndocs = nd;
    stats.chars = nchars;
  }

  // parity copies
  uint64_t copy_array(const std::string& name, void* out) {
    auto cp = [&](const void* d, uint64_t bytes) -> uint64_t {
      if (out && bytes) {
        HIPCHK(hipMemcpyAsync(out, d, bytes, hipMemcpyDefault, st));
        sync();
      }
      return bytes;
    };
    if (name.rfind("ref_", 0) == 0 && !refLoaded) throw InputError{CMSBWT_EARG, "load a reference first"};
    if (name == "ref_sa") return cp(dsa.p, (uint64_t)R.n * 4);
    if (name == "ref_isa") return cp(disa.p, (uint64_t)R.n * 4);
    if (name == "ref_lcp") return cp(dlcp.p, ((uint64_t)R.n + 1) * 4);
    if (name == "ref_plcp") return cp(dplcp.p, (uint64_t)R.n * 4);
    if (name == "ref_bwt") return cp(dbwt.p, R.n);
    if (name == "ref_ld") return R.ld ? cp(dld.p, (uint64_t)R.n * 4) : 0;
    if (name == "ref_pr") return cp(dpr.p, (uint64_t)R.n * 16);
    if (name == "ref_ir") return cp(dir.p, (uint64_t)R.n * 16);
    if (name == "ref_pfx") return R.pfx ? cp(dpfx.p, dpfx.n * 4) : 0;
    if (name == "ref_lvl") {  // the block-minima levels, concatenated
      uint64_t b = 0;
      for (int L = 0; L < R.nlvl; L++) {
        if (out) HIPCHK(hipMemcpyAsync((uint8_t*)out + b, R.lvl[L], (uint64_t)R.lvlLen[L] * 4, hipMemcpyDefault, st));
        b += (uint64_t)R.lvlLen[L] * 4;
      }
      if (out) sync();
      return b;
    }
    if (name == "coll_text") {
      if (!collLoaded) throw InputError{CMSBWT_EARG, "load a collection first"};
      return cp(dtext.p, hdoc.empty() ? 0 : hdoc.back());
    }
    if (name == "coll_off") {
      if (!collLoaded) throw InputError{CMSBWT_EARG, "load a collection first"};
      return cp(ddoc.p, hdoc.size() * 8);
    }
    if (name == "coll_meta") {
      collMeta[0] = sn;
      collMeta[1] = collChars;
      collMeta[2] = ndocs;
      if (out) memcpy(out, collMeta, 24);
      return 24;
    }
    if (name.rfind("h_", 0) == 0 && !walked) throw InputError{CMSBWT_EARG, "run ms_walk first"};
    if (name == "h_start") return cp(hStart.p, (uint64_t)H * 4);
    if (name == "h_pos") return cp(hPos.p, (uint64_t)H * 4);
    if (name == "h_len") return cp(hLen.p, (uint64_t)H * 4);
    if (name == "h_smaller") return cp(hSmall.p, H);
    if (name == "h_lchar") return cp(hChar.p, H);
    if (name == "h_isa") return cp(hIsa.p, (uint64_t)H * 4);
    if (name == "h_tonext") return cp(hTonext.p, (uint64_t)H * 4);
    if (name == "h_nexthead") return cp(hNext.p, (uint64_t)H * 2);
    if (name == "diff") { ensure_runs(); return cp(diff.p, ((uint64_t)R.n + 1) * 4); }
    if (name == "hashead") { ensure_runs(); return cp(hasHead.p, R.n); }
    if (!merged) throw InputError{CMSBWT_EARG, "run merge first"};
    if (dm.on) throw InputError{CMSBWT_EARG, "merge stage arrays are not kept by the sharded merge"};
    if (name == "bucket") return cp(bucket.p, (uint64_t)R.n * 8);
    if (name == "rank2head") {
      if (!keptT) throw InputError{CMSBWT_EARG, "rank2head is kept only with CMSBWT_KEEP_STAGES=1"};
      return cp(T.p, ((uint64_t)H + 1) * 4);
    }
    if (name == "head2rank") {
      if (out && saFlagged) {  // unresolved flags left in bit 31 (merge: flag31)
        mk_and_u32(saT.p, (uint64_t)H + 1, 0x7fffffffu, st);
        saFlagged = false;
      }
      return cp(saT.p, ((uint64_t)H + 1) * 4);
    }
    if (name == "bwtheads") return cp(bwtHeads.p, H);
    if (name == "counters") return cp(counter.p, ((uint64_t)H + 1) * 8);
    throw InputError{CMSBWT_EARG, "unknown array " + name};
  }
  // =====================================================================
  // Position-sharded merge over `world` ranks (dist_merge.hip, SURVEY.md
  // §8e): rank k owns reference positions [P_k, P_k+1) and the group labels
  // [G_k, G_k+1) of the head-string suffix sort.  The transport between the
  // calls (all-to-all, all-reduce, gather) is the caller's (cmsbwt.dist).
  struct DistMerge {
    bool on = false;  // the last merge was sharded (its runs live on rank 0)
    uint32_t world = 1, rank = 0, P0 = 0, P1 = 0, E = 0, Htot = 0;
    uint32_t labelBias = 0;  // added to every group label (tests: CMSBWT_DM_LABEL_BIAS)
    int rle = 1;
    bool check = false;
    std::vector<uint32_t> Psplit, Gsplit;
    DBuf<uint32_t> dPsplit, dGsplit, err;
    // document side (this rank's walk heads)
    DBuf<uint32_t> hPerm;          // send order -> head
    std::vector<uint64_t> hCnt;
    DBuf<uint32_t> grp, act;       // group label per head, unresolved heads
    uint32_t U = 0, dblH = 0;
    DBuf<uint32_t> aPerm;          // doubling send order -> index into act
    // position side (heads whose position this rank owns)
    uint32_t Hp = 0;
    DBuf<uint32_t> rPos, rLen, rIsa, rTon;
    DBuf<uint8_t> rSm, rCh;
    ItemSet IS;
    DBuf<uint32_t> itemOfSlot, Pm, gItem, headBase, nhr;
    DBuf<uint8_t> bwtSlot;
    DBuf<unsigned long long> counter;
    DBuf<uint32_t> pairItem, pairWordOff;
    uint32_t npairs = 0;
    uint64_t viol = 0;
    // writer: elements of the owned SA ranks (eBase, rOf, per-rank info,
    // element first/last chars ehl, inclusive run / symbol scans) and units
    // (E end phrases + SA ranks 1..n-1, all ranks' after the all-reduce)
    uint32_t Uw = 0, V = 0;
    DBuf<int64_t> bucket;
    DBuf<uint32_t> eBase, rOf, ehl;
    DBuf<uint4> info1;
    DBuf<uint4> segs;  // each element's segments (segs_pack), dm_units -> dm_emit
    DBuf<unsigned long long> info2, cum, runIn, symIn;  // symPacked: runIn holds both (symIn unused)
    bool symPacked = false;
    DBuf<uint32_t> uruns, uhl, uprev;
    DBuf<unsigned long long> runOff, symOff, locStart, gStart;
    DBuf<uint8_t> locChar, gChar;
    uint64_t Rloc = 0, Rn = 0, symbols = 0;
  } dm;
  void partition(const uint32_t* dest, uint64_t cnt, DBuf<uint32_t>& perm, std::vector<uint64_t>& counts);
  void dm_check_err(const char* where);
  ElemIn dm_elem_in();
  void dm_begin(uint32_t world, uint32_t rank, uint64_t heads_total, uint64_t docs_total, uint32_t flags, int rle);
  void dm_route_heads(uint64_t* counts);
  void dm_pack_heads(int32_t* out);
  void dm_group(const int32_t* recv, uint64_t nrecv, uint32_t* saCounts);
  void dm_labels(const uint32_t* saCounts, unsigned long long* back);
  uint64_t dm_dbl_init(const unsigned long long* labels);
  void dm_dbl_route(uint64_t h, uint64_t* counts);
  void dm_dbl_pack(int32_t* out);
  void dm_dbl_sort(const int32_t* recv, uint64_t nrecv, unsigned long long* res);
  uint64_t dm_dbl_apply(const unsigned long long* back);
  void dm_pack_ranks(int32_t* out);
  void dm_load_ranks(const int32_t* recv);
  void dm_route_halo(uint64_t* itemCounts, uint64_t* wordCounts);
  void dm_pack_halo(int32_t* hdr, int32_t* words);
  void dm_counter(const int32_t* hdr, uint64_t nh, const int32_t* words, uint64_t nw, uint64_t* out6);
  void dm_units(int64_t* out);
  uint64_t dm_emit(const int64_t* unitsAll);
  void dm_copy_stream(unsigned long long* start, uint8_t* chars);
  void dm_finish(const unsigned long long* const* starts, const uint8_t* const* chars, const uint64_t* counts,
                 const uint64_t* gstats);
};

}  // namespace cmsbwt

// The C ABI's context (engine.hip): one engine and its last error message.
struct cmsbwt_ctx {
  cmsbwt::Engine* e = nullptr;
  std::string err;
};
