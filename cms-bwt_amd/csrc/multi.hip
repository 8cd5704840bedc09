// multi.hip — cmsbwt_run over several GPUs in one process (SURVEY.md §8(b)
// `n_gpus`, §8(e)): the drop-in's multi-GPU path (`cmsbwt -n N`).
//
// One host thread and one Engine (device, stream, caching allocator) per
// rank; rank k runs on device (args.device + k) % devices.  Every rank indexes
// the reference, reads its byte range of the collection file (shard_bounds:
// ranges start at document starts, so the ranks' documents in rank order are
// the file's, FN:1138-1139) and walks its documents (FN:1138-1385).  The merge
// (FN:1387-1777) runs sharded by reference position with the dm_* stages of
// dist_merge.hip -- the sequence cmsbwt/dist.py drives over torch.distributed,
// here over an in-process transport:
//   PEER  pulls between the ranks' HBM buffers (hipMemcpyPeerAsync over xGMI;
//         device-local copies when ranks share a GPU).  All-to-alls: every
//         rank pulls its segments from every sender.  Reductions: each rank
//         reduces its 1/W chunk (pull + add), then pulls the other chunks.
//   RCCL  ncclSend/ncclRecv groups and ncclAllReduce on an ncclCommInitAll
//         communicator (one distinct GPU per rank; librccl opened at run time).
// Host-side exchanges (counts, statistics) go through a table shared by the
// rank threads between two barriers.  A rank that fails marks the group
// failed and the others leave at their next barrier; all ranks meet once
// more (a latch that ignores the failure) before any context is destroyed,
// so no rank frees a buffer another rank may still be reading.
//
// References below 1e6 symbols (the small path and its
// .counterSmallerThanHead_true, FN:919-924), -p runs (the cut depends on every
// byte before it), CMSBWT_DIST=gather, and steps that meet comparator
// ambiguity gather every rank's heads on rank 0 and run the
// one-GPU merge there (with its std::map replay).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <fstream>
#include <functional>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "ctx_view.h"
#include "host_index.h"
#include "host_reader.h"
#include "run_log.h"

namespace cmsbwt {
namespace {

#define MCHK(x)                                                                                   \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess)                                                                         \
      throw CtxError{CMSBWT_EDEVICE, std::string(#x) + " -> " + hipGetErrorString(e_) + " @" +     \
                                         std::to_string(__LINE__)};                               \
  } while (0)

// the rank thread's context: device buffers below come from its caching
// allocator (stream-ordered reuse on the rank's stream)
thread_local cmsbwt_ctx* t_ctx = nullptr;
template <class T>
struct Buf {
  T* p = nullptr;
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  ~Buf() { release(); }
  void alloc(uint64_t k) {
    release();
    p = (T*)ctx_alloc(t_ctx, std::max<uint64_t>(k, 1) * sizeof(T));
  }
  void release() {
    if (p) ctx_free(t_ctx, p);
    p = nullptr;
  }
};

__global__ void k_red_add_u32(uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] += b[i];
}
__global__ void k_red_add_i64(long long* __restrict__ a, const long long* __restrict__ b, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] += b[i];
}
__global__ void k_red_max_u8(uint8_t* __restrict__ a, const uint8_t* __restrict__ b, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = a[i] > b[i] ? a[i] : b[i];
}

enum class Red { SumU32, SumI64, MaxU8 };  // (int32 sums wrap like uint32)
uint64_t red_size(Red op) { return op == Red::SumU32 ? 4 : op == Red::SumI64 ? 8 : 1; }

void launch_red(Red op, void* a, const void* b, uint64_t n, hipStream_t st) {
  if (!n) return;
  const uint32_t g = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
  if (op == Red::SumU32) hipLaunchKernelGGL(k_red_add_u32, dim3(g), dim3(256), 0, st, (uint32_t*)a, (const uint32_t*)b, n);
  else if (op == Red::SumI64)
    hipLaunchKernelGGL(k_red_add_i64, dim3(g), dim3(256), 0, st, (long long*)a, (const long long*)b, n);
  else hipLaunchKernelGGL(k_red_max_u8, dim3(g), dim3(256), 0, st, (uint8_t*)a, (const uint8_t*)b, n);
  MCHK(hipGetLastError());
}

struct Aborted {};  // another rank failed: leave quietly

// test hook: CMSBWT_MULTI_FAIL_RANK=k makes rank k fail after its walk, while
// the other ranks enter the merge's exchanges (tests/test_gpu_cli_multi.py)
void inject_failure(int rank) {
  const char* e = getenv("CMSBWT_MULTI_FAIL_RANK");
  if (e && *e && atoi(e) == rank) throw CtxError{CMSBWT_EINTERNAL, "injected failure (CMSBWT_MULTI_FAIL_RANK)"};
}

// Rank threads of one run: barrier, failure flag, host exchange table.
class Group {
 public:
  explicit Group(int w) : world(w), tab(w), dev(w, 0) {}
  const int world;
  struct Slot {
    std::vector<uint64_t> v;
    const void* ptr = nullptr;
  };
  std::vector<Slot> tab;
  std::vector<int> dev;

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (failed) throw Aborted{};
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return;
    }
    cv.wait(lk, [&] { return gen != g || failed; });
    if (failed) throw Aborted{};
  }
  void fail() {
    std::function<void()> ab;
    {
      std::lock_guard<std::mutex> lk(mu);
      if (!failed && onFail) ab = onFail;
      failed = true;
      failedFlag = true;
      cv.notify_all();
    }
    // ranks blocked in a stream synchronisation behind an RCCL kernel wait on
    // a peer that never posts its side: abort the communicators so those
    // waits return an error and the ranks reach their latch.  The abort frees
    // the communicators, so it waits until no rank is inside an enqueue
    // (rccl() below: a rank checks the flag and enqueues under the shared
    // gate); a rank blocked inside an enqueue itself (a connection to the dead
    // peer) would hold the gate forever, and that call is what the abort
    // exists to end, so after kGateWait the abort proceeds regardless.
    if (ab) {
      std::unique_lock<std::shared_timed_mutex> lk(gate, std::defer_lock);
      (void)lk.try_lock_for(kGateWait);
      ab();
    }
  }
  bool has_failed() const { return failedFlag; }
  // RCCL enqueue section of one rank: refused once the group has failed, and
  // never concurrent with the abort of the communicators
  template <class F>
  void rccl(F&& f) {
    std::shared_lock<std::shared_timed_mutex> lk(gate);
    if (failedFlag) throw Aborted{};
    f();
  }
  std::function<void()> onFail;  // set before the rank threads start
  // every rank, failed or not, passes here once before its context goes away
  void final_latch() {
    std::unique_lock<std::mutex> lk(mu);
    if (++done == world) cv.notify_all();
    cv.wait(lk, [&] { return done == world; });
  }

 private:
  static constexpr std::chrono::seconds kGateWait{2};
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0, done = 0;
  uint64_t gen = 0;
  bool failed = false;
  std::atomic<bool> failedFlag{false};
  std::shared_timed_mutex gate;
};

// librccl entry points, resolved at run time (the PEER transport needs none)
struct Rccl {
  void* h = nullptr;
  decltype(&ncclCommInitAll) commInitAll = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclCommAbort) commAbort = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclAllReduce) allReduce = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclGetErrorString) errStr = nullptr;
  bool load(std::string& err) {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) { err = "cannot open librccl"; return false; }
    bool ok = true;
    auto sym = [&](auto& f, const char* s) {
      f = (std::remove_reference_t<decltype(f)>)dlsym(h, s);
      ok = ok && f;
    };
    sym(commInitAll, "ncclCommInitAll"); sym(commDestroy, "ncclCommDestroy"); sym(commAbort, "ncclCommAbort");
    sym(send, "ncclSend");
    sym(recv, "ncclRecv"); sym(allReduce, "ncclAllReduce"); sym(groupStart, "ncclGroupStart");
    sym(groupEnd, "ncclGroupEnd"); sym(errStr, "ncclGetErrorString");
    if (!ok) err = "librccl lacks an entry point";
    return ok;
  }
  void check(ncclResult_t r, const char* what) const {
    if (r != ncclSuccess)
      throw CtxError{CMSBWT_EDEVICE, std::string("RCCL ") + what + ": " + (errStr ? errStr(r) : "error")};
  }
};

// The exchanges of the sharded merge for one rank (cf. cmsbwt/dist.py Transport).
class Xfer {
 public:
  Xfer(Group& g, int rank, hipStream_t st, const Rccl* nccl, ncclComm_t comm)
      : g(g), rank(rank), W(g.world), st(st), nccl(nccl), comm(comm) {}

  std::vector<std::vector<uint64_t>> allgather(const std::vector<uint64_t>& v) {
    g.tab[rank].v = v;
    g.barrier();
    std::vector<std::vector<uint64_t>> out(W);
    for (int s = 0; s < W; s++) out[s] = g.tab[s].v;
    g.barrier();
    return out;
  }
  // per-destination counts -> per-source counts
  std::vector<uint64_t> counts(const std::vector<uint64_t>& send) {
    auto all = allgather(send);
    std::vector<uint64_t> r(W);
    for (int s = 0; s < W; s++) r[s] = all[s][rank];
    return r;
  }
  // send[k] = sc[k] elements of `elem` bytes for rank k (in rank order);
  // recv gets rc[s] elements from each rank s, in rank order
  void a2a(const void* send, uint64_t elem, const std::vector<uint64_t>& sc, const std::vector<uint64_t>& rc,
           void* recv) {
    if (nccl) {
      g.rccl([&] {
        nccl->check(nccl->groupStart(), "group start");
        uint64_t so = 0, ro = 0;
        bool open = true;
        try {
          for (int s = 0; s < W; s++) {
            if (sc[s]) nccl->check(nccl->send((const char*)send + so, sc[s] * elem, ncclUint8, s, comm, st), "send");
            if (rc[s]) nccl->check(nccl->recv((char*)recv + ro, rc[s] * elem, ncclUint8, s, comm, st), "recv");
            so += sc[s] * elem;
            ro += rc[s] * elem;
          }
          open = false;
          nccl->check(nccl->groupEnd(), "group end");
        } catch (...) {
          if (open) (void)nccl->groupEnd();  // (a group left open would swallow the next calls)
          throw;
        }
      });
      sync();
      return;
    }
    std::vector<uint64_t> off(W + 1, 0);
    for (int k = 0; k < W; k++) off[k + 1] = off[k] + sc[k] * elem;
    g.tab[rank].v = off;
    g.tab[rank].ptr = send;
    g.barrier();
    uint64_t ro = 0;
    for (int s = 0; s < W; s++) {
      const uint64_t b = rc[s] * elem;
      if (g.tab[s].v[rank + 1] - g.tab[s].v[rank] != b)
        throw CtxError{CMSBWT_EINTERNAL, "all-to-all: rank " + std::to_string(s) + " sends a different count"};
      pull((char*)recv + ro, (const char*)g.tab[s].ptr + g.tab[s].v[rank], s, b);
      ro += b;
    }
    sync();
    g.barrier();  // the senders' buffers stay until every pull is done
  }
  // in-place all-reduce of n elements
  void allreduce(void* buf, uint64_t n, Red op) {
    if (nccl) {
      const ncclDataType_t t = op == Red::SumU32 ? ncclUint32 : op == Red::SumI64 ? ncclInt64 : ncclUint8;
      g.rccl([&] {
        nccl->check(nccl->allReduce(buf, buf, n, t, op == Red::MaxU8 ? ncclMax : ncclSum, comm, st), "all-reduce");
      });
      sync();
      return;
    }
    const uint64_t es = red_size(op);
    auto chunk = [&](int k) { return std::make_pair(n * k / W, n * (k + 1) / W); };
    g.tab[rank].ptr = buf;
    g.barrier();
    {  // reduce-scatter: this rank's chunk, pulled from every other rank
      const auto [b, en] = chunk(rank);
      if (en > b) {
        Buf<uint8_t> tmp;
        tmp.alloc((en - b) * es);
        for (int s = 0; s < W; s++) {
          if (s == rank) continue;
          pull(tmp.p, (const char*)g.tab[s].ptr + b * es, s, (en - b) * es);
          launch_red(op, (char*)buf + b * es, tmp.p, en - b, st);  // stream order: tmp reused after the add
        }
        sync();
      }
    }
    g.barrier();
    for (int s = 0; s < W; s++) {  // all-gather of the reduced chunks
      if (s == rank) continue;
      const auto [b, en] = chunk(s);
      pull((char*)buf + b * es, (const char*)g.tab[s].ptr + b * es, s, (en - b) * es);
    }
    sync();
    g.barrier();
  }

  // a wait that fails because the group failed (aborted communicators) is
  // that failure's consequence, not a second error
  void sync() {
    const hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess && g.has_failed()) throw Aborted{};
    MCHK(e);
  }

  Group& g;
  const int rank, W;
  const hipStream_t st;

 private:
  void pull(void* dst, const void* src, int from, uint64_t bytes) {
    if (!bytes) return;
    if (g.dev[from] == g.dev[rank]) MCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    else MCHK(hipMemcpyPeerAsync(dst, g.dev[rank], src, g.dev[from], bytes, st));
  }
  const Rccl* nccl;
  ncclComm_t comm;
};

// What a rank reports to the main thread.
struct RankOut {
  int rc = 0;  // 0 ok, -1 left because another rank failed, else CMSBWT_E*
  std::string err;
  cmsbwt_stats st{};
  uint64_t sn = 0, heads = 0, chars = 0, ndocs = 0;
  bool tail = false;
  double tWalk = 0, tMerge = 0, tRanks = 0, tDbl = 0, tCounter = 0, tWrite = 0, tIndex = 0, tLoad = 0;
  double walkKernelMs = 0;
  bool gathered = false;
  // sharded merge, rank 0: phrasesSet.size() and First / Last rankToHead
  uint64_t positions = 0;
  int64_t first = -1, last = -1;
};

// The heavy stages go through the C ABI (engine.hip), so this file does not
// instantiate the engine's device code a second time.
void chk(int rc, cmsbwt_ctx* c) {
  if (rc) throw CtxError{rc, cmsbwt_last_error(c)};
}

// device bytes per head of the one-GPU merge at 1 % divergence (K ~ H;
// measured on the config-5 proxies)
constexpr double kGatherBytesPerHead = 135.0;

using Clock = std::chrono::steady_clock;
double since_ms(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// CMSBWT_MULTI_TIMING=1: host wall time of each exchange / stage of the
// sharded merge, per rank, on stderr (attributing the multi-rank overhead)
struct StageClock {
  bool on = false;
  int rank = 0;
  Clock::time_point t = Clock::now();
  std::string line;
  explicit StageClock(int r) : rank(r) {
    const char* e = getenv("CMSBWT_MULTI_TIMING");
    on = e && *e == '1';
  }
  void mark(const char* what) {
    if (!on) return;
    char b[64];
    snprintf(b, sizeof b, " %s %.2f", what, since_ms(t));
    line += b;
    t = Clock::now();
  }
  ~StageClock() {
    if (on) fprintf(stderr, "[multi-timing] rank %d:%s\n", rank, line.c_str());
  }
};

template <class T>
uint64_t sum_col(const std::vector<std::vector<uint64_t>>& m, int k) {
  uint64_t s = 0;
  for (auto& r : m) s += (T)r[k];
  return s;
}

// The one-GPU merge on rank 0 over every rank's heads (cmsbwt/dist.py
// gather_merge): heads concatenated in rank order (= document order), the
// per-position difference arrays summed and the head flags or-ed.
void gather_merge(Xfer& x, cmsbwt_ctx* ctx, int rle, RankOut& ro) {
  const int W = x.W, rank = x.rank;
  uint64_t nb = 0;
  chk(cmsbwt_copy_array(ctx, "diff", nullptr, &nb), ctx);  // the walk's run buckets exist
  const CtxView v = ctx_view(ctx);
  const uint32_t n = v.n;
  auto meta = x.allgather({v.H, v.ndocs, v.chars, v.orderInvariant ? 1ull : 0ull});
  uint64_t Htot = 0, E = 0, chars = 0;
  bool inv = true;
  for (auto& m : meta) { Htot += m[0]; E += m[1]; chars += m[2]; inv = inv && m[3]; }
  if (Htot >= 0xffffffffull) throw CtxError{CMSBWT_ELIMIT, "more than 2^32-2 heads (uint32 head indices)"};
  std::vector<uint64_t> sc(W, 0), rc(W, 0);
  sc[0] = v.H;
  if (rank == 0)
    for (int s = 0; s < W; s++) rc[s] = meta[s][0];
  const uint64_t sz[8] = {4, 4, 4, 1, 1, 4, 4, 2};  // h_start h_pos h_len h_smaller h_lchar h_isa h_tonext h_nexthead
  Buf<uint8_t> comb[8];
  for (int i = 0; i < 8; i++) {
    if (rank == 0) comb[i].alloc(Htot * sz[i]);
    x.a2a(v.heads[i], sz[i], sc, rc, comb[i].p);
  }
  Buf<int32_t> dsum;
  Buf<uint8_t> hmax;
  dsum.alloc((uint64_t)n + 1);
  hmax.alloc(n);
  MCHK(hipMemcpyAsync(dsum.p, v.diff, ((uint64_t)n + 1) * 4, hipMemcpyDeviceToDevice, v.st));
  MCHK(hipMemcpyAsync(hmax.p, v.hasHead, n, hipMemcpyDeviceToDevice, v.st));
  x.sync();
  x.allreduce(dsum.p, (uint64_t)n + 1, Red::SumU32);
  x.allreduce(hmax.p, n, Red::MaxU8);
  ro.gathered = true;
  if (rank != 0) return;
  const void* ptrs[10] = {comb[0].p, comb[1].p, comb[2].p, comb[3].p, comb[4].p,
                          comb[5].p, comb[6].p, comb[7].p, dsum.p,    hmax.p};
  chk(cmsbwt_walk_import(ctx, Htot, E, chars, inv ? 1u : 0u, ptrs), ctx);
  for (auto& c : comb) c.release();
  chk(cmsbwt_merge(ctx, rle), ctx);
}

// The position-sharded merge (include/cmsbwt.h "Multi-GPU merge"; the same
// sequence as cmsbwt/dist.py sharded_merge).  Returns false when the step has
// to be redone as a gather step (comparator ambiguity).
bool sharded_merge(Xfer& x, cmsbwt_ctx* ctx, int rle, RankOut& ro) {
  const int W = x.W, rank = x.rank;
  StageClock clk(rank);
  const CtxView v = ctx_view(ctx);
  const uint32_t n = v.n;
  const uint64_t H = v.H;
  auto meta = x.allgather({H, v.ndocs, v.chars, v.orderInvariant ? 1ull : 0ull});
  uint64_t Htot = 0, E = 0, chars = 0;
  bool inv = true;
  for (auto& m : meta) { Htot += m[0]; E += m[1]; chars += m[2]; inv = inv && m[3]; }
  auto tr = Clock::now();
  chk(cmsbwt_dm_begin(ctx, (uint32_t)W, (uint32_t)rank, Htot, E, inv ? 1u : 0u, rle), ctx);
  clk.mark("meta+begin");
  // 1-2. heads to the owners of their positions; items; initial labels
  std::vector<uint64_t> hc(W);
  chk(cmsbwt_dm_route_heads(ctx, hc.data()), ctx);
  const std::vector<uint64_t> rc = x.counts(hc);
  clk.mark("route+counts");
  uint64_t Hp = 0;
  for (auto c : rc) Hp += c;
  {
    Buf<int32_t> send, recv;
    send.alloc(H * 5);
    recv.alloc(Hp * 5);
    chk(cmsbwt_dm_pack_heads(ctx, send.p), ctx);
    x.a2a(send.p, 20, hc, rc, recv.p);
    clk.mark("pack+a2a_heads");
    send.release();
    Buf<uint32_t> sa;
    sa.alloc(3ull * n + 1);
    chk(cmsbwt_dm_group(ctx, recv.p, Hp, sa.p), ctx);
    clk.mark("group");
    recv.release();
    x.allreduce(sa.p, 3ull * n + 1, Red::SumU32);
    clk.mark("allreduce_sa");
    Buf<unsigned long long> back, labels;
    back.alloc(Hp);
    chk(cmsbwt_dm_labels(ctx, sa.p, (uint64_t*)back.p), ctx);
    sa.release();
    labels.alloc(H);
    x.a2a(back.p, 8, rc, hc, labels.p);
    clk.mark("labels+a2a");
    back.release();
    uint64_t u0 = 0;
    chk(cmsbwt_dm_dbl_init(ctx, (const uint64_t*)labels.p, &u0), ctx);
    clk.mark("dbl_init");
  }
  ro.tRanks = since_ms(tr);
  // phrasesSet.size(): distinct positions with items, over the owners
  const CtxView vg = ctx_view(ctx);
  const uint64_t posLocal = ctx_count_distinct(ctx, vg.dmItemPos, vg.dmItems);
  clk.mark("distinct");
  // 3. prefix doubling of the head string (FN:1455-1459); the count exchange
  // also sums the unresolved members
  auto td = Clock::now();
  uint64_t U = vg.dmU;
  for (uint64_t h = 1;; h *= 2) {
    std::vector<uint64_t> c(W);
    chk(cmsbwt_dm_dbl_route(ctx, h, c.data()), ctx);
    std::vector<uint64_t> cu = c;
    cu.push_back(U);
    auto all = x.allgather(cu);
    std::vector<uint64_t> r(W);
    uint64_t active = 0, nr = 0;
    for (int s = 0; s < W; s++) { r[s] = all[s][rank]; active += all[s][W]; nr += r[s]; }
    if (!active) break;
    Buf<int32_t> send, recv;
    Buf<unsigned long long> res, back;
    send.alloc(U * 2);
    recv.alloc(nr * 2);
    chk(cmsbwt_dm_dbl_pack(ctx, send.p), ctx);
    x.a2a(send.p, 8, c, r, recv.p);
    send.release();
    res.alloc(nr);
    chk(cmsbwt_dm_dbl_sort(ctx, recv.p, nr, (uint64_t*)res.p), ctx);
    recv.release();
    back.alloc(U);
    x.a2a(res.p, 8, r, c, back.p);
    chk(cmsbwt_dm_dbl_apply(ctx, (const uint64_t*)back.p, &U), ctx);
    clk.mark("dbl_round");
  }
  ro.tDbl = since_ms(td);
  clk.mark("dbl_end");
  // First / Last rankToHead (FN:1476-1477): ranks of global heads 0 and H-1
  // (the first head is rank 0's, the last one that of the last rank with heads)
  std::vector<uint64_t> fl{0, 0, H ? 1ull : 0ull};
  if (H) {
    const CtxView vd = ctx_view(ctx);
    uint32_t a = 0, b = 0;
    MCHK(hipMemcpyAsync(&a, vd.dmGrp, 4, hipMemcpyDeviceToHost, vd.st));
    MCHK(hipMemcpyAsync(&b, vd.dmGrp + (H - 1), 4, hipMemcpyDeviceToHost, vd.st));
    x.sync();
    fl = {a - vd.dmLabelBias, b - vd.dmLabelBias, 1};
  }
  // 4. head ranks / next-head ranks / BWT characters to the position owners
  auto tr2 = Clock::now();
  {
    Buf<int32_t> rk, rr;
    rk.alloc(H * 3);
    rr.alloc(Hp * 3);
    chk(cmsbwt_dm_pack_ranks(ctx, rk.p), ctx);
    x.a2a(rk.p, 12, hc, rc, rr.p);
    rk.release();
    chk(cmsbwt_dm_load_ranks(ctx, rr.p), ctx);
    clk.mark("ranks");
  }
  ro.tRanks += since_ms(tr2);
  // 5. counters with the halo of items reaching in from earlier ranks
  auto tc = Clock::now();
  std::vector<uint64_t> c6(6);
  {
    std::vector<uint64_t> ic(W), wc(W);
    chk(cmsbwt_dm_route_halo(ctx, ic.data(), wc.data()), ctx);
    uint64_t ni = 0, nw = 0;
    for (int k = 0; k < W; k++) { ni += ic[k]; nw += wc[k]; }
    Buf<int32_t> hdr, words, hin, win;
    hdr.alloc(ni * 6);
    words.alloc(nw);
    chk(cmsbwt_dm_pack_halo(ctx, hdr.p, words.p), ctx);
    const std::vector<uint64_t> ric = x.counts(ic), rwc = x.counts(wc);
    uint64_t nri = 0, nrw = 0;
    for (int k = 0; k < W; k++) { nri += ric[k]; nrw += rwc[k]; }
    hin.alloc(nri * 6);
    win.alloc(nrw);
    x.a2a(hdr.p, 24, ic, ric, hin.p);
    x.a2a(words.p, 4, wc, rwc, win.p);
    chk(cmsbwt_dm_counter(ctx, hin.p, nri, win.p, nrw, c6.data()), ctx);
    clk.mark("halo+counter");
  }
  ro.tCounter = since_ms(tc);
  std::vector<uint64_t> mine = c6;
  mine.push_back(posLocal);
  mine.insert(mine.end(), fl.begin(), fl.end());
  auto g = x.allgather(mine);  // bad good nothing viol errs keys | positions | first last has
  clk.mark("stats");
  uint64_t tot[7] = {0, 0, 0, 0, 0, 0, 0};
  for (auto& v : g)
    for (int k = 0; k < 7; k++) tot[k] += v[k];
  if (tot[4]) throw CtxError{CMSBWT_EINPUT, "counter target beyond the reference (reference UB)"};
  // comparator ambiguity (or the test hook CMSBWT_DM_FORCE_GATHER=1): redo
  // the step as a gather step, whose one-GPU merge on rank 0 holds every
  // head (~135 B per head at 1 % divergence) -- refused with
  // a clear error when that cannot fit rank 0's device
  const char* fg = getenv("CMSBWT_DM_FORCE_GATHER");
  if (tot[3] || (fg && *fg == '1')) {
    size_t fr = 0, total = 0;
    MCHK(hipMemGetInfo(&fr, &total));
    if ((double)Htot * kGatherBytesPerHead > 0.9 * (double)total)
      throw CtxError{CMSBWT_ELIMIT, "comparator ambiguity needs a gather step, and a one-GPU merge of " +
                                        std::to_string(Htot) + " heads (~" +
                                        std::to_string((uint64_t)((double)Htot * kGatherBytesPerHead) >> 30) +
                                        " GiB) does not fit rank 0's device (" + std::to_string(total >> 30) +
                                        " GiB)"};
    return false;
  }
  int64_t first = -1, last = -1;
  for (int s = 0; s < W; s++)
    if (g[s][9]) {
      if (first < 0) first = (int64_t)g[s][7] - 1;
      last = (int64_t)g[s][8] - 1;
    }
  // 6. writer units, emission, runs gathered on rank 0
  const uint64_t Uw = E + n - 1;
  uint64_t nloc = 0;
  {
    Buf<int64_t> units;
    units.alloc(2 * Uw);
    chk(cmsbwt_dm_units(ctx, units.p), ctx);
    x.allreduce(units.p, 2 * Uw, Red::SumI64);
    clk.mark("units+allreduce");
    chk(cmsbwt_dm_emit(ctx, units.p, &nloc), ctx);
    clk.mark("emit");
  }
  Buf<unsigned long long> starts;
  Buf<uint8_t> chs;
  starts.alloc(nloc);
  chs.alloc(nloc);
  chk(cmsbwt_dm_copy_stream(ctx, (uint64_t*)starts.p, chs.p), ctx);
  auto cnts = x.allgather({nloc});
  std::vector<uint64_t> sc(W, 0), rcv(W, 0), counts(W);
  sc[0] = nloc;
  uint64_t Rall = 0;
  for (int s = 0; s < W; s++) {
    counts[s] = cnts[s][0];
    if (rank == 0) rcv[s] = counts[s];
    Rall += rank == 0 ? counts[s] : 0;
  }
  Buf<unsigned long long> gst;
  Buf<uint8_t> gch;
  gst.alloc(Rall);
  gch.alloc(Rall);
  x.a2a(starts.p, 8, sc, rcv, gst.p);
  x.a2a(chs.p, 1, sc, rcv, gch.p);
  clk.mark("gather_runs");
  if (rank == 0) {
    std::vector<const unsigned long long*> sp(W);
    std::vector<const uint8_t*> cp(W);
    uint64_t o = 0;
    for (int s = 0; s < W; s++) {
      sp[s] = gst.p + o;
      cp[s] = gch.p + o;
      o += counts[s];
    }
    const uint64_t gstats[8] = {Htot, tot[5], E, chars, tot[0], tot[1], tot[2], tot[3]};
    chk(cmsbwt_dm_finish(ctx, (const uint64_t* const*)sp.data(), cp.data(), counts.data(), gstats), ctx);
    clk.mark("finish");
    ro.positions = tot[6];
    ro.first = first;
    ro.last = last;
  }
  return true;
}

}  // namespace

int run_multi(const cmsbwt_args* a, const char* ref_path, const char* coll_path, cmsbwt_stats* stats_out) {
  const int W = a->n_gpus;
  if (W < 2 || W > 64) return CMSBWT_EARG;
  // peer-access set-up selects devices on the caller's thread: give the
  // caller (e.g. the Python mirror next to torch) its current device back
  struct DeviceGuard {
    int d = -1;
    DeviceGuard() { if (hipGetDevice(&d) != hipSuccess) d = -1; }
    ~DeviceGuard() { if (d >= 0) (void)hipSetDevice(d); }
  } deviceGuard;
  const std::string out = a->outname;
  std::ofstream log(out + ".log");
  auto t0 = Clock::now();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1 || a->device < 0 || a->device >= ndev) {
    log << "HIP device " << a->device << " unavailable\n";
    return CMSBWT_EDEVICE;
  }
  log << "About to read ref\n";
  {
    FILE* f = fopen(ref_path, "r");  // FN:155-160
    if (!f) {
      log << "Error opening file of base sequence " << ref_path << ", errno=" << errno << '\n';
      return CMSBWT_EIO;
    }
    fclose(f);
  }
  std::string x, err;
  uint64_t fb = 0, rs = 0;
  if (!read_reference(ref_path, x, err, &fb, &rs)) {
    if (fb) log << "n = " << fb << '\n';
    log << err << '\n';
    return CMSBWT_EIO;
  }
  const uint64_t sn0 = [&] {  // FN:215-224
    struct stat sb;
    return stat(coll_path, &sb) == 0 ? (uint64_t)sb.st_size : ~0ull;
  }();
  if (sn0 == ~0ull) {
    cmsbwt_stats s0{};
    s0.ref_file_bytes = fb;
    s0.ref_read_size = rs;
    log_reference(log, s0, sn0, a->prefix, coll_path, 0);
    return CMSBWT_EIO;
  }
  Group g(W);
  std::vector<int> devs(W);
  for (int k = 0; k < W; k++) g.dev[k] = devs[k] = (a->device + k) % ndev;
  // transport
  Rccl nccl;
  std::vector<ncclComm_t> comms;
  std::atomic<bool> commsAborted{false};
  const bool useRccl = a->backend == CMSBWT_BACKEND_RCCL;
  if (useRccl) {
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) {
      log << "RCCL needs one distinct GPU per rank (" << W << " ranks, " << ndev << " devices)\n";
      return CMSBWT_EARG;
    }
    if (!nccl.load(err)) {
      log << err << '\n';
      return CMSBWT_EDEVICE;
    }
    comms.resize(W);
    if (nccl.commInitAll(comms.data(), W, devs.data()) != ncclSuccess) {
      log << "ncclCommInitAll failed\n";
      return CMSBWT_EDEVICE;
    }
    g.onFail = [&] {
      commsAborted = true;
      for (auto c : comms) (void)nccl.commAbort(c);
    };
  } else {
    for (int i = 0; i < W; i++)
      for (int j = 0; j < W; j++)
        if (devs[i] != devs[j] && hipSetDevice(devs[i]) == hipSuccess) {
          const hipError_t pe = hipDeviceEnablePeerAccess(devs[j], 0);
          if (pe != hipSuccess) (void)hipGetLastError();  // already enabled, or staged copies
        }
  }
  // ingest plan: byte ranges of the file read on the device, or (-p /
  // CMSBWT_HOST_READER) the host getline reader's documents split by bytes
  const char* hr = getenv("CMSBWT_HOST_READER");
  const bool hostRead = a->prefix != UINT64_MAX || (hr && *hr && *hr != '0');
  std::vector<uint64_t> bounds, docSplit(W + 1, 0);
  uint64_t fsz = sn0;
  Collection whole;
  if (!hostRead) {
    if (!shard_bounds(coll_path, (uint32_t)W, bounds, fsz, err)) {
      log << "Error opening file of sequence (" << coll_path << ")\n";
      return CMSBWT_EIO;
    }
  } else {
    if (!read_collection(coll_path, a->prefix, whole, err)) {
      log << err << '\n';
      return CMSBWT_EIO;
    }
    const uint64_t nd = whole.ndocs(), tot = whole.off.empty() ? 0 : whole.off.back();
    for (int k = 1; k < W; k++) {  // first document starting at or after k*tot/W
      const uint64_t B = tot * k / W;
      docSplit[k] = (uint64_t)(std::lower_bound(whole.off.begin(), whole.off.end() - 1, B) - whole.off.begin());
      docSplit[k] = std::max(docSplit[k], docSplit[k - 1]);
    }
    docSplit[W] = nd;
  }
  const char* dm = getenv("CMSBWT_DIST");
  const bool forceGather = dm && std::string(dm) == "gather";
  std::vector<RankOut> ro(W);
  std::vector<std::thread> th;
  for (int k = 0; k < W; k++)
    th.emplace_back([&, k] {
      cmsbwt_ctx* ctx = nullptr;
      RankOut& r = ro[k];
      try {
        try {
          if (const int crc = cmsbwt_ctx_create(devs[k], &ctx))
            throw CtxError{crc, "HIP device " + std::to_string(devs[k]) + " unavailable"};
          MCHK(hipSetDevice(devs[k]));
          t_ctx = ctx;
          Xfer xf(g, k, ctx_view(ctx).st, useRccl ? &nccl : nullptr, useRccl ? comms[k] : nullptr);
          auto ti = Clock::now();
          chk(cmsbwt_load_reference(ctx, (const uint8_t*)x.data(), x.size()), ctx);
          r.tIndex = since_ms(ti);
          auto tl = Clock::now();
          if (!hostRead) {
            chk(cmsbwt_load_collection_file_range(ctx, coll_path, (uint32_t)k, (uint32_t)W), ctx);
          } else {  // this rank's documents of the host reader's pass, without separators
            const uint64_t d0 = docSplit[k], d1 = docSplit[k + 1];
            std::vector<uint8_t> text;
            std::vector<uint64_t> off{0};
            for (uint64_t d = d0; d < d1; d++) {
              text.insert(text.end(), whole.text.begin() + whole.off[d], whole.text.begin() + whole.off[d + 1] - 1);
              off.push_back(text.size());
            }
            chk(cmsbwt_load_collection(ctx, text.data(), off.data(), d1 - d0), ctx);
          }
          r.tLoad = since_ms(tl);
          const CtxView vl = ctx_view(ctx);
          r.tail = vl.collTail;
          r.sn = vl.sn;
          r.chars = vl.chars;
          r.ndocs = vl.ndocs;
          const bool small = vl.n < 1000000;  // FN:1792
          auto tw = Clock::now();
          chk(cmsbwt_ms_walk(ctx), ctx);
          r.tWalk = since_ms(tw);
          const CtxView vw = ctx_view(ctx);
          r.heads = vw.H;
          r.walkKernelMs = vw.stats.ms_walk_kernel_ms;
          inject_failure(k);
          auto tm = Clock::now();
          if (small || hostRead || forceGather) {
            gather_merge(xf, ctx, a->rle ? 1 : 0, r);
          } else if (!sharded_merge(xf, ctx, a->rle ? 1 : 0, r)) {
            chk(cmsbwt_ms_walk(ctx), ctx);  // comparator ambiguity: the walk again, then a gather step
            gather_merge(xf, ctx, a->rle ? 1 : 0, r);
          }
          r.tMerge = since_ms(tm);
          if (k == 0) {
            auto tw2 = Clock::now();
            chk(cmsbwt_write_output(ctx, out.c_str(), a->rle ? 1 : 0), ctx);
            r.tWrite = since_ms(tw2);
          }
          const CtxView vf = ctx_view(ctx);
          r.st = vf.stats;
          r.st.device_peak_bytes = vf.devicePeak;
        } catch (const Aborted&) {
          r.rc = -1;
        } catch (const CtxError& ce) {
          r.rc = ce.code;
          r.err = ce.msg;
        } catch (const std::bad_alloc&) {
          r.rc = CMSBWT_ELIMIT;
          r.err = "host out of memory";
        } catch (const std::exception& ex) {
          r.rc = CMSBWT_EINTERNAL;
          r.err = std::string("internal error: ") + ex.what();
        }
      } catch (...) {
        r.rc = CMSBWT_EINTERNAL;
        r.err = "internal error: unknown exception";
      }
      if (r.rc > 0) g.fail();
      if (ctx) (void)hipStreamSynchronize(ctx_view(ctx).st);
      g.final_latch();
      cmsbwt_ctx_destroy(ctx);
    });
  for (auto& t : th) t.join();
  if (!commsAborted)  // (an aborted communicator is already freed)
    for (auto c : comms) nccl.commDestroy(c);
  // the first failing rank's error (ranks that left because of it report -1)
  for (int k = 0; k < W; k++)
    if (ro[k].rc > 0) {
      cmsbwt_stats s0{};
      s0.ref_file_bytes = fb;
      s0.ref_read_size = rs;
      log << "rank " << k << ": " << ro[k].err << '\n';
      return ro[k].rc;
    }
  // the log, with rank 0's merge statistics and global collection figures
  cmsbwt_stats s = ro[0].st;
  s.ref_file_bytes = fb;
  s.ref_read_size = rs;
  s.coll_file_bytes = fsz;
  s.sn_initial = std::min<uint64_t>(fsz, a->prefix);
  uint64_t chars = 0, ndocs = 0, size = 0;
  double tWalk = 0, kMax = 0;
  for (auto& r : ro) {
    chars += r.chars;
    ndocs += r.ndocs;
    size += r.chars + r.ndocs;
    tWalk = std::max(tWalk, r.tWalk);
    kMax = std::max(kMax, r.walkKernelMs);
  }
  s.chars = chars;
  s.ndocs = ndocs;
  s.t_ms_walk_s = tWalk / 1e3;
  s.ms_walk_kernel_ms = kMax;
  s.t_merge_s = ro[0].tMerge / 1e3;
  s.t_write_s = ro[0].tWrite / 1e3;
  if (!ro[0].gathered) {
    s.t_ranks_ms = ro[0].tRanks;
    s.t_libsais_int_ms = ro[0].tDbl;
    s.t_counter_ms = ro[0].tCounter;
    s.positions = ro[0].positions;
    s.first_rank_to_head = ro[0].first;
    s.last_rank_to_head = ro[0].last;
  }
  // the final _sn: the file size, or the collection text once a tail
  // document closes it (FN:1269-1275; only the last rank can hold one)
  uint64_t sn = hostRead ? whole.sn : fsz;
  if (!hostRead && ro[W - 1].tail && size < sn - 1) sn = size;
  s.sn = sn;
  const bool small = s.n < 1000000;
  log_reference(log, s, sn0, a->prefix, coll_path, (long long)ro[0].tIndex);
  log_collection_start(log, s, s.n);
  log << "Finished parsing file of length: " << sn << "\n";
  log_collection_end(log, s, small, sn, a->buffer_gb);
  log << "MS-walk kernel: " << kMax << " ms (slowest of " << W << " ranks); collection pass: "
      << (long long)since_ms(t0) << " ms\n";
  for (int k = 0; k < W; k++)
    log << "rank " << k << " (device " << devs[k] << "): documents " << ro[k].ndocs << ", heads " << ro[k].heads
        << ", index " << (long long)ro[k].tIndex << " ms, load " << (long long)ro[k].tLoad << " ms, walk "
        << (long long)ro[k].tWalk << " ms (kernel " << ro[k].walkKernelMs << " ms), merge "
        << (long long)ro[k].tMerge << " ms, HBM peak " << (ro[k].st.device_peak_bytes >> 20) << " MiB\n";
  log.flush();
  if (stats_out) *stats_out = s;
  if (a->verbose)
    fprintf(stderr, "ranks %d (%s) index %.3fs load %.3fs walk %.3fs (kernel %.2fms) merge %.3fs write %.3fs runs %llu\n",
            W, useRccl ? "rccl" : "peer", ro[0].tIndex / 1e3, ro[0].tLoad / 1e3, tWalk / 1e3, kMax,
            ro[0].tMerge / 1e3, ro[0].tWrite / 1e3, (unsigned long long)s.runs);
  return CMSBWT_OK;
}


// ---------------------------------------------------------------- rank groups
// The multi-GPU step as a C entry point over resident inputs (bench.py
// --gpus N without torchrun): W rank contexts the caller loads through the
// ctx API, and one call that runs the walk and the position-sharded merge on
// every rank (one host thread per rank, the transports above).
struct GroupImpl {
  int W = 0, backend = CMSBWT_BACKEND_PEER;
  std::vector<int> devs;
  std::vector<cmsbwt_ctx*> ctx;
  Rccl nccl;
  std::vector<ncclComm_t> comms;
  std::atomic<bool> aborted{false};
  std::string err;
};

}  // namespace cmsbwt

struct cmsbwt_group {
  cmsbwt::GroupImpl g;
};

using namespace cmsbwt;

extern "C" int cmsbwt_group_create(int world, int device, int backend, cmsbwt_group** out) {
  if (!out || world < 1 || world > 64) return CMSBWT_EARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1 || device < 0 || device >= ndev) return CMSBWT_EDEVICE;
  struct DeviceGuard {
    int d = -1;
    DeviceGuard() { if (hipGetDevice(&d) != hipSuccess) d = -1; }
    ~DeviceGuard() { if (d >= 0) (void)hipSetDevice(d); }
  } deviceGuard;
  auto* G = new (std::nothrow) cmsbwt_group;
  if (!G) return CMSBWT_ELIMIT;
  GroupImpl& g = G->g;
  g.W = world;
  g.backend = backend;
  for (int k = 0; k < world; k++) g.devs.push_back((device + k) % ndev);
  if (backend == CMSBWT_BACKEND_RCCL && world > 1) {
    std::vector<int> sorted = g.devs;
    std::sort(sorted.begin(), sorted.end());
    std::string err;
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end() || !g.nccl.load(err)) {
      delete G;
      return CMSBWT_EARG;
    }
    g.comms.resize(world);
    if (g.nccl.commInitAll(g.comms.data(), world, g.devs.data()) != ncclSuccess) {
      g.comms.clear();
      delete G;
      return CMSBWT_EDEVICE;
    }
  } else {
    for (int i = 0; i < world; i++)
      for (int j = 0; j < world; j++)
        if (g.devs[i] != g.devs[j] && hipSetDevice(g.devs[i]) == hipSuccess &&
            hipDeviceEnablePeerAccess(g.devs[j], 0) != hipSuccess)
          (void)hipGetLastError();  // already enabled, or staged copies
  }
  for (int k = 0; k < world; k++) {
    cmsbwt_ctx* c = nullptr;
    const int rc = cmsbwt_ctx_create(g.devs[k], &c);
    if (rc) {
      cmsbwt_group_destroy(G);
      return rc;
    }
    g.ctx.push_back(c);
  }
  *out = G;
  return CMSBWT_OK;
}

extern "C" cmsbwt_ctx* cmsbwt_group_ctx(cmsbwt_group* G, int rank) {
  if (!G || rank < 0 || rank >= G->g.W) return nullptr;
  return G->g.ctx[rank];
}

extern "C" const char* cmsbwt_group_last_error(const cmsbwt_group* G) { return G ? G->g.err.c_str() : ""; }

extern "C" int cmsbwt_group_step(cmsbwt_group* G, int rle, cmsbwt_rank_times* per_rank) {
  if (!G) return CMSBWT_EARG;
  GroupImpl& gi = G->g;
  if (gi.aborted) {
    gi.err = "the group's RCCL communicators were aborted by an earlier failure";
    return CMSBWT_EDEVICE;
  }
  const int W = gi.W;
  Group g(W);
  for (int k = 0; k < W; k++) g.dev[k] = gi.devs[k];
  const bool useRccl = gi.backend == CMSBWT_BACKEND_RCCL && W > 1;
  if (useRccl)
    g.onFail = [&] {
      gi.aborted = true;
      for (auto c : gi.comms) (void)gi.nccl.commAbort(c);
    };
  const char* dm = getenv("CMSBWT_DIST");
  const bool forceGather = dm && std::string(dm) == "gather";
  std::vector<RankOut> ro(W);
  std::vector<std::thread> th;
  for (int k = 0; k < W; k++)
    th.emplace_back([&, k] {
      cmsbwt_ctx* ctx = gi.ctx[k];
      RankOut& r = ro[k];
      try {
        try {
          MCHK(hipSetDevice(gi.devs[k]));
          t_ctx = ctx;
          Xfer xf(g, k, ctx_view(ctx).st, useRccl ? &gi.nccl : nullptr, useRccl ? gi.comms[k] : nullptr);
          const bool small = ctx_view(ctx).n < 1000000;  // FN:1792
          auto tw = Clock::now();
          chk(cmsbwt_ms_walk(ctx), ctx);
          r.tWalk = since_ms(tw);
          const CtxView vw = ctx_view(ctx);
          r.heads = vw.H;
          r.chars = vw.chars;
          r.walkKernelMs = vw.stats.ms_walk_kernel_ms;
          inject_failure(k);
          auto tm = Clock::now();
          if (W == 1) {
            chk(cmsbwt_merge(ctx, rle), ctx);
          } else if (small || forceGather) {
            gather_merge(xf, ctx, rle, r);
          } else if (!sharded_merge(xf, ctx, rle, r)) {
            chk(cmsbwt_ms_walk(ctx), ctx);  // comparator ambiguity: the walk again, then a gather step
            gather_merge(xf, ctx, rle, r);
          }
          MCHK(hipStreamSynchronize(ctx_view(ctx).st));
          r.tMerge = since_ms(tm);
          r.st.device_peak_bytes = ctx_view(ctx).devicePeak;
        } catch (const Aborted&) {
          r.rc = -1;
        } catch (const CtxError& ce) {
          r.rc = ce.code;
          r.err = ce.msg;
        } catch (const std::bad_alloc&) {
          r.rc = CMSBWT_ELIMIT;
          r.err = "host out of memory";
        } catch (const std::exception& ex) {
          r.rc = CMSBWT_EINTERNAL;
          r.err = std::string("internal error: ") + ex.what();
        }
      } catch (...) {
        r.rc = CMSBWT_EINTERNAL;
        r.err = "internal error: unknown exception";
      }
      if (r.rc > 0) g.fail();
      (void)hipStreamSynchronize(ctx_view(ctx).st);
      g.final_latch();
    });
  for (auto& t : th) t.join();
  for (int k = 0; k < W; k++) {
    if (per_rank) {
      cmsbwt_rank_times& o = per_rank[k];
      o.walk_ms = ro[k].tWalk;
      o.merge_ms = ro[k].tMerge;
      o.walk_kernel_ms = ro[k].walkKernelMs;
      o.heads = ro[k].heads;
      o.chars = ro[k].chars;
      o.device_peak_bytes = ro[k].st.device_peak_bytes;
      o.gathered = ro[k].gathered ? 1 : 0;
      o.device = gi.devs[k];
    }
  }
  for (int k = 0; k < W; k++)
    if (ro[k].rc > 0) {
      gi.err = "rank " + std::to_string(k) + ": " + ro[k].err;
      return ro[k].rc;
    }
  gi.err.clear();
  return CMSBWT_OK;
}

extern "C" void cmsbwt_group_destroy(cmsbwt_group* G) {
  if (!G) return;
  GroupImpl& g = G->g;
  for (auto c : g.ctx) cmsbwt_ctx_destroy(c);
  if (!g.aborted)  // (an aborted communicator is already freed)
    for (auto c : g.comms) g.nccl.commDestroy(c);
  delete G;
}
