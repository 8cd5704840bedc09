// coll_read.hip — the collection reader on the GPU.
//
// The reference reads the collection with std::getline(...).good()
// (FN:1138-1147, 1257-1275); host_reader.cpp restates that loop on the CPU.
// Here the raw file bytes are streamed into HBM and the line structure is
// resolved on the device, so the host only moves bytes (pread into pinned
// buffers, DMA to HBM) and the document layout is produced where the walk
// reads it.  Semantics (no -p prefix; with -p the host reader is used):
//   * only bytes up to the last '\n' are lines (an unterminated last line
//     makes good() false and is dropped);
//   * a content byte is kept unless its line starts with '>';
//   * a '\n' emits the separator 0x02 (= document end) when its line is empty
//     or starts with '>';
//   * a non-empty pending document at the end gets its separator on the host
//     (FN:1269-1275).
// Every emission depends only on the start of the byte's line, so tiles of
// 16 KiB are independent once each knows the last '\n' before it (an
// exclusive max-scan over per-tile last newlines).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "kernels.h"

namespace cmsbwt {

constexpr uint32_t kRdThreads = 256;
constexpr uint32_t kRdPerThread = kRdTile / kRdThreads;  // 64 bytes, 4 x uint4

__device__ __forceinline__ void rd_load(const uint8_t* __restrict__ raw, uint64_t a, uint8_t (&b)[kRdPerThread]) {
  const uint4* p = reinterpret_cast<const uint4*>(raw + a);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint4 v = p[k];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int q = 0; q < 4; q++) b[k * 16 + j * 4 + q] = (uint8_t)(w[j] >> (8 * q));
  }
}

// exclusive scan over the block's threads: max (op = 0) or sum (op = 1)
template <int OP, class T>
__device__ __forceinline__ T rd_block_scan(T v, T* sh, T& total) {
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o);
    if (lane >= (uint32_t)o) x = OP ? x + y : (y > x ? y : x);
  }
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  T pre = 0, tot = 0;
  for (uint32_t k = 0; k < kRdThreads / 64; k++) {
    if (k < wv) pre = OP ? pre + sh[k] : (sh[k] > pre ? sh[k] : pre);
    tot = OP ? tot + sh[k] : (sh[k] > tot ? sh[k] : tot);
  }
  __syncthreads();
  T ex = __shfl_up(x, 1);
  if (lane == 0) ex = 0;
  total = tot;
  return OP ? pre + ex : (pre > ex ? pre : ex);
}

// per tile: 1 + position of its last '\n' (0 when it has none)
__global__ void __launch_bounds__(kRdThreads) k_rd_lastnl(const uint8_t* __restrict__ raw, uint64_t len,
                                                          uint64_t* __restrict__ lastNl1) {
  __shared__ uint64_t sh[kRdThreads / 64];
  const uint64_t a = (uint64_t)blockIdx.x * kRdTile + threadIdx.x * kRdPerThread;
  uint8_t b[kRdPerThread];
  rd_load(raw, a, b);
  uint64_t m = 0;
#pragma unroll
  for (uint32_t k = 0; k < kRdPerThread; k++)
    if (b[k] == '\n' && a + k < len) m = a + k + 1;
  uint64_t tot;
  rd_block_scan<0>(m, sh, tot);
  if (threadIdx.x == 0) lastNl1[blockIdx.x] = tot;
}

// Per-thread line state at the start of its 64 bytes: ls = start of the line
// holding byte a (1 + last '\n' before a, or the tile carry).
struct RdState {
  uint64_t ls;
  bool hdr;
};

__device__ __forceinline__ RdState rd_state(const uint8_t* __restrict__ raw, uint64_t a, uint64_t len,
                                            const uint8_t (&b)[kRdPerThread], uint64_t carry, uint64_t* sh) {
  uint64_t m = 0;
#pragma unroll
  for (uint32_t k = 0; k < kRdPerThread; k++)
    if (b[k] == '\n' && a + k < len) m = a + k + 1;
  uint64_t tot;
  uint64_t ex = rd_block_scan<0>(m, sh, tot);
  RdState s;
  s.ls = ex > carry ? ex : carry;
  s.hdr = s.ls < len && raw[s.ls] == '>';
  return s;
}

// Walk the thread's bytes; f(k, byte, isSep) for each emission.
template <class F>
__device__ __forceinline__ void rd_walk(const uint8_t* __restrict__ raw, uint64_t a, uint64_t len,
                                        const uint8_t (&b)[kRdPerThread], RdState s, F f) {
#pragma unroll
  for (uint32_t k = 0; k < kRdPerThread; k++) {
    const uint64_t g = a + k;
    if (g >= len) break;
    if (b[k] == '\n') {
      if (g == s.ls || s.hdr) f(k, (uint8_t)kSep, true);
      s.ls = g + 1;
      const uint8_t nx = k + 1 < kRdPerThread ? b[k + 1] : raw[g + 1];  // raw is padded past len
      s.hdr = g + 1 < len && nx == '>';
    } else if (!s.hdr) {
      f(k, b[k], false);
    }
  }
}

__global__ void __launch_bounds__(kRdThreads) k_rd_count(const uint8_t* __restrict__ raw, uint64_t len,
                                                         const uint64_t* __restrict__ carry,
                                                         uint32_t* __restrict__ cnt, uint32_t* __restrict__ seps) {
  __shared__ uint64_t sh[kRdThreads / 64];
  __shared__ uint32_t sh32[kRdThreads / 64];
  const uint64_t a = (uint64_t)blockIdx.x * kRdTile + threadIdx.x * kRdPerThread;
  uint8_t b[kRdPerThread];
  rd_load(raw, a, b);
  RdState s = rd_state(raw, a, len, b, carry[blockIdx.x], sh);
  uint32_t ne = 0, ns = 0;
  rd_walk(raw, a, len, b, s, [&](uint32_t, uint8_t, bool sep) {
    ne++;
    ns += sep;
  });
  uint32_t te, ts;
  rd_block_scan<1>(ne, sh32, te);
  rd_block_scan<1>(ns, sh32, ts);
  if (threadIdx.x == 0) {
    cnt[blockIdx.x] = te;
    seps[blockIdx.x] = ts;
  }
}

// Emission: bytes staged in LDS at their tile-local offsets, then stored
// coalesced at outBase[tile]; separators also write the document offsets.
// A kept byte absent from the reference records min(outpos << 8 | byte).
__global__ void __launch_bounds__(kRdThreads) k_rd_emit(const uint8_t* __restrict__ raw, uint64_t len,
                                                        const uint64_t* __restrict__ carry,
                                                        const uint64_t* __restrict__ outBase,
                                                        const uint64_t* __restrict__ sepBase,
                                                        const uint8_t* __restrict__ present, uint8_t* __restrict__ out,
                                                        uint64_t* __restrict__ docOff,
                                                        unsigned long long* __restrict__ badByte) {
  __shared__ uint64_t sh[kRdThreads / 64];
  __shared__ uint32_t sh32[kRdThreads / 64];
  __shared__ uint8_t stage[kRdTile];
  __shared__ uint8_t pres[256];
  pres[threadIdx.x] = present[threadIdx.x];  // kRdThreads == 256
  const uint64_t a = (uint64_t)blockIdx.x * kRdTile + threadIdx.x * kRdPerThread;
  uint8_t b[kRdPerThread];
  rd_load(raw, a, b);
  RdState s = rd_state(raw, a, len, b, carry[blockIdx.x], sh);
  uint32_t ne = 0, ns = 0;
  rd_walk(raw, a, len, b, s, [&](uint32_t, uint8_t, bool sep) {
    ne++;
    ns += sep;
  });
  uint32_t te, ts;
  const uint32_t oe = rd_block_scan<1>(ne, sh32, te);
  const uint32_t os = rd_block_scan<1>(ns, sh32, ts);
  const uint64_t ob = outBase[blockIdx.x], sb = sepBase[blockIdx.x];
  uint32_t e = oe, q = os;
  unsigned long long bad = ~0ull;
  rd_walk(raw, a, len, b, s, [&](uint32_t, uint8_t c, bool sep) {
    stage[e] = c;
    if (sep) {
      docOff[sb + q + 1] = ob + e + 1;
      q++;
    } else if (!pres[c]) {
      const unsigned long long v = ((unsigned long long)(ob + e) << 8) | c;
      bad = v < bad ? v : bad;
    }
    e++;
  });
  if (bad != ~0ull) atomicMin(badByte, bad);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < te; k += kRdThreads) out[ob + k] = stage[k];
}

void launch_rd_lastnl(const uint8_t* raw, uint64_t len, uint64_t ntiles, uint64_t* lastNl1, hipStream_t st) {
  if (ntiles) hipLaunchKernelGGL(k_rd_lastnl, dim3((unsigned)ntiles), dim3(kRdThreads), 0, st, raw, len, lastNl1);
}
void launch_rd_count(const uint8_t* raw, uint64_t len, uint64_t ntiles, const uint64_t* carry, uint32_t* cnt,
                     uint32_t* seps, hipStream_t st) {
  if (ntiles)
    hipLaunchKernelGGL(k_rd_count, dim3((unsigned)ntiles), dim3(kRdThreads), 0, st, raw, len, carry, cnt, seps);
}
void launch_rd_emit(const uint8_t* raw, uint64_t len, uint64_t ntiles, const uint64_t* carry,
                    const uint64_t* outBase, const uint64_t* sepBase, const uint8_t* present, uint8_t* out,
                    uint64_t* docOff, unsigned long long* badByte, hipStream_t st) {
  if (ntiles)
    hipLaunchKernelGGL(k_rd_emit, dim3((unsigned)ntiles), dim3(kRdThreads), 0, st, raw, len, carry, outBase,
                       sepBase, present, out, docOff, badByte);
}

}  // namespace cmsbwt

// ---------------------------------------------------------------- output
// Plain .bwt expansion of the runs (FN:1631-1694 writes N + D - 1 bytes):
// bytes [o0, o0 + len) of the expanded BWT, 256 per thread; a thread finds
// the run holding its first byte by binary search over the run starts and
// walks forward.  Records are the packed 9-byte (u64 length, char) runs.
namespace cmsbwt {

__global__ void k_out_split(const uint8_t* __restrict__ rec, uint64_t R, unsigned long long* __restrict__ len,
                            uint8_t* __restrict__ chr) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= R) return;
  const uint8_t* r = rec + 9 * j;
  unsigned long long v = 0;
#pragma unroll
  for (int b = 0; b < 8; b++) v |= (unsigned long long)r[b] << (8 * b);
  len[j] = v;
  chr[j] = r[8];
}

constexpr uint32_t kOutPerThread = 256;

__global__ void k_out_expand(const unsigned long long* __restrict__ start, const uint8_t* __restrict__ chr, uint64_t R,
                             uint64_t o0, uint64_t len, uint8_t* __restrict__ out) {
  const uint64_t a = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kOutPerThread;
  if (a >= len) return;
  const uint64_t p0 = o0 + a;
  uint64_t lo = 0, hi = R;  // last run with start <= p0
  while (hi - lo > 1) {
    const uint64_t m = (lo + hi) >> 1;
    if (start[m] <= p0) lo = m; else hi = m;
  }
  uint64_t r = lo;
  uint64_t next = r + 1 < R ? start[r + 1] : ~0ull;
  uint8_t c = chr[r];
  const uint64_t e = a + kOutPerThread < len ? a + kOutPerThread : len;
  uint64_t k = a;
  while (k < e) {
    if (o0 + k >= next) {
      r++;
      c = chr[r];
      next = r + 1 < R ? start[r + 1] : ~0ull;
      continue;
    }
    uint64_t stop = next - o0 < e ? next - o0 : e;  // bytes of run r in [k, stop)
    for (; k < stop && (k & 15); k++) out[k] = c;
    const uint32_t w = 0x01010101u * c;
    for (; k + 16 <= stop; k += 16) *reinterpret_cast<uint4*>(out + k) = make_uint4(w, w, w, w);
    for (; k < stop; k++) out[k] = c;
  }
}

void launch_out_split(const uint8_t* rec, uint64_t R, unsigned long long* len, uint8_t* chr, hipStream_t st) {
  if (R) hipLaunchKernelGGL(k_out_split, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, st, rec, R, len, chr);
}
void launch_out_expand(const unsigned long long* start, const uint8_t* chr, uint64_t R, uint64_t o0, uint64_t len,
                       uint8_t* out, hipStream_t st) {
  const uint64_t th = (len + kOutPerThread - 1) / kOutPerThread;
  if (R && len)
    hipLaunchKernelGGL(k_out_expand, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, start, chr, R, o0, len,
                       out);
}

}  // namespace cmsbwt
