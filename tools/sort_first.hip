// Where the first rocPRIM radix sort of a process spends its time (tools only):
// device properties, allocation, the size query, the first and second sorts.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <chrono>
#include <cstdio>
#include <vector>
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define C(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void k_fill(uint32_t* k, uint32_t* v, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { k[i] = (i * 2654435761u) >> 8; v[i] = i; }
}
int main() {
  const uint32_t n = 10000000;
  double t = now();
  C(hipFree(nullptr));
  printf("init        %.3f s\n", now() - t); t = now();
  hipDeviceProp_t pr;
  C(hipGetDeviceProperties(&pr, 0));
  printf("props       %.3f s\n", now() - t); t = now();
  uint32_t *k0, *k1, *v0, *v1;
  C(hipMalloc(&k0, n * 4)); C(hipMalloc(&k1, n * 4)); C(hipMalloc(&v0, n * 4)); C(hipMalloc(&v1, n * 4));
  printf("alloc       %.3f s\n", now() - t); t = now();
  hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n);
  C(hipDeviceSynchronize());
  printf("fill        %.3f s\n", now() - t); t = now();
  for (int rep = 0; rep < 3; rep++) {
    size_t b = 0;
    C(rocprim::radix_sort_pairs(nullptr, b, k0, k1, v0, v1, (size_t)n, 0u, 24u, (hipStream_t)0));
    printf("query %d     %.3f s (%zu B)\n", rep, now() - t, b); t = now();
    void* tmp;
    C(hipMalloc(&tmp, b));
    printf("tmp alloc %d %.3f s\n", rep, now() - t); t = now();
    C(rocprim::radix_sort_pairs(tmp, b, k0, k1, v0, v1, (size_t)n, 0u, 24u, (hipStream_t)0));
    printf("enqueue %d   %.3f s\n", rep, now() - t); t = now();
    C(hipDeviceSynchronize());
    printf("sort %d      %.3f s\n", rep, now() - t); t = now();
    C(hipFree(tmp));
  }
  std::vector<uint32_t> h(n);
  C(hipMemcpy(h.data(), k1, n * 4, hipMemcpyDeviceToHost));
  for (uint32_t i = 1; i < n; i++) if (h[i - 1] > h[i]) { printf("not sorted\n"); return 1; }
  printf("sorted ok\n");
  return 0;
}
