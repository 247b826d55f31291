// Reference point only (not the product): hipCUB DeviceRadixSort::SortPairs on the C2 window's
// compact keys (u32, 24 bits) with u64 values, timed with hipEvents — what a vendor library onesweep
// achieves on this GPU for the same traffic as our 3 radix passes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void fill(uint32_t* k, uint64_t* v, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z ^= z >> 31;
    k[i] = (uint32_t)(z & 0xFFFFFF); v[i] = z >> 40;
  }
}
int main() {
  const size_t n = 1ull << 28;
  uint32_t *k0, *k1; uint64_t *v0, *v1;
  CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v0, n * 8)); CK(hipMalloc(&v1, n * 8));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, k0, v0, n);
  size_t tmp = 0;
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k0, k1, v0, v1, (int)n, 0, 24));
  void* t; CK(hipMalloc(&t, tmp));
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int it = 0; it < 2; ++it) CK(hipcub::DeviceRadixSort::SortPairs(t, tmp, k0, k1, v0, v1, (int)n, 0, 24));
  hipEventRecord(a);
  const int reps = 5;
  for (int it = 0; it < reps; ++it) CK(hipcub::DeviceRadixSort::SortPairs(t, tmp, k0, k1, v0, v1, (int)n, 0, 24));
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  printf("{\"hipcub_sortpairs_u32key_u64val_24bit_n\": %zu, \"ms\": %.3f}\n", n, ms / reps);
  // keys only
  for (int it = 0; it < 2; ++it) CK(hipcub::DeviceRadixSort::SortKeys(t, tmp, k0, k1, (int)n, 0, 24));
  hipEventRecord(a);
  for (int it = 0; it < reps; ++it) CK(hipcub::DeviceRadixSort::SortKeys(t, tmp, k0, k1, (int)n, 0, 24));
  hipEventRecord(b); hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  printf("{\"hipcub_sortkeys_u32_24bit_n\": %zu, \"ms\": %.3f}\n", n, ms / reps);
  return 0;
}
