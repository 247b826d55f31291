// Achievable HBM rate for the C2 scatter's byte mix (read 16 B, write 4 B per record), perfectly
// coalesced: the floor the speculative scatter is compared with.
//   hipcc -O3 --offload-arch=gfx950 stream_mix.hip -o stream_mix && ./stream_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_mix(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                             uint2* __restrict__ out, uint64_t n2) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (uint64_t)gridDim.x * 256) {
    const uint4 x = a[i], y = b[i];   // two records' keys, two records' values
    out[i] = make_uint2(x.x ^ y.x, x.z ^ y.z);
  }
}
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                              uint32_t* __restrict__ sink, uint64_t n2) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (uint64_t)gridDim.x * 256) {
    const uint4 x = a[i], y = b[i];
    acc ^= x.x ^ y.y ^ x.z ^ y.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint64_t n = 1ull << 28;   // records
  uint4 *a, *b;
  uint2* o;
  uint32_t* sink;
  hipMalloc(&a, n * 8);
  hipMalloc(&b, n * 8);
  hipMalloc(&o, n * 4);
  hipMalloc(&sink, 64);
  hipMemset(a, 1, n * 8);
  hipMemset(b, 2, n * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int grid : {1024, 2048, 4096, 8192}) {
    for (int which = 0; which < 2; ++which) {
      float best = 1e9f;
      for (int rep = 0; rep < 10; ++rep) {
        hipEventRecord(e0);
        if (which == 0) hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, a, b, o, n / 2);
        else hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, b, sink, n / 2);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep > 1 && ms < best) best = ms;
      }
      const double bytes = which == 0 ? 20.0 * n : 16.0 * n;
      printf("%s grid %5d: %.4f ms  %.2f TB/s\n", which == 0 ? "read16+write4" : "read16      ", grid, best,
             bytes / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
