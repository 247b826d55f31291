// LDS atomic throughput probe (not part of the library): one 1024-thread workgroup per CU, each
// lane issuing N adds at pseudo-random positions of a 2^S-entry LDS array, as k_bk_accum's
// accumulation does.  Variants: 64-bit add (no return), 32-bit add (no return), 32-bit add with
// return + a carry word on wrap, and 32-bit add with 4 records per lane.  Prints ns per record per CU.
//
// build: hipcc -O3 --offload-arch=gfx950 -o lds_atomic lds_atomic.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int BLOCK = 1024, N = 4096;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

template <int MODE, int S>
__global__ __launch_bounds__(BLOCK) void k_probe(uint64_t* out, uint32_t seed) {
  constexpr uint32_t W = 1u << S;
  __shared__ uint64_t s64[MODE == 0 ? W : 1];
  __shared__ uint32_t s32[MODE != 0 ? W : 1];
  __shared__ uint32_t s_hi[MODE == 2 ? W / 4 : 1];
  const int tid = threadIdx.x;
  for (uint32_t i = tid; i < W; i += BLOCK) {
    if constexpr (MODE == 0) s64[i] = 0;
    else s32[i] = 0;
    if constexpr (MODE == 2) if (i < W / 4) s_hi[i] = 0;
  }
  __syncthreads();
  uint32_t h = mix(seed ^ (blockIdx.x * BLOCK + tid));
  for (int r = 0; r < N; ++r) {
    h = h * 1664525u + 1013904223u;
    const uint32_t i = (h >> 8) & (W - 1), v = (h >> 20) & 0xFFFu;
    if constexpr (MODE == 0) {
      atomicAdd((unsigned long long*)&s64[i], (unsigned long long)v);
    } else if constexpr (MODE == 1) {
      atomicAdd(&s32[i], v);
    } else {
      const uint32_t old = atomicAdd(&s32[i], v);
      if (old + v < old) atomicAdd(&s_hi[i >> 2], 1u << (8 * (i & 3)));
    }
  }
  __syncthreads();
  uint64_t acc = 0;
  for (uint32_t i = tid; i < W; i += BLOCK) acc += MODE == 0 ? s64[i] : s32[i];
  if (MODE == 2) for (uint32_t i = tid; i < W / 4; i += BLOCK) acc += s_hi[i];
  atomicAdd((unsigned long long*)out, (unsigned long long)acc);
}

template <int MODE, int S>
void run(const char* name, int cus, uint64_t* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_probe<MODE, S><<<cus, BLOCK>>>(d, 1);
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k_probe<MODE, S><<<cus, BLOCK>>>(d, 2 + r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double recs = (double)cus * BLOCK * N * reps;
  printf("{\"variant\": \"%s\", \"S\": %d, \"ms\": %.4f, \"records_per_clk_per_cu_at_2.4GHz\": %.3f, \"G_records_per_s\": %.1f}\n",
         name, S, ms / reps, recs / cus / (ms * 1e-3) / 2.4e9, recs / (ms * 1e-3) / 1e9);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint64_t* d;
  hipMalloc(&d, 8);
  run<0, 14>("ds_add_u64", cus, d);
  run<1, 14>("ds_add_u32", cus, d);
  run<2, 14>("ds_add_rtn_u32+carry", cus, d);
  run<1, 15>("ds_add_u32", cus, d);
  run<0, 13>("ds_add_u64", cus, d);
  hipFree(d);
  return 0;
}
