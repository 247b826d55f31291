// gs_gen.hip — counter-based synthetic edge streams on the device.
// Bit-identical to oracle/gs_oracle.c (gso_gen_*), so CPU and GPU see the same windows.
#include <math.h>

#include <vector>

#include "gs_ops.hpp"

namespace gs {

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Perm {
  uint64_t mask, k0, k1, a0, a1;
  int sh;
  __device__ uint64_t operator()(uint64_t x) const {
    x = (x * k0 + a0) & mask;
    x ^= x >> sh;
    x = (x * k1 + a1) & mask;
    x ^= x >> sh;
    x = (x * k0 + a1) & mask;
    return x;
  }
};

__global__ __launch_bounds__(256) void k_gen_rmat(int scale, uint64_t n, uint64_t seed, uint32_t a, uint32_t ab,
                                                  uint32_t abc, int permute, int no_self_loops, uint64_t first,
                                                  Perm perm, int64_t* __restrict__ src, int64_t* __restrict__ dst) {
  const uint64_t V = 1ull << scale;
  const uint64_t per = (uint64_t)((scale + 1) / 2);
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256) {
    const uint64_t i = first + k;
    uint64_t u = 0, v = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
      if ((l & 1) == 0) r = splitmix64(seed, i * per + (uint64_t)(l >> 1));
      const uint32_t x = (l & 1) ? (uint32_t)(r >> 32) : (uint32_t)r;
      const uint64_t sb = (x >= ab), db = (x >= a && x < ab) || (x >= abc);
      u = (u << 1) | sb;
      v = (v << 1) | db;
    }
    if (no_self_loops && u == v) v = (u + 1 + splitmix64(seed ^ 0x5E1F100Bull, i) % (V - 1)) & (V - 1);
    if (permute) {
      u = perm(u);
      v = perm(v);
    }
    src[k] = (int64_t)u;
    dst[k] = (int64_t)v;
  }
}

__global__ __launch_bounds__(256) void k_gen_uniform(uint64_t V, uint64_t n, uint64_t seed, uint64_t first,
                                                     int64_t* __restrict__ src, int64_t* __restrict__ dst) {
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256) {
    const uint64_t i = first + k;
    const uint64_t s = splitmix64(seed, 2 * i) % V;
    const uint64_t d = (s + 1 + splitmix64(seed, 2 * i + 1) % (V - 1)) % V;
    src[k] = (int64_t)s;
    dst[k] = (int64_t)d;
  }
}

__global__ __launch_bounds__(256) void k_gen_values(uint64_t n, uint64_t seed, uint64_t first, int dtype,
                                                    void* __restrict__ val) {
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256) {
    const uint64_t r = splitmix64(seed ^ 0xA5A5A5A5F00DF00Dull, first + k);
    switch (dtype) {
      case GS_I32: ((int32_t*)val)[k] = (int32_t)(r & 0xFFFF); break;
      case GS_I64: ((int64_t*)val)[k] = (int64_t)(r & 0xFFFF); break;
      case GS_F32: ((float*)val)[k] = (float)(r >> 40) * (1.0f / 16777216.0f); break;
      case GS_F64: ((double*)val)[k] = (double)(r >> 11) * (1.0 / 9007199254740992.0); break;
    }
  }
}

// Zipf sources: the smallest k with cdf[k] > u (53-bit fixed point, cdf[V - 1] = 2^53)
__global__ __launch_bounds__(256) void k_gen_zipf(const uint64_t* __restrict__ cdf, uint64_t V, uint64_t n,
                                                  uint64_t seed, uint64_t first, int64_t* __restrict__ src,
                                                  int64_t* __restrict__ dst) {
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256) {
    const uint64_t i = first + k;
    const uint64_t u = splitmix64(seed ^ 0x21F0A5EDull, i) >> 11;
    uint64_t lo = 0, hi = V - 1;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (cdf[mid] > u) hi = mid;
      else lo = mid + 1;
    }
    src[k] = (int64_t)lo;
    dst[k] = (int64_t)(splitmix64(seed ^ 0xD5D5D5D5ull, i) % V);
  }
}

static unsigned gen_grid(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace gs

using namespace gs;

extern "C" {

gs_status gs_generate_rmat(gs_ctx* c, int32_t scale, uint64_t n, uint64_t seed, uint32_t a_fx, uint32_t b_fx,
                           uint32_t c_fx, int32_t permute, int32_t no_self_loops, uint64_t first_edge,
                           int64_t* src, int64_t* dst) {
  if (!c) return GS_EINVAL;
  if (scale < 1 || scale > 62 || (n && (!src || !dst)))
    return set_error(c, GS_EINVAL, "bad R-MAT arguments (scale %d)", scale);
  if ((uint64_t)a_fx + b_fx + c_fx >= (1ull << 32)) return set_error(c, GS_EINVAL, "a+b+c must be < 1");
  if (!n) return GS_OK;
  hipSetDevice(c->device);
  Perm p;
  p.mask = (1ull << scale) - 1;
  p.k0 = splitmix64(seed, 0x51) | 1ull;
  p.k1 = splitmix64(seed, 0x52) | 1ull;
  p.a0 = splitmix64(seed, 0x53);
  p.a1 = splitmix64(seed, 0x54);
  p.sh = scale > 1 ? (scale + 1) / 2 : 1;
  hipLaunchKernelGGL(k_gen_rmat, dim3(gen_grid(n)), dim3(256), 0, c->stream, scale, n, seed, a_fx, a_fx + b_fx,
                     a_fx + b_fx + c_fx, permute, no_self_loops, first_edge, p, src, dst);
  return hip_check(c, hipGetLastError(), "k_gen_rmat");
}

gs_status gs_generate_uniform(gs_ctx* c, uint64_t V, uint64_t n, uint64_t seed, uint64_t first_edge, int64_t* src,
                              int64_t* dst) {
  if (!c) return GS_EINVAL;
  if (V < 2 || (n && (!src || !dst))) return set_error(c, GS_EINVAL, "bad uniform arguments");
  if (!n) return GS_OK;
  hipSetDevice(c->device);
  hipLaunchKernelGGL(k_gen_uniform, dim3(gen_grid(n)), dim3(256), 0, c->stream, V, n, seed, first_edge, src, dst);
  return hip_check(c, hipGetLastError(), "k_gen_uniform");
}

gs_status gs_generate_zipf(gs_ctx* c, uint64_t V, double exponent, uint64_t n, uint64_t seed, uint64_t first_edge,
                           int64_t* src, int64_t* dst) {
  if (!c) return GS_EINVAL;
  if (V < 2 || V > (1ull << 32) || !(exponent > 0.0) || (n && (!src || !dst)))
    return set_error(c, GS_EINVAL, "bad Zipf arguments");
  if (!n) return GS_OK;
  hipSetDevice(c->device);
  if (c->zipf_v != V || c->zipf_s != exponent) {
    // the CDF table: a sequential double sum of pow() terms (the oracle's gso_zipf_cdf, same arithmetic)
    std::vector<uint64_t> cdf(V);
    double cum = 0.0;
    for (uint64_t k = 0; k < V; ++k) cum += pow((double)(k + 1), -exponent);
    const double total = cum;
    cum = 0.0;
    for (uint64_t k = 0; k < V; ++k) {
      cum += pow((double)(k + 1), -exponent);
      cdf[k] = (uint64_t)((cum / total) * 9007199254740992.0);
    }
    cdf[V - 1] = 1ull << 53;
    GS_TRY(ensure(c, c->zipf_cdf, V * 8));
    GS_HIP(hipMemcpy(c->zipf_cdf.p, cdf.data(), V * 8, hipMemcpyHostToDevice));
    c->zipf_v = V;
    c->zipf_s = exponent;
  }
  hipLaunchKernelGGL(k_gen_zipf, dim3(gen_grid(n)), dim3(256), 0, c->stream, c->zipf_cdf.as<uint64_t>(), V, n, seed,
                     first_edge, src, dst);
  return hip_check(c, hipGetLastError(), "k_gen_zipf");
}

gs_status gs_generate_values(gs_ctx* c, uint64_t n, uint64_t seed, uint64_t first_edge, int32_t dtype, void* val) {
  if (!c) return GS_EINVAL;
  if (dtype < GS_I32 || dtype > GS_F64 || (n && !val)) return set_error(c, GS_EINVAL, "bad value arguments");
  if (!n) return GS_OK;
  hipSetDevice(c->device);
  hipLaunchKernelGGL(k_gen_values, dim3(gen_grid(n)), dim3(256), 0, c->stream, n, seed, first_edge, dtype, val);
  return hip_check(c, hipGetLastError(), "k_gen_values");
}

}  // extern "C"
