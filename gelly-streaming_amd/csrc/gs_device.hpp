// gs_device.hpp — wave64 / inter-workgroup primitives shared by the gfx950 kernels.
//
// Conventions (cdna_hip_programming.md §1, §6 G16; MI355X_MICROARCH.md "Workgroup dispatch"):
//  - a wave is 64 lanes; ballots are 64-bit;
//  - look-back status words are single 8-byte granules written and read with agent-scope
//    relaxed atomics (global_store/load ... sc1), tagged with a per-call epoch so nothing has
//    to be zeroed between calls; multi-word payloads are stored sc1, drained with
//    `s_waitcnt vmcnt(0)`, then the flag granule is stored (the "sc1 payload -> vmcnt(0) ->
//    sc1 flag" hand-off);
//  - tiles are claimed in order from an atomic counter, so every tile a look-back waits on is
//    already running: the spin always terminates; it is still bounded and reports a timeout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

// number of set bits of `mask` in lanes below this one
__device__ __forceinline__ uint32_t mbcnt(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// lanes of the wave holding the same RADIX_BITS-bit digit as this lane (wave-level match_any)
template <int BITS>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t active) {
  uint64_t peers = active;
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const uint64_t m = ballot((d >> b) & 1u);
    peers &= ((d >> b) & 1u) ? m : ~m;
  }
  return peers;
}

template <typename T>
__device__ __forceinline__ T wave_inclusive_sum(T x) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    T y = __shfl_up(x, o, WAVE);
    if (l >= o) x += y;
  }
  return x;
}

__device__ __forceinline__ uint64_t wave_or(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, WAVE);
  return x;
}

// ---- look-back granules: [63:62] flag, [61:40] epoch, [39:0] value -------------------------
constexpr uint64_t FLAG_AGG = 1ull, FLAG_INC = 2ull;
constexpr uint32_t EPOCH_BITS = 22;
constexpr uint64_t VALUE_MASK = (1ull << 40) - 1;

__device__ __forceinline__ uint64_t granule(uint64_t flag, uint32_t epoch, uint64_t v) {
  return (flag << 62) | ((uint64_t)(epoch & ((1u << EPOCH_BITS) - 1)) << 40) | (v & VALUE_MASK);
}
__device__ __forceinline__ uint64_t g_flag(uint64_t g) { return g >> 62; }
__device__ __forceinline__ uint32_t g_epoch(uint64_t g) { return (uint32_t)(g >> 40) & ((1u << EPOCH_BITS) - 1); }
__device__ __forceinline__ uint64_t g_value(uint64_t g) { return g & VALUE_MASK; }

__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

constexpr uint32_t SPIN_LIMIT = 1u << 26;

// poll a granule until it carries `epoch` and a flag; bounded: sets *timeout and returns 0 on give-up
__device__ __forceinline__ uint64_t poll_granule(uint64_t* p, uint32_t epoch, uint32_t* timeout) {
  for (uint32_t spins = 0;; ++spins) {
    const uint64_t g = ld_agent(p);
    if (g_flag(g) != 0 && g_epoch(g) == (epoch & ((1u << EPOCH_BITS) - 1))) return g;
    if (spins >= SPIN_LIMIT) {
      atomicOr(timeout, 1u);
      return granule(FLAG_INC, epoch, 0);
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

}  // namespace gs
