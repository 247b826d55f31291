// gs_relabel.hip — compact vertex IDs for windows whose Long IDs are arbitrary (sparse, negative, wider
// than the composite-key budget).  The reference parses any Long (WindowTriangles.java:175-185) and
// its HashSet / keyBy work on the values themselves; the triangle pipeline packs two IDs into one
// 64-bit key, so a window whose IDs span more than TRI_MAX_BITS bits is relabeled first:
//   endpoints (2n, sign-flipped so unsigned order = Long order) -> stable LSD sort with positions ->
//   first-of-run flags -> exclusive scan -> compact ID of every endpoint (its rank among the distinct
//   IDs) + the sorted distinct IDs.
// The relabeling is order-preserving (compact ID order = Long order), so everything that compares IDs
// (orientation ties, a > v filters) is unchanged; what needs the original value (the JDK HashSet
// order of the self-pair term) maps back through the sorted distinct IDs.
#include "gs_ops.hpp"

namespace gs {

__global__ __launch_bounds__(256) void k_rl_keys(const int64_t* __restrict__ a, const int64_t* __restrict__ b, uint64_t n,
                                                 uint64_t* __restrict__ keys, uint32_t* __restrict__ pos) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    keys[2 * i] = (uint64_t)a[i] ^ (1ull << 63);
    keys[2 * i + 1] = (uint64_t)b[i] ^ (1ull << 63);
    pos[2 * i] = (uint32_t)(2 * i);
    pos[2 * i + 1] = (uint32_t)(2 * i + 1);
  }
}

template <typename K>
__global__ __launch_bounds__(256) void k_rl_flags(const K* __restrict__ keys, uint64_t R, uint64_t* __restrict__ flags) {
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < R; p += (uint64_t)gridDim.x * 256)
    flags[p] = (p == 0 || keys[p] != keys[p - 1]) ? 1u : 0u;
}

template <typename K>
__global__ __launch_bounds__(256) void k_rl_scatter(const K* __restrict__ keys, uint64_t key_xor,
                                                    const uint32_t* __restrict__ pos, const uint64_t* __restrict__ flags,
                                                    const uint64_t* __restrict__ excl, uint64_t R,
                                                    uint32_t* __restrict__ at, int64_t* __restrict__ uniq) {
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < R; p += (uint64_t)gridDim.x * 256) {
    const uint64_t rank = excl[p] + flags[p] - 1;
    at[pos[p]] = (uint32_t)rank;
    if (flags[p]) uniq[rank] = (int64_t)(((uint64_t)keys[p] ^ key_xor) ^ (1ull << 63));
  }
}

__global__ __launch_bounds__(256) void k_rl_cols(const uint32_t* __restrict__ at, uint64_t n, int64_t* __restrict__ ca,
                                                 int64_t* __restrict__ cb) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    ca[i] = at[2 * i];
    cb[i] = at[2 * i + 1];
  }
}

gs_status relabel_endpoints(gs_ctx* c, const int64_t* a, const int64_t* b, uint64_t n, const int64_t** ca,
                            const int64_t** cb, const int64_t** uniq, uint64_t* V) {
  const uint64_t R = 2 * n;
  if (R >= (1ull << 32)) return set_error(c, GS_EUNSUPPORTED, "relabel: more than 2^32 - 1 endpoints");
  GS_TRY(ensure(c, c->rl[0], R * 8));   // keys
  GS_TRY(ensure(c, c->rl[1], R * 4));   // positions
  GS_TRY(ensure(c, c->rl[2], R * 8 + 8));   // flags
  GS_TRY(ensure(c, c->rl[3], R * 8 + 8));   // exclusive scan
  GS_TRY(ensure(c, c->rl[4], R * 4));   // compact ID per endpoint
  GS_TRY(ensure(c, c->rl[5], R * 8));   // sorted distinct IDs
  GS_TRY(ensure(c, c->rl[6], n * 8 + 8));   // compact columns
  GS_TRY(ensure(c, c->rl[7], n * 8 + 8));
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192));
  const unsigned gR = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((R + 255) / 256, 8192));
  hipLaunchKernelGGL(k_rl_keys, dim3(g), dim3(256), 0, c->stream, a, b, n, c->rl[0].as<uint64_t>(),
                     c->rl[1].as<uint32_t>());
  GS_HIP(hipGetLastError());
  Sorted s;
  GS_TRY(sort_buffer(c, c->rl[0].as<uint64_t>(), c->rl[1].as<uint32_t>(), R, &s));
  uint64_t* flags = c->rl[2].as<uint64_t>();
  uint64_t* excl = c->rl[3].as<uint64_t>();
  if (s.wide) hipLaunchKernelGGL(k_rl_flags<uint64_t>, dim3(gR), dim3(256), 0, c->stream, (const uint64_t*)s.keys, R, flags);
  else hipLaunchKernelGGL(k_rl_flags<uint32_t>, dim3(gR), dim3(256), 0, c->stream, (const uint32_t*)s.keys, R, flags);
  GS_HIP(hipGetLastError());
  GS_TRY(xscan(c, flags, R, excl));
  if (s.wide)
    hipLaunchKernelGGL(k_rl_scatter<uint64_t>, dim3(gR), dim3(256), 0, c->stream, (const uint64_t*)s.keys, s.key_xor,
                       (const uint32_t*)s.vals, flags, excl, R, c->rl[4].as<uint32_t>(), c->rl[5].as<int64_t>());
  else
    hipLaunchKernelGGL(k_rl_scatter<uint32_t>, dim3(gR), dim3(256), 0, c->stream, (const uint32_t*)s.keys, s.key_xor,
                       (const uint32_t*)s.vals, flags, excl, R, c->rl[4].as<uint32_t>(), c->rl[5].as<int64_t>());
  hipLaunchKernelGGL(k_rl_cols, dim3(g), dim3(256), 0, c->stream, c->rl[4].as<uint32_t>(), n, c->rl[6].as<int64_t>(),
                     c->rl[7].as<int64_t>());
  GS_HIP(hipGetLastError());
  // distinct IDs = exclusive scan at R - 1 + flag at R - 1
  GS_HIP(hipMemcpyAsync(c->host_small + 16, excl + R - 1, 8, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small + 17, flags + R - 1, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *V = c->host_small[16] + c->host_small[17];
  *ca = c->rl[6].as<int64_t>();
  *cb = c->rl[7].as<int64_t>();
  *uniq = c->rl[5].as<int64_t>();
  return GS_OK;
}

// Compact ids of a window split over ranks (gs_window_triangles_dist): a rank's local compact ids
// (relabel_endpoints over its own records: ranks among ITS distinct ids) become ranks among the WHOLE
// window's sorted distinct ids G (every rank's distinct ids all-gathered and relabeled the same way, so
// every rank holds the same G).  Each local distinct id is searched in G once; the columns are gathered
// through that map in place.
__global__ __launch_bounds__(256) void k_rl_rank(const int64_t* __restrict__ loc, uint64_t nloc,
                                                 const int64_t* __restrict__ G, uint64_t ng, uint32_t* __restrict__ map) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nloc; i += (uint64_t)gridDim.x * 256) {
    const int64_t x = loc[i];
    uint64_t lo = 0, hi = ng;   // first position with G[p] >= x (x is in G)
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (G[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    map[i] = (uint32_t)lo;
  }
}

__global__ __launch_bounds__(256) void k_rl_map(int64_t* __restrict__ ca, int64_t* __restrict__ cb, uint64_t n,
                                                const uint32_t* __restrict__ map) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    ca[i] = map[ca[i]];
    cb[i] = map[cb[i]];
  }
}

gs_status relabel_to_global(gs_ctx* c, const int64_t* loc, uint64_t nloc, const int64_t* G, uint64_t ng, uint32_t* map,
                            int64_t* ca, int64_t* cb, uint64_t n) {
  if (!n) return GS_OK;
  const unsigned gl = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nloc + 255) / 256, 8192));
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192));
  hipLaunchKernelGGL(k_rl_rank, dim3(gl), dim3(256), 0, c->stream, loc, nloc, G, ng, map);
  hipLaunchKernelGGL(k_rl_map, dim3(g), dim3(256), 0, c->stream, ca, cb, n, (const uint32_t*)map);
  return hip_check(c, hipGetLastError(), "relabel_to_global");
}

}  // namespace gs
