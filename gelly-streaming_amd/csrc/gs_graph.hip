// gs_graph.hip — neighbourhood grouping (applyOnNeighbors) and the WindowTriangles operators.
//
//   gs_window_csr        <- the grouping half of applyOnNeighbors (GraphWindowStream.java:130-175)
//   gs_window_candidates <- applyOnNeighbors(GenerateCandidateEdges)   (WindowTriangles.java:83-116)
//   gs_window_triangles  <- slice(ALL) -> candidates -> CountTriangles -> sum(0) (WindowTriangles.java:61-66)
#include "gs_ops.hpp"
#include "gs_tricount.hpp"

namespace gs {

// sorted position p holds record index r (stable sort => arrival order inside each vertex):
// neighbours[p] = other endpoint of record r, vals[p] = value of its edge
template <int DIR>
__global__ __launch_bounds__(256) void k_gather_csr(const uint32_t* __restrict__ rec, uint32_t R,
                                                    const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                    const void* __restrict__ val, int vbytes,
                                                    int64_t* __restrict__ nbrs, void* __restrict__ vals) {
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < R; p += gridDim.x * 256u) {
    const uint32_t r = rec[p];
    uint32_t i = r;
    bool rev = (DIR == DIR_IN);
    if (DIR == DIR_ALL) {
      i = r >> 1;
      rev = r & 1u;
    }
    nbrs[p] = rev ? src[i] : dst[i];
    if (vals) {
      if (vbytes == 4) ((uint32_t*)vals)[p] = ((const uint32_t*)val)[i];
      else ((uint64_t*)vals)[p] = ((const uint64_t*)val)[i];
    }
  }
}


// ---------------------------------------------------------------------------------------------
// WindowTriangles: exact count of the reference's matched candidates without emitting them.
//   T = triangles of the window's simple undirected graph (GenerateCandidateEdges emits each
//       {b, c} pair of neighbours > v once per v; CountTriangles matches it iff b ~ c, and ALL
//       makes both (b,c) and (c,b) edge records) -> counted once each by the forward algorithm
//       on a (degree, id)-oriented CSR with sorted adjacency (merge intersection).
//   S = self-pair quirk (j = i emits (x, x); matched only if x has a self-loop) — needs
//       java.util.HashSet iteration order; only windows with self-loops have S != 0.
// ---------------------------------------------------------------------------------------------
constexpr uint64_t TRI_MAX_BITS = 28;

// composite symmetric adjacency keys (a << B | b), both directions; self-loops -> sentinel + flag
__global__ __launch_bounds__(256) void k_tri_sym(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                 uint64_t n, uint64_t key_xor, uint32_t B,
                                                 uint64_t* __restrict__ out, uint32_t* __restrict__ loop_bits,
                                                 unsigned long long* __restrict__ loops) {
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t a = (uint64_t)src[i] ^ key_xor, b = (uint64_t)dst[i] ^ key_xor;
    if (a != b) {
      out[2 * i] = (a << B) | b;
      out[2 * i + 1] = (b << B) | a;
    } else {
      out[2 * i] = sent;
      out[2 * i + 1] = sent;
      atomicOr(&loop_bits[a >> 5], 1u << (a & 31));
      atomicAdd(loops, 1ull);
    }
  }
}

// per vertex row of the unique symmetric adjacency: deg[v], rowstart[v]
struct RowOut {
  uint32_t* deg;
  uint32_t* rowstart;
  __device__ void store(uint32_t, int64_t k, uint64_t cnt, uint32_t end_pos) const {
    deg[k] = (uint32_t)cnt;
    rowstart[k] = end_pos + 1 - (uint32_t)cnt;
  }
};

__device__ __forceinline__ bool oriented(uint32_t du, uint32_t u, uint32_t dv, uint32_t v) {
  return du < dv || (du == dv && u < v);
}

constexpr int SCAN_BLOCK = 256, SCAN_ITEMS = 16, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

// keep flag per adjacency entry (u -> v kept iff (deg u, u) < (deg v, v)) + per-tile counts
__global__ __launch_bounds__(SCAN_BLOCK) void k_orient_count(const uint64_t* __restrict__ adj, uint32_t E2, uint32_t B,
                                                             const uint32_t* __restrict__ deg,
                                                             uint8_t* __restrict__ keep, uint32_t* __restrict__ tile_sum) {
  __shared__ uint32_t ws[SCAN_BLOCK / 64];
  const uint64_t mask = (1ull << B) - 1;
  uint32_t cnt = 0;
  const uint32_t base = blockIdx.x * SCAN_TILE;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint32_t p = base + j * SCAN_BLOCK + threadIdx.x;
    if (p < E2) {
      const uint64_t k = adj[p];
      const uint32_t u = (uint32_t)(k >> B), v = (uint32_t)(k & mask);
      const bool kp = oriented(deg[u], u, deg[v], v);
      keep[p] = kp;
      cnt += kp;
    }
  }
  cnt = wave_inclusive_sum(cnt);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < SCAN_BLOCK / 64; ++w) t += ws[w];
    tile_sum[blockIdx.x] = t;
  }
}

// exclusive scan of tile sums in one workgroup (tiles <= a few 10^5); writes total at [ntiles]
__global__ __launch_bounds__(1024) void k_scan_tiles(uint32_t* __restrict__ tile_sum, uint32_t ntiles) {
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < ntiles; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t x = i < ntiles ? tile_sum[i] : 0u;
    const uint32_t inc = wave_inclusive_sum(x);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint32_t off = carry;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += ws[w];
    if (i < ntiles) tile_sum[i] = off + inc - x;
    __syncthreads();
    if (threadIdx.x == 1023) carry = off + inc;
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_sum[ntiles] = carry;
}

// pos[p] = #kept before p (pos[E2] = M); kept entries compact into onbr (out-lists), the others into
// inbr (in-lists, at p - pos[p]); order preserved
__global__ __launch_bounds__(SCAN_BLOCK) void k_orient_scatter(const uint64_t* __restrict__ adj, uint32_t E2, uint32_t B,
                                                               const uint8_t* __restrict__ keep,
                                                               const uint32_t* __restrict__ tile_off,
                                                               uint32_t* __restrict__ pos, uint32_t* __restrict__ inbr,
                                                               uint32_t* __restrict__ onbr) {
  __shared__ uint32_t ws[SCAN_BLOCK / 64];
  const uint64_t mask = (1ull << B) - 1;
  const uint32_t base = blockIdx.x * SCAN_TILE;
  // blocked: thread t owns entries [base + t*ITEMS, +ITEMS) so the scan order is entry order
  const uint32_t first = base + threadIdx.x * SCAN_ITEMS;
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint32_t p = first + j;
    if (p < E2) cnt += keep[p];
  }
  const uint32_t inc = wave_inclusive_sum(cnt);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t off = tile_off[blockIdx.x] + inc - cnt;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += ws[w];
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const uint32_t p = first + j;
    if (p < E2) {
      pos[p] = off;
      const uint32_t x = (uint32_t)(adj[p] & mask);
      if (keep[p]) onbr[off++] = x;
      else inbr[p - off] = x;
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == SCAN_BLOCK - 1) pos[E2] = tile_off[gridDim.x];
}

}  // namespace gs

using namespace gs;

extern "C" {

gs_status gs_window_csr(gs_ctx* c, const gs_edge_batch* b, int32_t dir, gs_csr_out* out) {
  GS_TRY(check_batch(c, b, dir));
  if (!out || !out->n_vertices || !out->n_records) return set_error(c, GS_EINVAL, "bad gs_csr_out");
  GS_TRY(begin_call(c));
  const uint64_t R = dir == GS_DIR_ALL ? 2 * b->n : b->n;
  *out->n_records = R;
  if (R == 0) {
    *out->n_vertices = 0;
    if (out->offsets && out->capacity_vertices + 1 >= 1) {
      const uint64_t z = 0;
      GS_HIP(hipMemcpy(out->offsets, &z, 8, out->mem == GS_MEM_DEVICE ? hipMemcpyHostToDevice : hipMemcpyHostToHost));
    }
    return GS_OK;
  }
  const bool want_vals = out->vals && b->val_dtype != GS_NONE && b->val;
  hipEventRecord(c->ev[0], c->stream);
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, want_vals));
  Sorted s;
  GS_TRY(sort_window(c, src, dst, nullptr, 0, b->n, dir, PAY_IDX, &s));
  hipEventRecord(c->ev[2], c->stream);
  const size_t vb = dtype_bytes(b->val_dtype);
  const bool direct = out->mem == GS_MEM_DEVICE && out->capacity_vertices >= R && out->capacity_records >= R;
  int64_t *kd = out->keys, *nd = out->neighbors;
  uint64_t* od = out->offsets;
  void* vd = want_vals ? out->vals : nullptr;
  if (!direct) {
    GS_TRY(ensure(c, c->out_keys, R * 8));
    GS_TRY(ensure(c, c->out_a, (R + 1) * 8));
    GS_TRY(ensure(c, c->out_b, R * 8));
    kd = c->out_keys.as<int64_t>();
    od = c->out_a.as<uint64_t>();
    nd = c->out_b.as<int64_t>();
    if (want_vals) {
      GS_TRY(ensure(c, c->aux, R * vb));
      vd = c->aux.p;
    }
  }
  GS_HIP(hipMemsetAsync(od, 0, 8, c->stream));
  CsrOut o{kd, od};
  uint64_t U = 0;
  GS_TRY((s.wide ? launch_rbk<uint64_t, CountOp>(c, s, o, &U) : launch_rbk<uint32_t, CountOp>(c, s, o, &U)));
  const unsigned grid = (unsigned)std::min<uint64_t>((R + 255) / 256, 8192);
  switch (dir) {
    case GS_DIR_IN:
      hipLaunchKernelGGL(k_gather_csr<DIR_IN>, dim3(grid), dim3(256), 0, c->stream, (const uint32_t*)s.vals,
                         (uint32_t)R, src, dst, val, (int)vb, nd, vd);
      break;
    case GS_DIR_OUT:
      hipLaunchKernelGGL(k_gather_csr<DIR_OUT>, dim3(grid), dim3(256), 0, c->stream, (const uint32_t*)s.vals,
                         (uint32_t)R, src, dst, val, (int)vb, nd, vd);
      break;
    default:
      hipLaunchKernelGGL(k_gather_csr<DIR_ALL>, dim3(grid), dim3(256), 0, c->stream, (const uint32_t*)s.vals,
                         (uint32_t)R, src, dst, val, (int)vb, nd, vd);
  }
  GS_HIP(hipGetLastError());
  finish_times(c, s, U);
  *out->n_vertices = U;
  if (U > out->capacity_vertices || R > out->capacity_records)
    return set_error(c, GS_ECAPACITY, "csr needs %llu vertices / %llu records", (unsigned long long)U,
                     (unsigned long long)R);
  GS_TRY(deliver(c, out->keys, kd, U * 8, out->mem));
  GS_TRY(deliver(c, out->offsets, od, (U + 1) * 8, out->mem));
  GS_TRY(deliver(c, out->neighbors, nd, R * 8, out->mem));
  if (want_vals) GS_TRY(deliver(c, out->vals, vd, R * vb, out->mem));
  GS_TRY(host_wait(c));
  return GS_OK;
}

static gs_status triangles_impl(gs_ctx* c, const gs_edge_batch* b, uint32_t part, uint32_t nparts, uint64_t* count) {
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!count) return set_error(c, GS_EINVAL, "null output pointer");
  if (nparts == 0 || part >= nparts) return set_error(c, GS_EINVAL, "bad part %u of %u", part, nparts);
  GS_TRY(begin_call(c));
  *count = 0;
  if (b->n == 0) return GS_OK;
  hipEventRecord(c->ev[0], c->stream);
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  char* sm = c->small.as<char>();
  const uint64_t n = b->n;
  // key range of the window (same scan as the sort)
  GS_HIP(hipMemsetAsync(sm, 0, SM_TIMEOUT, c->stream));
  GS_HIP(hipMemsetAsync(sm + SM_COUNTERS, 0, SM_BASE - SM_COUNTERS, c->stream));
  GS_TRY(launch_keyinfo_all(c, src, dst, n));
  GS_HIP(hipMemcpyAsync(sm + SM_K0, src, 8, hipMemcpyDeviceToDevice, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small, sm, 16, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t mask = c->host_small[0], k0 = c->host_small[1];
  uint32_t B = mask ? 64 - __builtin_clzll(mask) : 1;
  uint64_t key_xor = k0 & ~((1ull << B) - 1);
  // IDs wider than the composite-key budget: relabel (order-preserving compact IDs); the originals
  // stay for the self-pair term's HashSet order
  const int64_t *osrc = src, *odst = dst, *uniq = nullptr;
  uint64_t nuniq = 0;
  if (B > TRI_MAX_BITS) {
    GS_TRY(relabel_endpoints(c, osrc, odst, n, &src, &dst, &uniq, &nuniq));
    B = nuniq > 1 ? 64 - __builtin_clzll(nuniq - 1) : 1;
    key_xor = 0;
    if (B > TRI_MAX_BITS)
      return set_error(c, GS_EUNSUPPORTED, "window triangles: %llu distinct vertices (> 2^%llu)",
                       (unsigned long long)nuniq, (unsigned long long)TRI_MAX_BITS);
  }
  const uint64_t R = 2 * n;
  // 1. symmetric composite keys (+ self-loop bitmap)
  GS_TRY(ensure(c, c->aux, R * 8));
  const size_t words = ((1ull << B) + 31) / 32;
  GS_TRY(ensure(c, c->tri_loops, words * 4));
  GS_HIP(hipMemsetAsync(c->tri_loops.p, 0, words * 4, c->stream));
  unsigned long long* d_loops = (unsigned long long*)(sm + SM_NUNIQUE);
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_tri_sym, dim3(g), dim3(256), 0, c->stream, src, dst, n, key_xor, B, c->aux.as<uint64_t>(),
                     c->tri_loops.as<uint32_t>(), d_loops);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 4, d_loops, 8, hipMemcpyDeviceToHost, c->stream));
  // 2. sort + unique -> symmetric simple adjacency, sorted by (u, v)
  Sorted s;
  GS_TRY(sort_buffer(c, c->aux.as<uint64_t>(), nullptr, R, &s));
  hipEventRecord(c->ev[1], c->stream);
  const uint64_t loops = c->host_small[4];
  GS_TRY(ensure(c, c->out_keys, R * 8));
  uint64_t E2 = 0;
  UniqueOut uo{c->out_keys.as<uint64_t>(), nullptr};
  GS_TRY((s.wide ? launch_rbk<uint64_t, CountOp>(c, s, uo, &E2) : launch_rbk<uint32_t, CountOp>(c, s, uo, &E2)));
  hipEventRecord(c->ev[2], c->stream);
  if (loops) E2 -= 1;   // the self-loop sentinel sorts last
  if (E2 == 0) {        // only self-loops: no triangle; the self-pair term needs >= 2 neighbours
    uint64_t S = 0;
    if (part == 0) GS_TRY(triangle_selfpair_term(c, osrc, odst, n, c->tri_loops.as<uint32_t>(), key_xor, uniq, nuniq, &S));
    *count = S;
    return GS_OK;
  }
  // 3. rows: degree + row start per vertex (segment by u = key >> B)
  const size_t V = 1ull << B;
  GS_TRY(ensure(c, c->out_a, V * 4));
  GS_TRY(ensure(c, c->out_b, V * 4));
  Sorted adj;
  adj.keys = c->out_keys.p;
  adj.wide = true;
  adj.key_xor = 0;
  adj.records = E2;
  GS_HIP(hipMemsetAsync(c->out_a.p, 0, V * 4, c->stream));   // vertices without edges: degree 0
  GS_TRY(ensure(c, c->tri_heavy, (V + E2 / 2 / TH_VCH + 64) * 8));   // (v, in-chunk) items
  GS_TRY(ensure(c, c->tri_range, V * 16));
  RowOut ro{c->out_a.as<uint32_t>(), c->out_b.as<uint32_t>()};
  uint64_t nv = 0;
  GS_TRY((launch_rbk<uint64_t, CountOp>(c, adj, ro, &nv, B)));
  // 4. orientation by (degree, id): keep flags, scan, compaction (order preserved)
  const uint32_t tiles = (uint32_t)((E2 + SCAN_TILE - 1) / SCAN_TILE);
  GS_TRY(ensure(c, c->tri_keep, E2 + 16));
  GS_TRY(ensure(c, c->tri_tiles, (tiles + 1) * 4));
  GS_TRY(ensure(c, c->tri_pos, (E2 + 1) * 4));
  GS_TRY(ensure(c, c->tri_ou, E2 * 4));
  GS_TRY(ensure(c, c->tri_onbr, E2 * 4));
  hipLaunchKernelGGL(k_orient_count, dim3(tiles), dim3(SCAN_BLOCK), 0, c->stream, c->out_keys.as<uint64_t>(),
                     (uint32_t)E2, B, c->out_a.as<uint32_t>(), c->tri_keep.as<uint8_t>(), c->tri_tiles.as<uint32_t>());
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, c->stream, c->tri_tiles.as<uint32_t>(), tiles);
  hipLaunchKernelGGL(k_orient_scatter, dim3(tiles), dim3(SCAN_BLOCK), 0, c->stream, c->out_keys.as<uint64_t>(),
                     (uint32_t)E2, B, c->tri_keep.as<uint8_t>(), c->tri_tiles.as<uint32_t>(),
                     c->tri_pos.as<uint32_t>(), c->tri_ou.as<uint32_t>(), c->tri_onbr.as<uint32_t>());
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[4], c->stream);
  const uint64_t M = E2 / 2;   // each undirected edge kept in exactly one direction
  GS_TRY(ensure(c, c->tri_queue, (M / TH_DMAX + 64) * 8));   // further in-list chunks: <= M / TH_DMAX
  // 5. intersections: vertex-centric LDS hash sets (k_tri_light), long out-lists in k_tri_heavy
  unsigned long long* d_total = (unsigned long long*)(sm + SM_NUNIQUE);
  uint32_t* d_nheavy = (uint32_t*)(sm + SM_COUNTERS) + 62;
  unsigned long long* d_probes = (unsigned long long*)(sm + SM_TRI_PROBES);
  GS_HIP(hipMemsetAsync(d_total, 0, 8, c->stream));
  GS_HIP(hipMemsetAsync(d_probes, 0, 8, c->stream));
  GS_HIP(hipMemsetAsync(d_nheavy, 0, 4, c->stream));
  uint32_t* d_err = (uint32_t*)(sm + SM_DEV_ERR);
  GS_HIP(hipMemsetAsync(d_err, 0, 4, c->stream));
  // LDS hash-set bucket cap: unlimited, or one bucket under GS_FLAG_TEST_TINY_TABLES (tests only)
  const uint32_t nb_cap = (c->flags & GS_FLAG_TEST_TINY_TABLES) ? 1u : 0xFFFFFFFFu;
  const uint64_t q0 = M * part / nparts, q1 = M * (part + 1) / nparts;   // this part's oriented edges
  uint2* out_range = reinterpret_cast<uint2*>(c->tri_range.p);
  uint2* in_range = out_range + V;
  uint32_t* d_nqueue = d_nheavy + 1;
  GS_HIP(hipMemsetAsync(d_nqueue, 0, 4, c->stream));
  hipLaunchKernelGGL(k_tri_rows, dim3((unsigned)std::min<uint64_t>((V + 255) / 256, 4096)), dim3(256), 0, c->stream,
                     c->out_a.as<uint32_t>(), c->out_b.as<uint32_t>(), c->tri_pos.as<uint32_t>(), (uint32_t)V,
                     out_range, in_range);
  const unsigned nvb = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((V + TH_WPB - 1) / TH_WPB, 8192));
  uint2* queue = c->tri_queue.as<uint2>();
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(k_tri_light, dim3(pass == 0 ? nvb : 4096u), dim3(TH_BLOCK), 0, c->stream,
                       c->tri_onbr.as<uint32_t>(), c->tri_ou.as<uint32_t>(), out_range, in_range, (uint32_t)V,
                       (uint32_t)q0, (uint32_t)q1, pass, queue, d_nqueue, c->tri_heavy.as<uint2>(), d_nheavy,
                       d_total, d_probes, nb_cap, d_err);
    GS_HIP(hipGetLastError());
  }
  hipEventRecord(c->ev[5], c->stream);
  hipLaunchKernelGGL(k_tri_heavy, dim3(GS_TH_HGRID), dim3(TH_HBLOCK), 0, c->stream, c->tri_onbr.as<uint32_t>(),
                     c->tri_ou.as<uint32_t>(), out_range, in_range, c->tri_heavy.as<uint2>(), d_nheavy, d_total,
                     d_probes, nb_cap, d_err);
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[3], c->stream);
  GS_HIP(hipMemcpyAsync(c->host_small, sm, 32, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small + 6, d_probes, 8, hipMemcpyDeviceToHost, c->stream));
  c->host_small[7] = 0;   // (the copy below fills the low 4 bytes)
  GS_HIP(hipMemcpyAsync(c->host_small + 7, d_err, 4, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if ((uint32_t)c->host_small[3] != 0) return set_error(c, GS_EDEVICE, "look-back spin timed out");
  if ((uint32_t)c->host_small[7] & GS_DERR_TABLE_FULL)
    return set_error(c, GS_EDEVICE, "window triangles: an LDS hash set filled up (counting aborted)");
  uint64_t T = c->host_small[2];
  {   // stage times (path 3): sym + sort, unique, rows + orientation, light count, heavy count
    gs_stage_times& t = c->times;
    t = gs_stage_times{};
    const int order[6] = {0, 1, 2, 4, 5, 3};
    for (int i = 0; i < 5; ++i) hipEventElapsedTime(&t.pass_ms[i], c->ev[order[i]], c->ev[order[i + 1]]);
    hipEventElapsedTime(&t.total_ms, c->ev[0], c->ev[3]);
    t.sort_passes = (uint32_t)s.passes;
    t.key_bits = B;
    t.records = E2;
    t.vertices = nv;
    t.partials = c->host_small[6];
    t.path = 3;
  }
  if (loops && part == 0) {   // self-pair candidates (x, x, true) matched by a self-loop on x (:105)
    uint64_t S = 0;
    GS_TRY(triangle_selfpair_term(c, osrc, odst, n, c->tri_loops.as<uint32_t>(), key_xor, uniq, nuniq, &S));
    T += S;
  }
  *count = T;
  return GS_OK;
}

gs_status gs_window_triangles(gs_ctx* c, const gs_edge_batch* b, uint64_t* count, int32_t* count_ref_wrapped,
                              int32_t* has_output) {
  if (!c) return GS_EINVAL;
  if (!count || !count_ref_wrapped || !has_output) return set_error(c, GS_EINVAL, "null output pointer");
  uint64_t T = 0;
  GS_TRY(triangles_impl(c, b, 0, 1, &T));
  *count = T;
  *count_ref_wrapped = (int32_t)(uint32_t)T;   // Integer sum(0) wraps (WindowTriangles.java:66, :126)
  *has_output = b && b->n > 0;   // every edge record forms a (v, t) group with edges > 0 (WindowTriangles.java:136)
  return GS_OK;
}

gs_status gs_window_triangles_part(gs_ctx* c, const gs_edge_batch* b, uint32_t part, uint32_t nparts,
                                   uint64_t* partial_count) {
  if (!c) return GS_EINVAL;
  return triangles_impl(c, b, part, nparts, partial_count);
}


}  // extern "C"
