// gs_hashset.hip — GenerateCandidateEdges on the GPU (WindowTriangles.java:83-116) and the
// triangle self-pair term, both of which depend on java.util.HashSet<Long> iteration order.
//
// For vertex v of a slice(ALL) window the reference
//   1. emits (v, t, false) for every neighbour record t, in arrival order               (:96-100)
//   2. builds HashSet(neighbours).toArray() = ids — JDK 8+ HashMap iteration order:    (:95, :101)
//        table capacity = 16 * 2^i, the smallest with k <= 0.75 * cap (k distinct ids),
//        bucket(x) = (h ^ h >>> 16) & (cap - 1), h = Long.hashCode(x) = (int)(x ^ x >>> 32),
//        buckets ascending, each bin in insertion (first-arrival) order
//   3. emits (ids[i], ids[j], true) for i < len-1, j >= i, ids[i] > v and ids[j] > v    (:104-114)
// Pipeline (all sorts are the stable onesweep of gs_radix.hpp):
//   ALL sort with record index -> CSR (arrival order) -> composite (vertex, neighbour) sort ->
//   distinct pairs with first arrival (segmented MIN) -> per-vertex k -> order key
//   (bucket, first arrival) -> sort, then stable sort by vertex -> ids per vertex in HashSet order.
// Bins that would be treeified (>= 9 entries at capacity >= 64) have a different JDK order; such
// windows are flagged (gs_pair_out.reserved = 1, "order unpinned").
#include "gs_ops.hpp"

namespace gs {

__device__ __forceinline__ uint64_t hs_capacity(uint64_t k) {
  uint64_t cap = 16;
  while (k * 4 > cap * 3) cap <<= 1;
  return cap;
}
__device__ __forceinline__ uint32_t hs_bucket(int64_t x, uint64_t cap) {
  const uint32_t h = (uint32_t)((uint64_t)x ^ ((uint64_t)x >> 32));
  return (h ^ (h >> 16)) & (uint32_t)(cap - 1);
}
// largest u with off[u] <= p (off ascending, off[0] = 0)
__device__ __forceinline__ uint32_t seg_of(const uint64_t* __restrict__ off, uint32_t U, uint64_t p) {
  uint32_t lo = 0, hi = U - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ---- generic exclusive scan of u64 (3 launches) ----------------------------------------------
constexpr int XS_BLOCK = 256, XS_ITEMS = 16, XS_TILE = XS_BLOCK * XS_ITEMS;

__global__ __launch_bounds__(XS_BLOCK) void k_xs_tiles(const uint64_t* __restrict__ in, uint64_t n,
                                                       uint64_t* __restrict__ tile_sum) {
  __shared__ uint64_t ws[XS_BLOCK / 64];
  uint64_t t = 0;
  const uint64_t base = (uint64_t)blockIdx.x * XS_TILE;
#pragma unroll
  for (int j = 0; j < XS_ITEMS; ++j) {
    const uint64_t p = base + (uint64_t)j * XS_BLOCK + threadIdx.x;
    if (p < n) t += in[p];
  }
  t = wave_inclusive_sum(t);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
    for (int w = 0; w < XS_BLOCK / 64; ++w) s += ws[w];
    tile_sum[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(1024) void k_xs_top(uint64_t* __restrict__ tile_sum, uint32_t ntiles) {
  __shared__ uint64_t ws[16];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < ntiles; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint64_t x = i < ntiles ? tile_sum[i] : 0ull;
    const uint64_t inc = wave_inclusive_sum(x);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint64_t off = carry;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += ws[w];
    if (i < ntiles) tile_sum[i] = off + inc - x;
    __syncthreads();
    if (threadIdx.x == 1023) carry = off + inc;
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_sum[ntiles] = carry;
}

__global__ __launch_bounds__(XS_BLOCK) void k_xs_apply(const uint64_t* __restrict__ in, uint64_t n,
                                                       const uint64_t* __restrict__ tile_off,
                                                       uint64_t* __restrict__ out) {
  __shared__ uint64_t ws[XS_BLOCK / 64];
  const uint64_t first = (uint64_t)blockIdx.x * XS_TILE + (uint64_t)threadIdx.x * XS_ITEMS;
  uint64_t v[XS_ITEMS];
  uint64_t t = 0;
#pragma unroll
  for (int j = 0; j < XS_ITEMS; ++j) {
    v[j] = (first + j < n) ? in[first + j] : 0ull;
    t += v[j];
  }
  const uint64_t inc = wave_inclusive_sum(t);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint64_t off = tile_off[blockIdx.x] + inc - t;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += ws[w];
#pragma unroll
  for (int j = 0; j < XS_ITEMS; ++j) {
    if (first + j < n) out[first + j] = off;
    off += v[j];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == XS_BLOCK - 1) out[n] = tile_off[gridDim.x];
}

// ---- pipeline kernels -------------------------------------------------------------------------
// per sorted record position p: neighbour (original ID), owning vertex, composite (u << B | x)
// (composite = (u << B) | rank(x): vertices are densely ranked, so any Long ID range fits 64 bits)
__global__ __launch_bounds__(256) void k_hs_prep(const uint32_t* __restrict__ rec, uint32_t R,
                                                 const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                 const uint64_t* __restrict__ off, const int64_t* __restrict__ vkeys,
                                                 uint32_t U, uint32_t B, int64_t* __restrict__ nbr,
                                                 uint32_t* __restrict__ useg, uint64_t* __restrict__ comp,
                                                 uint32_t* __restrict__ pidx) {
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < R; p += gridDim.x * 256u) {
    const uint32_t r = rec[p];
    const uint32_t i = r >> 1;
    const int64_t x = (r & 1u) ? src[i] : dst[i];   // ALL: r = 2i -> (src, dst), 2i+1 -> (dst, src)
    const uint32_t u = seg_of(off, U, p);
    uint32_t lo = 0, hi = U - 1;                      // rank of x among the window's vertices
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (vkeys[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    nbr[p] = x;
    useg[p] = u;
    comp[p] = ((uint64_t)u << B) | lo;
    pidx[p] = p;
  }
}

// distinct (u, x) with the first arrival position (segmented MIN over the stable sort's payload)
struct DistinctOut {
  uint64_t* keys;
  uint32_t* first;
  __device__ void store(uint32_t m, int64_t k, uint32_t a, uint32_t) const {
    keys[m] = (uint64_t)k;
    first[m] = a;
  }
};
// per-vertex start of its distinct entries (the vertex index is the shifted key)
struct StartOut {
  uint64_t* doff;
  __device__ void store(uint32_t, int64_t k, uint64_t cnt, uint32_t end_pos) const {
    doff[k + 1] = (uint64_t)end_pos + 1;
  }
};

__global__ __launch_bounds__(256) void k_hs_orderkey(const uint64_t* __restrict__ dkey, const uint32_t* __restrict__ dfirst,
                                                     uint32_t M, uint32_t B, const int64_t* __restrict__ vkeys,
                                                     const uint64_t* __restrict__ off, const uint64_t* __restrict__ doff,
                                                     uint64_t* __restrict__ okey, uint32_t* __restrict__ omid) {
  const uint64_t mask = (B >= 64) ? ~0ull : ((1ull << B) - 1);
  for (uint32_t m = blockIdx.x * 256u + threadIdx.x; m < M; m += gridDim.x * 256u) {
    const uint64_t k = dkey[m];
    const uint32_t u = (uint32_t)(k >> B);
    const int64_t x = vkeys[k & mask];
    const uint64_t cap = hs_capacity(doff[u + 1] - doff[u]);
    const uint32_t rel = dfirst[m] - (uint32_t)off[u];
    okey[m] = ((uint64_t)hs_bucket(x, cap) << 32) | rel;
    omid[m] = m;
  }
}

__global__ __launch_bounds__(256) void k_hs_vertex_of(const uint32_t* __restrict__ mid, const uint64_t* __restrict__ dkey,
                                                      uint32_t M, uint32_t B, uint64_t* __restrict__ ukey,
                                                      uint32_t* __restrict__ mid_out) {
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) {
    const uint32_t m = mid[q];
    ukey[q] = dkey[m] >> B;
    mid_out[q] = m;
  }
}

// ids in HashSet order (original IDs) + treeification check
__global__ __launch_bounds__(256) void k_hs_ids(const uint32_t* __restrict__ ord, const uint64_t* __restrict__ dkey,
                                                uint32_t M, uint32_t B, const int64_t* __restrict__ vkeys,
                                                const uint64_t* __restrict__ doff,
                                                uint32_t U, int64_t* __restrict__ ids, uint32_t* __restrict__ treeified) {
  const uint64_t mask = (B >= 64) ? ~0ull : ((1ull << B) - 1);
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) {
    const uint64_t k = dkey[ord[q]];
    const int64_t x = vkeys[k & mask];
    ids[q] = x;
    const uint32_t u = (uint32_t)(k >> B);
    const uint64_t end = doff[u + 1];
    const uint64_t cap = hs_capacity(end - doff[u]);
    if (cap >= 64 && q + 8 < end) {
      const uint64_t k8 = dkey[ord[q + 8]];
      const int64_t x8 = vkeys[k8 & mask];
      if (hs_bucket(x, cap) == hs_bucket(x8, cap)) atomicOr(treeified, 1u);
    }
  }
}

// gt[q] = ids[q] > v(u)   (signed Long order, WindowTriangles.java:108)
__global__ __launch_bounds__(256) void k_hs_gt(const int64_t* __restrict__ ids, uint32_t M, const uint64_t* __restrict__ doff,
                                               uint32_t U, const int64_t* __restrict__ vkeys, uint64_t* __restrict__ g) {
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) {
    const uint32_t u = seg_of(doff, U, q);
    g[q] = ids[q] > vkeys[u] ? 1ull : 0ull;
  }
}

// row q emits (ids[q], ids[j]) for j >= q with ids[j] > v; only rows q < end-1 with ids[q] > v (:104, :108)
__global__ __launch_bounds__(256) void k_hs_rowlen(const uint64_t* __restrict__ gx, uint32_t M,
                                                   const uint64_t* __restrict__ doff, uint32_t U,
                                                   const int64_t* __restrict__ ids, const int64_t* __restrict__ vkeys,
                                                   uint64_t* __restrict__ L) {
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) {
    const uint32_t u = seg_of(doff, U, q);
    const uint64_t end = doff[u + 1];
    const bool gt = ids[q] > vkeys[u];
    L[q] = (gt && q + 1 < end) ? (gx[end] - gx[q]) : 0ull;
  }
}

__global__ __launch_bounds__(256) void k_hs_emit_false(uint32_t R, const uint32_t* __restrict__ useg,
                                                       const uint64_t* __restrict__ doff, const uint64_t* __restrict__ LS,
                                                       const int64_t* __restrict__ vkeys, const int64_t* __restrict__ nbr,
                                                       int64_t* __restrict__ a, int64_t* __restrict__ b,
                                                       uint8_t* __restrict__ f) {
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < R; p += gridDim.x * 256u) {
    const uint32_t u = useg[p];
    const uint64_t pos = p + LS[doff[u]];
    a[pos] = vkeys[u];
    b[pos] = nbr[p];
    f[pos] = 0;
  }
}

__global__ __launch_bounds__(256) void k_hs_emit_pairs(uint32_t M, const uint64_t* __restrict__ doff, uint32_t U,
                                                       const uint64_t* __restrict__ off, const uint64_t* __restrict__ LS,
                                                       const int64_t* __restrict__ ids, const int64_t* __restrict__ vkeys,
                                                       int64_t* __restrict__ a, int64_t* __restrict__ b,
                                                       uint8_t* __restrict__ f) {
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) {
    if (LS[q + 1] == LS[q]) continue;
    const uint32_t u = seg_of(doff, U, q);
    const int64_t v = vkeys[u], xi = ids[q];
    uint64_t o = off[u + 1] + LS[q];
    const uint64_t end = doff[u + 1];
    for (uint64_t j = q; j < end; ++j) {
      const int64_t xj = ids[j];
      if (xj > v) {
        a[o] = xi;
        b[o] = xj;
        f[o] = 1;
        ++o;
      }
    }
  }
}

// self-pair term of WindowTriangles: matched (x, x, true) candidates need a self-loop on x
__global__ __launch_bounds__(256) void k_hs_selfpairs(const int64_t* __restrict__ ids, uint32_t M,
                                                      const uint64_t* __restrict__ doff, uint32_t U,
                                                      const int64_t* __restrict__ vkeys, const uint32_t* __restrict__ loops,
                                                      uint64_t key_xor, const int64_t* __restrict__ relabel,
                                                      uint64_t nrel, unsigned long long* __restrict__ S) {
  uint64_t t = 0;
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) {
    const uint32_t u = seg_of(doff, U, q);
    const int64_t v = vkeys[u], x = ids[q];
    if (q + 1 < doff[u + 1] && x > v) {   // rows i < len-1 emit (x, x) when x > v
      uint64_t c = (uint64_t)x ^ key_xor;
      if (relabel) {   // rank of x among the window's sorted distinct IDs
        uint64_t lo = 0, hi = nrel;
        while (lo < hi) {
          const uint64_t mid = (lo + hi) >> 1;
          if (relabel[mid] < x) lo = mid + 1;
          else hi = mid;
        }
        c = lo;
      }
      if ((loops[c >> 5] >> (c & 31)) & 1u) ++t;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if ((threadIdx.x & 63) == 0 && t) atomicAdd(S, (unsigned long long)t);
}

}  // namespace gs

using namespace gs;

namespace gs {

enum { HS_VKEYS, HS_OFF, HS_NBR, HS_USEG, HS_COMP, HS_PIDX, HS_DKEY, HS_DFIRST, HS_DOFF, HS_OKEY, HS_OMID,
       HS_UKEY, HS_ORD, HS_IDS, HS_G, HS_GX, HS_L, HS_LS, HS_TILES, HS_COUNT };

gs_status xscan(gs_ctx* c, const uint64_t* in, uint64_t n, uint64_t* out) {
  const uint32_t tiles = (uint32_t)std::max<uint64_t>(1, (n + XS_TILE - 1) / XS_TILE);
  GS_TRY(ensure(c, c->hs[HS_TILES], (size_t)(tiles + 1) * 8));
  uint64_t* ts = c->hs[HS_TILES].as<uint64_t>();
  hipLaunchKernelGGL(k_xs_tiles, dim3(tiles), dim3(XS_BLOCK), 0, c->stream, in, n, ts);
  hipLaunchKernelGGL(k_xs_top, dim3(1), dim3(1024), 0, c->stream, ts, tiles);
  hipLaunchKernelGGL(k_xs_apply, dim3(tiles), dim3(XS_BLOCK), 0, c->stream, in, n, (const uint64_t*)ts, out);
  return hip_check(c, hipGetLastError(), "exclusive scan");
}

static unsigned g256(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384)); }

// Distinct neighbour sets of every vertex of an ALL window, in HashSet order.  Results in c->hs[...]:
// HS_VKEYS[U] vertex IDs, HS_OFF[U+1] record offsets, HS_NBR[R] neighbours (arrival order),
// HS_USEG[R] vertex of each record, HS_DOFF[U+1] distinct offsets, HS_IDS[M] ids in HashSet order.
gs_status hashset_order(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, uint32_t* U_out,
                        uint32_t* M_out, uint64_t* key_xor_out, bool* treeified) {
  char* sm = c->small.as<char>();
  const uint64_t R = 2 * n;
  Sorted s;
  GS_TRY(sort_window(c, src, dst, nullptr, 0, n, DIR_ALL, PAY_IDX, &s));
  GS_TRY(ensure(c, c->hs[HS_VKEYS], R * 8));
  GS_TRY(ensure(c, c->hs[HS_OFF], (R + 1) * 8));
  GS_HIP(hipMemsetAsync(c->hs[HS_OFF].p, 0, 8, c->stream));
  CsrOut co{c->hs[HS_VKEYS].as<int64_t>(), c->hs[HS_OFF].as<uint64_t>()};
  uint64_t U = 0;
  GS_TRY((s.wide ? launch_rbk<uint64_t, CountOp>(c, s, co, &U) : launch_rbk<uint32_t, CountOp>(c, s, co, &U)));
  // copy the record order out of the sort buffers (the next sorts reuse them)
  GS_TRY(ensure(c, c->hs[HS_PIDX], R * 4));
  GS_TRY(ensure(c, c->hs[HS_NBR], R * 8));
  GS_TRY(ensure(c, c->hs[HS_USEG], R * 4));
  GS_TRY(ensure(c, c->hs[HS_COMP], R * 8));
  GS_TRY(ensure(c, c->hs[HS_ORD], R * 4));
  GS_HIP(hipMemcpyAsync(c->hs[HS_ORD].p, s.vals, R * 4, hipMemcpyDeviceToDevice, c->stream));
  const uint32_t B = U > 1 ? 64 - __builtin_clzll(U - 1) : 1;   // bits of a dense vertex rank
  hipLaunchKernelGGL(k_hs_prep, dim3(g256(R)), dim3(256), 0, c->stream, c->hs[HS_ORD].as<uint32_t>(), (uint32_t)R, src,
                     dst, c->hs[HS_OFF].as<uint64_t>(), c->hs[HS_VKEYS].as<int64_t>(), (uint32_t)U, B,
                     c->hs[HS_NBR].as<int64_t>(),
                     c->hs[HS_USEG].as<uint32_t>(), c->hs[HS_COMP].as<uint64_t>(), c->hs[HS_PIDX].as<uint32_t>());
  GS_HIP(hipGetLastError());
  // distinct (u, x) with first arrival
  Sorted s2;
  GS_TRY(sort_buffer(c, c->hs[HS_COMP].as<uint64_t>(), c->hs[HS_PIDX].as<uint32_t>(), R, &s2));
  GS_TRY(ensure(c, c->hs[HS_DKEY], R * 8));
  GS_TRY(ensure(c, c->hs[HS_DFIRST], R * 4));
  DistinctOut dout{c->hs[HS_DKEY].as<uint64_t>(), c->hs[HS_DFIRST].as<uint32_t>()};
  uint64_t M = 0;
  GS_TRY((s2.wide ? launch_rbk<uint64_t, ValueOp<uint32_t, OP_MIN>>(c, s2, dout, &M)
                  : launch_rbk<uint32_t, ValueOp<uint32_t, OP_MIN>>(c, s2, dout, &M)));
  // distinct offsets per vertex
  GS_TRY(ensure(c, c->hs[HS_DOFF], (U + 1) * 8));
  GS_HIP(hipMemsetAsync(c->hs[HS_DOFF].p, 0, 8, c->stream));
  Sorted sd;
  sd.keys = c->hs[HS_DKEY].p;
  sd.wide = true;
  sd.key_xor = 0;
  sd.records = M;
  StartOut so{c->hs[HS_DOFF].as<uint64_t>()};
  uint64_t U2 = 0;
  GS_TRY((launch_rbk<uint64_t, CountOp>(c, sd, so, &U2, B)));
  if (U2 != U) return set_error(c, GS_EDEVICE, "candidates: vertex count mismatch (%llu vs %llu)",
                                (unsigned long long)U2, (unsigned long long)U);
  // HashSet order: sort by (bucket, first arrival), then stably by vertex
  GS_TRY(ensure(c, c->hs[HS_OKEY], M * 8));
  GS_TRY(ensure(c, c->hs[HS_OMID], M * 4));
  hipLaunchKernelGGL(k_hs_orderkey, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_DKEY].as<uint64_t>(),
                     c->hs[HS_DFIRST].as<uint32_t>(), (uint32_t)M, B, c->hs[HS_VKEYS].as<int64_t>(),
                     c->hs[HS_OFF].as<uint64_t>(),
                     c->hs[HS_DOFF].as<uint64_t>(), c->hs[HS_OKEY].as<uint64_t>(), c->hs[HS_OMID].as<uint32_t>());
  GS_HIP(hipGetLastError());
  Sorted sa;
  GS_TRY(sort_buffer(c, c->hs[HS_OKEY].as<uint64_t>(), c->hs[HS_OMID].as<uint32_t>(), M, &sa));
  GS_TRY(ensure(c, c->hs[HS_UKEY], M * 8));
  hipLaunchKernelGGL(k_hs_vertex_of, dim3(g256(M)), dim3(256), 0, c->stream, (const uint32_t*)sa.vals,
                     c->hs[HS_DKEY].as<uint64_t>(), (uint32_t)M, B, c->hs[HS_UKEY].as<uint64_t>(),
                     c->hs[HS_OMID].as<uint32_t>());
  GS_HIP(hipGetLastError());
  Sorted sb;
  GS_TRY(sort_buffer(c, c->hs[HS_UKEY].as<uint64_t>(), c->hs[HS_OMID].as<uint32_t>(), M, &sb));
  GS_TRY(ensure(c, c->hs[HS_IDS], M * 8));
  uint32_t* d_tree = (uint32_t*)(sm + SM_TIMEOUT) + 1;   // spare word next to the timeout flag
  GS_HIP(hipMemsetAsync(d_tree, 0, 4, c->stream));
  hipLaunchKernelGGL(k_hs_ids, dim3(g256(M)), dim3(256), 0, c->stream, (const uint32_t*)sb.vals,
                     c->hs[HS_DKEY].as<uint64_t>(), (uint32_t)M, B, c->hs[HS_VKEYS].as<int64_t>(),
                     c->hs[HS_DOFF].as<uint64_t>(),
                     (uint32_t)U, c->hs[HS_IDS].as<int64_t>(), d_tree);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 6, sm + SM_TIMEOUT, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *treeified = (c->host_small[6] >> 32) != 0;
  *U_out = (uint32_t)U;
  *M_out = (uint32_t)M;
  *key_xor_out = s.key_xor;
  return GS_OK;
}

// S term of the triangle count (see gs_graph.hip): loops = self-loop bitmap over compact IDs
gs_status triangle_selfpair_term(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n,
                                 const uint32_t* loops, uint64_t loops_xor, const int64_t* relabel, uint64_t nrel,
                                 uint64_t* S) {
  uint32_t U = 0, M = 0;
  uint64_t key_xor = 0;
  bool tree = false;
  GS_TRY(hashset_order(c, src, dst, n, &U, &M, &key_xor, &tree));
  if (tree) return set_error(c, GS_EUNSUPPORTED, "triangles: a neighbour set would use a treeified HashMap bin");
  char* sm = c->small.as<char>();
  unsigned long long* d = (unsigned long long*)(sm + SM_TOTAL);
  GS_HIP(hipMemsetAsync(d, 0, 8, c->stream));
  hipLaunchKernelGGL(k_hs_selfpairs, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_IDS].as<int64_t>(), M,
                     c->hs[HS_DOFF].as<uint64_t>(), U, c->hs[HS_VKEYS].as<int64_t>(), loops, loops_xor, relabel,
                     nrel, d);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 7, d, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *S = c->host_small[7];
  return GS_OK;
}

}  // namespace gs

extern "C" {

gs_status gs_window_candidates(gs_ctx* c, const gs_edge_batch* b, gs_pair_out* out) {
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!out || !out->n_out || (out->capacity && (!out->a || !out->b || !out->is_candidate)))
    return set_error(c, GS_EINVAL, "bad gs_pair_out");
  GS_TRY(begin_call(c));
  out->reserved = 0;
  if (b->n == 0) {
    *out->n_out = 0;
    return GS_OK;
  }
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  const uint64_t R = 2 * b->n;
  uint32_t U = 0, M = 0;
  uint64_t key_xor = 0;
  bool tree = false;
  GS_TRY(hashset_order(c, src, dst, b->n, &U, &M, &key_xor, &tree));
  out->reserved = tree ? 1 : 0;   // 1 = a treeified bin: JDK order of that vertex not reproduced
  // rows: gt flags -> scan -> row lengths -> scan
  GS_TRY(ensure(c, c->hs[HS_G], (M + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_GX], (M + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_L], (M + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_LS], (M + 1) * 8));
  hipLaunchKernelGGL(k_hs_gt, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_IDS].as<int64_t>(), M,
                     c->hs[HS_DOFF].as<uint64_t>(), U, c->hs[HS_VKEYS].as<int64_t>(), c->hs[HS_G].as<uint64_t>());
  GS_HIP(hipGetLastError());
  GS_TRY(xscan(c, c->hs[HS_G].as<uint64_t>(), M, c->hs[HS_GX].as<uint64_t>()));
  hipLaunchKernelGGL(k_hs_rowlen, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_GX].as<uint64_t>(), M,
                     c->hs[HS_DOFF].as<uint64_t>(), U, c->hs[HS_IDS].as<int64_t>(), c->hs[HS_VKEYS].as<int64_t>(),
                     c->hs[HS_L].as<uint64_t>());
  GS_HIP(hipGetLastError());
  GS_TRY(xscan(c, c->hs[HS_L].as<uint64_t>(), M, c->hs[HS_LS].as<uint64_t>()));
  uint64_t P = 0;
  GS_HIP(hipMemcpyAsync(&c->host_small[7], c->hs[HS_LS].as<uint64_t>() + M, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  P = c->host_small[7];
  const uint64_t total = R + P;
  *out->n_out = total;
  if (total > out->capacity) return set_error(c, GS_ECAPACITY, "candidates need %llu records", (unsigned long long)total);
  int64_t *a = out->a, *bb = out->b;
  uint8_t* f = out->is_candidate;
  const bool direct = out->mem == GS_MEM_DEVICE;
  if (!direct) {
    GS_TRY(ensure(c, c->out_keys, total * 8));
    GS_TRY(ensure(c, c->out_a, total * 8));
    GS_TRY(ensure(c, c->out_b, total));
    a = c->out_keys.as<int64_t>();
    bb = c->out_a.as<int64_t>();
    f = c->out_b.as<uint8_t>();
  }
  hipLaunchKernelGGL(k_hs_emit_false, dim3(g256(R)), dim3(256), 0, c->stream, (uint32_t)R, c->hs[HS_USEG].as<uint32_t>(),
                     c->hs[HS_DOFF].as<uint64_t>(), c->hs[HS_LS].as<uint64_t>(), c->hs[HS_VKEYS].as<int64_t>(),
                     c->hs[HS_NBR].as<int64_t>(), a, bb, f);
  hipLaunchKernelGGL(k_hs_emit_pairs, dim3(g256(M)), dim3(256), 0, c->stream, M, c->hs[HS_DOFF].as<uint64_t>(), U,
                     c->hs[HS_OFF].as<uint64_t>(), c->hs[HS_LS].as<uint64_t>(), c->hs[HS_IDS].as<int64_t>(),
                     c->hs[HS_VKEYS].as<int64_t>(), a, bb, f);
  GS_HIP(hipGetLastError());
  if (!direct) {
    GS_HIP(hipMemcpyAsync(out->a, a, total * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(out->b, bb, total * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(out->is_candidate, f, total, hipMemcpyDeviceToHost, c->stream));
  }
  GS_TRY(host_wait(c));
  return GS_OK;
}

}  // extern "C"
