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

// Vertices are renumbered by degree before the adjacency is built: rank(x) orders (degree class, id),
// so in the renumbered graph "u -> v iff u < v" is the degree orientation.  Only the oriented keys
// (min rank << B | max rank) are sorted (n keys, not the 2n of a symmetric adjacency): unique -> the
// out-lists, sorted in orientation order; a second, narrow sort of the unique edges by target
// (B-bit keys, adjacency position as payload) groups them into in-lists.  Sorted out-lists are what
// halve the probes: for u -> v only the part of N+(u) above v can hold a w with v -> w, so each
// in-neighbour u of v contributes the suffix of N+(u) after v, and the in-list entry carries that
// suffix's range (R-MAT scale 20: sum of d+(u)^2 = 2.47 G probes -> sum of d+(d+-1)/2 = 1.23 G).
// Any total order gives the exact count; the degree classes only keep out-lists short.

// raw degree per (compact) vertex over the window's records: the bucket path's COUNT over both
// endpoints (bucket_reduce), scattered into a dense array.  Windows the bucket path does not take (id
// range too wide for its buckets) count with global atomics instead -- one request per endpoint, and
// an R-MAT hub's atomics serialize on its address, so each block first counts into an LDS table that
// keeps the first ids to claim a slot (the frequent ones, almost surely) and flushes it at the end.
__global__ __launch_bounds__(256) void k_tri_deg_scatter(const int64_t* __restrict__ keys, const int64_t* __restrict__ cnt,
                                                         uint64_t U, uint64_t key_xor, uint32_t* __restrict__ deg) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < U; i += (uint64_t)gridDim.x * 256)
    deg[(uint64_t)keys[i] ^ key_xor] = (uint32_t)cnt[i];
}

constexpr int DG_BLOCK = 512, DG_SLOTS = 4096;
__global__ __launch_bounds__(DG_BLOCK) void k_tri_deg(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      uint64_t n, uint64_t key_xor, uint32_t* __restrict__ deg) {
  __shared__ uint32_t s_key[DG_SLOTS], s_cnt[DG_SLOTS];
  for (int i = threadIdx.x; i < DG_SLOTS; i += DG_BLOCK) {
    s_key[i] = 0xFFFFFFFFu;
    s_cnt[i] = 0;
  }
  __syncthreads();
  auto add = [&](uint32_t x) {
    const uint32_t h = (x * 0x9E3779B1u) >> (32 - 12);
    uint32_t k = s_key[h];
    if (k == 0xFFFFFFFFu) {
      k = atomicCAS(&s_key[h], 0xFFFFFFFFu, x);
      if (k == 0xFFFFFFFFu) k = x;
    }
    if (k == x) atomicAdd(&s_cnt[h], 1u);
    else atomicAdd(&deg[x], 1u);
  };
  static_assert(DG_SLOTS == 1 << 12, "hash shift");
  for (uint64_t i = (uint64_t)blockIdx.x * DG_BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * DG_BLOCK) {
    add((uint32_t)((uint64_t)src[i] ^ key_xor));
    add((uint32_t)((uint64_t)dst[i] ^ key_xor));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < DG_SLOTS; i += DG_BLOCK)
    if (s_cnt[i]) atomicAdd(&deg[s_key[i]], s_cnt[i]);
}

// degree class: 0 for isolated ids, then two classes per octave
constexpr int RK_BLOCK = 256, RK_STEPS = 32, RK_WAVES = RK_BLOCK / WAVE, RK_TILE = RK_BLOCK * RK_STEPS, RK_NC = 64;
__device__ __forceinline__ uint32_t deg_class(uint32_t d) {
  if (!d) return 0;
  const uint32_t lz = 31u - (uint32_t)__clz(d);
  const uint32_t half = lz ? (d >> (lz - 1)) & 1u : 0u;
  return min((uint32_t)RK_NC - 1, 1u + 2u * lz + half);
}

// per tile of RK_TILE ids: ids per class -> cnt[class * tiles + tile]
__global__ __launch_bounds__(RK_BLOCK) void k_rank_count(const uint32_t* __restrict__ deg, uint32_t V, uint32_t tiles,
                                                         uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_c[RK_NC];
  const int tid = threadIdx.x;
  if (tid < RK_NC) s_c[tid] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RK_TILE;
  for (int j = 0; j < RK_STEPS; ++j) {
    const uint32_t x = base + j * RK_BLOCK + tid;
    if (x < V) atomicAdd(&s_c[deg_class(deg[x])], 1u);
  }
  __syncthreads();
  if (tid < RK_NC) cnt[tid * tiles + blockIdx.x] = s_c[tid];
}

// one block: exclusive scan of cnt[0 .. n) (class-major) in place
__global__ __launch_bounds__(1024) void k_rank_scan(uint32_t* __restrict__ cnt, uint32_t n) {
  __shared__ uint32_t s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t per = (n + 1023) / 1024, a = min(n, tid * per), b = min(n, a + per);
  uint32_t sum = 0;
  for (uint32_t i = a; i < b; ++i) sum += cnt[i];
  const uint32_t inc = wave_inclusive_sum(sum);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (int i = 0; i < w; ++i) run += s_w[i];
  for (uint32_t i = a; i < b; ++i) {
    const uint32_t x = cnt[i];
    cnt[i] = run;
    run += x;
  }
}

// rank[x] = ids of lower classes + ids of x's class below x (a stable partition: deterministic, so
// every rank of a multi-GPU job renumbers identically).  Wave w of a tile takes RK_STEPS groups of 64
// consecutive ids; a lane's place among equal classes comes from a 7-ballot match mask.
__global__ __launch_bounds__(RK_BLOCK) void k_rank_scatter(const uint32_t* __restrict__ deg, uint32_t V, uint32_t tiles,
                                                           const uint32_t* __restrict__ off, uint32_t* __restrict__ rank) {
  __shared__ uint32_t s_cnt[RK_WAVES][RK_NC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < RK_WAVES * RK_NC; i += RK_BLOCK) (&s_cnt[0][0])[i] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RK_TILE + (uint32_t)w * (RK_STEPS * WAVE);
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t cls[RK_STEPS], loc[RK_STEPS];
#pragma unroll
  for (int j = 0; j < RK_STEPS; ++j) {
    const uint32_t x = base + j * WAVE + lane;
    const uint32_t c = x < V ? deg_class(deg[x]) : 127u;
    uint64_t m = ~0ull;
#pragma unroll
    for (int bit = 0; bit < 7; ++bit) {
      const uint64_t bal = __ballot((c >> bit) & 1u);
      m &= ((c >> bit) & 1u) ? bal : ~bal;
    }
    cls[j] = c;
    uint32_t b0 = 0;
    if (c < RK_NC) b0 = s_cnt[w][c];
    loc[j] = b0 + (uint32_t)__popcll(m & lt);
    if (c < RK_NC && (m & lt) == 0) s_cnt[w][c] = b0 + (uint32_t)__popcll(m);   // the class's lowest lane
    wave_lds_sync();
  }
  __syncthreads();
  if (tid < RK_NC) {   // exclusive prefix over the waves, per class
    uint32_t run = 0;
    for (int k = 0; k < RK_WAVES; ++k) {
      const uint32_t t = s_cnt[k][tid];
      s_cnt[k][tid] = run;
      run += t;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RK_STEPS; ++j) {
    const uint32_t x = base + j * WAVE + lane;
    if (x < V) rank[x] = off[cls[j] * tiles + blockIdx.x] + s_cnt[w][cls[j]] + loc[j];
  }
}

// oriented composite keys (min rank << B | max rank); self-loops -> sentinel (sorts last) + bitmap
// and count
__global__ __launch_bounds__(256) void k_tri_okeys(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                   uint64_t n, uint64_t key_xor, uint32_t B,
                                                   const uint32_t* __restrict__ rank, uint64_t* __restrict__ out,
                                                   uint32_t* __restrict__ loop_bits, unsigned long long* __restrict__ loops) {
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t a = (uint64_t)src[i] ^ key_xor, b = (uint64_t)dst[i] ^ key_xor;
    uint64_t k = sent;
    if (a != b) {
      const uint64_t ra = rank[a], rb = rank[b];
      k = ra < rb ? (ra << B) | rb : (rb << B) | ra;
    } else {
      atomicOr(&loop_bits[a >> 5], 1u << (a & 31));
      atomicAdd(loops, 1ull);
    }
    out[i] = k;
  }
}

// the unique oriented edges (sorted keys u << B | v) -> out-lists: nbr[p] = v, out_range[u] =
// [first, last + 1) (ranges of absent vertices were zeroed); the transposed sort's keys: v
__global__ __launch_bounds__(256) void k_tri_out(const uint64_t* __restrict__ keys, uint32_t M, uint32_t B,
                                                 uint32_t* __restrict__ nbr, uint32_t* __restrict__ out_range,
                                                 uint64_t* __restrict__ tkey) {
  const uint64_t mask = (1ull << B) - 1;
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < M; p += gridDim.x * 256u) {
    const uint64_t k = keys[p];
    const uint32_t u = (uint32_t)(k >> B), v = (uint32_t)(k & mask);
    nbr[p] = v;
    tkey[p] = v;
    if (p == 0 || (uint32_t)(keys[p - 1] >> B) != u) out_range[2 * u] = p;
    if (p + 1 == M || (uint32_t)(keys[p + 1] >> B) != u) out_range[2 * u + 1] = p + 1;
  }
}

// the transposed sort's payload: for the edge u -> v at adjacency position p, the part of N+(u)
// past v, [p + 1, end of N+(u)) -- sorted by v it becomes the in-entries' suffix ranges
__global__ __launch_bounds__(256) void k_tri_sfx_pay(const uint64_t* __restrict__ keys, uint32_t M, uint32_t B,
                                                     const uint2* __restrict__ out_range, uint2* __restrict__ pay) {
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < M; p += gridDim.x * 256u)
    pay[p] = make_uint2(p + 1, out_range[(uint32_t)(keys[p] >> B)].y);
}

// the edges sorted by target: in_range[v] = [first, last + 1) of v's in-entries
__global__ __launch_bounds__(256) void k_tri_in(const uint32_t* __restrict__ skey, uint32_t M,
                                                uint32_t* __restrict__ in_range) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < M; i += gridDim.x * 256u) {
    const uint32_t v = skey[i];
    if (i == 0 || skey[i - 1] != v) in_range[2 * v] = i;
    if (i + 1 == M || skey[i + 1] != v) in_range[2 * v + 1] = i + 1;
  }
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
  const size_t V = 1ull << B;
  // 1. raw degrees (+ self-loop bitmap) -> degree-class ranks -> oriented composite keys of the ranks
  GS_TRY(ensure(c, c->aux, n * 8));
  const size_t words = (V + 31) / 32;
  GS_TRY(ensure(c, c->tri_loops, words * 4));
  GS_TRY(ensure(c, c->out_a, V * 4));
  GS_TRY(ensure(c, c->out_b, V * 4));
  const uint32_t rk_tiles = (uint32_t)((V + RK_TILE - 1) / RK_TILE);
  GS_TRY(ensure(c, c->tri_tiles, (size_t)rk_tiles * RK_NC * 4 + 8));
  GS_HIP(hipMemsetAsync(c->tri_loops.p, 0, words * 4, c->stream));
  GS_HIP(hipMemsetAsync(c->out_a.p, 0, V * 4, c->stream));
  unsigned long long* d_loops = (unsigned long long*)(sm + SM_NUNIQUE);
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 8192);
  uint32_t* deg = c->out_a.as<uint32_t>();
  uint32_t* rank = c->out_b.as<uint32_t>();
  uint32_t* rk_cnt = c->tri_tiles.as<uint32_t>();
  {
    GS_TRY(ensure(c, c->out_keys, std::min<uint64_t>(2 * n, V) * 8));
    GS_TRY(ensure(c, c->tri_sfx, std::min<uint64_t>(2 * n, V) * 8));
    uint64_t U = 0;
    const gs_status bs = bucket_reduce(c, src, dst, nullptr, n, DIR_ALL, OP_COUNT, GS_NONE, false, nullptr,
                                       c->out_keys.as<int64_t>(), c->tri_sfx.p, &U);
    if (bs == GS_OK) {
      if (U)
        hipLaunchKernelGGL(k_tri_deg_scatter, dim3((unsigned)std::min<uint64_t>((U + 255) / 256, 8192)), dim3(256), 0,
                           c->stream, c->out_keys.as<int64_t>(), c->tri_sfx.as<int64_t>(), U, key_xor, deg);
    } else if (bs == GS_EUNSUPPORTED) {
      hipLaunchKernelGGL(k_tri_deg, dim3((unsigned)std::min<uint64_t>((n + DG_BLOCK - 1) / DG_BLOCK, 1024)),
                         dim3(DG_BLOCK), 0, c->stream, src, dst, n, key_xor, deg);
    } else {
      return bs;
    }
  }
  hipLaunchKernelGGL(k_rank_count, dim3(rk_tiles), dim3(RK_BLOCK), 0, c->stream, deg, (uint32_t)V, rk_tiles, rk_cnt);
  hipLaunchKernelGGL(k_rank_scan, dim3(1), dim3(1024), 0, c->stream, rk_cnt, rk_tiles * RK_NC);
  hipLaunchKernelGGL(k_rank_scatter, dim3(rk_tiles), dim3(RK_BLOCK), 0, c->stream, deg, (uint32_t)V, rk_tiles, rk_cnt,
                     rank);
  GS_HIP(hipMemsetAsync(d_loops, 0, 8, c->stream));
  hipLaunchKernelGGL(k_tri_okeys, dim3(g), dim3(256), 0, c->stream, src, dst, n, key_xor, B, rank,
                     c->aux.as<uint64_t>(), c->tri_loops.as<uint32_t>(), d_loops);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 4, d_loops, 8, hipMemcpyDeviceToHost, c->stream));
  // ids of class 0 (no edge) = the offset of class 1 (the copy fills the low 4 bytes)
  c->host_small[5] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 5, rk_cnt + rk_tiles, 4, hipMemcpyDeviceToHost, c->stream));
  // 2. sort + unique -> the simple oriented graph, sorted by (u, v)
  Sorted s;
  GS_TRY(sort_buffer(c, c->aux.as<uint64_t>(), nullptr, n, &s, 2 * (int)B));
  hipEventRecord(c->ev[1], c->stream);
  const uint64_t loops = c->host_small[4];
  const uint64_t nv = V - (uint32_t)c->host_small[5];
  GS_TRY(ensure(c, c->out_keys, n * 8));
  uint64_t M = 0;
  UniqueOut uo{c->out_keys.as<uint64_t>(), nullptr};
  GS_TRY((s.wide ? launch_rbk<uint64_t, CountOp>(c, s, uo, &M) : launch_rbk<uint32_t, CountOp>(c, s, uo, &M)));
  hipEventRecord(c->ev[2], c->stream);
  if (loops) M -= 1;   // the self-loop sentinel sorts last
  if (M == 0) {        // only self-loops: no triangle; the self-pair term needs >= 2 neighbours
    uint64_t S = 0;
    if (part == 0) GS_TRY(triangle_selfpair_term(c, osrc, odst, n, c->tri_loops.as<uint32_t>(), key_xor, uniq, nuniq, &S));
    *count = S;
    return GS_OK;
  }
  // 3. out-lists, then in-lists (sorted by target) carrying each in-entry's suffix of N+(u)
  GS_TRY(ensure(c, c->tri_heavy, (V + M / TH_VCH + 64) * 8));   // (v, in-chunk) items
  GS_TRY(ensure(c, c->tri_range, V * 16));
  GS_TRY(ensure(c, c->tri_nbr, M * 4));
  GS_TRY(ensure(c, c->tri_sfx, M * 8));
  uint2* out_range = reinterpret_cast<uint2*>(c->tri_range.p);
  uint2* in_range = out_range + V;
  GS_HIP(hipMemsetAsync(c->tri_range.p, 0, V * 16, c->stream));
  const unsigned ge = (unsigned)std::min<uint64_t>((M + 255) / 256, 16384);
  uint32_t* nbr = c->tri_nbr.as<uint32_t>();
  // (the oriented keys in aux are consumed: aux takes the transposed sort's keys)
  hipLaunchKernelGGL(k_tri_out, dim3(ge), dim3(256), 0, c->stream, c->out_keys.as<uint64_t>(), (uint32_t)M, B, nbr,
                     reinterpret_cast<uint32_t*>(out_range), c->aux.as<uint64_t>());
  hipLaunchKernelGGL(k_tri_sfx_pay, dim3(ge), dim3(256), 0, c->stream, c->out_keys.as<uint64_t>(), (uint32_t)M, B,
                     out_range, c->tri_sfx.as<uint2>());
  GS_HIP(hipGetLastError());
  Sorted t;
  GS_TRY(sort_buffer(c, c->aux.as<uint64_t>(), c->tri_sfx.p, M, &t, (int)B, 8));
  if (t.wide || t.key_xor) return set_error(c, GS_EDEVICE, "window triangles: transposed keys wider than 32 bits");
  const uint2* sfx = (const uint2*)t.vals;   // the sort's payload buffer (valsA / valsB): read-only from here
  hipLaunchKernelGGL(k_tri_in, dim3(ge), dim3(256), 0, c->stream, (const uint32_t*)t.keys, (uint32_t)M,
                     reinterpret_cast<uint32_t*>(in_range));
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[4], c->stream);
  GS_TRY(ensure(c, c->tri_queue, (M / TH_DMAX + 64) * 8));   // further in-list chunks: <= M / TH_DMAX
  // 4. intersections: vertex-centric LDS hash sets (k_tri_light), long out-lists in k_tri_heavy
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
  // this part's middle vertices: those whose out-list starts in [q0, q1) of the adjacency
  const uint64_t q0 = M * part / nparts, q1 = M * (part + 1) / nparts;
  uint32_t* d_nqueue = d_nheavy + 1;
  GS_HIP(hipMemsetAsync(d_nqueue, 0, 4, c->stream));
  const unsigned nvb = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((V + TH_WPB - 1) / TH_WPB, 8192));
  uint2* queue = c->tri_queue.as<uint2>();
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(k_tri_light, dim3(pass == 0 ? nvb : 4096u), dim3(TH_BLOCK), 0, c->stream, nbr, sfx, out_range,
                       in_range, (uint32_t)V, (uint32_t)q0, (uint32_t)q1, pass, queue, d_nqueue,
                       c->tri_heavy.as<uint2>(), d_nheavy, d_total, d_probes, nb_cap, d_err);
    GS_HIP(hipGetLastError());
  }
  hipEventRecord(c->ev[5], c->stream);
  // heavy items: work per item, exclusive scan, then equal-work runs per block
  c->host_small[6] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 6, d_nheavy, 4, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint32_t nh = (uint32_t)c->host_small[6];
  if (nh) {
    GS_TRY(ensure(c, c->tri_hwork, (size_t)nh * 16 + 8));
    unsigned long long* hw = c->tri_hwork.as<unsigned long long>();
    hipLaunchKernelGGL(k_tri_hwork, dim3((unsigned)std::min<uint64_t>((nh + 3) / 4, 16384)), dim3(256), 0, c->stream,
                       sfx, in_range, c->tri_heavy.as<uint2>(), nh, hw);
    GS_HIP(hipGetLastError());
    GS_TRY(xscan(c, (const uint64_t*)hw, nh, (uint64_t*)hw + nh));
    hipLaunchKernelGGL(k_tri_heavy, dim3(GS_TH_HGRID), dim3(TH_HBLOCK), 0, c->stream, nbr, sfx, out_range, in_range,
                       c->tri_heavy.as<uint2>(), d_nheavy, (const unsigned long long*)hw + nh, d_total, d_probes,
                       nb_cap, d_err);
    GS_HIP(hipGetLastError());
  }
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
    t.records = M;     // unique undirected edges
    t.vertices = nv;   // vertices with edges
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
