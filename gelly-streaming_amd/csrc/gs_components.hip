// gs_components.hip — ConnectedComponents over a window stream:
//   library/ConnectedComponents.java:56-131 on WindowGraphAggregation.java:47-65 (GraphAggregation's
//   Merger, transientState = false): every window's edges are folded into a DisjointSet (UpdateCC ->
//   DisjointSet.union, example/util/DisjointSet.java:97-123) and merged into the running state
//   (CombineCC -> DisjointSet.merge :132-136).  The state after a window is the partition of every
//   vertex seen so far into weakly connected components.
//
// gs_window_components computes that state on the GPU from the window's edges and the previous state
// (vertex, label) rows, which join the window as edges vertex -- label:
//   1. ids: when they span <= 2^28 values, the ids minus a common base index a parent array directly
//      (present vertices found after the union-find and compacted by a scan); else compact IDs from
//      relabel_endpoints (sort of the 2(n + m) endpoints, order-preserving)
//   2. union-find with the larger root always linked under the smaller one (atomicCAS on the root,
//      find with pointer halving; parents only ever decrease, so stale reads only cost retries)
//   3. full compression: every vertex's root = the smallest compact ID of its component = the
//      smallest vertex (the IDs are order-preserving), the canonical label of the partition
// Which vertex the reference's DisjointSet keeps as a root depends on HashMap iteration order; the
// partition (what ConnectedComponentsTest and DisjointSet.toString observe) does not.
#include "gs_ops.hpp"

namespace gs {

__device__ __forceinline__ uint32_t cc_find(uint32_t* parent, uint32_t x) {
  uint32_t y = parent[x];
  if (y != x) {
    uint32_t z;
    while (y > (z = parent[y])) {   // pointer halving: x skips to its grandparent
      parent[x] = z;
      x = y;
      y = z;
    }
  }
  return y;
}

__global__ __launch_bounds__(256) void k_cc_init(uint32_t* __restrict__ parent, uint32_t n) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) parent[i] = i;
}

// one union per edge (compact endpoints at[2e], at[2e + 1])
__global__ __launch_bounds__(256) void k_cc_hook(const uint32_t* __restrict__ at, uint64_t ne, uint32_t* parent) {
  for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * 256) {
    uint32_t a = cc_find(parent, at[2 * e]), b = cc_find(parent, at[2 * e + 1]);
    while (a != b) {
      const uint32_t hi = a > b ? a : b, lo = a > b ? b : a;
      const uint32_t old = atomicCAS(&parent[hi], hi, lo);
      if (old == hi) break;      // hi was a root: linked under lo
      // hi got a parent meanwhile (always smaller): continue from its current root
      a = cc_find(parent, old);
      b = lo;
    }
  }
}

// the two-phase unions of k_cc_hook_ids_phase over compact endpoint pairs (the relabel path)
__global__ __launch_bounds__(256) void k_cc_hook_phase(const uint32_t* __restrict__ at, uint64_t ne, uint32_t* parent,
                                                       uint32_t mask, int phase, const uint32_t* __restrict__ gbits) {
  for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * 256) {
    if (((e & mask) == 0) != (phase == 0)) continue;
    const uint32_t x = at[2 * e], y = at[2 * e + 1];
    if (phase == 1) {
      if (gbits && ((gbits[x >> 5] >> (x & 31)) & (gbits[y >> 5] >> (y & 31)) & 1u)) continue;
      if (parent[x] == parent[y]) continue;
    }
    uint32_t a = cc_find(parent, x), b = cc_find(parent, y);
    while (a != b) {
      const uint32_t hi = a > b ? a : b, lo = a > b ? b : a;
      const uint32_t old = atomicCAS(&parent[hi], hi, lo);
      if (old == hi) break;
      a = cc_find(parent, old);
      b = lo;
    }
  }
}
// full compression (every compact id is present: no marks)
__global__ __launch_bounds__(256) void k_cc_compress_all(uint32_t* parent, uint32_t U) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < U; i += gridDim.x * 256u) {
    uint32_t r = parent[i];
    if (r == i) continue;
    while (parent[r] != r) r = parent[r];
    parent[i] = r;
  }
}

// roots (= smallest compact ID of the component) -> labels in original IDs
__global__ __launch_bounds__(256) void k_cc_emit(uint32_t* parent, const int64_t* __restrict__ uniq, uint32_t n,
                                                 int64_t* __restrict__ keys, int64_t* __restrict__ labels) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    uint32_t r = i;
    while (parent[r] != r) r = parent[r];
    keys[i] = uniq[i];
    labels[i] = uniq[r];
  }
}

__global__ __launch_bounds__(256) void k_cc_concat(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                   uint64_t n, int64_t* __restrict__ oa, int64_t* __restrict__ ob) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    oa[i] = a[i];
    ob[i] = b[i];
  }
}

// ---- direct ids (the window's ids span <= CC_DIRECT_BITS bits: no relabel) ---------------------------
constexpr uint32_t CC_DIRECT_BITS = 28;

// OR of (id ^ k0) over both columns, k0 = *k0p (the first id of the call)
__global__ __launch_bounds__(256) void k_cc_mask(const int64_t* __restrict__ a, const int64_t* __restrict__ b, uint64_t n,
                                                 const int64_t* __restrict__ k0p, unsigned long long* __restrict__ mask) {
  const uint64_t k0 = (uint64_t)*k0p;
  uint64_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    m |= ((uint64_t)a[i] ^ k0) | ((uint64_t)b[i] ^ k0);
  m = wave_or(m);
  if ((threadIdx.x & 63) == 0 && m) atomicOr(mask, (unsigned long long)m);
}

// unions over (a[e] ^ key_xor, b[e] ^ key_xor); a self-loop marks its vertex present (it has no link)
__global__ __launch_bounds__(256) void k_cc_hook_ids(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                     uint64_t n, uint64_t key_xor, uint32_t* parent,
                                                     uint8_t* __restrict__ mark) {
  for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (uint64_t)gridDim.x * 256) {
    const uint32_t x = (uint32_t)((uint64_t)a[e] ^ key_xor), y = (uint32_t)((uint64_t)b[e] ^ key_xor);
    if (x == y) {
      mark[x] = 1;
      continue;
    }
    uint32_t p = cc_find(parent, x), q = cc_find(parent, y);
    while (p != q) {
      const uint32_t hi = p > q ? p : q, lo = p > q ? q : p;
      const uint32_t old = atomicCAS(&parent[hi], hi, lo);
      if (old == hi) break;
      p = cc_find(parent, old);
      q = lo;
    }
  }
}

// (round 6) the same unions in two phases: the window's every (mask + 1)-th edge first (phase 0), then -- after a
// full compression, so every vertex those edges linked points at its tree's root -- the rest (phase 1), which
// skips an edge whose endpoints already share that root (on a skewed graph the sampled edges leave one giant
// tree, so most of the rest end after two parent reads: no find chains, no CAS, no pointer-halving writes)
__global__ __launch_bounds__(256) void k_cc_hook_ids_phase(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                           uint64_t n, uint64_t key_xor, uint32_t* parent,
                                                           uint8_t* __restrict__ mark, uint32_t mask, int phase,
                                                           const uint32_t* __restrict__ gbits) {
  for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (uint64_t)gridDim.x * 256) {
    if (((e & mask) == 0) != (phase == 0)) continue;
    const uint32_t x = (uint32_t)((uint64_t)a[e] ^ key_xor), y = (uint32_t)((uint64_t)b[e] ^ key_xor);
    if (x == y) {
      mark[x] = 1;
      continue;
    }
    if (phase == 1) {
      // both in the giant tree (an L2-resident bit per vertex), or one tree already (parents only move to
      // smaller ids): nothing to join
      if (gbits && ((gbits[x >> 5] >> (x & 31)) & (gbits[y >> 5] >> (y & 31)) & 1u)) continue;
      if (parent[x] == parent[y]) continue;
    }
    uint32_t p = cc_find(parent, x), q = cc_find(parent, y);
    while (p != q) {
      const uint32_t hi = p > q ? p : q, lo = p > q ? q : p;
      const uint32_t old = atomicCAS(&parent[hi], hi, lo);
      if (old == hi) break;
      p = cc_find(parent, old);
      q = lo;
    }
  }
}

// the giant tree after phase 0: the most frequent root among the parents of 1024 sampled edges' sources
// (one block; any root would be correct -- the bits only let edges skip that are joined already)
// (compact ids: at != nullptr, the sources at[2e] instead of a[e] ^ key_xor)
__global__ __launch_bounds__(1024) void k_cc_giant(const int64_t* __restrict__ a, const uint32_t* __restrict__ at,
                                                   uint64_t n, uint64_t key_xor, const uint32_t* __restrict__ parent,
                                                   uint32_t* __restrict__ giant) {
  __shared__ uint32_t s_r[1024];
  __shared__ unsigned long long s_best;
  const uint32_t t = threadIdx.x;
  const uint64_t e = (uint64_t)t * (n / 1024);
  s_r[t] = parent[at ? at[2 * e] : (uint32_t)((uint64_t)a[e] ^ key_xor)];
  if (t == 0) s_best = 0;
  __syncthreads();
  const uint32_t mine = s_r[t];
  uint32_t c = 0;
  for (int i = 0; i < 1024; ++i) c += s_r[i] == mine ? 1u : 0u;
  atomicMax(&s_best, ((unsigned long long)c << 32) | mine);
  __syncthreads();
  if (t == 0) *giant = (uint32_t)s_best;
}
// bit v of gbits: parent[v] is the giant root (after the compression, parent[v] is v's root)
__global__ __launch_bounds__(256) void k_cc_gbits(const uint32_t* __restrict__ parent, uint32_t V,
                                                  const uint32_t* __restrict__ giant, uint32_t* __restrict__ gbits) {
  const uint32_t g = *giant;
  for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < (V + 31) / 32; w += gridDim.x * 256u) {
    uint32_t bits = 0;
    for (uint32_t k = 0; k < 32 && w * 32 + k < V; ++k) bits |= (parent[w * 32 + k] == g ? 1u : 0u) << k;
    gbits[w] = bits;
  }
}

// full compression; a linked vertex is present and so is its root (every root of a linked tree is an
// endpoint: links only ever join the roots of trees that hold endpoints)
__global__ __launch_bounds__(256) void k_cc_compress(uint32_t* parent, uint32_t V, uint8_t* __restrict__ mark) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < V; i += gridDim.x * 256u) {
    uint32_t r = parent[i];
    if (r == i) continue;
    while (parent[r] != r) r = parent[r];
    parent[i] = r;
    mark[i] = 1;
    mark[r] = 1;
  }
}

__global__ __launch_bounds__(256) void k_cc_flags(const uint8_t* __restrict__ mark, uint32_t V, uint64_t* __restrict__ f) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < V; i += gridDim.x * 256u) f[i] = mark[i];
}

__global__ __launch_bounds__(256) void k_cc_emit_ids(const uint32_t* __restrict__ parent, const uint8_t* __restrict__ mark,
                                                     const uint64_t* __restrict__ pos, uint32_t V, uint64_t key_xor,
                                                     int64_t* __restrict__ keys, int64_t* __restrict__ labels) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < V; i += gridDim.x * 256u) {
    if (!mark[i]) continue;
    const uint64_t at = pos[i];
    keys[at] = (int64_t)(key_xor ^ i);
    labels[at] = (int64_t)(key_xor ^ parent[i]);
  }
}

}  // namespace gs

using namespace gs;

extern "C" {

gs_status gs_window_components(gs_ctx* c, const gs_edge_batch* b, const gs_partial_batch* prev, gs_vertex_out* out) {
  if (!c) return GS_EINVAL;
  GS_TRY(check_batch(c, b, GS_DIR_OUT));
  if (prev && prev->n && (!prev->keys || !prev->vals)) return set_error(c, GS_EINVAL, "bad previous state");
  if (prev && prev->n && prev->val_dtype != GS_I64) return set_error(c, GS_EINVAL, "state labels must be I64");
  if (!out || !out->n_out || (out->capacity && (!out->keys || !out->vals))) return set_error(c, GS_EINVAL, "bad gs_vertex_out");
  GS_TRY(begin_call(c));
  hipEventRecord(c->ev[0], c->stream);
  const uint64_t n = b->n, m = prev ? prev->n : 0, N = n + m;
  *out->n_out = 0;
  if (N == 0) return GS_OK;
  // 1. the state's (vertex, label) rows on the device (cc[0] / cc[1] rows [0, m)); the window's columns are read
  //    where they are (round 6: no copy of them into one edge list -- 16 B read + 16 B written per edge --
  //    unless the ids take the relabel path, which appends them at rows [m, N))
  GS_TRY(ensure(c, c->cc[0], N * 8));
  GS_TRY(ensure(c, c->cc[1], N * 8));
  int64_t* A = c->cc[0].as<int64_t>();
  int64_t* Bc = c->cc[1].as<int64_t>();
  const int64_t *src = nullptr, *dst = nullptr;
  if (n) {
    const void* val;
    GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  }
  if (m) {
    const hipMemcpyKind k = prev->mem == GS_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    GS_HIP(hipMemcpyAsync(A, prev->keys, m * 8, k, c->stream));
    GS_HIP(hipMemcpyAsync(Bc, prev->vals, m * 8, k, c->stream));
  }
  GS_HIP(hipGetLastError());
  // the two segments of pairs: the window's edges, the state's rows
  struct Seg {
    const int64_t *a, *b;
    uint64_t n;
  };
  const Seg seg[2] = {{src, dst, n}, {A, Bc, m}};
  const int64_t* k0p = n ? src : A;
  // 2a. ids spanning <= CC_DIRECT_BITS bits: union-find over the ids themselves (no relabel sort)
  {
    char* sm = c->small.as<char>();
    unsigned long long* dmask = (unsigned long long*)(sm + SM_TABLE);
    GS_HIP(hipMemsetAsync(dmask, 0, 8, c->stream));
    auto grid = [](uint64_t x) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((x + 255) / 256, 8192)); };
    for (const Seg& g : seg)
      if (g.n) hipLaunchKernelGGL(k_cc_mask, dim3(grid(g.n)), dim3(256), 0, c->stream, g.a, g.b, g.n, k0p, dmask);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(c->host_small + 12, dmask, 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(c->host_small + 13, k0p, 8, hipMemcpyDeviceToHost, c->stream));
    GS_TRY(host_wait(c));
    const uint64_t mask = c->host_small[12], k0 = c->host_small[13];
    const uint32_t B = mask ? 64 - __builtin_clzll(mask) : 1;
    if (B <= CC_DIRECT_BITS) {
      const uint64_t key_xor = k0 & ~((1ull << B) - 1);
      const uint32_t V = 1u << B;
      GS_TRY(ensure(c, c->cc[2], (size_t)V * 4));
      GS_TRY(ensure(c, c->out_b, (size_t)V));
      GS_TRY(ensure(c, c->rl[2], (size_t)V * 8 + 8));
      GS_TRY(ensure(c, c->rl[3], (size_t)V * 8 + 8));
      uint32_t* parent = c->cc[2].as<uint32_t>();
      uint8_t* mark = c->out_b.as<uint8_t>();
      const unsigned gv = (unsigned)std::min<uint64_t>((V + 255) / 256, 16384);
      hipLaunchKernelGGL(k_cc_init, dim3(gv), dim3(256), 0, c->stream, parent, V);
      GS_HIP(hipMemsetAsync(mark, 0, V, c->stream));
      hipEventRecord(c->ev[1], c->stream);
      // GS_CC_SAMPLE = k (a power of two): the two-phase unions over every k-th edge first (0 or 1: one pass
      // over every edge)
      static const int sample_env = getenv("GS_CC_SAMPLE") ? atoi(getenv("GS_CC_SAMPLE")) : 16;   // (8: +0.2-0.4 ms, 32: +0.2, 64: +0.6)
      if (sample_env > 1 && (sample_env & (sample_env - 1)) == 0 && N >= 65536) {
        for (const Seg& g : seg)
          if (g.n)
            hipLaunchKernelGGL(k_cc_hook_ids_phase, dim3(grid(g.n)), dim3(256), 0, c->stream, g.a, g.b, g.n, key_xor, parent,
                               mark, (uint32_t)sample_env - 1, 0, (const uint32_t*)nullptr);
        hipLaunchKernelGGL(k_cc_compress, dim3(gv), dim3(256), 0, c->stream, parent, V, mark);
        // the giant tree's vertices as a bit table (V / 8 bytes: L2-resident) for phase 1's skip test (the
        // larger segment's sources are sampled)
        static const int giant_env = getenv("GS_CC_GIANT") ? atoi(getenv("GS_CC_GIANT")) : 1;   // A/B
        uint32_t* gbits = nullptr;
        const Seg& big = n >= m ? seg[0] : seg[1];
        if (giant_env && big.n >= 1024) {
          GS_TRY(ensure(c, c->cc[3], (size_t)(V + 31) / 32 * 4 + 64));
          gbits = c->cc[3].as<uint32_t>();
          uint32_t* giant = gbits + (V + 31) / 32;
          hipLaunchKernelGGL(k_cc_giant, dim3(1), dim3(1024), 0, c->stream, big.a, (const uint32_t*)nullptr, big.n, key_xor,
                             parent, giant);
          hipLaunchKernelGGL(k_cc_gbits, dim3((unsigned)std::min<uint64_t>(((V + 31) / 32 + 255) / 256, 16384)), dim3(256),
                             0, c->stream, parent, V, giant, gbits);
        }
        for (const Seg& g : seg)
          if (g.n)
            hipLaunchKernelGGL(k_cc_hook_ids_phase, dim3(grid(g.n)), dim3(256), 0, c->stream, g.a, g.b, g.n, key_xor, parent,
                               mark, (uint32_t)sample_env - 1, 1, (const uint32_t*)gbits);
      } else {
        for (const Seg& g : seg)
          if (g.n)
            hipLaunchKernelGGL(k_cc_hook_ids, dim3(grid(g.n)), dim3(256), 0, c->stream, g.a, g.b, g.n, key_xor, parent, mark);
      }
      hipLaunchKernelGGL(k_cc_compress, dim3(gv), dim3(256), 0, c->stream, parent, V, mark);
      GS_HIP(hipGetLastError());
      hipEventRecord(c->ev[2], c->stream);
      uint64_t* flags = c->rl[2].as<uint64_t>();
      uint64_t* pos = c->rl[3].as<uint64_t>();
      hipLaunchKernelGGL(k_cc_flags, dim3(gv), dim3(256), 0, c->stream, mark, V, flags);
      GS_TRY(xscan(c, flags, V, pos));
      GS_HIP(hipMemcpyAsync(c->host_small + 12, pos + V, 8, hipMemcpyDeviceToHost, c->stream));
      GS_TRY(host_wait(c));
      const uint64_t U = c->host_small[12];
      *out->n_out = U;
      c->last_U = U;
      if (U > out->capacity) return set_error(c, GS_ECAPACITY, "components need %llu vertices", (unsigned long long)U);
      const bool direct = out->mem == GS_MEM_DEVICE;
      int64_t* kd = out->keys;
      int64_t* vd = (int64_t*)out->vals;
      if (!direct) {
        GS_TRY(ensure(c, c->out_keys, U * 8 + 8));
        GS_TRY(ensure(c, c->out_a, U * 8 + 8));
        kd = c->out_keys.as<int64_t>();
        vd = c->out_a.as<int64_t>();
      }
      hipLaunchKernelGGL(k_cc_emit_ids, dim3(gv), dim3(256), 0, c->stream, parent, mark, pos, V, key_xor, kd, vd);
      GS_HIP(hipGetLastError());
      hipEventRecord(c->ev[3], c->stream);
      if (!direct) {
        GS_TRY(deliver(c, out->keys, kd, U * 8, out->mem));
        GS_TRY(deliver(c, out->vals, vd, U * 8, out->mem));
      }
      GS_TRY(host_wait(c));
      gs_stage_times& t = c->times;
      t = gs_stage_times{};
      t.pass_ms[0] = event_ms(c->ev[0], c->ev[1]);   // staging + id range + init
      t.pass_ms[1] = event_ms(c->ev[1], c->ev[2]);   // union-find + compression
      t.pass_ms[2] = event_ms(c->ev[2], c->ev[3]);   // present vertices -> labels
      t.total_ms = event_ms(c->ev[0], c->ev[3]);
      t.records = N;
      t.vertices = U;
      t.key_bits = B;
      t.path = 4;
      return GS_OK;
    }
  }
  // 2b. compact IDs: the window's edges appended to the state's rows (one edge list for the relabel sort)
  if (n)
    hipLaunchKernelGGL(k_cc_concat, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 8192)), dim3(256), 0, c->stream,
                       src, dst, n, A + m, Bc + m);
  const int64_t *ca, *cb, *uniq;
  uint64_t U = 0;
  GS_TRY(relabel_endpoints(c, A, Bc, N, &ca, &cb, &uniq, &U));
  hipEventRecord(c->ev[1], c->stream);
  // 3. union-find over the compact endpoint pairs (rl[4]: at[2e], at[2e + 1])
  GS_TRY(ensure(c, c->cc[2], U * 4 + 4));
  uint32_t* parent = c->cc[2].as<uint32_t>();
  const unsigned gu = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((U + 255) / 256, 16384));
  const unsigned ge = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((N + 255) / 256, 16384));
  hipLaunchKernelGGL(k_cc_init, dim3(gu), dim3(256), 0, c->stream, parent, (uint32_t)U);
  {
    // the two-phase unions and the giant tree's bits, as the direct path (GS_CC_SAMPLE, GS_CC_GIANT)
    static const int sample_env = getenv("GS_CC_SAMPLE") ? atoi(getenv("GS_CC_SAMPLE")) : 16;
    static const int giant_env = getenv("GS_CC_GIANT") ? atoi(getenv("GS_CC_GIANT")) : 1;
    const uint32_t* at = c->rl[4].as<uint32_t>();
    if (sample_env > 1 && (sample_env & (sample_env - 1)) == 0 && N >= 65536) {
      hipLaunchKernelGGL(k_cc_hook_phase, dim3(ge), dim3(256), 0, c->stream, at, N, parent, (uint32_t)sample_env - 1, 0,
                         (const uint32_t*)nullptr);
      hipLaunchKernelGGL(k_cc_compress_all, dim3(gu), dim3(256), 0, c->stream, parent, (uint32_t)U);
      uint32_t* gbits = nullptr;
      if (giant_env) {
        GS_TRY(ensure(c, c->cc[3], (size_t)(U + 31) / 32 * 4 + 64));
        gbits = c->cc[3].as<uint32_t>();
        uint32_t* giant = gbits + (U + 31) / 32;
        hipLaunchKernelGGL(k_cc_giant, dim3(1), dim3(1024), 0, c->stream, (const int64_t*)nullptr, at, N, 0ull, parent, giant);
        hipLaunchKernelGGL(k_cc_gbits, dim3((unsigned)std::min<uint64_t>(((U + 31) / 32 + 255) / 256, 16384)), dim3(256), 0,
                           c->stream, parent, (uint32_t)U, giant, gbits);
      }
      hipLaunchKernelGGL(k_cc_hook_phase, dim3(ge), dim3(256), 0, c->stream, at, N, parent, (uint32_t)sample_env - 1, 1,
                         (const uint32_t*)gbits);
    } else {
      hipLaunchKernelGGL(k_cc_hook, dim3(ge), dim3(256), 0, c->stream, at, N, parent);
    }
  }
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[2], c->stream);
  // 4. labels
  *out->n_out = U;
  c->last_U = U;
  if (U > out->capacity) return set_error(c, GS_ECAPACITY, "components need %llu vertices", (unsigned long long)U);
  const bool direct = out->mem == GS_MEM_DEVICE;
  int64_t* kd = out->keys;
  int64_t* vd = (int64_t*)out->vals;
  if (!direct) {
    GS_TRY(ensure(c, c->out_keys, U * 8));
    GS_TRY(ensure(c, c->out_a, U * 8));
    kd = c->out_keys.as<int64_t>();
    vd = c->out_a.as<int64_t>();
  }
  hipLaunchKernelGGL(k_cc_emit, dim3(gu), dim3(256), 0, c->stream, parent, uniq, (uint32_t)U, kd, vd);
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[3], c->stream);
  if (!direct) {
    GS_TRY(deliver(c, out->keys, kd, U * 8, out->mem));
    GS_TRY(deliver(c, out->vals, vd, U * 8, out->mem));
  }
  GS_TRY(host_wait(c));
  gs_stage_times& t = c->times;
  t = gs_stage_times{};
  t.pass_ms[0] = event_ms(c->ev[0], c->ev[1]);   // staging + compact IDs
  t.pass_ms[1] = event_ms(c->ev[1], c->ev[2]);   // union-find
  t.pass_ms[2] = event_ms(c->ev[2], c->ev[3]);   // labels
  t.total_ms = event_ms(c->ev[0], c->ev[3]);
  t.records = N;
  t.vertices = U;
  t.path = 4;
  return GS_OK;
}

}  // extern "C"
