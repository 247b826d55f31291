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
// A vertex whose insertion sequence ever fills a bin to 9 nodes leaves that model (treeifyBin: a
// resize below capacity 64, a red-black tree bin above); those vertices are found exactly and re-run
// through a per-vertex JDK HashMap simulation (gs_pair_out.reserved reports which case occurred).
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
// dense rank table of the window's vertices when every id differs from the first sorted id only in its low
// bits (<= HS_RANK_BITS of them: the sort's key mask): rank[x ^ vkeys[0]] = u, so k_hs_prep ranks a
// neighbour with one read instead of a binary search
constexpr int HS_RANK_BITS = 28;
__global__ __launch_bounds__(256) void k_hs_rank(const int64_t* __restrict__ vkeys, uint32_t U, uint32_t* __restrict__ rank) {
  const uint64_t k0 = (uint64_t)vkeys[0];
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < U; u += gridDim.x * 256u) rank[(uint64_t)vkeys[u] ^ k0] = u;
}

__global__ __launch_bounds__(256) void k_hs_prep(const uint32_t* __restrict__ rec, uint32_t R,
                                                 const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                 const uint64_t* __restrict__ off, const int64_t* __restrict__ vkeys,
                                                 uint32_t U, uint32_t B, const uint32_t* __restrict__ rank,
                                                 int64_t* __restrict__ nbr,
                                                 uint32_t* __restrict__ useg, uint64_t* __restrict__ comp,
                                                 uint32_t* __restrict__ pidx) {
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < R; p += gridDim.x * 256u) {
    const uint32_t r = rec[p];
    const uint32_t i = r >> 1;
    const int64_t x = (r & 1u) ? src[i] : dst[i];   // ALL: r = 2i -> (src, dst), 2i+1 -> (dst, src)
    const uint32_t u = seg_of(off, U, p);
    uint32_t lo = 0, hi = U - 1;                      // rank of x among the window's vertices
    if (rank) {
      lo = rank[(uint64_t)x ^ (uint64_t)vkeys[0]];
    } else {
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (vkeys[mid] < x) lo = mid + 1;
        else hi = mid;
      }
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

// ids in plain-bin HashSet order (original IDs)
__global__ __launch_bounds__(256) void k_hs_ids(const uint32_t* __restrict__ ord, const uint64_t* __restrict__ dkey,
                                                uint32_t M, uint32_t B, const int64_t* __restrict__ vkeys,
                                                int64_t* __restrict__ ids) {
  const uint64_t mask = (B >= 64) ? ~0ull : ((1ull << B) - 1);
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) ids[q] = vkeys[dkey[ord[q]] & mask];
}

// gt[q] = ids[q] > v(u)   (signed Long order, WindowTriangles.java:108)
__global__ __launch_bounds__(256) void k_hs_gt(const int64_t* __restrict__ ids, uint32_t M, const uint64_t* __restrict__ doff,
                                               uint32_t U, const int64_t* __restrict__ vkeys, uint64_t* __restrict__ g) {
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u) {
    const uint32_t u = seg_of(doff, U, q);
    g[q] = ids[q] > vkeys[u] ? 1ull : 0ull;
  }
}

// ---- emission by output position (whole windows and chunks alike) ------------------------------------
// Output order (gs_window_candidates): the emitting vertices ascending ("slots": every vertex, or with a
// split the vertices this part owns); per slot its d edge records (v, t, false) in arrival order
// (:96-100), then its pair rows.  With G = the slot's ids > v in HashSet order (k of them), row r emits
// (G[r], G[r]), (G[r], G[r+1]), .., (G[r], G[k-1]) (:104-114: j >= i, both > v) for r < rows, where
// rows = k - 1 when the set's last id is > v (i < len - 1 excludes it) and k otherwise.  So a slot's
// block is d + rows*k - rows*(rows-1)/2 records and any position inverts in closed form: no per-row
// state, no thread-per-row loop.
struct CandMeta {     // one per slot, 32 bytes
  uint64_t nbr_off;   // first edge record (HS_NBR)
  uint64_t gbase;     // first id > v (HS_GIDS)
  uint32_t d;         // edge records
  uint32_t k;         // distinct ids > v
  uint32_t rows;      // pair rows
  uint32_t u;         // vertex index (HS_VKEYS)
};
static_assert(sizeof(CandMeta) == 32, "CandMeta");

__device__ __forceinline__ uint64_t tri_rows_before(uint64_t r, uint64_t k) { return r * k - r * (r - 1) / 2; }

// G: the ids > v of every vertex, compacted in HashSet order (position gx[q])
__global__ __launch_bounds__(256) void k_cand_gids(const int64_t* __restrict__ ids, const uint64_t* __restrict__ g,
                                                   const uint64_t* __restrict__ gx, uint32_t M,
                                                   int64_t* __restrict__ gids) {
  for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < M; q += gridDim.x * 256u)
    if (g[q]) gids[gx[q]] = ids[q];
}
// split: own[u] = 1 iff gs_owner_of assigns vertex u to `part`
__global__ __launch_bounds__(256) void k_cand_own(const int64_t* __restrict__ vkeys, uint32_t U, uint32_t nparts,
                                                  uint32_t part, uint64_t* __restrict__ own) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < U; u += gridDim.x * 256u)
    own[u] = owner_of(vkeys[u], nparts) == part ? 1ull : 0ull;
}
// slot metadata and block sizes (slot_of: exclusive scan of own, or null = every vertex is a slot)
__global__ __launch_bounds__(256) void k_cand_meta(const uint64_t* __restrict__ off, const uint64_t* __restrict__ doff,
                                                   const uint64_t* __restrict__ g, const uint64_t* __restrict__ gx,
                                                   uint32_t U, const uint64_t* __restrict__ own,
                                                   const uint64_t* __restrict__ slot_of, CandMeta* __restrict__ meta,
                                                   uint64_t* __restrict__ size) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < U; u += gridDim.x * 256u) {
    if (own && !own[u]) continue;
    const uint32_t s = slot_of ? (uint32_t)slot_of[u] : u;
    const uint64_t q0 = doff[u], q1 = doff[u + 1], gb = gx[q0], k = gx[q1] - gb;
    const uint64_t rows = k ? k - g[q1 - 1] : 0;
    CandMeta m;
    m.nbr_off = off[u];
    m.gbase = gb;
    m.d = (uint32_t)(off[u + 1] - off[u]);
    m.k = (uint32_t)k;
    m.rows = (uint32_t)rows;
    m.u = u;
    meta[s] = m;
    size[s] = m.d + tri_rows_before(rows, k);
  }
}

// One 256-position step [base, min(w1, base + 256)) by the general path: lane l takes positions
// base + 64 i + l; each position's slot is resolved against 64 consecutive block starts held one per lane
// (binary search through lane shuffles; a step that spans more than 64 slots takes the next 64), starting
// at slot sc (the slot of base or an earlier one).  Returns the slot of the step's last position.
// OT: the id columns' type -- int64_t (the reference's Long), or uint32_t holding id - idb (gs_candidates_next_u32).
template <typename OT>
__device__ __forceinline__ uint32_t cand_slow_step(const uint64_t* __restrict__ vs, uint32_t S,
                                                   const CandMeta* __restrict__ meta, const int64_t* __restrict__ vkeys,
                                                   const int64_t* __restrict__ nbr, const int64_t* __restrict__ gids,
                                                   uint64_t P0, uint64_t base, uint64_t w1, uint32_t sc, uint32_t lane,
                                                   OT* __restrict__ a, OT* __restrict__ b, uint8_t* __restrict__ f,
                                                   int64_t idb) {
  uint64_t o[4];
  uint32_t slot[4];
  bool need[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = base + (uint64_t)(i * 64) + lane;
    need[i] = o[i] < w1;
    slot[i] = sc;
  }
  for (uint32_t s0 = sc;; s0 += 64) {
    const uint64_t bj = (uint64_t)s0 + 1 + lane <= S ? vs[s0 + 1 + lane] : ~0ull;
    const uint64_t top = __shfl(bj, 63, 64);
    bool pend = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int pos = 0;   // block starts vs[s0 + 1 ..] at or below o[i]: 0..63 by halving, 64 past the window
#pragma unroll
      for (int st = 32; st > 0; st >>= 1) {
        const uint64_t v = __shfl(bj, pos + st - 1, 64);
        pos += v <= o[i] ? st : 0;
      }
      if (top <= o[i]) pos = 64;
      if (need[i] && pos < 64) {
        slot[i] = s0 + pos;
        need[i] = false;
      }
      pend |= need[i];
    }
    if (!__any(pend)) break;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (o[i] >= w1) continue;
    const uint32_t sl = slot[i];
    const CandMeta m = meta[sl];
    const uint64_t t = o[i] - vs[sl];
    int64_t av, bv;
    uint8_t fv;
    if (t < m.d) {
      av = vkeys[m.u];
      bv = nbr[m.nbr_off + t];
      fv = 0;
    } else if (m.rows) {
      // row r of the block: the largest r with r k - r (r - 1) / 2 <= q (closed form, then at most a
      // step or two of correction for the double rounding; the loops are bounded regardless)
      const uint64_t q = t - m.d, k = m.k, rows = m.rows;
      const double k2 = 2.0 * (double)k + 1.0;
      uint64_t r = (uint64_t)fmax(0.0, (k2 - sqrt(fmax(0.0, k2 * k2 - 8.0 * (double)q))) * 0.5);
      if (r >= rows) r = rows - 1;
      for (int g = 0; g < 64 && r > 0 && tri_rows_before(r, k) > q; ++g) --r;
      for (int g = 0; g < 64 && r + 1 < rows && tri_rows_before(r + 1, k) <= q; ++g) ++r;
      const uint64_t col = min(q - tri_rows_before(r, k), k - 1 - r);
      av = gids[m.gbase + r];
      bv = gids[m.gbase + r + col];
      fv = 1;
    } else {   // not reached: a block without pair rows holds only its edge records
      av = bv = 0;
      fv = 1;
    }
    a[o[i] - P0] = (OT)(av - idb);
    b[o[i] - P0] = (OT)(bv - idb);
    f[o[i] - P0] = fv;
  }
  return __shfl(slot[3], 63, 64);   // the slot of this step's last position (the next step starts there)
}

// slot of position w: invariant vs[lo] <= w and (hi == S or vs[hi] > w) (a 64-ary search; vs[0] = 0)
__device__ __forceinline__ uint32_t cand_find_slot(const uint64_t* __restrict__ vs, uint32_t S, uint64_t w,
                                                   uint32_t lane) {
  uint32_t lo = 0, hi = S;
  while (hi - lo > 1) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint64_t idx = (uint64_t)lo + (uint64_t)lane * step;
    const bool t = idx < hi && vs[idx] <= w;
    const uint64_t m = __ballot(t);
    const uint32_t L = 63 - __clzll(m);
    const uint32_t nlo = lo + L * step;
    hi = min(hi, nlo + step);
    lo = nlo;
  }
  return lo;
}

// The records at output positions [P0, P1), written to a/b/f[o - P0].  Each wave owns per_wave
// consecutive positions (a multiple of 256) and walks them 256 at a time, lane l taking positions
// base + 64 i + l: every store of a wave is one contiguous run (512 B of a, 512 B of b, 64 B of f).
// A wave finds the slot of its first position by a 64-ary search of the block starts vs[0..S].
// MODE 0: every step, by the fast path where it applies and cand_slow_step otherwise.  MODE 1: the fast
// steps only (the pair rows of one slot: ~99% of a window's steps), compiled without the general path
// so the kernel holds fewer registers and more of its stores are in flight; every other step's base is
// appended to `steps` (count in steps_n) for k_cand_emit_rest.  Kernels: k_cand_emit_all (MODE 0),
// k_cand_emit_fast (MODE 1).
#ifndef GS_CAND_LANE4
#define GS_CAND_LANE4 1   // fast path: four consecutive positions per lane (A/B: 0 = positions strided by 64)
#endif
#ifndef GS_CAND_CARRY
#define GS_CAND_CARRY 1   // fast path: a step after a fast step in the same slot starts from its row state (A/B: 0)
#endif
template <int MODE, typename OT>
__device__ __forceinline__ void cand_emit_body(const uint64_t* __restrict__ vs, uint32_t S,
                                               const CandMeta* __restrict__ meta, const int64_t* __restrict__ vkeys,
                                               const int64_t* __restrict__ nbr, const int64_t* __restrict__ gids,
                                               uint64_t P0, uint64_t P1, uint64_t per_wave,
                                               OT* __restrict__ a, OT* __restrict__ b,
                                               uint8_t* __restrict__ f, int f4, uint64_t* __restrict__ steps,
                                               uint32_t* __restrict__ steps_n, int64_t idb) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6;
  const uint64_t w0 = P0 + wave * per_wave;
  if (w0 >= P1) return;   // wave-uniform
  const uint64_t w1 = min(P1, w0 + per_wave);
  uint32_t sc = cand_find_slot(vs, S, w0, lane);
  // the current slot's block start / end and metadata, reloaded only when the step moves to another slot
  // (a fast step then issues no load before its id gathers; re-reading them every step put two dependent
  // loads in front of each step's stores)
  uint32_t cs = 0xFFFFFFFFu;
  uint64_t c_beg = 0, c_end = 0;
  CandMeta cm{};
#if GS_CAND_LANE4 && GS_CAND_CARRY
  // the row state (row, its length, offset into it) of position k_next in slot k_slot: what the previous fast
  // step's last lane walked to, so a fast step that follows one in the same slot skips the closed-form row search
  uint32_t k_r = 0, k_len = 0, k_off = 0, k_slot = 0xFFFFFFFFu;
  uint64_t k_next = ~0ull;
#endif
  for (uint64_t base = w0; base < w1; base += 256) {
    // Fast path: the step lies inside one slot's pair rows (most records of a window: the blocks of its
    // high-degree vertices are O(k^2)).  The slot's metadata is wave-uniform (scalar loads), the row of
    // the step's first position is found once, and each lane walks forward from it (a 256-position span
    // crosses at most ~23 rows: only a block's last rows are shorter than 12).
    const uint64_t e1 = min(w1, base + 256);
    if (cs != sc) {
      cs = sc;
      c_beg = vs[sc];
      c_end = vs[sc + 1];
      cm = meta[sc];
    }
    if (c_end >= e1) {
      const CandMeta m = cm;
      const uint64_t t0 = base - c_beg;
      if (t0 >= m.d && m.rows) {
        const uint64_t k = m.k, rows = m.rows, q0 = t0 - m.d;
        const int64_t* G = gids + m.gbase;
        const uint32_t rows32 = (uint32_t)rows;
#if GS_CAND_LANE4
        uint32_t r, len, off;
#if GS_CAND_CARRY
        if (k_next == base && k_slot == sc) {
          r = k_r;
          len = k_len;
          off = k_off;
        } else
#endif
        {
          const double k2 = 2.0 * (double)k + 1.0;
          uint64_t r0 = (uint64_t)fmax(0.0, (k2 - sqrt(fmax(0.0, k2 * k2 - 8.0 * (double)q0))) * 0.5);
          if (r0 >= rows) r0 = rows - 1;
          for (int g = 0; g < 64 && r0 > 0 && tri_rows_before(r0, k) > q0; ++g) --r0;
          for (int g = 0; g < 64 && r0 + 1 < rows && tri_rows_before(r0 + 1, k) <= q0; ++g) ++r0;
          r = (uint32_t)r0;
          len = (uint32_t)(k - r0);
          off = (uint32_t)(q0 - tri_rows_before(r0, k));
        }
        // lane l takes the step's positions base + 4l .. 4l + 3: its four records are consecutive (mostly in one
        // row), and a wave's a / b stores are one contiguous 1 KiB (u32) or 2 KiB (int64) run of 16-byte stores.
        // The row walk runs in 32 bits relative to the step's first row (row r holds k - r entries; off = q -
        // rows_before(r) < k + 256): one add and compare per row crossed, no 64-bit row products per record.
        off += 4u * lane;
        const uint64_t o0 = base + 4ull * lane;
        OT av[4], bv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j) ++off;
          for (int g = 0; g < 64 && r + 1 < rows32 && off >= len; ++g) {
            off -= len;
            --len;
            ++r;
          }
          const uint32_t col = min(off, len - 1);
          av[j] = (OT)(G[r] - idb);
          bv[j] = (OT)(G[r + col] - idb);
        }
#if GS_CAND_CARRY
        k_r = __shfl(r, 63, 64);   // the last lane's position is base + 255: one on is the next step's first
        k_len = __shfl(len, 63, 64);
        k_off = __shfl(off, 63, 64) + 1u;
        k_next = base + 256;
        k_slot = sc;
#endif
        if ((f4 & 2) && o0 + 4 <= e1) {   // a and b 16-byte aligned; o0 - P0 is a multiple of 4
          if constexpr (sizeof(OT) == 4) {
            *reinterpret_cast<uint4*>(a + (o0 - P0)) = make_uint4(av[0], av[1], av[2], av[3]);
            *reinterpret_cast<uint4*>(b + (o0 - P0)) = make_uint4(bv[0], bv[1], bv[2], bv[3]);
          } else {
            longlong2* pa = reinterpret_cast<longlong2*>(a + (o0 - P0));
            longlong2* pb = reinterpret_cast<longlong2*>(b + (o0 - P0));
            pa[0] = make_longlong2(av[0], av[1]);
            pa[1] = make_longlong2(av[2], av[3]);
            pb[0] = make_longlong2(bv[0], bv[1]);
            pb[1] = make_longlong2(bv[2], bv[3]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (o0 + j < e1) {
              a[o0 + j - P0] = av[j];
              b[o0 + j - P0] = bv[j];
            }
          }
        }
        if (!(f4 & 1)) {
          for (int j = 0; j < 4; ++j)
            if (o0 + j < e1) f[o0 + j - P0] = 1;
        }
#else
        const double k2 = 2.0 * (double)k + 1.0;
        uint64_t r0 = (uint64_t)fmax(0.0, (k2 - sqrt(fmax(0.0, k2 * k2 - 8.0 * (double)q0))) * 0.5);
        if (r0 >= rows) r0 = rows - 1;
        for (int g = 0; g < 64 && r0 > 0 && tri_rows_before(r0, k) > q0; ++g) --r0;
        for (int g = 0; g < 64 && r0 + 1 < rows && tri_rows_before(r0 + 1, k) <= q0; ++g) ++r0;
        // a lane's positions increase with i, so its row walk carries over; it runs in 32 bits relative to
        // the step's first row (row r holds k - r entries; off = q - rows_before(r) < k + 256), one add and
        // compare per row crossed instead of two 64-bit row products per record
        uint32_t r = (uint32_t)r0, len = (uint32_t)(k - r0);
        uint32_t off = (uint32_t)(q0 - tri_rows_before(r0, k)) + lane;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (i) off += 64;
          const uint64_t oi = base + (uint64_t)(i * 64) + lane;
          if (oi >= e1) continue;
          for (int g = 0; g < 64 && r + 1 < rows32 && off >= len; ++g) {
            off -= len;
            --len;
            ++r;
          }
          const uint32_t col = min(off, len - 1);
          a[oi - P0] = (OT)(G[r] - idb);
          b[oi - P0] = (OT)(G[r + col] - idb);
          if (!(f4 & 1)) f[oi - P0] = 1;
        }
#endif
        if (f4 & 1) {   // every flag of a pair row is 1: one 4-byte store per lane (256 B per wave) instead of four 64-B byte-store runs
          uint8_t* fr = f + (base - P0);   // base - P0 is a multiple of 256
          const uint64_t fo = 4ull * lane;
          if (base + fo + 4 <= e1) {
            *reinterpret_cast<uint32_t*>(fr + fo) = 0x01010101u;
          } else {
            for (uint32_t j = 0; j < 4; ++j)
              if (base + fo + j < e1) fr[fo + j] = 1;
          }
        }
        continue;   // sc still holds the next step's first position, or an earlier slot
      }
    }
    if constexpr (MODE == 1) {
      // the step goes to k_cand_emit_rest; here only the slot of the next step's first position (e1),
      // searched forward from sc over 64 block starts at a time
      if (lane == 0) steps[atomicAdd(steps_n, 1u)] = base;
      for (;;) {
        const uint64_t bj = (uint64_t)sc + 1 + lane <= S ? vs[sc + 1 + lane] : ~0ull;
        const uint32_t c = (uint32_t)__popcll(__ballot(bj <= e1));   // block starts at or below e1
        sc += c;
        if (c < 64) break;
      }
    } else {
      sc = cand_slow_step<OT>(vs, S, meta, vkeys, nbr, gids, P0, base, w1, sc, lane, a, b, f, idb);
    }
  }
}

#define GS_CAND_EMIT_ARGS                                                                                        \
  const uint64_t *__restrict__ vs, uint32_t S, const CandMeta *__restrict__ meta, const int64_t *__restrict__ vkeys, \
      const int64_t *__restrict__ nbr, const int64_t *__restrict__ gids, uint64_t P0, uint64_t P1, uint64_t per_wave,  \
      OT *__restrict__ a, OT *__restrict__ b, uint8_t *__restrict__ f, int f4, uint64_t *__restrict__ steps,           \
      uint32_t *__restrict__ steps_n, int64_t idb
#define GS_CAND_EMIT_PASS vs, S, meta, vkeys, nbr, gids, P0, P1, per_wave, a, b, f, f4, steps, steps_n, idb
template <typename OT>
__global__ __launch_bounds__(256) void k_cand_emit_all(GS_CAND_EMIT_ARGS) { cand_emit_body<0, OT>(GS_CAND_EMIT_PASS); }
#ifndef GS_CAND_FAST_WAVES
#define GS_CAND_FAST_WAVES 0   // A/B: a waves-per-SIMD target for k_cand_emit_fast (0 = the compiler's choice)
#endif
#if GS_CAND_FAST_WAVES
#define GS_CAND_FAST_ATTR __attribute__((amdgpu_waves_per_eu(GS_CAND_FAST_WAVES)))
#else
#define GS_CAND_FAST_ATTR
#endif
template <typename OT>
__global__ __launch_bounds__(256) GS_CAND_FAST_ATTR void k_cand_emit_fast(GS_CAND_EMIT_ARGS) {
  cand_emit_body<1, OT>(GS_CAND_EMIT_PASS);
}

// the steps k_cand_emit_fast left (their bases in steps[0 .. *steps_n)), one wave per step at a time
template <typename OT>
__global__ __launch_bounds__(256) void k_cand_emit_rest(const uint64_t* __restrict__ vs, uint32_t S,
                                                        const CandMeta* __restrict__ meta,
                                                        const int64_t* __restrict__ vkeys, const int64_t* __restrict__ nbr,
                                                        const int64_t* __restrict__ gids, uint64_t P0, uint64_t P1,
                                                        OT* __restrict__ a, OT* __restrict__ b,
                                                        uint8_t* __restrict__ f, const uint64_t* __restrict__ steps,
                                                        const uint32_t* __restrict__ steps_n, int64_t idb) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n = *steps_n;
  const uint32_t nw = gridDim.x * 4u;
  for (uint32_t i = (blockIdx.x * 256u + threadIdx.x) >> 6; i < n; i += nw) {   // wave-uniform
    const uint64_t base = steps[i];
    const uint32_t sc = cand_find_slot(vs, S, base, lane);
    cand_slow_step<OT>(vs, S, meta, vkeys, nbr, gids, P0, base, min(P1, base + 256), sc, lane, a, b, f, idb);
  }
}

// the block of vertex `x` in the session's output: first position and length (0 records if absent)
__global__ void k_cand_find(const int64_t* __restrict__ vkeys, uint32_t U, const uint64_t* __restrict__ vs, int64_t x,
                            unsigned long long* __restrict__ out) {
  uint32_t lo = 0, hi = U;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (vkeys[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  const bool hit = lo < U && vkeys[lo] == x;
  out[0] = hit ? vs[lo] : (lo < U ? vs[lo] : vs[U]);
  out[1] = hit ? vs[lo + 1] - vs[lo] : 0ull;
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

// ---- vertices whose JDK HashMap leaves the plain-bin model ------------------------------------
// Until some bin reaches 9 nodes the JDK map is the plain model at every step: stage capacity C
// (16, 32, ..., final) holds the first min(k, 3C/4 + 1) distinct ids (the insert that crosses the
// threshold lands before the resize), buckets only gain entries inside a stage, and resize splits keep
// insertion order.  So a vertex is "complex" iff for some stage C a bucket of (hash & (C-1)) over its
// first n_C arrivals reaches 9 -- one counter per (vertex, stage, bucket), filled with atomics.
// Complex vertices are then simulated exactly (k_hs_jdk).
__global__ __launch_bounds__(256) void k_hs_first(const uint32_t* __restrict__ dfirst, uint32_t M,
                                                  uint64_t* __restrict__ F) {
  for (uint32_t m = blockIdx.x * 256u + threadIdx.x; m < M; m += gridDim.x * 256u) F[dfirst[m]] = 1;
}
// counter space of a vertex: stages 16..cap hold 16+32+..+cap = 2cap - 16 buckets (k >= 9 only)
__global__ __launch_bounds__(256) void k_hs_csize(const uint64_t* __restrict__ doff, uint32_t U,
                                                  uint64_t* __restrict__ csz) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < U; u += gridDim.x * 256u) {
    const uint64_t k = doff[u + 1] - doff[u];
    csz[u] = k >= 9 ? 2 * hs_capacity(k) - 16 : 0;
  }
}
// arrival rank i of each distinct entry (FX = exclusive scan of the first-arrival flags), the
// arrival-ordered ids (arr), and the per-stage bucket counters; a counter reaching 9 marks the vertex
__global__ __launch_bounds__(256) void k_hs_detect(const uint64_t* __restrict__ dkey, const uint32_t* __restrict__ dfirst,
                                                   uint32_t M, uint32_t B, const int64_t* __restrict__ vkeys,
                                                   const uint64_t* __restrict__ doff, const uint64_t* __restrict__ FX,
                                                   const uint64_t* __restrict__ cbase, uint32_t* __restrict__ cnt,
                                                   int64_t* __restrict__ arr, uint32_t* __restrict__ cplx) {
  const uint64_t mask = (B >= 64) ? ~0ull : ((1ull << B) - 1);
  for (uint32_t m = blockIdx.x * 256u + threadIdx.x; m < M; m += gridDim.x * 256u) {
    const uint64_t key = dkey[m];
    const uint32_t u = (uint32_t)(key >> B);
    const uint64_t d0 = doff[u], k = doff[u + 1] - d0;
    if (k < 9) continue;
    const int64_t x = vkeys[key & mask];
    const uint64_t i = FX[dfirst[m]] - d0;
    arr[d0 + i] = x;
    const uint32_t h0 = (uint32_t)((uint64_t)x ^ ((uint64_t)x >> 32)), h = h0 ^ (h0 >> 16);
    const uint64_t capf = hs_capacity(k), base = cbase[u];
    for (uint64_t C = 16; C <= capf; C <<= 1) {
      const uint64_t nC = C == capf ? k : (3 * C / 4 + 1);
      if (i >= nC) continue;
      if (atomicAdd(&cnt[base + C - 16 + (h & (uint32_t)(C - 1))], 1u) == 8u) cplx[u] = 1;
    }
  }
}
// compact list of complex vertices (+ table sizes for their exact maps)
__global__ __launch_bounds__(256) void k_hs_clist(const uint32_t* __restrict__ cplx, uint32_t U,
                                                  const uint64_t* __restrict__ doff, uint32_t* __restrict__ nc,
                                                  uint32_t* __restrict__ list, uint64_t* __restrict__ tsz) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < U; u += gridDim.x * 256u) {
    if (!cplx[u]) continue;
    const uint32_t s = atomicAdd(nc, 1u);
    list[s] = u;
    tsz[s] = max(hs_capacity(doff[u + 1] - doff[u]), (uint64_t)64);   // early resizes stop at 64
  }
}

// One exact java.util.HashMap<Long> per complex vertex (JDK 8+ putVal / resize / treeifyBin /
// TreeNode.treeify / putTreeVal / balanceInsertion / rotations / moveRootToFront / split / untreeify;
// the same restatement as the oracle's hashset_order).  Nodes are indexed 0..k-1 in arrival order;
// the table is resized in place (old bin j feeds new bins j and j + oldCap only).
struct JNode {
  uint32_t hash;
  int32_t next, prev, parent, left, right;
  uint8_t red, tree, pad[2];
};
struct JMap {
  JNode* n;
  const int64_t* key;
  int32_t* tab;
  uint32_t cap, thr, size, flags;
};
__device__ int j_dir(const JMap& m, int32_t p, uint32_t h, int64_t k) {
  if (m.n[p].hash > h) return -1;
  if (m.n[p].hash < h) return 1;
  return k < m.key[p] ? -1 : 1;   // Long.compareTo; keys are distinct
}
__device__ int32_t j_rotl(JNode* n, int32_t root, int32_t p) {
  int32_t r, pp, rl;
  if (p >= 0 && (r = n[p].right) >= 0) {
    if ((rl = n[p].right = n[r].left) >= 0) n[rl].parent = p;
    if ((pp = n[r].parent = n[p].parent) < 0) {
      root = r;
      n[r].red = 0;
    } else if (n[pp].left == p) {
      n[pp].left = r;
    } else {
      n[pp].right = r;
    }
    n[r].left = p;
    n[p].parent = r;
  }
  return root;
}
__device__ int32_t j_rotr(JNode* n, int32_t root, int32_t p) {
  int32_t l, pp, lr;
  if (p >= 0 && (l = n[p].left) >= 0) {
    if ((lr = n[p].left = n[l].right) >= 0) n[lr].parent = p;
    if ((pp = n[l].parent = n[p].parent) < 0) {
      root = l;
      n[l].red = 0;
    } else if (n[pp].right == p) {
      n[pp].right = l;
    } else {
      n[pp].left = l;
    }
    n[l].right = p;
    n[p].parent = l;
  }
  return root;
}
__device__ int32_t j_balance(JNode* n, int32_t root, int32_t x) {
  n[x].red = 1;
  for (;;) {
    int32_t xp = n[x].parent, xpp, xppl, xppr;
    if (xp < 0) {
      n[x].red = 0;
      return x;
    }
    if (!n[xp].red || (xpp = n[xp].parent) < 0) return root;
    if (xp == (xppl = n[xpp].left)) {
      if ((xppr = n[xpp].right) >= 0 && n[xppr].red) {
        n[xppr].red = 0;
        n[xp].red = 0;
        n[xpp].red = 1;
        x = xpp;
      } else {
        if (x == n[xp].right) {
          root = j_rotl(n, root, x = xp);
          xpp = (xp = n[x].parent) < 0 ? -1 : n[xp].parent;
        }
        if (xp >= 0) {
          n[xp].red = 0;
          if (xpp >= 0) {
            n[xpp].red = 1;
            root = j_rotr(n, root, xpp);
          }
        }
      }
    } else {
      if (xppl >= 0 && n[xppl].red) {
        n[xppl].red = 0;
        n[xp].red = 0;
        n[xpp].red = 1;
        x = xpp;
      } else {
        if (x == n[xp].left) {
          root = j_rotr(n, root, x = xp);
          xpp = (xp = n[x].parent) < 0 ? -1 : n[xp].parent;
        }
        if (xp >= 0) {
          n[xp].red = 0;
          if (xpp >= 0) {
            n[xpp].red = 1;
            root = j_rotl(n, root, xpp);
          }
        }
      }
    }
  }
}
__device__ void j_root_front(JMap& m, int32_t root) {
  JNode* n = m.n;
  const uint32_t idx = n[root].hash & (m.cap - 1);
  const int32_t first = m.tab[idx];
  if (root != first) {
    m.tab[idx] = root;
    const int32_t rp = n[root].prev, rn = n[root].next;
    if (rn >= 0) n[rn].prev = rp;
    if (rp >= 0) n[rp].next = rn;
    if (first >= 0) n[first].prev = root;
    n[root].next = first;
    n[root].prev = -1;
  }
}
__device__ void j_treeify(JMap& m, int32_t hd) {
  JNode* n = m.n;
  int32_t root = -1;
  for (int32_t x = hd, nx; x >= 0; x = nx) {
    nx = n[x].next;
    n[x].left = n[x].right = -1;
    if (root < 0) {
      n[x].parent = -1;
      n[x].red = 0;
      root = x;
      continue;
    }
    for (int32_t p = root;;) {
      const int dir = j_dir(m, p, n[x].hash, m.key[x]);
      const int32_t xp = p;
      if ((p = dir <= 0 ? n[p].left : n[p].right) < 0) {
        n[x].parent = xp;
        if (dir <= 0) n[xp].left = x;
        else n[xp].right = x;
        root = j_balance(n, root, x);
        break;
      }
    }
  }
  j_root_front(m, root);
}
__device__ void j_untreeify(JNode* n, int32_t hd) {
  for (int32_t x = hd; x >= 0; x = n[x].next) {
    n[x].tree = 0;
    n[x].left = n[x].right = n[x].parent = -1;
  }
}
// m.cap is already the new capacity; old bin `index` splits into index / index + bit
__device__ void j_split(JMap& m, int32_t b, uint32_t index, uint32_t bit) {
  JNode* n = m.n;
  int32_t loH = -1, loT = -1, hiH = -1, hiT = -1;
  uint32_t lc = 0, hc = 0;
  for (int32_t e = b, nx; e >= 0; e = nx) {
    nx = n[e].next;
    n[e].next = -1;
    if ((n[e].hash & bit) == 0) {
      if ((n[e].prev = loT) < 0) loH = e;
      else n[loT].next = e;
      loT = e;
      ++lc;
    } else {
      if ((n[e].prev = hiT) < 0) hiH = e;
      else n[hiT].next = e;
      hiT = e;
      ++hc;
    }
  }
  if (loH >= 0) {
    m.tab[index] = loH;
    if (lc <= 6) j_untreeify(n, loH);
    else if (hiH >= 0) j_treeify(m, loH);
  }
  if (hiH >= 0) {
    m.tab[index + bit] = hiH;
    if (hc <= 6) j_untreeify(n, hiH);
    else if (loH >= 0) j_treeify(m, hiH);
  }
}
__device__ void j_resize(JMap& m) {
  const uint32_t ocap = m.cap, ncap = ocap ? ocap * 2 : 16;
  JNode* n = m.n;
  for (uint32_t i = ocap; i < ncap; ++i) m.tab[i] = -1;
  m.cap = ncap;
  for (uint32_t j = 0; j < ocap; ++j) {
    const int32_t e = m.tab[j];
    if (e < 0) continue;
    m.tab[j] = -1;
    if (n[e].next < 0) {
      m.tab[n[e].hash & (ncap - 1)] = e;
    } else if (n[e].tree) {
      j_split(m, e, j, ocap);
    } else {
      int32_t loH = -1, loT = -1, hiH = -1, hiT = -1;
      for (int32_t x = e, nx; x >= 0; x = nx) {
        nx = n[x].next;
        if ((n[x].hash & ocap) == 0) {
          if (loT < 0) loH = x;
          else n[loT].next = x;
          loT = x;
        } else {
          if (hiT < 0) hiH = x;
          else n[hiT].next = x;
          hiT = x;
        }
      }
      if (loT >= 0) {
        n[loT].next = -1;
        m.tab[j] = loH;
      }
      if (hiT >= 0) {
        n[hiT].next = -1;
        m.tab[j + ocap] = hiH;
      }
    }
  }
  m.thr = ncap / 4 * 3;
}
__device__ void j_treeify_bin(JMap& m, uint32_t hash) {
  if (m.cap < 64) {   // MIN_TREEIFY_CAPACITY: resize instead
    m.flags |= 2;
    j_resize(m);
    return;
  }
  JNode* n = m.n;
  const int32_t hd = m.tab[hash & (m.cap - 1)];
  int32_t tl = -1;
  for (int32_t e = hd; e >= 0; e = n[e].next) {
    n[e].tree = 1;
    n[e].prev = tl;
    tl = e;
  }
  m.flags |= 1;
  j_treeify(m, hd);
}
__device__ void j_put(JMap& m, int32_t x) {
  JNode* n = m.n;
  if (m.cap == 0) j_resize(m);
  const uint32_t h = n[x].hash, i = h & (m.cap - 1);
  n[x].next = n[x].prev = n[x].parent = n[x].left = n[x].right = -1;
  n[x].red = 0;
  n[x].tree = 0;
  int32_t p = m.tab[i];
  if (p < 0) {
    m.tab[i] = x;
  } else if (n[p].tree) {   // putTreeVal from the bin's root
    int32_t root = p;
    while (n[root].parent >= 0) root = n[root].parent;
    n[x].tree = 1;
    for (int32_t q = root;;) {
      const int dir = j_dir(m, q, h, m.key[x]);
      const int32_t xp = q;
      if ((q = dir <= 0 ? n[q].left : n[q].right) < 0) {
        const int32_t xpn = n[xp].next;
        n[x].next = xpn;
        if (dir <= 0) n[xp].left = x;
        else n[xp].right = x;
        n[xp].next = x;
        n[x].parent = n[x].prev = xp;
        if (xpn >= 0) n[xpn].prev = x;
        j_root_front(m, j_balance(n, root, x));
        break;
      }
    }
  } else {
    for (int bin = 0;; ++bin) {
      const int32_t e = n[p].next;
      if (e < 0) {
        n[p].next = x;
        if (bin >= 7) j_treeify_bin(m, h);   // TREEIFY_THRESHOLD - 1
        break;
      }
      p = e;
    }
  }
  if (++m.size > m.thr) j_resize(m);
}
// ---- the simulation in parallel over bin groups ---------------------------------------------------
// Until the table reaches capacity 64, a bin of 9 resizes the whole table (treeifyBin below
// MIN_TREEIFY_CAPACITY); from 64 on every bin evolves alone: a resize happens right after the insertion
// whose index equals the threshold 3C/4 (it depends on the count only), treeifyBin converts its own bin,
// and a resize splits old bin j into new bins j and j + C only.  So one thread per set simulates the
// insertions until the table reaches HS_JG bins (at most 3 HS_JG / 4 + 1 keys: the size threshold alone
// takes it there), exactly as the JDK (trees may already form from capacity 64), and from there the keys
// of one group g = hash & (HS_JG - 1) -- bins g, g + HS_JG, g + 2 HS_JG, ... at every capacity >= HS_JG --
// are simulated by their own thread, continuing from the table the prefix left: its keys in arrival
// order (k_hs_jdk_order), the resizes applied at the global insertion indices where they occur, its
// bins' chains walked in bin order at the end.  The critical path of a hub's set of ~10^5 ids drops
// from k inserts to ~k / HS_JG.
constexpr uint32_t HS_JG = 256;
__global__ __launch_bounds__(64) void k_hs_jdk_prefix(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nc,
                                                      const uint64_t* __restrict__ doff, const int64_t* __restrict__ arr,
                                                      const uint64_t* __restrict__ tbase, JNode* __restrict__ nodes,
                                                      int32_t* __restrict__ tabs, int64_t* __restrict__ ids,
                                                      uint32_t* __restrict__ p0, uint32_t* __restrict__ flags) {
  const uint32_t count = *nc;
  for (uint32_t s = blockIdx.x * 64u + threadIdx.x; s < count; s += gridDim.x * 64u) {
    const uint32_t u = list[s];
    const uint64_t d0 = doff[u], k = doff[u + 1] - d0;
    JMap m{nodes + d0, arr + d0, tabs + tbase[s], 0, 0, 0, 0};
    uint32_t j = 0;
    for (; j < k && m.cap < HS_JG; ++j) {
      const int64_t x = m.key[j];
      const uint32_t h0 = (uint32_t)((uint64_t)x ^ ((uint64_t)x >> 32));
      m.n[j].hash = h0 ^ (h0 >> 16);
      j_put(m, (int32_t)j);
    }
    if (m.flags) atomicOr(flags, m.flags);
    if (m.cap >= HS_JG) {   // the groups take it from here (the table of the keys before j stays for them)
      p0[s] = j;
      continue;
    }
    p0[s] = ~0u;   // the whole set stayed below capacity HS_JG: done here
    uint64_t o = d0;
    for (uint32_t b = 0; b < m.cap; ++b)
      for (int32_t e = m.tab[b]; e >= 0; e = m.n[e].next) ids[o++] = m.key[e];
  }
}

// one wave per set: the set's keys stably partitioned by group (hash & (HS_JG - 1)), as arrival indices,
// into ord[d0 ..] with the group starts in gofs[(HS_JG + 1) s ..] (two passes: counts, then positions)
__global__ __launch_bounds__(64) void k_hs_jdk_order(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nc,
                                                     const uint64_t* __restrict__ doff, const int64_t* __restrict__ arr,
                                                     const uint32_t* __restrict__ p0, uint32_t* __restrict__ ord,
                                                     uint32_t* __restrict__ gofs) {
  __shared__ uint32_t s_run[HS_JG];
  constexpr uint32_t PER = HS_JG / 64;   // groups per lane in the scans
  const uint32_t count = *nc, lane = threadIdx.x;
  for (uint32_t s = blockIdx.x; s < count; s += gridDim.x) {
    if (p0[s] == ~0u) continue;   // (uniform over the block)
    const uint32_t u = list[s];
    const uint64_t d0 = doff[u], k = doff[u + 1] - d0;
    for (uint32_t i = 0; i < PER; ++i) s_run[lane * PER + i] = 0;
    __syncthreads();
    for (int pass = 0; pass < 2; ++pass) {
      for (uint64_t j0 = 0; j0 < k; j0 += 64) {
        const uint64_t j = j0 + lane;
        const bool on = j < k;
        const uint64_t act = ballot(on);
        uint32_t g = 0;
        if (on) {
          const int64_t x = arr[d0 + j];
          const uint32_t h0 = (uint32_t)((uint64_t)x ^ ((uint64_t)x >> 32));
          g = (h0 ^ (h0 >> 16)) & (HS_JG - 1);
        }
        const uint64_t peers = match_digit<8>(g, act);
        static_assert(HS_JG == 256, "match_digit width");
        const uint32_t rank = mbcnt(peers);
        const bool leader = on && rank == 0;
        if (pass == 1 && on) ord[d0 + s_run[g] + rank] = (uint32_t)j;
        __syncthreads();
        if (leader) s_run[g] += (uint32_t)__popcll(peers);
        __syncthreads();
      }
      if (pass == 0) {   // counts -> group starts (lane l holds groups [PER l, PER l + PER))
        uint32_t c[PER], t = 0;
        for (uint32_t i = 0; i < PER; ++i) t += (c[i] = s_run[lane * PER + i]);
        uint32_t at = wave_inclusive_sum(t) - t;
        __syncthreads();
        for (uint32_t i = 0; i < PER; ++i) {
          s_run[lane * PER + i] = at;
          gofs[(uint64_t)(HS_JG + 1) * s + lane * PER + i] = at;
          at += c[i];
        }
        if (lane == 63) gofs[(uint64_t)(HS_JG + 1) * s + HS_JG] = at;
        __syncthreads();
      }
    }
    __syncthreads();
  }
}

// insertion at capacity >= HS_JG (no size bookkeeping: the resizes come from the caller's schedule)
__device__ void j_put_group(JMap& m, int32_t x) {
  JNode* n = m.n;
  const uint32_t h = n[x].hash, i = h & (m.cap - 1);
  n[x].next = n[x].prev = n[x].parent = n[x].left = n[x].right = -1;
  n[x].red = 0;
  n[x].tree = 0;
  int32_t p = m.tab[i];
  if (p < 0) {
    m.tab[i] = x;
  } else if (n[p].tree) {   // putTreeVal from the bin's root
    int32_t root = p;
    while (n[root].parent >= 0) root = n[root].parent;
    n[x].tree = 1;
    for (int32_t q = root;;) {
      const int dir = j_dir(m, q, h, m.key[x]);
      const int32_t xp = q;
      if ((q = dir <= 0 ? n[q].left : n[q].right) < 0) {
        const int32_t xpn = n[xp].next;
        n[x].next = xpn;
        if (dir <= 0) n[xp].left = x;
        else n[xp].right = x;
        n[xp].next = x;
        n[x].parent = n[x].prev = xp;
        if (xpn >= 0) n[xpn].prev = x;
        j_root_front(m, j_balance(n, root, x));
        break;
      }
    }
  } else {
    for (int bin = 0;; ++bin) {
      const int32_t e = n[p].next;
      if (e < 0) {
        n[p].next = x;
        if (bin >= 7) j_treeify_bin(m, h);   // TREEIFY_THRESHOLD - 1 (capacity >= 64: the bin itself)
        break;
      }
      p = e;
    }
  }
}

// the group's bins of a resize from m.cap to 2 m.cap (the split of j_resize, bins j = g mod HS_JG only)
__device__ void j_resize_group(JMap& m, uint32_t g) {
  const uint32_t ocap = m.cap, ncap = ocap * 2;
  JNode* n = m.n;
  for (uint32_t i = ocap + g; i < ncap; i += HS_JG) m.tab[i] = -1;
  m.cap = ncap;
  for (uint32_t j = g; j < ocap; j += HS_JG) {
    const int32_t e = m.tab[j];
    if (e < 0) continue;
    m.tab[j] = -1;
    if (n[e].next < 0) {
      m.tab[n[e].hash & (ncap - 1)] = e;
    } else if (n[e].tree) {
      j_split(m, e, j, ocap);
    } else {
      int32_t loH = -1, loT = -1, hiH = -1, hiT = -1;
      for (int32_t x = e, nx; x >= 0; x = nx) {
        nx = n[x].next;
        if ((n[x].hash & ocap) == 0) {
          if (loT < 0) loH = x;
          else n[loT].next = x;
          loT = x;
        } else {
          if (hiT < 0) hiH = x;
          else n[hiT].next = x;
          hiT = x;
        }
      }
      if (loT >= 0) {
        n[loT].next = -1;
        m.tab[j] = loH;
      }
      if (hiT >= 0) {
        n[hiT].next = -1;
        m.tab[j + ocap] = hiH;
      }
    }
  }
}

// thread per (set, group): the group's keys from capacity 64 on; then the sizes of its final bins
__global__ __launch_bounds__(64) void k_hs_jdk_group(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nc,
                                                     const uint64_t* __restrict__ doff, const int64_t* __restrict__ arr,
                                                     const uint64_t* __restrict__ tbase, const uint32_t* __restrict__ p0,
                                                     const uint32_t* __restrict__ ord, const uint32_t* __restrict__ gofs,
                                                     JNode* __restrict__ nodes, int32_t* __restrict__ tabs,
                                                     uint64_t* __restrict__ bcnt, uint32_t* __restrict__ flags) {
  const uint64_t total = (uint64_t)*nc * HS_JG;
  for (uint64_t t = (uint64_t)blockIdx.x * 64 + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 64) {
    const uint32_t s = (uint32_t)(t / HS_JG), g = (uint32_t)(t % HS_JG);
    const uint32_t P0 = p0[s];
    if (P0 == ~0u) continue;
    const uint32_t u = list[s];
    const uint64_t d0 = doff[u], k = doff[u + 1] - d0;
    // bin g of the prefix's table at capacity HS_JG (plain or tree, as the JDK left it)
    JMap m{nodes + d0, arr + d0, tabs + tbase[s], HS_JG, 0, 0, 0};
    JNode* n = m.n;
    const uint32_t* o = ord + d0;
    const uint32_t a = gofs[(uint64_t)(HS_JG + 1) * s + g], b = gofs[(uint64_t)(HS_JG + 1) * s + g + 1];
    uint32_t q = a;
    while (q < b && o[q] < P0) ++q;   // (the prefix inserted them)
    for (; q < b; ++q) {
      const uint32_t j = o[q];
      while ((uint64_t)m.cap * 3 / 4 < j) j_resize_group(m, g);   // the resizes after inserts 3C/4 < j
      const int64_t x = m.key[j];
      const uint32_t h0 = (uint32_t)((uint64_t)x ^ ((uint64_t)x >> 32));
      n[j].hash = h0 ^ (h0 >> 16);
      j_put_group(m, (int32_t)j);
    }
    while ((uint64_t)m.cap * 3 / 4 < k) j_resize_group(m, g);   // the resizes after the set's last inserts
    if (m.flags) atomicOr(flags, m.flags);
    uint64_t* bc = bcnt + tbase[s];
    for (uint32_t bin = g; bin < m.cap; bin += HS_JG) {
      uint64_t c = 0;
      for (int32_t e = m.tab[bin]; e >= 0; e = n[e].next) ++c;
      bc[bin] = c;
    }
  }
}

// thread per (set, group): the chains of the group's bins at their iteration positions
__global__ __launch_bounds__(64) void k_hs_jdk_write(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nc,
                                                     const uint64_t* __restrict__ doff, const int64_t* __restrict__ arr,
                                                     const uint64_t* __restrict__ tbase, const uint32_t* __restrict__ p0,
                                                     const JNode* __restrict__ nodes, const int32_t* __restrict__ tabs,
                                                     const uint64_t* __restrict__ bpos, int64_t* __restrict__ ids) {
  const uint64_t total = (uint64_t)*nc * HS_JG;
  for (uint64_t t = (uint64_t)blockIdx.x * 64 + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 64) {
    const uint32_t s = (uint32_t)(t / HS_JG), g = (uint32_t)(t % HS_JG);
    if (p0[s] == ~0u) continue;
    const uint32_t u = list[s];
    const uint64_t d0 = doff[u], k = doff[u + 1] - d0;
    uint64_t cap = 64;
    while (cap * 3 / 4 < k) cap <<= 1;
    const JNode* n = nodes + d0;
    const int32_t* tab = tabs + tbase[s];
    const uint64_t* bp = bpos + tbase[s];
    for (uint64_t bin = g; bin < cap; bin += HS_JG) {
      uint64_t at = d0 + (bp[bin] - bp[0]);
      for (int32_t e = tab[bin]; e >= 0; e = n[e].next) ids[at++] = arr[d0 + e];
    }
  }
}

// thread per complex vertex: insert its ids in arrival order, then write them in iteration order
// (GS_HS_JDK_SERIAL = 1: the round-4 kernel, for A/B; the default is the group-parallel one above)
__global__ __launch_bounds__(64) void k_hs_jdk(const uint32_t* __restrict__ list, const uint32_t* __restrict__ nc,
                                               const uint64_t* __restrict__ doff, const int64_t* __restrict__ arr,
                                               const uint64_t* __restrict__ tbase, JNode* __restrict__ nodes,
                                               int32_t* __restrict__ tabs, int64_t* __restrict__ ids,
                                               uint32_t* __restrict__ flags) {
  const uint32_t count = *nc;
  for (uint32_t s = blockIdx.x * 64u + threadIdx.x; s < count; s += gridDim.x * 64u) {
    const uint32_t u = list[s];
    const uint64_t d0 = doff[u], k = doff[u + 1] - d0;
    JMap m{nodes + d0, arr + d0, tabs + tbase[s], 0, 0, 0, 0};
    for (uint32_t j = 0; j < k; ++j) {
      const int64_t x = m.key[j];
      const uint32_t h0 = (uint32_t)((uint64_t)x ^ ((uint64_t)x >> 32));
      m.n[j].hash = h0 ^ (h0 >> 16);
      j_put(m, (int32_t)j);
    }
    uint64_t o = d0;
    for (uint32_t b = 0; b < m.cap; ++b)
      for (int32_t e = m.tab[b]; e >= 0; e = m.n[e].next) ids[o++] = m.key[e];
    if (m.flags) atomicOr(flags, m.flags);
  }
}

}  // namespace gs

using namespace gs;

namespace gs {

enum { HS_VKEYS, HS_OFF, HS_NBR, HS_USEG, HS_COMP, HS_PIDX, HS_DKEY, HS_DFIRST, HS_DOFF, HS_OKEY, HS_OMID,
       HS_UKEY, HS_ORD, HS_IDS, HS_G, HS_GX, HS_TILES, HS_F, HS_FX, HS_CSZ, HS_CBASE, HS_CNT, HS_CPLX,
       HS_CLIST, HS_TSZ, HS_TBASE, HS_ARR, HS_NODES, HS_TABS, HS_GIDS, HS_OWN, HS_SLOT, HS_META, HS_SIZE, HS_VS,
       HS_P0, HS_GORD, HS_GOFS, HS_BCNT, HS_BPOS, HS_COUNT };
static_assert(HS_COUNT <= 40, "gs_ctx::hs");

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
// Vertices that leave the plain-bin model get their exact JDK order (k_hs_detect, k_hs_jdk).
// *jdk_flags: bit 0 = some bin was treeified, bit 1 = some bin forced a resize below capacity 64.
static gs_status hashset_exact(gs_ctx* c, uint64_t R, uint64_t U, uint64_t M, uint32_t B, uint32_t* jdk_flags) {
  char* sm = c->small.as<char>();
  uint32_t* d_hs = (uint32_t*)(sm + SM_HS);   // [0] complex vertices, [1] JDK flags
  GS_HIP(hipMemsetAsync(d_hs, 0, 8, c->stream));
  // arrival rank of every distinct entry: scan of the first-arrival flags over record positions
  GS_TRY(ensure(c, c->hs[HS_F], (R + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_FX], (R + 1) * 8));
  GS_HIP(hipMemsetAsync(c->hs[HS_F].p, 0, R * 8, c->stream));
  hipLaunchKernelGGL(k_hs_first, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_DFIRST].as<uint32_t>(), (uint32_t)M,
                     c->hs[HS_F].as<uint64_t>());
  GS_TRY(xscan(c, c->hs[HS_F].as<uint64_t>(), R, c->hs[HS_FX].as<uint64_t>()));
  GS_TRY(ensure(c, c->hs[HS_CSZ], (U + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_CBASE], (U + 1) * 8));
  hipLaunchKernelGGL(k_hs_csize, dim3(g256(U)), dim3(256), 0, c->stream, c->hs[HS_DOFF].as<uint64_t>(), (uint32_t)U,
                     c->hs[HS_CSZ].as<uint64_t>());
  GS_TRY(xscan(c, c->hs[HS_CSZ].as<uint64_t>(), U, c->hs[HS_CBASE].as<uint64_t>()));
  c->host_small[6] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 6, c->hs[HS_CBASE].as<uint64_t>() + U, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t CT = c->host_small[6];
  *jdk_flags = 0;
  if (CT == 0) return GS_OK;   // no vertex with 9 or more distinct neighbours
  GS_TRY(ensure(c, c->hs[HS_CNT], CT * 4));
  GS_TRY(ensure(c, c->hs[HS_CPLX], U * 4));
  GS_TRY(ensure(c, c->hs[HS_ARR], M * 8));
  GS_HIP(hipMemsetAsync(c->hs[HS_CNT].p, 0, CT * 4, c->stream));
  GS_HIP(hipMemsetAsync(c->hs[HS_CPLX].p, 0, U * 4, c->stream));
  hipLaunchKernelGGL(k_hs_detect, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_DKEY].as<uint64_t>(),
                     c->hs[HS_DFIRST].as<uint32_t>(), (uint32_t)M, B, c->hs[HS_VKEYS].as<int64_t>(),
                     c->hs[HS_DOFF].as<uint64_t>(), c->hs[HS_FX].as<uint64_t>(), c->hs[HS_CBASE].as<uint64_t>(),
                     c->hs[HS_CNT].as<uint32_t>(), c->hs[HS_ARR].as<int64_t>(), c->hs[HS_CPLX].as<uint32_t>());
  GS_TRY(ensure(c, c->hs[HS_CLIST], U * 4));
  GS_TRY(ensure(c, c->hs[HS_TSZ], (U + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_TBASE], (U + 1) * 8));
  hipLaunchKernelGGL(k_hs_clist, dim3(g256(U)), dim3(256), 0, c->stream, c->hs[HS_CPLX].as<uint32_t>(), (uint32_t)U,
                     c->hs[HS_DOFF].as<uint64_t>(), d_hs, c->hs[HS_CLIST].as<uint32_t>(),
                     c->hs[HS_TSZ].as<uint64_t>());
  GS_HIP(hipGetLastError());
  c->host_small[6] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 6, d_hs, 4, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t nc = c->host_small[6] & 0xffffffffull;
  if (nc == 0) return GS_OK;
  GS_TRY(xscan(c, c->hs[HS_TSZ].as<uint64_t>(), nc, c->hs[HS_TBASE].as<uint64_t>()));
  c->host_small[6] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 6, c->hs[HS_TBASE].as<uint64_t>() + nc, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t T = c->host_small[6];
  GS_TRY(ensure(c, c->hs[HS_NODES], M * sizeof(JNode)));
  GS_TRY(ensure(c, c->hs[HS_TABS], T * 4));
  const unsigned grid = (unsigned)std::min<uint64_t>((nc + 63) / 64, 4096);
  static const bool serial = getenv("GS_HS_JDK_SERIAL") && atoi(getenv("GS_HS_JDK_SERIAL")) != 0;   // A/B
  if (serial) {
    hipLaunchKernelGGL(k_hs_jdk, dim3(grid), dim3(64), 0, c->stream, c->hs[HS_CLIST].as<uint32_t>(), d_hs,
                       c->hs[HS_DOFF].as<uint64_t>(), c->hs[HS_ARR].as<int64_t>(), c->hs[HS_TBASE].as<uint64_t>(),
                       c->hs[HS_NODES].as<JNode>(), c->hs[HS_TABS].as<int32_t>(), c->hs[HS_IDS].as<int64_t>(), d_hs + 1);
  } else {
    GS_TRY(ensure(c, c->hs[HS_P0], nc * 4 + 4));
    GS_TRY(ensure(c, c->hs[HS_GORD], M * 4 + 4));
    GS_TRY(ensure(c, c->hs[HS_GOFS], nc * (HS_JG + 1) * 4 + 4));
    GS_TRY(ensure(c, c->hs[HS_BCNT], (T + 1) * 8));
    GS_TRY(ensure(c, c->hs[HS_BPOS], (T + 1) * 8));
    const uint32_t* cl = c->hs[HS_CLIST].as<uint32_t>();
    uint32_t* p0 = c->hs[HS_P0].as<uint32_t>();
    hipLaunchKernelGGL(k_hs_jdk_prefix, dim3(grid), dim3(64), 0, c->stream, cl, d_hs, c->hs[HS_DOFF].as<uint64_t>(),
                       c->hs[HS_ARR].as<int64_t>(), c->hs[HS_TBASE].as<uint64_t>(), c->hs[HS_NODES].as<JNode>(),
                       c->hs[HS_TABS].as<int32_t>(), c->hs[HS_IDS].as<int64_t>(), p0, d_hs + 1);
    hipLaunchKernelGGL(k_hs_jdk_order, dim3((unsigned)std::min<uint64_t>(nc, 16384)), dim3(64), 0, c->stream, cl, d_hs,
                       c->hs[HS_DOFF].as<uint64_t>(), c->hs[HS_ARR].as<int64_t>(), (const uint32_t*)p0,
                       c->hs[HS_GORD].as<uint32_t>(), c->hs[HS_GOFS].as<uint32_t>());
    GS_HIP(hipMemsetAsync(c->hs[HS_BCNT].p, 0, (T + 1) * 8, c->stream));
    const unsigned ggrid = (unsigned)std::min<uint64_t>(nc * (HS_JG / 64), 65536);   // HS_JG threads (groups) per set
    hipLaunchKernelGGL(k_hs_jdk_group, dim3(ggrid), dim3(64), 0, c->stream, cl, d_hs, c->hs[HS_DOFF].as<uint64_t>(),
                       c->hs[HS_ARR].as<int64_t>(), c->hs[HS_TBASE].as<uint64_t>(), (const uint32_t*)p0,
                       (const uint32_t*)c->hs[HS_GORD].as<uint32_t>(), (const uint32_t*)c->hs[HS_GOFS].as<uint32_t>(),
                       c->hs[HS_NODES].as<JNode>(), c->hs[HS_TABS].as<int32_t>(), c->hs[HS_BCNT].as<uint64_t>(), d_hs + 1);
    GS_HIP(hipGetLastError());
    GS_TRY(xscan(c, c->hs[HS_BCNT].as<uint64_t>(), T, c->hs[HS_BPOS].as<uint64_t>()));
    hipLaunchKernelGGL(k_hs_jdk_write, dim3(ggrid), dim3(64), 0, c->stream, cl, d_hs, c->hs[HS_DOFF].as<uint64_t>(),
                       c->hs[HS_ARR].as<int64_t>(), c->hs[HS_TBASE].as<uint64_t>(), (const uint32_t*)p0,
                       (const JNode*)c->hs[HS_NODES].as<JNode>(), (const int32_t*)c->hs[HS_TABS].as<int32_t>(),
                       (const uint64_t*)c->hs[HS_BPOS].as<uint64_t>(), c->hs[HS_IDS].as<int64_t>());
  }
  GS_HIP(hipGetLastError());
  c->host_small[6] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 6, d_hs, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *jdk_flags = (uint32_t)(c->host_small[6] >> 32);
  return GS_OK;
}

gs_status hashset_order(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, uint32_t* U_out,
                        uint32_t* M_out, uint64_t* key_xor_out, uint32_t* jdk_flags) {
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
  // every id differs from the first in its low s.bits bits (the sort's key mask): a dense rank table when
  // that span is small (R-MAT s23 C5 window: 32 MB; k_hs_prep spent 23 ms in binary searches without it)
  // Only when the span is within a small multiple of the vertices (a small window with sparse ids would
  // otherwise take up to 1 GiB), and a table that cannot be allocated leaves the binary search.
  const uint32_t* rank = nullptr;
  const uint64_t span = 1ull << std::max(s.bits, 1);
  if (s.bits <= HS_RANK_BITS && span <= std::max<uint64_t>(16 * U, 1ull << 20)) {
    if (ensure(c, c->hs_rank, span * 4) == GS_OK) {
      hipLaunchKernelGGL(k_hs_rank, dim3(g256(U)), dim3(256), 0, c->stream, c->hs[HS_VKEYS].as<int64_t>(), (uint32_t)U,
                         c->hs_rank.as<uint32_t>());
      rank = c->hs_rank.as<uint32_t>();
    } else {
      (void)hipGetLastError();   // the failed allocation's sticky error: the search needs no table
      c->err.clear();
    }
  }
  hipLaunchKernelGGL(k_hs_prep, dim3(g256(R)), dim3(256), 0, c->stream, c->hs[HS_ORD].as<uint32_t>(), (uint32_t)R, src,
                     dst, c->hs[HS_OFF].as<uint64_t>(), c->hs[HS_VKEYS].as<int64_t>(), (uint32_t)U, B, rank,
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
  hipLaunchKernelGGL(k_hs_ids, dim3(g256(M)), dim3(256), 0, c->stream, (const uint32_t*)sb.vals,
                     c->hs[HS_DKEY].as<uint64_t>(), (uint32_t)M, B, c->hs[HS_VKEYS].as<int64_t>(),
                     c->hs[HS_IDS].as<int64_t>());
  GS_HIP(hipGetLastError());
  GS_TRY(hashset_exact(c, R, U, M, B, jdk_flags));
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
  uint32_t jdk_flags = 0;
  GS_TRY(hashset_order(c, src, dst, n, &U, &M, &key_xor, &jdk_flags));
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

// Layout of a window's candidate output (see k_cand_emit): the "> v" flags and their scan, the compacted
// ids G, per-slot metadata and block starts vs[0..S] (vs[S] = the record count).  nparts > 1: only the
// vertices gs_owner_of assigns to `part` are slots.
static gs_status cand_layout(gs_ctx* c, uint32_t U, uint32_t M, uint32_t nparts, uint32_t part, uint32_t* S_out,
                             uint64_t* total) {
  GS_TRY(ensure(c, c->hs[HS_G], (M + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_GX], (M + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_GIDS], (M + 1) * 8));
  hipLaunchKernelGGL(k_hs_gt, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_IDS].as<int64_t>(), M,
                     c->hs[HS_DOFF].as<uint64_t>(), U, c->hs[HS_VKEYS].as<int64_t>(), c->hs[HS_G].as<uint64_t>());
  GS_HIP(hipGetLastError());
  GS_TRY(xscan(c, c->hs[HS_G].as<uint64_t>(), M, c->hs[HS_GX].as<uint64_t>()));
  hipLaunchKernelGGL(k_cand_gids, dim3(g256(M)), dim3(256), 0, c->stream, c->hs[HS_IDS].as<int64_t>(),
                     c->hs[HS_G].as<uint64_t>(), c->hs[HS_GX].as<uint64_t>(), M, c->hs[HS_GIDS].as<int64_t>());
  GS_HIP(hipGetLastError());
  const uint64_t *own = nullptr, *slot_of = nullptr;
  uint32_t S = U;
  if (nparts > 1) {
    GS_TRY(ensure(c, c->hs[HS_OWN], (size_t)(U + 1) * 8));
    GS_TRY(ensure(c, c->hs[HS_SLOT], (size_t)(U + 1) * 8));
    hipLaunchKernelGGL(k_cand_own, dim3(g256(U)), dim3(256), 0, c->stream, c->hs[HS_VKEYS].as<int64_t>(), U, nparts,
                       part, c->hs[HS_OWN].as<uint64_t>());
    GS_HIP(hipGetLastError());
    GS_TRY(xscan(c, c->hs[HS_OWN].as<uint64_t>(), U, c->hs[HS_SLOT].as<uint64_t>()));
    c->host_small[6] = 0;
    GS_HIP(hipMemcpyAsync(&c->host_small[6], c->hs[HS_SLOT].as<uint64_t>() + U, 8, hipMemcpyDeviceToHost, c->stream));
    GS_TRY(host_wait(c));
    S = (uint32_t)c->host_small[6];
    own = c->hs[HS_OWN].as<uint64_t>();
    slot_of = c->hs[HS_SLOT].as<uint64_t>();
  }
  GS_TRY(ensure(c, c->hs[HS_META], (size_t)(S + 1) * sizeof(CandMeta)));
  GS_TRY(ensure(c, c->hs[HS_SIZE], (size_t)(S + 1) * 8));
  GS_TRY(ensure(c, c->hs[HS_VS], (size_t)(S + 1) * 8));
  hipLaunchKernelGGL(k_cand_meta, dim3(g256(U)), dim3(256), 0, c->stream, c->hs[HS_OFF].as<uint64_t>(),
                     c->hs[HS_DOFF].as<uint64_t>(), c->hs[HS_G].as<uint64_t>(), c->hs[HS_GX].as<uint64_t>(), U, own,
                     slot_of, c->hs[HS_META].as<CandMeta>(), c->hs[HS_SIZE].as<uint64_t>());
  GS_HIP(hipGetLastError());
  GS_TRY(xscan(c, c->hs[HS_SIZE].as<uint64_t>(), S, c->hs[HS_VS].as<uint64_t>()));
  c->host_small[7] = 0;
  GS_HIP(hipMemcpyAsync(&c->host_small[7], c->hs[HS_VS].as<uint64_t>() + S, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *S_out = S;
  *total = c->host_small[7];
  return GS_OK;
}

// records [P0, P1) of the layout into a / b / f (device); OT = uint32_t: the ids as id - idb
template <typename OT>
static gs_status cand_emit(gs_ctx* c, uint32_t S, uint64_t P0, uint64_t P1, OT* a, OT* b, uint8_t* f, int64_t idb = 0) {
  const uint64_t n = P1 - P0;
  if (n == 0) return GS_OK;
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((n + 4095) / 4096, 4096));
  const uint64_t waves = blocks * 4;
  const uint64_t per_wave = ((n + waves - 1) / waves + 255) / 256 * 256;
  // bit 0: the flag column 4-byte aligned; bit 1: a and b 16-byte aligned (the fast path's vector stores)
  const int f4 = (((uintptr_t)f & 3) == 0 ? 1 : 0) | ((((uintptr_t)a | (uintptr_t)b) & 15) == 0 ? 2 : 0);
  static const int split_env = getenv("GS_CAND_SPLIT") ? atoi(getenv("GS_CAND_SPLIT")) : 1;   // A/B
  const uint64_t* vs = c->hs[HS_VS].as<uint64_t>();
  const CandMeta* meta = c->hs[HS_META].as<CandMeta>();
  const int64_t *vkeys = c->hs[HS_VKEYS].as<int64_t>(), *nbr = c->hs[HS_NBR].as<int64_t>(),
                *gids = c->hs[HS_GIDS].as<int64_t>();
  if (split_env) {   // the pair-row steps in a lean kernel, then the steps it listed
    GS_TRY(ensure(c, c->cand_steps, (n / 256 + waves + 16) * 8 + 64));
    uint32_t* steps_n = reinterpret_cast<uint32_t*>(c->cand_steps.p);
    uint64_t* steps = c->cand_steps.as<uint64_t>() + 8;
    GS_HIP(hipMemsetAsync(steps_n, 0, 4, c->stream));
    // (k_cand_emit_fast holds 90 VGPRs: 5 waves per SIMD; held to 80 for 6 it spills and ran 0.99 -> 1.00 ms
    // per 2^28 records, profiles/r05/c5/)
    hipLaunchKernelGGL(k_cand_emit_fast<OT>, dim3((unsigned)blocks), dim3(256), 0, c->stream, vs, S, meta, vkeys, nbr,
                       gids, P0, P1, per_wave, a, b, f, f4, steps, steps_n, idb);
    hipLaunchKernelGGL(k_cand_emit_rest<OT>, dim3(1024), dim3(256), 0, c->stream, vs, S, meta, vkeys, nbr, gids, P0, P1,
                       a, b, f, (const uint64_t*)steps, (const uint32_t*)steps_n, idb);
  } else {
    hipLaunchKernelGGL(k_cand_emit_all<OT>, dim3((unsigned)blocks), dim3(256), 0, c->stream, vs, S, meta, vkeys, nbr,
                       gids, P0, P1, per_wave, a, b, f, f4, nullptr, nullptr, idb);
  }
  return hip_check(c, hipGetLastError(), "k_cand_emit");
}

}  // namespace gs

extern "C" {

gs_status gs_window_candidates_part(gs_ctx* c, const gs_edge_batch* b, uint32_t nparts, uint32_t part,
                                    gs_pair_out* out) {
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!out || !out->n_out || (out->capacity && (!out->a || !out->b || !out->is_candidate)))
    return set_error(c, GS_EINVAL, "bad gs_pair_out");
  if (nparts == 0 || part >= nparts) return set_error(c, GS_EINVAL, "part %u of %u", part, nparts);
  GS_TRY(begin_call(c));
  out->reserved = 0;
  if (b->n == 0) {
    *out->n_out = 0;
    return GS_OK;
  }
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  uint32_t U = 0, M = 0, S = 0;
  uint64_t key_xor = 0, total = 0;
  uint32_t jdk_flags = 0;
  GS_TRY(hashset_order(c, src, dst, b->n, &U, &M, &key_xor, &jdk_flags));
  out->reserved = jdk_flags;   // bit 0 = a treeified bin, bit 1 = a collision resize (both simulated exactly)
  GS_TRY(cand_layout(c, U, M, nparts, part, &S, &total));
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
  GS_TRY(cand_emit(c, S, 0, total, a, bb, f));
  if (!direct) {
    GS_HIP(hipMemcpyAsync(out->a, a, total * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(out->b, bb, total * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(out->is_candidate, f, total, hipMemcpyDeviceToHost, c->stream));
  }
  GS_TRY(host_wait(c));
  return GS_OK;
}

gs_status gs_window_candidates(gs_ctx* c, const gs_edge_batch* b, gs_pair_out* out) {
  return gs_window_candidates_part(c, b, 1, 0, out);
}

gs_status gs_candidates_begin_part(gs_ctx* c, const gs_edge_batch* b, uint32_t nparts, uint32_t part,
                                   uint64_t* total_records, uint32_t* jdk_flags) {
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!total_records) return set_error(c, GS_EINVAL, "null total_records");
  if (nparts == 0 || part >= nparts) return set_error(c, GS_EINVAL, "part %u of %u", part, nparts);
  GS_TRY(begin_call(c));
  c->cand_seq = c->call_seq;
  c->cand_total = c->cand_cursor = 0;
  c->cand_U = c->cand_S = 0;
  // the session's part and id range before the empty-batch return: an empty session after a part
  // session must not keep the earlier nparts (gs_candidates_vertex_range would refuse it)
  c->cand_nparts = nparts;
  c->cand_idmin = c->cand_idmax = 0;
  *total_records = 0;
  if (jdk_flags) *jdk_flags = 0;
  if (b->n == 0) return GS_OK;
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  uint32_t U = 0, M = 0, S = 0, fl = 0;
  uint64_t key_xor = 0, total = 0;
  GS_TRY(hashset_order(c, src, dst, b->n, &U, &M, &key_xor, &fl));
  // the window's smallest and largest ids (vkeys ascending), read back with the layout's sizes: whether the
  // session can emit 32-bit id columns (gs_candidates_next_u32)
  const int64_t* vk = c->hs[HS_VKEYS].as<int64_t>();
  GS_HIP(hipMemcpyAsync(&c->host_small[300], vk, 8, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(&c->host_small[301], vk + (U - 1), 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(cand_layout(c, U, M, nparts, part, &S, &total));   // (waits)
  c->cand_idmin = (int64_t)c->host_small[300];
  c->cand_idmax = (int64_t)c->host_small[301];
  c->cand_nparts = nparts;
  c->cand_U = U;
  c->cand_S = S;
  c->cand_total = total;
  *total_records = total;
  if (jdk_flags) *jdk_flags = fl;
  return GS_OK;
}

gs_status gs_candidates_begin(gs_ctx* c, const gs_edge_batch* b, uint64_t* total_records, uint32_t* jdk_flags) {
  return gs_candidates_begin_part(c, b, 1, 0, total_records, jdk_flags);
}

static gs_status cand_session(gs_ctx* c) {
  if (c->cand_seq != c->call_seq)
    return set_error(c, GS_EINVAL, "no candidates session (gs_candidates_begin; a later call on the ctx ends it)");
  return hip_check(c, hipSetDevice(c->device), "hipSetDevice");
}

}  // extern "C"

namespace gs {
// gs_candidates_next / gs_candidates_next_u32: OT = the id columns' type, idb = what the u32 columns are
// relative to
template <typename OT, class Out>
static gs_status cand_next(gs_ctx* c, Out* out, int64_t idb, uint64_t* first_record, int32_t* done) {
  const uint64_t P0 = c->cand_cursor, n = std::min<uint64_t>(out->capacity, c->cand_total - P0), P1 = P0 + n;
  if (first_record) *first_record = P0;
  *out->n_out = n;
  out->reserved = 0;
  if (n == 0) {
    if (done) *done = c->cand_cursor >= c->cand_total;
    if (c->cand_total > P0 && out->capacity == 0) return set_error(c, GS_ECAPACITY, "capacity 0");
    return GS_OK;
  }
  OT *a = out->a, *bb = out->b;
  uint8_t* f = out->is_candidate;
  const bool direct = out->mem == GS_MEM_DEVICE;
  if (!direct) {
    c->last_kind = 0;   // the staging buffers now hold candidate records, not a reduce's rows
    GS_TRY(ensure(c, c->out_keys, n * 8));
    GS_TRY(ensure(c, c->out_a, n * 8));
    GS_TRY(ensure(c, c->out_b, n));
    a = c->out_keys.as<OT>();
    bb = c->out_a.as<OT>();
    f = c->out_b.as<uint8_t>();
  }
  GS_TRY(cand_emit<OT>(c, c->cand_S, P0, P1, a, bb, f, idb));
  if (!direct) {
    GS_HIP(hipMemcpyAsync(out->a, a, n * sizeof(OT), hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(out->b, bb, n * sizeof(OT), hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(out->is_candidate, f, n, hipMemcpyDeviceToHost, c->stream));
    GS_TRY(host_wait(c));
  }
  // device output: the chunk is enqueued on the ctx stream and the call returns without waiting (the
  // record count is known on the host), so a consumer ordered after it on that stream -- or waiting on an
  // event recorded there -- streams chunk after chunk with no host round trip between them
  c->cand_cursor = P1;
  if (done) *done = P1 >= c->cand_total;
  return GS_OK;
}
}  // namespace gs

extern "C" {

gs_status gs_candidates_next(gs_ctx* c, gs_pair_out* out, uint64_t* first_record, int32_t* done) {
  if (!c) return GS_EINVAL;
  if (!out || !out->n_out || (out->capacity && (!out->a || !out->b || !out->is_candidate)))
    return set_error(c, GS_EINVAL, "bad gs_pair_out");
  GS_TRY(cand_session(c));
  return cand_next<int64_t>(c, out, 0, first_record, done);
}

gs_status gs_candidates_next_u32(gs_ctx* c, gs_pair_out_u32* out, int64_t* id_base, uint64_t* first_record,
                                 int32_t* done) {
  if (!c) return GS_EINVAL;
  if (!out || !out->n_out || !id_base || (out->capacity && (!out->a || !out->b || !out->is_candidate)))
    return set_error(c, GS_EINVAL, "bad gs_pair_out_u32");
  GS_TRY(cand_session(c));
  *id_base = c->cand_idmin;
  if (c->cand_total && (uint64_t)c->cand_idmax - (uint64_t)c->cand_idmin > 0xFFFFFFFFull)
    return set_error(c, GS_EUNSUPPORTED, "the window's ids span more than 2^32 values: gs_candidates_next");
  return cand_next<uint32_t>(c, out, c->cand_idmin, first_record, done);
}

gs_status gs_candidates_seek(gs_ctx* c, uint64_t record) {
  if (!c) return GS_EINVAL;
  GS_TRY(cand_session(c));
  if (record > c->cand_total)
    return set_error(c, GS_EINVAL, "seek to record %llu of %llu", (unsigned long long)record,
                     (unsigned long long)c->cand_total);
  c->cand_cursor = record;
  return GS_OK;
}

gs_status gs_candidates_vertex_range(gs_ctx* c, int64_t vertex, uint64_t* first_record, uint64_t* records) {
  if (!c) return GS_EINVAL;
  if (!first_record || !records) return set_error(c, GS_EINVAL, "null output");
  GS_TRY(cand_session(c));
  *first_record = *records = 0;
  if (c->cand_nparts > 1)   // (a part's slots are its own vertices only: the block table is not per vertex)
    return set_error(c, GS_EUNSUPPORTED, "gs_candidates_vertex_range on a part session (gs_candidates_begin_part)");
  if (c->cand_total == 0) return GS_OK;
  GS_TRY(ensure(c, c->cand_bounds, 64));
  auto* d = c->cand_bounds.as<unsigned long long>();
  hipLaunchKernelGGL(k_cand_find, dim3(1), dim3(1), 0, c->stream, c->hs[HS_VKEYS].as<int64_t>(), c->cand_U,
                     c->hs[HS_VS].as<uint64_t>(), vertex, d);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(&c->host_small[6], d, 16, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *first_record = c->host_small[6];
  *records = c->host_small[7];
  return GS_OK;
}

}  // extern "C"
