// gs_triangles.hip — WindowTriangles on one GPU and split over several.
//
//   gs_window_triangles       <- slice(ALL) -> GenerateCandidateEdges -> CountTriangles -> sum(0)
//                                (WindowTriangles.java:61-66, :83-140)
//   gs_window_triangles_part  one part of the count (balanced share of the work), for callers that
//                                hold the whole window on every rank
//   gs_tri_dist_*             the window split over ranks: local degrees (all-reduce), oriented edges
//                                routed to owner(u) (all-to-all), local out-lists (all-gather), each
//                                rank's balanced share of the count (all-reduce)
#include <climits>
#include <string.h>

#include <vector>

#include "gs_ops.hpp"
#include "gs_tricount.hpp"

namespace gs {

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
// and count; the sort's digit histograms of the 2B-bit keys on the way (sort_buffer hist_ready).
// U edges per lane per step: every column load, then every rank gather, is issued before the first is
// used, so a wave keeps 2U random gathers in flight (U = 1 ran at the latency of one gather chain).
template <int U>
__global__ __launch_bounds__(256) void k_tri_okeys(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                   uint64_t n, uint64_t key_xor, uint32_t B,
                                                   const uint32_t* __restrict__ rank, uint64_t* __restrict__ out,
                                                   uint32_t* __restrict__ loop_bits, unsigned long long* __restrict__ loops,
                                                   uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][8][RADIX];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = tid; i < 4 * 8 * RADIX; i += 256) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const int nd = (int)(2 * B + 7) / 8;
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U; i0 < n; i0 += stride) {   // wave-uniform trip count
    uint64_t a[U], b[U];
    uint32_t ra[U], rb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + 256 * u + tid;
      a[u] = b[u] = 0;
      if (i < n) { a[u] = (uint64_t)src[i] ^ key_xor; b[u] = (uint64_t)dst[i] ^ key_xor; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ra[u] = rb[u] = 0;
      if (i0 + 256 * u + tid < n && a[u] != b[u]) { ra[u] = rank[a[u]]; rb[u] = rank[b[u]]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + 256 * u + tid;
      const bool ok = i < n;
      uint64_t k = sent;
      if (ok) {
        if (a[u] != b[u]) {
          const uint64_t x = ra[u], y = rb[u];
          k = x < y ? (x << B) | y : (y << B) | x;
        } else {
          atomicOr(&loop_bits[a[u] >> 5], 1u << (a[u] & 31));
          atomicAdd(loops, 1ull);
        }
        out[i] = k;
      }
      wave_hist_add(h[w], k, ok, nd);
    }
  }
  __syncthreads();
  flush_hist<4>(h, nd, hist);
}

// The same keys in two passes when the rank table outgrows the Infinity Cache (V > 2^25: 128 MB; C4's
// scale 26 has a 256 MB table): pass 1 resolves the endpoints below H through the lower half of the
// table and parks the rest as id | ESC in a 2 x 32-bit pair; pass 2 resolves those through the upper
// half, orients, and counts the sort's histograms.  Each pass gathers from a half table that the cache
// keeps.  U as in k_tri_okeys.
constexpr uint32_t OK_ESC = 1u << 31;
template <int U>
__global__ __launch_bounds__(256) void k_tri_okeys_lo(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      uint64_t n, uint64_t key_xor, uint32_t H,
                                                      const uint32_t* __restrict__ rank, uint64_t* __restrict__ out,
                                                      uint32_t* __restrict__ loop_bits,
                                                      unsigned long long* __restrict__ loops) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
    uint64_t a[U], b[U];
    uint32_t xa[U], xb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + 256 * u;
      a[u] = b[u] = 0;
      if (i < n) { a[u] = (uint64_t)src[i] ^ key_xor; b[u] = (uint64_t)dst[i] ^ key_xor; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xa[u] = a[u] < H ? rank[a[u]] : ((uint32_t)a[u] | OK_ESC);
      xb[u] = b[u] < H ? rank[b[u]] : ((uint32_t)b[u] | OK_ESC);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + 256 * u;
      if (i >= n) continue;
      uint64_t k = ~0ull;   // a self-loop: the sentinel (pass 2 keeps it)
      if (a[u] != b[u]) {
        k = ((uint64_t)xa[u] << 32) | xb[u];
      } else {
        atomicOr(&loop_bits[a[u] >> 5], 1u << (a[u] & 31));
        atomicAdd(loops, 1ull);
      }
      out[i] = k;
    }
  }
}
template <int U>
__global__ __launch_bounds__(256) void k_tri_okeys_hi(uint64_t* __restrict__ keys, uint64_t n, uint32_t B,
                                                      const uint32_t* __restrict__ rank, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][8][RADIX];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = tid; i < 4 * 8 * RADIX; i += 256) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const int nd = (int)(2 * B + 7) / 8;
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U; i0 < n; i0 += stride) {   // wave-uniform trip count
    uint64_t x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + 256 * u + tid;
      x[u] = i < n ? keys[i] : ~0ull;
    }
    uint32_t xa[U], xb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xa[u] = (uint32_t)(x[u] >> 32);
      xb[u] = (uint32_t)x[u];
      if (x[u] != ~0ull) {
        if (xa[u] & OK_ESC) xa[u] = rank[xa[u] & ~OK_ESC];
        if (xb[u] & OK_ESC) xb[u] = rank[xb[u] & ~OK_ESC];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + 256 * u + tid;
      const bool ok = i < n;
      uint64_t k = sent;
      if (ok) {
        if (x[u] != ~0ull) {
          const uint64_t ra = xa[u], rb = xb[u];
          k = ra < rb ? (ra << B) | rb : (rb << B) | ra;
        }
        keys[i] = k;
      }
      wave_hist_add(h[w], k, ok, nd);
    }
  }
  __syncthreads();
  flush_hist<4>(h, nd, hist);
}

// ---- the same keys with cache-local rank gathers (round 6) -------------------------------------------
// The split above still gathers each endpoint's rank at random from a 128 MB half table (2^31 gathers at
// s26, each a 32-64 byte sector beyond L2: ~120 GB of fabric traffic, 38.6 ms).  Here the records are
// first partitioned by the top PB bits of their source id (one onesweep pass over a << 32 | b), so the
// records in flight all gather rank[a] from one 2^(B-PB)-entry slice of the table (1 MB at s26), which
// every XCD's L2 keeps; the second pass gathers rank[a] on its load and partitions b << 32 | rank(a) by the
// top bits of b; the last pass resolves rank(b) the same way, orients and counts the sort's histograms.
// Partition histograms of both endpoints (k_tri_phist) give the two passes their digit bases.
constexpr uint32_t OK_LOOP = 0xFFFFFFFFu;   // pass 2's rank(a) of a self-loop
struct TriPartA {   // pass 1 records: the window's columns -> a << 32 | b
  const int64_t* src;
  const int64_t* dst;
  uint64_t key_xor;
  __device__ __forceinline__ void load(uint32_t r, uint64_t& k, uint8_t&) const {
    const uint64_t a = ((uint64_t)src[r] ^ key_xor) & 0xFFFFFFFFull, b = ((uint64_t)dst[r] ^ key_xor) & 0xFFFFFFFFull;
    k = (a << 32) | b;
  }
};
struct TriPartB {   // pass 2 records: a << 32 | b -> b << 32 | rank(a), gathered from the partition's slice
  const uint64_t* keys;
  const uint32_t* rank;
  __device__ __forceinline__ void load(uint32_t r, uint64_t& k, uint8_t&) const {
    const uint64_t x = keys[r];
    const uint32_t a = (uint32_t)(x >> 32), b = (uint32_t)x;
    const uint32_t ra = rank[a];   // unconditional: the ITEMS gathers of a lane issue together
    k = ((uint64_t)b << 32) | (a != b ? ra : OK_LOOP);
  }
};

// 256-bin histograms of both endpoints' top bits (id >> sh): hist[0][..] sources, hist[1][..] targets.
// mask_out (tri_geometry's id scan, when it guesses the width from the previous window): also the OR of
// (id ^ src[0]) over both columns, as k_keyinfo's mask
__global__ __launch_bounds__(256) void k_tri_phist(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                   uint64_t n, uint64_t key_xor, uint32_t sh,
                                                   uint32_t* __restrict__ hist, unsigned long long* __restrict__ mask_out) {
  __shared__ uint32_t h[4][8][RADIX];
  const int tid = threadIdx.x, w = tid >> 6;
  const uint64_t k0 = (uint64_t)src[0];
  uint64_t m = 0;
  for (int i = tid; i < 4 * 8 * RADIX; i += 256) (&h[0][0][0])[i] = 0;
  __syncthreads();
  constexpr int U = 4;
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U; i0 < n; i0 += stride) {   // wave-uniform trip count
    uint64_t a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = min(i0 + 256 * u + tid, n - 1);
      a[u] = (uint64_t)src[i] ^ key_xor;
      b[u] = (uint64_t)dst[i] ^ key_xor;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t k = ((a[u] >> sh) & 255u) | (((b[u] >> sh) & 255u) << 8);
      wave_hist_add(h[w], k, i0 + 256 * u + tid < n, 2);
      if (mask_out) m |= (a[u] ^ key_xor ^ k0) | (b[u] ^ key_xor ^ k0);   // (clamped tail loads repeat an id)
    }
  }
  if (mask_out) {
    m = wave_or(m);
    if ((tid & 63) == 0 && m) atomicOr(mask_out, (unsigned long long)m);
  }
  __syncthreads();
  flush_hist<4>(h, 2, hist);
}

// pass 3: b << 32 | rank(a) (partitioned by b) -> oriented keys, self-loops, the sort's histograms
// (the histograms: of the nd bytes of key >> hshift -- the whole key, or u alone for the segmented sort)
template <int U>
__global__ __launch_bounds__(256) void k_tri_okeys_part(const uint64_t* __restrict__ in, uint64_t n, uint32_t B,
                                                        const uint32_t* __restrict__ rank, uint64_t* __restrict__ out,
                                                        uint32_t* __restrict__ loop_bits,
                                                        unsigned long long* __restrict__ loops,
                                                        uint32_t hshift, int nd, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][8][RADIX];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = tid; i < 4 * 8 * RADIX; i += 256) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U; i0 < n; i0 += stride) {   // wave-uniform trip count
    uint64_t x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = in[min(i0 + 256 * u + tid, n - 1)];
    uint32_t rb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) rb[u] = rank[(uint32_t)(x[u] >> 32)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + 256 * u + tid;
      const bool ok = i < n;
      const uint32_t b = (uint32_t)(x[u] >> 32), ra = (uint32_t)x[u];
      uint64_t k = sent;
      if (ok) {
        if (ra != OK_LOOP) {
          const uint64_t p = ra, q = rb[u];
          k = p < q ? (p << B) | q : (q << B) | p;
        } else {
          atomicOr(&loop_bits[b >> 5], 1u << (b & 31));
          atomicAdd(loops, 1ull);
        }
        out[i] = k;
      }
      wave_hist_add(h[w], k >> hshift, ok, nd);
    }
  }
  __syncthreads();
  flush_hist<4>(h, nd, hist);
}

// ---- segmented sort of the oriented keys (round 6) ------------------------------------------------------
// The oriented keys u << B | v need a full sort only so that each out-list comes out sorted (the count's
// suffix trick and the unique step); the order between lists is u's.  So the global LSD passes sort by u
// alone (ceil(B / 8) passes instead of ceil(2B / 8): s26 7 -> 4), and k_tri_segsort sorts each run of equal
// u by v in LDS: a block takes the runs that start in its tile of SS_T keys (to the end of the last one),
// up to SS_CAP keys, and sorts them stably by the local key (run index << B | v) in LDS passes of 8 bits.
// A run that does not fit is queued for k_tri_segsort_long (a block per run: in LDS when it fits, else
// stable 8-bit passes over the run in HBM through the free sort buffer).
#ifndef GS_SS_ITEMS
#define GS_SS_ITEMS 8
#endif
constexpr int SS_BLOCK = 512, SS_ITEMS = GS_SS_ITEMS, SS_CAP = SS_BLOCK * SS_ITEMS, SS_NW = SS_BLOCK / WAVE;
constexpr uint32_t SS_T = SS_CAP / 2;   // run starts per block
static_assert(SS_T <= (uint32_t)SS_CAP, "a block's tile must fit its LDS chunk");

struct SsLds {
  uint64_t k[SS_CAP];            // 64 KiB: the chunk's local keys between passes
  uint32_t whist[SS_NW][RADIX];  // per-wave digit counters, then their exclusive prefix over the waves
  uint32_t start[RADIX];         // the tile's digit starts
  uint32_t cnt[RADIX];           // the tile's digit counts
  uint32_t wtot[SS_NW];
  unsigned long long bound[4];
};

// stable ranks by digit dg[j] of up to SS_CAP elements held wave-striped (item j of lane l in wave w is
// element w * SS_ITEMS * 64 + j * 64 + l; valid below len): pos[j] = its place in digit order within the
// tile, sh.cnt[d] = the tile's count of digit d (as k_onesweep's ranking, gs_radix.hpp)
__device__ __forceinline__ void ss_rank(const uint32_t (&dg)[SS_ITEMS], uint32_t len, uint32_t (&pos)[SS_ITEMS], SsLds& sh) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < SS_NW * RADIX; i += SS_BLOCK) (&sh.whist[0][0])[i] = 0;
  __syncthreads();
  const uint32_t e0 = (uint32_t)w * (SS_ITEMS * WAVE) + lane;
#pragma unroll
  for (int j = 0; j < SS_ITEMS; ++j) {
    const bool valid = e0 + j * WAVE < len;
    const uint32_t d = valid ? dg[j] : 0u;
    const uint64_t peers = match_digit<RADIX_BITS>(d, ballot(valid));
    const uint32_t lt = mbcnt(peers);
    uint32_t base = 0;
    if (valid) base = sh.whist[w][d];
    pos[j] = base + lt;
    if (valid && lt == 0) sh.whist[w][d] = base + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  if (tid < RADIX) {
    uint32_t c = 0;
#pragma unroll
    for (int x = 0; x < SS_NW; ++x) {
      const uint32_t t = sh.whist[x][tid];
      sh.whist[x][tid] = c;
      c += t;
    }
    sh.cnt[tid] = c;
    const uint32_t inc = wave_inclusive_sum(c);
    if (lane == 63) sh.wtot[w] = inc;
    sh.start[tid] = inc - c;
  }
  __syncthreads();
  if (tid < RADIX) {
    uint32_t off = 0;
    for (int x = 0; x < w; ++x) off += sh.wtot[x];
    sh.start[tid] += off;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SS_ITEMS; ++j) pos[j] += e0 + j * WAVE < len ? sh.start[dg[j]] + sh.whist[w][dg[j]] : 0u;
}

// sort `len` (<= SS_CAP) keys at keys[s ..) by (u, v) in LDS, in place; runs of equal u are contiguous
__device__ void ss_sort_chunk(uint64_t* __restrict__ keys, uint64_t s, uint32_t len, uint32_t B, SsLds& sh) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t vmask = (1ull << B) - 1;
  const uint32_t e0 = (uint32_t)w * (SS_ITEMS * WAVE) + lane;
  uint64_t lk[SS_ITEMS];
  uint32_t ku[SS_ITEMS], hb[SS_ITEMS], wrun = 0;   // u of each element; heads up to it within the wave
#pragma unroll
  for (int j = 0; j < SS_ITEMS; ++j) {   // unconditional, clamped loads
    const uint32_t e = min(e0 + j * WAVE, len - 1);
    const uint64_t k = keys[s + e], kp = keys[s + (e ? e - 1 : 0)];
    ku[j] = (uint32_t)(k >> B);
    lk[j] = k & vmask;
    const bool head = e0 + j * WAVE < len && (e == 0 || (uint32_t)(kp >> B) != ku[j]);
    const uint64_t m = ballot(head);
    hb[j] = wrun + mbcnt(m) + (head ? 1u : 0u);   // inclusive
    wrun += (uint32_t)__popcll(m);
  }
  // run index of each element: heads up to it, less one (a block scan in element order)
  if (lane == 0) sh.wtot[w] = wrun;
  __syncthreads();
  uint32_t woff = 0, nruns = 0;
  for (int x = 0; x < SS_NW; ++x) {
    const uint32_t t = sh.wtot[x];
    woff += x < w ? t : 0u;
    nruns += t;
  }
  const uint32_t rbits = nruns > 1 ? 32u - (uint32_t)__clz(nruns - 1) : 0u;
  const int passes = (int)((B + rbits + 7) / 8);
#pragma unroll
  for (int j = 0; j < SS_ITEMS; ++j) lk[j] |= (uint64_t)(woff + hb[j] - 1) << B;
  for (int p = 0; p < passes; ++p) {
    uint32_t dg[SS_ITEMS], pos[SS_ITEMS];
#pragma unroll
    for (int j = 0; j < SS_ITEMS; ++j) dg[j] = (uint32_t)(lk[j] >> (8 * p)) & 255u;
    ss_rank(dg, len, pos, sh);
#pragma unroll
    for (int j = 0; j < SS_ITEMS; ++j)
      if (e0 + j * WAVE < len) sh.k[pos[j]] = lk[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SS_ITEMS; ++j) lk[j] = sh.k[min(e0 + j * WAVE, len - 1)];
    __syncthreads();   // (the next pass's counters and key writes)
  }
  // runs keep their places: element i of the sorted chunk has the u of the element that was at i
#pragma unroll
  for (int j = 0; j < SS_ITEMS; ++j)
    if (e0 + j * WAVE < len) keys[s + e0 + j * WAVE] = ((uint64_t)ku[j] << B) | (lk[j] & vmask);
}

__global__ __launch_bounds__(SS_BLOCK) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_tri_segsort(uint64_t* __restrict__ keys, uint64_t n, uint32_t B, uint32_t cap,
                                                          uint64_t* __restrict__ long_runs,
                                                          unsigned long long* __restrict__ n_long) {
  __shared__ SsLds sh;
  const int tid = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * SS_T, t1 = min(t0 + SS_T, n);
  if (tid < 2) sh.bound[tid] = tid == 0 ? ~0ull : 0ull;
  if (tid == 2) sh.bound[2] = n;
  __syncthreads();
  // the first and the last run start in [t0, t1)
  constexpr uint32_t PER = SS_T / SS_BLOCK;
  for (uint32_t j = 0; j < PER; ++j) {
    const uint64_t i = t0 + (uint64_t)j * SS_BLOCK + tid;
    if (i < t1 && (i == 0 || (keys[i - 1] >> B) != (keys[i] >> B))) {
      atomicMin(&sh.bound[0], (unsigned long long)i);
      atomicMax(&sh.bound[1], (unsigned long long)i);
    }
  }
  __syncthreads();
  const uint64_t s = sh.bound[0], h = sh.bound[1];
  if (s == ~0ull) return;   // the whole tile lies inside a run that starts before it
  // the end of the last run: the first run start at or after t1 (searched while the chunk still fits)
  const uint64_t uh = keys[h] >> B;
  for (uint64_t b0 = t1; b0 < n && b0 - s <= cap; b0 += SS_BLOCK) {
    const uint64_t i = b0 + tid;
    if (i < n && (keys[i] >> B) != uh) atomicMin(&sh.bound[2], (unsigned long long)i);
    __syncthreads();
    const bool found = sh.bound[2] != n;
    __syncthreads();   // (every thread has read it before the next window's atomics)
    if (found) break;
  }
  __syncthreads();
  const uint64_t e = sh.bound[2];
  uint64_t end = e;
  if (e - s > cap) {   // the last run goes to k_tri_segsort_long; the runs before it (inside the tile) stay here
    if (tid == 0) long_runs[atomicAdd(n_long, 1ull)] = h;
    end = h;
  }
  if (end > s + 1) ss_sort_chunk(keys, s, (uint32_t)(end - s), B, sh);
}

// the runs k_tri_segsort queued (their starts), a block each: the run's end, then its keys sorted by v in
// LDS (<= SS_CAP) or by stable passes of 8 bits over the run in HBM (keys -> tmp -> keys ..)
__global__ __launch_bounds__(SS_BLOCK) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_tri_segsort_long(uint64_t* __restrict__ keys, uint64_t* __restrict__ tmp,
                                                               uint64_t n, uint32_t B, uint32_t lds_max,
                                                               const uint64_t* __restrict__ runs,
                                                               const unsigned long long* __restrict__ n_runs) {
  __shared__ SsLds sh;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t nr = *n_runs, vmask = (1ull << B) - 1;
  for (uint64_t r = blockIdx.x; r < nr; r += gridDim.x) {
    const uint64_t h = runs[r], uh = keys[h] >> B;
    __syncthreads();
    if (tid == 0) sh.bound[2] = n;
    __syncthreads();
    for (uint64_t b0 = h + 1; b0 < n; b0 += SS_BLOCK) {
      const uint64_t i = b0 + tid;
      if (i < n && (keys[i] >> B) != uh) atomicMin(&sh.bound[2], (unsigned long long)i);
      __syncthreads();
      const bool found = sh.bound[2] != n;
      __syncthreads();
      if (found) break;
    }
    __syncthreads();
    const uint64_t e = sh.bound[2], L = e - h;
    if (uh == vmask) continue;   // the self-loop sentinels: equal keys
    if (L <= (uint64_t)lds_max) {
      ss_sort_chunk(keys, h, (uint32_t)L, B, sh);
      continue;
    }
    const int passes = (int)((B + 7) / 8);
    const uint32_t e0 = (uint32_t)w * (SS_ITEMS * WAVE) + lane;
    uint64_t* src = keys;
    uint64_t* dst = tmp;
    for (int p = 0; p < passes; ++p) {
      const uint32_t shift = 8u * (uint32_t)p;
      // the run's digit counts -> exclusive offsets (sh.bound[3] unused)
      __syncthreads();
      if (tid < RADIX) sh.whist[0][tid] = 0;
      __syncthreads();
      for (uint64_t i = h + tid; i < e; i += SS_BLOCK) atomicAdd(&sh.whist[0][(uint32_t)(src[i] >> shift) & 255u], 1u);
      __syncthreads();
      uint32_t goff = 0;   // thread d (< RADIX): the run's exclusive offset of digit d, carried over its tiles
      if (tid < RADIX) {
        const uint32_t c = sh.whist[0][tid];
        const uint32_t inc = wave_inclusive_sum(c);
        if (lane == 63) sh.wtot[w] = inc;
        goff = inc - c;
      }
      __syncthreads();
      if (tid < RADIX)
        for (int x = 0; x < w; ++x) goff += sh.wtot[x];
      // stable scatter, tile by tile in order
      for (uint64_t t = h; t < e; t += SS_CAP) {
        const uint32_t len = (uint32_t)min<uint64_t>(SS_CAP, e - t);
        uint64_t k[SS_ITEMS];
        uint32_t dg[SS_ITEMS], pos[SS_ITEMS];
#pragma unroll
        for (int j = 0; j < SS_ITEMS; ++j) {
          k[j] = src[t + min(e0 + j * WAVE, len - 1)];
          dg[j] = (uint32_t)(k[j] >> shift) & 255u;
        }
        __syncthreads();   // the previous tile's readers of sh.start / sh.k are done
        if (tid < RADIX) sh.k[SS_CAP - RADIX + tid] = goff;   // (parked: ss_rank reuses whist / start / cnt)
        ss_rank(dg, len, pos, sh);
        // global place: the digit's offset so far + the rank among this tile's keys of that digit
#pragma unroll
        for (int j = 0; j < SS_ITEMS; ++j)
          if (e0 + j * WAVE < len)
            dst[h + sh.k[SS_CAP - RADIX + dg[j]] + (pos[j] - sh.start[dg[j]])] = k[j];
        __syncthreads();
        if (tid < RADIX) goff += sh.cnt[tid];
      }
      uint64_t* x = src;
      src = dst;
      dst = x;
    }
    if (src != keys) {   // an odd number of passes: back into keys
      __syncthreads();
      for (uint64_t i = h + tid; i < e; i += SS_BLOCK) keys[i] = src[i];
    }
    (void)vmask;
  }
}

// the unique oriented edges (sorted keys u << B | v) -> out-lists: nbr[p] = v, out_range[u] =
// [first, last + 1) (ranges of absent vertices were zeroed)
__global__ __launch_bounds__(256) void k_tri_out(const uint64_t* __restrict__ keys, uint32_t M, uint32_t B,
                                                 uint32_t* __restrict__ nbr, uint32_t* __restrict__ out_range) {
  const uint64_t mask = (1ull << B) - 1;
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < M; p += gridDim.x * 256u) {
    const uint64_t k = keys[p];
    const uint32_t u = (uint32_t)(k >> B);
    nbr[p] = (uint32_t)(k & mask);
    if (p == 0 || (uint32_t)(keys[p - 1] >> B) != u) out_range[2 * u] = p;
    if (p + 1 == M || (uint32_t)(keys[p + 1] >> B) != u) out_range[2 * u + 1] = p + 1;
  }
}

// ---- the unique oriented edges straight into out-lists (wide keys, the whole window) -----------------
// One read of the sorted keys counts each tile's heads (a key other than its predecessor and other than the
// self-loop sentinel, which sorts last), an exclusive scan of the tile counts places them, and a second read
// writes nbr[p] = v and rowid[p] = u at each head's unique index p and the row bounds out_range[u] --
// instead of writing the unique keys (reduce-by-key) and reading them back to cut them into rows.
constexpr uint32_t UO_BLOCK = 256, UO_ITEMS = 16, UO_TILE = UO_BLOCK * UO_ITEMS;
// (hist, when not null: the transposed sort's digit histograms of the unique targets v (B bits), counted here
// -- tiles grid-strided over the blocks, so each block flushes its tables once -- for TriTpaySrc's first pass)
__global__ __launch_bounds__(UO_BLOCK) void k_tri_uo_count(const uint64_t* __restrict__ keys, uint64_t n, uint64_t sent,
                                                           uint64_t tiles, unsigned long long* __restrict__ tile_cnt,
                                                           uint32_t B, uint32_t* __restrict__ hist) {
  constexpr int NW = UO_BLOCK / WAVE;
  __shared__ uint32_t s_w[NW];
  __shared__ uint32_t s_h[NW][8][RADIX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nd = (int)(B + 7) / 8;
  const uint64_t vmask = (1ull << B) - 1;
  if (hist) {
    for (int i = threadIdx.x; i < NW * 8 * RADIX; i += UO_BLOCK) (&s_h[0][0][0])[i] = 0;
  }
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {   // block-uniform
    const uint64_t t0 = tile * UO_TILE;
    uint64_t k[UO_ITEMS], kp[UO_ITEMS];
#pragma unroll
    for (int j = 0; j < UO_ITEMS; ++j) {   // unconditional, clamped loads
      const uint64_t i = min(t0 + (uint64_t)j * UO_BLOCK + threadIdx.x, n - 1);
      k[j] = keys[i];
      kp[j] = keys[i ? i - 1 : 0];
    }
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < UO_ITEMS; ++j) {
      const uint64_t i = t0 + (uint64_t)j * UO_BLOCK + threadIdx.x;
      const bool head = i < n && k[j] != sent && (i == 0 || kp[j] != k[j]);
      c += head ? 1u : 0u;
      if (hist) wave_hist_add(s_h[w], k[j] & vmask, head, nd);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, WAVE);
    if (lane == 0) s_w[w] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
#pragma unroll
      for (int x = 0; x < NW; ++x) t += s_w[x];
      tile_cnt[tile] = t;
    }
    __syncthreads();   // (s_w of the next tile)
  }
  if (hist) {
    __syncthreads();
    flush_hist<NW>(s_h, nd, hist);
  }
}

__global__ __launch_bounds__(UO_BLOCK) void k_tri_uo_write(const uint64_t* __restrict__ keys, uint64_t n, uint64_t sent,
                                                           uint32_t B, const unsigned long long* __restrict__ tile_pre,
                                                           uint32_t* __restrict__ nbr, uint32_t* __restrict__ rowid,
                                                           uint32_t* __restrict__ out_range) {
  constexpr int NW = UO_BLOCK / WAVE;
  __shared__ uint32_t s_cnt[UO_ITEMS][NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t t0 = (uint64_t)blockIdx.x * UO_TILE;
  const uint64_t mask = (1ull << B) - 1;
  uint64_t k[UO_ITEMS], kp[UO_ITEMS], hb[UO_ITEMS];
#pragma unroll
  for (int j = 0; j < UO_ITEMS; ++j) {
    const uint64_t i = min(t0 + (uint64_t)j * UO_BLOCK + threadIdx.x, n - 1);
    k[j] = keys[i];
    kp[j] = keys[i ? i - 1 : 0];
  }
#pragma unroll
  for (int j = 0; j < UO_ITEMS; ++j) {
    const uint64_t i = t0 + (uint64_t)j * UO_BLOCK + threadIdx.x;
    hb[j] = __ballot(i < n && k[j] != sent && (i == 0 || kp[j] != k[j]));
    if (lane == 0) s_cnt[j][w] = (uint32_t)__popcll(hb[j]);
  }
  __syncthreads();
  uint64_t run = tile_pre[blockIdx.x];   // heads before this tile, then before round j
#pragma unroll
  for (int j = 0; j < UO_ITEMS; ++j) {
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int x = 0; x < NW; ++x) {
      const uint32_t c = s_cnt[j][x];
      tot += c;
      before += x < w ? c : 0u;
    }
    const uint64_t i = t0 + (uint64_t)j * UO_BLOCK + threadIdx.x;
    const uint64_t excl = run + before + mbcnt(hb[j]);   // heads before key i
    run += tot;
    if (i >= n || k[j] == sent) continue;
    const bool head = (hb[j] >> lane) & 1ull;
    const uint32_t u = (uint32_t)(k[j] >> B);
    if (head) {
      nbr[excl] = (uint32_t)(k[j] & mask);
      rowid[excl] = u;
      if (i == 0 || (uint32_t)(kp[j] >> B) != u) out_range[2 * u] = (uint32_t)excl;
    }
    const uint64_t kn = i + 1 < n ? keys[i + 1] : sent;   // the row ends at key i: the next key is another row's
    if (kn == sent || (uint32_t)(kn >> B) != u) out_range[2 * u + 1] = (uint32_t)(excl + (head ? 1u : 0u));
  }
}

// the transposed sort's first pass reads the out-lists directly (its histograms: k_tri_uo_count): record p ->
// key v = nbr[p], payload the
// suffix of N+(u) past v, [p + 1, end of N+(u)) (what k_tri_tpay would have written; u = rowid[p])
struct TriTpaySrc {
  const uint32_t* nbr;
  const uint32_t* rowid;
  const uint2* out_range;
  __device__ __forceinline__ void load(uint32_t r, uint32_t& k, uint64_t& v) const {
    k = nbr[r];
    v = ((uint64_t)out_range[rowid[r]].y << 32) | (uint64_t)(r + 1);
  }
};

// row (u) of each adjacency position of a slice, from the out-lists (one thread per u; d+(u) is
// small under the degree orientation)
__global__ __launch_bounds__(256) void k_tri_rowid(const uint2* __restrict__ out_range, uint32_t u0, uint32_t u1,
                                                   uint32_t p0, uint32_t* __restrict__ rowid) {
  for (uint32_t u = u0 + blockIdx.x * 256u + threadIdx.x; u < u1; u += gridDim.x * 256u) {
    const uint2 r = out_range[u];
    for (uint32_t p = r.x; p < r.y; ++p) rowid[p - p0] = u;
  }
}

// the transposed sort's input over the slice [p0, p1) of the adjacency: key v, payload the part of
// N+(u) past v, [p + 1, end of N+(u)) -- sorted by v it becomes the in-entries' suffix ranges; the
// digit histograms of the B-bit keys on the way.  Row of p: the sorted keys (whole window) or rowid.
template <bool ROWID>
__global__ __launch_bounds__(256) void k_tri_tpay(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ rowid,
                                                  const uint32_t* __restrict__ nbr, uint32_t p0, uint32_t p1,
                                                  uint32_t B, const uint2* __restrict__ out_range,
                                                  uint64_t* __restrict__ tkey, uint2* __restrict__ pay,
                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][8][RADIX];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = tid; i < 4 * 8 * RADIX; i += 256) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const int nd = (int)(B + 7) / 8;
  for (uint32_t q0 = p0 + blockIdx.x * 256u; q0 < p1; q0 += gridDim.x * 256u) {   // wave-uniform trip count
    const uint32_t p = q0 + tid;
    const bool ok = p < p1;
    uint32_t v = 0;
    if (ok) {
      uint32_t u;
      if constexpr (ROWID) u = rowid[p - p0];
      else u = (uint32_t)(keys[p] >> B);
      v = nbr[p];
      tkey[p - p0] = v;
      pay[p - p0] = make_uint2(p + 1, out_range[u].y);
    }
    wave_hist_add(h[w], v, ok, nd);
  }
  __syncthreads();
  flush_hist<4>(h, nd, hist);
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

// ---- the split over parts --------------------------------------------------------------------------
// counting work of u: the suffixes of N+(u) it hands out, d(d-1)/2, plus one unit per in-entry
__global__ __launch_bounds__(256) void k_tri_work(const uint2* __restrict__ out_range, uint32_t V,
                                                  unsigned long long* __restrict__ work) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < V; u += gridDim.x * 256u) {
    const uint64_t d = out_range[u].y - out_range[u].x;
    work[u] = d * (d + 1) / 2;
  }
}

// part `part` of nparts: the u-range [u0, u1) holding its equal share of the work (pre = exclusive
// prefix of k_tri_work, pre[V] = total), and that range's adjacency slice [p0, p1) -> out[0..3].
// Slice ends: a search in the sorted keys (okeys), else the prefix-built out_range of u0 / u1.
__global__ void k_tri_bounds(const unsigned long long* __restrict__ pre, uint32_t V, const uint2* __restrict__ out_range,
                             const uint64_t* __restrict__ okeys, uint32_t B, uint32_t M, uint32_t part, uint32_t nparts,
                             uint32_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const unsigned long long W = pre[V];
  auto lower = [&](unsigned long long t) {   // first u with pre[u] >= t
    uint32_t a = 0, b = V;
    while (a < b) {
      const uint32_t m = (a + b) >> 1;
      if (pre[m] < t) a = m + 1;
      else b = m;
    }
    return a;
  };
  auto pos = [&](uint32_t u) -> uint32_t {   // first adjacency position of a row >= u
    if (u >= V) return M;
    if (!okeys) return out_range[u].x;
    const uint64_t key = (uint64_t)u << B;
    uint32_t a = 0, b = M;
    while (a < b) {
      const uint32_t m = (a + b) >> 1;
      if (okeys[m] < key) a = m + 1;
      else b = m;
    }
    return a;
  };
  const uint32_t u0 = part == 0 ? 0u : lower(frac_share(W, part, nparts));
  const uint32_t u1 = part + 1 == nparts ? V : lower(frac_share(W, part + 1, nparts));
  out[0] = u0;
  out[1] = u1;
  out[2] = pos(u0);
  out[3] = max(pos(u0), pos(u1));
}

// out-lists from the (all-reduced) out-degrees: out_range[u] = [pre[u], pre[u] + d+(u))
__global__ __launch_bounds__(256) void k_tri_ranges(const uint32_t* __restrict__ dplus, const unsigned long long* __restrict__ pre,
                                                    uint32_t V, uint2* __restrict__ out_range) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < V; u += gridDim.x * 256u) {
    const uint32_t a = (uint32_t)pre[u];
    out_range[u] = make_uint2(a, a + dplus[u]);
  }
}

__global__ __launch_bounds__(256) void k_u32_to_u64(const uint32_t* __restrict__ in, uint32_t n,
                                                    unsigned long long* __restrict__ out) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) out[i] = in[i];
}

// d+(u) of the local out-lists (the build step of the split window)
__global__ __launch_bounds__(256) void k_tri_dplus(const uint2* __restrict__ out_range, uint32_t V, uint32_t* __restrict__ dplus) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < V; u += gridDim.x * 256u)
    dplus[u] = out_range[u].y - out_range[u].x;
}

// ---- routing oriented keys to owner(u): contiguous u ranges [split[q], split[q + 1]) of the degree
// order, cut at equal shares of the raw work (gs_tri_dist_route) ---------------------------------------
constexpr int RT_BLOCK = 256, RT_ITEMS = 16, RT_TILE = RT_BLOCK * RT_ITEMS, RT_MAXP = 64;
static_assert(sizeof(RtSplit) == (RT_MAXP + 1) * 4, "RtSplit");   // split[0] = 0 <= .. <= split[nparts] = V
__device__ __forceinline__ uint32_t tri_owner(uint64_t key, uint32_t B, uint32_t nparts, const RtSplit& sp) {
  const uint32_t u = (uint32_t)(key >> B);
  uint32_t a = 0, b = nparts;   // the last q with split[q] <= u
  while (b - a > 1) {
    const uint32_t m = (a + b) >> 1;
    if (sp.s[m] <= u) a = m;
    else b = m;
  }
  return a;
}
// raw (with duplicates) oriented out-degree of the local keys: dout[u] += 1 per key u << B | v
__global__ __launch_bounds__(256) void k_tri_dout(const uint64_t* __restrict__ keys, uint64_t n, uint32_t B,
                                                  uint32_t* __restrict__ dout) {
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t k = keys[i];
    if (k != sent) atomicAdd(&dout[k >> B], 1u);
  }
}
// raw work of u: dout(dout + 1) / 2
__global__ __launch_bounds__(256) void k_tri_rawwork(const uint32_t* __restrict__ dout, uint32_t V,
                                                     unsigned long long* __restrict__ w) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < V; u += gridDim.x * 256u) {
    const uint64_t d = dout[u];
    w[u] = d * (d + 1) / 2;
  }
}
// split points at equal shares of the work prefix pre (pre[V] = total): out[q], q = 0..P
__global__ void k_tri_split(const unsigned long long* __restrict__ pre, uint32_t V, uint32_t P,
                            unsigned long long* __restrict__ out) {
  const uint32_t q = threadIdx.x;
  if (q > P) return;
  const unsigned long long W = pre[V];
  uint32_t a = 0, b = V;
  const unsigned long long t = frac_share(W, q, P);
  while (a < b) {
    const uint32_t m = (a + b) >> 1;
    if (pre[m] < t) a = m + 1;
    else b = m;
  }
  out[q] = q == 0 ? 0u : q == P ? V : a;
}
__global__ __launch_bounds__(RT_BLOCK) void k_route_count(const uint64_t* __restrict__ keys, uint64_t n, uint32_t B,
                                                          uint32_t nparts, RtSplit sp, uint32_t tiles,
                                                          uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_c[RT_MAXP];
  const int tid = threadIdx.x;
  if (tid < RT_MAXP) s_c[tid] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * RT_TILE;
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  for (int j = 0; j < RT_ITEMS; ++j) {
    const uint64_t i = base + (uint64_t)j * RT_BLOCK + tid;
    if (i < n && keys[i] != sent) atomicAdd(&s_c[tri_owner(keys[i], B, nparts, sp)], 1u);
  }
  __syncthreads();
  if (tid < (int)nparts) cnt[(uint64_t)tid * tiles + blockIdx.x] = s_c[tid];
}
// (k_rank_scan: the exclusive scan, owner-major) then the scatter; order inside an owner is free
// (the owner sorts what it receives)
__global__ __launch_bounds__(RT_BLOCK) void k_route_scatter(const uint64_t* __restrict__ keys, uint64_t n, uint32_t B,
                                                            uint32_t nparts, RtSplit sp, uint32_t tiles,
                                                            const uint32_t* __restrict__ off, uint64_t* __restrict__ out) {
  __shared__ uint32_t s_c[RT_MAXP];
  const int tid = threadIdx.x;
  if (tid < (int)nparts) s_c[tid] = off[(uint64_t)tid * tiles + blockIdx.x];
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * RT_TILE;
  const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
  for (int j = 0; j < RT_ITEMS; ++j) {
    const uint64_t i = base + (uint64_t)j * RT_BLOCK + tid;
    if (i < n) {
      const uint64_t k = keys[i];
      if (k != sent) out[atomicAdd(&s_c[tri_owner(k, B, nparts, sp)], 1u)] = k;
    }
  }
}

// signed min / max of every endpoint id -> mm[0] (min), mm[1] (max)
__global__ __launch_bounds__(256) void k_tri_minmax(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                    uint64_t n, long long* __restrict__ mm) {
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const long long a = src[i], b = dst[i];
    lo = min(lo, min(a, b));
    hi = max(hi, max(a, b));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (long long)__shfl_xor(lo, o, WAVE));
    hi = max(hi, (long long)__shfl_xor(hi, o, WAVE));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

// self-loop bitmap + count of a window (the self-pair term of a gathered window)
__global__ __launch_bounds__(256) void k_tri_loops(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                   uint64_t n, uint64_t key_xor, uint32_t* __restrict__ loop_bits,
                                                   unsigned long long* __restrict__ loops) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t a = (uint64_t)src[i] ^ key_xor;
    if (a == ((uint64_t)dst[i] ^ key_xor)) {
      atomicOr(&loop_bits[a >> 5], 1u << (a & 31));
      atomicAdd(loops, 1ull);
    }
  }
}


// ---- boundary adjacency of a split window (gs_tri_dist_plan .. _assemble) ----------------------------
// The count share of rank `part` (u in its equal-work range C = [c0, c1)) reads the rows N+(u), u in C,
// and the rows N+(v) of their targets v; rank q built the rows of its route range R_q = [r_q, r_q+1),
// cut at equal shares of the raw work (duplicates included), so R_q is nearly C_q.  So instead of
// every row, a rank fetches the rows of C it did not build (contiguous: one all-to-all whose sizes every
// rank computes from the global d+) and then requests the rows of the targets it holds neither in C nor
// in R (one all-to-all of ids, one of rows).  dp = d+ (u64), pre =
// its exclusive prefix (the window positions of the rows).
struct BdGroups {   // group starts (ids) of up to 64 requesters (+ the end), by value
  uint64_t g[65];
};
// split points of every part: c_q (equal work), r_q (owner ranges), and the window position of each
__global__ void k_bd_bounds(const unsigned long long* __restrict__ prew, const unsigned long long* __restrict__ pre,
                            uint32_t V, RtSplit sp, uint32_t P, unsigned long long* __restrict__ out) {
  const uint32_t q = threadIdx.x;
  if (q > P) return;
  const unsigned long long W = prew[V];
  auto lower = [&](unsigned long long t) {   // first u with prew[u] >= t
    uint32_t a = 0, b = V;
    while (a < b) {
      const uint32_t m = (a + b) >> 1;
      if (prew[m] < t) a = m + 1;
      else b = m;
    }
    return a;
  };
  const uint32_t cq = q == 0 ? 0u : q == P ? V : lower(frac_share(W, q, P));
  const uint32_t rq = sp.s[q];   // the route split: rank q built the rows of [r_q, r_q+1)
  out[q] = cq;
  out[P + 1 + q] = rq;
  out[2 * (P + 1) + q] = pre[cq];
  out[3 * (P + 1) + q] = pre[rq];
}
// targets of the rows of C that this rank holds neither in C nor in R -> bitmap
__global__ __launch_bounds__(256) void k_bd_mark(const uint32_t* __restrict__ crows, uint64_t n, uint32_t c0, uint32_t c1,
                                                 uint32_t r0, uint32_t r1, uint32_t V,
                                                 const unsigned long long* __restrict__ dp, uint32_t* __restrict__ bits,
                                                 uint32_t* __restrict__ bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint32_t v = crows[i];
    if (v >= V) {
      atomicOr(bad, 1u);
      continue;
    }
    // (an empty row needs no request: nothing to intersect with)
    if (v - c0 >= c1 - c0 && v - r0 >= r1 - r0 && dp[v]) atomicOr(&bits[v >> 5], 1u << (v & 31));
  }
}
__global__ __launch_bounds__(256) void k_bd_popc(const uint32_t* __restrict__ bits, uint32_t words,
                                                 uint64_t* __restrict__ cnt) {
  for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < words; w += gridDim.x * 256u) cnt[w] = __popc(bits[w]);
}
// marked ids ascending (so grouped by owner) and their row lengths
__global__ __launch_bounds__(256) void k_bd_ids(const uint32_t* __restrict__ bits, uint32_t words,
                                                const uint64_t* __restrict__ pos, const unsigned long long* __restrict__ dp,
                                                uint32_t* __restrict__ ids, uint64_t* __restrict__ len) {
  for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < words; w += gridDim.x * 256u) {
    uint32_t b = bits[w];
    uint64_t p = pos[w];
    for (; b; b &= b - 1, ++p) {
      const uint32_t v = w * 32u + (uint32_t)__builtin_ctz(b);
      ids[p] = v;
      len[p] = dp[v];
    }
  }
}
// per owner q: the first requested id >= r_q, and the row elements before it
__global__ void k_bd_groups(const uint32_t* __restrict__ ids, uint64_t n, const uint64_t* __restrict__ rowpre,
                            const unsigned long long* __restrict__ bnd, uint32_t P, unsigned long long* __restrict__ out) {
  const uint32_t q = threadIdx.x;
  if (q > P) return;
  const uint64_t rq = bnd[P + 1 + q];
  uint64_t a = 0, b = n;
  while (a < b) {
    const uint64_t m = (a + b) >> 1;
    if (ids[m] < rq) a = m + 1;
    else b = m;
  }
  out[q] = a;
  out[P + 1 + q] = rowpre[a];
}
// row lengths of requested ids (serve): an id outside this rank's route range is a caller error
__global__ __launch_bounds__(256) void k_bd_serve_len(const uint32_t* __restrict__ ids, uint64_t n,
                                                      const unsigned long long* __restrict__ dp, uint32_t r0, uint32_t r1,
                                                      uint64_t* __restrict__ len, uint32_t* __restrict__ bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint32_t v = ids[i];
    const bool ok = v - r0 < r1 - r0;
    len[i] = ok ? dp[v] : 0ull;
    if (!ok) atomicOr(bad, 1u);
  }
}
// copy whole rows, one wave per id: serve (SERVE) from the local rows at pre[v] - base to the packed
// positions pos[i]; assemble from the packed received rows at pos[i] to the window positions pre[v]
template <bool SERVE>
__global__ __launch_bounds__(256) void k_bd_copy(const uint32_t* __restrict__ ids, uint64_t n,
                                                 const unsigned long long* __restrict__ pre, uint64_t base,
                                                 const uint64_t* __restrict__ pos, const unsigned long long* __restrict__ dp,
                                                 uint32_t r0, uint32_t r1, const uint32_t* __restrict__ from,
                                                 uint32_t* __restrict__ to) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; i < n; i += nw) {
    const uint32_t v = ids[i];
    if (SERVE && v - r0 >= r1 - r0) continue;   // flagged by k_bd_serve_len
    const uint64_t d = dp[v];
    const uint64_t s = SERVE ? pre[v] - base : pos[i], t = SERVE ? pos[i] : pre[v];
    for (uint64_t k = lane; k < d; k += 64) to[t + k] = from[s + k];
  }
}
// one value per group start, by value (serve: the element offset of each requester's rows)
__global__ void k_bd_pick(const uint64_t* __restrict__ pos, BdGroups g, uint32_t P, unsigned long long* __restrict__ out) {
  const uint32_t q = threadIdx.x;
  if (q <= P) out[q] = pos[g.g[q]];
}

}  // namespace gs

using namespace gs;

// ---- host side ---------------------------------------------------------------------------------------
namespace {

struct TriGeom {
  const int64_t *src = nullptr, *dst = nullptr;    // ids as counted (relabeled when wider than the budget)
  const int64_t *osrc = nullptr, *odst = nullptr;  // the window's own ids (the self-pair term)
  const int64_t* uniq = nullptr;                   // relabel table (sorted originals), or null
  uint64_t nuniq = 0, n = 0;
  uint32_t B = 1;
  uint64_t key_xor = 0;
  size_t V = 2;
  bool phist_ready = false;   // SM_HIST9 holds the top-8-bit histograms of src / dst at this B (tri_okeys)
};

void set_bits(TriGeom* g, uint32_t B) {
  g->B = B;
  g->V = 1ull << B;
}

// the window's id range -> B and key_xor; ids spanning more than TRI_MAX_BITS are relabeled
// (order-preserving compact IDs; the originals stay for the self-pair term's HashSet order)
gs_status tri_geometry(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, TriGeom* g) {
  char* sm = c->small.as<char>();
  GS_HIP(hipMemsetAsync(sm, 0, SM_TIMEOUT, c->stream));
  GS_HIP(hipMemsetAsync(sm + SM_COUNTERS, 0, SM_BASE - SM_COUNTERS, c->stream));
  // the id range; windows after the first also count the partitioned keys' histograms (tri_okeys) on the way,
  // at the width the previous window had (a miss -- another width -- only costs k_tri_phist's own scan later)
  static const int guess_env = getenv("GS_TRI_PHIST_GUESS") ? atoi(getenv("GS_TRI_PHIST_GUESS")) : 1;   // A/B
  const uint32_t guess = guess_env ? c->tri_guess_B : 0u;
  if (n && guess >= 8 && guess <= TRI_MAX_BITS) {
    GS_HIP(hipMemsetAsync(sm + SM_HIST9, 0, 2 * RADIX * 4, c->stream));
    hipLaunchKernelGGL(k_tri_phist, dim3((unsigned)std::min<uint64_t>((n + 1023) / 1024, 4096)), dim3(256), 0, c->stream,
                       src, dst, n, 0ull, guess - 8, (uint32_t*)(sm + SM_HIST9), (unsigned long long*)(sm + SM_MASK));
    GS_HIP(hipGetLastError());
  } else {
    GS_TRY(launch_keyinfo_all(c, src, dst, n, true));   // the id range (no histograms)
  }
  GS_HIP(hipMemcpyAsync(sm + SM_K0, src, 8, hipMemcpyDeviceToDevice, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small, sm, 16, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t mask = c->host_small[0], k0 = c->host_small[1];
  g->src = g->osrc = src;
  g->dst = g->odst = dst;
  g->n = n;
  set_bits(g, mask ? 64 - __builtin_clzll(mask) : 1);
  g->key_xor = k0 & ~((1ull << g->B) - 1);
  g->phist_ready = n && guess >= 8 && guess == g->B;   // (ids within B bits: (id ^ key_xor) >> (B - 8) = (id >> (B - 8)) & 255)
  if (g->B <= TRI_MAX_BITS) c->tri_guess_B = g->B;
  if (g->B > TRI_MAX_BITS) {
    g->phist_ready = false;
    GS_TRY(relabel_endpoints(c, src, dst, n, &g->src, &g->dst, &g->uniq, &g->nuniq));
    set_bits(g, g->nuniq > 1 ? 64 - __builtin_clzll(g->nuniq - 1) : 1);
    g->key_xor = 0;
    if (g->B > TRI_MAX_BITS)
      return set_error(c, GS_EUNSUPPORTED, "window triangles: %llu distinct vertices (> 2^%llu)",
                       (unsigned long long)g->nuniq, (unsigned long long)TRI_MAX_BITS);
  }
  return GS_OK;
}

// raw degree of every id over this window's (or this rank's) records: the bucket path's COUNT,
// else global atomics
gs_status tri_degrees(gs_ctx* c, const TriGeom& g, uint32_t* deg) {
  GS_HIP(hipMemsetAsync(deg, 0, g.V * 4, c->stream));
  if (g.n == 0) return GS_OK;
  GS_TRY(ensure(c, c->out_keys, std::min<uint64_t>(2 * g.n, g.V) * 8));
  GS_TRY(ensure(c, c->tri_sfx, std::min<uint64_t>(2 * g.n, g.V) * 8));
  uint64_t U = 0;
  const gs_status bs = bucket_reduce(c, g.src, g.dst, nullptr, g.n, DIR_ALL, OP_COUNT, GS_NONE, false, nullptr,
                                     c->out_keys.as<int64_t>(), c->tri_sfx.p, &U);
  if (bs == GS_OK) {
    if (U)
      hipLaunchKernelGGL(k_tri_deg_scatter, dim3((unsigned)std::min<uint64_t>((U + 255) / 256, 8192)), dim3(256), 0,
                         c->stream, c->out_keys.as<int64_t>(), c->tri_sfx.as<int64_t>(), U, g.key_xor, deg);
  } else if (bs == GS_EUNSUPPORTED) {
    hipLaunchKernelGGL(k_tri_deg, dim3((unsigned)std::min<uint64_t>((g.n + DG_BLOCK - 1) / DG_BLOCK, 1024)),
                       dim3(DG_BLOCK), 0, c->stream, g.src, g.dst, g.n, g.key_xor, deg);
  } else {
    return bs;
  }
  return hip_check(c, hipGetLastError(), "degrees");
}

// the degree sample of a large window: TRI_SAMPLE_SLICES contiguous slices spread evenly over the window,
// `per` records each, gathered into out_src / out_dst (a prefix alone misses most hubs of a window whose
// records arrive sorted by source, e.g. a replayed edge list: they would get class 0, the lowest rank,
// and their whole adjacency would become their out-list)
constexpr uint64_t TRI_SAMPLE_SLICES = 16;
__global__ __launch_bounds__(256) void k_tri_sample(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                    uint64_t n, uint64_t per, int64_t* __restrict__ out_src,
                                                    int64_t* __restrict__ out_dst) {
  const uint64_t stride = n / TRI_SAMPLE_SLICES, total = per * TRI_SAMPLE_SLICES;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256) {
    const uint64_t k = i / per, j = i - k * per, at = k * stride + j;
    out_src[i] = src[at];
    out_dst[i] = dst[at];
  }
}

// degree-class ranks; the ids without an edge (class 0) -> host_small[5] after the next wait
gs_status tri_ranks(gs_ctx* c, const TriGeom& g, const uint32_t* deg, uint32_t* rank) {
  const uint32_t rk_tiles = (uint32_t)((g.V + RK_TILE - 1) / RK_TILE);
  GS_TRY(ensure(c, c->tri_tiles, (size_t)rk_tiles * RK_NC * 4 + 8));
  uint32_t* rk_cnt = c->tri_tiles.as<uint32_t>();
  hipLaunchKernelGGL(k_rank_count, dim3(rk_tiles), dim3(RK_BLOCK), 0, c->stream, deg, (uint32_t)g.V, rk_tiles, rk_cnt);
  hipLaunchKernelGGL(k_rank_scan, dim3(1), dim3(1024), 0, c->stream, rk_cnt, rk_tiles * RK_NC);
  hipLaunchKernelGGL(k_rank_scatter, dim3(rk_tiles), dim3(RK_BLOCK), 0, c->stream, deg, (uint32_t)g.V, rk_tiles, rk_cnt,
                     rank);
  GS_HIP(hipGetLastError());
  c->host_small[5] = 0;   // (the copy fills the low 4 bytes)
  GS_HIP(hipMemcpyAsync(c->host_small + 5, rk_cnt + rk_tiles, 4, hipMemcpyDeviceToHost, c->stream));
  return GS_OK;
}

// oriented keys of the ranks into keys[0 .. n) (+ self-loop bitmap; loop count -> host_small[4] after
// the next wait; the digit histograms into SM_HIST)
// useg: histograms of u alone (the segmented sort) when the partitioned form runs -> *seg
gs_status tri_okeys(gs_ctx* c, const TriGeom& g, const uint32_t* rank, uint64_t* keys, bool useg = false,
                    bool* seg = nullptr) {
  if (seg) *seg = false;
  char* sm = c->small.as<char>();
  const size_t words = (g.V + 31) / 32;
  GS_TRY(ensure(c, c->tri_loops, words * 4));
  GS_HIP(hipMemsetAsync(c->tri_loops.p, 0, words * 4, c->stream));
  unsigned long long* d_loops = (unsigned long long*)(sm + SM_NUNIQUE);
  GS_HIP(hipMemsetAsync(d_loops, 0, 8, c->stream));
  GS_HIP(hipMemsetAsync(sm + SM_HIST, 0, 8 * 256 * 4, c->stream));
  static const int split_env = getenv("GS_TRI_OKEYS_SPLIT") ? atoi(getenv("GS_TRI_OKEYS_SPLIT")) : -1;   // A/B
  static const int unroll = getenv("GS_TRI_OKEYS_UNROLL") ? atoi(getenv("GS_TRI_OKEYS_UNROLL")) : 4;     // A/B: 1, 2, 4
  static const int part_env = getenv("GS_TRI_OKEYS_PART") ? atoi(getenv("GS_TRI_OKEYS_PART")) : -1;     // A/B
  const bool split = split_env >= 0 ? split_env != 0 : g.V > (1ull << 25);
  // partitioned on tables past the L2s (s24: 60.7 -> 58.9 ms, s26: 315.6 -> 305.2 ms; profiles/r06/tri/ab_okeys_part/)
  const bool part = g.n && g.n < (1ull << 32) && g.B >= 8 && (part_env >= 0 ? part_env != 0 : g.V > (1ull << 23));
  const int U = unroll >= 4 ? 4 : unroll >= 2 ? 2 : 1;
  const uint64_t steps = (g.n + 256ull * U - 1) / (256ull * U);
  if (part) {   // records partitioned by each endpoint in turn: L2-local rank gathers (TriPartA / TriPartB)
    const uint32_t sh = g.B - 8, R = (uint32_t)g.n, tiles = (R + SORT_TILE - 1) / SORT_TILE;
    uint32_t* ph = (uint32_t*)(sm + SM_HIST9);   // [2][256] partition histograms, then (SM_BASE9) their bases
    uint32_t* pb = (uint32_t*)(sm + SM_BASE9);
    uint32_t* ctr = (uint32_t*)(sm + SM_COUNTERS) + 56;
    GS_HIP(hipMemsetAsync(ctr, 0, 8, c->stream));
    if (!g.phist_ready) {   // (else tri_geometry's id scan counted them, with the width the previous window had)
      GS_HIP(hipMemsetAsync(ph, 0, 2 * RADIX * 4, c->stream));
      hipLaunchKernelGGL(k_tri_phist, dim3((unsigned)std::min<uint64_t>((g.n + 1023) / 1024, 4096)), dim3(256), 0, c->stream,
                         g.src, g.dst, g.n, g.key_xor, sh, ph, nullptr);
    }
    hipLaunchKernelGGL(k_digit_base, dim3(1), dim3(256), 0, c->stream, (const uint32_t*)ph, pb, 2);
    GS_TRY(ensure(c, c->keysA, g.n * 8));
    GS_TRY(ensure(c, c->keysB, g.n * 8));
    GS_TRY(ensure(c, c->sort_status, (size_t)tiles * RADIX * 8, true));
    uint64_t* ka = c->keysA.as<uint64_t>();
    uint64_t* kb = c->keysB.as<uint64_t>();
    const uint32_t ep1 = next_epoch(c, 0);
    hipLaunchKernelGGL((k_onesweep<uint64_t, uint8_t, false, SORT_BLOCK, SORT_ITEMS, TriPartA>), dim3(tiles), dim3(SORT_BLOCK),
                       0, c->stream, TriPartA{g.src, g.dst, g.key_xor}, ka, nullptr, R, 32 + sh, (const uint32_t*)pb,
                       c->sort_status.as<uint64_t>(), ctr, ep1, (uint32_t*)(sm + SM_TIMEOUT));
    const uint32_t ep2 = next_epoch(c, 0);
    hipLaunchKernelGGL((k_onesweep<uint64_t, uint8_t, false, SORT_BLOCK, SORT_ITEMS, TriPartB>), dim3(tiles), dim3(SORT_BLOCK),
                       0, c->stream, TriPartB{ka, rank}, kb, nullptr, R, 32 + sh, (const uint32_t*)pb + RADIX,
                       c->sort_status.as<uint64_t>(), ctr + 1, ep2, (uint32_t*)(sm + SM_TIMEOUT));
    const uint32_t hshift = useg ? g.B : 0u;
    const int nd = (int)((useg ? g.B : 2 * g.B) + 7) / 8;
    // keys per lane per step (A/B, s26 keys + sort: 4 -> 78.7, 8 -> 77.2, 16 -> 76.7 ms; ab_okeys_part/okp_u_*)
    static const int pu_env = getenv("GS_TRI_OKP_U") ? atoi(getenv("GS_TRI_OKP_U")) : 16;
    const int PU = pu_env >= 16 ? 16 : pu_env >= 8 ? 8 : 4;
    const unsigned gp = (unsigned)std::min<uint64_t>((g.n + 256ull * PU - 1) / (256ull * PU), 32768 / PU);
    if (PU == 16)
      hipLaunchKernelGGL(k_tri_okeys_part<16>, dim3(gp), dim3(256), 0, c->stream, kb, g.n, g.B, rank, keys,
                         c->tri_loops.as<uint32_t>(), d_loops, hshift, nd, (uint32_t*)(sm + SM_HIST));
    else if (PU == 8)
      hipLaunchKernelGGL(k_tri_okeys_part<8>, dim3(gp), dim3(256), 0, c->stream, kb, g.n, g.B, rank, keys,
                         c->tri_loops.as<uint32_t>(), d_loops, hshift, nd, (uint32_t*)(sm + SM_HIST));
    else
      hipLaunchKernelGGL(k_tri_okeys_part<4>, dim3(gp), dim3(256), 0, c->stream, kb, g.n, g.B, rank, keys,
                         c->tri_loops.as<uint32_t>(), d_loops, hshift, nd, (uint32_t*)(sm + SM_HIST));
    if (seg) *seg = useg;
    GS_HIP(hipGetLastError());
  } else if (g.n && split) {   // two passes over halves of the rank table (k_tri_okeys_lo / _hi)
    const unsigned glo = (unsigned)std::min<uint64_t>(steps, 16384 / U), ghi = (unsigned)std::min<uint64_t>(steps, 8192 / U);
    const uint32_t H = (uint32_t)(g.V / 2);
    uint32_t* lb = c->tri_loops.as<uint32_t>();
    uint32_t* hs = (uint32_t*)(sm + SM_HIST);
    if (U == 4) {
      hipLaunchKernelGGL(k_tri_okeys_lo<4>, dim3(glo), dim3(256), 0, c->stream, g.src, g.dst, g.n, g.key_xor, H, rank, keys, lb, d_loops);
      hipLaunchKernelGGL(k_tri_okeys_hi<4>, dim3(ghi), dim3(256), 0, c->stream, keys, g.n, g.B, rank, hs);
    } else if (U == 2) {
      hipLaunchKernelGGL(k_tri_okeys_lo<2>, dim3(glo), dim3(256), 0, c->stream, g.src, g.dst, g.n, g.key_xor, H, rank, keys, lb, d_loops);
      hipLaunchKernelGGL(k_tri_okeys_hi<2>, dim3(ghi), dim3(256), 0, c->stream, keys, g.n, g.B, rank, hs);
    } else {
      hipLaunchKernelGGL(k_tri_okeys_lo<1>, dim3(glo), dim3(256), 0, c->stream, g.src, g.dst, g.n, g.key_xor, H, rank, keys, lb, d_loops);
      hipLaunchKernelGGL(k_tri_okeys_hi<1>, dim3(ghi), dim3(256), 0, c->stream, keys, g.n, g.B, rank, hs);
    }
    GS_HIP(hipGetLastError());
  } else if (g.n) {
    const unsigned grid = (unsigned)std::min<uint64_t>(steps, 8192 / U);
    uint32_t* lb = c->tri_loops.as<uint32_t>();
    uint32_t* hs = (uint32_t*)(sm + SM_HIST);
    if (U == 4)
      hipLaunchKernelGGL(k_tri_okeys<4>, dim3(grid), dim3(256), 0, c->stream, g.src, g.dst, g.n, g.key_xor, g.B, rank, keys, lb, d_loops, hs);
    else if (U == 2)
      hipLaunchKernelGGL(k_tri_okeys<2>, dim3(grid), dim3(256), 0, c->stream, g.src, g.dst, g.n, g.key_xor, g.B, rank, keys, lb, d_loops, hs);
    else
      hipLaunchKernelGGL(k_tri_okeys<1>, dim3(grid), dim3(256), 0, c->stream, g.src, g.dst, g.n, g.key_xor, g.B, rank, keys, lb, d_loops, hs);
    GS_HIP(hipGetLastError());
  }
  GS_HIP(hipMemcpyAsync(c->host_small + 4, d_loops, 8, hipMemcpyDeviceToHost, c->stream));
  return GS_OK;
}

// the oriented keys sorted by u alone (LSD passes over bits B .. 2B; tri_okeys counted u's digit histograms),
// then each run of equal u by v (k_tri_segsort, k_tri_segsort_long) -> *out (wide keys, in keysA or keysB)
gs_status tri_seg_sort(gs_ctx* c, const TriGeom& g, const uint64_t* keys, Sorted* out) {
  char* sm = c->small.as<char>();
  const uint64_t n = g.n;
  const uint32_t R = (uint32_t)n, tiles = (R + SORT_TILE - 1) / SORT_TILE;
  const int passes = (int)(g.B + 7) / 8;
  hipLaunchKernelGGL(k_digit_base, dim3(1), dim3(256), 0, c->stream, (const uint32_t*)(sm + SM_HIST), (uint32_t*)(sm + SM_BASE),
                     passes);
  GS_TRY(ensure(c, c->keysA, n * 8));
  GS_TRY(ensure(c, c->keysB, n * 8));
  GS_TRY(ensure(c, c->sort_status, (size_t)tiles * RADIX * 8, true));
  uint64_t* ka = c->keysA.as<uint64_t>();
  uint64_t* kb = c->keysB.as<uint64_t>();
  const uint64_t* src = keys;
  for (int p = 0; p < passes; ++p) {
    GS_HIP(hipMemsetAsync((uint32_t*)(sm + SM_COUNTERS) + p, 0, 4, c->stream));
    const uint32_t ep = next_epoch(c, 0);
    hipLaunchKernelGGL((k_onesweep<uint64_t, uint8_t, false, SORT_BLOCK, SORT_ITEMS, BufSrc<uint64_t, uint8_t>>), dim3(tiles),
                       dim3(SORT_BLOCK), 0, c->stream, BufSrc<uint64_t, uint8_t>{src, nullptr, 0}, ka, nullptr, R,
                       g.B + 8u * (uint32_t)p, (const uint32_t*)(sm + SM_BASE) + p * RADIX, c->sort_status.as<uint64_t>(),
                       (uint32_t*)(sm + SM_COUNTERS) + p, ep, (uint32_t*)(sm + SM_TIMEOUT));
    src = ka;
    std::swap(ka, kb);
  }
  uint64_t* sorted = const_cast<uint64_t*>(src);   // (passes >= 1: B > 16 here)
  uint64_t* tmp = ka;                               // the other buffer
  // runs longer than the LDS chunk: their starts (at most one per k_tri_segsort block) in tri_tiles
  const uint64_t blocks = (n + SS_T - 1) / SS_T;
  GS_TRY(ensure(c, c->tri_tiles, (size_t)(blocks + 1) * 8));
  unsigned long long* d_nlong = (unsigned long long*)(sm + SM_TRI_MERGE);   // (tri_count zeroes it again)
  GS_HIP(hipMemsetAsync(d_nlong, 0, 8, c->stream));
  // GS_TRI_SEGSORT_CAP (tests): a smaller chunk, so more runs take the long kernel's HBM passes
  static const int cap_env = getenv("GS_TRI_SEGSORT_CAP") ? atoi(getenv("GS_TRI_SEGSORT_CAP")) : SS_CAP;
  const uint32_t cap = (uint32_t)std::max(1, std::min(cap_env, SS_CAP));
  hipLaunchKernelGGL(k_tri_segsort, dim3((unsigned)blocks), dim3(SS_BLOCK), 0, c->stream, sorted, n, g.B, cap,
                     c->tri_tiles.as<uint64_t>(), d_nlong);
  hipLaunchKernelGGL(k_tri_segsort_long, dim3(512), dim3(SS_BLOCK), 0, c->stream, sorted, tmp, n, g.B, cap,
                     (const uint64_t*)c->tri_tiles.as<uint64_t>(), (const unsigned long long*)d_nlong);
  GS_HIP(hipGetLastError());
  out->keys = sorted;
  out->vals = nullptr;
  out->wide = true;
  out->bits = 2 * (int)g.B;
  out->passes = passes;
  out->done_passes = passes;
  out->records = n;
  out->key_xor = 0;
  out->payload_bytes = 0;
  return GS_OK;
}

// sort + unique of n oriented keys -> c->out_keys[0 .. M); `sentinel`: the keys may end in self-loop
// sentinels (dropped)
gs_status tri_unique(gs_ctx* c, const uint64_t* keys, uint64_t n, uint32_t B, bool hist_ready, bool sentinel,
                     uint64_t* M, Sorted* s) {
  *M = 0;
  if (n == 0) return GS_OK;
  GS_TRY(sort_buffer(c, keys, nullptr, n, s, 2 * (int)B, 4, hist_ready, hist_ready ? sort_digit_bits(2 * (int)B) : 8));
  hipEventRecord(c->ev[1], c->stream);
  GS_TRY(ensure(c, c->out_keys, n * 8));
  UniqueOut uo{c->out_keys.as<uint64_t>(), nullptr};
  GS_TRY((s->wide ? launch_rbk<uint64_t, CountOp>(c, *s, uo, M) : launch_rbk<uint32_t, CountOp>(c, *s, uo, M)));
  if (sentinel && *M) {   // the self-loop sentinel sorts last
    uint64_t last = 0;
    GS_HIP(hipMemcpy(&last, c->out_keys.as<uint64_t>() + *M - 1, 8, hipMemcpyDeviceToHost));
    const uint64_t sent = (B * 2 >= 64) ? ~0ull : ((1ull << (2 * B)) - 1);
    if (last == sent) *M -= 1;
  }
  return GS_OK;
}

// the transposed sort of the whole window's M out-list entries by target, its first pass reading the out-lists
// (TriTpaySrc) with the digit histograms k_tri_uo_count counted -> *t (u32 keys, u64 payload (p + 1, end))
gs_status tri_tsort_fused(gs_ctx* c, uint32_t B, uint64_t M, const uint32_t* nbr, const uint32_t* rowid,
                          const uint2* out_range, Sorted* t) {
  char* sm = c->small.as<char>();
  const uint32_t R = (uint32_t)M, tiles = (R + SORT_TILE - 1) / SORT_TILE;
  const int passes = (int)(B + 7) / 8;
  hipLaunchKernelGGL(k_digit_base, dim3(1), dim3(256), 0, c->stream, (const uint32_t*)(sm + SM_HIST), (uint32_t*)(sm + SM_BASE),
                     passes);
  GS_TRY(ensure(c, c->keysA, M * 4));
  GS_TRY(ensure(c, c->keysB, M * 4));
  GS_TRY(ensure(c, c->valsA, M * 8));
  GS_TRY(ensure(c, c->valsB, M * 8));
  GS_TRY(ensure(c, c->sort_status, (size_t)tiles * RADIX * 8, true));
  uint32_t *ka = c->keysA.as<uint32_t>(), *kb = c->keysB.as<uint32_t>();
  uint64_t *va = c->valsA.as<uint64_t>(), *vb = c->valsB.as<uint64_t>();
  for (int p = 0; p < passes; ++p) {
    GS_HIP(hipMemsetAsync((uint32_t*)(sm + SM_COUNTERS) + p, 0, 4, c->stream));
    const uint32_t ep = next_epoch(c, 0);
    const uint32_t* base = (const uint32_t*)(sm + SM_BASE) + p * RADIX;
    uint32_t* ctr = (uint32_t*)(sm + SM_COUNTERS) + p;
    if (p == 0)
      hipLaunchKernelGGL((k_onesweep<uint32_t, uint64_t, true, SORT_BLOCK, SORT_ITEMS, TriTpaySrc>), dim3(tiles), dim3(SORT_BLOCK),
                         0, c->stream, TriTpaySrc{nbr, rowid, out_range}, ka, va, R, 0u, base, c->sort_status.as<uint64_t>(),
                         ctr, ep, (uint32_t*)(sm + SM_TIMEOUT));
    else
      hipLaunchKernelGGL((k_onesweep<uint32_t, uint64_t, true, SORT_BLOCK, SORT_ITEMS, BufSrc<uint32_t, uint64_t>>), dim3(tiles),
                         dim3(SORT_BLOCK), 0, c->stream, BufSrc<uint32_t, uint64_t>{kb, vb, 0}, ka, va, R, 8u * (uint32_t)p, base,
                         c->sort_status.as<uint64_t>(), ctr, ep, (uint32_t*)(sm + SM_TIMEOUT));
    std::swap(ka, kb);   // the pass's output is now kb / vb
    std::swap(va, vb);
  }
  GS_HIP(hipGetLastError());
  *t = Sorted{};
  t->keys = kb;
  t->vals = vb;
  t->bits = (int)B;
  t->passes = t->done_passes = passes;
  t->records = M;
  t->payload_bytes = 8;
  return GS_OK;
}

// The counting step over the out-lists (nbr, out_range; M edges) for part `part` of nparts: its
// balanced u-range's edges sorted by target (in-lists with suffix ranges), then the LDS hash-set
// kernels.  okeys: the sorted unique keys (row of every position), else rows come from out_range.
gs_status tri_count(gs_ctx* c, uint32_t B, size_t V, uint64_t M, const uint32_t* nbr, const uint2* out_range,
                    const uint64_t* okeys, uint32_t part, uint32_t nparts, uint64_t* T, uint64_t* probes,
                    const uint32_t* loops = nullptr, const uint32_t* rank = nullptr, uint64_t* active = nullptr,
                    const uint32_t* rowid_all = nullptr, bool tpay_fused = false) {
  char* sm = c->small.as<char>();
  *T = 0;
  *probes = 0;
  uint32_t u0 = 0, u1 = (uint32_t)V, p0 = 0, p1 = (uint32_t)M;
  if (nparts > 1) {
    GS_TRY(ensure(c, c->tri_hwork, (V * 2 + 2) * 8));
    unsigned long long* work = c->tri_hwork.as<unsigned long long>();
    const unsigned gv = (unsigned)std::min<uint64_t>((V + 255) / 256, 16384);
    hipLaunchKernelGGL(k_tri_work, dim3(gv), dim3(256), 0, c->stream, out_range, (uint32_t)V, work);
    GS_TRY(xscan(c, (const uint64_t*)work, V, (uint64_t*)work + V + 1));
    uint32_t* bnd = (uint32_t*)(sm + SM_TABLE);
    hipLaunchKernelGGL(k_tri_bounds, dim3(1), dim3(64), 0, c->stream, (const unsigned long long*)work + V + 1,
                       (uint32_t)V, out_range, okeys, B, (uint32_t)M, part, nparts, bnd);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(c->host_small + 12, bnd, 16, hipMemcpyDeviceToHost, c->stream));
    GS_TRY(host_wait(c));
    const uint32_t* hb = reinterpret_cast<const uint32_t*>(c->host_small + 12);
    u0 = hb[0];
    u1 = hb[1];
    p0 = hb[2];
    p1 = hb[3];
  }
  const uint64_t Ms = p1 - p0;   // this part's edges
  if (Ms == 0) {
    hipEventRecord(c->ev[4], c->stream);
    hipEventRecord(c->ev[5], c->stream);
    hipEventRecord(c->ev[3], c->stream);
    return GS_OK;
  }
  // 1. this part's edges by target: keys v, payload the suffix of N+(u) past v
  const unsigned ge = (unsigned)std::min<uint64_t>((Ms + 255) / 256, 16384);
  Sorted t;
  if (tpay_fused && rowid_all && nparts == 1) {   // the first pass reads the out-lists (TriTpaySrc; histograms: uo_count)
    GS_TRY(tri_tsort_fused(c, B, Ms, nbr, rowid_all, out_range, &t));
  } else {
  GS_TRY(ensure(c, c->aux, Ms * 8));
  GS_TRY(ensure(c, c->tri_sfx, Ms * 8));
  GS_HIP(hipMemsetAsync(sm + SM_HIST, 0, 8 * 256 * 4, c->stream));
  if (okeys) {
    hipLaunchKernelGGL(k_tri_tpay<false>, dim3(ge), dim3(256), 0, c->stream, okeys, nullptr, nbr, p0, p1, B, out_range,
                       c->aux.as<uint64_t>(), c->tri_sfx.as<uint2>(), (uint32_t*)(sm + SM_HIST));
  } else if (rowid_all) {   // the row of every position, written with the out-lists (k_tri_uo_write)
    hipLaunchKernelGGL(k_tri_tpay<true>, dim3(ge), dim3(256), 0, c->stream, nullptr, rowid_all + p0, nbr, p0, p1, B,
                       out_range, c->aux.as<uint64_t>(), c->tri_sfx.as<uint2>(), (uint32_t*)(sm + SM_HIST));
  } else {
    GS_TRY(ensure(c, c->tri_queue, Ms * 4));
    hipLaunchKernelGGL(k_tri_rowid, dim3((unsigned)std::min<uint64_t>((u1 - u0 + 255) / 256, 16384)), dim3(256), 0,
                       c->stream, out_range, u0, u1, p0, c->tri_queue.as<uint32_t>());
    hipLaunchKernelGGL(k_tri_tpay<true>, dim3(ge), dim3(256), 0, c->stream, nullptr, c->tri_queue.as<uint32_t>(), nbr,
                       p0, p1, B, out_range, c->aux.as<uint64_t>(), c->tri_sfx.as<uint2>(), (uint32_t*)(sm + SM_HIST));
  }
  GS_HIP(hipGetLastError());
  GS_TRY(sort_buffer(c, c->aux.as<uint64_t>(), c->tri_sfx.p, Ms, &t, (int)B, 8, true, sort_digit_bits((int)B)));
  }
  if (t.wide || t.key_xor) return set_error(c, GS_EDEVICE, "window triangles: transposed keys wider than 32 bits");
  const uint2* sfx = (const uint2*)t.vals;   // the sort's payload buffer (valsA / valsB): read-only from here
  uint2* in_range = const_cast<uint2*>(out_range) + V;
  GS_HIP(hipMemsetAsync(in_range, 0, V * 8, c->stream));
  hipLaunchKernelGGL(k_tri_in, dim3(ge), dim3(256), 0, c->stream, (const uint32_t*)t.keys, (uint32_t)Ms,
                     reinterpret_cast<uint32_t*>(in_range));
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[4], c->stream);
  // 2. intersections: vertex-centric LDS hash sets (k_tri_light), long out-lists in k_tri_heavy
  // (A/B of round 4, not kept: the light chunks in the heavy items' phase order, s24 light 7.1 -> 36 ms,
  // s26 42 -> 147 ms, profiles/r04/evidence/tri_*_lph.json)
  GS_TRY(ensure(c, c->tri_heavy, (V + Ms / TH_VCH + 64) * 8));   // (v, in-chunk) items
  GS_TRY(ensure(c, c->tri_queue, (std::min<uint64_t>(V, Ms) + Ms / TH_LCH + 64) * 8));   // light chunks
  unsigned long long* d_total = (unsigned long long*)(sm + SM_NUNIQUE);
  uint32_t* d_nheavy = (uint32_t*)(sm + SM_COUNTERS) + 62;
  unsigned long long* d_probes = (unsigned long long*)(sm + SM_TRI_PROBES);
  GS_HIP(hipMemsetAsync(d_total, 0, 8, c->stream));
  GS_HIP(hipMemsetAsync(d_probes, 0, 8, c->stream));
  GS_HIP(hipMemsetAsync(d_nheavy, 0, 8, c->stream));   // heavy items, queued chunks
  unsigned long long* d_active = active ? (unsigned long long*)(sm + SM_TRI_NV) : nullptr;
  if (d_active) GS_HIP(hipMemsetAsync(d_active, 0, 8, c->stream));
  uint32_t* d_err = (uint32_t*)(sm + SM_DEV_ERR);
  GS_HIP(hipMemsetAsync(d_err, 0, 4, c->stream));
  auto* d_merge = (unsigned long long*)(sm + SM_TRI_MERGE);
  GS_HIP(hipMemsetAsync(d_merge, 0, 8, c->stream));
  // LDS hash-set bucket cap: unlimited, or one bucket under GS_FLAG_TEST_TINY_TABLES (tests only)
  const uint32_t nb_cap = (c->flags & GS_FLAG_TEST_TINY_TABLES) ? 1u : 0xFFFFFFFFu;
  uint32_t* d_nqueue = d_nheavy + 1;
  uint2* queue = c->tri_queue.as<uint2>();
  hipLaunchKernelGGL(k_tri_lclass, dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((V + TH_LCBLOCK - 1) / TH_LCBLOCK,
                                                                                        4194304 / TH_LCBLOCK))),
                     dim3(TH_LCBLOCK), 0, c->stream, nbr, out_range, in_range, (uint32_t)V, 0u, 0xFFFFFFFFu, nb_cap, queue,
                     d_nqueue, c->tri_heavy.as<uint2>(), d_nheavy, d_active, d_merge);
  if (d_active && loops && rank) {
    const uint32_t words = (uint32_t)((V + 31) / 32);
    hipLaunchKernelGGL(k_tri_loop_only, dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((words + 255) / 256, 4096))),
                       dim3(256), 0, c->stream, loops, words, rank, out_range, in_range, d_active);
  }
  hipLaunchKernelGGL(k_tri_light, dim3(8192u), dim3(TH_BLOCK), 0, c->stream, nbr, sfx, out_range, in_range, queue,
                     d_nqueue, d_total, d_probes, nb_cap, d_err);
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[5], c->stream);
  // heavy items: work per item, exclusive scan, then equal-work runs per block
  c->host_small[6] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 6, d_nheavy, 4, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint32_t nh = (uint32_t)c->host_small[6];
  if (nh && GS_TH_PHASED) {   // items in phase order, claimed one at a time
    GS_TRY(ensure(c, c->tri_hwork, (size_t)nh * 4 + (TH_PHASES + 64) * 4));
    uint32_t* hist = c->tri_hwork.as<uint32_t>();
    uint32_t* claim = hist + TH_PHASES;
    uint32_t* order = hist + TH_PHASES + 64;
    GS_HIP(hipMemsetAsync(hist, 0, (TH_PHASES + 1) * 4, c->stream));
    const unsigned g = (unsigned)std::min<uint64_t>((nh + 255) / 256, 4096);
    hipLaunchKernelGGL(k_tri_hphase_count<TH_VCH>, dim3(g), dim3(256), 0, c->stream, sfx, in_range, c->tri_heavy.as<uint2>(),
                       nh, (uint32_t)M, hist);
    hipLaunchKernelGGL(k_tri_hphase_scan, dim3(1), dim3(256), 0, c->stream, hist);
    hipLaunchKernelGGL(k_tri_hphase_place<TH_VCH>, dim3(g), dim3(256), 0, c->stream, sfx, in_range, c->tri_heavy.as<uint2>(),
                       nh, (uint32_t)M, hist, order);
    hipLaunchKernelGGL(k_tri_heavy, dim3(GS_TH_HGRID), dim3(TH_HBLOCK), 0, c->stream, nbr, sfx, out_range, in_range,
                       c->tri_heavy.as<uint2>(), d_nheavy, nullptr, (const uint32_t*)order, claim, d_total, d_probes,
                       nb_cap, d_err);
    GS_HIP(hipGetLastError());
  } else if (nh) {
    GS_TRY(ensure(c, c->tri_hwork, (size_t)nh * 16 + 8));
    unsigned long long* hw = c->tri_hwork.as<unsigned long long>();
    hipLaunchKernelGGL(k_tri_hwork, dim3((unsigned)std::min<uint64_t>((nh + 3) / 4, 16384)), dim3(256), 0, c->stream,
                       sfx, in_range, c->tri_heavy.as<uint2>(), nh, hw);
    GS_HIP(hipGetLastError());
    GS_TRY(xscan(c, (const uint64_t*)hw, nh, (uint64_t*)hw + nh));
    hipLaunchKernelGGL(k_tri_heavy, dim3(GS_TH_HGRID), dim3(TH_HBLOCK), 0, c->stream, nbr, sfx, out_range, in_range,
                       c->tri_heavy.as<uint2>(), d_nheavy, (const unsigned long long*)hw + nh, nullptr, nullptr,
                       d_total, d_probes, nb_cap, d_err);
    GS_HIP(hipGetLastError());
  }
  hipEventRecord(c->ev[3], c->stream);
  GS_HIP(hipMemcpyAsync(c->host_small, sm, 32, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small + 6, d_probes, 8, hipMemcpyDeviceToHost, c->stream));
  c->host_small[7] = 0;   // (the copy below fills the low 4 bytes)
  GS_HIP(hipMemcpyAsync(c->host_small + 7, d_err, 4, hipMemcpyDeviceToHost, c->stream));
  if (d_active) GS_HIP(hipMemcpyAsync(c->host_small + 9, d_active, 8, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small + 10, d_merge, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if (active) *active = c->host_small[9];
  c->tri_merge = c->host_small[10];
  if ((uint32_t)c->host_small[3] != 0) return set_error(c, GS_EDEVICE, "look-back spin timed out");
  if ((uint32_t)c->host_small[7] & GS_DERR_TABLE_FULL)
    return set_error(c, GS_EDEVICE, "window triangles: an LDS hash set filled up (counting aborted)");
  *T = c->host_small[2];
  *probes = c->host_small[6];
  return GS_OK;
}

void tri_times(gs_ctx* c, const TriGeom& g, uint64_t M, uint64_t nv, uint64_t probes, int passes) {
  // stage times (path 3): ranks + keys + sort, unique, out-lists + transposed sort, light, heavy
  gs_stage_times& t = c->times;
  t = gs_stage_times{};
  const int order[6] = {0, 1, 2, 4, 5, 3};
  for (int i = 0; i < 5; ++i) t.pass_ms[i] = event_ms(c->ev[order[i]], c->ev[order[i + 1]]);
  t.total_ms = event_ms(c->ev[0], c->ev[3]);
  t.sort_passes = (uint32_t)passes;
  t.key_bits = g.B;
  t.records = M;     // unique undirected edges
  t.vertices = nv;   // vertices with edges
  t.partials = probes;
  t.escapes = c->tri_merge;
  t.path = 3;
}

// the whole window on this GPU; part / nparts: count only that share of the work
gs_status triangles_impl(gs_ctx* c, const gs_edge_batch* b, uint32_t part, uint32_t nparts, uint64_t* count) {
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
  TriGeom g;
  GS_TRY(tri_geometry(c, src, dst, b->n, &g));
  // 1. raw degrees -> degree-class ranks -> oriented composite keys of the ranks
  GS_TRY(ensure(c, c->out_a, g.V * 4));
  GS_TRY(ensure(c, c->out_b, g.V * 4));
  uint32_t* deg = c->out_a.as<uint32_t>();
  uint32_t* rank = c->out_b.as<uint32_t>();
  // The orientation needs only SOME total order of the ids (any order gives the exact count: each
  // triangle is counted once, at its lowest-ranked vertex); the degree classes keep the out-lists short.
  // A large window's classes come from the degrees of n / 4 of its edges, in 16 slices spread over the
  // window (round 4 took the first n / 4: R-MAT s26 ranks + keys + sort 98.2 -> 86.5 ms, count +0.9 ms,
  // window 329.0 -> 318.4 ms; s24 62.6 -> 61.3 ms, same box; profiles/r04/evidence/deg_sample/; a prefix
  // misses the hubs of a source-sorted window); the vertices-with-edges figure then comes from the count's
  // vertex pass (k_tri_lclass, k_tri_loop_only).  GS_TRI_DEG_SAMPLE = k overrides the 4 (1 = exact
  // degrees).  The split-window steps (gs_tri_dist_*) keep exact, all-reduced degrees.
  static const int deg_sample_env = getenv("GS_TRI_DEG_SAMPLE") ? atoi(getenv("GS_TRI_DEG_SAMPLE")) : 4;
  const uint64_t ds = deg_sample_env > 1 ? (uint64_t)deg_sample_env : 1;
  const bool sampled = ds > 1 && nparts == 1 && g.n >= (1ull << 26);
  {
    TriGeom gd = g;
    if (sampled) {   // n / ds records in TRI_SAMPLE_SLICES slices spread over the window (c->aux: the keys later)
      const uint64_t per = g.n / ds / TRI_SAMPLE_SLICES;
      GS_TRY(ensure(c, c->aux, g.n * 8));
      int64_t* ss = c->aux.as<int64_t>();
      hipLaunchKernelGGL(k_tri_sample, dim3(8192), dim3(256), 0, c->stream, g.src, g.dst, g.n, per, ss,
                         ss + per * TRI_SAMPLE_SLICES);
      GS_HIP(hipGetLastError());
      gd.src = ss;
      gd.dst = ss + per * TRI_SAMPLE_SLICES;
      gd.n = per * TRI_SAMPLE_SLICES;
    }
    GS_TRY(tri_degrees(c, gd, deg));
  }
  GS_TRY(tri_ranks(c, g, deg, rank));
  static const int uo_env = getenv("GS_TRI_FUSED_UNIQUE") ? atoi(getenv("GS_TRI_FUSED_UNIQUE")) : 1;   // A/B
  const bool fused = uo_env != 0 && 2 * g.B > 32;   // wide (u64) sorted keys
  // the segmented sort (with the partitioned keys): u-only LSD passes + each out-list sorted in LDS.  Off by
  // default: 3 passes fewer, but the LDS sort of the runs cost more than they did (s26 keys + sort 79.5 -> 98.3 ms,
  // s24 16.8 -> 21.5 ms; profiles/r06/tri/ab_segsort/).  GS_TRI_SEGSORT=1 turns it on (A/B).
  static const int seg_env = getenv("GS_TRI_SEGSORT") ? atoi(getenv("GS_TRI_SEGSORT")) : 0;
  bool seg = false;
  GS_TRY(ensure(c, c->aux, g.n * 8));
  GS_TRY(tri_okeys(c, g, rank, c->aux.as<uint64_t>(), fused && seg_env != 0 && g.B > 16, &seg));
  // 2. sort + unique -> the simple oriented graph, sorted by (u, v); 3. out-lists
  Sorted s;
  uint64_t M = 0;
  const uint32_t* rowid_all = nullptr;
  bool tpay_fused = false;
  uint2* out_range = nullptr;
  uint64_t loops = 0, nv = 0;
  if (fused) {
    if (seg) GS_TRY(tri_seg_sort(c, g, c->aux.as<uint64_t>(), &s));
    else GS_TRY(sort_buffer(c, c->aux.as<uint64_t>(), nullptr, g.n, &s, 2 * (int)g.B, 4, true, sort_digit_bits(2 * (int)g.B)));
    if (!s.wide) return set_error(c, GS_EDEVICE, "window triangles: oriented keys narrower than expected");
    hipEventRecord(c->ev[1], c->stream);
    const uint64_t* sk = static_cast<const uint64_t*>(s.keys);
    const uint64_t sent = (g.B * 2 >= 64) ? ~0ull : ((1ull << (2 * g.B)) - 1);
    const uint64_t tiles = (g.n + UO_TILE - 1) / UO_TILE;
    GS_TRY(ensure(c, c->tri_tiles, (size_t)(2 * tiles + 2) * 8));
    unsigned long long* tcnt = c->tri_tiles.as<unsigned long long>();
    unsigned long long* tpre = tcnt + tiles + 1;
    // (the whole window's count: the transposed sort's histograms on the way, for tri_count's fused first pass)
    static const int tfuse_env = getenv("GS_TRI_TPAY_FUSED") ? atoi(getenv("GS_TRI_TPAY_FUSED")) : 1;   // A/B
    tpay_fused = tfuse_env != 0 && nparts == 1;
    char* sm = c->small.as<char>();
    if (tpay_fused) GS_HIP(hipMemsetAsync(sm + SM_HIST, 0, 8 * 256 * 4, c->stream));
    hipLaunchKernelGGL(k_tri_uo_count, dim3((unsigned)std::min<uint64_t>(tiles, 2048)), dim3(UO_BLOCK), 0, c->stream, sk, g.n,
                       sent, tiles, tcnt, g.B, tpay_fused ? (uint32_t*)(sm + SM_HIST) : nullptr);
    GS_HIP(hipGetLastError());
    GS_TRY(xscan(c, (const uint64_t*)tcnt, tiles, (uint64_t*)tpre));
    GS_HIP(hipMemcpyAsync(c->host_small + 10, tpre + tiles, 8, hipMemcpyDeviceToHost, c->stream));
    GS_TRY(host_wait(c));
    M = c->host_small[10];
    loops = c->host_small[4];
    nv = g.V - (uint32_t)c->host_small[5];
    if (M >= (1ull << 32)) return set_error(c, GS_EINVAL, "window triangles: %llu unique edges (limit 2^32 - 1)",
                                            (unsigned long long)M);
    GS_TRY(ensure(c, c->tri_range, g.V * 16));
    GS_TRY(ensure(c, c->tri_nbr, M * 4 + 4));
    GS_TRY(ensure(c, c->out_keys, M * 4 + 4));
    out_range = reinterpret_cast<uint2*>(c->tri_range.p);
    GS_HIP(hipMemsetAsync(out_range, 0, g.V * 8, c->stream));
    hipLaunchKernelGGL(k_tri_uo_write, dim3((unsigned)tiles), dim3(UO_BLOCK), 0, c->stream, sk, g.n, sent, g.B,
                       (const unsigned long long*)tpre, c->tri_nbr.as<uint32_t>(), c->out_keys.as<uint32_t>(),
                       reinterpret_cast<uint32_t*>(out_range));
    GS_HIP(hipGetLastError());
    rowid_all = c->out_keys.as<uint32_t>();
    hipEventRecord(c->ev[2], c->stream);
  } else {
    GS_TRY(tri_unique(c, c->aux.as<uint64_t>(), g.n, g.B, true, false, &M, &s));
    loops = c->host_small[4];
    nv = g.V - (uint32_t)c->host_small[5];
    hipEventRecord(c->ev[2], c->stream);
    if (loops) M -= 1;   // the self-loop sentinel sorts last
    if (M) {
      GS_TRY(ensure(c, c->tri_range, g.V * 16));
      GS_TRY(ensure(c, c->tri_nbr, M * 4));
      out_range = reinterpret_cast<uint2*>(c->tri_range.p);
      GS_HIP(hipMemsetAsync(out_range, 0, g.V * 8, c->stream));
      hipLaunchKernelGGL(k_tri_out, dim3((unsigned)std::min<uint64_t>((M + 255) / 256, 16384)), dim3(256), 0,
                         c->stream, c->out_keys.as<uint64_t>(), (uint32_t)M, g.B, c->tri_nbr.as<uint32_t>(),
                         reinterpret_cast<uint32_t*>(out_range));
      GS_HIP(hipGetLastError());
    }
  }
  uint64_t T = 0, probes = 0;
  if (M) {
    // 4. the count
    uint64_t active = 0;
    GS_TRY(tri_count(c, g.B, g.V, M, c->tri_nbr.as<uint32_t>(), out_range, fused ? nullptr : c->out_keys.as<uint64_t>(),
                     part, nparts, &T, &probes, c->tri_loops.as<uint32_t>(), rank, sampled ? &active : nullptr,
                     rowid_all, tpay_fused));
    tri_times(c, g, M, sampled ? active : nv, probes, s.passes);
  }
  if (loops && part == 0) {   // self-pair candidates (x, x, true) matched by a self-loop on x (:105)
    uint64_t S = 0;
    GS_TRY(triangle_selfpair_term(c, g.osrc, g.odst, g.n, c->tri_loops.as<uint32_t>(), g.key_xor, g.uniq, g.nuniq, &S));
    T += S;
  }
  *count = T;
  return GS_OK;
}

// ---- the split window (gs_tri_dist_*) -------------------------------------------------------------
// geometry from the ranks' common id range (no relabel: a split window must span <= 2^28 ids)
gs_status tri_geometry_range(gs_ctx* c, int64_t gmin, int64_t gmax, TriGeom* g) {
  if (gmin > gmax) {   // no record anywhere
    set_bits(g, 1);
    g->key_xor = 0;
    return GS_OK;
  }
  const uint64_t d = (uint64_t)gmin ^ (uint64_t)gmax;
  set_bits(g, d ? 64 - __builtin_clzll(d) : 1);
  if (g->B > TRI_MAX_BITS)
    return set_error(c, GS_EUNSUPPORTED, "split window triangles: ids span more than 2^%llu values",
                     (unsigned long long)TRI_MAX_BITS);
  g->key_xor = (uint64_t)gmin & ~((1ull << g->B) - 1);
  return GS_OK;
}

gs_status dist_stage(gs_ctx* c, const gs_edge_batch* b, TriGeom* g) {
  // (the stage timings of the bucket / sort passes inside start at ev[0])
  hipEventRecord(c->ev[0], c->stream);
  const int64_t *src = nullptr, *dst = nullptr;
  const void* val;
  if (b->n) GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  g->src = g->osrc = src;
  g->dst = g->odst = dst;
  g->n = b->n;
  set_bits(g, c->tri_B ? c->tri_B : 1);
  g->key_xor = c->tri_key_xor;
  return GS_OK;
}

// Split window over ids that span more than 2^TRI_MAX_BITS values (any Long key,
// SimpleEdgeStream.java:173-183): every rank relabels its records to ranks among the WHOLE window's
// sorted distinct ids -- its own distinct ids (relabel_endpoints), all-gathered, relabeled again on every
// rank (the same G everywhere), then each local id searched in G once.  Order-preserving, as the
// single-GPU relabel (tri_geometry), so the orientation ties and the count are unchanged.  *lb: this
// rank's compact columns (device, the ctx's tri_rl), *vmax = |G| - 1.
gs_status tri_dist_relabel(gs_ctx* c, const gs_edge_batch* b, gs_edge_batch* lb, int64_t* vmax) {
  const uint32_t P = (uint32_t)c->comm_size;
  const uint64_t n = b->n;
  uint64_t nloc = 0;
  gs_status st = GS_OK;
  if (n) {
    const int64_t *src = nullptr, *dst = nullptr, *ca = nullptr, *cb = nullptr, *uq = nullptr;
    const void* val;
    st = stage_batch(c, b, &src, &dst, &val, false);
    if (st == GS_OK) st = relabel_endpoints(c, src, dst, n, &ca, &cb, &uq, &nloc);
    if (st == GS_OK) st = ensure(c, c->tri_rl[0], n * 8 + 8);
    if (st == GS_OK) st = ensure(c, c->tri_rl[1], n * 8 + 8);
    if (st == GS_OK) st = ensure(c, c->tri_rl[2], nloc * 8 + 8);
    if (st == GS_OK) st = hip_check(c, hipMemcpyAsync(c->tri_rl[0].p, ca, n * 8, hipMemcpyDeviceToDevice, c->stream), "relabel");
    if (st == GS_OK) st = hip_check(c, hipMemcpyAsync(c->tri_rl[1].p, cb, n * 8, hipMemcpyDeviceToDevice, c->stream), "relabel");
    if (st == GS_OK) st = hip_check(c, hipMemcpyAsync(c->tri_rl[2].p, uq, nloc * 8, hipMemcpyDeviceToDevice, c->stream), "relabel");
  }
  GS_TRY(comm_agree(c, st));
  std::vector<uint64_t> cnt(P);
  GS_TRY(comm_allgather_u64(c, nloc, cnt.data()));
  uint64_t T = 0;
  for (uint32_t p = 0; p < P; ++p) T += cnt[p];
  GS_TRY(ensure(c, c->tri_rl[3], T * 8 + 8));
  GS_TRY(comm_allgatherv(c, c->tri_rl[2].p, c->tri_rl[3].as<char>(), cnt.data(), 8));
  const int64_t *ga = nullptr, *gb = nullptr, *G = nullptr;
  uint64_t ng = 0;
  st = T ? relabel_endpoints(c, c->tri_rl[3].as<int64_t>(), c->tri_rl[3].as<int64_t>(), T, &ga, &gb, &G, &ng) : GS_OK;
  if (st == GS_OK && ng > (1ull << TRI_MAX_BITS))
    st = set_error(c, GS_EUNSUPPORTED, "split window triangles: %llu distinct vertices (> 2^%llu)", (unsigned long long)ng,
                   (unsigned long long)TRI_MAX_BITS);
  // (the gathered ids are consumed: tri_rl[3] holds the map)
  if (st == GS_OK && n)
    st = relabel_to_global(c, c->tri_rl[2].as<int64_t>(), nloc, G, ng, c->tri_rl[3].as<uint32_t>(), c->tri_rl[0].as<int64_t>(),
                           c->tri_rl[1].as<int64_t>(), n);
  GS_TRY(comm_agree(c, st));
  *lb = gs_edge_batch{c->tri_rl[0].as<int64_t>(), c->tri_rl[1].as<int64_t>(), nullptr, n, GS_NONE, GS_MEM_DEVICE, 0};
  *vmax = ng ? (int64_t)ng - 1 : 0;
  return GS_OK;
}

}  // namespace

extern "C" {

gs_status gs_tri_dist_range(gs_ctx* c, const gs_edge_batch* b, int64_t* minmax) {
  if (!c) return GS_EINVAL;
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!minmax) return set_error(c, GS_EINVAL, "null output pointer");
  GS_TRY(begin_call(c));
  minmax[0] = INT64_MAX;
  minmax[1] = INT64_MIN;
  if (b->n == 0) return GS_OK;
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  long long* mm = (long long*)(c->small.as<char>() + SM_TABLE);
  c->host_small[12] = (uint64_t)INT64_MAX;
  c->host_small[13] = (uint64_t)INT64_MIN;
  GS_HIP(hipMemcpyAsync(mm, c->host_small + 12, 16, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_tri_minmax, dim3((unsigned)std::min<uint64_t>((b->n + 255) / 256, 4096)), dim3(256), 0, c->stream,
                     src, dst, b->n, mm);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 12, mm, 16, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  minmax[0] = (int64_t)c->host_small[12];
  minmax[1] = (int64_t)c->host_small[13];
  return GS_OK;
}

gs_status gs_tri_dist_degrees(gs_ctx* c, const gs_edge_batch* b, int64_t gmin, int64_t gmax, uint32_t* deg, uint64_t* V) {
  if (!c) return GS_EINVAL;
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!V) return set_error(c, GS_EINVAL, "null output pointer");
  TriGeom g;
  GS_TRY(tri_geometry_range(c, gmin, gmax, &g));
  *V = g.V;
  c->tri_B = g.B;
  c->tri_key_xor = g.key_xor;
  if (!deg) return GS_OK;   // the query: V only
  GS_TRY(begin_call(c));
  GS_TRY(dist_stage(c, b, &g));
  GS_TRY(tri_degrees(c, g, deg));
  return host_wait(c);
}

gs_status gs_tri_dist_orient(gs_ctx* c, const gs_edge_batch* b, const uint32_t* deg, uint32_t* dout, uint64_t* loops) {
  if (!c) return GS_EINVAL;
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!deg || !dout || !loops) return set_error(c, GS_EINVAL, "null pointer");
  if (!c->tri_B) return set_error(c, GS_EINVAL, "gs_tri_dist_degrees first (the window's id geometry)");
  GS_TRY(begin_call(c));
  c->rt_n = ~0ull;
  TriGeom g;
  GS_TRY(dist_stage(c, b, &g));
  GS_TRY(ensure(c, c->out_b, g.V * 4));
  uint32_t* rank = c->out_b.as<uint32_t>();
  GS_TRY(tri_ranks(c, g, deg, rank));
  GS_TRY(ensure(c, c->aux, g.n * 8 + 8));
  GS_TRY(tri_okeys(c, g, rank, c->aux.as<uint64_t>()));
  GS_HIP(hipMemsetAsync(dout, 0, g.V * 4, c->stream));
  if (g.n)
    hipLaunchKernelGGL(k_tri_dout, dim3((unsigned)std::min<uint64_t>((g.n + 255) / 256, 16384)), dim3(256), 0, c->stream,
                       c->aux.as<uint64_t>(), g.n, g.B, dout);
  GS_HIP(hipGetLastError());
  GS_TRY(host_wait(c));
  *loops = c->host_small[4];
  c->rt_n = g.n;   // the oriented keys wait in c->aux for gs_tri_dist_route
  c->rt_seq = c->call_seq;
  return GS_OK;
}

gs_status gs_tri_dist_route(gs_ctx* c, const uint32_t* dout, uint32_t nparts, uint64_t* keys_out, uint64_t* counts) {
  if (!c) return GS_EINVAL;
  if (!dout || !counts) return set_error(c, GS_EINVAL, "null pointer");
  if (nparts < 1 || nparts > (uint32_t)RT_MAXP) return set_error(c, GS_EINVAL, "nparts %u outside [1, 64]", nparts);
  if (c->rt_n == ~0ull || c->rt_seq != c->call_seq) return set_error(c, GS_EINVAL, "gs_tri_dist_orient first");
  const uint64_t n = c->rt_n;
  if (n && !keys_out) return set_error(c, GS_EINVAL, "null keys_out");
  GS_HIP(hipSetDevice(c->device));
  (void)hipGetLastError();
  const uint32_t B = c->tri_B;
  const size_t V = 1ull << B;
  // split points at equal shares of the raw work (the same on every rank: dout is the all-reduced one)
  GS_TRY(ensure(c, c->tri_hwork, (V * 2 + 2) * 8));
  GS_TRY(ensure(c, c->tri_bd[3], 8 * 65 * 8));
  unsigned long long* w = c->tri_hwork.as<unsigned long long>();
  unsigned long long* sp_d = c->tri_bd[3].as<unsigned long long>() + 7 * 65;
  const unsigned gv = (unsigned)std::min<uint64_t>((V + 255) / 256, 16384);
  hipLaunchKernelGGL(k_tri_rawwork, dim3(gv), dim3(256), 0, c->stream, dout, (uint32_t)V, w);
  GS_TRY(xscan(c, (const uint64_t*)w, V, (uint64_t*)w + V + 1));
  hipLaunchKernelGGL(k_tri_split, dim3(1), dim3(128), 0, c->stream, (const unsigned long long*)w + V + 1, (uint32_t)V,
                     nparts, sp_d);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 64, sp_d, (nparts + 1) * 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  RtSplit sp;
  for (uint32_t q = 0; q <= nparts; ++q) {   // monotone owner ranges (route / plan / need / serve assume them)
    sp.s[q] = (uint32_t)std::min<uint64_t>(c->host_small[64 + q], V);
    if (q && sp.s[q] < sp.s[q - 1]) sp.s[q] = sp.s[q - 1];
  }
  sp.s[nparts] = (uint32_t)V;
  c->rt_split = sp;
  c->rt_nparts = nparts;
  const uint32_t tiles = (uint32_t)std::max<uint64_t>(1, (n + RT_TILE - 1) / RT_TILE);
  GS_TRY(ensure(c, c->tri_tiles, (size_t)tiles * nparts * 4 + 8));
  uint32_t* cnt = c->tri_tiles.as<uint32_t>();
  const uint64_t kept = n - c->host_small[4];
  if (n) {
    hipLaunchKernelGGL(k_route_count, dim3(tiles), dim3(RT_BLOCK), 0, c->stream, c->aux.as<uint64_t>(), n, B, nparts, sp,
                       tiles, cnt);
    hipLaunchKernelGGL(k_rank_scan, dim3(1), dim3(1024), 0, c->stream, cnt, tiles * nparts);
    hipLaunchKernelGGL(k_route_scatter, dim3(tiles), dim3(RT_BLOCK), 0, c->stream, c->aux.as<uint64_t>(), n, B, nparts,
                       sp, tiles, cnt, keys_out);
    GS_HIP(hipGetLastError());
    // owner o's keys start at cnt[o * tiles] (exclusive scan, owner-major)
    for (uint32_t o = 0; o < nparts; ++o)
      GS_HIP(hipMemcpyAsync((uint32_t*)(c->host_small + 16) + o, cnt + (size_t)o * tiles, 4, hipMemcpyDeviceToHost, c->stream));
  }
  GS_TRY(host_wait(c));
  const uint32_t* st = (const uint32_t*)(c->host_small + 16);
  for (uint32_t o = 0; o < nparts; ++o) counts[o] = n ? (o + 1 < nparts ? st[o + 1] : kept) - st[o] : 0;
  return GS_OK;
}

gs_status gs_tri_dist_build(gs_ctx* c, const uint64_t* keys, uint64_t n, uint32_t* nbr_out, uint32_t* dplus_out,
                            uint64_t* m_out) {
  if (!c) return GS_EINVAL;
  if (!m_out || !dplus_out || (n && (!keys || !nbr_out))) return set_error(c, GS_EINVAL, "null pointer");
  if (!c->tri_B) return set_error(c, GS_EINVAL, "gs_tri_dist_degrees first (the window's id geometry)");
  GS_TRY(begin_call(c));
  hipEventRecord(c->ev[0], c->stream);
  const uint32_t B = c->tri_B;
  const size_t V = 1ull << B;
  GS_TRY(ensure(c, c->tri_range, V * 16));
  uint2* out_range = reinterpret_cast<uint2*>(c->tri_range.p);
  GS_HIP(hipMemsetAsync(out_range, 0, V * 8, c->stream));
  uint64_t M = 0;
  if (n) {
    Sorted s;
    GS_TRY(tri_unique(c, keys, n, B, false, false, &M, &s));
    if (M)
      hipLaunchKernelGGL(k_tri_out, dim3((unsigned)std::min<uint64_t>((M + 255) / 256, 16384)), dim3(256), 0, c->stream,
                         c->out_keys.as<uint64_t>(), (uint32_t)M, B, nbr_out, reinterpret_cast<uint32_t*>(out_range));
  }
  hipLaunchKernelGGL(k_tri_dplus, dim3((unsigned)std::min<uint64_t>((V + 255) / 256, 16384)), dim3(256), 0, c->stream,
                     out_range, (uint32_t)V, dplus_out);
  GS_HIP(hipGetLastError());
  *m_out = M;
  return host_wait(c);
}

gs_status gs_tri_dist_count(gs_ctx* c, const uint32_t* nbr, uint64_t M, const uint32_t* dplus, uint32_t part,
                            uint32_t nparts, uint64_t* count) {
  if (!c) return GS_EINVAL;
  if (!count || !dplus || (M && !nbr)) return set_error(c, GS_EINVAL, "null pointer");
  if (nparts == 0 || part >= nparts) return set_error(c, GS_EINVAL, "bad part %u of %u", part, nparts);
  if (!c->tri_B) return set_error(c, GS_EINVAL, "gs_tri_dist_degrees first (the window's id geometry)");
  if (M >= (1ull << 32)) return set_error(c, GS_EINVAL, "split window: %llu edges (limit 2^32-1)", (unsigned long long)M);
  GS_TRY(begin_call(c));
  *count = 0;
  if (M == 0) return GS_OK;
  hipEventRecord(c->ev[0], c->stream);
  hipEventRecord(c->ev[1], c->stream);
  const uint32_t B = c->tri_B;
  const size_t V = 1ull << B;
  GS_TRY(ensure(c, c->tri_range, V * 16));
  GS_TRY(ensure(c, c->tri_d[5], (V + 1) * 16));
  unsigned long long* d64 = c->tri_d[5].as<unsigned long long>();
  uint2* out_range = reinterpret_cast<uint2*>(c->tri_range.p);
  const unsigned gv = (unsigned)std::min<uint64_t>((V + 255) / 256, 16384);
  hipLaunchKernelGGL(k_u32_to_u64, dim3(gv), dim3(256), 0, c->stream, dplus, (uint32_t)V, d64);
  GS_TRY(xscan(c, (const uint64_t*)d64, V, (uint64_t*)d64 + V));
  hipLaunchKernelGGL(k_tri_ranges, dim3(gv), dim3(256), 0, c->stream, dplus, (const unsigned long long*)d64 + V,
                     (uint32_t)V, out_range);
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[2], c->stream);
  uint64_t T = 0, probes = 0;
  GS_TRY(tri_count(c, B, V, M, nbr, out_range, nullptr, part, nparts, &T, &probes));
  TriGeom g;
  set_bits(&g, B);
  tri_times(c, g, M, 0, probes, 0);
  *count = T;
  return GS_OK;
}

// ---- boundary adjacency (see k_bd_bounds) -------------------------------------------------------------
static unsigned bd_grid(uint64_t n, uint64_t per) {
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, 16384));
}

gs_status gs_tri_dist_plan(gs_ctx* c, const uint32_t* dplus, uint32_t part, uint32_t nparts, uint64_t* send_elems,
                           uint64_t* recv_elems, uint64_t* M_out) {
  if (!c) return GS_EINVAL;
  if (!dplus || !send_elems || !recv_elems || !M_out) return set_error(c, GS_EINVAL, "null pointer");
  if (nparts == 0 || nparts > 64 || part >= nparts) return set_error(c, GS_EINVAL, "bad part %u of %u", part, nparts);
  if (!c->tri_B) return set_error(c, GS_EINVAL, "gs_tri_dist_degrees first (the window's id geometry)");
  if (c->rt_nparts != nparts) return set_error(c, GS_EINVAL, "gs_tri_dist_route over %u parts first", nparts);
  GS_TRY(begin_call(c));
  c->bd_ok = false;
  const uint32_t B = c->tri_B, P = nparts;
  const size_t V = 1ull << B;
  GS_TRY(ensure(c, c->tri_range, V * 16));
  GS_TRY(ensure(c, c->tri_d[5], (V + 1) * 16));
  GS_TRY(ensure(c, c->tri_hwork, (V * 2 + 2) * 8));
  GS_TRY(ensure(c, c->tri_bd[3], 8 * 65 * 8));
  unsigned long long* d64 = c->tri_d[5].as<unsigned long long>();   // d+ [0, V), prefix [V, 2V]
  unsigned long long* work = c->tri_hwork.as<unsigned long long>();
  unsigned long long* bnd = c->tri_bd[3].as<unsigned long long>();
  uint2* out_range = reinterpret_cast<uint2*>(c->tri_range.p);
  const unsigned gv = bd_grid(V, 256);
  hipLaunchKernelGGL(k_u32_to_u64, dim3(gv), dim3(256), 0, c->stream, dplus, (uint32_t)V, d64);
  GS_TRY(xscan(c, (const uint64_t*)d64, V, (uint64_t*)d64 + V));
  hipLaunchKernelGGL(k_tri_ranges, dim3(gv), dim3(256), 0, c->stream, dplus, (const unsigned long long*)d64 + V,
                     (uint32_t)V, out_range);
  hipLaunchKernelGGL(k_tri_work, dim3(gv), dim3(256), 0, c->stream, out_range, (uint32_t)V, work);
  GS_TRY(xscan(c, (const uint64_t*)work, V, (uint64_t*)work + V + 1));
  hipLaunchKernelGGL(k_bd_bounds, dim3(1), dim3(128), 0, c->stream, (const unsigned long long*)work + V + 1,
                     (const unsigned long long*)d64 + V, (uint32_t)V, c->rt_split, P, bnd);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 64, bnd, 4 * (P + 1) * 8, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small + 63, (const unsigned long long*)d64 + 2 * V, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t* h = c->host_small + 64;
  const uint64_t *cq = h, *rq = h + (P + 1), *pc = h + 2 * (P + 1), *pr = h + 3 * (P + 1);
  // C_a ∩ R_b as window positions: both are unions of whole rows, so the larger start / smaller end of
  // the two ranges bound it, and their positions bound its elements
  auto inter = [&](uint32_t a, uint32_t b) -> uint64_t {
    const uint64_t u0 = std::max(cq[a], rq[b]), u1 = std::min(cq[a + 1], rq[b + 1]);
    if (u0 >= u1) return 0;
    const uint64_t p0 = cq[a] >= rq[b] ? pc[a] : pr[b], p1 = cq[a + 1] <= rq[b + 1] ? pc[a + 1] : pr[b + 1];
    return p1 > p0 ? p1 - p0 : 0;
  };
  for (uint32_t q = 0; q < P; ++q) {
    send_elems[q] = inter(q, part);   // rows this rank built that rank q counts
    recv_elems[q] = inter(part, q);   // rows this rank counts that rank q built
  }
  c->bd_part = part;
  c->bd_nparts = P;
  c->bd_c0 = cq[part];
  c->bd_c1 = cq[part + 1];
  c->bd_r0 = rq[part];
  c->bd_r1 = rq[part + 1];
  c->bd_pc0 = pc[part];
  c->bd_pc1 = pc[part + 1];
  c->bd_pr0 = pr[part];
  c->bd_pr1 = pr[part + 1];
  c->bd_M = c->host_small[63];
  c->bd_nreq = 0;
  c->bd_ok = true;
  *M_out = c->bd_M;
  return GS_OK;
}

gs_status gs_tri_dist_need(gs_ctx* c, const uint32_t* crows, uint32_t* req_out, uint64_t capacity,
                           uint64_t* req_counts, uint64_t* req_elems, uint64_t* nreq) {
  if (!c) return GS_EINVAL;
  if (!req_counts || !req_elems || !nreq) return set_error(c, GS_EINVAL, "null pointer");
  if (!c->bd_ok) return set_error(c, GS_EINVAL, "gs_tri_dist_plan first");
  const uint64_t nc = c->bd_pc1 - c->bd_pc0;
  if (nc && !crows) return set_error(c, GS_EINVAL, "null crows");
  const uint32_t P = c->bd_nparts, B = c->tri_B;
  const size_t V = 1ull << B, words = (V + 31) / 32;
  GS_HIP(hipSetDevice(c->device));
  (void)hipGetLastError();
  const size_t boff = (words * 4 + 255) & ~(size_t)255;
  GS_TRY(ensure(c, c->tri_bd[0], V * 4 + 64));                        // the requested ids
  GS_TRY(ensure(c, c->tri_bd[1], (V + 1) * 8 * 2));                   // row lengths, their prefix
  GS_TRY(ensure(c, c->tri_bd[2], boff + (words + 1) * 8 * 2 + 64));  // bitmap, word counts, positions
  uint32_t* bits = c->tri_bd[2].as<uint32_t>();
  uint64_t* wcnt = reinterpret_cast<uint64_t*>(c->tri_bd[2].as<char>() + boff);
  uint64_t* wpos = wcnt + words + 1;
  uint32_t* bad = reinterpret_cast<uint32_t*>(wpos + words + 1);
  GS_HIP(hipMemsetAsync(bits, 0, words * 4, c->stream));
  GS_HIP(hipMemsetAsync(bad, 0, 4, c->stream));
  if (nc)
    hipLaunchKernelGGL(k_bd_mark, dim3(bd_grid(nc, 256)), dim3(256), 0, c->stream, crows, nc, (uint32_t)c->bd_c0,
                       (uint32_t)c->bd_c1, (uint32_t)c->bd_r0, (uint32_t)c->bd_r1, (uint32_t)V,
                       c->tri_d[5].as<unsigned long long>(), bits, bad);
  hipLaunchKernelGGL(k_bd_popc, dim3(bd_grid(words, 256)), dim3(256), 0, c->stream, bits, (uint32_t)words, wcnt);
  GS_TRY(xscan(c, wcnt, words, wpos));
  uint32_t* ids = c->tri_bd[0].as<uint32_t>();
  uint64_t* len = c->tri_bd[1].as<uint64_t>();
  uint64_t* rowpre = len + V + 1;
  const unsigned long long* d64 = c->tri_d[5].as<unsigned long long>();
  hipLaunchKernelGGL(k_bd_ids, dim3(bd_grid(words, 256)), dim3(256), 0, c->stream, bits, (uint32_t)words,
                     (const uint64_t*)wpos, d64, ids, len);
  GS_HIP(hipGetLastError());
  c->host_small[61] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 62, wpos + words, 8, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small + 61, bad, 4, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if ((uint32_t)c->host_small[61]) return set_error(c, GS_EINVAL, "gs_tri_dist_need: a row holds an id >= V");
  const uint64_t n = c->host_small[62];
  GS_TRY(xscan(c, len, n, rowpre));
  unsigned long long* g = c->tri_bd[3].as<unsigned long long>() + 4 * 65;
  hipLaunchKernelGGL(k_bd_groups, dim3(1), dim3(128), 0, c->stream, ids, n, (const uint64_t*)rowpre,
                     c->tri_bd[3].as<unsigned long long>(), P, g);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 64, g, 2 * (P + 1) * 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t* h = c->host_small + 64;
  for (uint32_t q = 0; q < P; ++q) {
    req_counts[q] = h[q + 1] - h[q];
    req_elems[q] = h[P + 1 + q + 1] - h[P + 1 + q];
  }
  c->bd_nreq = n;
  *nreq = n;
  if (n > capacity) return set_error(c, GS_ECAPACITY, "gs_tri_dist_need: %llu ids", (unsigned long long)n);
  if (n) GS_HIP(hipMemcpyAsync(req_out, ids, n * 4, hipMemcpyDeviceToDevice, c->stream));
  return host_wait(c);
}

gs_status gs_tri_dist_serve(gs_ctx* c, const uint32_t* nbr, const uint32_t* req_in, const uint64_t* counts_in,
                            uint32_t* rows_out, uint64_t capacity, uint64_t* send_elems) {
  if (!c) return GS_EINVAL;
  if (!counts_in || !send_elems) return set_error(c, GS_EINVAL, "null pointer");
  if (!c->bd_ok) return set_error(c, GS_EINVAL, "gs_tri_dist_plan first");
  const uint32_t P = c->bd_nparts;
  BdGroups gr;
  gr.g[0] = 0;
  for (uint32_t q = 0; q < P; ++q) gr.g[q + 1] = gr.g[q] + counts_in[q];
  const uint64_t n = gr.g[P];
  for (uint32_t q = 0; q < P; ++q) send_elems[q] = 0;
  if (n == 0) return GS_OK;
  if (!req_in || !nbr) return set_error(c, GS_EINVAL, "null pointer");
  GS_HIP(hipSetDevice(c->device));
  (void)hipGetLastError();
  GS_TRY(ensure(c, c->tri_bd[2], (n + 1) * 8 * 2 + 64));
  uint64_t* len = c->tri_bd[2].as<uint64_t>();
  uint64_t* pos = len + n + 1;
  uint32_t* bad = reinterpret_cast<uint32_t*>(pos + n + 1);
  GS_HIP(hipMemsetAsync(bad, 0, 4, c->stream));
  const unsigned long long* d64 = c->tri_d[5].as<unsigned long long>();
  hipLaunchKernelGGL(k_bd_serve_len, dim3(bd_grid(n, 256)), dim3(256), 0, c->stream, req_in, n, d64,
                     (uint32_t)c->bd_r0, (uint32_t)c->bd_r1, len, bad);
  GS_TRY(xscan(c, len, n, pos));
  unsigned long long* pk = c->tri_bd[3].as<unsigned long long>() + 6 * 65;
  hipLaunchKernelGGL(k_bd_pick, dim3(1), dim3(128), 0, c->stream, (const uint64_t*)pos, gr, P, pk);
  GS_HIP(hipGetLastError());
  c->host_small[61] = 0;
  GS_HIP(hipMemcpyAsync(c->host_small + 64, pk, (P + 1) * 8, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small + 61, bad, 4, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if ((uint32_t)c->host_small[61]) return set_error(c, GS_EINVAL, "gs_tri_dist_serve: a requested id is not this rank's");
  const uint64_t* h = c->host_small + 64;
  for (uint32_t q = 0; q < P; ++q) send_elems[q] = h[q + 1] - h[q];
  if (h[P] > capacity) return set_error(c, GS_ECAPACITY, "gs_tri_dist_serve: %llu row elements", (unsigned long long)h[P]);
  if (h[P] == 0) return GS_OK;
  if (!rows_out) return set_error(c, GS_EINVAL, "null rows_out");
  hipLaunchKernelGGL(k_bd_copy<true>, dim3(bd_grid(n, 4)), dim3(256), 0, c->stream, req_in, n,
                     d64 + (1ull << c->tri_B), c->bd_pr0, (const uint64_t*)pos, d64, (uint32_t)c->bd_r0, (uint32_t)c->bd_r1,
                     nbr, rows_out);
  GS_HIP(hipGetLastError());
  return host_wait(c);
}

gs_status gs_tri_dist_assemble(gs_ctx* c, const uint32_t* nbr, const uint32_t* crows, const uint32_t* rows_in,
                               uint32_t* full_out) {
  if (!c) return GS_EINVAL;
  if (!c->bd_ok) return set_error(c, GS_EINVAL, "gs_tri_dist_plan first");
  if (c->bd_M && !full_out) return set_error(c, GS_EINVAL, "null full_out");
  GS_HIP(hipSetDevice(c->device));
  (void)hipGetLastError();
  const uint64_t nr = c->bd_pr1 - c->bd_pr0, nc = c->bd_pc1 - c->bd_pc0, n = c->bd_nreq;
  if ((nr && !nbr) || (nc && !crows)) return set_error(c, GS_EINVAL, "null rows");
  // rows nobody sent stay id 0 (a valid id: a missing row can only miscount, never index past V)
  if (c->bd_M) GS_HIP(hipMemsetAsync(full_out, 0, c->bd_M * 4, c->stream));
  if (nr) GS_HIP(hipMemcpyAsync(full_out + c->bd_pr0, nbr, nr * 4, hipMemcpyDeviceToDevice, c->stream));
  if (nc) GS_HIP(hipMemcpyAsync(full_out + c->bd_pc0, crows, nc * 4, hipMemcpyDeviceToDevice, c->stream));
  if (n) {
    if (!rows_in) return set_error(c, GS_EINVAL, "null rows_in");
    const unsigned long long* d64 = c->tri_d[5].as<unsigned long long>();
    const uint64_t* rowpre = c->tri_bd[1].as<uint64_t>() + (1ull << c->tri_B) + 1;
    hipLaunchKernelGGL(k_bd_copy<false>, dim3(bd_grid(n, 4)), dim3(256), 0, c->stream, c->tri_bd[0].as<uint32_t>(), n,
                       d64 + (1ull << c->tri_B), 0ull, rowpre, d64, 0u, 0u, rows_in, full_out);
    GS_HIP(hipGetLastError());
  }
  return host_wait(c);
}

gs_status gs_window_triangles_selfpair(gs_ctx* c, const gs_edge_batch* b, uint64_t* S) {
  if (!c) return GS_EINVAL;
  GS_TRY(check_batch(c, b, GS_DIR_ALL));
  if (!S) return set_error(c, GS_EINVAL, "null output pointer");
  GS_TRY(begin_call(c));
  *S = 0;
  if (b->n == 0) return GS_OK;
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  TriGeom g;
  GS_TRY(tri_geometry(c, src, dst, b->n, &g));
  const size_t words = (g.V + 31) / 32;
  GS_TRY(ensure(c, c->tri_loops, words * 4));
  GS_HIP(hipMemsetAsync(c->tri_loops.p, 0, words * 4, c->stream));
  unsigned long long* d_loops = (unsigned long long*)(c->small.as<char>() + SM_NUNIQUE);
  GS_HIP(hipMemsetAsync(d_loops, 0, 8, c->stream));
  hipLaunchKernelGGL(k_tri_loops, dim3((unsigned)std::min<uint64_t>((b->n + 255) / 256, 8192)), dim3(256), 0, c->stream,
                     g.src, g.dst, g.n, g.key_xor, c->tri_loops.as<uint32_t>(), d_loops);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 4, d_loops, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if (c->host_small[4] == 0) return GS_OK;
  return triangle_selfpair_term(c, g.osrc, g.odst, g.n, c->tri_loops.as<uint32_t>(), g.key_xor, g.uniq, g.nuniq, S);
}

// The split window with the ctx communicator: every rank passes its own records of the window
gs_status gs_window_triangles_dist(gs_ctx* c, const gs_edge_batch* b, uint64_t* count, int32_t* count_ref_wrapped,
                                   int32_t* has_output) {
  if (!c) return GS_EINVAL;
  if (!count || !count_ref_wrapped || !has_output) return set_error(c, GS_EINVAL, "null output pointer");
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  const uint32_t P = (uint32_t)c->comm_size, me = (uint32_t)c->comm_rank;
  // 1. the common id range, the window's record count and every rank's status in ONE collective (each
  //    rank's [failed, min, max, records] row; round 5 ran an agreement, a MIN, a MAX and a SUM, each with
  //    its own host wait).  Later steps agree on their status before the collective that follows them.
  int64_t mm[2];
  const gs_status rs = gs_tri_dist_range(c, b, mm);
  const std::string rerr = c->err;
  const uint64_t mine[4] = {rs != GS_OK ? 1ull : 0ull, (uint64_t)mm[0], (uint64_t)mm[1], rs == GS_OK ? b->n : 0};
  std::vector<uint64_t> rows((size_t)P * 4);
  GS_TRY(comm_allgather_words(c, mine, 4, rows.data()));
  if (rs != GS_OK) return set_error(c, rs, "%s", rerr.c_str());
  int64_t gmin = INT64_MAX, gmax = INT64_MIN;
  uint64_t total_n = 0;
  for (uint32_t p = 0; p < P; ++p) {
    if (rows[4 * p]) return set_error(c, GS_ECOMM, "rank %u failed its local step of the window", p);
    gmin = std::min(gmin, (int64_t)rows[4 * p + 1]);
    gmax = std::max(gmax, (int64_t)rows[4 * p + 2]);
    total_n += rows[4 * p + 3];
  }
  *count = 0;
  *count_ref_wrapped = 0;
  *has_output = total_n > 0;
  if (total_n == 0) return GS_OK;
  // ids spanning more than 2^TRI_MAX_BITS values, or an id space more than 4x sparser than the window's
  // endpoints (the dense per-id tables -- degrees, out-degrees, d+ -- are all-reduced, 4 B per id each):
  // steps 2-5 run on compact ids of the whole window (step 6, the self-pair term, keeps the original
  // records: its HashSet order needs the values)
  const gs_edge_batch* lb = b;
  gs_edge_batch rb{};
  const uint64_t dx = (uint64_t)gmin ^ (uint64_t)gmax;
  const int span_bits = dx ? 64 - __builtin_clzll(dx) : 1;
  if (span_bits > (int)TRI_MAX_BITS || (span_bits > 20 && (1ull << span_bits) > 8 * total_n)) {
    int64_t vmax = 0;
    GS_TRY(tri_dist_relabel(c, b, &rb, &vmax));
    lb = &rb;
    gmin = 0;
    gmax = vmax;
  }
  // 2. degrees, summed over ranks
  uint64_t V = 0;
  gs_status st = gs_tri_dist_degrees(c, lb, gmin, gmax, nullptr, &V);
  if (st == GS_OK) st = ensure(c, c->tri_d[1], V * 4);
  uint32_t* deg = c->tri_d[1].as<uint32_t>();
  if (st == GS_OK) st = gs_tri_dist_degrees(c, lb, gmin, gmax, deg, &V);
  GS_TRY(comm_agree(c, st));
  GS_TRY(comm_allreduce(c, deg, V, NCCL_T_U32, NCCL_OP_SUM));
  // 3. oriented edges; their raw out-degrees summed (the route's owner ranges cut the raw work in equal
  //    shares, the same on every rank); keys to owner(u): counts matrix, then the rows
  std::vector<uint64_t> send(P), recv(P);
  uint64_t loops = 0;
  GS_TRY(ensure(c, c->tri_d[6], V * 4 + 4));
  uint32_t* dout = c->tri_d[6].as<uint32_t>();
  GS_TRY(comm_agree(c, gs_tri_dist_orient(c, lb, deg, dout, &loops)));
  GS_TRY(comm_allreduce(c, dout, V, NCCL_T_U32, NCCL_OP_SUM));
  st = ensure(c, c->tri_d[2], lb->n * 8 + 8);
  if (st == GS_OK) st = gs_tri_dist_route(c, dout, P, c->tri_d[2].as<uint64_t>(), send.data());
  GS_TRY(comm_agree(c, st));
  GS_TRY(ensure(c, c->tri_d[0], 64 + (size_t)P * P * 8));
  uint64_t* dmat = (uint64_t*)(c->tri_d[0].as<char>() + 64);
  GS_HIP(hipMemsetAsync(dmat, 0, (size_t)P * P * 8, c->stream));
  memcpy(c->host_small + 16, send.data(), P * 8);
  GS_HIP(hipMemcpyAsync(dmat + (size_t)me * P, c->host_small + 16, P * 8, hipMemcpyHostToDevice, c->stream));
  GS_TRY(comm_allreduce(c, dmat, (size_t)P * P, NCCL_T_U64, NCCL_OP_SUM));
  uint64_t nrecv = 0;
  for (uint32_t p = 0; p < P; ++p) {   // column me of the matrix: what each rank sends me
    GS_HIP(hipMemcpyAsync(c->host_small + 16 + p, dmat + (size_t)p * P + me, 8, hipMemcpyDeviceToHost, c->stream));
  }
  GS_TRY(host_wait(c));
  for (uint32_t p = 0; p < P; ++p) nrecv += (recv[p] = c->host_small[16 + p]);
  GS_TRY(ensure(c, c->tri_d[3], nrecv * 8 + 8));
  GS_TRY(exchange_rows(c, c->tri_d[2].as<char>(), send.data(), c->tri_d[3].as<char>(), recv.data(), 8));
  GS_TRY(gs_comm_allreduce_sum_u64(c, &loops));
  // 4. local out-lists; out-degrees summed (every u has one owner).  Then the boundary adjacency
  //    instead of every row: the rows of this rank's count range (one all-to-all, sizes known to every
  //    rank from the global d+), then the rows of their targets it holds in neither range (ids
  //    requested, rows served: two all-to-alls), assembled at their window positions
  GS_TRY(ensure(c, c->tri_d[4], nrecv * 4 + 4));
  GS_TRY(ensure(c, c->tri_d[1], V * 4));   // the degrees are consumed: d+ reuses the buffer
  uint32_t* dplus = c->tri_d[1].as<uint32_t>();
  uint32_t* nbr = c->tri_d[4].as<uint32_t>();
  uint64_t m = 0;
  GS_TRY(comm_agree(c, gs_tri_dist_build(c, c->tri_d[3].as<uint64_t>(), nrecv, nbr, dplus, &m)));
  GS_TRY(comm_allreduce(c, dplus, V, NCCL_T_U32, NCCL_OP_SUM));
  std::vector<uint64_t> s1(P), r1(P), rc(P), re(P), qc(P), qe(P), se(P), one(P, 1);
  uint64_t M = 0, nreq = 0;
  GS_TRY(comm_agree(c, gs_tri_dist_plan(c, dplus, me, P, s1.data(), r1.data(), &M)));
  uint64_t nc = 0;
  for (uint32_t p = 0; p < P; ++p) nc += r1[p];
  GS_TRY(ensure(c, c->tri_d[2], nc * 4 + 4));   // the routed keys are consumed: the count range's rows
  uint32_t* crows = c->tri_d[2].as<uint32_t>();
  GS_TRY(exchange_rows(c, (const char*)nbr, s1.data(), (char*)crows, r1.data(), 4));
  GS_TRY(ensure(c, c->tri_d[3], V * 4 + 4));    // the received keys are consumed: the ids requested
  uint32_t* req = c->tri_d[3].as<uint32_t>();
  GS_TRY(comm_agree(c, gs_tri_dist_need(c, crows, req, V, rc.data(), re.data(), &nreq)));
  // (ids, row elements) each rank asks of each other: one 16-byte row per peer
  GS_TRY(ensure(c, c->tri_d[0], 64 + (size_t)P * 32));
  uint64_t* pairs = (uint64_t*)(c->tri_d[0].as<char>() + 64);
  for (uint32_t p = 0; p < P; ++p) {
    c->host_small[64 + 2 * p] = rc[p];
    c->host_small[65 + 2 * p] = re[p];
  }
  GS_HIP(hipMemcpyAsync(pairs, c->host_small + 64, (size_t)P * 16, hipMemcpyHostToDevice, c->stream));
  GS_TRY(exchange_rows(c, (const char*)pairs, one.data(), (char*)(pairs + 2 * P), one.data(), 16));
  GS_HIP(hipMemcpyAsync(c->host_small + 64, pairs + 2 * P, (size_t)P * 16, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  uint64_t nin = 0, nel = 0, nrows = 0;
  for (uint32_t p = 0; p < P; ++p) {
    nin += (qc[p] = c->host_small[64 + 2 * p]);
    nel += (qe[p] = c->host_small[65 + 2 * p]);
    nrows += re[p];
  }
  GS_TRY(ensure(c, c->tri_d[6], nin * 4 + 4));
  GS_TRY(exchange_rows(c, (const char*)req, rc.data(), c->tri_d[6].as<char>(), qc.data(), 4));
  GS_TRY(ensure(c, c->tri_d[7], nel * 4 + 4));
  GS_TRY(comm_agree(c, gs_tri_dist_serve(c, nbr, c->tri_d[6].as<uint32_t>(), qc.data(), c->tri_d[7].as<uint32_t>(),
                                         nel, se.data())));
  GS_TRY(ensure(c, c->tri_d[8], nrows * 4 + 4));
  GS_TRY(exchange_rows(c, c->tri_d[7].as<char>(), se.data(), c->tri_d[8].as<char>(), re.data(), 4));
  GS_TRY(ensure(c, c->tri_d[9], M * 4 + 4));
  GS_TRY(comm_agree(c, gs_tri_dist_assemble(c, nbr, crows, c->tri_d[8].as<uint32_t>(), c->tri_d[9].as<uint32_t>())));
  // 5. this rank's share of the count, summed
  uint64_t T = 0;
  GS_TRY(comm_agree(c, gs_tri_dist_count(c, c->tri_d[9].as<uint32_t>(), M, dplus, me, P, &T)));
  // 6. the self-pair term needs whole neighbour sets: windows with self-loops gather the records
  if (loops) {
    std::vector<uint64_t> ns(P);
    GS_TRY(comm_allgather_u64(c, b->n, ns.data()));
    const int64_t *src, *dst;
    const void* val;
    GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
    GS_TRY(ensure(c, c->tri_d[3], total_n * 16 + 16));
    int64_t* all = c->tri_d[3].as<int64_t>();
    GS_TRY(comm_allgatherv(c, src, (char*)all, ns.data(), 8));
    GS_TRY(comm_allgatherv(c, dst, (char*)(all + total_n), ns.data(), 8));
    GS_TRY(host_wait(c));
    gs_status sp = GS_OK;
    if (me == 0) {
      const gs_edge_batch wb{all, all + total_n, nullptr, total_n, GS_NONE, GS_MEM_DEVICE, 0};
      uint64_t S = 0;
      sp = gs_window_triangles_selfpair(c, &wb, &S);
      T += S;
    }
    GS_TRY(comm_agree(c, sp));
  }
  GS_TRY(gs_comm_allreduce_sum_u64(c, &T));
  *count = T;
  *count_ref_wrapped = (int32_t)(uint32_t)T;
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
