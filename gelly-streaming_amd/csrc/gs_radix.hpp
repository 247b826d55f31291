// gs_radix.hpp — stable LSD radix sort of a window's keyed records on gfx950.
//
// Replaces Flink's keyBy(NeighborKeySelector) + per-key window state grouping
// (SimpleEdgeStream.java:153-183, GraphWindowStream.java:49-53): after the sort every
// vertex's records are contiguous and, because every pass is stable, in arrival order.
//
// Pipeline per window (all HBM-bound integer work, no MFMA):
//   k_keyinfo   one read of the keys: OR of (key ^ key0) -> which bits vary, and the
//               histograms of the four low key bytes (LDS, per-wave copies);
//   k_digit_base exclusive scan of each pass's 256-bin histogram (1 block);
//   k_onesweep  one launch per 8-bit digit: dynamic tile claim, wave64 ballot match for
//               the rank inside a wave, LDS digit counters, decoupled look-back over tiles
//               for the global digit offsets, LDS exchange so the scatter writes runs of
//               consecutive addresses.  The first pass reads the raw int64 edge columns
//               and does the direction expansion (OUT / IN / ALL) on the fly.
// Keys are compacted to 32 bits whenever only the low 32 bits vary (vertex IDs < 2^32 or
// any window whose IDs share their high half) — halving key traffic in every pass.
#pragma once
#include <type_traits>

#include "gs_device.hpp"

namespace gs {

constexpr int RADIX_BITS = 8;
constexpr int RADIX = 1 << RADIX_BITS;

enum : int { DIR_IN = 0, DIR_OUT = 1, DIR_ALL = 2 };

// ---- first-pass record sources (direction expansion, SimpleEdgeStream.java:153-171) -------
// record r: OUT key=src[r], nbr=dst[r]; IN key=dst[r], nbr=src[r];
// ALL r=2i -> (src[i], dst[i]), r=2i+1 -> (dst[i], src[i])  (UndirectEdges :359-365)
enum : int { PAY_NONE = 0, PAY_VAL = 1, PAY_NBR = 2, PAY_IDX = 3 };

template <typename K, typename V, int DIR, int PAY>
struct EdgeSrc {
  const int64_t* src;
  const int64_t* dst;
  const V* val;       // PAY_VAL: edge values
  uint64_t key_xor;   // compaction: ukey = key ^ key_xor, truncated to K
  __device__ __forceinline__ void load(uint32_t r, K& k, V& v) const {
    uint32_t i = r;
    bool rev = (DIR == DIR_IN);
    if (DIR == DIR_ALL) { i = r >> 1; rev = r & 1u; }
    const int64_t a = rev ? dst[i] : src[i];
    k = (K)((uint64_t)a ^ key_xor);
    if constexpr (PAY == PAY_VAL) v = val[i];
    else if constexpr (PAY == PAY_NBR) v = (V)(rev ? src[i] : dst[i]);
    else if constexpr (PAY == PAY_IDX) v = (V)r;
  }
};

template <typename K, typename V>
struct BufSrc {
  const K* keys;
  const V* vals;
  uint64_t key_xor;  // unused
  __device__ __forceinline__ void load(uint32_t r, K& k, V& v) const {
    k = keys[r];
    if constexpr (!std::is_same_v<V, uint8_t>) v = vals[r];   // no payload: V = uint8_t
  }
};

// u64 key buffer (composite keys) -> key type K: k = (K)(key ^ key_xor)
template <typename K, typename V>
struct ConvSrc {
  const uint64_t* keys;
  const V* vals;
  uint64_t key_xor;
  __device__ __forceinline__ void load(uint32_t r, K& k, V& v) const {
    k = (K)(keys[r] ^ key_xor);
    if constexpr (!std::is_same_v<V, uint8_t>) v = vals[r];   // no payload: V = uint8_t
  }
};

// One key into this wave's 256-bin histograms of its nd low bytes (hw = [nd][RADIX] in LDS).  The
// bin of the wave's first lane is counted once per wave (a popcount): skewed digits -- R-MAT hubs,
// the top byte of narrow keys -- would otherwise serialize 64 lanes on one LDS counter (triangles
// s24: 4.0 ms per 2 GB of keys).  Every lane of the wave must call it (ballots).
__device__ __forceinline__ void wave_hist_add(uint32_t (*hw)[RADIX], uint64_t k, bool valid, int nd) {
  const uint64_t lt = (1ull << (threadIdx.x & 63)) - 1;
  for (int b = 0; b < nd; ++b) {
    const uint32_t d = (uint32_t)(k >> (8 * b)) & 255u;
    const uint32_t L = __builtin_amdgcn_readfirstlane(d);
    const uint64_t same = __ballot(valid && d == L);
    if (valid && d == L) {
      if ((same & lt) == 0) atomicAdd(&hw[b][L], (uint32_t)__popcll(same));
    } else if (valid) {
      atomicAdd(&hw[b][d], 1u);
    }
  }
}
// a block's per-wave tables h[NW][8][RADIX] (nd bytes used) into the global histograms
template <int NW>
__device__ __forceinline__ void flush_hist(uint32_t (*h)[8][RADIX], int nd, uint32_t* __restrict__ hist_out) {
  for (int i = threadIdx.x; i < nd * RADIX; i += blockDim.x) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) c += h[w][0][i];
    if (c) atomicAdd(&hist_out[i], c);
  }
}

// XOR-mask of a key buffer + the 256-bin histograms of its nd low bytes (the caller's bound on the
// key width), one table per wave (wave_hist_add)
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_keyinfo_buf(const uint64_t* __restrict__ keys, uint64_t n, int nd,
                                                     unsigned long long* __restrict__ mask_out,
                                                     uint32_t* __restrict__ hist_out /*[8][256]*/) {
  __shared__ uint32_t h[4][8][RADIX];   // [wave][byte][bin]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < 4 * 8 * RADIX; i += 256) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const uint64_t k0 = keys[0];
  uint64_t m = 0;
  auto add = [&](uint64_t k, bool valid) {
    m |= valid ? k ^ k0 : 0ull;
    wave_hist_add(h[w], k, valid, nd);
  };
  const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(keys);
  const uint64_t npair = n >> 1;
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  // every lane runs the same trip count (the ballots need the whole wave)
  for (uint64_t q0 = (uint64_t)blockIdx.x * 256u; q0 < npair; q0 += stride) {
    const uint64_t q = q0 + tid;
    const bool ok = q < npair;
    const ulonglong2 x = ok ? k2[q] : make_ulonglong2(0, 0);
    add(x.x, ok);
    add(x.y, ok);
  }
  if (n & 1) {
    if (blockIdx.x == 0 && w == 0) add(keys[n - 1], lane == 0);
  }
  m = wave_or(m);
  if (lane == 0 && m) atomicOr(mask_out, (unsigned long long)m);
  __syncthreads();
  flush_hist<4>(h, nd, hist_out);
}

// ---- k_keyinfo ------------------------------------------------------------------------------
// nd = number of low key bytes to histogram (the ctx predicts it from the previous window; a
// window that needs more gets k_hist_bytes for the rest)
template <int DIR, bool VEC>
__global__ __launch_bounds__(256) void k_keyinfo(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                 uint64_t n, int nd, unsigned long long* __restrict__ mask_out,
                                                 uint32_t* __restrict__ hist_out /*[4][256]*/) {
  __shared__ uint32_t h[4][4][RADIX];  // [wave][byte][bin]
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = tid; i < 4 * 4 * RADIX; i += 256) (&h[0][0][0])[i] = 0;
  __syncthreads();
  const uint64_t k0 = (uint64_t)((DIR == DIR_IN) ? dst[0] : src[0]);
  uint64_t m = 0;
  auto add = [&](uint64_t k) {
    m |= k ^ k0;
    if (nd > 0) atomicAdd(&h[w][0][k & 255u], 1u);   // nd = 0: the mask alone
    if (nd > 1) atomicAdd(&h[w][1][(k >> 8) & 255u], 1u);
    if (nd > 2) atomicAdd(&h[w][2][(k >> 16) & 255u], 1u);
    if (nd > 3) atomicAdd(&h[w][3][(k >> 24) & 255u], 1u);
  };
  if constexpr (!VEC) {   // columns not 16-byte aligned (caller-provided slices)
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + tid; i < n; i += stride) {
      if (DIR != DIR_IN) add((uint64_t)src[i]);
      if (DIR != DIR_OUT) add((uint64_t)dst[i]);
    }
  } else {
  // 16-byte loads, 4 in flight per column per thread: 8 keys per column per iteration
  const uint64_t npair = n >> 1;
  const longlong2* s2 = reinterpret_cast<const longlong2*>(src);
  const longlong2* d2 = reinterpret_cast<const longlong2*>(dst);
  const uint64_t stride = (uint64_t)gridDim.x * 1024u;
  for (uint64_t q = (uint64_t)blockIdx.x * 1024u + tid; q < npair; q += stride) {
    longlong2 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t qq = q + 256u * u;
      if (qq < npair) {
        if (DIR != DIR_IN) a[u] = s2[qq];
        if (DIR != DIR_OUT) b[u] = d2[qq];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (q + 256u * u < npair) {
        if (DIR != DIR_IN) { add((uint64_t)a[u].x); add((uint64_t)a[u].y); }
        if (DIR != DIR_OUT) { add((uint64_t)b[u].x); add((uint64_t)b[u].y); }
      }
    }
  }
  if ((n & 1) && blockIdx.x == 0 && tid == 0) {
    if (DIR != DIR_IN) add((uint64_t)src[n - 1]);
    if (DIR != DIR_OUT) add((uint64_t)dst[n - 1]);
  }
  }
  m = wave_or(m);
  if ((tid & 63) == 0 && m) atomicOr(mask_out, (unsigned long long)m);
  __syncthreads();
  for (int i = tid; i < nd * RADIX; i += 256) {
    const uint32_t c = h[0][0][i] + h[1][0][i] + h[2][0][i] + h[3][0][i];
    if (c) atomicAdd(&hist_out[i], c);
  }
}

// histograms of key bytes [b0, b1) of (key ^ key_xor) — the bytes keyinfo did not predict
template <int DIR>
__global__ __launch_bounds__(256) void k_hist_bytes(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                    uint64_t n, uint64_t key_xor, int b0, int b1,
                                                    uint32_t* __restrict__ hist_out /*[8][256]*/) {
  __shared__ uint32_t h[8][RADIX];
  const int tid = threadIdx.x;
  for (int i = tid; i < 8 * RADIX; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  auto add = [&](uint64_t k) {
    k ^= key_xor;
    for (int b = b0; b < b1; ++b) atomicAdd(&h[b][(k >> (8 * b)) & 255u], 1u);
  };
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + tid; i < n; i += stride) {
    if (DIR != DIR_IN) add((uint64_t)src[i]);
    if (DIR != DIR_OUT) add((uint64_t)dst[i]);
  }
  __syncthreads();
  for (int i = tid + b0 * RADIX; i < b1 * RADIX; i += 256) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&hist_out[i], c);
  }
}

// hist[p][256] -> base[p][256] exclusive scans, one wave-parallel scan per pass (block = 256)
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_digit_base(const uint32_t* __restrict__ hist, uint32_t* __restrict__ base,
                                                    int passes) {
  __shared__ uint32_t wsum[4];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  for (int p = 0; p < passes; ++p) {
    const uint32_t c = hist[p * RADIX + tid];
    const uint32_t inc = wave_inclusive_sum(c);
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (int i = 0; i < w; ++i) off += wsum[i];
    base[p * RADIX + tid] = off + inc - c;
    __syncthreads();
  }
}

// ---- wider digits (9 bits: one LSD pass less where 8-bit digits would leave a pass 1-2 bits wide) --
// The histograms of every DBITS-bit digit of a u64 key buffer, one table per wave as wave_hist_add (the
// wave's leading bin counted once), into hist_out[nd][1 << DBITS]
template <int DBITS>
__global__ __launch_bounds__(256) void k_hist_digits(const uint64_t* __restrict__ keys, uint64_t n, int nd,
                                                     uint32_t* __restrict__ hist_out) {
  constexpr int R = 1 << DBITS, MAXD = (64 + DBITS - 1) / DBITS;
  __shared__ uint32_t h[4][MAXD * R];
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = tid; i < 4 * MAXD * R; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  const uint64_t lt = (1ull << (tid & 63)) - 1;
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  for (uint64_t q0 = (uint64_t)blockIdx.x * 256u; q0 < n; q0 += stride) {   // same trip count on every lane
    const uint64_t q = q0 + tid;
    const bool valid = q < n;
    const uint64_t k = valid ? keys[q] : 0ull;
    for (int b = 0; b < nd; ++b) {
      const uint32_t d = (uint32_t)(k >> (DBITS * b)) & (R - 1);
      const uint32_t L = __builtin_amdgcn_readfirstlane(d);
      const uint64_t same = __ballot(valid && d == L);
      if (valid && d == L) {
        if ((same & lt) == 0) atomicAdd(&h[w][b * R + L], (uint32_t)__popcll(same));
      } else if (valid) {
        atomicAdd(&h[w][b * R + d], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < nd * R; i += 256) {
    const uint32_t c = h[0][i] + h[1][i] + h[2][i] + h[3][i];
    if (c) atomicAdd(&hist_out[i], c);
  }
}

// hist[p][R] -> base[p][R] exclusive scans (block = R threads)
template <int DBITS>
__global__ __launch_bounds__(1 << DBITS) void k_digit_base_bits(const uint32_t* __restrict__ hist, uint32_t* __restrict__ base,
                                                               int passes) {
  constexpr int R = 1 << DBITS, NW = R / WAVE;
  __shared__ uint32_t wsum[NW];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  for (int p = 0; p < passes; ++p) {
    const uint32_t c = hist[p * R + tid];
    const uint32_t inc = wave_inclusive_sum(c);
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (int i = 0; i < w; ++i) off += wsum[i];
    base[p * R + tid] = off + inc - c;
    __syncthreads();
  }
}

// ---- k_onesweep ------------------------------------------------------------------------------
// One stable counting-sort pass on digit (key >> shift) & (2^DBITS - 1) over records [0, n).
// Tile = BLOCK*ITEMS records, wave-striped (wave w owns records [w*ITEMS*64, (w+1)*ITEMS*64)
// of the tile, item j at lane l is record j*64 + l), so (wave, item, lane) order == record order
// and ranking in that order keeps the pass stable.
// DBITS: digit width (8 for the full LSD sort; 4-6 for the bucket path's partition passes).
// KO: stored key type — the bucket path's last pass stores only the low 16 bits (the bucket-local
// vertex index; the bucket itself is implied by the position).
template <typename K, typename V, bool HAS_V, int BLOCK, int ITEMS, class Src, int DBITS = RADIX_BITS,
          typename KO = K>
__global__ __launch_bounds__(BLOCK) void k_onesweep(Src src, KO* __restrict__ kout, V* __restrict__ vout, uint32_t n,
                                                    uint32_t shift, const uint32_t* __restrict__ digit_base,
                                                    uint64_t* __restrict__ status, uint32_t* __restrict__ tile_ctr,
                                                    uint32_t epoch, uint32_t* __restrict__ timeout) {
  constexpr int RADIX = 1 << DBITS;
  static_assert(BLOCK >= RADIX && BLOCK % WAVE == 0, "one thread per digit");
  constexpr int NW = BLOCK / WAVE;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int XBYTES = (sizeof(K) > sizeof(V) || !HAS_V) ? sizeof(K) : sizeof(V);
  // per-wave digit counters: 16-bit for wider digits (a tile's counts fit; 512 bins x 8 waves in 8 KiB keeps
  // two blocks per CU with an 8-byte exchange tile)
  using WH = std::conditional_t<(DBITS > 8), uint16_t, uint32_t>;
  static_assert(DBITS <= 8 || TILE < 65536, "16-bit wave counters");
  __shared__ WH s_whist[NW][RADIX];
  __shared__ uint32_t s_start[RADIX];
  __shared__ uint32_t s_goff[RADIX];
  __shared__ uint32_t s_wtot[NW];
  __shared__ uint32_t s_tile;
  __shared__ __attribute__((aligned(16))) unsigned char s_x[TILE * XBYTES];
  K* s_keys = reinterpret_cast<K*>(s_x);
  V* s_vals = reinterpret_cast<V*>(s_x);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < NW * RADIX; i += BLOCK) (&s_whist[0][0])[i] = 0;
  if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t tbase = tile * (uint32_t)TILE;
  if (tbase >= n) return;   // defensive: a stale counter can never index past the input
  const uint32_t tile_n = min((uint32_t)TILE, n - tbase);

  // load (wave-striped) + rank within the wave, in record order
  K key[ITEMS];
  V val[ITEMS];
  uint32_t pos[ITEMS];
  const uint32_t wrec = tbase + (uint32_t)wid * (ITEMS * WAVE) + lane;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t r = wrec + j * WAVE;
    src.load(r < n ? r : n - 1, key[j], val[j]);   // unconditional: a load under a branch serialises
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t r = wrec + j * WAVE;
    const bool valid = r < n;
    const uint32_t d = valid ? (uint32_t)(key[j] >> shift) & (RADIX - 1) : 0u;
    const uint64_t active = ballot(valid);
    const uint64_t peers = match_digit<DBITS>(d, active);
    const uint32_t lt = mbcnt(peers);
    uint32_t base = 0;
    if (valid) base = s_whist[wid][d];
    pos[j] = base + lt;
    if (valid && lt == 0) s_whist[wid][d] = (WH)(base + (uint32_t)__popcll(peers));
  }
  __syncthreads();

  // per digit: wave prefix, tile count, publish aggregate, then decoupled look-back
  uint32_t cnt = 0;
  if (tid < RADIX) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t c = s_whist[w][tid];
      s_whist[w][tid] = (WH)cnt;
      cnt += c;
    }
    uint64_t* st = status + (uint64_t)tile * RADIX + tid;
    if (tile == 0) st_agent(st, granule(FLAG_INC, epoch, (uint64_t)digit_base[tid] + cnt));
    else st_agent(st, granule(FLAG_AGG, epoch, cnt));
  }
  // exclusive scan of the digit counts -> tile-local digit starts
  if (tid < RADIX) {
    const uint32_t inc = wave_inclusive_sum(cnt);
    if (lane == (RADIX < WAVE ? RADIX - 1 : WAVE - 1)) s_wtot[wid] = inc;
    s_start[tid] = inc - cnt;
  }
  __syncthreads();
  if (tid < RADIX) {
    uint32_t off = 0;
    for (int w = 0; w < wid; ++w) off += s_wtot[w];
    s_start[tid] += off;
    uint64_t excl;
    if (tile == 0) {
      excl = digit_base[tid];
    } else {
      excl = 0;
      for (int64_t k = (int64_t)tile - 1; k >= 0; --k) {
        const uint64_t g = poll_granule(status + (uint64_t)k * RADIX + tid, epoch, timeout);
        excl += g_value(g);
        if (g_flag(g) == FLAG_INC) break;
      }
      st_agent(status + (uint64_t)tile * RADIX + tid, granule(FLAG_INC, epoch, excl + cnt));
    }
    s_goff[tid] = (uint32_t)excl;
  }
  __syncthreads();

  // exchange keys through LDS into digit order, then scatter runs of consecutive addresses
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t r = wrec + j * WAVE;
    if (r < n) {
      const uint32_t d = (uint32_t)(key[j] >> shift) & (RADIX - 1);
      pos[j] += s_start[d] + s_whist[wid][d];
      s_keys[pos[j]] = key[j];
    }
  }
  __syncthreads();
  uint32_t gpos[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = (uint32_t)j * BLOCK + tid;
    if (i < tile_n) {
      const K k = s_keys[i];
      const uint32_t d = (uint32_t)(k >> shift) & (RADIX - 1);
      gpos[j] = s_goff[d] + i - s_start[d];
      kout[gpos[j]] = (KO)k;
    }
  }
  if constexpr (HAS_V) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t r = wrec + j * WAVE;
      if (r < n) s_vals[pos[j]] = val[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = (uint32_t)j * BLOCK + tid;
      if (i < tile_n) vout[gpos[j]] = s_vals[i];
    }
  }
}

}  // namespace gs
