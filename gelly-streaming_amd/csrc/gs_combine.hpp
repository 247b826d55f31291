// gs_combine.hpp — the last LSD pass fused with the per-vertex combine.
//
// After passes 0..P-2 the records are sorted by the low key digits.  The last pass ranks each tile
// by the top digit; inside the tile the records are then sorted by the FULL key (stable ranking
// keeps the low-digit order), so every vertex's records in that tile are adjacent.  This kernel
// reduces each such run in LDS (the EdgesReduce / EdgesFold combine, GraphWindowStream.java:62-121)
// and scatters one (vertex, partial) per run instead of every record.  A vertex whose records span
// k tiles leaves k adjacent partials; k_reduce_by_key with the merge op finishes them.
//
// Output layout: partials of digit d are written densely from digit_base[d] (the record-count
// region start, known from the histogram); the look-back runs on per-digit RUN counts, so region d
// ends at the last tile's inclusive granule.  k_region_table / k_compact_runs squeeze the gaps out.
#pragma once
#include "gs_radix.hpp"
#include "gs_rbk.hpp"

namespace gs {

// merge op for the partials the combine pass emits (In = Acc of the combine op)
template <class Op>
struct MergeOf {
  using type = Op;  // ValueOp<T, OP>: In == Acc == T
};
struct CountMergeOp {
  using In = uint64_t;
  using Acc = uint64_t;
  static constexpr bool HAS_V = true;
  __device__ static Acc from(In v) { return v; }
  __device__ static Acc combine(Acc a, Acc b) { return a + b; }
};
template <>
struct MergeOf<CountOp> {
  using type = CountMergeOp;
};
struct DegMaxMergeOp {
  using In = DegMax;
  using Acc = DegMax;
  static constexpr bool HAS_V = true;
  __device__ static Acc from(In v) { return v; }
  __device__ static Acc combine(Acc a, Acc b) { return DegMaxOp::combine(a, b); }
};
template <>
struct MergeOf<DegMaxOp> {
  using type = DegMaxMergeOp;
};

template <typename K, class Op, int BLOCK, int ITEMS, class Src>
__global__ __launch_bounds__(BLOCK) void k_onesweep_combine(Src src, K* __restrict__ kout,
                                                            typename Op::Acc* __restrict__ aout, uint32_t n,
                                                            uint32_t shift, const uint32_t* __restrict__ digit_base,
                                                            uint64_t* __restrict__ status,
                                                            uint32_t* __restrict__ tile_ctr, uint32_t epoch,
                                                            uint32_t* __restrict__ timeout) {
  static_assert(BLOCK >= RADIX && BLOCK % WAVE == 0, "one thread per digit");
  using In = typename Op::In;
  using Acc = typename Op::Acc;
  using S = Seg<Acc>;
  constexpr int NW = BLOCK / WAVE;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int PT = TILE + TILE / 32 + 2;
  using V = std::conditional_t<Op::HAS_V, In, uint8_t>;
  __shared__ uint32_t s_whist[NW][RADIX];
  __shared__ uint32_t s_start[RADIX];
  __shared__ uint32_t s_rcnt[RADIX];
  __shared__ uint32_t s_rstart[RADIX];
  __shared__ uint32_t s_hcnt[BLOCK + 1];   // heads before each thread's first record (+ total)
  __shared__ uint32_t s_hmask[BLOCK];      // each thread's head bitmask
  __shared__ uint32_t s_goff[RADIX];
  __shared__ uint32_t s_wtot[NW];
  __shared__ S s_wagg[NW];
  __shared__ uint32_t s_tile;
  __shared__ K s_keys[PT];
  __shared__ __attribute__((aligned(16))) V s_vals[Op::HAS_V ? PT : 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < NW * RADIX; i += BLOCK) (&s_whist[0][0])[i] = 0;
  if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t tbase = tile * (uint32_t)TILE;
  if (tbase >= n) return;
  const uint32_t tile_n = min((uint32_t)TILE, n - tbase);

  // 1. load (wave-striped) + stable rank by the top digit (as k_onesweep)
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
    const uint64_t peers = match_digit<RADIX_BITS>(d, active);
    const uint32_t lt = mbcnt(peers);
    uint32_t base = 0;
    if (valid) base = s_whist[wid][d];
    pos[j] = base + lt;
    if (valid && lt == 0) s_whist[wid][d] = base + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  uint32_t cnt = 0;
  if (tid < RADIX) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t c = s_whist[w][tid];
      s_whist[w][tid] = cnt;
      cnt += c;
    }
    const uint32_t inc = wave_inclusive_sum(cnt);
    if (lane == 63) s_wtot[wid] = inc;
    s_start[tid] = inc - cnt;
  }
  __syncthreads();
  if (tid < RADIX) {
    uint32_t off = 0;
    for (int w = 0; w < wid; ++w) off += s_wtot[w];
    s_start[tid] += off;
  }
  __syncthreads();

  // 2. records into LDS in full-key order (padded for the blocked reads below)
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t r = wrec + j * WAVE;
    if (r < n) {
      const uint32_t d = (uint32_t)(key[j] >> shift) & (RADIX - 1);
      const uint32_t p = pos[j] + s_start[d] + s_whist[wid][d];
      s_keys[pad32(p)] = key[j];
      if constexpr (Op::HAS_V) s_vals[pad32(p)] = val[j];
    }
  }
  __syncthreads();

  // 3. tile-local reduce-by-key: thread owns ITEMS consecutive sorted records
  const uint32_t first = (uint32_t)tid * ITEMS;
  const uint32_t mine = first < tile_n ? min((uint32_t)ITEMS, tile_n - first) : 0u;
  S agg;
  agg.cnt = 0;
  agg.valid = mine > 0;
  uint32_t headmask = 0;
  {
    K pk = first > 0 ? s_keys[pad32(first - 1)] : (K)0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      if ((uint32_t)j < mine) {
        const K k = s_keys[pad32(first + j)];
        In x{};
        if constexpr (Op::HAS_V) x = s_vals[pad32(first + j)];
        const bool head = (first + j == 0) || k != pk;
        const Acc a = Op::from(x);
        if (head) {
          headmask |= 1u << j;
          agg.cnt++;
          agg.v = a;
        } else {
          agg.v = (j == 0) ? a : Op::combine(agg.v, a);
        }
        pk = k;
      }
    }
  }
  S inc = agg;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    S y;
    y.cnt = __shfl_up(inc.cnt, o, WAVE);
    y.valid = __shfl_up(inc.valid, o, WAVE);
    y.v = shfl_up_acc(inc.v, o);
    if (lane >= o) inc = seg_combine<Op>(y, inc);
  }
  S excl;
  excl.cnt = __shfl_up(inc.cnt, 1, WAVE);
  excl.valid = __shfl_up(inc.valid, 1, WAVE);
  excl.v = shfl_up_acc(inc.v, 1);
  if (lane == 0) {
    excl.valid = 0;
    excl.cnt = 0;
  }
  if (lane == 63) s_wagg[wid] = inc;
  __syncthreads();
  S start;
  start.cnt = 0;
  start.valid = 0;
  for (int w = 0; w < wid; ++w) start = seg_combine<Op>(start, s_wagg[w]);
  start = seg_combine<Op>(start, excl);
  s_hcnt[tid] = start.cnt;
  s_hmask[tid] = headmask;
  if (tid == BLOCK - 1) s_hcnt[BLOCK] = start.cnt + __popc(headmask);

  // runs that END at item j of this thread: partial kept in ra[j] (static index: stays in registers);
  // key re-read from LDS and run index recomputed from the head mask at scatter time
  Acc ra[ITEMS];
  uint32_t endmask = 0;
  {
    Acc run = start.v;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      if ((uint32_t)j < mine) {
        const K k = s_keys[pad32(first + j)];
        In x{};
        if constexpr (Op::HAS_V) x = s_vals[pad32(first + j)];
        const Acc a = Op::from(x);
        run = (headmask & (1u << j)) ? a : Op::combine(run, a);
        const uint32_t nx = first + j + 1;
        if (nx >= tile_n || s_keys[pad32(nx)] != k) endmask |= 1u << j;
        ra[j] = run;
      }
    }
  }
  __syncthreads();

  // 4. per digit: runs of digit d = heads in its record range [s_start[d], s_start[d] + cnt) — read off the
  //    owners' head masks (no atomics: runs of one digit are adjacent, so per-run counters would all collide)
  if (tid < RADIX) {
    auto heads_before = [&](uint32_t p) -> uint32_t {
      if (p >= tile_n) return s_hcnt[BLOCK];
      const uint32_t t = p / ITEMS, o = p % ITEMS;
      return s_hcnt[t] + __popc(s_hmask[t] & ((1u << o) - 1u));
    };
    const uint32_t h0 = heads_before(s_start[tid]);
    const uint32_t rc = cnt ? heads_before(s_start[tid] + cnt) - h0 : 0u;
    s_rcnt[tid] = rc;
    uint64_t* st = status + (uint64_t)tile * RADIX + tid;
    if (tile == 0) st_agent(st, granule(FLAG_INC, epoch, (uint64_t)digit_base[tid] + rc));
    else st_agent(st, granule(FLAG_AGG, epoch, rc));
    s_rstart[tid] = h0;   // runs are in digit order: the first run of digit d has index H(start of d)
  }
  __syncthreads();
  if (tid < RADIX) {
    uint64_t ex;
    if (tile == 0) {
      ex = digit_base[tid];
    } else {
      ex = 0;
      for (int64_t k = (int64_t)tile - 1; k >= 0; --k) {
        const uint64_t g = poll_granule(status + (uint64_t)k * RADIX + tid, epoch, timeout);
        ex += g_value(g);
        if (g_flag(g) == FLAG_INC) break;
      }
      st_agent(status + (uint64_t)tile * RADIX + tid, granule(FLAG_INC, epoch, ex + s_rcnt[tid]));
    }
    s_goff[tid] = (uint32_t)ex;
  }
  __syncthreads();

  // 5. scatter the partials
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    if (endmask & (1u << j)) {
      const K k = s_keys[pad32(first + j)];
      const uint32_t ri = start.cnt + __popc(headmask & ((2u << j) - 1u)) - 1u;
      const uint32_t d = (uint32_t)(k >> shift) & (RADIX - 1);
      const uint32_t g = s_goff[d] + ri - s_rstart[d];
      kout[g] = k;
      aout[g] = ra[j];
    }
  }
}

// region d of the partial array = [digit_base[d], end[d]); end from the last tile's INCLUSIVE granule.
// table[0..255] = physical starts, table[256..512] = logical starts (table[512] = total partials)
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_region_table(const uint64_t* __restrict__ status, uint32_t last_tile,
                                                             const uint32_t* __restrict__ digit_base,
                                                             uint32_t* __restrict__ table,
                                                             unsigned long long* __restrict__ total) {
  __shared__ uint32_t ws[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t base = digit_base[tid];
  const uint32_t end = (uint32_t)g_value(status[(uint64_t)last_tile * RADIX + tid]);
  const uint32_t len = end - base;
  const uint32_t inc = wave_inclusive_sum(len);
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t off = 0;
  for (int i = 0; i < w; ++i) off += ws[i];
  table[tid] = base;
  table[RADIX + tid] = off + inc - len;
  if (tid == RADIX - 1) {
    table[2 * RADIX] = off + inc;
    *total = off + inc;
  }
}

template <typename K, typename Acc>
__global__ __launch_bounds__(256) void k_compact_runs(const K* __restrict__ kin, const Acc* __restrict__ ain,
                                                      const uint32_t* __restrict__ table, uint32_t total,
                                                      K* __restrict__ kout, Acc* __restrict__ aout) {
  __shared__ uint32_t s_phys[RADIX];
  __shared__ uint32_t s_log[RADIX + 1];
  for (int i = threadIdx.x; i < RADIX; i += 256) s_phys[i] = table[i];
  for (int i = threadIdx.x; i <= RADIX; i += 256) s_log[i] = table[RADIX + i];
  __syncthreads();
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    int lo = 0, hi = RADIX - 1;   // last region with logical start <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_log[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t p = s_phys[lo] + (i - s_log[lo]);
    kout[i] = kin[p];
    aout[i] = ain[p];
  }
}

}  // namespace gs
