// gs_rbk.hpp — single-pass segmented reduce (reduce-by-key) over the sorted window.
//
// Replaces Flink's per-edge reducing / folding window state:
//   reduceOnEdges  EdgesReduceFunction.reduce   GraphWindowStream.java:107-121 (+ project(0,2) :102-103)
//   foldNeighbors  EdgesFoldFunction.fold        GraphWindowStream.java:67-87
// Input: keys sorted (stable, so each vertex's values are in arrival order) + payload.
// Output: one (vertex, aggregate) per run of equal keys, vertices ascending.
//
// Edge-balanced: every thread owns ITEMS consecutive records regardless of where vertex
// boundaries fall, so a hub vertex with millions of records is spread over many tiles and
// carried across them by a decoupled look-back on (#segment heads, trailing partial) — the
// segmented-scan operator  (c1,v1) (+) (c2,v2) = (c1+c2, c2 > 0 ? v2 : op(v1, v2)).
// One read of keys+payload, one write per vertex: the HBM roofline kernel of the window.
#pragma once
#include <type_traits>

#include "gs_device.hpp"

namespace gs {

// ---- built-in associative ops (Java semantics) ------------------------------------------------
__device__ __forceinline__ double java_min(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && __signbit(b)) return b;
  return (a <= b) ? a : b;
}
__device__ __forceinline__ double java_max(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && __signbit(a)) return b;
  return (a >= b) ? a : b;
}
__device__ __forceinline__ float java_min(float a, float b) {
  if (a != a) return a;
  if (a == 0.0f && b == 0.0f && __signbitf(b)) return b;
  return (a <= b) ? a : b;
}
__device__ __forceinline__ float java_max(float a, float b) {
  if (a != a) return a;
  if (a == 0.0f && b == 0.0f && __signbitf(a)) return b;
  return (a >= b) ? a : b;
}

enum : int { OP_SUM = 0, OP_MIN = 1, OP_MAX = 2, OP_COUNT = 3 };

// T in {int32_t, int64_t, float, double}; Acc == T; integer sums wrap (unsigned adds)
template <typename T, int OP>
struct ValueOp {
  using In = T;
  using Acc = T;
  static constexpr bool HAS_V = true;
  __device__ static Acc from(In v) { return v; }
  __device__ static Acc combine(Acc a, Acc b) {
    if constexpr (OP == OP_SUM) {
      if constexpr (std::is_integral_v<T>) return (T)((std::make_unsigned_t<T>)a + (std::make_unsigned_t<T>)b);
      else return a + b;
    } else if constexpr (OP == OP_MIN) {
      if constexpr (std::is_integral_v<T>) return b < a ? b : a;
      else return java_min(a, b);
    } else {
      if constexpr (std::is_integral_v<T>) return b > a ? b : a;
      else return java_max(a, b);
    }
  }
};

struct CountOp {
  using In = uint8_t;  // no payload
  using Acc = uint64_t;
  static constexpr bool HAS_V = false;
  __device__ static Acc from(In) { return 1; }
  __device__ static Acc combine(Acc a, Acc b) { return a + b; }
};

struct DegMax {
  uint64_t cnt;
  int64_t mx;
};
struct DegMaxOp {
  using In = int64_t;  // neighbour ID
  using Acc = DegMax;
  static constexpr bool HAS_V = true;
  __device__ static Acc from(In v) { return {1ull, v}; }
  __device__ static Acc combine(Acc a, Acc b) { return {a.cnt + b.cnt, b.mx > a.mx ? b.mx : a.mx}; }
};

// ---- outputs -------------------------------------------------------------------------------------
// reduceOnEdges: vals[u] = acc;  foldNeighbors: vals[u] = op(init, acc)
template <class Op, bool HAS_INIT>
struct ValueOut {
  int64_t* keys;
  typename Op::Acc* vals;
  typename Op::Acc init;
  __device__ void store(uint32_t u, int64_t k, typename Op::Acc a, uint32_t) const {
    keys[u] = k;
    vals[u] = HAS_INIT ? Op::combine(init, a) : a;
  }
};
struct CountOut {
  int64_t* keys;
  int64_t* vals;
  int64_t init;
  __device__ void store(uint32_t u, int64_t k, uint64_t a, uint32_t) const {
    keys[u] = k;
    vals[u] = (int64_t)((uint64_t)init + a);
  }
};
// distinct keys of a sorted array (key_xor = 0): keys[u] = key, counts[u] = multiplicity (optional)
struct UniqueOut {
  uint64_t* keys;
  uint32_t* counts;
  __device__ void store(uint32_t u, int64_t k, uint64_t a, uint32_t) const {
    keys[u] = (uint64_t)k;
    if (counts) counts[u] = (uint32_t)a;
  }
};
// CSR: offsets[u+1] = one past the last record of vertex u (offsets[0] = 0 is set by the host)
struct CsrOut {
  int64_t* keys;
  uint64_t* offsets;
  __device__ void store(uint32_t u, int64_t k, uint64_t, uint32_t end_pos) const {
    keys[u] = k;
    offsets[u + 1] = (uint64_t)end_pos + 1;
  }
};
struct DegMaxOut {
  int64_t* keys;
  int64_t* deg;
  int64_t* mx;
  int64_t init_max;
  __device__ void store(uint32_t u, int64_t k, DegMax a, uint32_t) const {
    keys[u] = k;
    deg[u] = (int64_t)a.cnt;
    mx[u] = a.mx > init_max ? a.mx : init_max;
  }
};
template <typename Acc>
struct Seg {
  uint32_t cnt;    // segment heads
  uint32_t valid;  // 0 = identity
  Acc v;           // trailing partial
};

template <typename Acc>
__device__ __forceinline__ Acc shfl_up_acc(Acc a, int o) {
  static_assert(sizeof(Acc) % 4 == 0, "acc of dwords");
  union U {
    Acc a;
    uint32_t w[sizeof(Acc) / 4];
  } u;
  u.a = a;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(Acc) / 4); ++i) u.w[i] = __shfl_up(u.w[i], o, WAVE);
  return u.a;
}

template <typename Acc>
__device__ __forceinline__ Acc shfl_down_acc(Acc a, int o) {
  union U {
    Acc a;
    uint32_t w[sizeof(Acc) / 4];
  } u;
  u.a = a;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(Acc) / 4); ++i) u.w[i] = __shfl_down(u.w[i], o, WAVE);
  return u.a;
}
template <typename Acc>
__device__ __forceinline__ Acc shfl_acc(Acc a, int src) {
  union U {
    Acc a;
    uint32_t w[sizeof(Acc) / 4];
  } u;
  u.a = a;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(Acc) / 4); ++i) u.w[i] = __shfl(u.w[i], src, WAVE);
  return u.a;
}

template <class Op>
__device__ __forceinline__ Seg<typename Op::Acc> seg_combine(Seg<typename Op::Acc> a, Seg<typename Op::Acc> b) {
  if (!b.valid) return a;
  if (!a.valid) return b;
  Seg<typename Op::Acc> r;
  r.cnt = a.cnt + b.cnt;
  r.valid = 1;
  r.v = b.cnt > 0 ? b.v : Op::combine(a.v, b.v);
  return r;
}

constexpr int accum_slots(int bytes) { return (bytes + 7) / 8; }

template <typename Acc>
__device__ __forceinline__ void store_acc(uint64_t* p, Acc a) {
  union {
    Acc a;
    uint64_t w[accum_slots(sizeof(Acc))];
  } u;
  u.w[accum_slots(sizeof(Acc)) - 1] = 0;
  u.a = a;
#pragma unroll
  for (int i = 0; i < accum_slots(sizeof(Acc)); ++i) st_agent(p + i, u.w[i]);
}
template <typename Acc>
__device__ __forceinline__ Acc load_acc(uint64_t* p) {
  union {
    Acc a;
    uint64_t w[accum_slots(sizeof(Acc))];
  } u;
#pragma unroll
  for (int i = 0; i < accum_slots(sizeof(Acc)); ++i) u.w[i] = ld_agent(p + i);
  return u.a;
}

__device__ __forceinline__ uint32_t pad32(uint32_t i) { return i + (i >> 5); }

// keys: sorted compact keys; vals: payload in the same order (unused when !Op::HAS_V)
template <typename K, class Op, class Out, int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_reduce_by_key(const K* __restrict__ keys, const typename Op::In* __restrict__ vals,
                                                         uint32_t n, uint64_t key_xor, uint32_t key_shift, Out out,
                                                         uint64_t* __restrict__ st_word,
                                                         uint64_t* __restrict__ st_agg, uint64_t* __restrict__ st_inc,
                                                         uint32_t* __restrict__ tile_ctr, uint32_t ntiles, uint32_t epoch,
                                                         uint32_t* __restrict__ timeout, unsigned long long* __restrict__ n_unique) {
  using Acc = typename Op::Acc;
  using In = typename Op::In;
  using S = Seg<Acc>;
  constexpr int NW = BLOCK / WAVE;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int SLOTS = accum_slots(sizeof(Acc));
  __shared__ K s_k[TILE + TILE / 32 + 2];
  __shared__ __attribute__((aligned(16))) In s_v[Op::HAS_V ? TILE + TILE / 32 + 2 : 1];
  __shared__ S s_wagg[NW];
  __shared__ S s_prefix;
  __shared__ K s_prev, s_next;
  __shared__ uint32_t s_tile;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  if (tile >= ntiles) return;   // defensive: a stale counter can never index past the input
  const uint32_t tbase = tile * (uint32_t)TILE;
  const uint32_t tile_n = min((uint32_t)TILE, n - tbase);

  // striped coalesced load into padded LDS
  K lk[ITEMS];
  In lv[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {   // unconditional (clamped) loads: a load under a branch serialises
    const uint32_t i = min((uint32_t)j * BLOCK + tid, tile_n - 1);
    lk[j] = keys[tbase + i];
    if constexpr (Op::HAS_V) lv[j] = vals[tbase + i];
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = (uint32_t)j * BLOCK + tid;
    if (i < tile_n) {
      s_k[pad32(i)] = lk[j] >> key_shift;
      if constexpr (Op::HAS_V) s_v[pad32(i)] = lv[j];
    }
  }
  if (tid == 0) {
    s_prev = tbase > 0 ? (K)(keys[tbase - 1] >> key_shift) : (K)0;
    s_next = (tbase + tile_n < n) ? (K)(keys[tbase + tile_n] >> key_shift) : (K)0;
  }
  __syncthreads();

  // thread-local: ITEMS consecutive records
  const uint32_t first = (uint32_t)tid * ITEMS;
  const uint32_t mine = first < tile_n ? min((uint32_t)ITEMS, tile_n - first) : 0u;
  K prevk = first == 0 ? s_prev : s_k[pad32(first - 1)];
  const bool has_prev = (tbase + first) > 0;
  S agg;
  agg.cnt = 0;
  agg.valid = mine > 0;
  uint32_t headmask = 0;
  {
    K pk = prevk;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      if ((uint32_t)j < mine) {
        const K k = s_k[pad32(first + j)];
        In x{};
        if constexpr (Op::HAS_V) x = s_v[pad32(first + j)];
        const bool head = (j == 0) ? (!has_prev || k != pk) : (k != pk);
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

  // block exclusive segmented scan of thread aggregates
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
  if (lane == 0) { excl.valid = 0; excl.cnt = 0; }
  if (lane == 63) s_wagg[wid] = inc;
  __syncthreads();

  // tile aggregate -> publish -> wave-parallel decoupled look-back (wave 0: lane l inspects tile-1-l,
  // 64 predecessors per round; the nearest INCLUSIVE granule ends the walk)
  if (wid == 0) {
    S tot = s_wagg[0];
    for (int w = 1; w < NW; ++w) tot = seg_combine<Op>(tot, s_wagg[w]);
    S pre;
    pre.cnt = 0;
    pre.valid = 0;
    uint64_t* w0 = st_word + tile;
    if (tile == 0) {
      if (lane == 0) {
        store_acc(st_inc, tot.v);
        drain_stores();
        st_agent(w0, granule(FLAG_INC, epoch, tot.cnt));
      }
    } else {
      if (lane == 0) {
        store_acc(st_agg + (uint64_t)tile * SLOTS, tot.v);
        drain_stores();
        st_agent(w0, granule(FLAG_AGG, epoch, tot.cnt));
      }
      for (int64_t k = (int64_t)tile - 1;; k -= WAVE) {
        const int64_t kk = k - lane;
        uint64_t g = 0;
        if (kk >= 0) g = poll_granule(st_word + kk, epoch, timeout);
        const bool is_inc = kk >= 0 && g_flag(g) == FLAG_INC;
        const uint64_t incm = ballot(is_inc);
        const int stop = incm ? __builtin_ctzll(incm) : WAVE - 1;   // farthest lane that counts
        S x;
        x.valid = (kk >= 0 && lane <= stop) ? 1u : 0u;
        x.cnt = x.valid ? (uint32_t)g_value(g) : 0u;
        if (x.valid) x.v = load_acc<Acc>((is_inc ? st_inc : st_agg) + (uint64_t)kk * SLOTS);
        // ordered reduction: higher lane = earlier tile
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
          S y;
          y.cnt = __shfl_down(x.cnt, o, WAVE);
          y.valid = __shfl_down(x.valid, o, WAVE);
          y.v = shfl_down_acc(x.v, o);
          if (lane + o < WAVE) x = seg_combine<Op>(y, x);
        }
        S r;
        r.cnt = __shfl(x.cnt, 0, WAVE);
        r.valid = __shfl(x.valid, 0, WAVE);
        r.v = shfl_acc(x.v, 0);
        pre = seg_combine<Op>(r, pre);
        if (incm || k < WAVE) break;   // wave-uniform: an INCLUSIVE was seen or tile 0 covered
      }
      const S all = seg_combine<Op>(pre, tot);
      if (lane == 0) {
        store_acc(st_inc + (uint64_t)tile * SLOTS, all.v);
        drain_stores();
        st_agent(w0, granule(FLAG_INC, epoch, all.cnt));
      }
    }
    if (lane == 0) {
      if (tile == ntiles - 1) *n_unique = (unsigned long long)seg_combine<Op>(pre, tot).cnt;
      s_prefix = pre;
    }
  }
  __syncthreads();

  S wpre = s_prefix;
  for (int w = 0; w < wid; ++w) wpre = seg_combine<Op>(wpre, s_wagg[w]);
  const S start = seg_combine<Op>(wpre, excl);

  // walk: write each segment that ends inside this thread's range
  Acc run = start.v;
  uint32_t hidx = start.cnt;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    if ((uint32_t)j < mine) {
      const K k = s_k[pad32(first + j)];
      In x{};
      if constexpr (Op::HAS_V) x = s_v[pad32(first + j)];
      const Acc a = Op::from(x);
      if (headmask & (1u << j)) {
        run = a;
        hidx++;
      } else {
        run = Op::combine(run, a);
      }
      bool end;
      const uint32_t nx = first + j + 1;
      if (nx < tile_n) end = s_k[pad32(nx)] != k;
      else end = (tbase + nx >= n) || (s_next != k);
      if (end) out.store(hidx - 1, (int64_t)(key_xor ^ (uint64_t)k), run, tbase + first + j);
    }
  }
}

}  // namespace gs
