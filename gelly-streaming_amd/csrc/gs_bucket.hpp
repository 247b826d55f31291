// gs_bucket.hpp — the bucket path for the associative built-ins (reduceOnEdges / foldNeighbors with
// SUM, MIN, MAX, COUNT or the degree / max-neighbour fold).
//
// The reference folds each (vertex, window) group with Flink's reducing / folding window state
// (GraphWindowStream.java:62-87, 101-121).  For an associative and commutative op the fold needs
// the records GROUPED by vertex, not ORDERED within a vertex, so a full LSD sort is more than the
// op requires.  This path sorts only the HIGH bits:
//
//   c = key - base                 (base = window's smallest vertex, or a predicted lower bound)
//   bucket = c >> S                (S = 13..15: 2^S vertices whose accumulators fit one CU's LDS)
//   k_bk_info    one read of the keys: min / max and the histogram of the bucket index;
//   k_bk_plan    one block: per-pass digit bases, bucket starts, the work items;
//   k_onesweep   1-2 LSD passes of 4-6-bit digits over the bucket index (long runs per digit, so
//                the scatter writes are near-sequential); the last pass stores only the low 16 bits;
//   k_bk_accum   one persistent workgroup per CU takes items (bucket, record range), adds every
//                record into LDS accumulators with LDS atomics (ds_add/min/max), then writes the
//                bucket's vertices in ascending order (wave ballot compaction) to a staging area;
//                buckets larger than one item leave LDS slabs that k_bk_merge combines;
//   k_bk_emit    staging -> (vertex, value) outputs, vertices ascending (the sort path's order).
// Integer results are bit-exact (wrapping adds, min / max); f64 / f32 sums are summed in f64 in
// LDS-atomic order, within the API's 1e-5 relative tolerance.  Float MIN / MAX keep the sort path
// (Java's Math.min/max NaN and signed-zero rules have no LDS atomic).
#pragma once
#include <limits>
#include <type_traits>

#include "gs_radix.hpp"
#include "gs_rbk.hpp"

namespace gs {

constexpr int BK_MAXB = 2048;          // buckets (the bucket index has <= 11 bits)
constexpr int BK_INFO_BLOCK = 512;
// (k_bk_accum, packed records, A/B of round 3: the next group's loads in flight during this group's
// atomics, C2 accumulate 0.345 vs 0.331 ms: removed)
#ifndef GS_BK_ACC_BLOCK
#define GS_BK_ACC_BLOCK 1024
#endif
#ifndef GS_BK_ACC_PER_CU
#define GS_BK_ACC_PER_CU 1
#endif
#ifndef GS_BK_PREFETCH
#define GS_BK_PREFETCH 0   // k_bk_accum: the next item's first loads issued before the current item's finalize
                           // (A/B, round 6: accumulate 0.2560 -> 0.2728 ms on C2 -- the barrier after the finalize
                           // waits for them, so they hide nothing and hold VGPRs: off)
#endif
#ifndef GS_BK_FUSED_RESET
#define GS_BK_FUSED_RESET 1   // k_bk_accum: each wave resets its own finalized entries (no block-wide init pass)
#endif
#ifndef GS_BK_S8
#define GS_BK_S8 14   // 2^S vertices per bucket with 8-byte accumulators (BkVal)
#endif
constexpr int BK_ACC_BLOCK = GS_BK_ACC_BLOCK;     // 16 waves: one workgroup per CU (LDS-bound)
constexpr int BK_NW = BK_ACC_BLOCK / WAVE;
constexpr int BK_PLAN_BLOCK = 1024;

struct BkItem {
  uint32_t bucket, begin, end, slab;   // slab = ~0u: the bucket is one item (finalize directly)
};

struct BkStage {
  uint32_t* k;   // compact vertex (c)
  void* a;       // per-vertex accumulator (policy type)
  int64_t* b;    // second accumulator (degree fold: max neighbour)
};

struct BkPlanOut {
  uint32_t* digit_base;    // [2][256]
  uint32_t* bucket_start;  // [NB + 1]
  uint32_t* bucket_count;  // [NB]   outputs per bucket (written by finalize)
  uint32_t* b_items;       // [NB]
  uint32_t* b_slab;        // [NB]   first slab of a multi-item bucket
  uint32_t* mlist;         // [NB]   multi-item buckets
  BkItem* items;
  uint32_t* n_items;       // device scalars
  uint32_t* n_multi;
  // speculative partition (k_sp_scatter_pack): bucket_start holds the regions (read, not written),
  // the counts are the cursors' advance (clamped to the region).  counts_out (either mode, optional):
  // every bucket's count, which the next window's regions are sized from
  const uint32_t* cursor = nullptr;
  uint32_t* counts_out = nullptr;
  unsigned long long* occupied = nullptr;   // speculative: [0] lowest, [1] highest bucket with records
  uint32_t* claim = nullptr;                // k_bk_accum's item counter, zeroed here
  uint32_t* max_items = nullptr;            // the most items of one bucket (k_bk_merge_groups skips when <= 16)
};

// speculative partition: a bucket's region is split into SP_NSEG segments, one per XCD slot, each with
// its own cursor (cursor[x * BK_MAXB + b]).  A region of e - s = T + SP_NSEG·SP_PADSEG records (T the
// predicted count with its relative slack, 4-aligned) gives segment x its share of T,
// T·pre[x] / pre[SP_NSEG] (pre[x] = the window's records in the tiles of slots before x, i.e.
// k_sp_scatter_pack's tile -> slot map), plus SP_PADSEG records of absolute slack.
#ifndef GS_SP_XCD
#define GS_SP_XCD 1
#endif
constexpr uint32_t SP_NSEG = GS_SP_XCD ? 8 : 1;
#ifndef GS_SP_MATCH
#define GS_SP_MATCH 1   // k_sp_scatter (folds): wave-aggregated ranking for the first lane's bucket
#endif
constexpr uint32_t SP_PAD = 1024;                  // absolute slack per bucket
constexpr uint32_t SP_PADSEG = SP_PAD / SP_NSEG;   // ... per segment
static_assert(SP_PADSEG % 4 == 0, "segment starts stay 4-aligned");
// the cursor buffer: SP_NSEG x BK_MAXB cursors | SP_NSEG x BK_MAXB segment ends | ... starts.  k_sp_regions
// writes all three; the later kernels read segment bounds from the tables (no division in their loops).
constexpr uint32_t SP_END_OFF = SP_NSEG * BK_MAXB;
constexpr uint32_t SP_LO_OFF = 2 * SP_NSEG * BK_MAXB;
constexpr uint32_t SP_CUR_WORDS = 3 * SP_NSEG * BK_MAXB;
__device__ __forceinline__ uint32_t sp_lo(const uint32_t* cur, uint32_t x, uint32_t b) {
  return cur[SP_LO_OFF + x * BK_MAXB + b];
}
__device__ __forceinline__ uint32_t sp_hi(const uint32_t* cur, uint32_t x, uint32_t b) {
  return cur[SP_END_OFF + x * BK_MAXB + b];
}
struct SpSlots {
  uint32_t pre[SP_NSEG + 1];
};
// frac[x] = pre[x] / pre[SP_NSEG] in 0.32 fixed point (non-decreasing in x; k_sp_regions)
__device__ inline uint32_t sp_seg_start(uint32_t s, uint32_t e, uint32_t x, const uint32_t* frac) {
  if (x == 0) return s;
  if (x >= SP_NSEG) return e;
  const uint32_t T = e - s - SP_NSEG * SP_PADSEG;
  return s + ((uint32_t)(((uint64_t)T * frac[x]) >> 32) & ~3u) + x * SP_PADSEG;
}

// ---- policies: LDS accumulator layout and the op ------------------------------------------------
template <typename T>
__device__ __forceinline__ T bits_as(uint64_t r) {
  if constexpr (sizeof(T) == 8) return __builtin_bit_cast(T, r);
  else return __builtin_bit_cast(T, (uint32_t)r);
}

// value ops: SUM / MIN / MAX over I32 / I64, SUM over F32 / F64 (accumulated in f64)
template <typename T, int OP>
struct BkVal {
  using Raw = std::conditional_t<sizeof(T) == 4, uint32_t, uint64_t>;
  using Load = Raw;                   // what the scatter loads (Raw: what it stores)
  static constexpr bool REL = false;  // payload stored as an offset from the window base
  using A = std::conditional_t<std::is_floating_point_v<T>, double, T>;
  static constexpr int S = sizeof(A) == 8 ? GS_BK_S8 : 15;
  static constexpr uint32_t W = 1u << S;
  static constexpr bool HAS_V = true;
  static constexpr int PAY = PAY_VAL;
  // presence of a vertex: one byte each (a plain ds_write_b8, no atomic) where it fits next to 8-byte
  // accumulators (128 + 16 KB); a bitmap with ds_or for 4-byte accumulators (2^15 of them)
  static constexpr bool PB = sizeof(A) == 8;
  static constexpr uint32_t PW = PB ? W / 4 : W / 32;   // presence words
  struct Lds {
    A acc[W];
    uint32_t pm[PW];
  };
  // Float SUM (f32 / f64 values, f64 accumulators) starts from -0.0, the additive identity of IEEE
  // arithmetic: x + -0.0 is x for every x, so a vertex whose values are all -0.0 sums to -0.0 as the
  // reference's reduce (which starts from the first value) does -- from +0.0 it summed to +0.0.  A sum that
  // cancels ends at +0.0, so an accumulator that still holds -0.0's bits has seen no record or only -0.0
  // values, which mark presence themselves: the presence byte is written for those records only.
  static constexpr bool FLOAT_SUM = OP == OP_SUM && std::is_floating_point_v<T>;
  __device__ static A identity() {
    if constexpr (FLOAT_SUM) return -0.0;
    if constexpr (OP == OP_SUM) return A(0);
    else if constexpr (OP == OP_MIN) return std::numeric_limits<A>::max();
    else return std::numeric_limits<A>::lowest();
  }
  __device__ static A combine(A a, A b) {
    if constexpr (OP == OP_SUM) {
      if constexpr (std::is_integral_v<A>) return (A)((std::make_unsigned_t<A>)a + (std::make_unsigned_t<A>)b);
      else return a + b;
    } else if constexpr (OP == OP_MIN) return b < a ? b : a;
    else return b > a ? b : a;
  }
  __device__ static void init(Lds& s, int tid) {
    for (uint32_t i = tid; i < W; i += BK_ACC_BLOCK) s.acc[i] = identity();
    for (uint32_t i = tid; i < PW; i += BK_ACC_BLOCK) s.pm[i] = 0;
  }
  // entries [lo, hi) back to the identity by one wave (lo, hi multiples of 32: whole presence words)
  __device__ static void init_range(Lds& s, uint32_t lo, uint32_t hi, int lane) {
    for (uint32_t i = lo + lane; i < hi; i += WAVE) s.acc[i] = identity();
    constexpr uint32_t PER_WORD = PB ? 4 : 32;
    for (uint32_t i = lo / PER_WORD + lane; i < hi / PER_WORD; i += WAVE) s.pm[i] = 0;
  }
  __device__ static void add(Lds& s, uint32_t i, Raw r) {
    const T v = bits_as<T>(r);
    if constexpr (OP == OP_SUM) {
      if constexpr (std::is_integral_v<T>) {
        using U = std::conditional_t<sizeof(T) == 8, unsigned long long, unsigned int>;
        atomicAdd((U*)&s.acc[i], (U)v);
      } else {
        atomicAdd(&s.acc[i], (double)v);
        if (__double_as_longlong((double)v) == (long long)0x8000000000000000ull) mark(s, i);   // -0.0
        return;
      }
    } else if constexpr (OP == OP_MIN) {
      using I = std::conditional_t<sizeof(T) == 8, long long, int>;
      atomicMin((I*)&s.acc[i], (I)v);
    } else {
      using I = std::conditional_t<sizeof(T) == 8, long long, int>;
      atomicMax((I*)&s.acc[i], (I)v);
    }
    mark(s, i);
  }
  __device__ static void mark(Lds& s, uint32_t i) {
    if constexpr (PB) reinterpret_cast<uint8_t*>(s.pm)[i] = 1;
    else atomicOr(&s.pm[i >> 5], 1u << (i & 31));
  }
  // packed records (k_dp/sp_scatter_pack, integer ops): r is a narrow value in [0, PK_ESC) unless esc.
  // An integer accumulator that left its identity has seen a record, and narrow values cannot bring it
  // back (a 64-bit SUM of values in [1, 2^16) over < 2^32 records never wraps to 0; a MIN / MAX of them is
  // never the extreme identity), so presence needs its byte only for escaped values and, for SUM, zero
  // values.  A 32-bit SUM can wrap to exactly 0 (2^16 records of 2^16 - 1 ... ), so Integer SUM marks
  // every record.
  static constexpr bool INFER_PRESENCE = std::is_integral_v<T>;
  static constexpr bool SUM_MARKS_ALL = OP == OP_SUM && sizeof(A) == 4;
  static constexpr bool OP_IS_SUM = OP == OP_SUM;
  __device__ static void add_packed(Lds& s, uint32_t i, Raw r, bool esc) {
    const T v = bits_as<T>(r);
    if constexpr (OP == OP_SUM) {
      using U = std::conditional_t<sizeof(T) == 8, unsigned long long, unsigned int>;
      atomicAdd((U*)&s.acc[i], (U)v);
    } else if constexpr (OP == OP_MIN) {
      using I = std::conditional_t<sizeof(T) == 8, long long, int>;
      atomicMin((I*)&s.acc[i], (I)v);
    } else {
      using I = std::conditional_t<sizeof(T) == 8, long long, int>;
      atomicMax((I*)&s.acc[i], (I)v);
    }
    if (SUM_MARKS_ALL || esc || (OP == OP_SUM && r == 0)) mark(s, i);
  }
  // the common packed record: a narrow value that needs no presence byte (not escaped; for SUM not 0)
  __device__ static void add_narrow(Lds& s, uint32_t i, uint32_t r) {
    if constexpr (OP == OP_SUM) {
      using U = std::conditional_t<sizeof(T) == 8, unsigned long long, unsigned int>;
      atomicAdd((U*)&s.acc[i], (U)r);
    } else if constexpr (OP == OP_MIN) {
      using I = std::conditional_t<sizeof(T) == 8, long long, int>;
      atomicMin((I*)&s.acc[i], (I)r);
    } else {
      using I = std::conditional_t<sizeof(T) == 8, long long, int>;
      atomicMax((I*)&s.acc[i], (I)r);
    }
  }
  __device__ static bool present(const Lds& s, uint32_t i) {
    const bool m = PB ? reinterpret_cast<const uint8_t*>(s.pm)[i] != 0 : ((s.pm[i >> 5] >> (i & 31)) & 1u) != 0;
    if constexpr (INFER_PRESENCE) return m || s.acc[i] != identity();
    else if constexpr (FLOAT_SUM) return m || __double_as_longlong(s.acc[i]) != (long long)0x8000000000000000ull;
    else return m;
  }
  __device__ static void stage(BkStage st, uint32_t pos, const Lds& s, uint32_t i) { ((A*)st.a)[pos] = s.acc[i]; }
  static constexpr uint32_t PWORDS = PW;   // presence words merged by OR
  __device__ static void merge_el(Lds* d, const Lds* g, uint32_t i) { d->acc[i] = combine(d->acc[i], g->acc[i]); }
  __device__ static void merge_pw(Lds* d, const Lds* g, uint32_t w) { d->pm[w] |= g->pm[w]; }
  struct Out {
    int64_t* keys;
    T* vals;
    T init;
    bool has_init;
    // the same output into other arrays (k_bk_owner_emit: a chunk's rows staged in LDS)
    __device__ Out retarget(int64_t* k, void* v, int64_t*) const { return Out{k, (T*)v, init, has_init}; }
  };
  __device__ static void emit(const Out& o, uint64_t u, int64_t key, BkStage st, uint32_t j, int64_t) {
    const A a = ((const A*)st.a)[j];
    o.keys[u] = key;
    if constexpr (std::is_floating_point_v<T>) {
      o.vals[u] = o.has_init ? (T)((double)o.init + a) : (T)a;
    } else {
      o.vals[u] = o.has_init ? ValueOp<T, OP>::combine(o.init, a) : a;
    }
  }
};

// COUNT: the number of incident records (foldNeighbors' init + count)
struct BkCount {
  using Raw = uint8_t;
  using Load = Raw;
  static constexpr bool REL = false;
  using A = uint32_t;
  static constexpr int S = 15;
  static constexpr uint32_t W = 1u << S;
  static constexpr bool HAS_V = false;
  static constexpr int PAY = PAY_NONE;
  struct Lds {
    uint32_t cnt[W];
  };
  __device__ static void init(Lds& s, int tid) {
    for (uint32_t i = tid; i < W; i += BK_ACC_BLOCK) s.cnt[i] = 0;
  }
  __device__ static void init_range(Lds& s, uint32_t lo, uint32_t hi, int lane) {
    for (uint32_t i = lo + lane; i < hi; i += WAVE) s.cnt[i] = 0;
  }
  __device__ static void add(Lds& s, uint32_t i, Raw) { atomicAdd(&s.cnt[i], 1u); }
  __device__ static bool present(const Lds& s, uint32_t i) { return s.cnt[i] != 0; }
  __device__ static void stage(BkStage st, uint32_t pos, const Lds& s, uint32_t i) { ((uint32_t*)st.a)[pos] = s.cnt[i]; }
  static constexpr uint32_t PWORDS = 0;
  __device__ static void merge_el(Lds* d, const Lds* g, uint32_t i) { d->cnt[i] += g->cnt[i]; }
  __device__ static void merge_pw(Lds*, const Lds*, uint32_t) {}
  struct Out {
    int64_t* keys;
    int64_t* vals;
    int64_t init;
    __device__ Out retarget(int64_t* k, void* v, int64_t*) const { return Out{k, (int64_t*)v, init}; }
  };
  __device__ static void emit(const Out& o, uint64_t u, int64_t key, BkStage st, uint32_t j, int64_t) {
    o.keys[u] = key;
    o.vals[u] = (int64_t)((uint64_t)o.init + ((const uint32_t*)st.a)[j]);
  }
};

// degree / max-neighbour fold (TestSlice.java:233-239's shape)
struct BkDeg {
  using Raw = uint64_t;   // neighbour ID
  using Load = Raw;
  static constexpr bool REL = false;
  using A = uint32_t;
  static constexpr int S = 13;
  static constexpr uint32_t W = 1u << S;
  static constexpr bool HAS_V = true;
  static constexpr int PAY = PAY_NBR;
  struct Lds {
    long long mx[W];
    uint32_t cnt[W];
  };
  __device__ static void init(Lds& s, int tid) {
    for (uint32_t i = tid; i < W; i += BK_ACC_BLOCK) {
      s.cnt[i] = 0;
      s.mx[i] = std::numeric_limits<long long>::lowest();
    }
  }
  __device__ static void init_range(Lds& s, uint32_t lo, uint32_t hi, int lane) {
    for (uint32_t i = lo + lane; i < hi; i += WAVE) {
      s.cnt[i] = 0;
      s.mx[i] = std::numeric_limits<long long>::lowest();
    }
  }
  __device__ static void add(Lds& s, uint32_t i, Raw r) {
    atomicAdd(&s.cnt[i], 1u);
    atomicMax(&s.mx[i], (long long)r);
  }
  __device__ static bool present(const Lds& s, uint32_t i) { return s.cnt[i] != 0; }
  __device__ static void stage(BkStage st, uint32_t pos, const Lds& s, uint32_t i) {
    ((uint32_t*)st.a)[pos] = s.cnt[i];
    st.b[pos] = s.mx[i];
  }
  static constexpr uint32_t PWORDS = 0;
  __device__ static void merge_el(Lds* d, const Lds* g, uint32_t i) {
    d->cnt[i] += g->cnt[i];
    d->mx[i] = max(d->mx[i], g->mx[i]);
  }
  __device__ static void merge_pw(Lds*, const Lds*, uint32_t) {}
  struct Out {
    int64_t* keys;
    int64_t* deg;
    int64_t* mx;
    int64_t init_max;
    __device__ Out retarget(int64_t* k, void* v, int64_t* v2) const { return Out{k, (int64_t*)v, v2, init_max}; }
  };
  __device__ static void emit(const Out& o, uint64_t u, int64_t key, BkStage st, uint32_t j, int64_t) {
    o.keys[u] = key;
    o.deg[u] = (int64_t)((const uint32_t*)st.a)[j];
    const int64_t m = st.b[j];
    o.mx[u] = m > o.init_max ? m : o.init_max;
  }
};

// degree / max-neighbour fold with the neighbour kept as a 32-bit offset from the window's vertex
// base: 8 bytes of LDS per vertex (S = 14, half the buckets of BkDeg) and 4-byte payloads.  Valid
// while every neighbour lies in [base, base + 2^32): k_dp_scatter flags any that does not and the
// host reruns the window with BkDeg.
struct BkDeg32 {
  using Raw = uint32_t;    // stored payload: neighbour - base
  using Load = uint64_t;   // loaded neighbour ID
  using A = uint32_t;
  static constexpr bool REL = true;
  static constexpr int S = 14;
  static constexpr uint32_t W = 1u << S;
  static constexpr bool HAS_V = true;
  static constexpr int PAY = PAY_NBR;
  struct Lds {
    uint32_t mx[W];
    uint32_t cnt[W];
  };
  __device__ static void init(Lds& s, int tid) {
    for (uint32_t i = tid; i < W; i += BK_ACC_BLOCK) {
      s.cnt[i] = 0;
      s.mx[i] = 0;
    }
  }
  __device__ static void init_range(Lds& s, uint32_t lo, uint32_t hi, int lane) {
    for (uint32_t i = lo + lane; i < hi; i += WAVE) {
      s.cnt[i] = 0;
      s.mx[i] = 0;
    }
  }
  __device__ static void add(Lds& s, uint32_t i, Raw r) {
    atomicAdd(&s.cnt[i], 1u);
    atomicMax(&s.mx[i], r);
  }
  __device__ static bool present(const Lds& s, uint32_t i) { return s.cnt[i] != 0; }
  __device__ static void stage(BkStage st, uint32_t pos, const Lds& s, uint32_t i) {
    ((uint32_t*)st.a)[pos] = s.cnt[i];
    st.b[pos] = s.mx[i];
  }
  static constexpr uint32_t PWORDS = 0;
  __device__ static void merge_el(Lds* d, const Lds* g, uint32_t i) {
    d->cnt[i] += g->cnt[i];
    d->mx[i] = max(d->mx[i], g->mx[i]);
  }
  __device__ static void merge_pw(Lds*, const Lds*, uint32_t) {}
  using Out = BkDeg::Out;
  __device__ static void emit(const Out& o, uint64_t u, int64_t key, BkStage st, uint32_t j, int64_t base) {
    o.keys[u] = key;
    o.deg[u] = (int64_t)((const uint32_t*)st.a)[j];
    const int64_t m = (int64_t)((uint64_t)base + (uint32_t)st.b[j]);
    o.mx[u] = m > o.init_max ? m : o.init_max;
  }
};

// ---- record sources ------------------------------------------------------------------------------
// window edge columns, key relative to `base` (direction expansion as in EdgeSrc)
template <typename V, int DIR, int PAY>
struct BaseSrc {
  const int64_t* src;
  const int64_t* dst;
  const V* val;
  int64_t base;
  __device__ __forceinline__ void load(uint32_t r, uint32_t& k, V& v) const {
    uint32_t i = r;
    bool rev = (DIR == DIR_IN);
    if (DIR == DIR_ALL) { i = r >> 1; rev = r & 1u; }
    const int64_t a = rev ? dst[i] : src[i];
    k = (uint32_t)((uint64_t)a - (uint64_t)base);
    if constexpr (PAY == PAY_VAL) v = val[i];
    else if constexpr (PAY == PAY_NBR) v = (V)(rev ? src[i] : dst[i]);
  }
};

// partitioned records: 16-bit bucket-local index + payload
template <typename V>
struct PartSrc {
  const uint16_t* keys;
  const V* vals;
  __device__ __forceinline__ void load(uint32_t r, uint32_t& k, V& v) const {
    k = keys[r];
    if constexpr (!std::is_same_v<V, uint8_t>) v = vals[r];
  }
};

// packed partitioned records (integer SUM / MIN / MAX, k_dp_scatter_pack): one u32 per record,
// bucket-local index in the low 16 bits, the value in the high 16 bits when it lies in [0, PK_ESC),
// else PK_ESC there and the full value at the same position of `wide`
constexpr uint32_t PK_ESC = 0xFFFFu;
template <typename V>
struct PackSrc {
  const uint32_t* rec;
  const V* wide;
};
template <class P, class = void>
struct has_add_packed : std::false_type {};
template <class P>
struct has_add_packed<P, std::void_t<decltype(&P::add_packed)>> : std::bool_constant<P::INFER_PRESENCE> {};
// packed records whose common case needs only the LDS atomic (k_bk_accum's add4)
template <class P, bool = has_add_packed<P>::value>
struct fast_packed : std::false_type {};
template <class P>
struct fast_packed<P, true> : std::bool_constant<!P::SUM_MARKS_ALL> {};
template <class Src>
struct is_pack_src : std::false_type {};
template <typename V>
struct is_pack_src<PackSrc<V>> : std::true_type {};
template <class Src>
struct is_part_src : std::false_type {};
template <typename V>
struct is_part_src<PartSrc<V>> : std::bool_constant<sizeof(V) == 1 || sizeof(V) == 4 || sizeof(V) == 8> {};

template <typename V>
__device__ __forceinline__ uint32_t pk_narrow(V v) {
  using U = std::conditional_t<sizeof(V) == 8, uint64_t, uint32_t>;
  const U u = (U)v;
  return u < (U)PK_ESC ? (uint32_t)u : PK_ESC;
}

// ---- k_bk_info: min / max of the keys and the bucket histogram (relative to a predicted base) ----
// mm[0] = max(~flip(key)) (i.e. min), mm[1] = max(flip(key)), mm[2] = keys outside the prediction
template <int DIR, bool VEC>
__global__ __launch_bounds__(BK_INFO_BLOCK) void k_bk_info(const int64_t* __restrict__ src,
                                                           const int64_t* __restrict__ dst, uint64_t n,
                                                           int64_t base, int S, uint32_t nb,
                                                           uint32_t* __restrict__ hist,
                                                           unsigned long long* __restrict__ mm) {
  __shared__ uint32_t h[BK_MAXB];
  const int tid = threadIdx.x;
  for (int i = tid; i < BK_MAXB; i += BK_INFO_BLOCK) h[i] = 0;
  __syncthreads();
  uint64_t lo = 0, hi = 0;   // max of ~flip, max of flip
  uint32_t ovf = 0;
  auto add = [&](int64_t k) {
    const uint64_t f = (uint64_t)k ^ (1ull << 63);
    lo = max(lo, ~f);
    hi = max(hi, f);
    const uint64_t d = ((uint64_t)k - (uint64_t)base) >> S;
    if (k < base || d >= nb) ++ovf;
    else atomicAdd(&h[d], 1u);
  };
  if constexpr (!VEC) {
    const uint64_t stride = (uint64_t)gridDim.x * BK_INFO_BLOCK;
    for (uint64_t i = (uint64_t)blockIdx.x * BK_INFO_BLOCK + tid; i < n; i += stride) {
      if (DIR != DIR_IN) add(src[i]);
      if (DIR != DIR_OUT) add(dst[i]);
    }
  } else {
    const uint64_t npair = n >> 1;
    const longlong2* s2 = reinterpret_cast<const longlong2*>(src);
    const longlong2* d2 = reinterpret_cast<const longlong2*>(dst);
    constexpr int U = 4;
    const uint64_t stride = (uint64_t)gridDim.x * BK_INFO_BLOCK * U;
    for (uint64_t q = (uint64_t)blockIdx.x * BK_INFO_BLOCK * U + tid; q < npair; q += stride) {
      longlong2 a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t qq = q + (uint64_t)BK_INFO_BLOCK * u;
        if (qq < npair) {
          if (DIR != DIR_IN) a[u] = s2[qq];
          if (DIR != DIR_OUT) b[u] = d2[qq];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (q + (uint64_t)BK_INFO_BLOCK * u < npair) {
          if (DIR != DIR_IN) { add(a[u].x); add(a[u].y); }
          if (DIR != DIR_OUT) { add(b[u].x); add(b[u].y); }
        }
      }
    }
    if ((n & 1) && blockIdx.x == 0 && tid == 0) {
      if (DIR != DIR_IN) add(src[n - 1]);
      if (DIR != DIR_OUT) add(dst[n - 1]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = max(lo, (uint64_t)__shfl_xor((unsigned long long)lo, o, WAVE));
    hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, o, WAVE));
    ovf += __shfl_xor(ovf, o, WAVE);
  }
  if ((tid & 63) == 0) {
    atomicMax(&mm[0], (unsigned long long)lo);
    atomicMax(&mm[1], (unsigned long long)hi);
    if (ovf) atomicAdd(&mm[2], (unsigned long long)ovf);
  }
  __syncthreads();
  for (uint32_t i = tid; i < nb; i += BK_INFO_BLOCK) {
    const uint32_t c = h[i];
    if (c) atomicAdd(&hist[i], c);
  }
}

// block-wide exclusive scan of one u32 per thread (BLOCK = BK_PLAN_BLOCK); returns the total
// (1024-thread blocks only: it reads BK_PLAN_BLOCK / WAVE wave sums; block_excl_scan<BLOCK> for others)
__device__ __forceinline__ uint32_t bk_block_scan(uint32_t x, uint32_t* s_w, uint32_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = BK_PLAN_BLOCK / WAVE;
  const uint32_t inc = wave_inclusive_sum(x);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t v = s_w[i];
    off += i < w ? v : 0u;
    tot += v;
  }
  __syncthreads();
  total = tot;
  return off + inc - x;
}

// ---- k_bk_plan: digit bases of the partition passes, bucket starts, work items (one block) -------
#ifndef GS_BK_LPT
#define GS_BK_LPT 1
#endif
constexpr int BK_LPT_CLASSES = 64;
// pass p ranks digit (bucket >> (p * w)) & (2^w - 1); bucket b's records end up at
// [bucket_start[b], bucket_start[b + 1]).  Items: a bucket of cnt records is split into
// ceil(cnt / item_recs) items; multi-item buckets get consecutive slabs.
static __global__ __launch_bounds__(BK_PLAN_BLOCK) void k_bk_plan(const uint32_t* __restrict__ hist, uint32_t nb,
                                                                  int passes, int w, uint32_t item_recs,
                                                                  BkPlanOut o) {
  __shared__ uint32_t s_dh[2][256];
  __shared__ uint32_t s_w[BK_PLAN_BLOCK / WAVE];
  __shared__ uint32_t s_maxit;
  const int tid = threadIdx.x;
  for (int i = tid; i < 2 * 256; i += BK_PLAN_BLOCK) (&s_dh[0][0])[i] = 0;
  if (tid == 0) s_maxit = 0;
  if (tid == 0 && o.claim) *o.claim = 0;
  __syncthreads();
  // two buckets per thread (BK_MAXB = 2 * BK_PLAN_BLOCK)
  const uint32_t b0 = 2 * tid, b1 = 2 * tid + 1;
  const bool spec = o.cursor != nullptr;
  auto count = [&](uint32_t b) -> uint32_t {
    if (b >= nb) return 0u;
    if (!spec) return hist[b];
    uint32_t n = 0;
    for (uint32_t x = 0; x < SP_NSEG; ++x) n += min(o.cursor[x * BK_MAXB + b], sp_hi(o.cursor, x, b)) - sp_lo(o.cursor, x, b);
    return n;
  };
  const uint32_t c0 = count(b0), c1 = count(b1);
  const uint32_t dmask = (1u << w) - 1;
  for (int p = 0; p < passes; ++p) {
    if (c0) atomicAdd(&s_dh[p][(b0 >> (p * w)) & dmask], c0);
    if (c1) atomicAdd(&s_dh[p][(b1 >> (p * w)) & dmask], c1);
  }
  uint32_t total;
  const uint32_t start0 = bk_block_scan(c0 + c1, s_w, total);
  if (spec) {   // the occupied buckets (the next window's predicted range)
    __shared__ uint32_t s_lo, s_hi;
    if (tid == 0) {
      s_lo = ~0u;
      s_hi = 0;
    }
    __syncthreads();
    if (c0 | c1) {
      atomicMin(&s_lo, c0 ? b0 : b1);
      atomicMax(&s_hi, c1 ? b1 : b0);
    }
    __syncthreads();
    if (tid == 0) {
      o.occupied[0] = s_lo;
      o.occupied[1] = s_hi;
    }
  }
  if (o.counts_out) {   // every bucket slot (0 past nb): the next window's regions read them
    o.counts_out[b0] = c0;
    o.counts_out[b1] = c1;
  }
  if (!spec) {
    if (b0 < nb) o.bucket_start[b0] = start0;
    if (b1 < nb) o.bucket_start[b1] = start0 + c0;
    if (tid == 0) o.bucket_start[nb] = total;
  }
  // digit bases (s_dh complete after the scan's barriers)
  if (tid < passes) {   // <= 256 digits per pass, one thread each
    uint32_t run = 0;
    for (uint32_t d = 0; d <= dmask; ++d) {
      o.digit_base[tid * 256 + d] = run;
      run += s_dh[tid][d];
    }
  }
  // items
  auto nitems = [&](uint32_t c) { return c == 0 ? 0u : (c + item_recs - 1) / item_recs; };
  const uint32_t i0 = nitems(c0), i1 = nitems(c1);
  const uint32_t m0 = i0 > 1 ? i0 : 0u, m1 = i1 > 1 ? i1 : 0u;
  uint32_t n_items, n_slabs, n_multi;
  const uint32_t first0 = bk_block_scan(i0 + i1, s_w, n_items);
  const uint32_t slab0 = bk_block_scan(m0 + m1, s_w, n_slabs);
  const uint32_t mb0 = bk_block_scan((m0 ? 1u : 0u) + (m1 ? 1u : 0u), s_w, n_multi);
#if GS_BK_LPT
  // claim order: largest items first (k_bk_accum's workgroups take items from a counter, so the small
  // ones fill the gaps at the end instead of a large one starting last): a counting sort over
  // BK_LPT_CLASSES size classes, descending; the order within a class is free
  __shared__ uint32_t s_cls[BK_LPT_CLASSES];
  for (int i = tid; i < BK_LPT_CLASSES; i += BK_PLAN_BLOCK) s_cls[i] = 0;
  __syncthreads();
  auto size_class = [&](uint32_t n) -> uint32_t {   // larger items -> smaller class
    return BK_LPT_CLASSES - 1 - min<uint32_t>(BK_LPT_CLASSES - 1, (uint32_t)((uint64_t)n * BK_LPT_CLASSES / (item_recs + 1)));
  };
  // a bucket's items are ni - 1 full ones and its last piece: one atomic for each group (a hub bucket of
  // a Zipf stream has hundreds of items; one atomic per item serialised the plan's thread)
  auto count_items = [&](uint32_t b, uint32_t c, uint32_t ni) {
    if (b >= nb || !ni) return;
    if (ni > 1) atomicAdd(&s_cls[size_class(item_recs)], ni - 1);
    atomicAdd(&s_cls[size_class(c - (ni - 1) * item_recs)], 1u);
  };
  count_items(b0, c0, i0);
  count_items(b1, c1, i1);
  __syncthreads();
  static_assert(BK_LPT_CLASSES == WAVE, "one wave scans the classes");
  if (tid < WAVE) {
    const uint32_t x = s_cls[tid];
    s_cls[tid] = wave_inclusive_sum(x) - x;
  }
  __syncthreads();
#endif
  auto emit_bucket = [&](uint32_t b, uint32_t c, uint32_t ni, uint32_t first, uint32_t slab, uint32_t mb) {
    if (b >= nb) return;
    o.bucket_count[b] = 0;
    o.b_items[b] = ni;
    o.b_slab[b] = slab;
    if (ni > 1) o.mlist[mb] = b;
    if (!ni) return;
#if GS_BK_LPT
    const uint32_t fpos = ni > 1 ? atomicAdd(&s_cls[size_class(item_recs)], ni - 1) : 0u;   // the full items
    const uint32_t lpos = atomicAdd(&s_cls[size_class(c - (ni - 1) * item_recs)], 1u);     // the last piece
#endif
    for (uint32_t k = 0; k < ni; ++k) {
      BkItem it;
      it.bucket = b;
      it.begin = k * item_recs;   // relative; made absolute below
      it.end = min(c, (k + 1) * item_recs);
      it.slab = ni > 1 ? slab + k : ~0u;
#if GS_BK_LPT
      o.items[k + 1 < ni ? fpos + k : lpos] = it;
#else
      o.items[first + k] = it;
#endif
    }
  };
  emit_bucket(b0, c0, i0, first0, slab0, mb0);
  emit_bucket(b1, c1, i1, first0 + i0, slab0 + m0, mb0 + (m0 ? 1u : 0u));
  if (o.max_items) {   // (s_maxit complete after the item scans' barriers)
    if (i0 > 1 || i1 > 1) atomicMax(&s_maxit, max(i0, i1));
    __syncthreads();
  }
  if (tid == 0) {
    if (o.max_items) *o.max_items = s_maxit;
    *o.n_items = n_items;
    *o.n_multi = n_multi;
  }
}

// ---- direct partition: the whole bucket index in ONE scatter pass ----------------------------------
// A tile is the records of dp_tile_edges<DIR>() consecutive edges (at most DP_TILE records, so a
// per-bucket count fits u16).
//   k_dp_hist     per-tile bucket counts cnt[t][b] (u16, row-contiguous) + vertex min / max;
//   k_dp_up       per chunk of DP_CHUNK tiles and bucket: the chunk's count;
//   k_dp_spine    per bucket: exclusive scan of the chunk counts over chunks, bucket totals;
//   (k_bk_plan    bucket starts from the totals, work items)
//   k_dp_down     every tile's absolute write offset per bucket: off[t][b] (u32);
//   k_dp_scatter  ranks the tile's records by bucket in LDS (LDS atomics: the order inside a bucket
//                 is free, the ops are associative and commutative) and writes each bucket's run of
//                 (16-bit bucket-local index, payload) at off[t][b].
// Against the 2-pass LSD partition (k_onesweep twice) this moves 8 + 26 B per 8-byte-payload record
// instead of 8 + 28 + 22.
#ifndef GS_DP_ITEMS
#define GS_DP_ITEMS 10
#endif
#ifndef GS_DP_XCD
#define GS_DP_XCD 1
#endif
// 1: payloads go straight from registers to their global slot (off[t][b] + rank) instead of through
// LDS; the tile's LDS drops to the staged keys + tables (two blocks per CU).  Measured on C2 (scatter,
// ms): staged 10 items 1.65; direct 6 items 1.75 (staged 6 items 1.89); direct 8 and 10 items spill at
// the 64-VGPR cap of two blocks per CU (2.20, 3.17).  Kept off; the A/B stays buildable.
#ifndef GS_DP_VDIRECT
#define GS_DP_VDIRECT 0
#endif
constexpr int DP_BLOCK = 1024;
constexpr int DP_ITEMS = GS_DP_ITEMS;
constexpr uint32_t DP_TILE = DP_BLOCK * DP_ITEMS;   // 10240 records < 2^16
constexpr uint32_t DP_CHUNK = 64;                   // tiles per up / down-sweep chunk
// packed path (k_dp_scatter_pack): its own tile, 6 B of LDS per record (the histogram runs on the same tiles)
#ifndef GS_PK_ITEMS
#define GS_PK_ITEMS 16   // C2 scatter (ms): 10 items 1.18, 12 1.17, 14 1.144, 16 1.149 (fewer tiles: offsets 0.056 -> 0.043)
#endif
constexpr int PK_ITEMS = GS_PK_ITEMS;
static_assert(DP_BLOCK * PK_ITEMS < 65536 && DP_BLOCK * DP_ITEMS < 65536, "per-tile bucket counts are u16");
template <int DIR, int ITEMS = DP_ITEMS>
__host__ __device__ constexpr uint32_t dp_tile_edges() {
  return DIR == DIR_ALL ? DP_BLOCK * ITEMS / 2 : DP_BLOCK * ITEMS;
}
// k_dp_scatter grid: the full tiles (in 8 XCD slots) + one block for the partial tile
template <int DIR, int ITEMS = DP_ITEMS>
__host__ __device__ inline uint32_t dp_scatter_grid(uint64_t n) {
  return (uint32_t)((n / dp_tile_edges<DIR, ITEMS>() + 7) / 8 * 8 + 1);
}

// Persistent, software-pipelined: the next tile's keys are in flight while this
// tile's counts go through LDS.  VEC: the tile's keys as 16-byte pairs (columns 16-byte aligned).
template <int DIR, bool VEC, int ITEMS>
__global__ __launch_bounds__(DP_BLOCK) void k_dp_hist(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      uint64_t n, uint32_t nt, int64_t base, int S, uint32_t nbp,
                                                      uint16_t* __restrict__ cnt,
                                                      unsigned long long* __restrict__ mm) {
  __shared__ uint32_t h[BK_MAXB];
  __shared__ unsigned long long s_mm[3][DP_BLOCK / WAVE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr uint32_t TE = dp_tile_edges<DIR, ITEMS>();
  constexpr int U = VEC ? (TE / 2 + DP_BLOCK - 1) / DP_BLOCK : (TE + DP_BLOCK - 1) / DP_BLOCK;
  using L = std::conditional_t<VEC, longlong2, int64_t>;
  uint64_t lo = 0, hi = 0;   // max of ~flip(key), max of flip(key)
  uint32_t ovf = 0;
  auto add = [&](int64_t k) {
    const uint64_t f = (uint64_t)k ^ (1ull << 63);
    lo = max(lo, ~f);
    hi = max(hi, f);
    const uint64_t d = ((uint64_t)k - (uint64_t)base) >> S;
    if (k < base || d >= nbp) ++ovf;
    else atomicAdd(&h[d], 1u);
  };
  // element u of tile tt: a 16-byte pair index (VEC) or an edge index
  auto first = [&](uint32_t tt) { return VEC ? ((uint64_t)tt * TE) >> 1 : (uint64_t)tt * TE; };
  auto last = [&](uint32_t tt) { const uint64_t e1 = min(n, (uint64_t)(tt + 1) * TE); return VEC ? e1 >> 1 : e1; };
  // loads are unconditional (indices clamped into the tile; the host picks VEC only when every tile
  // holds a whole pair): a load under a branch gets a register copy at the join that waits for it,
  // which serialises the tile's loads
  auto load = [&](uint32_t tt, L (&a)[U], L (&b)[U]) {
    const uint64_t q0 = first(tt), q1 = last(tt);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t q = min(q0 + (uint64_t)u * DP_BLOCK + tid, q1 - 1);
      if (DIR != DIR_IN) a[u] = reinterpret_cast<const L*>(src)[q];
      if (DIR != DIR_OUT) b[u] = reinterpret_cast<const L*>(dst)[q];
    }
  };
  L ca[U], cb[U];
  uint32_t t = blockIdx.x;
  if (t < nt) load(t, ca, cb);
  for (; t < nt; t += gridDim.x) {
    for (uint32_t i = tid; i < nbp; i += DP_BLOCK) h[i] = 0;
    L na[U], nb2[U];
    load(t + gridDim.x < nt ? t + gridDim.x : t, na, nb2);   // prefetch (the last round reloads this tile)
    __syncthreads();
    const uint64_t q0 = first(t), q1 = last(t);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (q0 + (uint64_t)u * DP_BLOCK + tid < q1) {
        if constexpr (VEC) {
          if (DIR != DIR_IN) { add(ca[u].x); add(ca[u].y); }
          if (DIR != DIR_OUT) { add(cb[u].x); add(cb[u].y); }
        } else {
          if (DIR != DIR_IN) add(ca[u]);
          if (DIR != DIR_OUT) add(cb[u]);
        }
      }
    }
    if (VEC && tid == 0) {   // TE is even: only the window's last edge can be unpaired
      const uint64_t e1 = min(n, (uint64_t)(t + 1) * TE);
      if (e1 & 1) {
        if (DIR != DIR_IN) add(src[e1 - 1]);
        if (DIR != DIR_OUT) add(dst[e1 - 1]);
      }
    }
    __syncthreads();
    uint16_t* row = cnt + (uint64_t)t * nbp;
    for (uint32_t i = tid; i < nbp; i += DP_BLOCK) row[i] = (uint16_t)h[i];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ca[u] = na[u];
      cb[u] = nb2[u];
    }
    __syncthreads();
  }
  // one atomic per block and word (thousands of blocks on three words would serialise)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = max(lo, (uint64_t)__shfl_xor((unsigned long long)lo, o, WAVE));
    hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, o, WAVE));
    ovf += __shfl_xor(ovf, o, WAVE);
  }
  if (lane == 0) {
    s_mm[0][w] = lo;
    s_mm[1][w] = hi;
    s_mm[2][w] = ovf;
  }
  __syncthreads();
  if (tid == 0) {
    unsigned long long a = 0, b = 0, o2 = 0;
    for (int i = 0; i < DP_BLOCK / WAVE; ++i) {
      a = max(a, s_mm[0][i]);
      b = max(b, s_mm[1][i]);
      o2 += s_mm[2][i];
    }
    atomicMax(&mm[0], a);
    atomicMax(&mm[1], b);
    if (o2) atomicAdd(&mm[2], o2);
  }
}

// chunk counts: csum[c][b] = sum of cnt[t][b] over the chunk's tiles
static __global__ __launch_bounds__(256) void k_dp_up(const uint16_t* __restrict__ cnt, uint32_t nt, uint32_t nbp,
                                                      uint32_t* __restrict__ csum) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nbp) return;
  const uint32_t c = blockIdx.y, t0 = c * DP_CHUNK, t1 = min(nt, t0 + DP_CHUNK);
  uint32_t s = 0;
#pragma unroll 8
  for (uint32_t t = t0; t < t1; ++t) s += cnt[(uint64_t)t * nbp + b];
  csum[(uint64_t)c * nbp + b] = s;
}

// per bucket (one lane each, 64 per block): exclusive scan of csum over chunks, in place; totals
static __global__ __launch_bounds__(1024) void k_dp_spine(uint32_t* __restrict__ csum, uint32_t nch, uint32_t nbp,
                                                          uint32_t* __restrict__ total) {
  __shared__ uint32_t s[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * 64 + lane;
  const uint32_t per = (nch + 15) / 16, c0 = min(nch, w * per), c1 = min(nch, c0 + per);
  uint32_t sum = 0;
  if (b < nbp) {
#pragma unroll 8
    for (uint32_t c = c0; c < c1; ++c) sum += csum[(uint64_t)c * nbp + b];
  }
  s[w][lane] = sum;
  __syncthreads();
  uint32_t run = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t v = s[i][lane];
    run += i < w ? v : 0u;
    tot += v;
  }
  if (b < nbp) {
    for (uint32_t c = c0; c < c1; ++c) {
      const uint32_t v = csum[(uint64_t)c * nbp + b];
      csum[(uint64_t)c * nbp + b] = run;
      run += v;
    }
    if (w == 0) total[b] = tot;
  }
}

// off[t][b] = bucket_start[b] + (records of bucket b in tiles before t)
static __global__ __launch_bounds__(256) void k_dp_down(const uint16_t* __restrict__ cnt,
                                                        const uint32_t* __restrict__ csum,
                                                        const uint32_t* __restrict__ bucket_start, uint32_t nt,
                                                        uint32_t nbp, uint32_t* __restrict__ off) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nbp) return;
  const uint32_t c = blockIdx.y, t0 = c * DP_CHUNK, t1 = min(nt, t0 + DP_CHUNK);
  uint32_t run = bucket_start[b] + csum[(uint64_t)c * nbp + b];
  for (uint32_t t = t0; t < t1; ++t) {
    const uint64_t i = (uint64_t)t * nbp + b;
    const uint32_t k = cnt[i];
    off[i] = run;
    run += k;
  }
}

// raw record r of the window: the low half of its key (the bucket math is mod 2^32) and its payload
template <typename V, int DIR, int PAY>
__device__ __forceinline__ void dp_load_raw(const BaseSrc<V, DIR, PAY>& es, uint32_t r, uint32_t& klo, V& v) {
  uint32_t i = r;
  bool rev = DIR == DIR_IN;
  if constexpr (DIR == DIR_ALL) {
    i = r >> 1;
    rev = r & 1u;
  }
  klo = reinterpret_cast<const uint32_t*>(rev ? es.dst : es.src)[2 * (uint64_t)i];
  if constexpr (PAY == PAY_VAL) v = es.val[i];
  else if constexpr (PAY == PAY_NBR) v = (V)(rev ? es.src : es.dst)[i];
}

// One full tile per block (1 block per CU: LDS-bound); blocks b and b + 8 share an XCD under
// round-robin dispatch (speed only), so XCD slot b & 7 owns a contiguous range of tiles and the
// blocks an XCD runs at once write adjacent runs of each bucket through one L2 (without it: +14 %).
// The last block takes the window's partial tile.  Every load is unconditional (clamped indices):
// a load under a branch gets a register copy at the join that waits for it and serialises the tile
// (2.02 -> 1.59 ms on C2).  Measured and dropped: a persistent loop prefetching the
// next tile (2.20 ms), 2-8 unrolled tiles per block (1.68-2.43 ms), 5120-record tiles at 2 blocks
// per CU (1.71 ms), keys and values staged in turn through one region for 2 blocks per CU (1.81 ms
// at 8192 records, 2.21 at 10240: the 64-VGPR cap spills).
// V: loaded payload; VO: stored payload (REL: VO = V - base, out-of-range payloads set *rel_bad)
#if GS_DP_VDIRECT
#define GS_DP_SCATTER_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))   // two 16-wave blocks per CU
#else
#define GS_DP_SCATTER_ATTR
#endif
template <typename V, int DIR, int PAY, typename VO = V, bool REL = false>
__global__ __launch_bounds__(DP_BLOCK) GS_DP_SCATTER_ATTR void k_dp_scatter(BaseSrc<V, DIR, PAY> es, uint64_t n, int S, uint32_t nbp,
                                                         const uint32_t* __restrict__ off,
                                                         uint16_t* __restrict__ k16, VO* __restrict__ vout,
                                                         uint32_t* __restrict__ rel_bad,
                                                         const unsigned long long* __restrict__ mm) {
  constexpr bool HAS_V = PAY != PAY_NONE;
  if (mm[2]) return;   // keys outside the predicted range: the window is rerun
  constexpr bool STAGE_V = HAS_V && !GS_DP_VDIRECT;
  __shared__ uint32_t s_key[DP_TILE];                // (bucket << 16) | bucket-local index, bucket order
  __shared__ VO s_val[STAGE_V ? DP_TILE : 1];
  __shared__ uint32_t s_cnt[BK_MAXB];                // counts, then run starts inside the tile
  __shared__ uint32_t s_delta[BK_MAXB];              // global position - tile position of bucket b's run
  __shared__ uint32_t s_w[DP_BLOCK / WAVE];
  const int tid = threadIdx.x;
  constexpr uint32_t TE = dp_tile_edges<DIR>();
  const uint32_t nfull = (uint32_t)(n / TE);   // tile nfull, if any, is the window's partial last one
  const uint32_t base32 = (uint32_t)es.base, lmask = (1u << S) - 1;
  const uint32_t b0 = 2 * tid, b1 = 2 * tid + 1;   // BK_MAXB = 2 * DP_BLOCK
  const uint32_t bl0 = min(b0, nbp - 1), bl1 = min(b1, nbp - 1);
  bool bad = false;

  auto process = [&](auto full, uint32_t nrec, const uint32_t (&klo)[DP_ITEMS], const V (&vv)[DP_ITEMS],
                     uint32_t o0, uint32_t o1) {
    constexpr bool FULL = decltype(full)::value;
    for (uint32_t i = tid; i < nbp; i += DP_BLOCK) s_cnt[i] = 0;
    __syncthreads();
    uint32_t kb[DP_ITEMS], rk[DP_ITEMS];
#pragma unroll
    for (int u = 0; u < DP_ITEMS; ++u) {
      const uint32_t c = klo[u] - base32;
      kb[u] = ((c >> S) << 16) | (c & lmask);
      if (FULL || (uint32_t)u * DP_BLOCK + tid < nrec) rk[u] = atomicAdd(&s_cnt[kb[u] >> 16], 1u);
    }
    __syncthreads();
    const uint32_t c0 = b0 < nbp ? s_cnt[b0] : 0u, c1 = b1 < nbp ? s_cnt[b1] : 0u;
    uint32_t total;
    const uint32_t st0 = bk_block_scan(c0 + c1, s_w, total);
    // unconditional: entries past nbp are never read, and a branch here would make the compiler
    // wait for every outstanding load (the prefetch) before the offsets it guards
    s_cnt[b0] = st0;
    s_delta[b0] = o0 - st0;
    s_cnt[b1] = st0 + c0;
    s_delta[b1] = o1 - (st0 + c0);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < DP_ITEMS; ++u) {
      if (FULL || (uint32_t)u * DP_BLOCK + tid < nrec) {
        const uint32_t pos = s_cnt[kb[u] >> 16] + rk[u];
        s_key[pos] = kb[u];
        VO vo{};
        if constexpr (REL) {
          const uint64_t rel = (uint64_t)vv[u] - (uint64_t)es.base;
          bad |= (rel >> 32) != 0;
          vo = (VO)rel;
        } else if constexpr (HAS_V) {
          vo = vv[u];
        }
        if constexpr (STAGE_V) s_val[pos] = vo;
        else if constexpr (HAS_V) vout[s_delta[kb[u] >> 16] + pos] = vo;
      }
    }
    __syncthreads();
    if constexpr (FULL) {
#pragma unroll
      for (int u = 0; u < DP_ITEMS; ++u) {
        const uint32_t j = (uint32_t)u * DP_BLOCK + tid;
        const uint32_t kv = s_key[j];
        const uint32_t d = s_delta[kv >> 16] + j;
        k16[d] = (uint16_t)kv;
        if constexpr (STAGE_V) vout[d] = s_val[j];
      }
    } else {
      for (uint32_t j = tid; j < nrec; j += DP_BLOCK) {
        const uint32_t kv = s_key[j];
        const uint32_t d = s_delta[kv >> 16] + j;
        k16[d] = (uint16_t)kv;
        if constexpr (STAGE_V) vout[d] = s_val[j];
      }
    }
  };
  // tile tt holds records [tt * DP_TILE, + nrec); indices clamped into the tile
  auto load_tile = [&](uint32_t tt, uint32_t nrec, uint32_t (&klo)[DP_ITEMS], V (&vv)[DP_ITEMS]) {
    const uint32_t r0 = tt * DP_TILE;
#pragma unroll
    for (int u = 0; u < DP_ITEMS; ++u) dp_load_raw(es, r0 + min((uint32_t)u * DP_BLOCK + tid, nrec - 1), klo[u], vv[u]);
  };
  auto load_off = [&](uint32_t tt, uint32_t& o0, uint32_t& o1) {
    const uint32_t* orow = off + (uint64_t)tt * nbp;
    o0 = orow[bl0];
    o1 = orow[bl1];
  };
  using Full = std::integral_constant<bool, true>;
  uint32_t ka[DP_ITEMS];
  V va[DP_ITEMS];
  {   // one full tile per block
#if GS_DP_XCD
    const uint32_t per = (nfull + 7) / 8;
    const uint32_t t = blockIdx.x == gridDim.x - 1 ? nfull : (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
#else
    const uint32_t t = blockIdx.x;
#endif
    if (t < nfull) {
      uint32_t o0, o1;
      load_off(t, o0, o1);
      load_tile(t, DP_TILE, ka, va);
      process(Full{}, DP_TILE, ka, va, o0, o1);
    }
  }
  if ((uint64_t)nfull * TE < n && blockIdx.x == gridDim.x - 1) {   // the partial last tile
    const uint32_t nrec = (uint32_t)((n - (uint64_t)nfull * TE) * (DIR == DIR_ALL ? 2 : 1));
    uint32_t o0, o1;
    load_off(nfull, o0, o1);
    load_tile(nfull, nrec, ka, va);
    process(std::integral_constant<bool, false>{}, nrec, ka, va, o0, o1);
  }
  if constexpr (REL) {
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(rel_bad, 1u);
  }
}

// ---- packed scatter: integer SUM / MIN / MAX, 4 bytes per partitioned record ----------------------
// The same tile, ranking and per-tile offsets as k_dp_scatter, but each record leaves as one u32
// (bucket-local index | narrow value << 16, PackSrc) instead of a u16 key plus an 8-byte value: the
// partition written and read back shrinks from 10 to 4 bytes per record.  A value outside
// [0, PK_ESC) is an escape: PK_ESC in the record, the full value at the record's position of `wide`
// (written from this kernel, read by k_bk_accum only for escapes; n_esc counts them so the host can
// fall back to k_dp_scatter for windows where escapes are common).  LDS is 6 bytes per record
// (76 KiB per 10240-record tile), so two 1024-thread blocks share a CU and one block's loads overlap
// the other's LDS and store phases (k_dp_scatter: one block per CU).
// mm[2] != 0 (k_dp_hist saw a key outside the predicted range): every block exits at once and the
// host reruns the window with the measured range.
#ifndef GS_PK_WAVES
#define GS_PK_WAVES 4   // waves per SIMD: 4 = one 16-wave block per CU (8: two, with the 64-VGPR cap)
#endif
template <typename V, int DIR, int ITEMS>
__global__ __launch_bounds__(DP_BLOCK) __attribute__((amdgpu_waves_per_eu(GS_PK_WAVES, GS_PK_WAVES)))
void k_dp_scatter_pack(BaseSrc<V, DIR, PAY_VAL> es, uint64_t n, int S, uint32_t nbp,
                       const uint32_t* __restrict__ off, uint32_t* __restrict__ rec, V* __restrict__ wide,
                       const unsigned long long* __restrict__ mm, unsigned long long* __restrict__ n_esc) {
  constexpr uint32_t TILE = DP_BLOCK * ITEMS;
  __shared__ uint32_t s_key[TILE];         // (bucket << 16) | bucket-local index, bucket order
  __shared__ uint16_t s_v16[TILE];         // narrow value, same order
  __shared__ uint32_t s_cnt[BK_MAXB];      // counts, then run starts inside the tile
  __shared__ uint32_t s_delta[BK_MAXB];    // global position - tile position of bucket b's run
  __shared__ uint32_t s_w[DP_BLOCK / WAVE];
  if (mm[2]) return;
  const int tid = threadIdx.x;
  constexpr uint32_t TE = dp_tile_edges<DIR, ITEMS>();
  const uint32_t nfull = (uint32_t)(n / TE);
  const uint32_t base32 = (uint32_t)es.base, lmask = (1u << S) - 1;
  const uint32_t b0 = 2 * tid, b1 = 2 * tid + 1;   // BK_MAXB = 2 * DP_BLOCK
  const uint32_t bl0 = min(b0, nbp - 1), bl1 = min(b1, nbp - 1);
  uint32_t t, nrec = TILE;
  if (blockIdx.x == gridDim.x - 1) {   // the window's partial last tile
    if ((uint64_t)nfull * TE >= n) return;
    t = nfull;
    nrec = (uint32_t)((n - (uint64_t)nfull * TE) * (DIR == DIR_ALL ? 2 : 1));
  } else {   // XCD slot b & 7 owns a contiguous range of full tiles (k_dp_scatter)
    const uint32_t per = (nfull + 7) / 8;
    t = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (t >= nfull) return;
  }
  const uint32_t r0 = t * TILE;
  const uint32_t* orow = off + (uint64_t)t * nbp;
  const uint32_t o0 = orow[bl0], o1 = orow[bl1];
  uint32_t kb[ITEMS], v16[ITEMS];
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {   // unconditional loads, clamped into the tile (k_dp_scatter)
    uint32_t kl;
    V vv;
    dp_load_raw(es, r0 + min((uint32_t)u * DP_BLOCK + tid, nrec - 1), kl, vv);
    const uint32_t c = kl - base32;
    kb[u] = ((c >> S) << 16) | (c & lmask);
    v16[u] = pk_narrow(vv);
  }
  for (uint32_t i = tid; i < nbp; i += DP_BLOCK) s_cnt[i] = 0;
  __syncthreads();
  uint32_t rk[ITEMS];
#pragma unroll
  for (int u = 0; u < ITEMS; ++u)
    if ((uint32_t)u * DP_BLOCK + tid < nrec) rk[u] = atomicAdd(&s_cnt[kb[u] >> 16], 1u);
  __syncthreads();
  const uint32_t c0 = b0 < nbp ? s_cnt[b0] : 0u, c1 = b1 < nbp ? s_cnt[b1] : 0u;
  uint32_t total;
  const uint32_t st0 = bk_block_scan(c0 + c1, s_w, total);
  s_cnt[b0] = st0;   // unconditional: entries past nbp are never read
  s_delta[b0] = o0 - st0;
  s_cnt[b1] = st0 + c0;
  s_delta[b1] = o1 - (st0 + c0);
  __syncthreads();
  uint32_t esc = 0;
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint32_t j = (uint32_t)u * DP_BLOCK + tid;
    if (j < nrec) {
      const uint32_t pos = s_cnt[kb[u] >> 16] + rk[u];
      s_key[pos] = kb[u];
      s_v16[pos] = (uint16_t)v16[u];
      if (v16[u] == PK_ESC) {   // rare: reload the full value for its slot of `wide`
        const uint32_t r = r0 + j;
        wide[s_delta[kb[u] >> 16] + pos] = es.val[DIR == DIR_ALL ? r >> 1 : r];
        ++esc;
      }
    }
  }
  __syncthreads();
  auto put = [&](uint32_t j) {
    const uint32_t kv = s_key[j];
    rec[s_delta[kv >> 16] + j] = (kv & 0xFFFFu) | ((uint32_t)s_v16[j] << 16);
  };
  if (nrec == TILE) {
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) put((uint32_t)u * DP_BLOCK + tid);
  } else {
    for (uint32_t j = tid; j < nrec; j += DP_BLOCK) put(j);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) esc += __shfl_xor(esc, o, WAVE);
  if ((tid & 63) == 0 && esc) atomicAdd(n_esc, (unsigned long long)esc);
}

// ---- speculative partition: the packed scatter without a histogram pass -------------------------
// Consecutive windows of one stream spread their records over the buckets alike (a bucket is the sum
// of 2^S vertices' degrees).  So bucket b gets a REGION sized from the previous window's count of b
// (k_sp_regions: t·R/R_prev + 1/16, 4-aligned, + SP_PAD records), and a tile reserves its run of each
// bucket with one returning atomicAdd on b's cursor instead of reading the offsets that k_dp_hist +
// the scans computed: the window's keys are read once, not twice, and the per-tile count / offset
// matrices (0.1 GB at C2) go away.  The reservation is issued before the tile's records go through LDS
// and used after, so its latency hides behind the LDS scatter.  Each XCD slot reserves from its own
// segment of the region (GS_SP_XCD): runs written at the same time by one XCD's blocks stay adjacent
// in one L2, and each cursor sees 1/8 of the atomics.  A run that would pass its segment's end is
// written to a trash area instead, and a key outside the predicted range is dropped; both count in
// mm[2], every later launch exits and the host reruns the window through k_dp_hist (which cannot
// miss).  Record order inside a bucket follows the atomics: integer SUM / MIN / MAX only (exact in
// any order).

// bucket regions from the previous window's counts (one block): starts, cursors, mm reset
static __global__ __launch_bounds__(BK_PLAN_BLOCK) void k_sp_regions(const uint32_t* __restrict__ prev, uint32_t nb,
                                                                     uint64_t r_prev, uint64_t r_now,
                                                                     uint32_t* __restrict__ bucket_start,
                                                                     uint32_t* __restrict__ cursor, SpSlots slots,
                                                                     unsigned long long* __restrict__ mm,
                                                                     unsigned long long* __restrict__ n_esc) {
  __shared__ uint32_t s_w[BK_PLAN_BLOCK / WAVE];
  __shared__ uint32_t s_frac[SP_NSEG + 1];
  const int tid = threadIdx.x;
  const uint32_t b0 = 2 * tid, b1 = 2 * tid + 1;   // BK_MAXB = 2 * BK_PLAN_BLOCK
  if (tid <= (int)SP_NSEG) {   // each slot's share of the records (visible after the scan's barrier)
    const uint32_t all = slots.pre[SP_NSEG];
    const uint64_t f = all ? ((uint64_t)slots.pre[tid] << 32) / all : 0;
    s_frac[tid] = (uint32_t)min(f, (uint64_t)0xFFFFFFFFu);
  }
  auto cap = [&](uint32_t b) -> uint32_t {
    if (b >= nb) return 0u;
    const uint64_t t = (uint64_t)prev[b] * r_now / (r_prev ? r_prev : 1);
    return (uint32_t)((t + (t >> 4) + 3) & ~3ull) + SP_PAD;
  };
  const uint32_t c0 = cap(b0), c1 = cap(b1);
  uint32_t total;
  const uint32_t s0 = bk_block_scan(c0 + c1, s_w, total);
  if (b0 < nb) bucket_start[b0] = s0;
  if (b1 < nb) bucket_start[b1] = s0 + c0;
  // segment x of bucket b: [lo, hi); its cursor starts at lo
  uint32_t l0 = s0, l1 = s0 + c0;
  for (uint32_t x = 0; x < SP_NSEG; ++x) {
    const uint32_t h0 = sp_seg_start(s0, s0 + c0, x + 1, s_frac), h1 = sp_seg_start(s0 + c0, s0 + c0 + c1, x + 1, s_frac);
    if (b0 < nb) {
      cursor[x * BK_MAXB + b0] = l0;
      cursor[SP_LO_OFF + x * BK_MAXB + b0] = l0;
      cursor[SP_END_OFF + x * BK_MAXB + b0] = h0;
    }
    if (b1 < nb) {
      cursor[x * BK_MAXB + b1] = l1;
      cursor[SP_LO_OFF + x * BK_MAXB + b1] = l1;
      cursor[SP_END_OFF + x * BK_MAXB + b1] = h1;
    }
    l0 = h0;
    l1 = h1;
  }
  if (tid == 0) bucket_start[nb] = total;
  if (tid < 4) mm[tid] = 0;
  if (tid == 4) *n_esc = 0;
}

// the host's bound on k_sp_regions' total (sum of t <= r_now)
__host__ __device__ inline uint64_t sp_capacity(uint64_t r_now, uint32_t nb) {
  return r_now + (r_now >> 4) + (uint64_t)nb * (SP_PAD + 4);
}

// Branch-free: a lane past the window's last record or holding a key outside the predicted range
// ranks into the dummy bucket BK_MAXB, whose run (the tile's last) goes to the trash area, so every
// tile -- the partial last one too -- stores all TILE slots in one unrolled loop.  The exact key
// range is not tracked here: on a hit every key lay in the predicted range, and k_bk_plan reports the
// occupied buckets for the next prediction; on a miss the window's rerun measures it.
//
// LDS traffic per record (what bounds this kernel once the loads overlap: a timing-only build without
// column loads and record stores still took 0.75 ms of the 1.3 ms C2 scatter): the rank (one returning
// LDS atomic on the bucket's count), one 8-byte read of the bucket's run entry (tile start | global
// start), one 8-byte write of the record's slot (packed record | global position) in bucket order and
// one linear 8-byte read of it in the store loop -- three random LDS accesses and one linear.  The
// reservations (one returning atomicAdd per (tile, bucket) on the XCD slot's cursor) are known before
// the LDS scatter, so the slot already carries the record's global position and the store loop needs
// no table lookup.  Escaped values (rare) are written to `wide` by the scattering lane, which still
// knows the record's column index.
//
// Block shape: SPK_BLOCK threads x SPK_ITEMS records.  512 x 16 with the 1024-bucket tables (72 KiB of
// LDS, <= 128 VGPRs): two blocks per CU, so one block's loads are in flight while the other ranks,
// scatters and stores (C2: 1.08 ms against 1.14 ms for one 1024 x 16 block per CU).
#ifndef GS_SPK_BLOCK
#define GS_SPK_BLOCK 512
#endif
#ifndef GS_SPK_ITEMS
#define GS_SPK_ITEMS 16
#endif
#ifndef GS_SPK_NT
#define GS_SPK_NT 0
#endif
#ifndef GS_SPK_LATE
#define GS_SPK_LATE 0   // 1: run deltas written after the LDS scatter (the reservations' latency hides behind it)
#endif
#ifndef GS_SPK_WAVES
#define GS_SPK_WAVES 4   // waves per SIMD: one 1024-thread block or two 512-thread blocks per CU
#endif
constexpr int SPK_BLOCK = GS_SPK_BLOCK, SPK_ITEMS = GS_SPK_ITEMS;
constexpr uint32_t SPK_TILE = (uint32_t)SPK_BLOCK * SPK_ITEMS;
static_assert(BK_MAXB % SPK_BLOCK == 0 && SPK_TILE <= 65536 && SPK_ITEMS <= 32, "tile / bucket-table shape");
template <int DIR>
__host__ __device__ constexpr uint32_t spk_tile_edges() {
  return DIR == DIR_ALL ? SPK_TILE / 2 : SPK_TILE;
}
// grid: the full tiles (in 8 XCD slots) + one block for the partial tile
template <int DIR>
__host__ __device__ inline uint32_t spk_grid(uint64_t n) {
  return (uint32_t)((n / spk_tile_edges<DIR>() + 7) / 8 * 8 + 1);
}

// block-wide exclusive scan of one u32 per thread (BLOCK threads); returns the total
template <int BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* s_w, uint32_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = BLOCK / WAVE;
  const uint32_t inc = wave_inclusive_sum(x);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t v = s_w[i];
    off += i < w ? v : 0u;
    tot += v;
  }
  total = tot;
  return off + inc - x;
}

// The bucket a thread reserves (k of its BPT): k-major (tid + k * BLOCK), so one wave-instruction of
// the reservation atomics covers 64 consecutive cursors -- 256 B, four 64-byte atomic transactions at the
// memory side -- instead of 64 cursors two apart (eight transactions).  The run order inside a tile follows
// the threads and is free (a run is contiguous either way).  A/B: GS_SPK_KMAJOR=0 (tid * BPT + k).
#ifndef GS_SPK_VEC
#define GS_SPK_VEC 1   // k_sp_scatter_pack: two records per lane and 16-byte column loads on full aligned tiles
#endif
#ifndef GS_SPK_KMAJOR
#define GS_SPK_KMAJOR 1
#endif
#define SP_BK(k) (GS_SPK_KMAJOR ? (uint32_t)tid + (uint32_t)(k) * (uint32_t)BLOCK : (uint32_t)tid * BPT + (uint32_t)(k))
template <typename V, int DIR, int NB>
__global__ __launch_bounds__(SPK_BLOCK) __attribute__((amdgpu_waves_per_eu(GS_SPK_WAVES, GS_SPK_WAVES)))
void k_sp_scatter_pack(BaseSrc<V, DIR, PAY_VAL> es, uint64_t n, int S, uint32_t nbp,
                       uint32_t* __restrict__ cursor, uint32_t* __restrict__ rec, V* __restrict__ wide,
                       uint32_t trash, unsigned long long* __restrict__ mm, unsigned long long* __restrict__ n_esc,
                       uint32_t xmask) {
  constexpr int ITEMS = SPK_ITEMS, BLOCK = SPK_BLOCK;
  constexpr int BPT = NB >= BLOCK ? NB / BLOCK : 1;   // buckets per thread
  static_assert(NB <= BK_MAXB && (NB % BLOCK == 0 || NB < BLOCK), "bucket table shape");
  constexpr uint32_t TILE = SPK_TILE;
  constexpr uint32_t ESC = 1u << 31, DUMMY = (uint32_t)NB << 16;   // kb: escaped value / dummy bucket
  __shared__ uint64_t s_slot[TILE];   // bucket order; early: packed << 32 | global position,
                                      // late: packed << 32 | tile record << 12 | bucket
#if GS_SPK_LATE
  __shared__ uint32_t s_st[NB + 1];    // run starts in the tile
  __shared__ uint32_t s_del[NB + 1];   // global start - tile start of each run
#else
  __shared__ uint64_t s_run[NB + 1];   // global start of the run << 32 | its start in the tile
#endif
  // per-bucket counts (the rank atomics): in the slots' space, read into registers before the scan's
  // barrier
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_slot);
  static_assert((NB + 1) * 4 <= TILE * 8 && TILE <= (1u << 20), "counts fit the slot array");
  __shared__ uint32_t s_w[BLOCK / WAVE];
  __shared__ uint32_t s_ovf[BLOCK / WAVE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr uint32_t TE = spk_tile_edges<DIR>();
  const uint32_t nfull = (uint32_t)(n / TE);
  const uint32_t lmask = (1u << S) - 1;
  uint32_t t, nrec = TILE;
  if (blockIdx.x == gridDim.x - 1) {   // the window's partial last tile
    if ((uint64_t)nfull * TE >= n) return;
    t = nfull;
    nrec = (uint32_t)((n - (uint64_t)nfull * TE) * (DIR == DIR_ALL ? 2 : 1));
  } else {   // XCD slot b & 7 owns a contiguous range of full tiles (k_dp_scatter)
    const uint32_t per = (nfull + 7) / 8;
    t = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (t >= nfull) return;
  }
  const uint32_t r0 = t * TILE;
  // this block's XCD slot: its segment (xmask 0: one segment per bucket, the merges' sorted runs)
  const uint32_t xs = SP_NSEG == 1 ? 0u : blockIdx.x & xmask;
  auto col_index = [&](uint32_t j) -> uint32_t { return DIR == DIR_ALL ? (r0 + j) >> 1 : r0 + j; };
  // this thread's buckets (BPT consecutive ones): their segment ends, issued before the columns
  uint32_t send[BPT];
#pragma unroll
  for (int k = 0; k < BPT; ++k) send[k] = cursor[SP_END_OFF + xs * BK_MAXB + min(SP_BK(k), nbp - 1)];
  cursor += xs * BK_MAXB;
  // loads: unconditional, clamped into the tile (k_dp_scatter).  Full OUT / IN tiles of 16-byte aligned
  // columns (GS_SPK_VEC): two consecutive records per lane and load -- 16-byte key loads (and 16- or 8-byte
  // value loads) instead of 8-byte ones, half the load instructions for the same bytes; record u of a
  // thread is then 2 ((u >> 1) BLOCK + tid) + (u & 1) of the tile (jof), which the ranking, the escapes and
  // the dead-lane check use -- the LDS slots and the stores do not depend on it.
  const int64_t* kcol = DIR == DIR_IN ? es.dst : es.src;
  const bool vec = GS_SPK_VEC && DIR != DIR_ALL && nrec == TILE &&
                   ((((uintptr_t)kcol) | ((uintptr_t)es.val)) & 15u) == 0;
  auto jof = [&](int u) -> uint32_t {
    return vec ? 2u * ((uint32_t)(u >> 1) * BLOCK + tid) + (uint32_t)(u & 1) : (uint32_t)u * BLOCK + tid;
  };
  int64_t kk[ITEMS];
  V vv[ITEMS];
  if (vec) {
#pragma unroll
    for (int u = 0; u < ITEMS; u += 2) {
      const uint32_t r = r0 + 2u * ((uint32_t)(u >> 1) * BLOCK + tid);
      const ulonglong2 k2 = *reinterpret_cast<const ulonglong2*>(kcol + r);
      kk[u] = (int64_t)k2.x;
      kk[u + 1] = (int64_t)k2.y;
      if constexpr (sizeof(V) == 8) {
        const ulonglong2 v2 = *reinterpret_cast<const ulonglong2*>(es.val + r);
        vv[u] = (V)v2.x;
        vv[u + 1] = (V)v2.y;
      } else {
        const uint2 v2 = *reinterpret_cast<const uint2*>(es.val + r);
        vv[u] = (V)v2.x;
        vv[u + 1] = (V)v2.y;
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
      const uint32_t r = r0 + min((uint32_t)u * BLOCK + tid, nrec - 1);
      uint32_t i = r;
      bool rev = DIR == DIR_IN;
      if constexpr (DIR == DIR_ALL) {
        i = r >> 1;
        rev = r & 1u;
      }
#if GS_SPK_NT   // A/B: the columns are read once: non-temporal loads
      kk[u] = __builtin_nontemporal_load(&(rev ? es.dst : es.src)[i]);
      vv[u] = __builtin_nontemporal_load(&es.val[i]);
#else
      kk[u] = (rev ? es.dst : es.src)[i];
      vv[u] = es.val[i];
#endif
    }
  }
  for (uint32_t i = tid; i < nbp; i += BLOCK) s_cnt[i] = 0;
  if (tid == 0) s_cnt[NB] = 0;
  // kb: ESC | bucket << 16 | bucket-local vertex (DUMMY for dead lanes / keys outside the range);
  // vr: narrow value (PK_ESC for an escape) << 16 | rank in the tile's run
  uint32_t kb[ITEMS], vr[ITEMS];
  uint32_t ovf = 0;
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint32_t j = jof(u);
    const uint64_t d = (uint64_t)kk[u] - (uint64_t)es.base;
    const bool in = (d >> S) < nbp, live = j < nrec;
    ovf += (live && !in) ? 1u : 0u;
    const uint32_t nv = pk_narrow(vv[u]);
    kb[u] = (live && in) ? ((uint32_t)(d >> S) << 16) | ((uint32_t)d & lmask) | (nv == PK_ESC ? ESC : 0u) : DUMMY;
    vr[u] = nv << 16;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) vr[u] |= atomicAdd(&s_cnt[(kb[u] >> 16) & 0x7FFFu], 1u);
  __syncthreads();
  // reserve this thread's runs on the slot's cursors
  uint32_t cb[BPT], ob[BPT], sum = 0;
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    const uint32_t b = SP_BK(k);
    cb[k] = b < nbp ? s_cnt[b] : 0u;
    sum += cb[k];
  }
#pragma unroll
  for (int k = 0; k < BPT; ++k) ob[k] = cb[k] ? atomicAdd(&cursor[SP_BK(k)], cb[k]) : 0u;
  uint32_t total;
  uint32_t st = block_excl_scan<BLOCK>(sum, s_w, total);   // total: records in the predicted range
  // A run that does not fit its segment goes to the trash area [trash, trash + TILE) past every region,
  // at its tile position (nothing reads the trash).
#if GS_SPK_LATE
  // late: the scatter needs only the tile starts; the reservations are waited for after it
  uint32_t sb[BPT];
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    sb[k] = st;
    if (SP_BK(k) < NB) s_st[SP_BK(k)] = st;
    st += cb[k];
  }
  if (tid == 0) s_st[NB] = total;   // the dummy run: the tile's last
  __syncthreads();
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint32_t b = (kb[u] >> 16) & 0x7FFFu;
    const uint32_t packed = (kb[u] & 0xFFFFu) | (vr[u] & 0xFFFF0000u);
    s_slot[s_st[b] + (vr[u] & 0xFFFFu)] = ((uint64_t)packed << 32) | (jof(u) << 12) | b;
  }
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    const bool drop = cb[k] && ob[k] + cb[k] > send[k];
    ovf += drop ? 1u : 0u;
    if (SP_BK(k) < NB) s_del[SP_BK(k)] = drop ? trash : ob[k] - sb[k];
  }
  if (tid == 0) s_del[NB] = trash;
  __syncthreads();
  uint32_t esc = 0;
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint32_t j = (uint32_t)u * BLOCK + tid;
    const uint64_t e = s_slot[j];
    const uint32_t g = j + s_del[(uint32_t)e & 0xFFFu];
    const uint32_t packed = (uint32_t)(e >> 32);
    rec[g] = packed;
    if ((packed >> 16) == PK_ESC && ((uint32_t)e & 0xFFFu) != (uint32_t)NB) {   // rare: the full value into `wide`
      wide[g] = es.val[col_index(((uint32_t)e >> 12) & 0xFFFFFu)];
      ++esc;
    }
  }
#else
  // early: every slot carries its record's global position, so the store loop needs no table lookup
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    const bool drop = cb[k] && ob[k] + cb[k] > send[k];
    ovf += drop ? 1u : 0u;
    if (SP_BK(k) < NB) s_run[SP_BK(k)] = ((uint64_t)(drop ? trash + st : ob[k]) << 32) | st;
    st += cb[k];
  }
  if (tid == 0) s_run[NB] = ((uint64_t)(trash + total) << 32) | total;   // the dummy run: the tile's last
  __syncthreads();
  uint32_t escm = 0;
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint64_t e = s_run[(kb[u] >> 16) & 0x7FFFu];
    const uint32_t rk = vr[u] & 0xFFFFu;
    const uint32_t packed = (kb[u] & 0xFFFFu) | (vr[u] & 0xFFFF0000u);
    s_slot[(uint32_t)e + rk] = ((uint64_t)packed << 32) | ((uint32_t)(e >> 32) + rk);
    escm |= (kb[u] & ESC) ? 1u << u : 0u;
  }
  uint32_t esc = 0;
  for (; escm; escm &= escm - 1, ++esc) {   // the full value from the column into the record's slot of `wide`
    const int u = __builtin_ctz(escm);
    uint32_t ku = 0, ru = 0;
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {   // (register arrays indexed by a runtime u would go to scratch)
      ku = q == u ? kb[q] : ku;
      ru = q == u ? vr[q] : ru;
    }
    const uint32_t g = (uint32_t)(s_run[(ku >> 16) & 0x7FFFu] >> 32) + (ru & 0xFFFFu);
    wide[g] = es.val[col_index(jof(u))];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint64_t e = s_slot[(uint32_t)u * BLOCK + tid];
    rec[(uint32_t)e] = (uint32_t)(e >> 32);
  }
#endif
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    esc += __shfl_xor(esc, o, WAVE);
    ovf += __shfl_xor(ovf, o, WAVE);
  }
  if (lane == 0) {
    if (esc) atomicAdd(n_esc, (unsigned long long)esc);
    s_ovf[w] = ovf;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t o2 = 0;
    for (int i = 0; i < BLOCK / WAVE; ++i) o2 += s_ovf[i];
    if (o2) atomicAdd(&mm[2], (unsigned long long)o2);
  }
}
// The same speculative partition for the unpacked records (k_dp_scatter's layout: a 16-bit bucket-local
// index in k16, the payload in vout): 8-byte values (Double sums, windows whose values escape), COUNT
// (no payload) and the degree / max-neighbour folds (the neighbour, or REL: its 32-bit offset from the
// window base, flagged in *rel_bad when it does not fit).  Same regions, segments, cursors, dummy bucket
// and trash area as k_sp_scatter_pack.  Float SUM accumulates in LDS-atomic order anyway (1e-5).
// Block shape (round 3, as k_sp_scatter_pack): SPU_BLOCK x SPU_ITEMS records with bucket tables sized for
// the window's buckets (NB), so two or more blocks share a CU (8-byte payload: 68 KiB of LDS at NB 1024).
#ifndef GS_SPU_BLOCK
#define GS_SPU_BLOCK 512
#endif
#ifndef GS_SPU_ITEMS
#define GS_SPU_ITEMS 10
#endif
constexpr int SPU_BLOCK = GS_SPU_BLOCK, SPU_ITEMS = GS_SPU_ITEMS;
constexpr uint32_t SPU_TILE = (uint32_t)SPU_BLOCK * SPU_ITEMS;
static_assert(SPU_TILE < 65536, "tile positions in 16 bits");
template <int DIR>
__host__ __device__ constexpr uint32_t spu_tile_edges() {
  return DIR == DIR_ALL ? SPU_TILE / 2 : SPU_TILE;
}
template <int DIR>
__host__ __device__ inline uint32_t spu_grid(uint64_t n) {
  return (uint32_t)((n / spu_tile_edges<DIR>() + 7) / 8 * 8 + 1);
}
template <typename V, int DIR, int PAY, typename VO, bool REL, int NB>
__global__ __launch_bounds__(SPU_BLOCK) __attribute__((amdgpu_waves_per_eu(4))) void k_sp_scatter(
    BaseSrc<V, DIR, PAY> es, uint64_t n, int S, uint32_t nbp, uint32_t* __restrict__ cursor,
    uint16_t* __restrict__ k16, VO* __restrict__ vout, uint32_t trash, uint32_t* __restrict__ rel_bad,
    unsigned long long* __restrict__ mm, uint32_t xmask) {
  constexpr bool HAS_V = PAY != PAY_NONE;
  constexpr int BLOCK = SPU_BLOCK, ITEMS = SPU_ITEMS, BPT = NB / BLOCK;   // buckets per thread
  static_assert(NB % BLOCK == 0 && NB <= BK_MAXB, "bucket table shape");
  constexpr uint32_t TILE = SPU_TILE;
  constexpr uint32_t DUMMY = (uint32_t)NB << 16;
  __shared__ uint32_t s_key[TILE];                // (bucket << 16) | bucket-local index, bucket order
  __shared__ VO s_val[HAS_V ? TILE : 1];
  __shared__ uint32_t s_cnt[NB + 1];
  __shared__ uint32_t s_delta[NB + 1];
  __shared__ uint32_t s_w[BLOCK / WAVE];
  __shared__ uint32_t s_ovf[BLOCK / WAVE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr uint32_t TE = spu_tile_edges<DIR>();
  const uint32_t nfull = (uint32_t)(n / TE);
  const uint32_t lmask = (1u << S) - 1;
  uint32_t t, nrec = TILE;
  if (blockIdx.x == gridDim.x - 1) {   // the window's partial last tile
    if ((uint64_t)nfull * TE >= n) return;
    t = nfull;
    nrec = (uint32_t)((n - (uint64_t)nfull * TE) * (DIR == DIR_ALL ? 2 : 1));
  } else {   // XCD slot b & 7 owns a contiguous range of full tiles (k_dp_scatter)
    const uint32_t per = (nfull + 7) / 8;
    t = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (t >= nfull) return;
  }
  const uint32_t r0 = t * TILE;
  const uint32_t xs = SP_NSEG == 1 ? 0u : blockIdx.x & xmask;
  uint32_t send[BPT];
#pragma unroll
  for (int k = 0; k < BPT; ++k) send[k] = sp_hi(cursor, xs, min(SP_BK(k), nbp - 1));
  cursor += xs * BK_MAXB;
  int64_t kk[ITEMS];
  V vv[ITEMS];
  // full OUT / IN tiles of 16-byte aligned columns: two records per lane and load, as k_sp_scatter_pack
  // (GS_SPK_VEC; record u of a thread is jof(u) of the tile, which only the dead-lane check uses)
  static_assert(ITEMS % 2 == 0, "two records per lane and load");
  const int64_t* kcol = DIR == DIR_IN ? es.dst : es.src;
  const void* pcol = PAY == PAY_VAL ? (const void*)es.val : PAY == PAY_NBR ? (const void*)(DIR == DIR_IN ? es.src : es.dst)
                                                                          : (const void*)kcol;
  const bool vec = GS_SPK_VEC && DIR != DIR_ALL && nrec == TILE && ((((uintptr_t)kcol) | ((uintptr_t)pcol)) & 15u) == 0;
  auto jof = [&](int u) -> uint32_t {
    return vec ? 2u * ((uint32_t)(u >> 1) * BLOCK + tid) + (uint32_t)(u & 1) : (uint32_t)u * BLOCK + tid;
  };
  if (vec) {
#pragma unroll
    for (int u = 0; u < ITEMS; u += 2) {
      const uint32_t r = r0 + 2u * ((uint32_t)(u >> 1) * BLOCK + tid);
      const ulonglong2 k2 = *reinterpret_cast<const ulonglong2*>(kcol + r);
      kk[u] = (int64_t)k2.x;
      kk[u + 1] = (int64_t)k2.y;
      if constexpr (PAY == PAY_NBR) {
        const ulonglong2 v2 = *reinterpret_cast<const ulonglong2*>((const int64_t*)pcol + r);
        vv[u] = (V)v2.x;
        vv[u + 1] = (V)v2.y;
      } else if constexpr (PAY == PAY_VAL && sizeof(V) == 8) {
        const ulonglong2 v2 = *reinterpret_cast<const ulonglong2*>(es.val + r);
        vv[u] = __builtin_bit_cast(V, v2.x);
        vv[u + 1] = __builtin_bit_cast(V, v2.y);
      } else if constexpr (PAY == PAY_VAL && sizeof(V) == 4) {
        const uint2 v2 = *reinterpret_cast<const uint2*>(es.val + r);
        vv[u] = __builtin_bit_cast(V, v2.x);
        vv[u + 1] = __builtin_bit_cast(V, v2.y);
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {   // every load first, unconditional and clamped into the tile
      const uint32_t r = r0 + min((uint32_t)u * BLOCK + tid, nrec - 1);
      uint32_t i = r;
      bool rev = DIR == DIR_IN;
      if constexpr (DIR == DIR_ALL) {
        i = r >> 1;
        rev = r & 1u;
      }
      kk[u] = (rev ? es.dst : es.src)[i];
      if constexpr (PAY == PAY_VAL) vv[u] = es.val[i];
      else if constexpr (PAY == PAY_NBR) vv[u] = (V)(rev ? es.src : es.dst)[i];
    }
  }
  uint32_t ovf = 0, kb[ITEMS];
  bool bad = false;
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint32_t j = jof(u);
    const uint64_t d = (uint64_t)kk[u] - (uint64_t)es.base;
    const bool in = (d >> S) < nbp, live = j < nrec;
    ovf += (live && !in) ? 1u : 0u;
    kb[u] = (live && in) ? ((uint32_t)(d >> S) << 16) | ((uint32_t)d & lmask) : DUMMY;
  }
  for (uint32_t i = tid; i < nbp; i += BLOCK) s_cnt[i] = 0;
  if (tid == 0) s_cnt[NB] = 0;
  __syncthreads();
  uint32_t rk[ITEMS];
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    if constexpr (GS_SP_MATCH && PAY == PAY_NBR) {
      // folds (C3's hub-heavy streams): the lanes sharing the wave's first lane's bucket take one atomic
      // for all of them instead of serialising same-address LDS atomics (Zipf C3 scatter 1.82 -> 1.44 ms;
      // R-MAT C3 +2 %, Double reduce +6 %: value reduces keep the plain atomics)
      const uint32_t b = kb[u] >> 16, L = __builtin_amdgcn_readfirstlane(b);
      const uint64_t same = __ballot(b == L);
      uint32_t base = 0;
      if ((threadIdx.x & 63) == 0) base = atomicAdd(&s_cnt[L], (uint32_t)__popcll(same));
      base = __builtin_amdgcn_readfirstlane(base);
      rk[u] = b == L ? base + mbcnt(same) : atomicAdd(&s_cnt[b], 1u);
    } else {
      rk[u] = atomicAdd(&s_cnt[kb[u] >> 16], 1u);
    }
  }
  __syncthreads();
  uint32_t cb[BPT], ob[BPT], sum = 0;
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    const uint32_t b = SP_BK(k);
    cb[k] = b < nbp ? s_cnt[b] : 0u;
    sum += cb[k];
  }
#pragma unroll
  for (int k = 0; k < BPT; ++k) ob[k] = cb[k] ? atomicAdd(&cursor[SP_BK(k)], cb[k]) : 0u;
  uint32_t total;
  uint32_t st = block_excl_scan<BLOCK>(sum, s_w, total);   // (bk_block_scan assumes 1024 threads)
  uint32_t sb[BPT];
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    sb[k] = st;
    s_cnt[SP_BK(k)] = st;   // (entries past nbp are never read)
    st += cb[k];
  }
  if (tid == 0) s_cnt[NB] = total;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint32_t pos = s_cnt[kb[u] >> 16] + rk[u];
    s_key[pos] = kb[u];
    if constexpr (REL) {   // a dead or outside lane's payload is never checked (it goes to the trash)
      const uint64_t rel = (uint64_t)vv[u] - (uint64_t)es.base;
      bad |= kb[u] != DUMMY && (rel >> 32) != 0;
      s_val[pos] = (VO)rel;
    } else if constexpr (HAS_V) {
      s_val[pos] = (VO)vv[u];
    }
  }
#pragma unroll
  for (int k = 0; k < BPT; ++k) {
    const bool drop = cb[k] && ob[k] + cb[k] > send[k];
    s_delta[SP_BK(k)] = (drop ? trash : ob[k]) - sb[k];
    ovf += drop ? 1u : 0u;
  }
  if (tid == 0) s_delta[NB] = trash;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < ITEMS; ++u) {
    const uint32_t j = (uint32_t)u * BLOCK + tid;
    const uint32_t kv = s_key[j];
    const uint32_t g = s_delta[kv >> 16] + j;
    k16[g] = (uint16_t)kv;
    if constexpr (HAS_V) vout[g] = s_val[j];
  }
  if constexpr (REL) {
    if (__any(bad) && lane == 0) atomicOr(rel_bad, 1u);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ovf += __shfl_xor(ovf, o, WAVE);
  if (lane == 0) s_ovf[w] = ovf;
  __syncthreads();
  if (tid == 0) {
    uint32_t o2 = 0;
    for (int i = 0; i < BLOCK / WAVE; ++i) o2 += s_ovf[i];
    if (o2) atomicAdd(&mm[2], (unsigned long long)o2);
  }
}

// ---- k_bk_accum: persistent; LDS accumulation of (bucket, record range) items ---------------------
// Finalize (shared with k_bk_merge): the bucket's vertices in ascending order -> staging at the
// bucket's record offset (a bucket has at least as many records as vertices).
// RESET (k_bk_accum): each wave then returns its own entries to the identity -- the next item needs no
// block-wide init pass and no barrier for it.
template <class P, bool RESET = false>
__device__ __forceinline__ void bk_finalize(typename P::Lds& s, uint32_t bucket, uint32_t stage_at,
                                            BkStage st, uint32_t* bucket_count, uint32_t* s_wc) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr uint32_t PER = P::W / BK_NW;   // entries per wave
  const uint32_t e0 = (uint32_t)w * PER;
  uint32_t cnt = 0;
  for (uint32_t j = 0; j < PER; j += WAVE) cnt += (uint32_t)__popcll(ballot(P::present(s, e0 + j + lane)));
  if (lane == 0) s_wc[w] = cnt;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < BK_NW; ++i) {
    const uint32_t v = s_wc[i];
    off += i < w ? v : 0u;
    tot += v;
  }
  const uint32_t cbase = bucket << P::S;
  for (uint32_t j = 0; j < PER; j += WAVE) {
    const uint32_t e = e0 + j + lane;
    const bool p = P::present(s, e);
    const uint64_t m = ballot(p);
    if (p) {
      const uint32_t pos = stage_at + off + mbcnt(m);
      st.k[pos] = cbase | e;
      P::stage(st, pos, s, e);
    }
    off += (uint32_t)__popcll(m);
  }
  if constexpr (RESET) {
    static_assert(PER % 32 == 0, "a wave's entries are whole presence words");
    P::init_range(s, e0, e0 + PER, lane);
  }
  if (tid == 0) bucket_count[bucket] = tot;
}

#ifdef GS_BK_TRACE
constexpr uint32_t BK_TRACE_MAX = 16384;
__device__ uint64_t g_bk_trace[BK_TRACE_MAX][4];
#endif
// The item loop is pipelined (round 6): wave 0 claims the NEXT item, reads its descriptor and bucket start,
// computes its pieces (speculative packed partition) and loads their unaligned head / tail records while the
// other waves finish the current item's stream; the block then finalizes the current item, re-initializes
// the table and starts the next one with all of that already in LDS and registers.  Before, each item began
// with a chain of dependent global-memory latencies (claim -> descriptor -> bucket start -> segment bounds ->
// head / tail records, one record after another) behind two barriers, with no stream load in flight on the CU.
template <class P, class Src, int UNROLL>
__global__ __launch_bounds__(BK_ACC_BLOCK) void k_bk_accum(Src src, const BkItem* __restrict__ items,
                                                           const uint32_t* __restrict__ n_items_p,
                                                           const uint32_t* __restrict__ bucket_start,
                                                           uint32_t* __restrict__ ctr,
                                                           typename P::Lds* __restrict__ slabs, BkStage st,
                                                           uint32_t* __restrict__ bucket_count,
                                                           const unsigned long long* __restrict__ mm,
                                                           const uint32_t* __restrict__ seg_cur) {
  __shared__ typename P::Lds s;
  __shared__ uint32_t s_item[2], s_b0[2];   // two slots: the current item and the one wave 0 stages
  __shared__ BkItem s_m[2];
  __shared__ uint32_t s_wc[BK_NW];
  __shared__ uint32_t s_pre4[2][SP_NSEG + 1], s_qb[2][SP_NSEG];   // packed records: the item's pieces as one stream
  using Raw = typename P::Raw;
  constexpr bool PACKED = is_pack_src<Src>::value;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  if (mm[2]) return;   // keys outside the predicted range: the window is rerun
  const uint32_t n_items = *n_items_p;
  // packed records: one record into LDS (the value from `wide` when escaped)
  auto add1 = [&](const auto& sr, uint32_t q, uint32_t x) {
    const uint32_t v16 = x >> 16;
    const bool esc = v16 == PK_ESC;
    if constexpr (has_add_packed<P>::value) P::add_packed(s, x & (P::W - 1), !esc ? (Raw)v16 : (Raw)sr.wide[q], esc);
    else P::add(s, x & (P::W - 1), !esc ? (Raw)v16 : (Raw)sr.wide[q]);
  };
  // wave 0: claim an item into slot b and stage its descriptor, bucket start and (speculative packed
  // partition) its pieces; lane 6x + j (< 6 SP_NSEG) loads record j of piece x's unaligned head (j < 3) or
  // tail, which it adds once the table is ready (hh: it holds one)
  uint32_t hq = 0, hx = 0;
  bool hh = false;
  auto prepare = [&](int b) {
    uint32_t it = 0;
    if (lane == 0) it = atomicAdd(ctr, 1u);
    it = __shfl(it, 0, WAVE);
    if (lane == 0) s_item[b] = it;
    hh = false;
    if (it >= n_items) return;
    const BkItem m = items[it];
    const uint32_t b0 = bucket_start[m.bucket];
    if (lane == 0) {
      s_m[b] = m;
      s_b0[b] = b0;
    }
    if constexpr (PACKED) {
      if (seg_cur) {
        // the item's pieces of the bucket's SP_NSEG segments, in segment order, as ONE stream of 16-byte
        // groups (a loop per segment drained and refilled the loads in flight at each segment boundary):
        // lane x < SP_NSEG takes segment x's piece [p0, p1) and publishes its groups' place in the stream
        const bool on = lane < (int)SP_NSEG;
        const uint32_t x = on ? (uint32_t)lane : 0u;
        const uint32_t sg = sp_lo(seg_cur, x, m.bucket);
        const uint32_t nx = on ? min(seg_cur[x * BK_MAXB + m.bucket], sp_hi(seg_cur, x, m.bucket)) - sg : 0u;
        const uint32_t at = wave_inclusive_sum(nx) - nx;   // records of the bucket in the segments before x
        const uint32_t lo = max(m.begin, at), hi = min(m.end, at + nx);
        uint32_t p0 = 0, p1 = 0;
        if (on && lo < hi) {
          p0 = sg + (lo - at);
          p1 = sg + (hi - at);
        }
        const uint32_t a0 = min(p1, (p0 + 3) & ~3u), a1 = max(a0, p1 & ~3u);
        const uint32_t n4 = (a1 - a0) / 4;
        const uint32_t e4 = wave_inclusive_sum(n4);
        if (on) {
          s_pre4[b][x + 1] = e4;
          s_qb[b][x] = a0 / 4 - (e4 - n4);   // group g of piece x: uint4 index g + s_qb[x]
        }
        if (lane == 0) s_pre4[b][0] = 0;
        const uint32_t px = (uint32_t)lane / 6, j = (uint32_t)lane % 6;
        const uint32_t xp0 = __shfl(p0, (int)px, WAVE), xa0 = __shfl(a0, (int)px, WAVE);
        const uint32_t xa1 = __shfl(a1, (int)px, WAVE), xp1 = __shfl(p1, (int)px, WAVE);
        const uint32_t q = j < 3 ? xp0 + j : xa1 + (j - 3);
        hh = px < SP_NSEG && (j < 3 ? q < xa0 : q < xp1);
        if (hh) {
          hq = q;
          hx = src.rec[q];
        }
      }
    }
  };
  if (tid < WAVE) prepare(0);
  P::init(s, tid);
  __syncthreads();
  constexpr int U4 = UNROLL / 2 > 0 ? UNROLL / 2 : 1;
  // (GS_BK_PREFETCH) the next item's first group of 16-byte loads, issued before this item's finalize
  uint4 xp[U4];
  uint32_t qp[U4];
  bool pf = false;
  for (int sl = 0;; sl ^= 1) {
    const uint32_t it = s_item[sl];
    if (it >= n_items) break;
    const BkItem m = s_m[sl];
    const uint32_t b0 = s_b0[sl];
#ifdef GS_BK_TRACE
    const uint64_t t_item0 = wall_clock64();
#endif
    if constexpr (PACKED) {
      // packed records: 16-byte loads (4 records per lane per load: 4x the bytes in flight of 4-byte
      // loads; the 4-byte version was latency-bound); unaligned heads and tails record by record
      const uint4* rec4 = reinterpret_cast<const uint4*>(src.rec);
      constexpr uint32_t STEP = BK_ACC_BLOCK * U4;
      // n4 groups of 4 records, group g at uint4 index q4_of(g) of the partition
      auto stream = [&](uint32_t n4, auto q4_of) {
        for (uint32_t g4 = tid; g4 < n4; g4 += STEP) {
          uint4 x[U4];
          uint32_t qi[U4];
          if (pf) {   // the first group, loaded before the previous item's finalize
#pragma unroll
            for (int u = 0; u < U4; ++u) {
              x[u] = xp[u];
              qi[u] = qp[u];
            }
            pf = false;
          } else {
#pragma unroll
            for (int u = 0; u < U4; ++u) {   // unconditional, clamped: see k_dp_hist
              const uint32_t g = g4 + (uint32_t)u * BK_ACC_BLOCK;
              qi[u] = q4_of(g < n4 ? g : n4 - 1);
              x[u] = rec4[qi[u]];
            }
          }
          // every load of the group issued before the first use (the scheduler moved the first
          // group's decode, and its wait, between the loads)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int u = 0; u < U4; ++u) {
            if (g4 + (uint32_t)u * BK_ACC_BLOCK >= n4) continue;
            const uint32_t q = 4 * qi[u];
            if constexpr (fast_packed<P>::value) {
              // one branch per 4 records: the common case (narrow values, for SUM non-zero) is 4 LDS atomics
              // and nothing else; escapes and zero SUM values (presence bytes, the wide value) take add1.
              // (A branch per record cost ~4 scalar instructions each: the accumulate ran 7x more SALU than
              // LDS instructions.)
              const uint32_t h0 = x[u].x >> 16, h1 = x[u].y >> 16, h2 = x[u].z >> 16, h3 = x[u].w >> 16;
              bool rare = (h0 == PK_ESC) | (h1 == PK_ESC) | (h2 == PK_ESC) | (h3 == PK_ESC);
              if constexpr (P::OP_IS_SUM) rare |= (h0 == 0u) | (h1 == 0u) | (h2 == 0u) | (h3 == 0u);
              if (!rare) {
                P::add_narrow(s, x[u].x & (P::W - 1), h0);
                P::add_narrow(s, x[u].y & (P::W - 1), h1);
                P::add_narrow(s, x[u].z & (P::W - 1), h2);
                P::add_narrow(s, x[u].w & (P::W - 1), h3);
                continue;
              }
            }
            add1(src, q, x[u].x);
            add1(src, q + 1, x[u].y);
            add1(src, q + 2, x[u].z);
            add1(src, q + 3, x[u].w);
          }
        }
        pf = false;   // (a thread with no group in this item drops its prefetch)
      };
      if (!seg_cur) {   // records [r0, r1) of the partition
        const uint32_t r0 = b0 + m.begin, r1 = b0 + m.end;
        const uint32_t a0 = min(r1, (r0 + 3) & ~3u), a1 = max(a0, r1 & ~3u);
        if (r0 + tid < a0) add1(src, r0 + tid, src.rec[r0 + tid]);
        if (a1 + tid < r1) add1(src, a1 + tid, src.rec[a1 + tid]);
        stream((a1 - a0) / 4, [&](uint32_t g) { return a0 / 4 + g; });
      } else {
        if (hh) add1(src, hq, hx);   // wave 0's staged head / tail records
        // group g of the stream lies in the last piece x with s_pre4[x] <= g (empty pieces share their
        // start with the next one): the pieces' bounds in registers, a branch-free select per load (a
        // cursor walking s_pre4 in LDS put an LDS read and its wait between consecutive loads)
        // (as a sum of the bases' steps: a select chain compiled to a table in scratch memory)
        uint32_t pre[SP_NSEG], dq[SP_NSEG];
#pragma unroll
        for (uint32_t x = 0; x < SP_NSEG; ++x) {
          pre[x] = s_pre4[sl][x];
          dq[x] = x ? s_qb[sl][x] - s_qb[sl][x - 1] : s_qb[sl][0];
        }
        stream(s_pre4[sl][SP_NSEG], [&](uint32_t g) {
          uint32_t b = dq[0];
#pragma unroll
          for (uint32_t x = 1; x < SP_NSEG; ++x) b += g >= pre[x] ? dq[x] : 0u;
          return g + b;
        });
      }
    } else {
    auto range = [&](uint32_t r0, uint32_t r1) {   // records [r0, r1) of the partition into LDS
    if constexpr (is_part_src<Src>::value) {
      // unpacked partition (2-byte keys + the payload, k_dp_scatter / k_sp_scatter): 4 consecutive records
      // per lane and step -- one 8-byte load of their keys, one (4-byte values) or two (8-byte values)
      // 16-byte loads of their values; an unaligned head and the tail record by record.  (A 2-byte key
      // load and an 8-byte value load per record kept too few bytes in flight: Double C2's accumulate
      // ran at 4.3 TB/s.)
      using V = std::remove_cv_t<std::remove_pointer_t<decltype(src.vals)>>;
      constexpr bool HV = !std::is_same_v<V, uint8_t>;
      auto add1 = [&](uint32_t q) {
        uint32_t k;
        V v{};
        src.load(q, k, v);
        P::add(s, k & (P::W - 1), (Raw)v);
      };
      const uint32_t a0 = min(r1, (r0 + 3) & ~3u), a1 = max(a0, r1 & ~3u);
      if (r0 + tid < a0) add1(r0 + tid);
      constexpr int U4 = UNROLL / 2 > 0 ? UNROLL / 2 : 1;
      constexpr uint32_t STEP = BK_ACC_BLOCK * U4;
      const uint32_t q_end = a1 / 4;
      const uint2* k4 = reinterpret_cast<const uint2*>(src.keys);
      for (uint32_t q4 = a0 / 4 + tid; q4 < q_end; q4 += STEP) {
        uint2 kx[U4];
        V vx[U4][4];
#pragma unroll
        for (int u = 0; u < U4; ++u) {   // unconditional, clamped (see k_dp_hist)
          const uint32_t qq = min(q4 + (uint32_t)u * BK_ACC_BLOCK, q_end - 1);
          kx[u] = k4[qq];
          if constexpr (HV && sizeof(V) == 4) {
            const uint4 w = reinterpret_cast<const uint4*>(src.vals)[qq];
            vx[u][0] = __builtin_bit_cast(V, w.x);
            vx[u][1] = __builtin_bit_cast(V, w.y);
            vx[u][2] = __builtin_bit_cast(V, w.z);
            vx[u][3] = __builtin_bit_cast(V, w.w);
          } else if constexpr (HV && sizeof(V) == 8) {
            const ulonglong2 w0 = reinterpret_cast<const ulonglong2*>(src.vals)[2 * qq];
            const ulonglong2 w1 = reinterpret_cast<const ulonglong2*>(src.vals)[2 * qq + 1];
            vx[u][0] = __builtin_bit_cast(V, w0.x);
            vx[u][1] = __builtin_bit_cast(V, w0.y);
            vx[u][2] = __builtin_bit_cast(V, w1.x);
            vx[u][3] = __builtin_bit_cast(V, w1.y);
          } else {
            vx[u][0] = vx[u][1] = vx[u][2] = vx[u][3] = V{};
          }
        }
#pragma unroll
        for (int u = 0; u < U4; ++u) {
          if (q4 + (uint32_t)u * BK_ACC_BLOCK < q_end) {
            P::add(s, (kx[u].x & 0xFFFFu) & (P::W - 1), (Raw)vx[u][0]);
            P::add(s, (kx[u].x >> 16) & (P::W - 1), (Raw)vx[u][1]);
            P::add(s, (kx[u].y & 0xFFFFu) & (P::W - 1), (Raw)vx[u][2]);
            P::add(s, (kx[u].y >> 16) & (P::W - 1), (Raw)vx[u][3]);
          }
        }
      }
      if (a1 + tid < r1) add1(a1 + tid);
    } else {
      for (uint32_t r = r0 + tid; r < r1; r += BK_ACC_BLOCK * UNROLL) {
        uint32_t k[UNROLL];
        Raw v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          const uint32_t q = r + (uint32_t)u * BK_ACC_BLOCK;
          src.load(q < r1 ? q : r1 - 1, k[u], v[u]);   // unconditional: see k_dp_hist
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          const uint32_t q = r + (uint32_t)u * BK_ACC_BLOCK;
          if (q < r1) P::add(s, k[u] & (P::W - 1), v[u]);
        }
      }
    }
    };
    if (!seg_cur) {
      range(b0 + m.begin, b0 + m.end);
    } else {   // speculative partition: the item's span of the bucket's SP_NSEG segments, in order
      uint32_t at = 0;   // records of the bucket in the segments before x
      for (uint32_t x = 0; x < SP_NSEG && at < m.end; ++x) {
        const uint32_t sg = sp_lo(seg_cur, x, m.bucket);
        const uint32_t nx = min(seg_cur[x * BK_MAXB + m.bucket], sp_hi(seg_cur, x, m.bucket)) - sg;
        const uint32_t lo = max(m.begin, at), hi = min(m.end, at + nx);
        if (lo < hi) range(sg + (lo - at), sg + (hi - at));
        at += nx;
      }
    }
    }
    // the next item: wave 0 claims and stages it in the other slot while the other waves finish this one
    if (tid < WAVE) prepare(sl ^ 1);
    __syncthreads();
#if GS_BK_PREFETCH
    if constexpr (PACKED) {   // the next item's first group in flight during this item's finalize
      const int nx = sl ^ 1;
      if (seg_cur && s_item[nx] < n_items && s_pre4[nx][SP_NSEG]) {
        const uint32_t n4n = s_pre4[nx][SP_NSEG];
        uint32_t pre[SP_NSEG], dq[SP_NSEG];
#pragma unroll
        for (uint32_t x = 0; x < SP_NSEG; ++x) {
          pre[x] = s_pre4[nx][x];
          dq[x] = x ? s_qb[nx][x] - s_qb[nx][x - 1] : s_qb[nx][0];
        }
        const uint4* rec4 = reinterpret_cast<const uint4*>(src.rec);
#pragma unroll
        for (int u = 0; u < U4; ++u) {
          const uint32_t g0 = (uint32_t)tid + (uint32_t)u * BK_ACC_BLOCK, g = g0 < n4n ? g0 : n4n - 1;
          uint32_t b = dq[0];
#pragma unroll
          for (uint32_t x = 1; x < SP_NSEG; ++x) b += g >= pre[x] ? dq[x] : 0u;
          qp[u] = g + b;
          xp[u] = rec4[qp[u]];
        }
        pf = true;
      }
    }
#endif
    bool reset = false;
    if (m.slab == ~0u) {
      bk_finalize<P, GS_BK_FUSED_RESET != 0>(s, m.bucket, b0, st, bucket_count, s_wc);
      reset = GS_BK_FUSED_RESET != 0;
    } else {
      // dump the LDS accumulators (k_bk_merge, a later launch, combines the bucket's slabs)
      const uint4* ls = reinterpret_cast<const uint4*>(&s);
      uint4* gs = reinterpret_cast<uint4*>(slabs + m.slab);
      for (uint32_t i = tid; i < sizeof(typename P::Lds) / 16; i += BK_ACC_BLOCK) gs[i] = ls[i];
    }
    __syncthreads();
#ifdef GS_BK_TRACE   // tuning builds only: per item (workgroup, item, wall clock at 100 MHz, records)
    if (tid == 0 && it < BK_TRACE_MAX) {
      g_bk_trace[it][0] = blockIdx.x;
      g_bk_trace[it][1] = t_item0;
      g_bk_trace[it][2] = wall_clock64();
      g_bk_trace[it][3] = m.end - m.begin;
    }
#endif
    if (!reset) {   // (block-uniform: the item's slab)
      P::init(s, tid);
      __syncthreads();
    }
  }
}

// Slabs of a multi-item bucket merged into its first slab, BK_MS_SLICES blocks per bucket, each over
// one slice of the vertex range (a hub bucket can leave hundreds of slabs: one block per bucket
// merged them serially).  Fixed element -> thread map: deterministic merge order.  Two levels: slab k
// of a bucket with more than BK_MS_GROUPS slabs is first merged into slab k mod BK_MS_GROUPS
// (k_bk_merge_groups: a Zipf hub bucket's ~700 slabs as 16 chains of ~44 instead of one of 700, which
// ran the C3 Zipf merge at 0.19 ms), then slabs 1 .. 15 into slab 0 (k_bk_merge_slices).
constexpr uint32_t BK_MS_SLICES = 64, BK_MS_BLOCK = 256, BK_MS_GROUPS = 16;

// level 1: work unit (multi bucket, slice, group z): slabs z + 16, z + 32, ... into slab z
template <class P>
__global__ __launch_bounds__(BK_MS_BLOCK) void k_bk_merge_groups(const uint32_t* __restrict__ mlist,
                                                                 const uint32_t* __restrict__ n_multi_p,
                                                                 const uint32_t* __restrict__ b_items,
                                                                 const uint32_t* __restrict__ b_slab,
                                                                 typename P::Lds* __restrict__ slabs,
                                                                 const unsigned long long* __restrict__ mm,
                                                                 const uint32_t* __restrict__ max_items) {
  if (mm[2] || *max_items <= BK_MS_GROUPS) return;   // (every bucket's slabs fit level 2: C2's 2-3)
  const uint32_t units = *n_multi_p * BK_MS_SLICES * BK_MS_GROUPS;
  constexpr uint32_t EL = P::W / BK_MS_SLICES, PWS = (P::PWORDS + BK_MS_SLICES - 1) / BK_MS_SLICES;
  for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {
    const uint32_t mb = u / (BK_MS_SLICES * BK_MS_GROUPS), rem = u % (BK_MS_SLICES * BK_MS_GROUPS);
    const uint32_t sl = rem / BK_MS_GROUPS, z = rem % BK_MS_GROUPS;
    const uint32_t b = mlist[mb];
    const uint32_t n = b_items[b], f = b_slab[b];
    if (z + BK_MS_GROUPS >= n) continue;   // (block-uniform)
    typename P::Lds* __restrict__ d = slabs + f + z;
    const typename P::Lds* __restrict__ rest = slabs + f + z + BK_MS_GROUPS;   // slab z + 16 (k + 1)
    const uint32_t nk = (n - z - 1) / BK_MS_GROUPS;                            // slabs in this chain
    const uint32_t e0 = sl * EL, w0 = sl * PWS;
    for (uint32_t i = threadIdx.x; i < EL; i += BK_MS_BLOCK) {
#pragma unroll 8
      for (uint32_t k = 0; k < nk; ++k) P::merge_el(d, rest + (size_t)k * BK_MS_GROUPS, e0 + i);
    }
    for (uint32_t w = threadIdx.x; w < PWS && w0 + w < P::PWORDS; w += BK_MS_BLOCK) {
#pragma unroll 8
      for (uint32_t k = 0; k < nk; ++k) P::merge_pw(d, rest + (size_t)k * BK_MS_GROUPS, w0 + w);
    }
  }
}
template <class P>
__global__ __launch_bounds__(BK_MS_BLOCK) void k_bk_merge_slices(const uint32_t* __restrict__ mlist,
                                                                 const uint32_t* __restrict__ n_multi_p,
                                                                 const uint32_t* __restrict__ b_items,
                                                                 const uint32_t* __restrict__ b_slab,
                                                                 typename P::Lds* __restrict__ slabs,
                                                                 const unsigned long long* __restrict__ mm) {
  if (mm[2]) return;
  const uint32_t n_multi = *n_multi_p;
  // blocks loop over the multi-item buckets (the grid is sized without a read-back of their number: one
  // block per possible bucket and slice left ~65 K blocks exiting at once for C2's ~30, 16 us of dispatch)
  for (uint32_t mb = blockIdx.x; mb < n_multi; mb += gridDim.x) {
    const uint32_t b = mlist[mb];
    const uint32_t n = b_items[b], f = b_slab[b];
    // d and the other slabs never overlap (restrict): d's elements stay in registers across the slabs and
    // the slab loads of an unrolled group issue together (a dependent read-modify-write of d per slab made
    // the merge latency-bound: Zipf hub buckets of ~100 slabs, C3 0.78 ms)
    typename P::Lds* __restrict__ d = slabs + f;
    const typename P::Lds* __restrict__ rest = slabs + f + 1;
    const uint32_t nk = min(n, BK_MS_GROUPS) - 1;   // the group heads 1 .. 15 (k_bk_merge_groups)
    constexpr uint32_t EL = P::W / BK_MS_SLICES, PWS = (P::PWORDS + BK_MS_SLICES - 1) / BK_MS_SLICES;
    const uint32_t e0 = blockIdx.y * EL, w0 = blockIdx.y * PWS;
    for (uint32_t i = threadIdx.x; i < EL; i += BK_MS_BLOCK) {
#pragma unroll 8
      for (uint32_t k = 0; k < nk; ++k) P::merge_el(d, rest + k, e0 + i);
    }
    for (uint32_t w = threadIdx.x; w < PWS && w0 + w < P::PWORDS; w += BK_MS_BLOCK) {
#pragma unroll 8
      for (uint32_t k = 0; k < nk; ++k) P::merge_pw(d, rest + k, w0 + w);
    }
  }
}

// finalize a multi-item bucket from its merged first slab
template <class P>
__global__ __launch_bounds__(BK_ACC_BLOCK) void k_bk_merge(const uint32_t* __restrict__ mlist,
                                                           const uint32_t* __restrict__ n_multi_p,
                                                           const uint32_t* __restrict__ b_items,
                                                           const uint32_t* __restrict__ b_slab,
                                                           const uint32_t* __restrict__ bucket_start,
                                                           const typename P::Lds* __restrict__ slabs, BkStage st,
                                                           uint32_t* __restrict__ bucket_count,
                                                           const unsigned long long* __restrict__ mm) {
  __shared__ typename P::Lds s;
  __shared__ uint32_t s_wc[BK_NW];
  const int tid = threadIdx.x;
  if (mm[2]) return;
  const uint32_t n_multi = *n_multi_p;
  for (uint32_t mb = blockIdx.x; mb < n_multi; mb += gridDim.x) {   // (grid: see k_bk_merge_slices)
    const uint32_t b = mlist[mb];
    const uint32_t f = b_slab[b];
    {
      const uint4* gs = reinterpret_cast<const uint4*>(slabs + f);
      uint4* ls = reinterpret_cast<uint4*>(&s);
      for (uint32_t i = tid; i < sizeof(typename P::Lds) / 16; i += BK_ACC_BLOCK) ls[i] = gs[i];
    }
    __syncthreads();
    bk_finalize<P>(s, b, bucket_start[b], st, bucket_count, s_wc);
    __syncthreads();   // (the next bucket's slab overwrites s)
  }
}

// ---- k_bk_emit: staging -> outputs, vertices ascending --------------------------------------------
template <class P>
// host (GS_FLAG_ASYNC_OUTPUT): block 0 first writes the window's whole read-back block -- the plan's and the
// scatter's words, U (every bucket's count, final after the merges), the timeout flag and the escapes --
// into pinned host memory, then `seq` behind a system-scope fence; the host returns on it while the other
// blocks still emit (the outputs are complete in stream order).
__global__ __launch_bounds__(256) void k_bk_emit(const uint32_t* __restrict__ bucket_start,
                                                 const uint32_t* __restrict__ bucket_count, uint32_t nb,
                                                 BkStage st, int64_t base, typename P::Out o,
                                                 unsigned long long* __restrict__ n_out,
                                                 const unsigned long long* __restrict__ mm,
                                                 const uint32_t* __restrict__ timeout,
                                                 const unsigned long long* __restrict__ n_esc,
                                                 unsigned long long* __restrict__ res,
                                                 unsigned long long* __restrict__ host = nullptr, uint64_t seq = 0) {
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (blockIdx.x == 0 && tid == 0) {   // the read-back block: [timeout flag, escapes] after mm / ns
    res[0] = *timeout;
    res[1] = *n_esc;
  }
  if (host && blockIdx.x == 0) {
    uint64_t tot = 0;
    if (!mm[2])
      for (uint32_t i = tid; i < nb; i += 256) tot += bucket_count[i];
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) tot += __shfl_xor(tot, o2, WAVE);
    __shared__ uint64_t s_tot[4];
    if (lane == 0) s_tot[w] = tot;
    __syncthreads();
    if (tid == 0) {
      const unsigned long long* ns = mm + 4;   // SM_BK_N = SM_BK_MM + 32: the plan's counts, two words
      host[0] = mm[0];
      host[1] = mm[1];
      host[2] = mm[2];
      host[3] = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
      host[4] = ns[0];
      host[5] = ns[1];
      host[6] = *timeout;
      host[7] = *n_esc;
      __threadfence_system();
      __hip_atomic_store(host + 8, (unsigned long long)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (mm[2]) return;
  const uint32_t b = blockIdx.x;
  uint32_t part = 0;
  for (uint32_t i = tid; i < b; i += 256) part += bucket_count[i];
#pragma unroll
  for (int o2 = 32; o2 > 0; o2 >>= 1) part += __shfl_xor(part, o2, WAVE);
  if (lane == 0) s_w[w] = part;
  __syncthreads();
  const uint64_t off = (uint64_t)s_w[0] + s_w[1] + s_w[2] + s_w[3];
  const uint32_t n = bucket_count[b], j0 = bucket_start[b];
  for (uint32_t i = tid; i < n; i += 256) {
    const uint32_t j = j0 + i;
    P::emit(o, off + i, (int64_t)((uint64_t)base + st.k[j]), st, j, base);
  }
  if (b == nb - 1 && tid == 0) *n_out = off + n;
}

// ---- the keyBy exchange's emit (gs_dist.hip): staging -> packed rows grouped by owner ----------------
// Instead of k_bk_emit's ascending (vertex, value) output, which gs_window_reduce_dist then partitioned by
// owner and packed: per bucket, its rows per owner (k_bk_owner_count), an owner-major scan (k_owner_scan),
// then each bucket's rows written straight into the exchange's rows of their owner, in vertex order
// (k_bk_owner_emit).  Row: key (1 word; 2 when a key of this window lies outside [0, 2^32)), the value
// (vw words, as P::emit converts it), [the maximum (mw words)].
// Each bucket's rows in BK_OE_SLICES slices (grid (buckets, slices)): a C2 window has ~7 K rows per bucket,
// which one block per bucket walked in 256-row steps (owner count 27 us, emit 65 us at one block per bucket)
constexpr uint32_t BK_OE_SLICES = 8;
__global__ __launch_bounds__(256) void k_bk_owner_count(const uint32_t* __restrict__ bucket_start,
                                                        const uint32_t* __restrict__ bucket_count, uint32_t nb,
                                                        const uint32_t* __restrict__ stk, int64_t base, uint32_t nparts,
                                                        uint32_t* __restrict__ cnt, unsigned long long* __restrict__ wide,
                                                        const unsigned long long* __restrict__ mm,
                                                        const uint32_t* __restrict__ timeout,
                                                        const unsigned long long* __restrict__ n_esc,
                                                        unsigned long long* __restrict__ res) {
  __shared__ uint32_t s_c[64];
  const int tid = threadIdx.x;
  const uint32_t b = blockIdx.x;
  if (b == 0 && blockIdx.y == 0 && tid == 0) {   // the read-back block: [timeout flag, escapes] (as k_bk_emit)
    res[0] = *timeout;
    res[1] = *n_esc;
  }
  if (tid < 64) s_c[tid] = 0;
  __syncthreads();
  if (mm[2]) return;
  const uint64_t lt = (1ull << (tid & 63)) - 1;
  const uint32_t nbk = bucket_count[b], sl = blockIdx.y;
  const uint32_t r0 = (uint32_t)((uint64_t)nbk * sl / BK_OE_SLICES), r1 = (uint32_t)((uint64_t)nbk * (sl + 1) / BK_OE_SLICES);
  const uint32_t n = r1 - r0, j0 = bucket_start[b] + r0;
  bool w = false;
  constexpr int U = 4;   // rows per lane per step: their loads issued together
  for (uint32_t i0 = 0; i0 < n; i0 += 256 * U) {   // same trip count on every lane (ballots)
    uint32_t kc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + (uint32_t)u * 256 + tid;
      kc[u] = i < n ? stk[j0 + i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool valid = i0 + (uint32_t)u * 256 + tid < n;
      const int64_t key = (int64_t)((uint64_t)base + kc[u]);
      w |= valid && ((uint64_t)key >> 32) != 0;
      const uint32_t o = valid ? owner_of(key, nparts) : 0u;
      const uint64_t peers = match_digit<6>(o, ballot(valid));
      if (valid && (peers & lt) == 0) atomicAdd(&s_c[o], (uint32_t)__popcll(peers));
    }
  }
  if (wide && __any(w) && (tid & 63) == 0) atomicOr(wide, 1ull);
  __syncthreads();
  if (tid < (int)nparts) cnt[(uint64_t)tid * nb * BK_OE_SLICES + b * BK_OE_SLICES + sl] = s_c[tid];
}

template <class P>
__global__ __launch_bounds__(256) void k_bk_owner_emit(const uint32_t* __restrict__ bucket_start,
                                                       const uint32_t* __restrict__ bucket_count, uint32_t nb,
                                                       BkStage st, int64_t base, typename P::Out o, uint32_t nparts,
                                                       const uint32_t* __restrict__ off, uint32_t* __restrict__ rows,
                                                       const unsigned long long* __restrict__ wide, int vw, int mw,
                                                       const unsigned long long* __restrict__ mm) {
  __shared__ int64_t s_key[256];
  __shared__ uint64_t s_v[256];
  __shared__ int64_t s_v2[256];
  __shared__ uint32_t s_wc[4][64];   // per wave: rows of each owner in this chunk
  __shared__ uint32_t s_run[64];     // per owner: rows of this bucket written before this chunk
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (mm[2]) return;
  const uint32_t b = blockIdx.x, sl = blockIdx.y;
  const uint32_t nbk = bucket_count[b];
  const uint32_t r0 = (uint32_t)((uint64_t)nbk * sl / BK_OE_SLICES), r1 = (uint32_t)((uint64_t)nbk * (sl + 1) / BK_OE_SLICES);
  const uint32_t n = r1 - r0, j0 = bucket_start[b] + r0;
  const uint64_t cslot = (uint64_t)b * BK_OE_SLICES + sl, cstride = (uint64_t)nb * BK_OE_SLICES;
  const uint32_t kw = (*wide & 1ull) ? 2u : 1u, rw = kw + (uint32_t)vw + (uint32_t)mw;
  const typename P::Out lo = o.retarget(s_key, s_v, s_v2);
  const uint64_t lt = (1ull << lane) - 1;
  if (tid < 64) s_run[tid] = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += 256) {
    (&s_wc[0][0])[tid] = 0;
    __syncthreads();
    const uint32_t i = i0 + tid;
    const bool valid = i < n;
    uint32_t ow = 0, r = 0;
    if (valid) {
      const uint32_t j = j0 + i;
      const int64_t key = (int64_t)((uint64_t)base + st.k[j]);
      P::emit(lo, (uint64_t)tid, key, st, j, base);   // this row's key and converted value(s), in LDS
      ow = owner_of(key, nparts);
    }
    const uint64_t peers = match_digit<6>(ow, ballot(valid));
    if (valid) {
      r = (uint32_t)__popcll(peers & lt);
      if (r == 0) s_wc[w][ow] = (uint32_t)__popcll(peers);
    }
    __syncthreads();
    if (valid) {
      uint32_t before = s_run[ow];
      for (int x = 0; x < w; ++x) before += s_wc[x][ow];
      const uint64_t pos = (uint64_t)off[(uint64_t)ow * cstride + cslot] + before + r;
      uint32_t* wr = rows + pos * rw;
      const uint64_t k = (uint64_t)s_key[tid];
      wr[0] = (uint32_t)k;
      if (kw == 2) wr[1] = (uint32_t)(k >> 32);
      if (vw == 1) {
        wr[kw] = reinterpret_cast<const uint32_t*>(s_v)[tid];
      } else {
        const uint64_t v = s_v[tid];
        wr[kw] = (uint32_t)v;
        wr[kw + 1] = (uint32_t)(v >> 32);
      }
      if (mw) {
        const uint64_t m = (uint64_t)s_v2[tid];
        wr[kw + vw] = (uint32_t)m;
        wr[kw + vw + 1] = (uint32_t)(m >> 32);
      }
    }
    __syncthreads();
    if (tid < (int)nparts) s_run[tid] += s_wc[0][tid] + s_wc[1][tid] + s_wc[2][tid] + s_wc[3][tid];
    __syncthreads();   // (the next chunk clears s_wc)
  }
}

}  // namespace gs
