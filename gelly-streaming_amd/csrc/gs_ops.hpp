// gs_ops.hpp — helpers shared by the operator translation units (engine, graph).
#pragma once
#include <algorithm>

#include "gs_internal.hpp"
#include "gs_radix.hpp"
#include "gs_rbk.hpp"
#include "gs_combine.hpp"

#define GS_TRY(x)                       \
  do {                                  \
    gs_status _s = (x);                 \
    if (_s != GS_OK) return _s;         \
  } while (0)
#define GS_HIP(x) GS_TRY(hip_check(c, (x), #x))

namespace gs {

// owner(v) of the multi-GPU keyBy (gs_owner_of): a murmur3 finaliser of the vertex, scaled to nparts
__host__ __device__ inline uint32_t owner_of(int64_t v, uint32_t nparts) {
  uint64_t x = (uint64_t)v;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)(((x >> 32) * (uint64_t)nparts) >> 32);
}

// one block: exclusive scan of cnt[0 .. n) (owner-major) in place; totals[o] = partials of owner o, *n_out
// (optional) = all of them (gs_dist.hip's owner partition; the bucket path's owner-grouped emit)
static __global__ __launch_bounds__(1024) void k_owner_scan(uint32_t* __restrict__ cnt, uint32_t n, uint32_t tiles,
                                                            uint32_t nparts, unsigned long long* __restrict__ totals,
                                                            unsigned long long* __restrict__ n_out) {
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_tot;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t per = (n + 1023) / 1024, a = min(n, tid * per), b = min(n, a + per);
  uint32_t sum = 0;
  for (uint32_t i = a; i < b; ++i) sum += cnt[i];
  const uint32_t inc = wave_inclusive_sum(sum);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int i = 0; i < 16; ++i) {
    off += i < w ? s_w[i] : 0u;
    tot += s_w[i];
  }
  uint32_t run = off + inc - sum;
  for (uint32_t i = a; i < b; ++i) {
    const uint32_t x = cnt[i];
    cnt[i] = run;
    run += x;
  }
  if (tid == 0) {
    s_tot = tot;
    if (n_out) *n_out = tot;
  }
  __syncthreads();
  if (tid < (int)nparts) {
    const uint32_t lo = cnt[(uint64_t)tid * tiles], hi = tid + 1 < (int)nparts ? cnt[(uint64_t)(tid + 1) * tiles] : s_tot;
    totals[tid] = hi - lo;
  }
}

// send row per peer p: [rows for p, flags] (flags: 1 = wide keys on this rank, 2 = this rank failed);
// then the key-width flag is cleared for the next window's k_owner_count (no memset per window; a flag
// left set by a failed window only widens that next window's keys)
// With `miss` / `timeout` (the owner-grouped emit of a window whose read-back the caller defers): 4 = this
// rank's speculative partition missed (every rank then sends its counts again after this rank reruns), 2 =
// its look-back timed out
static __global__ void k_send_rows(const unsigned long long* __restrict__ totals, unsigned long long* __restrict__ wide,
                            uint32_t nparts, unsigned long long* __restrict__ send,
                            const unsigned long long* __restrict__ miss, const uint32_t* __restrict__ timeout) {
  const uint32_t p = threadIdx.x;
  const unsigned long long fl = (*wide & 1ull) | (miss && miss[2] ? 4ull : 0ull) | (timeout && *timeout ? 2ull : 0ull);
  if (p < nparts) {
    send[2 * p] = totals[p];
    send[2 * p + 1] = fl;
  }
  __syncthreads();
  if (p == 0) *wide = 0;
}

// tile shapes (overridable with -D for tuning builds: make VARIANT="-DGS_SORT_ITEMS=24")
#ifndef GS_SORT_BLOCK
#define GS_SORT_BLOCK 512
#endif
#ifndef GS_SORT_ITEMS
#define GS_SORT_ITEMS 16
#endif
#ifndef GS_RBK_BLOCK
#define GS_RBK_BLOCK 256
#endif
#ifndef GS_RBK_ITEMS
#define GS_RBK_ITEMS 16
#endif
#ifndef GS_COMB_BLOCK
#define GS_COMB_BLOCK 256
#endif
#ifndef GS_COMB_ITEMS
#define GS_COMB_ITEMS 12
#endif
constexpr int COMB_BLOCK = GS_COMB_BLOCK, COMB_ITEMS = GS_COMB_ITEMS, COMB_TILE = COMB_BLOCK * COMB_ITEMS;
constexpr int SORT_BLOCK = GS_SORT_BLOCK, SORT_ITEMS = GS_SORT_ITEMS, SORT_TILE = SORT_BLOCK * SORT_ITEMS;
constexpr int RBK_BLOCK = GS_RBK_BLOCK, RBK_ITEMS = GS_RBK_ITEMS, RBK_TILE = RBK_BLOCK * RBK_ITEMS;

// ---- reduce-by-key launch ----------------------------------------------------------------------
template <typename K, class Op, class Out>
inline gs_status launch_rbk(gs_ctx* c, const Sorted& s, Out o, uint64_t* n_unique_host, uint32_t key_shift = 0) {
  char* sm = c->small.as<char>();
  const uint32_t R = (uint32_t)s.records;
  const uint32_t tiles = (R + RBK_TILE - 1) / RBK_TILE;
  constexpr int SLOTS = accum_slots(sizeof(typename Op::Acc));
  GS_TRY(ensure(c, c->rbk_word, (size_t)tiles * 8, true));
  GS_TRY(ensure(c, c->rbk_agg, (size_t)tiles * 8 * SLOTS));
  GS_TRY(ensure(c, c->rbk_inc, (size_t)tiles * 8 * SLOTS));
  const uint32_t ep = next_epoch(c, 0);
  GS_HIP(hipMemsetAsync((uint32_t*)(sm + SM_COUNTERS) + 63, 0, 4, c->stream));   // fresh tile counter per launch
  hipLaunchKernelGGL((k_reduce_by_key<K, Op, Out, RBK_BLOCK, RBK_ITEMS>), dim3(tiles), dim3(RBK_BLOCK), 0, c->stream,
                     (const K*)s.keys, (const typename Op::In*)s.vals, R, s.key_xor, key_shift, o,
                     c->rbk_word.as<uint64_t>(),
                     c->rbk_agg.as<uint64_t>(), c->rbk_inc.as<uint64_t>(), (uint32_t*)(sm + SM_COUNTERS) + 63, tiles,
                     ep, (uint32_t*)(sm + SM_TIMEOUT), (unsigned long long*)(sm + SM_NUNIQUE));
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[3], c->stream);
  GS_HIP(hipMemcpyAsync(c->host_small, sm, 32, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if ((uint32_t)c->host_small[3] != 0) return set_error(c, GS_EDEVICE, "look-back spin timed out");
  *n_unique_host = c->host_small[2];
  return GS_OK;
}

inline void finish_times(gs_ctx* c, const Sorted& s, uint64_t U) {
  hipEventSynchronize(c->ev[3]);
  float a = 0, b = 0, d = 0;
  a = event_ms(c->ev[0], c->ev[1]);
  b = event_ms(c->ev[1], c->ev[2]);
  d = event_ms(c->ev[2], c->ev[3]);
  c->times.keyinfo_ms = a;
  c->times.sort_ms = b;
  c->times.reduce_ms = d;
  c->times.total_ms = a + b + d;
  c->times.sort_passes = (uint32_t)s.passes;
  c->times.key_bits = (uint32_t)s.bits;
  c->times.records = s.records;
  c->times.vertices = U;
  const int launched = s.done_passes + (s.fused ? 1 : 0);
  for (int p = 0; p < 8; ++p) {
    float t = 0;
    if (p < launched) t = event_ms(c->pass_ev[p], c->pass_ev[p + 1]);
    c->times.pass_ms[p] = t;
  }
  c->times.sort_passes = (uint32_t)launched;
  if (!s.fused) c->times.partials = 0;
  c->times.key_bytes = s.wide ? 8 : 4;
  c->times.payload_bytes = (uint32_t)s.payload_bytes;
  c->times.fused_last = s.fused ? 1u : 0u;
  c->times.path = 0;
  if (c->timing != GS_TIMING_STAGES) {   // the window's start event was not recorded (stage_event)
    c->times.keyinfo_ms = c->times.sort_ms = c->times.reduce_ms = c->times.total_ms = 0.f;
    for (int p = 0; p < 8; ++p) c->times.pass_ms[p] = 0.f;
  }
}

// Copy U staged outputs to the caller (host or device) — only when the direct write was impossible.
inline gs_status deliver(gs_ctx* c, void* dst, const void* staged, size_t bytes, int mem) {
  if (!bytes || dst == staged) return GS_OK;
  GS_HIP(hipMemcpyAsync(dst, staged, bytes, mem == GS_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                        c->stream));
  return GS_OK;
}

inline gs_status check_batch(gs_ctx* c, const gs_edge_batch* b, int dir) {
  if (!c) return GS_EINVAL;
  if (!b) return set_error(c, GS_EINVAL, "null batch");
  if (dir < 0 || dir > 2) return set_error(c, GS_EINVAL, "bad EdgeDirection %d", dir);
  if (b->n && (!b->src || !b->dst)) return set_error(c, GS_EINVAL, "null src/dst");
  if (b->val_dtype < GS_I32 || b->val_dtype > GS_NONE) return set_error(c, GS_EINVAL, "bad dtype %d", b->val_dtype);
  const uint64_t R = dir == GS_DIR_ALL ? 2 * b->n : b->n;
  if (R >= (1ull << 32)) return set_error(c, GS_EINVAL, "window has %llu records; limit is 2^32-1",
                                          (unsigned long long)R);
  return GS_OK;
}

// reduce / fold / degree fold: any window size (chunked above one pass's record cap, gs_engine.hip)
inline gs_status check_batch_any(gs_ctx* c, const gs_edge_batch* b, int dir) {
  if (!c) return GS_EINVAL;
  if (!b) return set_error(c, GS_EINVAL, "null batch");
  if (dir < 0 || dir > 2) return set_error(c, GS_EINVAL, "bad EdgeDirection %d", dir);
  if (b->n && (!b->src || !b->dst)) return set_error(c, GS_EINVAL, "null src/dst");
  if (b->val_dtype < GS_I32 || b->val_dtype > GS_NONE) return set_error(c, GS_EINVAL, "bad dtype %d", b->val_dtype);
  if (b->n >= (1ull << 62)) return set_error(c, GS_EINVAL, "window has %llu edges", (unsigned long long)b->n);
  return GS_OK;
}

// The last radix pass fused with the per-vertex combine (gs_combine.hpp), then the merge of the
// few partials a vertex leaves when its records straddle tiles.  `s` holds passes 0..P-2.
template <typename K, class Op, class Out>
inline gs_status reduce_fused(gs_ctx* c, const Sorted& s, Out o, uint64_t* U) {
  using Acc = typename Op::Acc;
  using V = std::conditional_t<Op::HAS_V, typename Op::In, uint8_t>;
  using MOp = typename MergeOf<Op>::type;
  char* sm = c->small.as<char>();
  const uint32_t R = (uint32_t)s.records;
  const int lp = s.passes - 1;
  const uint32_t tiles = (R + COMB_TILE - 1) / COMB_TILE;
  GS_TRY(ensure(c, c->part_k, (size_t)R * sizeof(K)));
  GS_TRY(ensure(c, c->part_a, (size_t)R * sizeof(Acc)));
  GS_TRY(ensure(c, c->comp_k, (size_t)R * sizeof(K)));
  GS_TRY(ensure(c, c->comp_a, (size_t)R * sizeof(Acc)));
  GS_TRY(ensure(c, c->sort_status, (size_t)tiles * RADIX * 8, true));
  const uint32_t ep = next_epoch(c, 0);
  uint32_t* ctr = (uint32_t*)(sm + SM_COUNTERS) + 40;
  GS_HIP(hipMemsetAsync(ctr, 0, 4, c->stream));
  const uint32_t* base = (const uint32_t*)(sm + SM_BASE) + lp * RADIX;
  BufSrc<K, V> bs{(const K*)s.keys, Op::HAS_V ? (const V*)s.vals : nullptr, 0};
  hipLaunchKernelGGL((k_onesweep_combine<K, Op, COMB_BLOCK, COMB_ITEMS, BufSrc<K, V>>), dim3(tiles), dim3(COMB_BLOCK),
                     0, c->stream, bs, c->part_k.as<K>(), c->part_a.as<Acc>(), R, 8u * lp, base,
                     c->sort_status.as<uint64_t>(), ctr, ep, (uint32_t*)(sm + SM_TIMEOUT));
  GS_HIP(hipGetLastError());
  hipEventRecord(c->pass_ev[s.done_passes + 1], c->stream);
  uint32_t* table = (uint32_t*)(sm + SM_TABLE);
  hipLaunchKernelGGL(k_region_table, dim3(1), dim3(RADIX), 0, c->stream, c->sort_status.as<uint64_t>(), tiles - 1, base,
                     table, (unsigned long long*)(sm + SM_TOTAL));
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(c->host_small + 5, sm + SM_TOTAL, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t parts = c->host_small[5];
  c->times.partials = parts;
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((parts + 255) / 256, 8192));
  hipLaunchKernelGGL((k_compact_runs<K, Acc>), dim3(g), dim3(256), 0, c->stream, c->part_k.as<K>(), c->part_a.as<Acc>(),
                     table, (uint32_t)parts, c->comp_k.as<K>(), c->comp_a.as<Acc>());
  GS_HIP(hipGetLastError());
  Sorted m = s;
  m.keys = c->comp_k.p;
  m.vals = c->comp_a.p;
  m.records = parts;
  if (parts == 0) {
    *U = 0;
    return GS_OK;
  }
  return launch_rbk<K, MOp>(c, m, o, U);
}

}  // namespace gs
