// gs_ops.hpp — helpers shared by the operator translation units (engine, graph).
#pragma once
#include <algorithm>

#include "gs_internal.hpp"
#include "gs_radix.hpp"
#include "gs_rbk.hpp"

#define GS_TRY(x)                       \
  do {                                  \
    gs_status _s = (x);                 \
    if (_s != GS_OK) return _s;         \
  } while (0)
#define GS_HIP(x) GS_TRY(hip_check(c, (x), #x))

namespace gs {

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
  GS_HIP(hipStreamSynchronize(c->stream));
  if ((uint32_t)c->host_small[3] != 0) return set_error(c, GS_EDEVICE, "look-back spin timed out");
  *n_unique_host = c->host_small[2];
  return GS_OK;
}

inline void finish_times(gs_ctx* c, const Sorted& s, uint64_t U) {
  hipEventSynchronize(c->ev[3]);
  float a = 0, b = 0, d = 0;
  hipEventElapsedTime(&a, c->ev[0], c->ev[1]);
  hipEventElapsedTime(&b, c->ev[1], c->ev[2]);
  hipEventElapsedTime(&d, c->ev[2], c->ev[3]);
  c->times.keyinfo_ms = a;
  c->times.sort_ms = b;
  c->times.reduce_ms = d;
  c->times.total_ms = a + b + d;
  c->times.sort_passes = (uint32_t)s.passes;
  c->times.key_bits = (uint32_t)s.bits;
  c->times.records = s.records;
  c->times.vertices = U;
  for (int p = 0; p < 8; ++p) {
    float t = 0;
    if (p < s.passes) hipEventElapsedTime(&t, c->pass_ev[p], c->pass_ev[p + 1]);
    c->times.pass_ms[p] = t;
  }
  c->times.key_bytes = s.wide ? 8 : 4;
  c->times.payload_bytes = (uint32_t)s.payload_bytes;
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

}  // namespace gs
