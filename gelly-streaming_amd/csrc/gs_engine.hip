// gs_engine.hip — C ABI lifecycle, window sort orchestration and the reduce / fold operators.
//
//   gs_window_reduce          <- GraphWindowStream.reduceOnEdges  (GraphWindowStream.java:101-121)
//   gs_window_fold            <- GraphWindowStream.foldNeighbors  (GraphWindowStream.java:62-87)
//   gs_window_fold_degree_max <- foldNeighbors with a degree / max-neighbour EdgesFold
// Window = one columnar batch: keyinfo -> LSD onesweep passes -> reduce-by-key.
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>

#include "gs_ops.hpp"

using namespace gs;

namespace gs {


gs_status set_error(gs_ctx* c, gs_status s, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
    // a failed call may have left the look-back timeout word set (e.g. a later kernel of the call timed out
    // after an earlier read-back saw it zero): the next call clears it (begin_call)
    c->timeout_clean = false;
  }
  return s;
}

gs_status host_wait(gs_ctx* c) {
  static const bool blocking = getenv("GS_BLOCKING_WAIT") != nullptr;   // A/B switch for measurements
  if (blocking) return hip_check(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  if (!c->sync_ev) GS_HIP(hipEventCreateWithFlags(&c->sync_ev, hipEventDisableTiming));
  GS_HIP(hipEventRecord(c->sync_ev, c->stream));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(c->sync_ev);
    if (e == hipSuccess) return GS_OK;
    if (e != hipErrorNotReady) return hip_check(c, e, "hipEventQuery");
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
  }
  (void)hipGetLastError();   // "not ready" is a poll result, not an error for the next launch check
  return hip_check(c, hipEventSynchronize(c->sync_ev), "hipEventSynchronize");
}

gs_status hip_check(gs_ctx* c, hipError_t e, const char* what) {
  if (e == hipSuccess) return GS_OK;
  return set_error(c, e == hipErrorOutOfMemory ? GS_ENOMEM : GS_EDEVICE, "%s: %s", what, hipGetErrorString(e));
}

gs_status ensure(gs_ctx* c, DevBuf& b, size_t bytes, bool zero) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return GS_OK;
  if (b.p) {
    GS_TRY(host_wait(c));
    GS_HIP(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  size_t want = bytes + bytes / 8;  // headroom for slightly larger windows
  GS_HIP(hipMalloc(&b.p, want));
  b.bytes = want;
  if (zero) GS_HIP(hipMemsetAsync(b.p, 0, want, c->stream));
  return GS_OK;
}

// Epochs tag look-back granules so no status buffer is cleared between launches.
uint32_t next_epoch(gs_ctx* c, size_t) {
  c->epoch++;
  if (c->epoch >= (1u << EPOCH_BITS) - 1) {
    if (c->sort_status.p) hipMemsetAsync(c->sort_status.p, 0, c->sort_status.bytes, c->stream);
    if (c->rbk_word.p) hipMemsetAsync(c->rbk_word.p, 0, c->rbk_word.bytes, c->stream);
    c->epoch = 1;
  }
  return c->epoch;
}

gs_status begin_call(gs_ctx* c) {
  ++c->call_seq;   // ends a chunked-candidates session (its sets live in shared workspace)
  c->last_kind = 0;   // the staged output buffers are about to be reused: nothing left to fetch
  (void)hipGetLastError();
  GS_HIP(hipSetDevice(c->device));
  // the look-back timeout word: cleared unless the previous call's read-back saw it zero (the bucket
  // path reads it back with every window, so back-to-back windows skip this launch)
  // (a resumed deferred window, gs_dist.hip: its read-back of the word is already on the host and checked
  // by the resumed call)
  if (!c->timeout_clean && !c->oe.resume) GS_HIP(hipMemsetAsync(c->small.as<char>() + SM_TIMEOUT, 0, 8, c->stream));
  c->timeout_clean = false;
  return GS_OK;
}

gs_status stage_batch(gs_ctx* c, const gs_edge_batch* b, const int64_t** src, const int64_t** dst, const void** val,
                      bool need_val) {
  const size_t vb = dtype_bytes(b->val_dtype);
  if (b->mem == GS_MEM_DEVICE) {
    *src = b->src;
    *dst = b->dst;
    *val = b->val;
    return GS_OK;
  }
  const size_t eb = b->n * sizeof(int64_t);
  GS_TRY(ensure(c, c->in_src, eb));
  GS_TRY(ensure(c, c->in_dst, eb));
  GS_HIP(hipMemcpyAsync(c->in_src.p, b->src, eb, hipMemcpyHostToDevice, c->stream));
  GS_HIP(hipMemcpyAsync(c->in_dst.p, b->dst, eb, hipMemcpyHostToDevice, c->stream));
  *src = c->in_src.as<int64_t>();
  *dst = c->in_dst.as<int64_t>();
  *val = nullptr;
  if (need_val && vb) {
    GS_TRY(ensure(c, c->in_val, b->n * vb));
    GS_HIP(hipMemcpyAsync(c->in_val.p, b->val, b->n * vb, hipMemcpyHostToDevice, c->stream));
    *val = c->in_val.p;
  }
  return GS_OK;
}

static inline unsigned grid_for(uint64_t n, unsigned per_block, unsigned cap) {
  const uint64_t g = (n + per_block - 1) / per_block;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

template <int DIR>
static gs_status launch_keyinfo(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, bool mask_only = false) {
  char* sm = c->small.as<char>();
  const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  const int nd = mask_only ? 0 : std::min(4, std::max(1, c->hist_digits));
  if (vec)
    hipLaunchKernelGGL((k_keyinfo<DIR, true>), dim3(grid_for(n, 2048, 2048)), dim3(256), 0, c->stream, src, dst, n,
                       nd, (unsigned long long*)(sm + SM_MASK), (uint32_t*)(sm + SM_HIST));
  else
    hipLaunchKernelGGL((k_keyinfo<DIR, false>), dim3(grid_for(n, 2048, 2048)), dim3(256), 0, c->stream, src, dst, n,
                       nd, (unsigned long long*)(sm + SM_MASK), (uint32_t*)(sm + SM_HIST));
  return hip_check(c, hipGetLastError(), "k_keyinfo");
}
gs_status launch_keyinfo_all(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, bool mask_only) {
  return launch_keyinfo<DIR_ALL>(c, src, dst, n, mask_only);
}

template <int DIR>
static gs_status launch_hist_bytes(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, uint64_t key_xor,
                                   int b0, int b1) {
  char* sm = c->small.as<char>();
  GS_HIP(hipMemsetAsync(sm + SM_HIST + b0 * 256 * 4, 0, (b1 - b0) * 256 * 4, c->stream));
  hipLaunchKernelGGL(k_hist_bytes<DIR>, dim3(grid_for(n, 256 * 8, 2048)), dim3(256), 0, c->stream, src, dst, n,
                     key_xor, b0, b1, (uint32_t*)(sm + SM_HIST));
  return hip_check(c, hipGetLastError(), "k_hist_bytes");
}

template <typename K, typename V, bool HAS_V, class Src, int DBITS = RADIX_BITS>
static gs_status launch_pass(gs_ctx* c, Src src, K* kout, V* vout, uint32_t R, int pass, uint32_t shift) {
  char* sm = c->small.as<char>();
  const uint32_t tiles = (R + SORT_TILE - 1) / SORT_TILE;
  const uint32_t ep = next_epoch(c, 0);
  const uint32_t* base = DBITS == RADIX_BITS ? (const uint32_t*)(sm + SM_BASE) + pass * RADIX
                                             : (const uint32_t*)(sm + SM_BASE9) + pass * (1 << DBITS);
  GS_HIP(hipMemsetAsync((uint32_t*)(sm + SM_COUNTERS) + pass, 0, 4, c->stream));
  hipLaunchKernelGGL((k_onesweep<K, V, HAS_V, SORT_BLOCK, SORT_ITEMS, Src, DBITS>), dim3(tiles), dim3(SORT_BLOCK), 0,
                     c->stream, src, kout, vout, R, shift, base, c->sort_status.as<uint64_t>(),
                     (uint32_t*)(sm + SM_COUNTERS) + pass, ep, (uint32_t*)(sm + SM_TIMEOUT));
  return hip_check(c, hipGetLastError(), "k_onesweep");
}

template <typename K, typename V, bool HAS_V, int DIR, int PAY>
static gs_status run_passes(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, uint32_t R,
                            Sorted* out) {
  K* ka = c->keysA.as<K>();
  K* kb = c->keysB.as<K>();
  V* va = c->valsA.as<V>();
  V* vb = c->valsB.as<V>();
  EdgeSrc<K, V, DIR, PAY> es{src, dst, (const V*)val, out->key_xor};
  hipEventRecord(c->pass_ev[0], c->stream);
  GS_TRY((launch_pass<K, V, HAS_V>(c, es, ka, va, R, 0, 0)));
  hipEventRecord(c->pass_ev[1], c->stream);
  for (int p = 1; p < out->done_passes; ++p) {
    BufSrc<K, V> bs{ka, HAS_V ? va : nullptr, 0};
    GS_TRY((launch_pass<K, V, HAS_V>(c, bs, kb, vb, R, p, 8u * p)));
    hipEventRecord(c->pass_ev[p + 1], c->stream);
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  out->payload_bytes = HAS_V ? (int)sizeof(V) : 0;
  out->keys = ka;
  out->vals = HAS_V ? (void*)va : nullptr;
  return GS_OK;
}

template <typename K, int DIR>
static gs_status dispatch_payload(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, int vbytes,
                                  uint32_t R, int payload, Sorted* out) {
  switch (payload) {
    case PAY_NONE: return run_passes<K, uint8_t, false, DIR, PAY_NONE>(c, src, dst, val, R, out);
    case PAY_VAL:
      if (vbytes == 4) return run_passes<K, uint32_t, true, DIR, PAY_VAL>(c, src, dst, val, R, out);
      return run_passes<K, uint64_t, true, DIR, PAY_VAL>(c, src, dst, val, R, out);
    case PAY_NBR: return run_passes<K, uint64_t, true, DIR, PAY_NBR>(c, src, dst, val, R, out);
    case PAY_IDX: return run_passes<K, uint32_t, true, DIR, PAY_IDX>(c, src, dst, val, R, out);
  }
  return set_error(c, GS_EINVAL, "bad payload kind %d", payload);
}

template <int DIR>
static gs_status sort_dir(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, int vbytes,
                          uint64_t n, int payload, Sorted* out, bool leave_last) {
  char* sm = c->small.as<char>();
  const uint64_t R = (DIR == DIR_ALL) ? 2 * n : n;
  GS_HIP(hipMemsetAsync(sm, 0, SM_TIMEOUT, c->stream));                            // mask, k0, n_unique
  GS_HIP(hipMemsetAsync(sm + SM_COUNTERS, 0, SM_BASE - SM_COUNTERS, c->stream));   // counters, hist
  GS_TRY(launch_keyinfo<DIR>(c, src, dst, n));
  const int64_t* k0p = (DIR == DIR_IN) ? dst : src;
  GS_HIP(hipMemcpyAsync(sm + SM_K0, k0p, 8, hipMemcpyDeviceToDevice, c->stream));
  GS_HIP(hipMemcpyAsync(c->host_small, sm, 16, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint64_t mask = c->host_small[0], k0 = c->host_small[1];
  const int bits = mask ? 64 - __builtin_clzll(mask) : 0;
  out->bits = bits;
  out->wide = bits > 32;
  out->passes = std::max(1, (bits + RADIX_BITS - 1) / RADIX_BITS);
  out->done_passes = leave_last ? std::max(1, out->passes - 1) : out->passes;
  out->records = R;
  out->key_xor = out->wide ? (1ull << 63) : (k0 & 0xFFFFFFFF00000000ull);
  const int have = std::min(4, std::max(1, c->hist_digits));
  if (out->wide) GS_TRY(launch_hist_bytes<DIR>(c, src, dst, n, out->key_xor, 0, out->passes));   // sign-flipped bytes
  else if (out->passes > have) GS_TRY(launch_hist_bytes<DIR>(c, src, dst, n, out->key_xor, have, out->passes));
  c->hist_digits = std::min(4, out->passes);
  hipLaunchKernelGGL(k_digit_base, dim3(1), dim3(256), 0, c->stream, (const uint32_t*)(sm + SM_HIST),
                     (uint32_t*)(sm + SM_BASE), out->passes);
  GS_HIP(hipGetLastError());
  hipEventRecord(c->ev[1], c->stream);
  const size_t kb = out->wide ? 8 : 4;
  const size_t vb = payload == PAY_NONE ? 0 : payload == PAY_IDX ? 4 : payload == PAY_NBR ? 8 : (size_t)vbytes;
  const uint64_t tiles = (R + SORT_TILE - 1) / SORT_TILE;
  GS_TRY(ensure(c, c->keysA, R * kb));
  GS_TRY(ensure(c, c->keysB, R * kb));
  if (vb) {
    GS_TRY(ensure(c, c->valsA, R * vb));
    GS_TRY(ensure(c, c->valsB, R * vb));
  }
  GS_TRY(ensure(c, c->sort_status, tiles * RADIX * 8, true));
  if (out->wide) return dispatch_payload<uint64_t, DIR>(c, src, dst, val, vbytes, (uint32_t)R, payload, out);
  return dispatch_payload<uint32_t, DIR>(c, src, dst, val, vbytes, (uint32_t)R, payload, out);
}

template <typename K, typename V, bool HAS_V, int DBITS = RADIX_BITS>
static gs_status buffer_passes(gs_ctx* c, const uint64_t* keys, const V* vals, uint32_t R, Sorted* out) {
  K* ka = c->keysA.as<K>();
  K* kb = c->keysB.as<K>();
  V* va = c->valsA.as<V>();
  V* vb = c->valsB.as<V>();
  ConvSrc<K, V> cs{keys, HAS_V ? vals : nullptr, out->key_xor};
  hipEventRecord(c->pass_ev[0], c->stream);
  GS_TRY((launch_pass<K, V, HAS_V, ConvSrc<K, V>, DBITS>(c, cs, ka, va, R, 0, 0)));
  hipEventRecord(c->pass_ev[1], c->stream);
  for (int p = 1; p < out->passes; ++p) {
    BufSrc<K, V> bs{ka, HAS_V ? va : nullptr, 0};
    GS_TRY((launch_pass<K, V, HAS_V, BufSrc<K, V>, DBITS>(c, bs, kb, vb, R, p, (uint32_t)DBITS * p)));
    hipEventRecord(c->pass_ev[p + 1], c->stream);
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  out->keys = ka;
  out->vals = HAS_V ? (void*)va : nullptr;
  out->payload_bytes = HAS_V ? (int)sizeof(V) : 0;
  return GS_OK;
}

// 9-bit digits are off by default: on the s26 triangle window one pass less of each sort still cost more
// than it saved (6 x 9-bit passes of the oriented keys 96.8-98.7 vs 89.8 ms for 7 x 8-bit, the transposed
// sort 40 vs 36.6 ms; same box, profiles/r05/tri/d9_ab/): each 512-bin pass looks back over twice the
// digits, ranks with 9 ballots and writes runs of half the length.  GS_SORT_DIGIT9=1 turns them on (A/B).
int sort_digit_bits(int bits) {
  static const bool on = getenv("GS_SORT_DIGIT9") && getenv("GS_SORT_DIGIT9")[0] == '1';
  return on && bits > 0 && (bits + 8) / 9 < (bits + 7) / 8 ? 9 : 8;
}

gs_status sort_buffer(gs_ctx* c, const uint64_t* keys, const void* vals, uint64_t n, Sorted* out, int bits_hint,
                      int val_bytes, bool hist_ready, int digit_bits) {
  char* sm = c->small.as<char>();
  if (digit_bits == 9 && !hist_ready) return set_error(c, GS_EINVAL, "sort_buffer: 9-bit digits need a known key width");
  const int nd = std::min(8, std::max(1, (bits_hint + 7) / 8));
  int bits = bits_hint;
  uint64_t k0 = 0;
  GS_HIP(hipMemsetAsync(sm, 0, SM_TIMEOUT, c->stream));   // mask, k0, unique count (reduce-by-key after us)
  if (!hist_ready) {   // mask + histograms of the hinted bytes, then the measured width
    GS_HIP(hipMemsetAsync(sm + SM_COUNTERS, 0, SM_BASE - SM_COUNTERS, c->stream));
    hipLaunchKernelGGL(k_keyinfo_buf, dim3(grid_for(n, 512, 2048)), dim3(256), 0, c->stream, keys, n, nd,
                       (unsigned long long*)(sm + SM_MASK), (uint32_t*)(sm + SM_HIST));
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(sm + SM_K0, keys, 8, hipMemcpyDeviceToDevice, c->stream));
    GS_HIP(hipMemcpyAsync(c->host_small, sm, 16, hipMemcpyDeviceToHost, c->stream));
    GS_TRY(host_wait(c));
    const uint64_t mask = c->host_small[0];
    k0 = c->host_small[1];
    bits = mask ? 64 - __builtin_clzll(mask) : 0;
    if (bits > 8 * nd) return set_error(c, GS_EDEVICE, "sort_buffer: keys wider than the %d-bit hint", bits_hint);
  }
  // (hist_ready: the producer of the keys filled SM_HIST for bits_hint-bit keys; no host round trip)
  out->bits = bits;
  out->wide = bits > 32;
  const bool d9 = digit_bits == 9;
  out->passes = std::max(1, (bits + (d9 ? 8 : RADIX_BITS - 1)) / (d9 ? 9 : RADIX_BITS));
  out->done_passes = out->passes;
  out->records = n;
  out->key_xor = (out->wide || hist_ready) ? 0 : (k0 & 0xFFFFFFFF00000000ull);
  if (d9) {   // the 9-bit digits' histograms: one more read of the keys
    GS_HIP(hipMemsetAsync(sm + SM_HIST9, 0, (size_t)out->passes * 512 * 4, c->stream));
    if (n)
      hipLaunchKernelGGL(k_hist_digits<9>, dim3(grid_for(n, 256 * 8, 2048)), dim3(256), 0, c->stream, keys, n, out->passes,
                         (uint32_t*)(sm + SM_HIST9));
    hipLaunchKernelGGL(k_digit_base_bits<9>, dim3(1), dim3(512), 0, c->stream, (const uint32_t*)(sm + SM_HIST9),
                       (uint32_t*)(sm + SM_BASE9), out->passes);
  } else {
    hipLaunchKernelGGL(k_digit_base, dim3(1), dim3(256), 0, c->stream, (const uint32_t*)(sm + SM_HIST),
                       (uint32_t*)(sm + SM_BASE), out->passes);
  }
  GS_HIP(hipGetLastError());
  const size_t kb = out->wide ? 8 : 4;
  const uint64_t tiles = (n + SORT_TILE - 1) / SORT_TILE;
  GS_TRY(ensure(c, c->keysA, n * kb));
  GS_TRY(ensure(c, c->keysB, n * kb));
  if (vals && val_bytes != 4 && val_bytes != 8) return set_error(c, GS_EINVAL, "sort_buffer: %d-byte payload", val_bytes);
  if (vals) {
    GS_TRY(ensure(c, c->valsA, n * val_bytes));
    GS_TRY(ensure(c, c->valsB, n * val_bytes));
  }
  GS_TRY(ensure(c, c->sort_status, tiles * (d9 ? 512 : RADIX) * 8, true));
  const auto* v4 = (const uint32_t*)vals;
  const auto* v8 = (const uint64_t*)vals;
  if (d9) {
    if (out->wide) {
      if (!vals) return buffer_passes<uint64_t, uint8_t, false, 9>(c, keys, nullptr, (uint32_t)n, out);
      return val_bytes == 8 ? buffer_passes<uint64_t, uint64_t, true, 9>(c, keys, v8, (uint32_t)n, out)
                            : buffer_passes<uint64_t, uint32_t, true, 9>(c, keys, v4, (uint32_t)n, out);
    }
    if (!vals) return buffer_passes<uint32_t, uint8_t, false, 9>(c, keys, nullptr, (uint32_t)n, out);
    return val_bytes == 8 ? buffer_passes<uint32_t, uint64_t, true, 9>(c, keys, v8, (uint32_t)n, out)
                          : buffer_passes<uint32_t, uint32_t, true, 9>(c, keys, v4, (uint32_t)n, out);
  }
  if (out->wide) {
    if (!vals) return buffer_passes<uint64_t, uint8_t, false>(c, keys, nullptr, (uint32_t)n, out);
    return val_bytes == 8 ? buffer_passes<uint64_t, uint64_t, true>(c, keys, v8, (uint32_t)n, out)
                          : buffer_passes<uint64_t, uint32_t, true>(c, keys, v4, (uint32_t)n, out);
  }
  if (!vals) return buffer_passes<uint32_t, uint8_t, false>(c, keys, nullptr, (uint32_t)n, out);
  return val_bytes == 8 ? buffer_passes<uint32_t, uint64_t, true>(c, keys, v8, (uint32_t)n, out)
                        : buffer_passes<uint32_t, uint32_t, true>(c, keys, v4, (uint32_t)n, out);
}

gs_status sort_window(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, int val_bytes,
                      uint64_t n_edges, int dir, int payload, Sorted* out, bool leave_last) {
  switch (dir) {
    case DIR_IN: return sort_dir<DIR_IN>(c, src, dst, val, val_bytes, n_edges, payload, out, leave_last);
    case DIR_OUT: return sort_dir<DIR_OUT>(c, src, dst, val, val_bytes, n_edges, payload, out, leave_last);
    case DIR_ALL: return sort_dir<DIR_ALL>(c, src, dst, val, val_bytes, n_edges, payload, out, leave_last);
  }
  return set_error(c, GS_EINVAL, "bad direction %d", dir);
}

namespace {
// ---- reduce / fold ---------------------------------------------------------------------------------
template <typename T, int OP>
static gs_status value_rbk(gs_ctx* c, const Sorted& s, int64_t* keys, void* vals, bool has_init, const void* init,
                           uint64_t* U) {
  using Op = ValueOp<T, OP>;
  ValueOut<Op, true> oi{keys, (T*)vals, has_init ? *(const T*)init : T{}};
  ValueOut<Op, false> on{keys, (T*)vals, T{}};
  if (s.wide) {
    if (has_init) return reduce_fused<uint64_t, Op>(c, s, oi, U);
    return reduce_fused<uint64_t, Op>(c, s, on, U);
  }
  if (has_init) return reduce_fused<uint32_t, Op>(c, s, oi, U);
  return reduce_fused<uint32_t, Op>(c, s, on, U);
}

template <typename T>
static gs_status value_rbk_op(gs_ctx* c, int op, const Sorted& s, int64_t* keys, void* vals, bool has_init,
                              const void* init, uint64_t* U) {
  switch (op) {
    case OP_SUM: return value_rbk<T, OP_SUM>(c, s, keys, vals, has_init, init, U);
    case OP_MIN: return value_rbk<T, OP_MIN>(c, s, keys, vals, has_init, init, U);
    case OP_MAX: return value_rbk<T, OP_MAX>(c, s, keys, vals, has_init, init, U);
  }
  return set_error(c, GS_EINVAL, "bad op %d", op);
}

}  // namespace

}  // namespace gs

// =================================================================================================
// C ABI
// =================================================================================================
extern "C" {

int32_t gs_abi_version(void) { return GS_ABI_VERSION; }

gs_status gs_device_count(int32_t* n) {
  if (!n) return GS_EINVAL;
  *n = 0;
  int d = 0;
  if (hipGetDeviceCount(&d) != hipSuccess) {
    (void)hipGetLastError();
    return GS_EDEVICE;
  }
  *n = d;
  return GS_OK;
}

gs_status gs_create(const gs_config* cfg, gs_ctx** out) {
  if (!out) return GS_EINVAL;
  *out = nullptr;
  gs_ctx* c = new (std::nothrow) gs_ctx();
  if (!c) return GS_ENOMEM;
  c->device = cfg ? cfg->device : 0;
  c->flags = cfg ? cfg->flags : 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= c->device) {
    delete c;
    return GS_EDEVICE;
  }
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return GS_EDEVICE;
  }
  c->own_stream = true;
  for (auto& e : c->ev) hipEventCreate(&e);
  for (auto& e : c->pass_ev) hipEventCreate(&e);
  if (hipHostMalloc((void**)&c->host_small, HOST_SMALL_WORDS * 8, hipHostMallocDefault) != hipSuccess ||
      ensure(c, c->small, SM_BYTES, true) != GS_OK) {
    gs_destroy(c);
    return GS_ENOMEM;
  }
  if (cfg && cfg->reserve_edges) {
    const uint64_t R = 2 * cfg->reserve_edges;
    if (ensure(c, c->keysA, R * 4) || ensure(c, c->keysB, R * 4) || ensure(c, c->valsA, R * 8) ||
        ensure(c, c->valsB, R * 8)) {
      gs_destroy(c);
      return GS_ENOMEM;
    }
  }
  hipStreamSynchronize(c->stream);
  *out = c;
  return GS_OK;
}

void gs_destroy(gs_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->comm) gs_comm_destroy(c);
  for (DevBuf& b : c->hs)
    if (b.p) hipFree(b.p);
  for (DevBuf* b : {&c->part_k, &c->part_a, &c->comp_k, &c->comp_a,
                    &c->in_src, &c->in_dst, &c->in_val, &c->keysA, &c->keysB, &c->valsA, &c->valsB, &c->sort_status,
                    &c->rbk_word, &c->rbk_agg, &c->rbk_inc, &c->small, &c->out_keys, &c->out_a, &c->out_b, &c->aux,
                    &c->bk_meta, &c->bk_items, &c->bk_slabs, &c->dp_cnt, &c->dp_csum, &c->dp_off, &c->tri_loops, &c->tri_tiles, &c->tri_sfx, &c->tri_nbr, &c->tri_heavy, &c->tri_range, &c->tri_queue, &c->tri_hwork, &c->tri_d[0], &c->tri_d[1], &c->tri_d[2], &c->tri_d[3], &c->tri_d[4], &c->tri_d[5], &c->tri_d[6], &c->tri_d[7], &c->tri_d[8], &c->tri_d[9], &c->cc[0], &c->cc[1], &c->cc[2], &c->cc[3],
                    &c->pr_a, &c->pr_b, &c->pr_f, &c->pr_key, &c->pr_val, &c->pr_gk, &c->pr_gv, &c->pr_small,
                    &c->tx_text, &c->tx_cnt, &c->tx_starts, &c->zipf_cdf,
                    &c->dist_k, &c->dist_v, &c->dist_v2, &c->dist_k2, &c->dist_v3, &c->dist_v4, &c->dist_cnt,
                    &c->dist_x, &c->dist_x2, &c->comm_scratch, &c->cand_bounds, &c->cand_steps, &c->hs_rank, &c->ck_k[0], &c->ck_k[1], &c->ck_a[0],
                    &c->ck_a[1], &c->ck_b[0], &c->ck_b[1], &c->sp[0].tot, &c->sp[1].tot, &c->sp_cur})
    if (b->p) hipFree(b->p);
  for (DevBuf& b : c->rl)
    if (b.p) hipFree(b.p);
  for (DevBuf& b : c->tri_bd)
    if (b.p) hipFree(b.p);
  for (DevBuf& b : c->tri_rl)
    if (b.p) hipFree(b.p);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  for (auto& e : c->pass_ev)
    if (e) hipEventDestroy(e);
  if (c->sync_ev) hipEventDestroy(c->sync_ev);
  if (c->host_small) hipHostFree(c->host_small);
  if (c->rb_host) hipHostFree(c->rb_host);
  if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
  delete c;
}

const char* gs_last_error(const gs_ctx* c) { return c ? c->err.c_str() : "null context"; }

gs_status gs_set_timing(gs_ctx* c, int32_t level) {
  if (!c) return GS_EINVAL;
  if (level < GS_TIMING_OFF || level > GS_TIMING_STAGES) return set_error(c, GS_EINVAL, "bad timing level %d", level);
  c->timing = level;
  return GS_OK;
}

gs_status gs_set_stream(gs_ctx* c, void* s) {
  if (!c) return GS_EINVAL;
  (void)hipGetLastError();
  GS_HIP(hipSetDevice(c->device));
  // the handle must be a live stream of this process's HIP runtime on the ctx's device (NULL = the
  // device's default stream); anything else fails here, not at the next window's first launch
  if (s) {
    const hipError_t q = hipStreamQuery((hipStream_t)s);
    if (q != hipSuccess && q != hipErrorNotReady) {
      (void)hipGetLastError();
      return set_error(c, GS_EDEVICE, "gs_set_stream: %p is not a HIP stream of this process: %s", s,
                       hipGetErrorString(q));
    }
    int dev = -1;
    if (hipStreamGetDevice((hipStream_t)s, &dev) == hipSuccess && dev != c->device)
      return set_error(c, GS_EINVAL, "gs_set_stream: stream %p belongs to device %d, the ctx to device %d", s, dev,
                       c->device);
    (void)hipGetLastError();
  }
  if (c->stream) GS_HIP(hipStreamSynchronize(c->stream));
  if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
  c->stream = (hipStream_t)s;
  c->own_stream = false;
  return GS_OK;
}

gs_status gs_synchronize(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  return hip_check(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
}

void* gs_alloc_pinned(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}
void gs_free_pinned(void* p) {
  if (p) hipHostFree(p);
}

gs_status gs_last_stage_times(const gs_ctx* c, gs_stage_times* out) {
  if (!c || !out) return GS_EINVAL;
  *out = c->times;
  return GS_OK;
}

static gs_status finish_vertex_out(gs_ctx* c, gs_vertex_out* out, const int64_t* kd, const void* vd, size_t ob,
                                   uint64_t U, bool direct) {
  *out->n_out = U;
  c->last_U = U;   // the staged rows gs_fetch_last_output can deliver after GS_ECAPACITY
  c->last_ob = ob;
  c->last_kind = direct ? 0 : 1;
  if (U > out->capacity) return set_error(c, GS_ECAPACITY, "output needs %llu vertices", (unsigned long long)U);
  GS_TRY(deliver(c, out->keys, kd, U * 8, out->mem));
  GS_TRY(deliver(c, out->vals, vd, U * ob, out->mem));
  if (!direct) GS_TRY(host_wait(c));
  return GS_OK;
}

// ---- windows above one pass's record cap (gs_set_max_window_records) ---------------------------------
// Edges per pass: max_records / (records per edge); for a host batch also what the free HBM holds (the
// staged columns plus the pass's workspace, ~64 B per record).  0 = the window runs in one pass.
static uint64_t chunk_edges(gs_ctx* c, const gs_edge_batch* b, int32_t dir) {
  if (c->in_chunk) return 0;
  const uint64_t per = dir == GS_DIR_ALL ? 2 : 1;
  uint64_t cap = c->max_records / per;
  if (b->mem == GS_MEM_HOST && b->n >= (1ull << 26)) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      const uint64_t per_edge = 16 + dtype_bytes(b->val_dtype) + 64 * per;
      cap = std::min<uint64_t>(cap, std::max<uint64_t>(1ull << 24, (uint64_t)(fr / 2) / per_edge));
    }
  }
  return b->n > cap ? std::max<uint64_t>(cap, 1) : 0;
}

// grow a device buffer keeping its first `keep` bytes
static gs_status grow_keep(gs_ctx* c, DevBuf& d, size_t bytes, size_t keep) {
  if (d.bytes >= bytes) return GS_OK;
  DevBuf n;
  GS_TRY(ensure(c, n, bytes));
  if (keep) GS_HIP(hipMemcpyAsync(n.p, d.p, keep, hipMemcpyDeviceToDevice, c->stream));
  GS_TRY(host_wait(c));
  if (d.p) GS_HIP(hipFree(d.p));
  d = n;
  return GS_OK;
}

// The window in chunks of `ce` whole edges: each chunk's per-vertex partials (op with no init; COUNT ->
// I64 counts; the degree fold -> degree + maximum) are appended after the running partials in one buffer,
// and the two merged (gs_merge_partials / gs_merge_degree_max_partials) into the other buffer; the last
// merge applies foldNeighbors' init and writes the caller's output.  Integer ops are associative and
// commutative, so the result is the one-pass window's bit for bit; float sums change order only.
static gs_status window_chunked(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, bool has_init,
                                const void* init, bool deg, int64_t init_max, gs_vertex_out* vout,
                                gs_degree_out* dout, uint64_t ce) {
  struct InChunk {
    gs_ctx* c;
    explicit InChunk(gs_ctx* x) : c(x) {
      c->in_chunk = true;
      c->oe.nparts = 0;   // the chunks' partials and merges emit ascending rows (gs_window_reduce_dist partitions them)
    }
    ~InChunk() { c->in_chunk = false; }
  } guard(c);
  const uint64_t per = dir == GS_DIR_ALL ? 2 : 1;
  const size_t vb = dtype_bytes(b->val_dtype);
  const size_t ob = (deg || op == GS_OP_COUNT) ? 8 : vb;
  const int32_t pdt = (deg || op == GS_OP_COUNT) ? GS_I64 : b->val_dtype;
  // a merge takes the running partials plus one chunk's: keep that under one pass's 2^32 - 1 rows by
  // shrinking the chunk as the distinct vertices accumulate (a window of more distinct vertices than
  // that cannot be merged in one pass: GS_EUNSUPPORTED)
  const uint64_t pass_rows = (1ull << 32) - 1;
  int x = 0;
  uint64_t acc = 0;   // running partials in ck_*[x][0, acc)
  for (uint64_t k = 0, e0 = 0; e0 < b->n; ++k) {
    if (acc + per > pass_rows)
      return set_error(c, GS_EUNSUPPORTED, "chunked window: %llu distinct vertices leave no room for a chunk",
                       (unsigned long long)acc);
    const uint64_t ne = std::min<uint64_t>({ce, b->n - e0, (pass_rows - acc) / per}), Rc = ne * per;
    gs_edge_batch cb = *b;
    cb.src = b->src + e0;
    cb.dst = b->dst + e0;
    if (b->val) cb.val = (const char*)b->val + e0 * vb;
    cb.n = ne;
    GS_TRY(grow_keep(c, c->ck_k[x], (acc + Rc) * 8 + 64, acc * 8));
    GS_TRY(grow_keep(c, c->ck_a[x], (acc + Rc) * ob + 64, acc * ob));
    if (deg) GS_TRY(grow_keep(c, c->ck_b[x], (acc + Rc) * 8 + 64, acc * 8));
    uint64_t Uc = 0;
    if (deg) {
      gs_degree_out po{c->ck_k[x].as<int64_t>() + acc, c->ck_a[x].as<int64_t>() + acc, c->ck_b[x].as<int64_t>() + acc,
                       Rc, &Uc, GS_MEM_DEVICE, 0};
      GS_TRY(gs_window_fold_degree_max(c, &cb, dir, INT64_MIN, &po));
    } else {
      gs_vertex_out po{c->ck_k[x].as<int64_t>() + acc, c->ck_a[x].as<char>() + acc * ob, Rc, &Uc, GS_MEM_DEVICE, 0};
      GS_TRY(gs_window_reduce(c, &cb, dir, op, &po));
    }
    const uint64_t n = acc + Uc;
    e0 += ne;
    const bool last = e0 == b->n;
    if (k == 0 && !last) {   // nothing to merge with yet
      acc = n;
      continue;
    }
    const gs_partial_batch pb{c->ck_k[x].as<int64_t>(), c->ck_a[x].p, deg ? c->ck_b[x].as<int64_t>() : nullptr, n, pdt,
                              GS_MEM_DEVICE};
    const int y = x ^ 1;
    if (last) {   // the caller's output, with the fold's init
      if (deg) return gs_merge_degree_max_partials(c, &pb, init_max, dout);
      return gs_merge_partials(c, &pb, op, has_init ? init : nullptr, vout);
    }
    GS_TRY(ensure(c, c->ck_k[y], n * 8 + 64));
    GS_TRY(ensure(c, c->ck_a[y], n * ob + 64));
    uint64_t Um = 0;
    if (deg) {
      GS_TRY(ensure(c, c->ck_b[y], n * 8 + 64));
      gs_degree_out mo{c->ck_k[y].as<int64_t>(), c->ck_a[y].as<int64_t>(), c->ck_b[y].as<int64_t>(), n, &Um,
                       GS_MEM_DEVICE, 0};
      GS_TRY(gs_merge_degree_max_partials(c, &pb, INT64_MIN, &mo));
    } else {
      gs_vertex_out mo{c->ck_k[y].as<int64_t>(), c->ck_a[y].p, n, &Um, GS_MEM_DEVICE, 0};
      GS_TRY(gs_merge_partials(c, &pb, op, nullptr, &mo));
    }
    x = y;
    acc = Um;
  }
  // one chunk only (not reached: chunk_edges returns 0 then)
  return set_error(c, GS_EINVAL, "chunked window: no chunks");
}

// GS_FLAG_ASYNC_OUTPUT for one window: the bucket path may leave its read-back to the emit kernel's first block
// (bucket_wait) when the outputs go straight to the caller's device buffers; cleared on every exit
struct RbAllow {
  gs_ctx* c;
  RbAllow(gs_ctx* c_, bool direct) : c(c_) {
    c->rb_allow = (c->flags & GS_FLAG_ASYNC_OUTPUT) && direct && c->timing != GS_TIMING_STAGES && !c->oe.nparts;
  }
  ~RbAllow() {
    c->rb_allow = false;
    c->rb_pending = false;
  }
};

static gs_status window_fold_impl(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, bool has_init,
                                  const void* init, gs_vertex_out* out) {
  GS_TRY(check_batch_any(c, b, dir));
  if (op < GS_OP_SUM || op > GS_OP_COUNT) return set_error(c, GS_EINVAL, "bad op %d", op);
  if (const uint64_t ce = chunk_edges(c, b, dir)) {
    if (!out || !out->n_out || (out->capacity && (!out->keys || !out->vals)))
      return set_error(c, GS_EINVAL, "bad gs_vertex_out");
    if (op != GS_OP_COUNT && (b->val_dtype == GS_NONE || (b->n && !b->val)))
      return set_error(c, GS_EINVAL, "op %d needs edge values", op);
    if (has_init && !init) return set_error(c, GS_EINVAL, "null init");
    return window_chunked(c, b, dir, op, has_init, init, false, 0, out, nullptr, ce);
  }
  GS_TRY(check_batch(c, b, dir));
  if (!out || !out->n_out || (out->capacity && (!out->keys || !out->vals)))
    return set_error(c, GS_EINVAL, "bad gs_vertex_out");
  if (op < GS_OP_SUM || op > GS_OP_COUNT) return set_error(c, GS_EINVAL, "bad op %d", op);
  if (op != GS_OP_COUNT && (b->val_dtype == GS_NONE || (b->n && !b->val)))
    return set_error(c, GS_EINVAL, "op %d needs edge values", op);
  if (has_init && !init) return set_error(c, GS_EINVAL, "null init");
  GS_TRY(begin_call(c));
  const uint64_t R = dir == GS_DIR_ALL ? 2 * b->n : b->n;
  if (R == 0) {
    *out->n_out = 0;
    return GS_OK;
  }
  stage_event(c, c->ev[0]);
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, op != GS_OP_COUNT));
  const int vbytes = (int)dtype_bytes(b->val_dtype);
  const size_t ob = op == GS_OP_COUNT ? 8 : (size_t)vbytes;
  const bool direct = out->mem == GS_MEM_DEVICE && out->capacity >= R;
  const RbAllow rb(c, direct);
  int64_t* kd = out->keys;
  void* vd = out->vals;
  if (!direct) {
    GS_TRY(ensure(c, c->out_keys, R * 8));
    GS_TRY(ensure(c, c->out_a, R * ob));
    kd = c->out_keys.as<int64_t>();
    vd = c->out_a.p;
  }
  uint64_t U = 0;
  const gs_status bs = bucket_reduce(c, src, dst, val, b->n, dir, op, b->val_dtype, has_init, init, kd, vd, &U);
  if (bs != GS_EUNSUPPORTED) {
    GS_TRY(bs);
    return finish_vertex_out(c, out, kd, vd, ob, U, direct);
  }
  c->oe.done = false;   // (an attempt that launched the owner-grouped emit, then gave up) the output is the sort path's
  Sorted s;
  GS_TRY(sort_window(c, src, dst, val, vbytes, b->n, dir, op == GS_OP_COUNT ? PAY_NONE : PAY_VAL, &s, true));
  s.fused = true;
  hipEventRecord(c->ev[2], c->stream);
  if (op == GS_OP_COUNT) {
    CountOut o{kd, (int64_t*)vd, has_init ? *(const int64_t*)init : 0};
    GS_TRY((s.wide ? reduce_fused<uint64_t, CountOp>(c, s, o, &U) : reduce_fused<uint32_t, CountOp>(c, s, o, &U)));
  } else {
    switch (b->val_dtype) {
      case GS_I32: GS_TRY(value_rbk_op<int32_t>(c, op, s, kd, vd, has_init, init, &U)); break;
      case GS_I64: GS_TRY(value_rbk_op<int64_t>(c, op, s, kd, vd, has_init, init, &U)); break;
      case GS_F32: GS_TRY(value_rbk_op<float>(c, op, s, kd, vd, has_init, init, &U)); break;
      case GS_F64: GS_TRY(value_rbk_op<double>(c, op, s, kd, vd, has_init, init, &U)); break;
    }
  }
  finish_times(c, s, U);
  return finish_vertex_out(c, out, kd, vd, ob, U, direct);
}

gs_status gs_fetch_last_output(gs_ctx* c, gs_vertex_out* out) {
  if (!c) return GS_EINVAL;
  if (c->last_kind != 1) return set_error(c, GS_EINVAL, "no staged (vertex, value) output to fetch");
  if (!out || !out->n_out || (c->last_U && (!out->keys || !out->vals))) return set_error(c, GS_EINVAL, "bad gs_vertex_out");
  *out->n_out = c->last_U;
  if (c->last_U > out->capacity) return set_error(c, GS_ECAPACITY, "output needs %llu vertices", (unsigned long long)c->last_U);
  GS_TRY(deliver(c, out->keys, c->out_keys.as<int64_t>(), c->last_U * 8, out->mem));
  GS_TRY(deliver(c, out->vals, c->out_a.p, c->last_U * c->last_ob, out->mem));
  return host_wait(c);
}

gs_status gs_fetch_last_degree_output(gs_ctx* c, gs_degree_out* out) {
  if (!c) return GS_EINVAL;
  if (c->last_kind != 2) return set_error(c, GS_EINVAL, "no staged degree / max output to fetch");
  if (!out || !out->n_out || (c->last_U && (!out->keys || !out->degree || !out->max_neighbor)))
    return set_error(c, GS_EINVAL, "bad gs_degree_out");
  *out->n_out = c->last_U;
  if (c->last_U > out->capacity) return set_error(c, GS_ECAPACITY, "output needs %llu vertices", (unsigned long long)c->last_U);
  GS_TRY(deliver(c, out->keys, c->out_keys.as<int64_t>(), c->last_U * 8, out->mem));
  GS_TRY(deliver(c, out->degree, c->out_a.p, c->last_U * 8, out->mem));
  GS_TRY(deliver(c, out->max_neighbor, c->out_b.p, c->last_U * 8, out->mem));
  return host_wait(c);
}

gs_status gs_window_reduce(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, gs_vertex_out* out) {
  return window_fold_impl(c, b, dir, op, false, nullptr, out);
}

gs_status gs_window_fold(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, const void* init,
                         gs_vertex_out* out) {
  return window_fold_impl(c, b, dir, op, true, init, out);
}

gs_status gs_set_max_window_records(gs_ctx* c, uint64_t max_records) {
  if (!c) return GS_EINVAL;
  const uint64_t lim = (1ull << 32) - 1;
  c->max_records = max_records == 0 || max_records > lim ? lim : std::max<uint64_t>(max_records, 2);
  return GS_OK;
}

gs_status gs_window_fold_degree_max(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int64_t init_max,
                                    gs_degree_out* out) {
  GS_TRY(check_batch_any(c, b, dir));
  if (!out || !out->n_out || (out->capacity && (!out->keys || !out->degree || !out->max_neighbor)))
    return set_error(c, GS_EINVAL, "bad gs_degree_out");
  if (const uint64_t ce = chunk_edges(c, b, dir)) return window_chunked(c, b, dir, 0, false, nullptr, true, init_max,
                                                                        nullptr, out, ce);
  GS_TRY(check_batch(c, b, dir));
  GS_TRY(begin_call(c));
  const uint64_t R = dir == GS_DIR_ALL ? 2 * b->n : b->n;
  if (R == 0) {
    *out->n_out = 0;
    return GS_OK;
  }
  stage_event(c, c->ev[0]);
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, false));
  const bool direct = out->mem == GS_MEM_DEVICE && out->capacity >= R;
  const RbAllow rb(c, direct);
  int64_t *kd = out->keys, *dd = out->degree, *md = out->max_neighbor;
  if (!direct) {
    GS_TRY(ensure(c, c->out_keys, R * 8));
    GS_TRY(ensure(c, c->out_a, R * 8));
    GS_TRY(ensure(c, c->out_b, R * 8));
    kd = c->out_keys.as<int64_t>();
    dd = c->out_a.as<int64_t>();
    md = c->out_b.as<int64_t>();
  }
  uint64_t U = 0;
  const gs_status bs = bucket_degree_max(c, src, dst, b->n, dir, init_max, kd, dd, md, &U);
  if (bs != GS_EUNSUPPORTED) {
    GS_TRY(bs);
  } else {
    c->oe.done = false;   // the output is the sort path's
    Sorted s;
    GS_TRY(sort_window(c, src, dst, nullptr, 0, b->n, dir, PAY_NBR, &s, true));
    s.fused = true;
    hipEventRecord(c->ev[2], c->stream);
    DegMaxOut o{kd, dd, md, init_max};
    GS_TRY((s.wide ? reduce_fused<uint64_t, DegMaxOp>(c, s, o, &U) : reduce_fused<uint32_t, DegMaxOp>(c, s, o, &U)));
    finish_times(c, s, U);
  }
  *out->n_out = U;
  c->last_U = U;
  c->last_ob = 8;
  c->last_kind = direct ? 0 : 2;
  if (U > out->capacity) return set_error(c, GS_ECAPACITY, "output needs %llu vertices", (unsigned long long)U);
  GS_TRY(deliver(c, out->keys, kd, U * 8, out->mem));
  GS_TRY(deliver(c, out->degree, dd, U * 8, out->mem));
  GS_TRY(deliver(c, out->max_neighbor, md, U * 8, out->mem));
  if (!direct) GS_TRY(host_wait(c));
  return GS_OK;
}

}  // extern "C"
