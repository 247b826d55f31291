// gs_bucket.hip — host side of the bucket path (gs_bucket.hpp) for reduceOnEdges / foldNeighbors
// with the associative built-ins (GraphWindowStream.java:62-87, 101-121).
//
// A window fits the path when its vertex range (max - min + 1) covers at most BK_MAXB buckets of
// 2^S vertices (S = 13..15 by accumulator size: 2^24..2^26 vertices) and the op has an LDS
// atomic: integer SUM / MIN / MAX, float SUM, COUNT, the degree / max-neighbour fold.  Anything
// else returns GS_EUNSUPPORTED and the caller sorts (gs_engine.hip).
//
// Two partition front ends feed the same LDS accumulation:
//   direct  (default, stage_times.path = 2): per-tile bucket histograms, an offset table and ONE
//           scatter pass (k_dp_*);
//   onesweep (GS_FLAG_BK_ONESWEEP, path = 1): 1-2 stable LSD passes of 4-6-bit digits over the
//           bucket index (k_onesweep with a global digit histogram), kept as the A/B baseline.
#include <algorithm>

#include "gs_ops.hpp"
#include <atomic>
#include <chrono>
// GS_TIMING_DOMINANT brackets the scatter and (1) the accumulate with dispatch-carried events; 0: the scatter
// only (the accumulate's time then comes from windows timed at GS_TIMING_STAGES)
#ifndef GS_DOM_ACCUM
#define GS_DOM_ACCUM 1
#endif

#include "gs_bucket.hpp"

namespace gs {

#ifndef GS_BK_ITEM_LOG
#define GS_BK_ITEM_LOG 17
#endif
#ifndef GS_BK_UNROLL
#define GS_BK_UNROLL 8
#endif
constexpr uint32_t BK_ITEM = 1u << GS_BK_ITEM_LOG;

namespace {

// internal: the window does not fit the compact (32-bit offset) policy; rerun with the wide one
constexpr gs_status GS_RETRY_WIDE = -100;

struct BkMeta {   // offsets (u32 units) inside ctx->bk_meta
  static constexpr size_t HIST = 0, DBASE = HIST + BK_MAXB, BSTART = DBASE + 512, BCOUNT = BSTART + BK_MAXB + 4,
                          BITEMS = BCOUNT + BK_MAXB, BSLAB = BITEMS + BK_MAXB, MLIST = BSLAB + BK_MAXB,
                          MAXIT = MLIST + BK_MAXB,   // the most items of one bucket (k_bk_merge_groups)
                          TOTAL = MAXIT + 4;
};

struct BkGeom {
  int64_t base = 0;
  uint32_t nb = 1;
  int passes = 0, w = 0;
};

int64_t key_min(const uint64_t* h) { return (int64_t)(~h[0] ^ (1ull << 63)); }
int64_t key_max(const uint64_t* h) { return (int64_t)(h[1] ^ (1ull << 63)); }

// base for the next window: 0 when the IDs are small non-negative numbers, else the window's minimum
int64_t predict_base(int64_t kmin, int64_t kmax, int S) {
  return (kmin >= 0 && ((uint64_t)kmax >> S) < (uint64_t)BK_MAXB) ? 0 : kmin;
}

template <int DIR>
gs_status launch_info(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, int64_t base, int S) {
  char* sm = c->small.as<char>();
  uint32_t* hist = c->bk_meta.as<uint32_t>() + BkMeta::HIST;
  GS_HIP(hipMemsetAsync(sm + SM_BK_MM, 0, 32, c->stream));
  GS_HIP(hipMemsetAsync(hist, 0, BK_MAXB * 4, c->stream));
  const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 4095) / 4096, 1024));
  if (vec)
    hipLaunchKernelGGL((k_bk_info<DIR, true>), dim3(grid), dim3(BK_INFO_BLOCK), 0, c->stream, src, dst, n, base, S,
                       (uint32_t)BK_MAXB, hist, (unsigned long long*)(sm + SM_BK_MM));
  else
    hipLaunchKernelGGL((k_bk_info<DIR, false>), dim3(grid), dim3(BK_INFO_BLOCK), 0, c->stream, src, dst, n, base, S,
                       (uint32_t)BK_MAXB, hist, (unsigned long long*)(sm + SM_BK_MM));
  return hip_check(c, hipGetLastError(), "k_bk_info");
}

template <int DIR, int ITEMS>
gs_status launch_dp_hist(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, uint32_t nt, int64_t base,
                         int S, uint32_t nbp) {
  char* sm = c->small.as<char>();
  auto* mm = (unsigned long long*)(sm + SM_BK_MM);
  GS_HIP(hipMemsetAsync(mm, 0, 32, c->stream));
  // VEC reads whole 16-byte pairs: every tile must hold one (only the last tile can be shorter)
  const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0 &&
                   n % dp_tile_edges<DIR, ITEMS>() != 1;
  const unsigned grid = std::max<uint32_t>(1, std::min<uint32_t>(nt, (uint32_t)c->n_cu));
  uint16_t* cnt = c->dp_cnt.as<uint16_t>();
  if (vec)
    hipLaunchKernelGGL((k_dp_hist<DIR, true, ITEMS>), dim3(grid), dim3(DP_BLOCK), 0, c->stream, src, dst, n, nt, base, S, nbp,
                       cnt, mm);
  else
    hipLaunchKernelGGL((k_dp_hist<DIR, false, ITEMS>), dim3(grid), dim3(DP_BLOCK), 0, c->stream, src, dst, n, nt, base, S,
                       nbp, cnt, mm);
  return hip_check(c, hipGetLastError(), "k_dp_hist");
}

// one partition pass: digit (key >> shift) & (2^DB - 1); K -> KO keys, payload V
template <int DB, typename K, typename KO, typename V, bool HAS_V, class Src>
gs_status launch_part(gs_ctx* c, Src src, KO* kout, V* vout, uint32_t R, int pass, uint32_t shift) {
  char* sm = c->small.as<char>();
  const uint32_t tiles = (R + SORT_TILE - 1) / SORT_TILE;
  const uint32_t ep = next_epoch(c, 0);
  GS_HIP(hipMemsetAsync((uint32_t*)(sm + SM_COUNTERS) + 48 + pass, 0, 4, c->stream));
  hipLaunchKernelGGL((k_onesweep<K, V, HAS_V, SORT_BLOCK, SORT_ITEMS, Src, DB, KO>), dim3(tiles), dim3(SORT_BLOCK), 0,
                     c->stream, src, kout, vout, R, shift,
                     (const uint32_t*)(c->bk_meta.as<uint32_t>() + BkMeta::DBASE) + pass * 256,
                     c->sort_status.as<uint64_t>(), (uint32_t*)(sm + SM_COUNTERS) + 48 + pass, ep,
                     (uint32_t*)(sm + SM_TIMEOUT));
  return hip_check(c, hipGetLastError(), "k_onesweep(bucket)");
}

template <typename K, typename KO, typename V, bool HAS_V, class Src>
gs_status launch_part_w(gs_ctx* c, int w, Src src, KO* kout, V* vout, uint32_t R, int pass, uint32_t shift) {
  switch (w) {
    case 4: return launch_part<4, K, KO, V, HAS_V>(c, src, kout, vout, R, pass, shift);
    case 5: return launch_part<5, K, KO, V, HAS_V>(c, src, kout, vout, R, pass, shift);
    case 6: return launch_part<6, K, KO, V, HAS_V>(c, src, kout, vout, R, pass, shift);
    case 8: return launch_part<8, K, KO, V, HAS_V>(c, src, kout, vout, R, pass, shift);
  }
  return set_error(c, GS_EINVAL, "bucket path: bad digit width %d", w);
}

void choose_passes(uint32_t nb, int* passes, int* w) {
  const int nbits = nb <= 1 ? 0 : 32 - __builtin_clz(nb - 1);
  if (nbits == 0) { *passes = 0; *w = 0; }
  else if (nbits <= 4) { *passes = 1; *w = 4; }
  else if (nbits <= 5) { *passes = 1; *w = 5; }
  else if (nbits <= 6) { *passes = 1; *w = 6; }
  else if (nbits <= 8) { *passes = 1; *w = 8; }
  else if (nbits <= 10) { *passes = 2; *w = 5; }
  else { *passes = 2; *w = 6; }
}

// records per accumulation work item: about GS_BK_ITEMS_PER_CU items per CU, at least 2^14 records
#ifndef GS_BK_ITEMS_PER_CU
#define GS_BK_ITEMS_PER_CU 3   // C2 (ms, one box): 4 items 1.712, 3 items 1.662 (fewer multi-item buckets: merge 0.066 -> 0.029), 2 items 1.685, 6 items 1.785
#endif
uint32_t item_records(gs_ctx* c, uint64_t R) {
  const uint64_t per = R / (GS_BK_ITEMS_PER_CU * (uint64_t)std::max(1, c->n_cu));
  return (uint32_t)std::max<uint64_t>(BK_ITEM, std::min<uint64_t>(per, 1u << 20));
}

gs_status ensure_cu(gs_ctx* c) {
  if (!c->n_cu) {
    int cu = 0;
    GS_HIP(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, c->device));
    c->n_cu = std::max(1, cu);
  }
  return GS_OK;
}

// k_bk_plan over meta[HIST] (bucket totals): bucket starts, work items, multi-item buckets
template <class P>
// R: records (or, with cursor, the regions' total capacity) -- sizes the item and slab buffers.
// cursor / counts_out: see BkPlanOut (speculative partition).
gs_status launch_plan(gs_ctx* c, uint64_t R, uint32_t nb, int passes, int w, uint32_t item_recs,
                      const uint32_t* cursor = nullptr, uint32_t* counts_out = nullptr,
                      unsigned long long* occupied = nullptr) {
  char* sm = c->small.as<char>();
  uint32_t* meta = c->bk_meta.as<uint32_t>();
  const uint64_t max_items = R / item_recs + nb + 1;
  const uint64_t max_slabs = 2 * (R / item_recs) + 2;
  GS_TRY(ensure(c, c->bk_items, max_items * sizeof(BkItem)));
  GS_TRY(ensure(c, c->bk_slabs, max_slabs * sizeof(typename P::Lds)));
  uint32_t* ns = (uint32_t*)(sm + SM_BK_N);
  BkPlanOut po{meta + BkMeta::DBASE, meta + BkMeta::BSTART, meta + BkMeta::BCOUNT, meta + BkMeta::BITEMS,
               meta + BkMeta::BSLAB, meta + BkMeta::MLIST, c->bk_items.as<BkItem>(), ns + 0, ns + 1,
               cursor, counts_out, occupied, ns + 2, meta + BkMeta::MAXIT};
  hipLaunchKernelGGL(k_bk_plan, dim3(1), dim3(BK_PLAN_BLOCK), 0, c->stream, meta + BkMeta::HIST, nb, passes, w,
                     item_recs, po);
  return hip_check(c, hipGetLastError(), "k_bk_plan");
}

// The back end both front ends share: LDS accumulation of the partitioned records (or of the
// columns themselves when the window is one bucket), merge of multi-item buckets, emit; then ONE
// read-back of the window's scalars (vertex range, outside-prediction count, U, items, escapes,
// timeout) into host_small[0..7].  The caller waits (host_wait) and interprets them.  Records
// pass_ev[ev0 + 1 .. ev0 + 3] after the three launches.  Every launch exits at once when the
// histogram saw a key outside the predicted range (mm[2] != 0).
template <class P, class Src>
gs_status bucket_accumulate(gs_ctx* c, Src rs, uint64_t R, uint32_t nb, int64_t base, typename P::Out o, int ev0,
                           const uint32_t* seg_cur = nullptr) {
  char* sm = c->small.as<char>();
  uint32_t* meta = c->bk_meta.as<uint32_t>();
  uint32_t* ns = (uint32_t*)(sm + SM_BK_N);
  const auto* mm = (const unsigned long long*)(sm + SM_BK_MM);
  BkStage st{c->keysA.as<uint32_t>(), c->valsA.p,
             (std::is_same_v<P, BkDeg> || std::is_same_v<P, BkDeg32>) ? c->aux.as<int64_t>() : nullptr};
  auto* slabs = c->bk_slabs.as<typename P::Lds>();
  // the direct path's accumulate (ev0 2) is a dominant kernel: its own start (pass_ev[7]) and stop events
  const bool dom = GS_DOM_ACCUM && ev0 == 2 && c->timing == GS_TIMING_DOMINANT;
  launch_dominant(c, dom ? c->pass_ev[7] : nullptr, dom ? c->pass_ev[ev0 + 1] : nullptr, k_bk_accum<P, Src, GS_BK_UNROLL>,
                  dim3(c->n_cu * GS_BK_ACC_PER_CU), dim3(BK_ACC_BLOCK), rs, (const BkItem*)c->bk_items.as<BkItem>(),
                  (const uint32_t*)(ns + 0), (const uint32_t*)(meta + BkMeta::BSTART), ns + 2, slabs, st,
                  meta + BkMeta::BCOUNT, mm, seg_cur);
  GS_HIP(hipGetLastError());
  stage_event(c, c->pass_ev[ev0 + 1]);
  // blocks loop over the multi-item buckets (their number stays on the device)
  const unsigned mgrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)nb, R / BK_ITEM + 1, 64}));
  const unsigned fgrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)nb, R / BK_ITEM + 1, (uint64_t)c->n_cu}));
  hipLaunchKernelGGL((k_bk_merge_groups<P>), dim3(2048), dim3(BK_MS_BLOCK), 0, c->stream, meta + BkMeta::MLIST, ns + 1,
                     meta + BkMeta::BITEMS, meta + BkMeta::BSLAB, slabs, mm, (const uint32_t*)(meta + BkMeta::MAXIT));
  hipLaunchKernelGGL((k_bk_merge_slices<P>), dim3(mgrid, BK_MS_SLICES), dim3(BK_MS_BLOCK), 0, c->stream,
                     meta + BkMeta::MLIST, ns + 1, meta + BkMeta::BITEMS, meta + BkMeta::BSLAB, slabs, mm);
  hipLaunchKernelGGL((k_bk_merge<P>), dim3(fgrid), dim3(BK_ACC_BLOCK), 0, c->stream, meta + BkMeta::MLIST, ns + 1,
                     meta + BkMeta::BITEMS, meta + BkMeta::BSLAB, meta + BkMeta::BSTART, slabs, st,
                     meta + BkMeta::BCOUNT, mm);
  GS_HIP(hipGetLastError());
  stage_event(c, c->pass_ev[ev0 + 2]);
  if (c->oe.nparts) {   // gs_window_reduce_dist: the exchange's rows instead of the ascending output
    const OwnerEmit& e = c->oe;
    hipLaunchKernelGGL(k_bk_owner_count, dim3(nb, BK_OE_SLICES), dim3(256), 0, c->stream, (const uint32_t*)(meta + BkMeta::BSTART),
                       (const uint32_t*)(meta + BkMeta::BCOUNT), nb, (const uint32_t*)st.k, base, e.nparts, e.cnt, e.wide,
                       mm, (const uint32_t*)(sm + SM_TIMEOUT), (const unsigned long long*)(sm + SM_BK_ESC),
                       (unsigned long long*)(sm + SM_BK_X));
    hipLaunchKernelGGL(k_owner_scan, dim3(1), dim3(1024), 0, c->stream, e.cnt, nb * BK_OE_SLICES * e.nparts,
                       nb * BK_OE_SLICES, e.nparts, e.totals,
                       (unsigned long long*)(sm + SM_BK_MM + 24));
    hipLaunchKernelGGL((k_bk_owner_emit<P>), dim3(nb, BK_OE_SLICES), dim3(256), 0, c->stream, (const uint32_t*)(meta + BkMeta::BSTART),
                       (const uint32_t*)(meta + BkMeta::BCOUNT), nb, st, base, o, e.nparts, (const uint32_t*)e.cnt, e.rows,
                       (const unsigned long long*)e.wide, e.vw, e.mw, mm);
    // the counts exchange's send rows too, before the read-back: after its wait the caller goes straight
    // to the collective
    hipLaunchKernelGGL(k_send_rows, dim3(1), dim3(64), 0, c->stream, (const unsigned long long*)e.totals, e.wide,
                       e.nparts, e.send, mm, (const uint32_t*)(sm + SM_TIMEOUT));
    c->oe.done = true;
  } else {
    // GS_FLAG_ASYNC_OUTPUT (the entry point allowed it for this window): the emit's first block writes the
    // read-back block into pinned host memory and bucket_wait spins on it -- the host does not wait for the
    // emit (its outputs are complete in stream order), and there is no copy launch
    const bool early = c->rb_allow && !c->in_chunk;
    if (early && !c->rb_host) {
      if (hipHostMalloc((void**)&c->rb_host, 128, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
          hipHostGetDevicePointer((void**)&c->rb_dev, c->rb_host, 0) != hipSuccess)
        return set_error(c, GS_ENOMEM, "pinned read-back block");
      c->rb_host[8] = 0;
    }
    const uint64_t seq = early ? ++c->rb_seq : 0;
    hipLaunchKernelGGL((k_bk_emit<P>), dim3(nb), dim3(256), 0, c->stream, meta + BkMeta::BSTART, meta + BkMeta::BCOUNT,
                       nb, st, base, o, (unsigned long long*)(sm + SM_BK_MM + 24), mm, (const uint32_t*)(sm + SM_TIMEOUT),
                       (const unsigned long long*)(sm + SM_BK_ESC), (unsigned long long*)(sm + SM_BK_X),
                       early ? (unsigned long long*)c->rb_dev : nullptr, seq);
    if (early) {
      GS_HIP(hipGetLastError());
      c->rb_pending = true;
      return GS_OK;
    }
  }
  GS_HIP(hipGetLastError());
  stage_event(c, c->pass_ev[ev0 + 3]);
  stage_event(c, c->ev[3]);
  static_assert(SM_BK_N == SM_BK_MM + 32 && SM_BK_X == SM_BK_MM + 48, "one read-back block");
  GS_HIP(hipMemcpyAsync(c->host_small, sm + SM_BK_MM, 64, hipMemcpyDeviceToHost, c->stream));
  return GS_OK;
}

gs_status bucket_wait(gs_ctx* c) {
  if (!c->rb_pending) return host_wait(c);
  c->rb_pending = false;
  volatile uint64_t* h = c->rb_host;
  const uint64_t seq = c->rb_seq;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0; h[8] != seq; ++spin) {
    // every 4096 polls: past 2 ms of spinning, wait for the stream instead (a long window, or a fault: its
    // error surfaces there); the block must then be there
    if ((spin & 4095) == 4095 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
      GS_TRY(hip_check(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize"));
      if (h[8] != seq) return set_error(c, GS_EDEVICE, "bucket path: the read-back block never arrived");
      break;
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  for (int i = 0; i < 8; ++i) c->host_small[i] = h[i];
  return GS_OK;
}

// after host_wait: the accumulate's results (GS_EDEVICE on a look-back timeout)
gs_status bucket_results(gs_ctx* c, uint64_t* U, uint32_t* n_items) {
  if ((uint32_t)c->host_small[6] != 0) return set_error(c, GS_EDEVICE, "look-back spin timed out");
  c->timeout_clean = true;   // read back as zero at the end of this window (begin_call skips its clear)
  *U = c->host_small[3];
  *n_items = (uint32_t)c->host_small[4];
  return GS_OK;
}

void bucket_times(gs_ctx* c, int path, int passes, int launches, uint32_t key_bits, uint64_t R, uint64_t U,
                  size_t vb, uint32_t n_items) {
  // only the events this timing level recorded are read (each hipEventElapsedTime is a driver call on the
  // window's critical path: the host turnaround between two windows)
  const bool all = c->timing == GS_TIMING_STAGES;
  float a = 0, b = 0, d = 0;
  if (all) {
    a = event_ms(c->ev[0], c->ev[1]);
    b = event_ms(c->ev[1], c->ev[2]);
    d = event_ms(c->ev[2], c->ev[3]);
  }
  gs_stage_times& t = c->times;
  t = gs_stage_times{};
  t.keyinfo_ms = a;
  t.sort_ms = b;
  t.reduce_ms = d;
  t.total_ms = a + b + d;
  t.sort_passes = (uint32_t)passes;
  t.key_bits = key_bits;
  t.records = R;
  t.vertices = U;
  if (all)
    for (int p = 0; p < launches && p < 8; ++p) t.pass_ms[p] = event_ms(c->pass_ev[p], c->pass_ev[p + 1]);
  t.key_bytes = 2;
  t.payload_bytes = (uint32_t)vb;
  t.partials = n_items;
  t.fused_last = 0;
  t.path = (uint32_t)path;
  if (!all) {   // only the events stage_event recorded at this level
    if (c->timing == GS_TIMING_DOMINANT && path == 2) {   // the scatter and the accumulate (launch_dominant)
      if (passes) t.pass_ms[1] = event_ms(c->pass_ev[1], c->pass_ev[2]);
      if (GS_DOM_ACCUM) t.pass_ms[2] = event_ms(c->pass_ev[7], c->pass_ev[3]);
    }
  }
}

template <class P>
gs_status ensure_stage(gs_ctx* c, uint64_t R) {
  constexpr size_t vb = P::HAS_V ? sizeof(typename P::Raw) : 0;
  constexpr size_t ab = std::max(sizeof(typename P::A), vb);
  GS_TRY(ensure(c, c->keysA, R * 4));
  GS_TRY(ensure(c, c->keysB, R * 4));
  GS_TRY(ensure(c, c->valsA, R * std::max<size_t>(ab, 4)));
  if (P::HAS_V) GS_TRY(ensure(c, c->valsB, R * vb));
  if (std::is_same_v<P, BkDeg> || std::is_same_v<P, BkDeg32>) GS_TRY(ensure(c, c->aux, R * 8));
  return GS_OK;
}

// ---- direct front end: hist -> offsets -> one scatter -------------------------------------------------
// The whole window is enqueued against the PREDICTED vertex range (the previous window's base and
// bucket count; the first window of a ctx assumes small non-negative IDs and BK_MAXB buckets) with
// no host round trip inside it: k_dp_hist counts the keys outside the prediction and every later
// launch exits at once when there are any.  One read-back at the end brings the measured range,
// that count, U and the escape count; only a missed prediction reruns the window (with the measured
// range, which cannot miss).
// Integer SUM / MIN / MAX partition through k_dp_scatter_pack (4-byte records) unless the previous
// window of this ctx had more than 1/8 escapes; every other op through k_dp_scatter.
// Events: ev[1] / pass_ev[0] after the histogram; pass_ev[0..2] around the offset scans and the
// scatter; then accumulate / merge / emit.
template <class P, int DIR, int ITEMS>
gs_status bucket_direct_t(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, uint64_t n,
                          typename P::Out o, uint64_t* U, bool pack) {
  using Raw = typename P::Raw;
  constexpr int S = P::S;
  constexpr bool CAN_PACK = P::PAY == PAY_VAL && !P::REL && std::is_integral_v<typename P::A>;
  char* sm = c->small.as<char>();
  const uint64_t R = (DIR == DIR_ALL) ? 2 * n : n;
  GS_TRY(ensure(c, c->bk_meta, BkMeta::TOTAL * 4, true));
  GS_TRY(ensure_cu(c));
  uint32_t* meta = c->bk_meta.as<uint32_t>();
  constexpr uint32_t TE = dp_tile_edges<DIR, ITEMS>();
  const uint32_t nt = (uint32_t)((n + TE - 1) / TE);
  const uint32_t nch = (nt + DP_CHUNK - 1) / DP_CHUNK;
  GS_TRY(ensure(c, c->dp_cnt, (size_t)nt * BK_MAXB * 2));
  GS_TRY(ensure(c, c->dp_csum, (size_t)nch * BK_MAXB * 4));
  GS_TRY(ensure(c, c->dp_off, (size_t)nt * BK_MAXB * 4));
  GS_TRY(ensure_stage<P>(c, R));
  int64_t base = c->bk_base;
  uint32_t nb = c->bk_nbp ? c->bk_nbp : (uint32_t)BK_MAXB;
  const uint32_t item_recs = item_records(c, R);
  // speculative partition: windows whose bucket counts the previous bucket-path window of this ctx
  // measured in the same geometry (base, S, direction); packed records through k_sp_scatter_pack, the
  // others through k_sp_scatter
  constexpr bool SPEC_OK = (CAN_PACK && ITEMS == PK_ITEMS) || ITEMS == DP_ITEMS;
  bool spec = false, spec_missed = false;
  uint64_t cap = R;
  // the speculative scatter's tile: k_sp_scatter_pack (SPK_BLOCK x SPK_ITEMS) or k_sp_scatter (DP_TILE)
  const uint64_t TRASH = std::max<uint64_t>(SPK_TILE, SPU_TILE);
  const uint64_t SPTE = !pack ? spu_tile_edges<DIR>() : spk_tile_edges<DIR>();
  auto& sp = c->sp[c->sp_slot];
  if constexpr (SPEC_OK) {
    GS_TRY(ensure(c, sp.tot, BK_MAXB * 4, true));
    GS_TRY(ensure(c, c->sp_cur, SP_CUR_WORDS * 4));
    // merges (slot 1) speculate with ONE segment per bucket: their rows are sender runs sorted by
    // vertex, so a tile holds few buckets and a bucket's records come from the tiles of one XCD slot
    // -- proportional per-slot segments would overflow.  A tile reserves one run per bucket it
    // touches (a handful), so the single cursor sees few atomics.
    spec = !(c->flags & GS_FLAG_NO_SPEC) && sp.ok && sp.skip == 0 && sp.base == base && sp.S == S &&
           sp.dir == DIR && nb > 1 && sp_capacity(R, nb) + TRASH < (1ull << 32);   // u32 positions + trash
    if (sp.skip > 0) --sp.skip;
    if (spec) {
      cap = sp_capacity(R, nb);
      GS_TRY(ensure_stage<P>(c, cap + TRASH));   // + the trash area of dropped runs
    }
  }
  uint16_t* cnt = c->dp_cnt.as<uint16_t>();
  uint32_t* csum = c->dp_csum.as<uint32_t>();
  uint16_t* k16 = c->keysB.as<uint16_t>();
  Raw* vpart = P::HAS_V ? c->valsB.as<Raw>() : nullptr;
  uint32_t* rel_bad = (uint32_t*)(sm + SM_BK_N) + 3;
  auto* mm = (unsigned long long*)(sm + SM_BK_MM);
  bool part = false;
  int64_t kmin = 0, kmax = 0;
  for (int attempt = 0;; ++attempt) {
    if constexpr (SPEC_OK) {
      // gs_window_reduce_dist's deferred window (OwnerEmit::defer; not the 32-bit-neighbour policies, whose
      // read-back can still ask for the wide one): the launches return at once, the resumed call skips them
      const bool defer = !P::REL && c->oe.nparts && c->oe.defer;
      if (spec && attempt == 0 && defer && c->oe.resume) {
        c->oe.resume = false;
        if (!c->host_small[2]) {   // hit
          kmin = (int64_t)((uint64_t)base + (c->host_small[0] << S));
          kmax = (int64_t)((uint64_t)base + (c->host_small[1] << S) + ((1ull << S) - 1));
          part = true;
          break;
        }
        sp.skip = 8;
        spec = false;
        spec_missed = true;
        continue;
      }
      if (spec && attempt == 0) {
        // regions from the previous window's counts -> the scatter reserves runs with atomics ->
        // items from the cursors (the counts the next window predicts from) -> accumulate
        // each XCD slot's share of the records (k_sp_scatter_pack: slot x owns full tiles [x·per, (x+1)·per),
        // the partial last tile runs in slot 0)
        SpSlots slots{};
        const uint32_t xmask = c->sp_slot == 0 ? 7u : 0u;
        if (!xmask) {   // segment 0 = the whole region
          for (uint32_t x = 1; x <= SP_NSEG; ++x) slots.pre[x] = (uint32_t)R;
        } else {
          const uint64_t tr = (DIR == DIR_ALL ? 2 : 1) * SPTE, nfull = n / SPTE, per = (nfull + 7) / 8;
          uint64_t acc = 0;
          for (uint32_t x = 0; x < SP_NSEG; ++x) {
            slots.pre[x] = (uint32_t)acc;
            const uint64_t lo = std::min<uint64_t>(nfull, SP_NSEG == 1 ? 0 : x * per);
            const uint64_t hi = SP_NSEG == 1 ? nfull : std::min<uint64_t>(nfull, (x + 1) * per);
            acc += (hi - lo) * tr + (x == 0 ? R - nfull * tr : 0);
          }
          slots.pre[SP_NSEG] = (uint32_t)acc;   // == R
        }
        hipLaunchKernelGGL(k_sp_regions, dim3(1), dim3(BK_PLAN_BLOCK), 0, c->stream, (const uint32_t*)sp.tot.as<uint32_t>(),
                           nb, sp.R, R, meta + BkMeta::BSTART, c->sp_cur.as<uint32_t>(), slots, mm,
                           (unsigned long long*)(sm + SM_BK_ESC));
        if constexpr (P::REL) GS_HIP(hipMemsetAsync(rel_bad, 0, 4, c->stream));
        stage_event(c, c->ev[1]);
        stage_event(c, c->pass_ev[0]);
        stage_event(c, c->pass_ev[1]);
        using Load = typename P::Load;
        const BaseSrc<Load, DIR, P::PAY> ls{src, dst, (const Load*)val, base};
        uint32_t* cur = c->sp_cur.as<uint32_t>();
        hipEvent_t e0 = c->pass_ev[1], e1 = c->pass_ev[2];
        uint32_t* kp = c->keysB.as<uint32_t>();
        auto* esc = (unsigned long long*)(sm + SM_BK_ESC);
        const uint32_t trash = (uint32_t)cap;
        if constexpr (CAN_PACK && ITEMS == PK_ITEMS) {
          // the bucket tables sized for the window's buckets (1024: 8 KiB less LDS, one bucket per thread)
          if (pack && nb <= 1024)
            launch_dominant(c, e0, e1, k_sp_scatter_pack<Load, DIR, 1024>, dim3(spk_grid<DIR>(n)), dim3(SPK_BLOCK), ls, n,
                            S, nb, cur, kp, vpart, trash, mm, esc, xmask);
          else if (pack)
            launch_dominant(c, e0, e1, k_sp_scatter_pack<Load, DIR, BK_MAXB>, dim3(spk_grid<DIR>(n)), dim3(SPK_BLOCK), ls,
                            n, S, nb, cur, kp, vpart, trash, mm, esc, xmask);
        }
        if constexpr (ITEMS == DP_ITEMS) {
          if (!pack) {
            if (nb <= 1024)
              launch_dominant(c, e0, e1, k_sp_scatter<Load, DIR, P::PAY, Raw, P::REL, 1024>, dim3(spu_grid<DIR>(n)),
                              dim3(SPU_BLOCK), ls, n, S, nb, cur, k16, vpart, trash, rel_bad, mm, xmask);
            else
              launch_dominant(c, e0, e1, k_sp_scatter<Load, DIR, P::PAY, Raw, P::REL, BK_MAXB>, dim3(spu_grid<DIR>(n)),
                              dim3(SPU_BLOCK), ls, n, S, nb, cur, k16, vpart, trash, rel_bad, mm, xmask);
          }
        }
        GS_HIP(hipGetLastError());
        stage_event(c, c->pass_ev[2]);
        stage_event(c, c->ev[2]);
        GS_TRY(launch_plan<P>(c, cap, nb, 0, 0, item_recs, cur, sp.tot.as<uint32_t>(), mm));
        part = true;
        if (pack) GS_TRY((bucket_accumulate<P>(c, PackSrc<Raw>{c->keysB.as<uint32_t>(), vpart}, cap, nb, base, o, 2, cur)));
        else GS_TRY((bucket_accumulate<P>(c, PartSrc<Raw>{k16, vpart}, cap, nb, base, o, 2, cur)));
        if (defer) return GS_PENDING_LOCAL;
        GS_TRY(bucket_wait(c));
        if (!c->host_small[2]) {   // hit: every key in the range; the plan reported the occupied buckets
          kmin = (int64_t)((uint64_t)base + (c->host_small[0] << S));
          kmax = (int64_t)((uint64_t)base + (c->host_small[1] << S) + ((1ull << S) - 1));
          break;
        }
        // missed (a run past its segment, or a key outside the range): rerun through the histogram,
        // which measures the range (and reruns once more if the prediction missed it); the next 8
        // windows do not speculate
        sp.skip = 8;
        spec = false;
        spec_missed = true;
        continue;
      }
    }
    // 1. per-tile bucket counts against the predicted base and width (the window's one read of
    //    the keys before the scatter) + the measured range and the keys outside the prediction
    GS_TRY((launch_dp_hist<DIR, ITEMS>(c, src, dst, n, nt, base, S, nb)));
    GS_HIP(hipMemsetAsync(sm + SM_BK_ESC, 0, 8, c->stream));
    stage_event(c, c->ev[1]);
    stage_event(c, c->pass_ev[0]);

    // 2. offsets: chunk counts, per-bucket spine (-> meta[HIST] totals), plan, per-tile offsets
    part = nb > 1;
    const dim3 g2((nb + 255) / 256, nch);
    hipLaunchKernelGGL(k_dp_up, g2, dim3(256), 0, c->stream, cnt, nt, nb, csum);
    hipLaunchKernelGGL(k_dp_spine, dim3((nb + 63) / 64), dim3(1024), 0, c->stream, csum, nch, nb, meta + BkMeta::HIST);
    GS_HIP(hipGetLastError());
    GS_TRY(launch_plan<P>(c, R, nb, 0, 0, item_recs, nullptr, SPEC_OK ? sp.tot.as<uint32_t>() : nullptr));
    if (part) {
      hipLaunchKernelGGL(k_dp_down, g2, dim3(256), 0, c->stream, cnt, csum, meta + BkMeta::BSTART, nt, nb,
                         c->dp_off.as<uint32_t>());
      GS_HIP(hipGetLastError());
    }
    stage_event(c, c->pass_ev[1], !part);   // (a partitioned window's scatter carries its own events)

    // 3. the scatter: bucket-local index + payload in bucket order
    if constexpr (P::REL) {
      if (!part) return GS_RETRY_WIDE;   // offsets are checked by the scatter only
    }
    using Load = typename P::Load;
    const BaseSrc<Load, DIR, P::PAY> ls{src, dst, (const Load*)val, base};
    if (part) {
      const unsigned grid = dp_scatter_grid<DIR, ITEMS>(n);
      const uint32_t* off = c->dp_off.as<uint32_t>();
      const auto* mmc = (const unsigned long long*)mm;
      if constexpr (CAN_PACK) {
        if (pack) {
          launch_dominant(c, c->pass_ev[1], c->pass_ev[2], k_dp_scatter_pack<Load, DIR, ITEMS>, dim3(grid), dim3(DP_BLOCK),
                          ls, n, S, nb, off, c->keysB.as<uint32_t>(), vpart, mmc, (unsigned long long*)(sm + SM_BK_ESC));
          GS_HIP(hipGetLastError());
        }
      }
      if constexpr (ITEMS == DP_ITEMS) if (!pack) {
        if constexpr (P::REL) GS_HIP(hipMemsetAsync(rel_bad, 0, 4, c->stream));
        launch_dominant(c, c->pass_ev[1], c->pass_ev[2], k_dp_scatter<Load, DIR, P::PAY, Raw, P::REL>, dim3(grid),
                        dim3(DP_BLOCK), ls, n, S, nb, c->dp_off.as<uint32_t>(), k16, vpart, rel_bad, mmc);
        GS_HIP(hipGetLastError());
      }
    }
    stage_event(c, c->pass_ev[2], !part);
    stage_event(c, c->ev[2]);

    // 4-6. accumulate, merge, emit; one read-back
    if (part) {
      if (pack) GS_TRY((bucket_accumulate<P>(c, PackSrc<Raw>{c->keysB.as<uint32_t>(), vpart}, R, nb, base, o, 2)));
      else GS_TRY((bucket_accumulate<P>(c, PartSrc<Raw>{k16, vpart}, R, nb, base, o, 2)));
    } else if constexpr (!P::REL) {
      const BaseSrc<Raw, DIR, P::PAY> es{src, dst, (const Raw*)val, base};
      GS_TRY((bucket_accumulate<P>(c, es, R, nb, base, o, 2)));
    }
    GS_TRY(bucket_wait(c));
    kmin = key_min(c->host_small);
    kmax = key_max(c->host_small);
    if ((((uint64_t)kmax - (uint64_t)kmin) >> S) >= (uint64_t)BK_MAXB) return GS_EUNSUPPORTED;
    if (!c->host_small[2]) break;
    if (attempt > (spec_missed ? 1 : 0))
      return set_error(c, GS_EDEVICE, "bucket path: keys outside the measured vertex range");
    base = predict_base(kmin, kmax, S);   // missed prediction: rerun with the measured range
    nb = (uint32_t)((((uint64_t)kmax - (uint64_t)base) >> S) + 1);
  }
  {   // the next window predicts this base and this width rounded up to a power of two
    const uint32_t need = (uint32_t)((((uint64_t)kmax - (uint64_t)base) >> S) + 1);
    uint32_t p2 = 1;
    while (p2 < need) p2 <<= 1;
    c->bk_base = base;
    c->bk_nbp = std::min<uint32_t>(p2, BK_MAXB);
  }
  uint32_t n_items = 0;
  GS_TRY(bucket_results(c, U, &n_items));
  if constexpr (P::REL) {
    if ((uint32_t)(c->host_small[5] >> 32) != 0) return GS_RETRY_WIDE;   // a neighbour outside base + 2^32
  }
  if constexpr (CAN_PACK) {
    // escapes common (> 1/8 of the records): the next 16 windows store 8-byte values, then packing
    // is tried again
    int& wide = c->bk_wide_vals[c->sp_slot];
    if (pack && c->host_small[7] > R / 8) wide = 16;
    else if (!pack && wide > 0) --wide;
  }
  const uint64_t esc = pack ? c->host_small[7] : 0;
  const uint32_t key_bits = nb <= 1 ? (uint32_t)S : (uint32_t)(S + 32 - __builtin_clz(nb - 1));
  const size_t pb = pack ? 2 : (P::HAS_V ? sizeof(Raw) : 0);   // packed: 2 key + 2 value bytes per record
  bucket_times(c, 2, part ? 1 : 0, 5, key_bits, R, *U, pb, n_items);
  c->times.key_bytes = 2;
  c->times.escapes = esc;
  c->times.packed = pack ? 1u : 0u;
  c->times.speculative = spec ? 1u : spec_missed ? 2u : 0u;
  if constexpr (SPEC_OK) {   // the counts plan wrote to sp_tot are this geometry's
    if (part) {
      sp.ok = true;
      sp.base = base;
      sp.S = S;
      sp.dir = DIR;
      sp.R = R;
    }
  }
  return GS_OK;
}

template <class P, int DIR>
gs_status bucket_direct(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, uint64_t n,
                        typename P::Out o, uint64_t* U) {
  constexpr bool CAN_PACK = P::PAY == PAY_VAL && !P::REL && std::is_integral_v<typename P::A>;
  if constexpr (CAN_PACK) {
    if (c->bk_wide_vals[c->sp_slot] <= 0 && !(c->flags & GS_FLAG_NO_PACK))
      return bucket_direct_t<P, DIR, PK_ITEMS>(c, src, dst, val, n, o, U, true);
  }
  return bucket_direct_t<P, DIR, DP_ITEMS>(c, src, dst, val, n, o, U, false);
}

// ---- onesweep front end (GS_FLAG_BK_ONESWEEP): global histogram -> 1-2 stable LSD passes ----------
template <class P, int DIR>
gs_status bucket_onesweep(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, uint64_t n,
                          typename P::Out o, uint64_t* U) {
  using Raw = typename P::Raw;
  constexpr bool HAS_V = P::HAS_V;
  constexpr int S = P::S;
  char* sm = c->small.as<char>();
  const uint64_t R = (DIR == DIR_ALL) ? 2 * n : n;
  GS_TRY(ensure(c, c->bk_meta, BkMeta::TOTAL * 4, true));
  GS_TRY(ensure_cu(c));

  // 1. vertex range + bucket histogram against the predicted base
  int64_t base = c->bk_base;
  GS_TRY(launch_info<DIR>(c, src, dst, n, base, S));
  GS_HIP(hipMemcpyAsync(c->host_small, sm + SM_BK_MM, 24, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const int64_t kmin = key_min(c->host_small), kmax = key_max(c->host_small);
  if ((((uint64_t)kmax - (uint64_t)kmin) >> S) >= (uint64_t)BK_MAXB) return GS_EUNSUPPORTED;
  if (c->host_small[2]) {
    base = kmin;
    GS_TRY(launch_info<DIR>(c, src, dst, n, base, S));
  }
  c->bk_base = predict_base(kmin, kmax, S);
  BkGeom g;
  g.base = base;
  g.nb = (uint32_t)((((uint64_t)kmax - (uint64_t)base) >> S) + 1);
  choose_passes(g.nb, &g.passes, &g.w);

  // 2. plan
  const uint32_t item_recs = item_records(c, R);
  GS_TRY(launch_plan<P>(c, R, g.nb, g.passes, g.w, item_recs));
  stage_event(c, c->ev[1]);
  stage_event(c, c->pass_ev[0]);

  // 3. partition passes over the bucket index; the last stores the 16-bit bucket-local index
  GS_TRY(ensure_stage<P>(c, R));
  const uint32_t tiles = (uint32_t)((R + SORT_TILE - 1) / SORT_TILE);
  GS_TRY(ensure(c, c->sort_status, (size_t)tiles * 256 * 8, true));
  using ESrc = BaseSrc<Raw, DIR, P::PAY>;
  const ESrc es{src, dst, (const Raw*)val, base};
  uint16_t* k16 = c->keysB.as<uint16_t>();
  Raw* vpart = HAS_V ? c->valsB.as<Raw>() : nullptr;
  if (g.passes == 1) {
    GS_TRY((launch_part_w<uint32_t, uint16_t, Raw, HAS_V>(c, g.w, es, k16, vpart, (uint32_t)R, 0, S)));
    stage_event(c, c->pass_ev[1]);
  } else if (g.passes == 2) {
    uint32_t* k32 = c->keysA.as<uint32_t>();
    Raw* vmid = HAS_V ? c->valsA.as<Raw>() : nullptr;
    GS_TRY((launch_part_w<uint32_t, uint32_t, Raw, HAS_V>(c, g.w, es, k32, vmid, (uint32_t)R, 0, S)));
    stage_event(c, c->pass_ev[1]);
    const BufSrc<uint32_t, Raw> bs{k32, vmid, 0};
    GS_TRY((launch_part_w<uint32_t, uint16_t, Raw, HAS_V>(c, g.w, bs, k16, vpart, (uint32_t)R, 1, S + g.w)));
    stage_event(c, c->pass_ev[2]);
  }
  stage_event(c, c->ev[2]);

  // 4-6. accumulate, merge, emit
  uint32_t n_items = 0;
  if (g.passes == 0)
    GS_TRY((bucket_accumulate<P>(c, es, R, g.nb, base, o, g.passes)));
  else
    GS_TRY((bucket_accumulate<P>(c, PartSrc<Raw>{k16, vpart}, R, g.nb, base, o, g.passes)));
  GS_TRY(bucket_wait(c));
  GS_TRY(bucket_results(c, U, &n_items));
  const uint32_t key_bits = g.nb <= 1 ? (uint32_t)S : (uint32_t)(S + 32 - __builtin_clz(g.nb - 1));
  bucket_times(c, 1, g.passes, g.passes + 3, key_bits, R, *U, HAS_V ? sizeof(Raw) : 0, n_items);
  return GS_OK;
}

template <class P>
gs_status bucket_dir(gs_ctx* c, int dir, const int64_t* src, const int64_t* dst, const void* val, uint64_t n,
                     typename P::Out o, uint64_t* U) {
  const bool os = c->flags & GS_FLAG_BK_ONESWEEP;
  switch (dir) {
    case DIR_IN:
      return os ? bucket_onesweep<P, DIR_IN>(c, src, dst, val, n, o, U) : bucket_direct<P, DIR_IN>(c, src, dst, val, n, o, U);
    case DIR_OUT:
      return os ? bucket_onesweep<P, DIR_OUT>(c, src, dst, val, n, o, U)
                : bucket_direct<P, DIR_OUT>(c, src, dst, val, n, o, U);
    case DIR_ALL:
      return os ? bucket_onesweep<P, DIR_ALL>(c, src, dst, val, n, o, U)
                : bucket_direct<P, DIR_ALL>(c, src, dst, val, n, o, U);
  }
  return set_error(c, GS_EINVAL, "bad direction %d", dir);
}

template <typename T, int OP>
gs_status bucket_value(gs_ctx* c, int dir, const int64_t* src, const int64_t* dst, const void* val, uint64_t n,
                       bool has_init, const void* init, int64_t* keys, void* vals, uint64_t* U) {
  using P = BkVal<T, OP>;
  typename P::Out o{keys, (T*)vals, has_init ? *(const T*)init : T{}, has_init};
  return bucket_dir<P>(c, dir, src, dst, val, n, o, U);
}

template <typename T>
gs_status bucket_value_op(gs_ctx* c, int op, int dir, const int64_t* src, const int64_t* dst, const void* val,
                          uint64_t n, bool has_init, const void* init, int64_t* keys, void* vals, uint64_t* U) {
  switch (op) {
    case OP_SUM: return bucket_value<T, OP_SUM>(c, dir, src, dst, val, n, has_init, init, keys, vals, U);
    case OP_MIN:
      if constexpr (std::is_integral_v<T>) return bucket_value<T, OP_MIN>(c, dir, src, dst, val, n, has_init, init, keys, vals, U);
      break;
    case OP_MAX:
      if constexpr (std::is_integral_v<T>) return bucket_value<T, OP_MAX>(c, dir, src, dst, val, n, has_init, init, keys, vals, U);
      break;
  }
  return GS_EUNSUPPORTED;
}

}  // namespace

gs_status bucket_reduce(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, uint64_t n, int dir,
                        int op, int dtype, bool has_init, const void* init, int64_t* keys, void* vals, uint64_t* U) {
  if (c->flags & GS_FLAG_SORT_ONLY) return GS_EUNSUPPORTED;
  if (op == OP_COUNT) {
    BkCount::Out o{keys, (int64_t*)vals, has_init ? *(const int64_t*)init : 0};
    return bucket_dir<BkCount>(c, dir, src, dst, nullptr, n, o, U);
  }
  switch (dtype) {
    case GS_I32: return bucket_value_op<int32_t>(c, op, dir, src, dst, val, n, has_init, init, keys, vals, U);
    case GS_I64: return bucket_value_op<int64_t>(c, op, dir, src, dst, val, n, has_init, init, keys, vals, U);
    case GS_F32: return bucket_value_op<float>(c, op, dir, src, dst, val, n, has_init, init, keys, vals, U);
    case GS_F64: return bucket_value_op<double>(c, op, dir, src, dst, val, n, has_init, init, keys, vals, U);
  }
  return GS_EUNSUPPORTED;
}

gs_status bucket_degree_max(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, int dir, int64_t init_max,
                            int64_t* keys, int64_t* deg, int64_t* mx, uint64_t* U) {
  if (c->flags & GS_FLAG_SORT_ONLY) return GS_EUNSUPPORTED;
  BkDeg::Out o{keys, deg, mx, init_max};
  if (!(c->flags & GS_FLAG_BK_ONESWEEP)) {   // neighbours as 32-bit offsets: 2^14 vertices per bucket
    const gs_status st = bucket_dir<BkDeg32>(c, dir, src, dst, nullptr, n, o, U);
    if (st != GS_RETRY_WIDE) return st;
  }
  return bucket_dir<BkDeg>(c, dir, src, dst, nullptr, n, o, U);
}

}  // namespace gs

#ifdef GS_BK_TRACE
// tuning builds only (tools/accum_trace.py): the last accumulate's per-item records
extern "C" __attribute__((visibility("default"))) int gs_debug_bk_trace(void* dst, uint32_t n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(gs::g_bk_trace), (size_t)std::min<uint32_t>(n, gs::BK_TRACE_MAX) * 32, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
