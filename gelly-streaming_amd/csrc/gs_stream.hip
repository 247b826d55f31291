// gs_stream.hip — the columnar event-time window-buffer operator behind the C ABI (gs_stream_*).
//
// The reference gets its windows from Flink: slice() keys the edge stream and assigns tumbling
// event-time windows (SimpleEdgeStream.java:153-171 -> keyBy(...).timeWindow(size)), and the window
// operator buffers each (vertex, window)'s records and fires the window function when the watermark
// passes the window's end (GraphWindowStream.java:49-53, 62-182; Flink 1.0.3 WindowOperator +
// EventTimeTrigger + TumblingEventTimeWindows).  The GPU path needs a whole window as ONE columnar
// batch, so this operator owns the windowing for the built-in operators:
//
//   assignment   start = ts - ts % size (Java's truncating remainder), end = start + size
//   buffering    per open window, columns appended in arrival order into pinned host memory
//   firing       a window fires when the watermark reaches end - 1 (EventTimeTrigger: watermark >=
//                maxTimestamp); its result carries the timestamp end - 1 (the window's maxTimestamp)
//   watermarks   explicit (gs_stream_watermark), or ascending: max timestamp seen - 1 after every
//                append (AscendingTimestampExtractor, SimpleEdgeStream.java:90-94 / WindowTriangles.java
//                :225-230); gs_stream_flush = the end of a finite source (watermark Long.MAX_VALUE)
//   late records records of an already fired window (the reference's ascending timestamps never
//                produce any): GS_LATE_REFIRE, as Flink 1.0.3's WindowOperator (no lateness check: a
//                fresh pane whose end - 1 timer fires at the next watermark), or GS_LATE_DROP; both count
//
// Pipelining: a fired window's columns go to one of two device slots with hipMemcpyAsync on the
// operator's copy stream; the window's kernels run on the ctx stream when the caller polls.  So the
// copy of window k+1 (fired before the poll of window k) overlaps window k's kernels, and the host
// keeps appending while both run.  Results are copied into pinned host buffers the poll hands out.
#include <string.h>

#include <chrono>
#include <deque>
#include <map>
#include <thread>
#include <vector>

#include "gs_ops.hpp"

using namespace gs;

namespace {

struct PinnedCols {   // one window's host columns (pinned)
  int64_t start = 0;
  int64_t* src = nullptr;
  int64_t* dst = nullptr;
  char* val = nullptr;
  uint64_t n = 0, cap = 0;
};

struct Slot {   // device columns of one in-flight window
  int64_t* src = nullptr;
  int64_t* dst = nullptr;
  char* val = nullptr;
  uint64_t cap = 0;
  hipEvent_t copied = nullptr;
  bool busy = false;
};

struct Fired {   // a window whose columns are on their way to (or in) a device slot
  int64_t start = 0;
  uint64_t n = 0;
  Slot* slot = nullptr;
  PinnedCols* cols = nullptr;   // pinned staging: returned to the pool once the copy has landed
  double fired_at = 0;          // host seconds (latency from fire to result)
};

struct DirectWin {   // GS_STAGE_DIRECT: an open window's columns already on the device
  Slot* slot = nullptr;
  uint64_t n = 0;
};

struct Result {   // one window's result; its rows live in the pinned buffers below
  gs_window_result r{};
  int64_t* keys = nullptr;
  char* vals = nullptr;
  int64_t* vals2 = nullptr;
  uint64_t cap = 0;
};

// host copy into the pinned window buffers: large blocks split over threads (one thread streams
// ~5-10 GB/s of host memory; a 2^28-edge window is 6 GB)
// host memory the DMA engines can read directly (hipHostMalloc / registered); pageable memory is not
bool is_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();   // a pageable pointer: clear the error the query left
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

void par_memcpy(void* dst, const void* src, size_t bytes) {
  constexpr size_t PART = 64ull << 20;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned T = (unsigned)std::min<size_t>(hw, bytes / PART);
  if (T <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (bytes + T - 1) / T;
  for (unsigned t = 0; t < T; ++t) {
    const size_t a = std::min(bytes, t * per), b = std::min(bytes, a + per);
    th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

// the end of the run of records from i whose timestamps lie in [lo, hi], and their maximum into *mx;
// long scans split over threads (each thread: the first record outside the range in its chunk and
// the maximum before it)
uint64_t run_end(const int64_t* ts, uint64_t i, uint64_t n, int64_t lo, int64_t hi, int64_t* mx) {
  constexpr uint64_t PART = 1ull << 22;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned T = (unsigned)std::min<uint64_t>(hw, (n - i) / PART);
  auto scan = [&](uint64_t a, uint64_t b, uint64_t* out, int64_t* m) {
    int64_t x = INT64_MIN;
    uint64_t q = a;
    for (; q < b && ts[q] >= lo && ts[q] <= hi; ++q) x = std::max(x, ts[q]);
    *out = q;
    *m = x;
  };
  if (T <= 1) {
    uint64_t j;
    int64_t m;
    scan(i, n, &j, &m);
    *mx = std::max(*mx, m);
    return j;
  }
  std::vector<uint64_t> ends(T);
  std::vector<int64_t> ms(T);
  std::vector<std::thread> th;
  const uint64_t per = (n - i + T - 1) / T;
  for (unsigned t = 0; t < T; ++t) {
    const uint64_t a = std::min(n, i + t * per), b = std::min(n, a + per);
    th.emplace_back([&, a, b, t] { scan(a, b, &ends[t], &ms[t]); });
  }
  for (auto& x : th) x.join();
  for (unsigned t = 0; t < T; ++t) {
    *mx = std::max(*mx, ms[t]);
    const uint64_t b = std::min(n, std::min(n, i + t * per) + per);
    if (ends[t] < b) return ends[t];
  }
  return n;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct gs_stream {
  gs_ctx* c = nullptr;
  gs_stream_config cfg{};
  size_t vb = 0;                       // value bytes (0: NullValue)
  std::vector<char> init;              // foldNeighbors init value
  std::map<int64_t, PinnedCols*> open; // open windows by start
  std::vector<PinnedCols*> pool;       // free pinned column buffers
  int64_t watermark = INT64_MIN;
  int64_t max_ts = INT64_MIN;
  uint64_t late = 0, fired_total = 0, edges_total = 0;
  hipStream_t copy = nullptr;
  std::vector<Slot*> slots;            // every device slot (owned)
  std::vector<Slot*> free_slots;
  int in_flight = 0;                   // pinned staging: fired windows holding a slot (at most 2)
  std::map<int64_t, DirectWin> dopen;  // GS_STAGE_DIRECT: open windows by start
  std::deque<Fired> fired;
  std::deque<Result*> ready;
  std::vector<Result*> rpool;
  Result* current = nullptr;           // handed out by the last poll
  std::string err;
  hipEvent_t appended = nullptr;       // direct staging from pinned columns: the append's DMAs are done
};

namespace {

void free_cols(PinnedCols* p) {
  if (!p) return;
  hipHostFree(p->src);
  hipHostFree(p->dst);
  if (p->val) hipHostFree(p->val);
  delete p;
}

gs_status grow_cols(gs_stream* s, PinnedCols* p, uint64_t need) {
  if (need <= p->cap) return GS_OK;
  uint64_t cap = std::max<uint64_t>(need, std::max<uint64_t>(p->cap * 2, s->cfg.max_window_edges ? s->cfg.max_window_edges : 1024));
  int64_t *ns = nullptr, *nd = nullptr;
  char* nv = nullptr;
  if (hipHostMalloc((void**)&ns, cap * 8, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&nd, cap * 8, hipHostMallocDefault) != hipSuccess ||
      (s->vb && hipHostMalloc((void**)&nv, cap * s->vb, hipHostMallocDefault) != hipSuccess)) {
    if (ns) hipHostFree(ns);
    if (nd) hipHostFree(nd);
    return gs::set_error(s->c, GS_ENOMEM, "gs_stream: pinned allocation of %llu edges failed", (unsigned long long)cap);
  }
  if (p->n) {
    memcpy(ns, p->src, p->n * 8);
    memcpy(nd, p->dst, p->n * 8);
    if (s->vb) memcpy(nv, p->val, p->n * s->vb);
  }
  if (p->src) hipHostFree(p->src);
  if (p->dst) hipHostFree(p->dst);
  if (p->val) hipHostFree(p->val);
  p->src = ns;
  p->dst = nd;
  p->val = nv;
  p->cap = cap;
  return GS_OK;
}

PinnedCols* take_cols(gs_stream* s) {
  if (!s->pool.empty()) {
    PinnedCols* p = s->pool.back();
    s->pool.pop_back();
    p->n = 0;
    return p;
  }
  return new PinnedCols();
}

// device columns of >= n edges; the first `keep` edges survive a reallocation (direct staging grows a
// window's slot while records arrive)
gs_status ensure_slot(gs_stream* s, Slot& sl, uint64_t n, uint64_t keep = 0) {
  gs_ctx* c = s->c;
  if (!sl.copied) GS_HIP(hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming));
  if (n <= sl.cap) return GS_OK;
  const uint64_t cap = std::max<uint64_t>(std::max<uint64_t>(n, sl.cap * 2), s->cfg.max_window_edges);
  int64_t *ns = nullptr, *nd = nullptr;
  char* nv = nullptr;
  GS_HIP(hipMalloc((void**)&ns, cap * 8));
  GS_HIP(hipMalloc((void**)&nd, cap * 8));
  if (s->vb) GS_HIP(hipMalloc((void**)&nv, cap * s->vb));
  if (keep) {
    GS_HIP(hipMemcpyAsync(ns, sl.src, keep * 8, hipMemcpyDeviceToDevice, s->copy));
    GS_HIP(hipMemcpyAsync(nd, sl.dst, keep * 8, hipMemcpyDeviceToDevice, s->copy));
    if (s->vb) GS_HIP(hipMemcpyAsync(nv, sl.val, keep * s->vb, hipMemcpyDeviceToDevice, s->copy));
    GS_HIP(hipStreamSynchronize(s->copy));
  }
  if (sl.src) hipFree(sl.src);
  if (sl.dst) hipFree(sl.dst);
  if (sl.val) hipFree(sl.val);
  sl.src = ns;
  sl.dst = nd;
  sl.val = nv;
  sl.cap = cap;
  return GS_OK;
}

Slot* take_slot(gs_stream* s) {
  if (!s->free_slots.empty()) {
    Slot* sl = s->free_slots.back();
    s->free_slots.pop_back();
    return sl;
  }
  Slot* sl = new Slot();
  s->slots.push_back(sl);
  return sl;
}

Result* take_result(gs_stream* s, uint64_t rows) {
  Result* r = nullptr;
  if (!s->rpool.empty()) {
    r = s->rpool.back();
    s->rpool.pop_back();
  } else {
    r = new Result();
  }
  if (rows > r->cap) {
    if (r->keys) hipHostFree(r->keys);
    if (r->vals) hipHostFree(r->vals);
    if (r->vals2) hipHostFree(r->vals2);
    r->keys = nullptr;
    r->vals = nullptr;
    r->vals2 = nullptr;
    const uint64_t cap = std::max<uint64_t>(rows, 1024);
    if (hipHostMalloc((void**)&r->keys, cap * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&r->vals, cap * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&r->vals2, cap * 8, hipHostMallocDefault) != hipSuccess) {
      r->cap = 0;
      s->rpool.push_back(r);
      return nullptr;
    }
    r->cap = cap;
  }
  r->r = gs_window_result{};
  return r;
}

void free_result(Result* r) {
  if (!r) return;
  if (r->keys) hipHostFree(r->keys);
  if (r->vals) hipHostFree(r->vals);
  if (r->vals2) hipHostFree(r->vals2);
  delete r;
}

// the window's kernels (ctx stream, after its copy landed) and the D2H of its results
gs_status process_one(gs_stream* s) {
  gs_ctx* c = s->c;
  Fired f = s->fired.front();
  s->fired.pop_front();
  Slot& sl = *f.slot;
  GS_HIP(hipStreamWaitEvent(c->stream, sl.copied, 0));
  const int64_t end = f.start + s->cfg.window_ms;
  gs_edge_batch b{sl.src, sl.dst, s->vb ? sl.val : nullptr, f.n, s->cfg.val_dtype, GS_MEM_DEVICE, end};
  const uint64_t R = s->cfg.dir == GS_DIR_ALL ? 2 * f.n : f.n;
  Result* res = take_result(s, s->cfg.kind == GS_STREAM_TRIANGLES ? 1 : R);
  if (!res) return gs::set_error(c, GS_ENOMEM, "gs_stream: pinned result allocation failed");
  gs_window_result& r = res->r;
  r.window_start = f.start;
  r.window_end = end;
  r.max_timestamp = end - 1;
  r.edges = f.n;
  uint64_t U = 0;
  gs_status st = GS_OK;
  switch (s->cfg.kind) {
    case GS_STREAM_REDUCE:
    case GS_STREAM_FOLD: {
      gs_vertex_out o{res->keys, res->vals, res->cap, &U, GS_MEM_HOST, 0};
      st = s->cfg.kind == GS_STREAM_REDUCE ? gs_window_reduce(c, &b, s->cfg.dir, s->cfg.op, &o)
                                            : gs_window_fold(c, &b, s->cfg.dir, s->cfg.op, s->init.data(), &o);
      r.keys = res->keys;
      r.vals = res->vals;
      break;
    }
    case GS_STREAM_DEGREE_MAX: {
      gs_degree_out o{res->keys, (int64_t*)res->vals, res->vals2, res->cap, &U, GS_MEM_HOST, 0};
      st = gs_window_fold_degree_max(c, &b, s->cfg.dir, s->cfg.init_max, &o);
      r.keys = res->keys;
      r.vals = res->vals;
      r.vals2 = res->vals2;
      break;
    }
    case GS_STREAM_TRIANGLES: {
      int32_t has = 0;
      st = gs_window_triangles(c, &b, &r.triangles, &r.triangles_ref, &has);
      r.has_output = has;
      break;
    }
  }
  // the slot is free once the kernels that read it are done (the calls above end with a host wait),
  // and the window's pinned columns (copied before those kernels ran) can be refilled
  sl.busy = false;
  s->free_slots.push_back(f.slot);
  if (s->cfg.staging != GS_STAGE_DIRECT) --s->in_flight;
  if (f.cols) s->pool.push_back(f.cols);
  if (st != GS_OK) {
    s->rpool.push_back(res);
    return st;
  }
  r.n_vertices = U;
  if (s->cfg.kind != GS_STREAM_TRIANGLES) r.has_output = U > 0;
  r.latency_ms = (now_s() - f.fired_at) * 1e3;
  s->ready.push_back(res);
  return GS_OK;
}

// fire the window starting at `start`.  Pinned staging: enqueue its copy into a free device slot (at
// most two windows in flight: the oldest runs first when both slots are taken).  Direct staging: its
// columns are already on their way (appends copied them); mark the end of its copies.
gs_status fire(gs_stream* s, int64_t start) {
  gs_ctx* c = s->c;
  Fired f;
  f.start = start;
  if (s->cfg.staging == GS_STAGE_DIRECT) {
    auto it = s->dopen.find(start);
    DirectWin w = it->second;
    s->dopen.erase(it);
    if (w.n == 0) {
      s->free_slots.push_back(w.slot);
      return GS_OK;
    }
    GS_HIP(hipEventRecord(w.slot->copied, s->copy));
    w.slot->busy = true;
    f.n = w.n;
    f.slot = w.slot;
  } else {
    auto it = s->open.find(start);
    PinnedCols* p = it->second;
    s->open.erase(it);
    if (p->n == 0) {   // no records: Flink creates no window, nothing is emitted
      s->pool.push_back(p);
      return GS_OK;
    }
    while (s->in_flight >= 2) GS_TRY(process_one(s));   // double buffering: the oldest window runs first
    Slot* sl = take_slot(s);
    GS_TRY(ensure_slot(s, *sl, p->n));
    GS_HIP(hipMemcpyAsync(sl->src, p->src, p->n * 8, hipMemcpyHostToDevice, s->copy));
    GS_HIP(hipMemcpyAsync(sl->dst, p->dst, p->n * 8, hipMemcpyHostToDevice, s->copy));
    if (s->vb) GS_HIP(hipMemcpyAsync(sl->val, p->val, p->n * s->vb, hipMemcpyHostToDevice, s->copy));
    GS_HIP(hipEventRecord(sl->copied, s->copy));
    sl->busy = true;
    ++s->in_flight;
    f.n = p->n;
    f.slot = sl;
    f.cols = p;
  }
  f.fired_at = now_s();
  s->fired.push_back(f);
  s->fired_total++;
  s->edges_total += f.n;
  return GS_OK;
}

// pinned buffers whose copy has landed go back to the pool
void reclaim(gs_stream* s) {
  for (Fired& f : s->fired) {
    if (f.cols && hipEventQuery(f.slot->copied) == hipSuccess) {
      s->pool.push_back(f.cols);
      f.cols = nullptr;
    }
  }
}

gs_status advance(gs_stream* s, int64_t wm) {
  if (wm <= s->watermark) return GS_OK;
  s->watermark = wm;
  // fire every open window with end - 1 <= watermark, oldest first
  const bool direct = s->cfg.staging == GS_STAGE_DIRECT;
  while (direct ? !s->dopen.empty() : !s->open.empty()) {
    const int64_t start = direct ? s->dopen.begin()->first : s->open.begin()->first;
    if (start + s->cfg.window_ms - 1 > wm) break;
    GS_TRY(fire(s, start));
  }
  return GS_OK;
}

}  // namespace

extern "C" {

gs_status gs_stream_create(gs_ctx* c, const gs_stream_config* cfg, gs_stream** out) {
  if (!c) return GS_EINVAL;
  if (!cfg || !out) return set_error(c, GS_EINVAL, "gs_stream_create: null argument");
  *out = nullptr;
  if (cfg->window_ms <= 0) return set_error(c, GS_EINVAL, "gs_stream_create: window size must be > 0");
  if (cfg->dir < 0 || cfg->dir > 2) return set_error(c, GS_EINVAL, "bad EdgeDirection %d", cfg->dir);
  if (cfg->kind < GS_STREAM_REDUCE || cfg->kind > GS_STREAM_TRIANGLES) return set_error(c, GS_EINVAL, "bad stream kind");
  if (cfg->val_dtype < GS_I32 || cfg->val_dtype > GS_NONE) return set_error(c, GS_EINVAL, "bad dtype %d", cfg->val_dtype);
  if ((cfg->kind == GS_STREAM_REDUCE || cfg->kind == GS_STREAM_FOLD) &&
      (cfg->op < GS_OP_SUM || cfg->op > GS_OP_COUNT || (cfg->op != GS_OP_COUNT && cfg->val_dtype == GS_NONE)))
    return set_error(c, GS_EINVAL, "bad op %d for dtype %d", cfg->op, cfg->val_dtype);
  if (cfg->kind == GS_STREAM_FOLD && !cfg->init) return set_error(c, GS_EINVAL, "foldNeighbors needs an init value");
  if (cfg->staging != GS_STAGE_PINNED && cfg->staging != GS_STAGE_DIRECT) return set_error(c, GS_EINVAL, "bad staging mode");
  if (cfg->late_mode != GS_LATE_REFIRE && cfg->late_mode != GS_LATE_DROP) return set_error(c, GS_EINVAL, "bad late mode");
  gs_stream* s = new (std::nothrow) gs_stream();
  if (!s) return GS_ENOMEM;
  s->c = c;
  s->cfg = *cfg;
  s->vb = (cfg->kind == GS_STREAM_REDUCE || cfg->kind == GS_STREAM_FOLD) ? dtype_bytes(cfg->val_dtype) : 0;
  if (cfg->kind == GS_STREAM_FOLD) {
    const size_t ib = cfg->op == GS_OP_COUNT ? 8 : dtype_bytes(cfg->val_dtype);
    s->init.assign((const char*)cfg->init, (const char*)cfg->init + ib);
  }
  s->cfg.init = nullptr;
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&s->copy, hipStreamNonBlocking) != hipSuccess) {
    delete s;
    return set_error(c, GS_EDEVICE, "gs_stream_create: copy stream");
  }
  *out = s;
  return GS_OK;
}

void gs_stream_destroy(gs_stream* s) {
  if (!s) return;
  hipSetDevice(s->c->device);
  if (s->copy) hipStreamSynchronize(s->copy);
  hipStreamSynchronize(s->c->stream);
  for (auto& kv : s->open) free_cols(kv.second);
  for (Fired& f : s->fired) free_cols(f.cols);
  for (PinnedCols* p : s->pool) free_cols(p);
  for (Slot* sl : s->slots) {
    if (sl->src) hipFree(sl->src);
    if (sl->dst) hipFree(sl->dst);
    if (sl->val) hipFree(sl->val);
    if (sl->copied) hipEventDestroy(sl->copied);
    delete sl;
  }
  for (Result* r : s->ready) free_result(r);
  for (Result* r : s->rpool) free_result(r);
  free_result(s->current);
  if (s->copy) hipStreamDestroy(s->copy);
  if (s->appended) hipEventDestroy(s->appended);
  delete s;
}

gs_status gs_stream_append(gs_stream* s, const int64_t* src, const int64_t* dst, const void* val, const int64_t* ts,
                           uint64_t n) {
  if (!s) return GS_EINVAL;
  gs_ctx* c = s->c;
  if (n && (!src || !dst || !ts || (s->vb && !val))) return set_error(c, GS_EINVAL, "gs_stream_append: null column");
  const int64_t size = s->cfg.window_ms;
  reclaim(s);
  // runs of consecutive records of one window are copied as one block (ascending timestamps: one run
  // per window).  The run test is a range check: the timestamps of window `start` are [start, start +
  // size) for start > 0, (start - size, start] for start < 0 and (-size, size) for start 0 (Java's
  // truncating remainder).
  uint64_t i = 0;
  int64_t mx = s->max_ts;
  // direct staging from caller-pinned columns (gs_alloc_pinned, a Java direct buffer registered with
  // HIP): the copies are DMAs straight from them at PCIe rate, no runtime staging copy; the append
  // returns once they have read the columns (the caller may refill them)
  const bool pinned_src = s->cfg.staging == GS_STAGE_DIRECT && n && is_pinned(src) && is_pinned(dst) &&
                          (!s->vb || is_pinned(val));
  bool queued = false;
  while (i < n) {
    const int64_t start = ts[i] - ts[i] % size;
    const int64_t lo = start > 0 ? start : start - size + 1, hi = start < 0 ? start : start + size - 1;
    const uint64_t j = run_end(ts, i, n, lo, hi, &mx);
    const uint64_t k = j - i;
    const bool late = start + size - 1 <= s->watermark;   // the window already fired
    if (late) s->late += k;
    if (late && s->cfg.late_mode == GS_LATE_DROP) {
      // dropped (counted above)
    } else if (s->cfg.staging == GS_STAGE_DIRECT) {   // (a late run opens a fresh pane: GS_LATE_REFIRE)
      auto it = s->dopen.find(start);
      if (it == s->dopen.end()) it = s->dopen.emplace(start, DirectWin{take_slot(s), 0}).first;
      DirectWin& w = it->second;
      GS_TRY(ensure_slot(s, *w.slot, w.n + k, w.n));
      // pageable host -> HBM on the copy stream (the runtime stages it); overlaps the kernels of
      // windows that already fired
      GS_HIP(hipMemcpyAsync(w.slot->src + w.n, src + i, k * 8, hipMemcpyHostToDevice, s->copy));
      GS_HIP(hipMemcpyAsync(w.slot->dst + w.n, dst + i, k * 8, hipMemcpyHostToDevice, s->copy));
      if (s->vb)
        GS_HIP(hipMemcpyAsync(w.slot->val + w.n * s->vb, (const char*)val + i * s->vb, k * s->vb,
                              hipMemcpyHostToDevice, s->copy));
      w.n += k;
      queued = true;
    } else {
      auto it = s->open.find(start);
      PinnedCols* p;
      if (it == s->open.end()) {
        p = take_cols(s);
        p->start = start;
        s->open.emplace(start, p);
      } else {
        p = it->second;
      }
      GS_TRY(grow_cols(s, p, p->n + k));
      par_memcpy(p->src + p->n, src + i, k * 8);
      par_memcpy(p->dst + p->n, dst + i, k * 8);
      if (s->vb) par_memcpy(p->val + p->n * s->vb, (const char*)val + i * s->vb, k * s->vb);
      p->n += k;
    }
    i = j;
  }
  if (pinned_src && queued) {
    if (!s->appended) GS_HIP(hipEventCreateWithFlags(&s->appended, hipEventDisableTiming));
    GS_HIP(hipEventRecord(s->appended, s->copy));
    GS_HIP(hipEventSynchronize(s->appended));
  }
  s->max_ts = mx;
  if (s->cfg.watermark_mode == GS_WATERMARK_ASCENDING && s->max_ts != INT64_MIN) GS_TRY(advance(s, s->max_ts - 1));
  return GS_OK;
}

gs_status gs_stream_watermark(gs_stream* s, int64_t watermark) {
  if (!s) return GS_EINVAL;
  return advance(s, watermark);
}

gs_status gs_stream_flush(gs_stream* s) {
  if (!s) return GS_EINVAL;
  return advance(s, INT64_MAX);
}

gs_status gs_stream_poll(gs_stream* s, int32_t wait, gs_window_result* out) {
  if (!s || !out) return s ? set_error(s->c, GS_EINVAL, "gs_stream_poll: null result") : GS_EINVAL;
  if (s->current) {   // the previous poll's buffers are recycled now
    s->rpool.push_back(s->current);
    s->current = nullptr;
  }
  // run the oldest fired window when nothing is ready: always when waiting, else only once its
  // copy has landed (a non-blocking poll never waits on the copy)
  if (s->ready.empty() && !s->fired.empty()) {
    const Fired& f = s->fired.front();
    if (wait || hipEventQuery(f.slot->copied) == hipSuccess) GS_TRY(process_one(s));
  }
  reclaim(s);
  if (s->ready.empty()) {
    *out = gs_window_result{};
    return GS_EAGAIN;
  }
  s->current = s->ready.front();
  s->ready.pop_front();
  *out = s->current->r;
  return GS_OK;
}

gs_status gs_stream_stats(const gs_stream* s, gs_stream_stats_t* out) {
  if (!s || !out) return GS_EINVAL;
  out->watermark = s->watermark;
  out->open_windows = s->open.size() + s->dopen.size();
  out->fired_windows = s->fired_total;
  out->pending_windows = s->fired.size() + s->ready.size();
  out->late_records = s->late;
  out->edges_fired = s->edges_total;
  return GS_OK;
}

}  // extern "C"
