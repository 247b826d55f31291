// gs_internal.hpp — host-side context, workspace and the window sort shared by all operators.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include <string>

#include "../../include/gelly_hip.h"

namespace gs {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

// Result of the window sort: compact keys + payload in key order (stable).
// gs_window_reduce_dist's local window: with nparts set, the bucket path's last stage writes the
// exchange's packed rows grouped by owner (k_bk_owner_count / k_owner_scan / k_bk_owner_emit) instead of
// the ascending (vertex, value) output, and sets `done` (a window that took another path leaves it unset:
// the caller partitions that output itself)
struct OwnerEmit {
  uint32_t nparts = 0;                   // 0: off
  uint32_t* rows = nullptr;              // packed rows, owner-major
  uint32_t* cnt = nullptr;               // [nparts][buckets] rows per (owner, bucket) -> write offsets
  unsigned long long* totals = nullptr;  // [nparts] rows per owner
  unsigned long long* wide = nullptr;    // key-width flag
  int vw = 0, mw = 0;                    // value / maximum words per row
  unsigned long long* send = nullptr;    // [nparts][2] the counts exchange's send rows (k_send_rows)
  bool done = false;
  // defer: a speculative window returns GS_PENDING_LOCAL right after its launches (no host wait); the
  // caller's next wait brings its read-back block, and the same call again with `resume` checks it
  // (a missed speculation reruns there) and completes the window
  bool defer = false, resume = false;
};
constexpr gs_status GS_PENDING_LOCAL = -101;   // internal (never returned across the ABI)

struct Sorted {
  void* keys = nullptr;     // uint32_t or uint64_t
  void* vals = nullptr;     // payload (nullptr when none)
  bool wide = false;        // 64-bit keys
  uint64_t key_xor = 0;     // key = key_xor ^ compact
  uint64_t records = 0;
  int bits = 0, passes = 0;
  int payload_bytes = 0;
  int done_passes = 0;      // passes executed (passes - 1 when the last is left to a fused pass)
  bool fused = false;       // the last pass ran fused with the combine (gs_combine.hpp)
};

// split points of the split-window triangle route: owner q holds the degree-order ranks
// [s[q], s[q + 1]) (up to 64 parts); passed to kernels by value
struct RtSplit {
  uint32_t s[65];
};

}  // namespace gs

struct gs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  uint32_t epoch = 0;
  bool timeout_clean = false;      // SM_TIMEOUT known zero (begin_call)
  int timing = GS_TIMING_STAGES;   // gs_set_timing: which stage events a window records (stage_event)
  int hist_digits = 4;   // key-byte histograms keyinfo computes (learned from the previous window)
  uint32_t flags = 0;    // gs_config.flags
  int64_t bk_base = 0;   // bucket path: predicted lower bound of the next window's vertex IDs
  uint32_t bk_nbp = 0;   // direct bucket path: predicted bucket count (0 = BK_MAXB)
  int bk_wide_vals[2] = {0, 0};   // per sp_slot: a merge's wide partial sums must not unpack the windows
  // the last window call's output: U rows of ob-byte values, staged in out_keys / out_a (/ out_b) when
  // last_kind is 1 (vertex, value) or 2 (degree / max) -- gs_fetch_last_output after GS_ECAPACITY
  uint64_t last_U = 0;
  size_t last_ob = 0;
  int last_kind = 0;  // direct bucket path: > 0 = windows left that store 8-byte values (escapes were common)
  int n_cu = 0;          // compute units (persistent grids)
  // chunked windows (gs_set_max_window_records): records per engine pass, running partials (ping-pong)
  uint64_t max_records = (1ull << 32) - 1;
  bool in_chunk = false;
  gs::DevBuf ck_k[2], ck_a[2], ck_b[2];
  // chunked candidate emission (gs_candidates_begin / _next): the window's HashSet-ordered sets stay in
  // hs[] until the next entry point call on the ctx (call_seq) ends the session
  uint64_t call_seq = 0, cand_seq = ~0ull, cand_total = 0, cand_cursor = 0;
  uint32_t cand_U = 0, cand_S = 0, cand_nparts = 1;
  int64_t cand_idmin = 0, cand_idmax = 0;   // the session's id range (gs_candidates_next_u32)
  gs::DevBuf cand_bounds, cand_steps;   // (cand_steps: the steps k_cand_emit<1> leaves to k_cand_emit_rest)
  // input staging (host batches)
  gs::DevBuf in_src, in_dst, in_val;
  // sort ping-pong
  gs::DevBuf keysA, keysB, valsA, valsB;
  // look-back granules
  gs::DevBuf sort_status, rbk_word, rbk_agg, rbk_inc;
  // small scalars: see gs_engine.hip layout
  gs::DevBuf small;
  // output staging
  gs::DevBuf out_keys, out_a, out_b, aux;
  // fused last pass: partials with gaps, compacted partials
  gs::DevBuf part_k, part_a, comp_k, comp_a;
  // triangles
  gs::DevBuf tri_loops, tri_tiles, tri_sfx, tri_nbr, tri_heavy, tri_range, tri_queue, tri_hwork;
  gs::DevBuf tri_d[10];          // split-window triangles (gs_window_triangles_dist)
  gs::DevBuf cc[4];              // connected components (gs_components.hip; [3]: the giant tree's bits)
  uint32_t tri_guess_B = 0;      // triangles: the previous window's id width (its partition histograms ride the id scan)
  uint32_t tri_B = 0;            // split-window triangles: id geometry of the current window
  uint64_t tri_key_xor = 0;
  // split-window triangles, boundary adjacency (gs_tri_dist_plan / _need / _serve / _assemble): this
  // rank's count range [bd_c0, bd_c1) and route range [bd_r0, bd_r1) of the degree order with their
  // adjacency positions (bd_p*), the window's unique edges bd_M, the ids it requested (tri_bd[0]) and
  // the prefix of their row lengths (tri_bd[1])
  uint32_t bd_part = 0, bd_nparts = 0;
  uint64_t bd_c0 = 0, bd_c1 = 0, bd_r0 = 0, bd_r1 = 0, bd_pc0 = 0, bd_pc1 = 0, bd_pr0 = 0, bd_pr1 = 0, bd_M = 0;
  uint64_t bd_nreq = 0;
  bool bd_ok = false;
  // the route step's split points (owner ranges of the degree order) and the oriented keys it waits
  // for (rt_n local keys in aux, valid while rt_seq == call_seq)
  gs::RtSplit rt_split{};
  uint64_t rt_n = ~0ull, rt_seq = 0;
  uint32_t rt_nparts = 0;
  gs::DevBuf tri_bd[4];
  gs::DevBuf tri_rl[4];          // split-window triangles over wide ids: compact columns, local / all ids
  // HashSet-order pipeline (gs_hashset.hip)
  gs::DevBuf hs[40];
  gs::DevBuf hs_rank;            // dense vertex-rank table of the window (k_hs_rank)
  // bucket path (gs_bucket.hip): plan tables, work items, LDS slabs of multi-item buckets
  gs::DevBuf bk_meta, bk_items, bk_slabs;
  // direct partition: per-tile bucket counts (u16), chunk sums, per-tile write offsets
  gs::DevBuf dp_cnt, dp_csum, dp_off;
  // speculative partition (k_sp_scatter*): per stream of windows, the last window's bucket counts, the
  // geometry they were taken in and the windows left before the next try after a miss; slot 0 = the
  // caller's windows, slot 1 = the multi-GPU merges (their rows spread over the buckets unlike the
  // windows', so they keep their own counts); bucket cursors shared
  struct SpState {
    gs::DevBuf tot;
    bool ok = false;
    int S = 0, dir = -1, skip = 0;
    int64_t base = 0;
    uint64_t R = 0;
  } sp[2];
  int sp_slot = 0;
  uint64_t tri_merge = 0;   // the last count's sum of d+(u) + d+(v) over its oriented edges (tri_times)
  gs::OwnerEmit oe;         // gs_window_reduce_dist: the bucket path emits the exchange's rows (gs_dist.hip)
  gs::DevBuf sp_cur;
  // stage-2 candidate count (gs_pairs.hip): staged input columns, packed keys / payloads, group sums
  gs::DevBuf pr_a, pr_b, pr_f, pr_key, pr_val, pr_gk, pr_gv, pr_small;
  // edge text parser (gs_text.hip): staged text, tile newline counts, record starts
  gs::DevBuf tx_text, tx_cnt, tx_starts;
  // multi-GPU keyBy (gs_dist.hip): staging of the local reduce, owner-grouped partials, received rows,
  // per-tile owner counts; the ctx communicator (gs_comm.hip): an RCCL ncclComm_t (comm_kind
  // GS_COMM_KIND_RCCL) or an in-process gs_comm_group (GS_COMM_KIND_GROUP; comm_scratch: its all-reduce)
  gs::DevBuf dist_k, dist_v, dist_v2, dist_k2, dist_v3, dist_v4, dist_cnt, dist_x, dist_x2;
  void* comm = nullptr;
  int comm_kind = 0;
  int comm_size = 0, comm_rank = 0;
  gs::DevBuf comm_scratch;
  // relabeling of arbitrary vertex IDs (gs_relabel.hip)
  gs::DevBuf rl[8];
  // Zipf generator: CDF table of (zipf_v, zipf_s)
  gs::DevBuf zipf_cdf;
  uint64_t zipf_v = 0;
  double zipf_s = 0.0;
  hipEvent_t ev[6] = {};
  hipEvent_t sync_ev = nullptr;   // host_wait: polled completion event
  hipEvent_t pass_ev[9] = {};
  gs_stage_times times{};
  uint64_t* host_small = nullptr;  // pinned mirror of small scalars
  // GS_FLAG_ASYNC_OUTPUT: the bucket path's read-back block, written into pinned host memory by the emit
  // kernel's first block (rb_dev is its device address) and followed by a sequence word the host spins on
  uint64_t* rb_host = nullptr;
  uint64_t* rb_dev = nullptr;
  uint64_t rb_seq = 0;
  bool rb_allow = false;     // set by the entry point for this window (direct device outputs, not STAGES)
  bool rb_pending = false;   // the last bucket_accumulate left its read-back to bucket_wait
};

namespace gs {

// small-buffer layout (bytes)
constexpr size_t SM_MASK = 0;          // u64 OR(key ^ key0)
constexpr size_t SM_K0 = 8;            // u64 key0 (device copy)
constexpr size_t SM_NUNIQUE = 16;      // u64
constexpr size_t SM_TIMEOUT = 24;      // u32
constexpr size_t SM_COUNTERS = 32;     // u32[64] tile counters
constexpr size_t SM_HIST = 32 + 256;   // u32[8][256]
constexpr size_t SM_BASE = SM_HIST + 8 * 256 * 4;  // u32[8][256]
constexpr size_t SM_TOTAL = SM_BASE + 8 * 256 * 4;   // u64 partial count of the fused pass
constexpr size_t SM_TABLE = SM_TOTAL + 64;            // u32[513] region table of the fused pass
constexpr size_t SM_BK_MM = SM_TABLE + 520 * 4;    // u64[4] bucket path: min', max', outside, U
constexpr size_t SM_BK_N = SM_BK_MM + 32;            // u32[4] bucket path: items, multi buckets, claim ctr
constexpr size_t SM_BK_X = SM_BK_N + 16;            // u64[2] bucket path: copies of the timeout flag and the escape
                                                    // count (k_bk_emit), so the window reads back one 64-byte block
constexpr size_t SM_TRI_PROBES = SM_BK_X + 16;      // u64 triangles: hash probes of the counting step
constexpr size_t SM_TRI_NV = SM_TRI_PROBES + 8;     // u64 triangles: vertices with an edge (k_tri_lclass)
constexpr size_t SM_BK_ESC = SM_TRI_PROBES + 16;    // u64 packed scatter: escaped values
constexpr size_t SM_DEV_ERR = SM_BK_ESC + 8;        // u32 device error flags (GS_DERR_*)
constexpr size_t SM_HS = SM_DEV_ERR + 8;            // u32[4] HashSet order: complex vertices, JDK flags
constexpr size_t SM_TRI_MERGE = SM_HS + 16;      // u64 triangles: sum of d+(u) + d+(v) over the oriented edges
constexpr size_t SM_HIST9 = SM_TRI_MERGE + 8;      // u32[8][512] digit histograms of a 9-bit-digit sort
constexpr size_t SM_BASE9 = SM_HIST9 + 8 * 512 * 4;  // u32[8][512] their exclusive scans
constexpr size_t SM_BYTES = SM_BASE9 + 8 * 512 * 4;
// device error flags (SM_DEV_ERR): a kernel that cannot finish its work sets one and returns
constexpr uint32_t GS_DERR_TABLE_FULL = 1u;         // an LDS hash set filled up (triangle counting)
constexpr size_t HOST_SMALL_WORDS = 512;            // pinned u64 mirror of small scalars

gs_status set_error(gs_ctx* c, gs_status s, const char* fmt, ...);
gs_status hip_check(gs_ctx* c, hipError_t e, const char* what);
gs_status ensure(gs_ctx* c, DevBuf& b, size_t bytes, bool zero = false);
uint32_t next_epoch(gs_ctx* c, size_t status_bytes_hint);

// Sort the window's records by key (stable).  payload: 0 none, 1 value (val_bytes 4|8),
// 2 neighbour (int64), 3 record index (u32).  src/dst/val are device pointers.
// leave_last: run passes 0..P-2 only (at least one) so the caller can fuse the last pass.
gs_status sort_window(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, int val_bytes,
                      uint64_t n_edges, int dir, int payload, Sorted* out, bool leave_last = false);

// Sort an unsigned 64-bit key buffer (stable), optional u32 payload; keys of <= 32 varying bits are
// compacted to u32 (key = key_xor ^ compact).  `keys` must be 16-byte aligned.
// bits_hint: an upper bound on the key width (the histograms cover only those bytes); payload of
// val_bytes (4 or 8) per key, or none.  hist_ready: the kernel that wrote the keys (all < 2^bits_hint)
// already filled the digit histograms (SM_HIST, wave_hist_add): no scan, no host round trip
// digit_bits 9 (hist_ready callers only: bits_hint is then the key width): 9-bit digits, their histograms
// from one extra read of the keys -- one LSD pass less where 8-bit digits would leave a last pass of 1-2 bits
gs_status sort_buffer(gs_ctx* c, const uint64_t* keys, const void* vals, uint64_t n, Sorted* out,
                      int bits_hint = 64, int val_bytes = 4, bool hist_ready = false, int digit_bits = 8);
// the digit width for a sort of `bits`-bit keys: 8, or with GS_SORT_DIGIT9=1 9 when that saves a pass
int sort_digit_bits(int bits);

// HashSet-ordered distinct neighbour sets of an ALL window (gs_hashset.hip)
gs_status hashset_order(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, uint32_t* U_out,
                        uint32_t* M_out, uint64_t* key_xor_out, uint32_t* jdk_flags);
// WindowTriangles self-pair term for windows with self-loops (loops: bitmap over compact IDs: x ^ loops_xor,
// or, for a relabeled window, the rank of x among the sorted distinct IDs `relabel[0 .. nrel)`)
gs_status triangle_selfpair_term(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n,
                                 const uint32_t* loops, uint64_t loops_xor, const int64_t* relabel, uint64_t nrel,
                                 uint64_t* S);
// ctx communicator helpers (gs_comm.hip; RCCL enums: ncclInt64 4, ncclUint32 3, ncclUint64 5; ncclSum 0,
// ncclMax 2, ncclMin 3): in-place all-reduce of a device buffer; every rank's u64 to the host;
// grouped send / recv of owner-grouped rows
constexpr int NCCL_T_U32 = 3, NCCL_T_I64 = 4, NCCL_T_U64 = 5, NCCL_OP_SUM = 0, NCCL_OP_MAX = 2, NCCL_OP_MIN = 3;
constexpr int GS_COMM_KIND_RCCL = 1, GS_COMM_KIND_GROUP = 2;
gs_status comm_allreduce(gs_ctx* c, void* buf, size_t count, int nccl_dtype, int nccl_op);
gs_status comm_alltoall(gs_ctx* c, const void* send, void* recv, size_t count, int nccl_dtype);
gs_status comm_allgather_u64(gs_ctx* c, uint64_t mine, uint64_t* all);
gs_status comm_allgather_words(gs_ctx* c, const uint64_t* mine, int W, uint64_t* all);
gs_status comm_agree(gs_ctx* c, gs_status local);
// skip_self: this rank's own rows (send[me] == recv[me]) stay in sendbuf -- not copied, and the receive
// buffer holds only the peers' rows
gs_status exchange_rows(gs_ctx* c, const char* sendbuf, const uint64_t* send, char* recvbuf, const uint64_t* recv,
                        size_t row, bool skip_self = false);
gs_status comm_allgatherv(gs_ctx* c, const void* sendbuf, char* recvbuf, const uint64_t* counts, size_t row);
// exclusive scan of n u64 (gs_hashset.hip)
gs_status xscan(gs_ctx* c, const uint64_t* in, uint64_t n, uint64_t* out);
// order-preserving compaction of the IDs of two columns (gs_relabel.hip): *ca / *cb = ranks among the
// *V sorted distinct IDs *uniq (device buffers of the ctx, valid until the next relabel)
gs_status relabel_endpoints(gs_ctx* c, const int64_t* a, const int64_t* b, uint64_t n, const int64_t** ca,
                            const int64_t** cb, const int64_t** uniq, uint64_t* V);
// local compact columns ca / cb (ranks among the nloc sorted distinct ids loc) -> ranks among the ng
// sorted distinct ids G (loc ⊂ G), in place; map: nloc u32 of scratch
gs_status relabel_to_global(gs_ctx* c, const int64_t* loc, uint64_t nloc, const int64_t* G, uint64_t ng, uint32_t* map,
                            int64_t* ca, int64_t* cb, uint64_t n);
// Bucket path (gs_bucket.hip) for the associative built-ins; GS_EUNSUPPORTED (no message) when the
// window or op does not fit it and the caller should take the sort path.  keys/vals: device.
gs_status bucket_reduce(gs_ctx* c, const int64_t* src, const int64_t* dst, const void* val, uint64_t n, int dir,
                        int op, int dtype, bool has_init, const void* init, int64_t* keys, void* vals, uint64_t* U);
gs_status bucket_degree_max(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, int dir, int64_t init_max,
                            int64_t* keys, int64_t* deg, int64_t* mx, uint64_t* U);
// Wait on the host for the ctx stream: poll a completion event for up to 2 ms, then block.  The host
// reads small results mid-window (vertex range, output count); a blocking wait's wake-up latency is
// paid twice per window otherwise.
gs_status host_wait(gs_ctx* c);
// at the start of a public call: drain the thread's sticky HIP error (a failed call of the host process,
// e.g. torch's, would otherwise surface at our next post-launch hipGetLastError), select the device and
// clear the look-back timeout word
gs_status begin_call(gs_ctx* c);
// after bucket_accumulate: the read-back block in host_small[0..7] (a host-memory spin when the window's
// read-back went through rb_host, else host_wait)
gs_status bucket_wait(gs_ctx* c);
// milliseconds between two recorded events; 0 (and no sticky error left behind) when either was not
// recorded on this call's path -- hipEventElapsedTime's hipErrorInvalidHandle must not reach the next
// launch check as "invalid resource handle"
inline float event_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();
    ms = 0.f;
  }
  return ms;
}

// a stage-time event (gs_set_timing): recorded at GS_TIMING_STAGES, and at GS_TIMING_DOMINANT only when
// `dominant` (the bucket path's scatter / accumulate brackets); never at GS_TIMING_OFF
inline void stage_event(gs_ctx* c, hipEvent_t e, bool dominant = false) {
  if (c->timing == GS_TIMING_STAGES || (dominant && c->timing == GS_TIMING_DOMINANT)) hipEventRecord(e, c->stream);
}
// a dominant kernel (the bucket path's scatter and accumulate): at GS_TIMING_DOMINANT its start / stop
// events ride on its own dispatch (hipExtLaunchKernelGGL) -- an event record of its own is a packet
// between two kernels, ~5-10 us of idle GPU each; otherwise a plain launch, bracketed by the caller's
// stage_event records at GS_TIMING_STAGES
template <typename F, typename... A>
inline void launch_dominant(gs_ctx* c, hipEvent_t e0, hipEvent_t e1, F k, dim3 grid, dim3 block, A... args) {
  if (c->timing == GS_TIMING_DOMINANT) hipExtLaunchKernelGGL(k, grid, block, 0, c->stream, e0, e1, 0, args...);
  else hipLaunchKernelGGL(k, grid, block, 0, c->stream, args...);
}

// k_keyinfo over both columns (ALL): mask at SM_MASK, byte histograms at SM_HIST
gs_status launch_keyinfo_all(gs_ctx* c, const int64_t* src, const int64_t* dst, uint64_t n, bool mask_only = false);

// Stage a batch on the device (copies host columns into ctx buffers); returns device pointers.
gs_status stage_batch(gs_ctx* c, const gs_edge_batch* b, const int64_t** src, const int64_t** dst,
                      const void** val, bool need_val);

// floor(W * q / P) for q <= P without the 64-bit overflow of W * q (equal-work split points)
__host__ __device__ inline unsigned long long frac_share(unsigned long long W, unsigned long long q, unsigned long long P) {
  return (W / P) * q + (W % P) * q / P;
}

inline size_t dtype_bytes(int dt) { return (dt == GS_I32 || dt == GS_F32) ? 4 : (dt == GS_NONE ? 0 : 8); }

}  // namespace gs
