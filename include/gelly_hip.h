/*
 * gelly_hip.h — C ABI of libgellyhip.so, the MI355X (gfx950) engine behind the
 * per-tumbling-window neighbourhood path of gelly-streaming.
 *
 * The reference (Ren91/gelly-streaming, Java on Flink 1.0.3) has no native code.
 * Its per-window path is
 *
 *   SimpleEdgeStream.slice(Time[, EdgeDirection])      SimpleEdgeStream.java:139-171
 *     -> GraphWindowStream.reduceOnEdges(EdgesReduce)    GraphWindowStream.java:101-121
 *     -> GraphWindowStream.foldNeighbors(init, EdgesFold) GraphWindowStream.java:62-87
 *     -> GraphWindowStream.applyOnNeighbors(EdgesApply)  GraphWindowStream.java:130-182
 *   and the WindowTriangles example                     example/WindowTriangles.java:51-140
 *
 * Flink runs those per (vertex, window) record by record.  This ABI takes ONE
 * tumbling window as a columnar (SoA) edge batch and returns the per-vertex
 * results for the whole window; the Java window-buffer operator described in
 * INTEGRATION.md calls it once per window end.  Every entry point below names
 * the reference interface it replaces.
 *
 * Conventions
 *  - Plain C: no C++ or torch types cross this boundary.
 *  - Nothing throws or aborts across the ABI.  Every call returns gs_status;
 *    gs_last_error(ctx) holds the message of the last failure on that ctx.
 *    The Java wrapper maps a non-zero status to an Exception, matching the
 *    `throws Exception` of EdgesReduce.java:43 / EdgesFold.java:47 / EdgesApply.java:47.
 *  - Buffers are caller-owned.  `mem` says whether a pointer is host memory
 *    (pageable or from gs_alloc_pinned) or device memory (HBM) on ctx's device.
 *    No pointer is retained after a call returns.
 *  - A ctx is not re-entrant: one ctx per Flink subtask thread.  Distinct ctxs
 *    are independent (own stream, own workspace).
 *  - Keys are Java Long vertex IDs (int64).  Output keys are ascending.
 */
#ifndef GELLY_HIP_H
#define GELLY_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: gs_tri_dist_route lost two parameters (gs_tri_dist_orient runs first), the JNI candidates
 *    natives changed return types, and the in-process comm group (gs_comm_group_*),
 *    gs_candidates_begin_part and gs_device_count were added. */
#define GS_ABI_VERSION 2

#if defined(__GNUC__) || defined(__clang__)
#define GS_API __attribute__((visibility("default")))
#else
#define GS_API
#endif

typedef int32_t gs_status;
enum {
  GS_OK = 0,
  GS_EINVAL = -1,       /* bad argument (null pointer, unknown enum, n too large)          */
  GS_ECAPACITY = -2,    /* output capacity too small; *n_out holds the size needed          */
  GS_EDEVICE = -3,      /* HIP runtime / kernel failure                                     */
  GS_ECOMM = -4,        /* collective failure (multi-GPU)                                   */
  GS_ENOMEM = -5,       /* device or pinned allocation failed                               */
  GS_EUNSUPPORTED = -6, /* op/dtype combination not offered by the engine                   */
  GS_EAGAIN = -7        /* gs_stream_poll: no window result ready (non-blocking poll)        */
};

/* org.apache.flink.graph.EdgeDirection, same ordinals (IN, OUT, ALL).
 * OUT: key = src, neighbour = dst            (SimpleEdgeStream.java:160-162)
 * IN : key = dst, neighbour = src (reverse)  (SimpleEdgeStream.java:157-159, 332-341)
 * ALL: both records, e then e.reverse(), in that arrival order (SimpleEdgeStream.java:163-167, 354-365) */
typedef enum gs_dir { GS_DIR_IN = 0, GS_DIR_OUT = 1, GS_DIR_ALL = 2 } gs_dir;

/* Built-in associative reducers that replace a user EdgesReduce / EdgesFold lambda.
 * SUM/MIN/MAX fold the edge values of a vertex in its window (Java semantics:
 * two's-complement wrap for I32/I64, Math.min/Math.max for floats, float sums
 * within 1e-5 relative of the arrival-order fold).  COUNT yields the number of
 * incident edge records (I64) and ignores values. */
typedef enum gs_op { GS_OP_SUM = 0, GS_OP_MIN = 1, GS_OP_MAX = 2, GS_OP_COUNT = 3 } gs_op;

/* Edge value type EV: Integer, Long, Float, Double, or NullValue (GS_NONE). */
typedef enum gs_dtype { GS_I32 = 0, GS_I64 = 1, GS_F32 = 2, GS_F64 = 3, GS_NONE = 4 } gs_dtype;

typedef enum gs_mem { GS_MEM_HOST = 0, GS_MEM_DEVICE = 1 } gs_mem;

typedef struct gs_ctx gs_ctx;

/* gs_config.flags */
#define GS_FLAG_SORT_ONLY 1u   /* reduce / fold: always take the full LSD sort + reduce-by-key path */
#define GS_FLAG_BK_ONESWEEP 2u /* bucket path: partition with 1-2 LSD passes instead of the one-pass
                                  direct scatter (A/B measurement; same results)                   */
#define GS_FLAG_NO_PACK 4u     /* bucket path: integer SUM/MIN/MAX keep 8-byte partitioned values
                                  instead of 4-byte packed records (A/B measurement; same results)  */
#define GS_FLAG_TEST_TINY_TABLES 8u /* TEST ONLY: triangle counting sizes its LDS hash sets at one
                                  bucket, so sets overflow and the call must fail with GS_EDEVICE   */
#define GS_FLAG_NO_SPEC 16u    /* bucket path: no speculative partition (packed windows always count
                                  per-tile bucket histograms first; A/B measurement; same results)  */
#define GS_FLAG_TEST_FORCE_EXCHANGE 32u /* TEST ONLY: gs_window_*_dist on a one-rank communicator still
                                  runs the owner partition, the exchange (to itself) and the merge   */
#define GS_FLAG_ASYNC_OUTPUT 64u /* gs_window_reduce / gs_window_fold / gs_window_fold_degree_max with
                                  DEVICE outputs (GS_MEM_DEVICE, capacity >= the window's records):
                                  the call returns once the window's sizes are known (*n_out), while
                                  the last kernel may still be writing the outputs; they are complete
                                  in the order of the ctx's stream (gs_set_stream), so a caller that
                                  reads them on that stream -- or after gs_synchronize -- needs no
                                  wait.  Host outputs and every other entry point are unchanged.
                                  Default (0): every call returns with its outputs complete.        */

typedef struct gs_config {
  int32_t device;          /* HIP device ordinal                                           */
  uint32_t flags;          /* GS_FLAG_* (0 = defaults)                                     */
  uint64_t reserve_edges;  /* pre-size the workspace for windows of this many edges (0 = lazy) */
} gs_config;

/* One tumbling window's edges, structure-of-arrays: Edge<Long, EV> = Tuple3(f0 src, f1 dst, f2 value).
 * `val` may be NULL when val_dtype == GS_NONE (NullValue edges, e.g. WindowTriangles.java:185). */
typedef struct gs_edge_batch {
  const int64_t* src;
  const int64_t* dst;
  const void* val;
  uint64_t n;              /* edges in the window (before direction expansion)             */
  int32_t val_dtype;       /* gs_dtype                                                     */
  int32_t mem;             /* gs_mem of src/dst/val                                        */
  int64_t window_end_ms;   /* TimeWindow end; results carry end-1 (maxTimestamp)          */
} gs_edge_batch;

/* Per-vertex output: Tuple2<K, EV>(vertex, value) as emitted by reduceOnEdges' project(0, 2). */
typedef struct gs_vertex_out {
  int64_t* keys;           /* [capacity] ascending vertex IDs                              */
  void* vals;              /* [capacity] values (batch dtype; I64 for COUNT)               */
  uint64_t capacity;
  uint64_t* n_out;         /* host pointer: number of vertices written / needed           */
  int32_t mem;             /* gs_mem of keys/vals                                          */
  int32_t reserved;
} gs_vertex_out;

/* Degree / max-neighbour fold output: (vertex, degree, max neighbour ID). */
typedef struct gs_degree_out {
  int64_t* keys;
  int64_t* degree;
  int64_t* max_neighbor;
  uint64_t capacity;
  uint64_t* n_out;
  int32_t mem;
  int32_t reserved;
} gs_degree_out;

/* Grouped neighbourhoods of one window (CSR), the input EdgesWindowFunction.apply
 * hands to a user EdgesApply (GraphWindowStream.java:144-175): for vertex u,
 * neighbours/values [offsets[u], offsets[u+1]) in arrival order, duplicates kept. */
typedef struct gs_csr_out {
  int64_t* keys;           /* [capacity_vertices]                                          */
  uint64_t* offsets;       /* [capacity_vertices + 1]                                      */
  int64_t* neighbors;      /* [capacity_records]                                           */
  void* vals;              /* [capacity_records] or NULL                                   */
  uint64_t capacity_vertices;
  uint64_t capacity_records;
  uint64_t* n_vertices;
  uint64_t* n_records;
  int32_t mem;
  int32_t reserved;
} gs_csr_out;

/* Candidate records of WindowTriangles.GenerateCandidateEdges (WindowTriangles.java:83-116):
 * Tuple3<Long, Long, Boolean>(a, b, isCandidate).  The flag is stored as one byte. */
typedef struct gs_pair_out {
  int64_t* a;
  int64_t* b;
  uint8_t* is_candidate;
  uint64_t capacity;
  uint64_t* n_out;         /* records written / needed (two-phase: call with capacity 0 to size) */
  int32_t mem;
  int32_t reserved;
} gs_pair_out;

/* ---- lifecycle ---------------------------------------------------------------------- */
GS_API int32_t gs_abi_version(void);
/* HIP devices visible to this process (*n); a Flink job sizes its GPU operators' parallelism by it and
 * puts subtask i on device i % n. */
GS_API gs_status gs_device_count(int32_t* n);
GS_API gs_status gs_create(const gs_config* cfg, gs_ctx** out);
GS_API void gs_destroy(gs_ctx* ctx);
GS_API const char* gs_last_error(const gs_ctx* ctx);
/* Run this ctx's work on an existing hipStream_t (e.g. torch.cuda.current_stream()); NULL = the
 * device's default stream.  gs_create gives each ctx a stream of its own until this is called. */
GS_API gs_status gs_set_stream(gs_ctx* ctx, void* hip_stream);
GS_API gs_status gs_synchronize(gs_ctx* ctx);
GS_API void* gs_alloc_pinned(size_t bytes);
GS_API void gs_free_pinned(void* p);

/* ---- per-window neighbourhood operators ------------------------------------------- */

/* Replaces GraphWindowStream.reduceOnEdges(EdgesReduce) (GraphWindowStream.java:101-121)
 * with a built-in reducer: one (vertex, reduced value) per vertex with >=1 incident record. */
GS_API gs_status gs_window_reduce(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir, int32_t op,
                           gs_vertex_out* out);

/* Replaces GraphWindowStream.foldNeighbors(initialValue, EdgesFold) (GraphWindowStream.java:62-87)
 * for an associative fold over edge values: acc = op(... op(op(init, v1), v2) ...).
 * `init` points to one host value of the batch dtype (I64 for COUNT). */
GS_API gs_status gs_window_fold(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir, int32_t op,
                         const void* init, gs_vertex_out* out);

/* Replaces foldNeighbors with the degree / max-neighbour fold of TestSlice.java:233-239's shape:
 * acc.f0 = vertex, acc.f1 += 1, acc.f2 = max(acc.f2, neighbour), starting from (v, 0, init_max). */
GS_API gs_status gs_window_fold_degree_max(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir,
                                    int64_t init_max, gs_degree_out* out);

/* Windows of any size for reduce / fold / the degree fold (SimpleEdgeStream.java:159-167: keyBy puts
 * no cap on a window).  One pass of the engine takes at most max_records direction-expanded records
 * (default and upper bound 2^32 - 1: 32-bit record positions); a host batch is also cut so that each
 * pass's columns and workspace fit the device's free HBM.  A larger window runs in chunks of whole
 * edges, each reduced to per-vertex partials (gs_window_reduce_partials' local half) and merged into
 * a running set of partials (gs_merge_partials; foldNeighbors' init applied once, at the end).
 * Integer results are bit-exact; float sums stay within the API's 1e-5 relative tolerance.  Tests
 * set a small max_records to force chunking; 0 restores the default. */
GS_API gs_status gs_set_max_window_records(gs_ctx* ctx, uint64_t max_records);

/* The grouping half of applyOnNeighbors (GraphWindowStream.java:130-175): the window's
 * neighbourhoods as a CSR in arrival order, for a host-side user EdgesApply to iterate. */
GS_API gs_status gs_window_csr(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir, gs_csr_out* out);

/* applyOnNeighbors(GenerateCandidateEdges) on slice(ALL) (WindowTriangles.java:62-63, 83-116).
 * Records per vertex v: (v, t, false) per neighbour record in arrival order, then the candidate
 * pairs (ids[i], ids[j], true), i < len-1, j >= i, ids[i] > v, ids[j] > v, where ids is v's
 * neighbour set in java.util.HashSet (JDK 8+) iteration order.  Vertices ascend.  A neighbour set
 * whose insertion ever fills a HashMap bin to 9 nodes is simulated exactly (treeifyBin's resize below
 * capacity 64, red-black tree bins above); out->reserved reports it: bit 0 = a tree bin, bit 1 = a
 * collision resize. */
GS_API gs_status gs_window_candidates(gs_ctx* ctx, const gs_edge_batch* batch, gs_pair_out* out);

/* The same records in chunks, for consumers that stream them (a window's output is O(sum d^2): a 1e8-edge
 * R-MAT scale-23 window emits 1.6e11 records, 2.7 TB).  gs_candidates_begin builds the window's
 * HashSet-ordered neighbour sets once and returns the number of records gs_window_candidates would
 * write; each gs_candidates_next then writes the next min(out->capacity, remaining) records, in
 * gs_window_candidates' order (*first_record = the global position of the chunk's first record; a
 * vertex's records may straddle chunks), and sets *done after the last.  With device output
 * (out->mem == GS_MEM_DEVICE) the chunk is only enqueued on the ctx stream: the call returns without
 * waiting for it, and the records are there for work ordered after it on that stream (gs_set_stream) or
 * after gs_synchronize; host output returns with the records copied.  The session lives in the ctx
 * workspace: any other entry point called on the ctx ends it (gs_candidates_next then fails with
 * GS_EINVAL). */
GS_API gs_status gs_candidates_begin(gs_ctx* ctx, const gs_edge_batch* batch, uint64_t* total_records,
                                     uint32_t* jdk_flags);
GS_API gs_status gs_candidates_next(gs_ctx* ctx, gs_pair_out* out, uint64_t* first_record, int32_t* done);
/* gs_candidates_next with the ids as 32-bit columns: a[i] = *id_base + a32[i] (likewise b), *id_base = the
 * window's smallest id, the same records in the same order at 9 bytes instead of 17 (no reference
 * counterpart: a consumer on the device that takes compact ids, e.g. WindowTriangles' counting stage,
 * reads half the bytes).  GS_EUNSUPPORTED when the window's ids span more than 2^32 values. */
typedef struct gs_pair_out_u32 {
  uint32_t* a;
  uint32_t* b;
  uint8_t* is_candidate;
  uint64_t capacity;
  uint64_t* n_out;
  int32_t mem;
  int32_t reserved;
} gs_pair_out_u32;
GS_API gs_status gs_candidates_next_u32(gs_ctx* ctx, gs_pair_out_u32* out, int64_t* id_base, uint64_t* first_record,
                                        int32_t* done);
/* A session over one part of a window split by owner (the chunked gs_window_candidates_part, below):
 * only the vertices v with gs_owner_of(v, nparts) == part emit; the batch holds every edge incident to
 * them in stream order (a Flink subtask behind an owner partitioner: GpuCandidatesOperator).
 * gs_candidates_vertex_range is not offered on such a session (GS_EUNSUPPORTED). */
GS_API gs_status gs_candidates_begin_part(gs_ctx* ctx, const gs_edge_batch* batch, uint32_t nparts, uint32_t part,
                                          uint64_t* total_records, uint32_t* jdk_flags);
/* Random access into the session (no reference counterpart: a consumer that restarts mid-window, or
 * several consumers that split the output, e.g. one per downstream pair-keyed subtask).
 * gs_candidates_seek moves the cursor: the next gs_candidates_next starts at `record` (<= the total).
 * gs_candidates_vertex_range gives the block of one vertex: its records (edge records, then its pair rows)
 * are [*first_record, *first_record + *records); a vertex absent from the window has *records = 0 and
 * *first_record = where it would start.  Neither ends the session. */
GS_API gs_status gs_candidates_seek(gs_ctx* ctx, uint64_t record);
GS_API gs_status gs_candidates_vertex_range(gs_ctx* ctx, int64_t vertex, uint64_t* first_record, uint64_t* records);

/* Multi-GPU candidates (partition by owner(v), no exchange of pairs): only the vertices
 * v with gs_owner_of(v, nparts) == part emit, with exactly the records gs_window_candidates gives them
 * over the same batch.  The batch must hold every edge incident to those vertices, in stream order
 * (distributed.candidates_window routes each edge to the owners of its two endpoints, rank order
 * = stream order); the union over parts is the whole window's output. */
GS_API gs_status gs_window_candidates_part(gs_ctx* ctx, const gs_edge_batch* batch, uint32_t nparts,
                                           uint32_t part, gs_pair_out* out);

/* The whole WindowTriangles pipeline for one window (WindowTriangles.java:61-66):
 * slice(ALL) -> GenerateCandidateEdges -> keyBy(0,1) CountTriangles -> timeWindowAll sum(0).
 * *count is the exact 64-bit count; *count_ref_wrapped is the Integer the reference emits
 * (mod 2^32 as signed).  *has_output = 0 when the window has no edge (no record is emitted). */
GS_API gs_status gs_window_triangles(gs_ctx* ctx, const gs_edge_batch* batch, uint64_t* count,
                              int32_t* count_ref_wrapped, int32_t* has_output);

/* One share of WindowTriangles for a caller that holds the whole window: part `part` of `nparts`
 * counts the triangles u -> v -> w whose first vertex u lies in the part's range of the degree order,
 * the ranges cut at equal shares of the work sum_u d+(u)(d+(u)+1)/2 (plus the self-pair term on part
 * 0); the parts sum (an all-reduce) to gs_window_triangles' count. */
GS_API gs_status gs_window_triangles_part(gs_ctx* ctx, const gs_edge_batch* batch, uint32_t part,
                                          uint32_t nparts, uint64_t* partial_count);

/* ---- WindowTriangles over a window split across ranks ------------------------
 * Every rank holds only its own records of the window (the reference's subtasks after slice()).
 * The steps, with the collective the caller runs after each (torch.distributed, the JVM's, or the
 * ctx communicator: gs_window_triangles_dist does all of them over RCCL or the comm group):
 *   1. gs_tri_dist_range     local [min, max] id            -> all-reduce min of [0], max of [1]
 *   2. gs_tri_dist_degrees   local raw degrees deg[V]       -> all-reduce (sum, u32) of deg
 *      (deg == NULL: *V only, to size the buffer; V = 2^bits of the common id span, <= 2^28: a window
 *      whose ids span more is relabeled to the whole window's compact ids first, as gs_window_triangles_dist
 *      does inside and distributed.relabel_window shows for a caller)
 *   3a. gs_tri_dist_orient   oriented edges (u << B | v, u < v in the degree order), kept in the ctx
 *      for 3b; dout[V] = their count per u (raw, duplicates included); *loops = local self-loops
 *                                                           -> all-reduce (sum, u32) of dout; of loops
 *   3b. gs_tri_dist_route    owner ranges of the degree order cut at equal shares of the raw work
 *      dout(dout+1)/2 (the same on every rank, so a rank builds nearly the rows it will count); the keys
 *      grouped by owner(u) into keys_out, counts[p] rows for rank p   -> all-to-all of the rows
 *   4. gs_tri_dist_build     the received rows deduplicated into this rank's out-lists: nbr_out[m]
 *      (targets, sorted per u) and dplus_out[V] (d+(u) of the owned u, 0 elsewhere)
 *                                                           -> all-reduce (sum, u32) of dplus
 *      Boundary adjacency (north_star: "all-gathers boundary adjacency"; not every row): the count share
 *      of a rank reads the rows of its equal-work range C of the degree order and the rows of their
 *      targets; it built the rows of its route range R.
 *   4a. gs_tri_dist_plan     from the global dplus: send_elems[p] = elements of this rank's rows that
 *      rank p counts, recv_elems[p] = elements of the rows this rank counts that rank p built; *M =
 *      the window's unique edges                            -> all-to-all of nbr (those sizes) = crows
 *   4b. gs_tri_dist_need     the targets of crows held in neither C nor R, ascending (so grouped by
 *      owner) into req_out[capacity]; per owner: ids and row elements
 *                                                           -> all-to-all of (ids, elements) per peer,
 *                                                              then of the ids (req_counts sizes)
 *   4c. gs_tri_dist_serve    the rows of the ids other ranks requested (req_in grouped by requester,
 *      counts_in[p] ids from rank p) packed into rows_out[capacity]; send_elems[p] per requester
 *                                                           -> all-to-all of the rows (send_elems / the
 *                                                              req_elems of 4b)
 *   4d. gs_tri_dist_assemble nbr, crows and the received rows at their window positions: full_out[M]
 *      holds every row this rank's count share reads (the rest is zero)
 *   5. gs_tri_dist_count     this rank's share (part = rank, nparts = ranks) of the count over
 *      full_out                                             -> all-reduce (sum) of the counts
 *   6. windows with self-loops (summed loops > 0): the self-pair term needs whole neighbour sets, so
 *      the records are gathered and rank 0 adds gs_window_triangles_selfpair of the whole window.
 * Exchanged per window: 4 B per id (deg, dout, dplus), 8 B per local record (step 3) and 4 B per element of the
 * boundary rows a rank reads but did not build (step 4; R-MAT s22-s24: 0.16-0.47 of the all-gathered
 * adjacency at 2-8 ranks).  Buffers: deg, keys_out, keys, nbr_out, dplus_out, crows,
 * req_out, req_in, rows_out, rows_in, full_out, nbr, dplus are device memory; counts and sizes host. */
GS_API gs_status gs_tri_dist_range(gs_ctx* ctx, const gs_edge_batch* local, int64_t* minmax /* [2] */);
GS_API gs_status gs_tri_dist_degrees(gs_ctx* ctx, const gs_edge_batch* local, int64_t id_min, int64_t id_max,
                                     uint32_t* deg, uint64_t* V);
GS_API gs_status gs_tri_dist_orient(gs_ctx* ctx, const gs_edge_batch* local, const uint32_t* deg,
                                    uint32_t* dout /* [V] */, uint64_t* loops /* host */);
GS_API gs_status gs_tri_dist_route(gs_ctx* ctx, const uint32_t* dout, uint32_t nparts,
                                   uint64_t* keys_out /* [local n] */, uint64_t* counts /* host [nparts] */);
GS_API gs_status gs_tri_dist_build(gs_ctx* ctx, const uint64_t* keys, uint64_t n, uint32_t* nbr_out /* [n] */,
                                   uint32_t* dplus_out /* [V] */, uint64_t* m_out);
GS_API gs_status gs_tri_dist_plan(gs_ctx* ctx, const uint32_t* dplus, uint32_t part, uint32_t nparts,
                                  uint64_t* send_elems /* host [nparts] */, uint64_t* recv_elems /* host [nparts] */,
                                  uint64_t* M);
GS_API gs_status gs_tri_dist_need(gs_ctx* ctx, const uint32_t* crows, uint32_t* req_out, uint64_t capacity,
                                  uint64_t* req_counts /* host [nparts] */, uint64_t* req_elems /* host [nparts] */,
                                  uint64_t* nreq);
GS_API gs_status gs_tri_dist_serve(gs_ctx* ctx, const uint32_t* nbr, const uint32_t* req_in,
                                   const uint64_t* counts_in /* host [nparts] */, uint32_t* rows_out, uint64_t capacity,
                                   uint64_t* send_elems /* host [nparts] */);
GS_API gs_status gs_tri_dist_assemble(gs_ctx* ctx, const uint32_t* nbr, const uint32_t* crows, const uint32_t* rows_in,
                                      uint32_t* full_out /* [M] */);
GS_API gs_status gs_tri_dist_count(gs_ctx* ctx, const uint32_t* nbr, uint64_t M, const uint32_t* dplus, uint32_t part,
                                   uint32_t nparts, uint64_t* partial_count);
/* The self-pair term alone (WindowTriangles.java:105: (x, x) candidates matched by a self-loop on x)
 * of a whole window. */
GS_API gs_status gs_window_triangles_selfpair(gs_ctx* ctx, const gs_edge_batch* window, uint64_t* S);
/* Steps 1-6 with the ctx communicator (gs_comm_init / gs_comm_init_group); every rank gets the
 * window's count. */
GS_API gs_status gs_window_triangles_dist(gs_ctx* ctx, const gs_edge_batch* local, uint64_t* count,
                                          int32_t* count_ref_wrapped, int32_t* has_output);

/* Two-phase output without recomputation: after a window call returned GS_ECAPACITY (with the needed
 * size in *n_out) and before the next call on the ctx, deliver the rows it left staged.  Covers
 * gs_window_reduce / gs_window_fold / gs_merge_partials / gs_window_reduce_dist (gs_fetch_last_output)
 * and the degree / max variants (gs_fetch_last_degree_output). */
GS_API gs_status gs_fetch_last_output(gs_ctx* ctx, gs_vertex_out* out);
GS_API gs_status gs_fetch_last_degree_output(gs_ctx* ctx, gs_degree_out* out);

/* ---- multi-GPU keyBy (SimpleEdgeStream.java:159-167) ---------------------------------- */
/* A window spread over nparts ranks: every rank pre-reduces its own slice, the per-vertex partials
 * travel to their owner, the owner merges them.  owner(v) = gs_owner_of(v, nparts), a hash of the
 * vertex as Flink's keyBy is (which subtask owns a vertex is not observable in the output).  The
 * exchange between the halves is the caller's (e.g. an all-to-all in torch.distributed or the JVM), or
 * the ctx-owned RCCL communicator (gs_comm_init + gs_window_*_dist). */
GS_API uint32_t gs_owner_of(int64_t vertex, uint32_t nparts);

/* Partials grouped by owner: rows of owner 0, then owner 1, ...; keys ascend within an owner. */
typedef struct gs_partials_out {
  int64_t* keys;           /* [capacity]                                                        */
  void* vals;              /* [capacity] partial values (batch dtype; I64 for COUNT; degrees)   */
  int64_t* vals2;          /* [capacity] degree/max fold: maxima (NULL otherwise)               */
  uint64_t capacity;
  uint64_t* n_out;         /* host: rows written / needed                                       */
  uint64_t* owner_counts;  /* host: [nparts] rows per owner                                     */
  int32_t mem;
  int32_t reserved;
} gs_partials_out;

/* Rows an owner received (any order, any number of rows per vertex). */
typedef struct gs_partial_batch {
  const int64_t* keys;
  const void* vals;
  const int64_t* vals2;    /* degree/max fold: maxima                                           */
  uint64_t n;
  int32_t val_dtype;       /* gs_dtype of vals (I64 for COUNT partials and degrees)             */
  int32_t mem;
} gs_partial_batch;

/* The first half of reduceOnEdges / foldNeighbors across ranks: this rank's slice reduced with `op`
 * (no init; COUNT partials are I64 counts), partitioned by owner on the device. */
GS_API gs_status gs_window_reduce_partials(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir, int32_t op,
                                           uint32_t nparts, gs_partials_out* out);
/* The same for the degree / max-neighbour fold: vals = degrees (I64), vals2 = maxima (no init). */
GS_API gs_status gs_window_fold_degree_max_partials(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir,
                                                    uint32_t nparts, gs_partials_out* out);
/* The second half: merge the partials this owner received with `op` (COUNT partials add up);
 * `init` (NULL for reduceOnEdges) is foldNeighbors' initial value, applied once per vertex. */
GS_API gs_status gs_merge_partials(gs_ctx* ctx, const gs_partial_batch* partials, int32_t op, const void* init,
                                   gs_vertex_out* out);
GS_API gs_status gs_merge_degree_max_partials(gs_ctx* ctx, const gs_partial_batch* partials, int64_t init_max,
                                              gs_degree_out* out);

/* The ctx communicator: every gs_window_*_dist call and gs_comm_allreduce_sum_u64 run over it.  Two
 * kinds, the same collectives and results:
 *  - RCCL (one rank per process and GPU; RCCL is loaded at gs_comm_init time).  Rank 0 calls
 *    gs_comm_unique_id and ships the 128 bytes to every rank out of band; every rank calls gs_comm_init.
 *  - an in-process thread group (one rank per ctx, all ctxs in one process, on one or several GPUs):
 *    gs_comm_group_create once, then gs_comm_init_group(ctx_r, group, r) for every rank r, and each
 *    rank's calls from its own thread (a JVM driving several GPUs without RCCL; the tests run P ranks
 *    on one GPU this way).  The group checks that the ranks enter the same collectives with matching
 *    sizes; a mismatch, a failed copy or a rank missing for GS_COMM_TIMEOUT_MS (env, default 120000)
 *    breaks the group: every rank's call returns GS_ECOMM.  gs_comm_group_destroy drops the creator's
 *    reference; the group lives until every ctx has left it (gs_comm_destroy / gs_destroy).
 * nranks <= GS_COMM_MAX_RANKS. */
#define GS_COMM_MAX_RANKS 64
typedef struct gs_comm_group gs_comm_group;
GS_API gs_status gs_comm_unique_id(void* id128);
GS_API gs_status gs_comm_init(gs_ctx* ctx, int32_t nranks, int32_t rank, const void* id128);
GS_API gs_status gs_comm_group_create(int32_t nranks, gs_comm_group** group);
GS_API void gs_comm_group_destroy(gs_comm_group* group);
GS_API gs_status gs_comm_init_group(gs_ctx* ctx, gs_comm_group* group, int32_t rank);
GS_API gs_status gs_comm_destroy(gs_ctx* ctx);
/* *value = the sum of *value over the communicator's ranks (e.g. per-rank triangle counts). */
GS_API gs_status gs_comm_allreduce_sum_u64(gs_ctx* ctx, uint64_t* value);
/* Partials -> all-to-all (counts, then rows) over the ctx communicator -> merge: `out` receives the
 * vertices this rank owns. */
GS_API gs_status gs_window_reduce_dist(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir, int32_t op,
                                       const void* init, gs_vertex_out* out);
GS_API gs_status gs_window_fold_degree_max_dist(gs_ctx* ctx, const gs_edge_batch* batch, int32_t dir,
                                                int64_t init_max, gs_degree_out* out);

/* ConnectedComponents over a window stream (library/ConnectedComponents.java:56-131 through
 * WindowGraphAggregation.java:47-65): the running DisjointSet state after this window -- the previous
 * state's (vertex, label) rows (NULL or n = 0 for the first window) merged with the window's edges
 * (direction ignored: weakly connected).  out: every vertex seen so far, ascending, with the smallest
 * vertex of its component (I64 labels); the partition is the reference's, the label is canonical (which
 * vertex DisjointSet keeps as root depends on HashMap iteration order).  Feed the output back as `prev`
 * for the next window (transientState = false). */
GS_API gs_status gs_window_components(gs_ctx* ctx, const gs_edge_batch* window, const gs_partial_batch* prev,
                                      gs_vertex_out* out);

/* Candidate records of one window as produced by GenerateCandidateEdges (gs_pair_out layout). */
typedef struct gs_pair_batch {
  const int64_t* a;
  const int64_t* b;
  const uint8_t* is_candidate;   /* Boolean f2: non-zero = true                                  */
  uint64_t n;
  int32_t mem;             /* gs_mem of a/b/is_candidate                                       */
  int32_t reserved;
} gs_pair_batch;

/* Stage 2 of WindowTriangles for callers that keep GenerateCandidateEdges and count downstream:
 * keyBy(0, 1).timeWindow(w).apply(CountTriangles).timeWindowAll(w).sum(0)
 * (WindowTriangles.java:64-66, CountTriangles :119-140).  The records (one window) are grouped by the
 * ordered pair (a, b); a group with at least one edge record (is_candidate = 0) emits its number of
 * candidate records; the all-window sum adds them.  *count = exact sum, *count_ref_wrapped = the
 * Integer the reference emits, *has_output = 0 when no group emits (the reference emits no record),
 * *groups = records CountTriangles emits.  IDs of a and of b must each span < 2^32 (GS_EUNSUPPORTED). */
GS_API gs_status gs_window_count_candidates(gs_ctx* ctx, const gs_pair_batch* pairs, uint64_t* count,
                                            int32_t* count_ref_wrapped, int32_t* has_output, uint64_t* groups);

/* Edge text input of the examples: env.readTextFile(path).map(s.split("\\s") -> Long.parseLong of
 * fields 0..2) (WindowTriangles.java:175-185).  Records end at '\n' (a trailing '\r' is dropped; text
 * after the last '\n' is a record when non-empty); fields are separated by exactly one whitespace
 * char; fields after the third are ignored.  Outputs src, dst, ts (the edge value the example turns
 * into the event time) in record order.  Two-phase: *n_out = records (GS_ECAPACITY when capacity is
 * short).  A record where the reference's map would throw gives GS_EINVAL and its index in
 * *bad_record (~0 otherwise).  text < 4 GiB per call. */
GS_API gs_status gs_parse_edges_text(gs_ctx* ctx, const char* text, uint64_t bytes, int32_t in_mem, int64_t* src,
                                     int64_t* dst, int64_t* ts, uint64_t capacity, int32_t out_mem,
                                     uint64_t* n_out, uint64_t* bad_record);

/* ---- the window-buffer operator: event-time tumbling windows over a record stream -------- */
/* Replaces slice(size[, dir]) -> keyBy(vertex).timeWindow(size) -> the window function for the built-in
 * operators (SimpleEdgeStream.java:153-171, GraphWindowStream.java:49-53, 62-182; Flink 1.0.3
 * TumblingEventTimeWindows + EventTimeTrigger): records are appended with their event timestamps,
 * buffered per window (start = ts - ts % size, Java remainder) in pinned host memory, and a window
 * fires when the watermark reaches end - 1; its result carries the timestamp end - 1.  A fired
 * window's columns are copied to HBM on the operator's own copy stream, so window k+1's copy overlaps
 * window k's kernels.  Results come back in firing order from gs_stream_poll.  Records of a window
 * that already fired: gs_stream_config.late_mode. */
typedef struct gs_stream gs_stream;
enum { GS_STREAM_REDUCE = 0, GS_STREAM_FOLD = 1, GS_STREAM_DEGREE_MAX = 2, GS_STREAM_TRIANGLES = 3 };
enum { GS_WATERMARK_EXPLICIT = 0,    /* gs_stream_watermark only                                   */
       GS_WATERMARK_ASCENDING = 1 }; /* AscendingTimestampExtractor: max timestamp seen - 1        */
enum { GS_STAGE_PINNED = 0, GS_STAGE_DIRECT = 1 };
/* Records of a window that already fired.  GS_LATE_REFIRE (default): Flink 1.0.3's WindowOperator has no
 * lateness check -- the record goes into fresh window state (the fired pane was purged,
 * EventTimeTrigger FIRE_AND_PURGE) and registers a timer at end - 1, already behind the watermark, which
 * fires at the next watermark: the window fires again with only its late records.  GS_LATE_DROP: they
 * are dropped (Flink >= 1.1 with allowedLateness 0).  Both count them in late_records.  No reference
 * fixture covers late records: parity unpinned. */
enum { GS_LATE_REFIRE = 0, GS_LATE_DROP = 1 };

typedef struct gs_stream_config {
  int64_t window_ms;       /* tumbling window size (Time.milliseconds)                          */
  int32_t kind;            /* GS_STREAM_*: reduceOnEdges / foldNeighbors / degree-max / triangles */
  int32_t dir;             /* gs_dir (GS_STREAM_TRIANGLES: slice(ALL) regardless)               */
  int32_t op;              /* gs_op for REDUCE / FOLD                                           */
  int32_t val_dtype;       /* gs_dtype of appended values (GS_NONE: no value column)            */
  int32_t watermark_mode;  /* GS_WATERMARK_*                                                    */
  int32_t staging;         /* GS_STAGE_PINNED: records copied into pinned window buffers, the
                              window's H2D at firing; GS_STAGE_DIRECT: each append is copied straight
                              into the window's device columns on the copy stream -- by DMA from the
                              caller's columns when they are pinned (gs_alloc_pinned; the append
                              returns once the DMA has read them), else through HIP's pageable staging */
  const void* init;        /* FOLD: one value of the result dtype (copied at create)           */
  int64_t init_max;        /* DEGREE_MAX: initial maximum                                       */
  uint64_t max_window_edges; /* expected window size: pinned / device buffers are sized for it  */
  int32_t late_mode;       /* GS_LATE_*                                                         */
  int32_t reserved;
} gs_stream_config;

typedef struct gs_window_result {
  int64_t window_start, window_end;
  int64_t max_timestamp;   /* end - 1: the timestamp of every record this window emits          */
  uint64_t edges;          /* records the window held                                           */
  uint64_t n_vertices;     /* rows in keys / vals / vals2                                       */
  const int64_t* keys;     /* pinned host rows, valid until the next gs_stream_poll             */
  const void* vals;        /* REDUCE / FOLD values; DEGREE_MAX degrees (I64)                    */
  const int64_t* vals2;    /* DEGREE_MAX maxima                                                 */
  uint64_t triangles;      /* TRIANGLES: exact count                                            */
  int32_t triangles_ref;   /* TRIANGLES: the Integer the reference emits                        */
  int32_t has_output;      /* 0: the reference emits no record for this window                  */
  double latency_ms;       /* host time from the window's firing to its result                  */
} gs_window_result;

typedef struct gs_stream_stats_t {
  int64_t watermark;
  uint64_t open_windows, fired_windows, pending_windows, late_records, edges_fired;
} gs_stream_stats_t;

GS_API gs_status gs_stream_create(gs_ctx* ctx, const gs_stream_config* cfg, gs_stream** out);
GS_API void gs_stream_destroy(gs_stream* stream);
/* Append n records in arrival order (host columns; `val` NULL for NullValue streams). */
GS_API gs_status gs_stream_append(gs_stream* stream, const int64_t* src, const int64_t* dst, const void* val,
                                  const int64_t* ts, uint64_t n);
GS_API gs_status gs_stream_watermark(gs_stream* stream, int64_t watermark);
/* End of a finite source: watermark Long.MAX_VALUE, every open window fires. */
GS_API gs_status gs_stream_flush(gs_stream* stream);
/* The next window result in firing order; GS_EAGAIN when none is ready (wait = 0). */
GS_API gs_status gs_stream_poll(gs_stream* stream, int32_t wait, gs_window_result* out);
GS_API gs_status gs_stream_stats(const gs_stream* stream, gs_stream_stats_t* out);

/* ---- synthetic streams (bit-identical to oracle/gs_oracle.c) ------------------------ */
/* R-MAT: 2^scale vertices, probabilities a, b, c (d = 1-a-b-c) as 32-bit fixed point,
 * optional seeded vertex permutation, optional self-loop removal (rewired, count kept). */
GS_API gs_status gs_generate_rmat(gs_ctx* ctx, int32_t scale, uint64_t n, uint64_t seed, uint32_t a_fx,
                           uint32_t b_fx, uint32_t c_fx, int32_t permute, int32_t no_self_loops,
                           uint64_t first_edge, int64_t* src_dev, int64_t* dst_dev);
/* Uniform: src, dst in [0, V), dst != src. */
GS_API gs_status gs_generate_uniform(gs_ctx* ctx, uint64_t num_vertices, uint64_t n, uint64_t seed,
                              uint64_t first_edge, int64_t* src_dev, int64_t* dst_dev);
/* Zipf(exponent) sources over [0, V) (P(k) ~ (k+1)^-exponent: hubs at the lowest IDs), uniform
 * destinations — the power-law source stream of BASELINE config C3 (V = 2^24, exponent 1.1). */
GS_API gs_status gs_generate_zipf(gs_ctx* ctx, uint64_t num_vertices, double exponent, uint64_t n, uint64_t seed,
                                  uint64_t first_edge, int64_t* src_dev, int64_t* dst_dev);
/* Edge values: I64 = splitmix64(seed, i) & 0xFFFF; F64 = top 53 bits / 2^53; I32/F32 likewise. */
GS_API gs_status gs_generate_values(gs_ctx* ctx, uint64_t n, uint64_t seed, uint64_t first_edge,
                             int32_t dtype, void* val_dev);

/* ---- instrumentation ----------------------------------------------------------------- */
/* Wall time (ms, device events on ctx's stream) of each stage of the last window call. */
typedef struct gs_stage_times {
  float keyinfo_ms, sort_ms, reduce_ms, total_ms;
  uint32_t sort_passes, key_bits;
  uint64_t records, vertices;
  float pass_ms[8];        /* each onesweep launch (device events around the launch)         */
  uint32_t key_bytes, payload_bytes;  /* sorted key / payload widths                          */
  uint64_t partials;       /* (vertex, partial) pairs left by the fused last pass               */
  uint32_t fused_last;     /* 1: pass_ms[sort_passes] is the last pass fused with the combine   */
  uint32_t path;           /* 0: LSD sort + reduce-by-key;
                              1: bucket path, onesweep partition (pass_ms[0..sort_passes) = LSD
                                 passes, then accumulate, merge, emit; partials = work items);
                              2: bucket path, direct partition (keyinfo_ms = per-tile histogram,
                                 pass_ms[0..4] = offset scans, scatter, accumulate, merge, emit);
                              3: window triangles (pass_ms[0..4] = symmetric keys + sort, unique,
                                 rows + orientation, light count, heavy count; records = unique
                                 adjacency entries, vertices = vertices with edges, partials = hash
                                 probes of the counting step, sort_passes = LSD passes)          */
  uint32_t packed;         /* path 2: 1 = 4-byte packed partition records (k_dp_scatter_pack)    */
  uint32_t speculative;    /* path 2: 0 = per-tile histogram + offsets (k_dp_hist);
                              1 = speculative partition (regions from the previous window's counts,
                                  runs reserved with atomics: keyinfo_ms = regions, pass_ms[0] = 0);
                              2 = speculative partition missed, window rerun through k_dp_hist   */
  uint64_t escapes;        /* path 2, packed: values stored in full (outside [0, 0xFFFF));
                              path 3: sum over the oriented edges u -> v of d+(u) + d+(v), the list
                                 entries a per-edge merge intersection would read (a roofline term)   */
} gs_stage_times;
GS_API gs_status gs_last_stage_times(const gs_ctx* ctx, gs_stage_times* out);
/* Which device events a window records for gs_last_stage_times (diagnostics; replaces nothing in the
 * reference).  GS_TIMING_STAGES (the default): every stage of every path.  GS_TIMING_DOMINANT: on the
 * bucket path (path 2) only the partition scatter and the accumulate (pass_ms[1], pass_ms[2], from
 * events carried by those two kernels' own dispatches; every other time reads 0) -- each separate event
 * record costs the stream a few microseconds, ~30 us per C2 window at the default.  GS_TIMING_OFF: none on the bucket path.  path / packed /
 * speculative / escapes and the counts stay valid at every level. */
#define GS_TIMING_OFF 0
#define GS_TIMING_DOMINANT 1
#define GS_TIMING_STAGES 2
GS_API gs_status gs_set_timing(gs_ctx* ctx, int32_t level);

#ifdef __cplusplus
}
#endif
#endif /* GELLY_HIP_H */
