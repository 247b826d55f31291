// gs_comm.hip — the ctx communicator behind the multi-rank window steps.
//
// The split-window orchestrations (gs_window_reduce_dist / _fold_degree_max_dist in gs_dist.hip,
// gs_window_triangles_dist in gs_triangles.hip) use five collectives only: an in-place all-reduce, a
// fixed-size all-to-all, a grouped exchange of owner-grouped rows, an all-gather of variable-size rows,
// and the status agreement built on the all-reduce.  Two backends implement them:
//
//   RCCL (gs_comm_init)         one rank per process and GPU, the production path over xGMI; librccl is
//                               resolved with dlopen at gs_comm_init, so the library has no link
//                               dependency on it.
//   thread group                one rank per ctx, every ctx in THIS process (gs_comm_group_create +
//   (gs_comm_init_group)        gs_comm_init_group): each rank is a caller thread; a collective is a host
//                               barrier, device copies that pull the peers' buffers (same or different
//                               GPUs: hipMemcpyDefault over the unified address space) and a second
//                               barrier before any rank may reuse its buffers.  This is how one process
//                               (a JVM, a test) drives P ranks on one or several GPUs without RCCL, and
//                               how the multi-rank orchestration is exercised at P = 2..64 on a single
//                               GPU (RCCL refuses two ranks on one device).
//
// The group also checks what RCCL cannot: every rank must enter the same collective with matching sizes
// (a send count must equal its receiver's recv count); a mismatch, a rank that never arrives (timeout,
// GS_COMM_TIMEOUT_MS, default 120 s) or a failed copy breaks the group and every rank's call returns
// GS_ECOMM instead of hanging.
#include <dlfcn.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

#include "gs_ops.hpp"

namespace gs {

// ---- RCCL, resolved at run time -----------------------------------------------------------------------
// ncclUniqueId is 128 bytes; ncclComm_t an opaque pointer; the enums are RCCL's values (gs_internal.hpp).
typedef void* nccl_comm_t;
struct NcclId {
  char internal[128];
};
struct NcclApi {
  int (*GetUniqueId)(void*) = nullptr;
  int (*CommInitRank)(nccl_comm_t*, int, NcclId, int) = nullptr;
  int (*CommDestroy)(nccl_comm_t) = nullptr;
  int (*Send)(const void*, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
  int (*Recv)(void*, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
  int (*AllToAll)(const void*, void*, size_t, int, nccl_comm_t, hipStream_t) = nullptr;
  int (*AllReduce)(const void*, void*, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
  int (*GroupStart)() = nullptr;
  int (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(int) = nullptr;
  bool ok = false;
};
constexpr int NCCL_UINT8 = 1;

// resolved once per process; a function-local static is initialised exactly once even when several
// ctxs (Flink subtask threads) reach it concurrently
static NcclApi load_nccl() {
  NcclApi api;
  void* h = nullptr;
  if (dlsym(RTLD_DEFAULT, "ncclCommInitRank")) h = RTLD_DEFAULT;   // already loaded (e.g. by torch)
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return api;
  auto sym = [&](const char* n) { return dlsym(h, n); };
  api.GetUniqueId = (int (*)(void*))sym("ncclGetUniqueId");
  api.CommInitRank = (int (*)(nccl_comm_t*, int, NcclId, int))sym("ncclCommInitRank");
  api.CommDestroy = (int (*)(nccl_comm_t))sym("ncclCommDestroy");
  api.Send = (int (*)(const void*, size_t, int, int, nccl_comm_t, hipStream_t))sym("ncclSend");
  api.Recv = (int (*)(void*, size_t, int, int, nccl_comm_t, hipStream_t))sym("ncclRecv");
  api.AllToAll = (int (*)(const void*, void*, size_t, int, nccl_comm_t, hipStream_t))sym("ncclAllToAll");
  api.AllReduce = (int (*)(const void*, void*, size_t, int, int, nccl_comm_t, hipStream_t))sym("ncclAllReduce");
  api.GroupStart = (int (*)())sym("ncclGroupStart");
  api.GroupEnd = (int (*)())sym("ncclGroupEnd");
  api.GetErrorString = (const char* (*)(int))sym("ncclGetErrorString");
  api.ok = api.GetUniqueId && api.CommInitRank && api.CommDestroy && api.Send && api.Recv && api.AllToAll &&
           api.AllReduce && api.GroupStart && api.GroupEnd && api.GetErrorString;
  return api;
}

static NcclApi& nccl() {
  static NcclApi api = load_nccl();
  return api;
}

static gs_status nccl_check(gs_ctx* c, int r, const char* what) {
  if (r == 0) return GS_OK;
  return set_error(c, GS_ECOMM, "%s: %s", what, nccl().GetErrorString ? nccl().GetErrorString(r) : "RCCL error");
}

static size_t nccl_bytes(int dt) { return dt == NCCL_T_U32 ? 4 : dt == NCCL_UINT8 ? 1 : 8; }

}  // namespace gs

// ---- the in-process thread group ------------------------------------------------------------------
struct gs_comm_group {
  enum Kind { NONE = 0, ALLREDUCE, ALLTOALL, EXCHANGE, ALLGATHERV };
  struct Post {
    int kind = NONE;
    size_t count = 0, row = 0;
    int dtype = 0, op = 0;
    const void* send = nullptr;
    const uint64_t* scount = nullptr;   // EXCHANGE: rows to each peer; ALLGATHERV: rows of every rank
  };
  int P = 0;
  std::mutex m;
  std::condition_variable cv;
  uint64_t gen = 0;
  int arrived = 0;
  bool broken = false;
  std::string why;
  std::atomic<int> refs{1};
  std::vector<uint8_t> joined;
  std::vector<Post> post;
};

namespace gs {

static int group_timeout_ms() {
  static const int ms = getenv("GS_COMM_TIMEOUT_MS") ? atoi(getenv("GS_COMM_TIMEOUT_MS")) : 120000;
  return ms > 0 ? ms : 120000;
}

static void group_break(gs_comm_group* g, const std::string& why) {
  std::lock_guard<std::mutex> lk(g->m);
  if (!g->broken) g->why = why;
  g->broken = true;
  g->cv.notify_all();
}

static gs_status group_barrier(gs_ctx* c, gs_comm_group* g) {
  std::unique_lock<std::mutex> lk(g->m);
  if (g->broken) return set_error(c, GS_ECOMM, "comm group broken: %s", g->why.c_str());
  const uint64_t gen = g->gen;
  if (++g->arrived == g->P) {
    g->arrived = 0;
    ++g->gen;
    g->cv.notify_all();
    return GS_OK;
  }
  const bool woke = g->cv.wait_for(lk, std::chrono::milliseconds(group_timeout_ms()),
                                   [&] { return g->gen != gen || g->broken; });
  if (g->gen != gen) return GS_OK;   // (the barrier completed, even if the group broke after it)
  if (!woke && !g->broken) {
    g->broken = true;
    g->why = "rank " + std::to_string(c->comm_rank) + " timed out waiting for its peers";
    g->cv.notify_all();
  }
  return set_error(c, GS_ECOMM, "comm group broken: %s", g->why.c_str());
}

// post this rank's part, then the first barrier: on return every rank's post is readable until the
// second barrier (group_end).  The inputs are complete on the device (the ctx stream drained) first.
static gs_status group_begin(gs_ctx* c, gs_comm_group* g, const gs_comm_group::Post& p) {
  gs_status st = host_wait(c);
  if (st != GS_OK) {
    group_break(g, "rank " + std::to_string(c->comm_rank) + ": " + c->err);
    return st;
  }
  {   // a broken group takes no new post: a rank that saw a mismatch below and returned must not
      // overwrite its post while a slower peer still runs the same check
    std::lock_guard<std::mutex> lk(g->m);
    if (g->broken) return set_error(c, GS_ECOMM, "comm group broken: %s", g->why.c_str());
    g->post[c->comm_rank] = p;
  }
  GS_TRY(group_barrier(c, g));
  const gs_comm_group::Post& a = g->post[0];
  for (int q = 0; q < g->P; ++q) {   // the same check on every rank: all agree on a mismatch
    const gs_comm_group::Post& b = g->post[q];
    if (b.kind != a.kind || b.row != a.row || b.dtype != a.dtype || b.op != a.op ||
        (a.kind != gs_comm_group::EXCHANGE && a.kind != gs_comm_group::ALLGATHERV && b.count != a.count)) {
      set_error(c, GS_ECOMM, "comm group: rank %d entered collective %d (count %zu) where rank 0 entered %d (count %zu)",
                q, b.kind, b.count, a.kind, a.count);
      const std::string why = c->err;
      group_break(g, why);   // every rank breaks it (the same check): later collectives fail, none races on post[]
      return GS_ECOMM;
    }
  }
  return GS_OK;
}

// the pulls are enqueued on this rank's stream: wait for them, then the second barrier (no rank reuses
// a buffer a peer may still be reading)
static gs_status group_end(gs_ctx* c, gs_comm_group* g, gs_status st) {
  if (st == GS_OK) st = host_wait(c);
  if (st != GS_OK) {
    group_break(g, "rank " + std::to_string(c->comm_rank) + ": " + c->err);
    return st;
  }
  return group_barrier(c, g);
}

template <typename T, int OP>
__global__ __launch_bounds__(256) void k_group_reduce(const T* __restrict__ in, size_t n, int P, T* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    T a = in[i];
    for (int p = 1; p < P; ++p) {
      const T b = in[(size_t)p * n + i];
      a = OP == NCCL_OP_SUM ? (T)(a + b) : OP == NCCL_OP_MAX ? (b > a ? b : a) : (b < a ? b : a);
    }
    out[i] = a;
  }
}

template <typename T>
static void launch_group_reduce(gs_ctx* c, const void* in, size_t n, int P, int op, void* out) {
  const unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 8192));
  if (op == NCCL_OP_SUM)
    hipLaunchKernelGGL((k_group_reduce<T, NCCL_OP_SUM>), dim3(grid), dim3(256), 0, c->stream, (const T*)in, n, P, (T*)out);
  else if (op == NCCL_OP_MAX)
    hipLaunchKernelGGL((k_group_reduce<T, NCCL_OP_MAX>), dim3(grid), dim3(256), 0, c->stream, (const T*)in, n, P, (T*)out);
  else
    hipLaunchKernelGGL((k_group_reduce<T, NCCL_OP_MIN>), dim3(grid), dim3(256), 0, c->stream, (const T*)in, n, P, (T*)out);
}

// all-reduce: every rank pulls all P buffers into its scratch (rank order), the second barrier, then
// reduces them into its own buffer (every rank sums in the same order: identical results)
static gs_status group_allreduce(gs_ctx* c, void* buf, size_t count, int dt, int op) {
  gs_comm_group* g = (gs_comm_group*)c->comm;
  if (dt != NCCL_T_U32 && dt != NCCL_T_I64 && dt != NCCL_T_U64) return set_error(c, GS_EINVAL, "comm group: dtype %d", dt);
  if (op != NCCL_OP_SUM && op != NCCL_OP_MAX && op != NCCL_OP_MIN) return set_error(c, GS_EINVAL, "comm group: op %d", op);
  gs_comm_group::Post p;
  p.kind = gs_comm_group::ALLREDUCE;
  p.count = count;
  p.dtype = dt;
  p.op = op;
  p.send = buf;
  const size_t bytes = count * nccl_bytes(dt);
  gs_status st = ensure(c, c->comm_scratch, bytes * g->P + 16);   // (before the barrier: ensure may wait)
  if (st != GS_OK) {
    group_break(g, "rank " + std::to_string(c->comm_rank) + ": " + c->err);
    return st;
  }
  GS_TRY(group_begin(c, g, p));
  for (int q = 0; q < g->P && st == GS_OK && bytes; ++q)
    st = hip_check(c, hipMemcpyAsync(c->comm_scratch.as<char>() + (size_t)q * bytes, g->post[q].send, bytes, hipMemcpyDefault,
                                     c->stream), "comm group all-reduce pull");
  GS_TRY(group_end(c, g, st));
  if (!count) return GS_OK;
  if (dt == NCCL_T_U32) launch_group_reduce<uint32_t>(c, c->comm_scratch.p, count, g->P, op, buf);
  else if (dt == NCCL_T_I64) launch_group_reduce<int64_t>(c, c->comm_scratch.p, count, g->P, op, buf);
  else launch_group_reduce<uint64_t>(c, c->comm_scratch.p, count, g->P, op, buf);
  return hip_check(c, hipGetLastError(), "k_group_reduce");
}

// all-to-all of `bytes` per peer: rank r pulls block r of every peer's send buffer into block p of its
// own receive buffer
static gs_status group_alltoall(gs_ctx* c, const void* send, void* recv, size_t bytes) {
  gs_comm_group* g = (gs_comm_group*)c->comm;
  gs_comm_group::Post p;
  p.kind = gs_comm_group::ALLTOALL;
  p.count = bytes;
  p.send = send;
  GS_TRY(group_begin(c, g, p));
  gs_status st = GS_OK;
  const int me = c->comm_rank;
  for (int q = 0; q < g->P && st == GS_OK && bytes; ++q)
    st = hip_check(c, hipMemcpyAsync((char*)recv + (size_t)q * bytes, (const char*)g->post[q].send + (size_t)me * bytes, bytes,
                                     hipMemcpyDefault, c->stream), "comm group all-to-all pull");
  return group_end(c, g, st);
}

// owner-grouped rows: peer q's rows for this rank start after the rows it sends ranks 0 .. me-1; their
// number must equal recv[q]
static gs_status group_exchange(gs_ctx* c, const char* sendbuf, const uint64_t* send, char* recvbuf, const uint64_t* recv,
                                size_t row, bool skip_self) {
  gs_comm_group* g = (gs_comm_group*)c->comm;
  gs_comm_group::Post p;
  p.kind = gs_comm_group::EXCHANGE;
  p.row = row;
  p.send = sendbuf;
  p.scount = send;
  GS_TRY(group_begin(c, g, p));
  gs_status st = GS_OK;
  const int me = c->comm_rank;
  uint64_t ro = 0;
  for (int q = 0; q < g->P && st == GS_OK; ++q) {
    if (skip_self && q == me) continue;
    const gs_comm_group::Post& pq = g->post[q];
    uint64_t off = 0;
    for (int k = 0; k < me; ++k) off += pq.scount[k];
    const uint64_t n = pq.scount[me];
    if (n != recv[q]) {
      st = set_error(c, GS_ECOMM, "comm group exchange: rank %d sends %llu rows to rank %d, which expects %llu", q,
                     (unsigned long long)n, me, (unsigned long long)recv[q]);
      break;
    }
    if (n)
      st = hip_check(c, hipMemcpyAsync(recvbuf + ro * row, (const char*)pq.send + off * row, n * row, hipMemcpyDefault, c->stream),
                     "comm group exchange pull");
    ro += n;
  }
  return group_end(c, g, st);
}

static gs_status group_allgatherv(gs_ctx* c, const void* sendbuf, char* recvbuf, const uint64_t* counts, size_t row) {
  gs_comm_group* g = (gs_comm_group*)c->comm;
  gs_comm_group::Post p;
  p.kind = gs_comm_group::ALLGATHERV;
  p.row = row;
  p.send = sendbuf;
  p.scount = counts;
  GS_TRY(group_begin(c, g, p));
  gs_status st = GS_OK;
  uint64_t at = 0;
  for (int q = 0; q < g->P && st == GS_OK; ++q) {
    const uint64_t n = counts[q];
    if (g->post[q].scount[q] != n) {
      st = set_error(c, GS_ECOMM, "comm group all-gather: rank %d holds %llu rows, expected %llu", q,
                     (unsigned long long)g->post[q].scount[q], (unsigned long long)n);
      break;
    }
    if (n)
      st = hip_check(c, hipMemcpyAsync(recvbuf + at * row, g->post[q].send, n * row, hipMemcpyDefault, c->stream),
                     "comm group all-gather pull");
    at += n;
  }
  return group_end(c, g, st);
}

static bool is_group(const gs_ctx* c) { return c->comm_kind == GS_COMM_KIND_GROUP; }

// ---- the primitives (gs_internal.hpp) -------------------------------------------------------------------
gs_status exchange_rows(gs_ctx* c, const char* sendbuf, const uint64_t* send, char* recvbuf, const uint64_t* recv,
                        size_t row, bool skip_self) {
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  if (is_group(c)) return group_exchange(c, sendbuf, send, recvbuf, recv, row, skip_self);
  NcclApi& A = nccl();
  const int P = c->comm_size;
  bool any = false;   // nothing to or from any peer (e.g. one rank): no group at all
  for (int p = 0; p < P; ++p)
    if (!(skip_self && p == c->comm_rank)) any |= send[p] != 0 || recv[p] != 0;
  if (!any) return GS_OK;
  GS_TRY(nccl_check(c, A.GroupStart(), "ncclGroupStart"));
  uint64_t so = 0, ro = 0;
  for (int p = 0; p < P; ++p) {
    if (skip_self && p == c->comm_rank) {
      so += send[p];
      continue;
    }
    if (send[p]) GS_TRY(nccl_check(c, A.Send(sendbuf + so * row, send[p] * row, NCCL_UINT8, p, c->comm, c->stream), "ncclSend"));
    if (recv[p]) GS_TRY(nccl_check(c, A.Recv(recvbuf + ro * row, recv[p] * row, NCCL_UINT8, p, c->comm, c->stream), "ncclRecv"));
    so += send[p];
    ro += recv[p];
  }
  return nccl_check(c, A.GroupEnd(), "ncclGroupEnd");
}

gs_status comm_allreduce(gs_ctx* c, void* buf, size_t count, int nccl_dtype, int nccl_op) {
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  if (is_group(c)) return group_allreduce(c, buf, count, nccl_dtype, nccl_op);
  return nccl_check(c, nccl().AllReduce(buf, buf, count, nccl_dtype, nccl_op, c->comm, c->stream), "ncclAllReduce");
}

gs_status comm_alltoall(gs_ctx* c, const void* send, void* recv, size_t count, int nccl_dtype) {
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  if (is_group(c)) return group_alltoall(c, send, recv, count * nccl_bytes(nccl_dtype));
  return nccl_check(c, nccl().AllToAll(send, recv, count, nccl_dtype, c->comm, c->stream), "ncclAllToAll");
}

// Status agreement before the next collective: every rank reports whether its local step failed
// (all-reduce MAX of one flag), so a failure on one rank ends the call on all of them with an error
// instead of leaving the others blocked in a collective.  Returns the local status (its message kept),
// GS_ECOMM when only another rank failed.
gs_status comm_agree(gs_ctx* c, gs_status local) {
  if (!c->comm) return local;
  const std::string msg = c->err;
  GS_TRY(ensure(c, c->dist_x, 64 + (size_t)c->comm_size * 32, true));   // (word 0: gs_dist.hip's key-width flag)
  uint64_t* d = c->dist_x.as<uint64_t>() + 1;
  c->host_small[200] = local != GS_OK ? 1 : 0;
  GS_HIP(hipMemcpyAsync(d, c->host_small + 200, 8, hipMemcpyHostToDevice, c->stream));
  GS_TRY(comm_allreduce(c, d, 1, NCCL_T_U64, NCCL_OP_MAX));
  GS_HIP(hipMemcpyAsync(c->host_small + 201, d, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if (local != GS_OK) return set_error(c, local, "%s", msg.c_str());
  if (c->host_small[201]) return set_error(c, GS_ECOMM, "another rank failed its local step of the window");
  return GS_OK;
}

// every rank's u64 -> all[0 .. comm_size) on the host (a sum of one-hot rows)
gs_status comm_allgather_u64(gs_ctx* c, uint64_t mine, uint64_t* all) {
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  const int P = c->comm_size;
  GS_TRY(ensure(c, c->dist_cnt, 1024 + (size_t)P * 8));
  uint64_t* d = (uint64_t*)(c->dist_cnt.as<char>() + 512);
  GS_HIP(hipMemsetAsync(d, 0, P * 8, c->stream));
  c->host_small[100] = mine;   // pinned source (HOST_SMALL_WORDS = 512; results land in [8, 8 + P))
  GS_HIP(hipMemcpyAsync(d + c->comm_rank, c->host_small + 100, 8, hipMemcpyHostToDevice, c->stream));
  GS_TRY(comm_allreduce(c, d, P, NCCL_T_U64, NCCL_OP_SUM));
  GS_HIP(hipMemcpyAsync(c->host_small + 8, d, P * 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  memcpy(all, c->host_small + 8, P * 8);
  return GS_OK;
}

// every rank's W words -> all[p * W + j] on the host (a sum of one-hot rows; W * comm_size <= 256)
gs_status comm_allgather_words(gs_ctx* c, const uint64_t* mine, int W, uint64_t* all) {
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  const int P = c->comm_size;
  if (W < 1 || (size_t)W * P > 256) return set_error(c, GS_EINVAL, "comm_allgather_words: %d x %d words", W, P);
  GS_TRY(ensure(c, c->dist_cnt, 1024 + (size_t)P * W * 8));
  uint64_t* d = (uint64_t*)(c->dist_cnt.as<char>() + 512);
  GS_HIP(hipMemsetAsync(d, 0, (size_t)P * W * 8, c->stream));
  memcpy(c->host_small + 100, mine, (size_t)W * 8);   // pinned source; results land in [200, 200 + P W)
  GS_HIP(hipMemcpyAsync(d + (size_t)c->comm_rank * W, c->host_small + 100, (size_t)W * 8, hipMemcpyHostToDevice, c->stream));
  GS_TRY(comm_allreduce(c, d, (size_t)P * W, NCCL_T_U64, NCCL_OP_SUM));
  GS_HIP(hipMemcpyAsync(c->host_small + 200, d, (size_t)P * W * 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  memcpy(all, c->host_small + 200, (size_t)P * W * 8);
  return GS_OK;
}

// every rank's `mine` rows (row bytes each) concatenated in rank order into recvbuf; counts[p] = rows of
// rank p (comm_allgather_u64)
gs_status comm_allgatherv(gs_ctx* c, const void* sendbuf, char* recvbuf, const uint64_t* counts, size_t row) {
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  if (is_group(c)) return group_allgatherv(c, sendbuf, recvbuf, counts, row);
  NcclApi& A = nccl();
  const int P = c->comm_size, me = c->comm_rank;
  uint64_t off = 0;
  std::vector<uint64_t> at(P);
  for (int p = 0; p < P; ++p) {
    at[p] = off;
    off += counts[p];
  }
  if (counts[me]) GS_HIP(hipMemcpyAsync(recvbuf + at[me] * row, sendbuf, counts[me] * row, hipMemcpyDeviceToDevice, c->stream));
  GS_TRY(nccl_check(c, A.GroupStart(), "ncclGroupStart"));
  for (int p = 0; p < P; ++p) {
    if (p == me) continue;
    if (counts[me]) GS_TRY(nccl_check(c, A.Send(sendbuf, counts[me] * row, NCCL_UINT8, p, c->comm, c->stream), "ncclSend"));
    if (counts[p]) GS_TRY(nccl_check(c, A.Recv(recvbuf + at[p] * row, counts[p] * row, NCCL_UINT8, p, c->comm, c->stream), "ncclRecv"));
  }
  return nccl_check(c, A.GroupEnd(), "ncclGroupEnd");
}

}  // namespace gs

using namespace gs;

extern "C" {

gs_status gs_comm_unique_id(void* id128) {
  if (!id128) return GS_EINVAL;
  NcclApi& A = nccl();
  if (!A.ok) return GS_ECOMM;
  return A.GetUniqueId(id128) == 0 ? GS_OK : GS_ECOMM;
}

gs_status gs_comm_init(gs_ctx* c, int32_t nranks, int32_t rank, const void* id128) {
  if (!c) return GS_EINVAL;
  if (!id128 || nranks < 1 || nranks > GS_COMM_MAX_RANKS || rank < 0 || rank >= nranks)
    return set_error(c, GS_EINVAL, "bad communicator arguments (%d ranks, rank %d)", nranks, rank);
  NcclApi& A = nccl();
  if (!A.ok) return set_error(c, GS_ECOMM, "RCCL not found (librccl.so.1)");
  GS_TRY(gs_comm_destroy(c));
  GS_HIP(hipSetDevice(c->device));
  NcclId id;
  memcpy(id.internal, id128, 128);
  nccl_comm_t comm = nullptr;
  GS_TRY(nccl_check(c, A.CommInitRank(&comm, nranks, id, rank), "ncclCommInitRank"));
  c->comm = comm;
  c->comm_kind = GS_COMM_KIND_RCCL;
  c->comm_size = nranks;
  c->comm_rank = rank;
  return GS_OK;
}

gs_status gs_comm_group_create(int32_t nranks, gs_comm_group** out) {
  if (!out) return GS_EINVAL;
  *out = nullptr;
  if (nranks < 1 || nranks > GS_COMM_MAX_RANKS) return GS_EINVAL;
  gs_comm_group* g = new (std::nothrow) gs_comm_group();
  if (!g) return GS_ENOMEM;
  g->P = nranks;
  g->joined.assign(nranks, 0);
  g->post.resize(nranks);
  *out = g;
  return GS_OK;
}

static void group_release(gs_comm_group* g) {
  if (g && g->refs.fetch_sub(1) == 1) delete g;
}

void gs_comm_group_destroy(gs_comm_group* g) { group_release(g); }

gs_status gs_comm_init_group(gs_ctx* c, gs_comm_group* g, int32_t rank) {
  if (!c) return GS_EINVAL;
  if (!g || rank < 0 || rank >= g->P) return set_error(c, GS_EINVAL, "bad comm group arguments (rank %d)", rank);
  GS_TRY(gs_comm_destroy(c));
  {
    std::lock_guard<std::mutex> lk(g->m);
    if (g->joined[rank]) return set_error(c, GS_EINVAL, "comm group: rank %d already joined", rank);
    g->joined[rank] = 1;
  }
  g->refs.fetch_add(1);
  c->comm = g;
  c->comm_kind = GS_COMM_KIND_GROUP;
  c->comm_size = g->P;
  c->comm_rank = rank;
  return GS_OK;
}

gs_status gs_comm_destroy(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  if (c->comm && c->comm_kind == GS_COMM_KIND_RCCL && nccl().ok) nccl().CommDestroy(c->comm);
  if (c->comm && c->comm_kind == GS_COMM_KIND_GROUP) {
    gs_comm_group* g = (gs_comm_group*)c->comm;
    {
      std::lock_guard<std::mutex> lk(g->m);
      g->joined[c->comm_rank] = 0;
    }
    group_release(g);
  }
  c->comm = nullptr;
  c->comm_kind = 0;
  c->comm_size = 0;
  return GS_OK;
}

// exact triangle count etc. add up over ranks: all-reduce (sum) of one u64
gs_status gs_comm_allreduce_sum_u64(gs_ctx* c, uint64_t* value) {
  if (!c || !value) return GS_EINVAL;
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  GS_TRY(ensure(c, c->dist_cnt, 1024));
  uint64_t* d = c->dist_cnt.as<uint64_t>();
  c->host_small[8] = *value;
  GS_HIP(hipMemcpyAsync(d, c->host_small + 8, 8, hipMemcpyHostToDevice, c->stream));
  GS_TRY(comm_allreduce(c, d, 1, NCCL_T_U64, NCCL_OP_SUM));
  GS_HIP(hipMemcpyAsync(c->host_small + 8, d, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *value = c->host_small[8];
  return GS_OK;
}

}  // extern "C"
