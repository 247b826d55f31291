// gs_pairs.hip — stage 2 of WindowTriangles over materialised candidate records:
//   keyBy(0, 1).timeWindow(w).apply(CountTriangles).timeWindowAll(w).sum(0)
//   (example/WindowTriangles.java:64-66; CountTriangles.apply :119-140)
// Per (a, b) group the reference counts candidate (true) and edge (false) records and emits the
// candidate count when edges > 0; the all-window sum adds the emitted Integers.
//
// Device pipeline (all HBM-bound integer work):
//   k_pr_minmax  min / max of a and of b (one pass over 16 B per record)
//   k_pr_pack    key = (a - amin) << 32 | (b - bmin) (injective when both spans are < 2^32),
//                payload = 1 for a candidate, 2^32 for an edge record
//   gs_window_reduce(SUM) groups the keys: a group's sum holds #candidates in its low word and
//                #edges in its high word (the window's records are < 2^32 per group)
//   k_pr_count   sum of low words over groups whose high word is non-zero; number of such groups
#include "gs_ops.hpp"

using namespace gs;

namespace {

constexpr int PR_BLOCK = 256;

__device__ __forceinline__ uint64_t flip(int64_t x) { return (uint64_t)x ^ (1ull << 63); }

// mm[0] = max ~flip(a), mm[1] = max flip(a), mm[2] = max ~flip(b), mm[3] = max flip(b)
__global__ __launch_bounds__(PR_BLOCK) void k_pr_minmax(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                        uint64_t n, unsigned long long* __restrict__ mm) {
  uint64_t r[4] = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * PR_BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * PR_BLOCK) {
    const uint64_t fa = flip(a[i]), fb = flip(b[i]);
    r[0] = max(r[0], ~fa);
    r[1] = max(r[1], fa);
    r[2] = max(r[2], ~fb);
    r[3] = max(r[3], fb);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r[k] = max(r[k], (uint64_t)__shfl_xor((unsigned long long)r[k], o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicMax(&mm[k], (unsigned long long)r[k]);
  }
}

__global__ __launch_bounds__(PR_BLOCK) void k_pr_pack(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                      const uint8_t* __restrict__ f, uint64_t n, int64_t amin,
                                                      int64_t bmin, int64_t* __restrict__ key,
                                                      int64_t* __restrict__ val) {
  for (uint64_t i = (uint64_t)blockIdx.x * PR_BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * PR_BLOCK) {
    const uint64_t ra = (uint64_t)a[i] - (uint64_t)amin, rb = (uint64_t)b[i] - (uint64_t)bmin;
    key[i] = (int64_t)((ra << 32) | rb);
    val[i] = f[i] ? 1 : (int64_t)(1ull << 32);
  }
}

// out[0] = sum of #candidates over emitting groups, out[1] = emitting groups
__global__ __launch_bounds__(PR_BLOCK) void k_pr_count(const int64_t* __restrict__ gv, uint64_t U,
                                                       unsigned long long* __restrict__ out) {
  uint64_t s = 0, g = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * PR_BLOCK + threadIdx.x; i < U; i += (uint64_t)gridDim.x * PR_BLOCK) {
    const uint64_t v = (uint64_t)gv[i];
    if (v >> 32) {
      s += v & 0xFFFFFFFFull;
      ++g;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += (uint64_t)__shfl_xor((unsigned long long)s, o, 64);
    g += (uint64_t)__shfl_xor((unsigned long long)g, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && (s | g)) {
    atomicAdd(&out[0], (unsigned long long)s);
    atomicAdd(&out[1], (unsigned long long)g);
  }
}

uint32_t grid_for(const gs_ctx* c, uint64_t n) {
  const uint64_t want = (n + PR_BLOCK - 1) / PR_BLOCK;
  const uint64_t cap = (uint64_t)std::max(1, c->n_cu) * 16;
  return (uint32_t)std::max<uint64_t>(1, std::min(want, cap));
}

}  // namespace

extern "C" gs_status gs_window_count_candidates(gs_ctx* c, const gs_pair_batch* p, uint64_t* count,
                                                int32_t* count_ref_wrapped, int32_t* has_output,
                                                uint64_t* groups) {
  if (!c) return GS_EINVAL;
  if (!p || !count || !count_ref_wrapped || !has_output || !groups)
    return set_error(c, GS_EINVAL, "count_candidates: null argument");
  if (p->n && (!p->a || !p->b || !p->is_candidate))
    return set_error(c, GS_EINVAL, "count_candidates: null column");
  if (p->mem != GS_MEM_HOST && p->mem != GS_MEM_DEVICE) return set_error(c, GS_EINVAL, "count_candidates: bad mem");
  if (p->n >= (1ull << 32)) return set_error(c, GS_EINVAL, "count_candidates: more than 2^32 - 1 records");
  *count = 0;
  *count_ref_wrapped = 0;
  *has_output = 0;
  *groups = 0;
  GS_HIP(hipSetDevice(c->device));
  GS_TRY(begin_call(c));
  const uint64_t n = p->n;
  if (n == 0) return GS_OK;
  const int64_t *a = p->a, *b = p->b;
  const uint8_t* f = p->is_candidate;
  if (p->mem == GS_MEM_HOST) {
    GS_TRY(ensure(c, c->pr_a, n * 8));
    GS_TRY(ensure(c, c->pr_b, n * 8));
    GS_TRY(ensure(c, c->pr_f, n));
    GS_HIP(hipMemcpyAsync(c->pr_a.p, a, n * 8, hipMemcpyHostToDevice, c->stream));
    GS_HIP(hipMemcpyAsync(c->pr_b.p, b, n * 8, hipMemcpyHostToDevice, c->stream));
    GS_HIP(hipMemcpyAsync(c->pr_f.p, f, n, hipMemcpyHostToDevice, c->stream));
    a = c->pr_a.as<int64_t>();
    b = c->pr_b.as<int64_t>();
    f = c->pr_f.as<uint8_t>();
  }
  GS_TRY(ensure(c, c->pr_small, 64));
  unsigned long long* mm = c->pr_small.as<unsigned long long>();
  GS_HIP(hipMemsetAsync(mm, 0, 64, c->stream));
  const uint32_t grid = grid_for(c, n);
  hipLaunchKernelGGL(k_pr_minmax, dim3(grid), dim3(PR_BLOCK), 0, c->stream, a, b, n, mm);
  GS_HIP(hipGetLastError());
  uint64_t h[4];
  GS_HIP(hipMemcpyAsync(h, mm, 32, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const int64_t amin = (int64_t)(~h[0] ^ (1ull << 63)), amax = (int64_t)(h[1] ^ (1ull << 63));
  const int64_t bmin = (int64_t)(~h[2] ^ (1ull << 63)), bmax = (int64_t)(h[3] ^ (1ull << 63));
  int64_t amin_ = amin, bmin_ = bmin;
  if ((uint64_t)amax - (uint64_t)amin >= (1ull << 32) || (uint64_t)bmax - (uint64_t)bmin >= (1ull << 32)) {
    // IDs spanning 2^32 or more: order-preserving compact IDs of a and b (one ID space, < 2n values);
    // grouping by (a, b) is unchanged
    const int64_t* uniq = nullptr;
    uint64_t V = 0;
    GS_TRY(relabel_endpoints(c, a, b, n, &a, &b, &uniq, &V));
    amin_ = 0;
    bmin_ = 0;
  }
  GS_TRY(ensure(c, c->pr_key, n * 8));
  GS_TRY(ensure(c, c->pr_val, n * 8));
  GS_TRY(ensure(c, c->pr_gk, n * 8));
  GS_TRY(ensure(c, c->pr_gv, n * 8));
  hipLaunchKernelGGL(k_pr_pack, dim3(grid), dim3(PR_BLOCK), 0, c->stream, a, b, f, n, amin_, bmin_,
                     c->pr_key.as<int64_t>(), c->pr_val.as<int64_t>());
  GS_HIP(hipGetLastError());
  gs_edge_batch kb{c->pr_key.as<int64_t>(), c->pr_key.as<int64_t>(), c->pr_val.p, n, GS_I64, GS_MEM_DEVICE, 0};
  uint64_t U = 0;
  gs_vertex_out go{c->pr_gk.as<int64_t>(), c->pr_gv.p, n, &U, GS_MEM_DEVICE, 0};
  GS_TRY(gs_window_reduce(c, &kb, GS_DIR_OUT, GS_OP_SUM, &go));
  GS_HIP(hipMemsetAsync(mm, 0, 16, c->stream));
  hipLaunchKernelGGL(k_pr_count, dim3(grid_for(c, U)), dim3(PR_BLOCK), 0, c->stream, c->pr_gv.as<int64_t>(), U, mm);
  GS_HIP(hipGetLastError());
  GS_HIP(hipMemcpyAsync(h, mm, 16, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  *count = h[0];
  *count_ref_wrapped = (int32_t)(uint32_t)h[0];
  *groups = h[1];
  *has_output = h[1] != 0;
  return GS_OK;
}
