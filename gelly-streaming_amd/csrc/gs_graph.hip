// gs_graph.hip — neighbourhood grouping (applyOnNeighbors).
//
//   gs_window_csr        <- the grouping half of applyOnNeighbors (GraphWindowStream.java:130-175)
// (WindowTriangles: gs_triangles.hip)
#include "gs_ops.hpp"

namespace gs {

// sorted position p holds record index r (stable sort => arrival order inside each vertex):
// neighbours[p] = other endpoint of record r, vals[p] = value of its edge
template <int DIR>
__global__ __launch_bounds__(256) void k_gather_csr(const uint32_t* __restrict__ rec, uint32_t R,
                                                    const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                    const void* __restrict__ val, int vbytes,
                                                    int64_t* __restrict__ nbrs, void* __restrict__ vals) {
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < R; p += gridDim.x * 256u) {
    const uint32_t r = rec[p];
    uint32_t i = r;
    bool rev = (DIR == DIR_IN);
    if (DIR == DIR_ALL) {
      i = r >> 1;
      rev = r & 1u;
    }
    nbrs[p] = rev ? src[i] : dst[i];
    if (vals) {
      if (vbytes == 4) ((uint32_t*)vals)[p] = ((const uint32_t*)val)[i];
      else ((uint64_t*)vals)[p] = ((const uint64_t*)val)[i];
    }
  }
}


}  // namespace gs

using namespace gs;

extern "C" {

gs_status gs_window_csr(gs_ctx* c, const gs_edge_batch* b, int32_t dir, gs_csr_out* out) {
  GS_TRY(check_batch(c, b, dir));
  if (!out || !out->n_vertices || !out->n_records) return set_error(c, GS_EINVAL, "bad gs_csr_out");
  GS_TRY(begin_call(c));
  const uint64_t R = dir == GS_DIR_ALL ? 2 * b->n : b->n;
  *out->n_records = R;
  if (R == 0) {
    *out->n_vertices = 0;
    if (out->offsets && out->capacity_vertices + 1 >= 1) {
      const uint64_t z = 0;
      GS_HIP(hipMemcpy(out->offsets, &z, 8, out->mem == GS_MEM_DEVICE ? hipMemcpyHostToDevice : hipMemcpyHostToHost));
    }
    return GS_OK;
  }
  const bool want_vals = out->vals && b->val_dtype != GS_NONE && b->val;
  hipEventRecord(c->ev[0], c->stream);
  const int64_t *src, *dst;
  const void* val;
  GS_TRY(stage_batch(c, b, &src, &dst, &val, want_vals));
  Sorted s;
  GS_TRY(sort_window(c, src, dst, nullptr, 0, b->n, dir, PAY_IDX, &s));
  hipEventRecord(c->ev[2], c->stream);
  const size_t vb = dtype_bytes(b->val_dtype);
  const bool direct = out->mem == GS_MEM_DEVICE && out->capacity_vertices >= R && out->capacity_records >= R;
  int64_t *kd = out->keys, *nd = out->neighbors;
  uint64_t* od = out->offsets;
  void* vd = want_vals ? out->vals : nullptr;
  if (!direct) {
    GS_TRY(ensure(c, c->out_keys, R * 8));
    GS_TRY(ensure(c, c->out_a, (R + 1) * 8));
    GS_TRY(ensure(c, c->out_b, R * 8));
    kd = c->out_keys.as<int64_t>();
    od = c->out_a.as<uint64_t>();
    nd = c->out_b.as<int64_t>();
    if (want_vals) {
      GS_TRY(ensure(c, c->aux, R * vb));
      vd = c->aux.p;
    }
  }
  GS_HIP(hipMemsetAsync(od, 0, 8, c->stream));
  CsrOut o{kd, od};
  uint64_t U = 0;
  GS_TRY((s.wide ? launch_rbk<uint64_t, CountOp>(c, s, o, &U) : launch_rbk<uint32_t, CountOp>(c, s, o, &U)));
  const unsigned grid = (unsigned)std::min<uint64_t>((R + 255) / 256, 8192);
  switch (dir) {
    case GS_DIR_IN:
      hipLaunchKernelGGL(k_gather_csr<DIR_IN>, dim3(grid), dim3(256), 0, c->stream, (const uint32_t*)s.vals,
                         (uint32_t)R, src, dst, val, (int)vb, nd, vd);
      break;
    case GS_DIR_OUT:
      hipLaunchKernelGGL(k_gather_csr<DIR_OUT>, dim3(grid), dim3(256), 0, c->stream, (const uint32_t*)s.vals,
                         (uint32_t)R, src, dst, val, (int)vb, nd, vd);
      break;
    default:
      hipLaunchKernelGGL(k_gather_csr<DIR_ALL>, dim3(grid), dim3(256), 0, c->stream, (const uint32_t*)s.vals,
                         (uint32_t)R, src, dst, val, (int)vb, nd, vd);
  }
  GS_HIP(hipGetLastError());
  finish_times(c, s, U);
  *out->n_vertices = U;
  if (U > out->capacity_vertices || R > out->capacity_records)
    return set_error(c, GS_ECAPACITY, "csr needs %llu vertices / %llu records", (unsigned long long)U,
                     (unsigned long long)R);
  GS_TRY(deliver(c, out->keys, kd, U * 8, out->mem));
  GS_TRY(deliver(c, out->offsets, od, (U + 1) * 8, out->mem));
  GS_TRY(deliver(c, out->neighbors, nd, R * 8, out->mem));
  if (want_vals) GS_TRY(deliver(c, out->vals, vd, R * vb, out->mem));
  GS_TRY(host_wait(c));
  return GS_OK;
}

}  // extern "C"
