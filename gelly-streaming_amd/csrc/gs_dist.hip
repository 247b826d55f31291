// gs_dist.hip — multi-GPU keyBy for reduceOnEdges / foldNeighbors behind the C ABI.
//
// The reference spreads a window over subtasks with keyBy(NeighborKeySelector) (SimpleEdgeStream.java
// :159-167): every record travels to the subtask that owns its key.  Here every rank pre-reduces its
// own slice of the window (the bucket path), and only the per-vertex partials travel:
//
//   gs_window_reduce_partials      local reduce -> partials grouped by owner(v) = gs_owner_of(v, nparts)
//                                  (a stable device-side partition: ascending keys within each owner),
//                                  per-owner counts to the host
//   (exchange)                     the caller's all-to-all (torch.distributed / Java), or the ctx-owned
//                                  RCCL communicator below
//   gs_merge_partials              the owner combines what it received (op: SUM / MIN / MAX; COUNT
//                                  partials merge by SUM; foldNeighbors' init applied once, here)
//   gs_window_reduce_dist          all three with the ctx's RCCL communicator (gs_comm_init)
//
// The owner is a hash of the vertex, as Flink's keyBy is; which rank owns a vertex is not observable in
// the reference's output (per-vertex records, compared as unordered sets).  Integer results stay
// bit-exact (the ops are associative and commutative); float sums move within the 1e-5 tolerance.
// RCCL is resolved at gs_comm_init time (dlopen / the process's already-loaded RCCL, e.g. torch's), so
// libgellyhip.so itself has no RCCL dependency.
#include <string.h>

#include <string>
#include <vector>

#include "gs_ops.hpp"

namespace gs {

// owner_of: gs_ops.hpp (shared with the candidate split, gs_hashset.hip)

constexpr int OW_BLOCK = 256, OW_ITEMS = 8, OW_TILE = OW_BLOCK * OW_ITEMS, OW_MAXP = 64;
constexpr size_t BK_MAXB_DIST = 2048;   // the bucket path's most buckets (gs_bucket.hpp BK_MAXB) ...
constexpr size_t BK_OE_SLICES_DIST = 8;  // ... and slices per bucket (BK_OE_SLICES): OwnerEmit's counts

// per tile: partials per owner -> cnt[owner * tiles + tile]; *wide |= 1 when a key lies outside
// [0, 2^32) (the exchange then sends 8-byte keys).  MAXP 8: each thread counts its rows per owner in
// registers, one wave sum per owner, one LDS atomic per wave and owner (per-row LDS atomics on a few
// addresses serialise: 29 us for a C2 window's partials at one owner); MAXP 64: per-row LDS atomics.
template <int MAXP>
__global__ __launch_bounds__(OW_BLOCK) void k_owner_count(const int64_t* __restrict__ keys, uint64_t U, uint32_t nparts,
                                                          uint32_t tiles, uint32_t* __restrict__ cnt,
                                                          unsigned long long* __restrict__ wide) {
  __shared__ uint32_t s_c[OW_MAXP];
  const int tid = threadIdx.x;
  if (tid < OW_MAXP) s_c[tid] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * OW_TILE;
  bool w = false;
  uint32_t mine[MAXP <= 8 ? MAXP : 1] = {};
#pragma unroll
  for (int u = 0; u < OW_ITEMS; ++u) {
    const uint64_t i = base + (uint64_t)u * OW_BLOCK + tid;
    if (i < U) {
      const int64_t k = keys[i];
      w |= (uint64_t)k >> 32 != 0;
      const uint32_t o = owner_of(k, nparts);
      if constexpr (MAXP <= 8) {
#pragma unroll
        for (int j = 0; j < MAXP; ++j) mine[j] += o == (uint32_t)j ? 1u : 0u;
      } else {
        atomicAdd(&s_c[o], 1u);
      }
    }
  }
  if constexpr (MAXP <= 8) {
#pragma unroll
    for (int j = 0; j < MAXP; ++j) {
      if (j >= (int)nparts) break;
      const uint32_t t = wave_inclusive_sum(mine[j]);
      if ((tid & 63) == 63 && t) atomicAdd(&s_c[j], t);
    }
  }
  if (wide && __any(w) && (tid & 63) == 0) atomicOr(wide, 1ull);
  __syncthreads();
  if (tid < (int)nparts) cnt[(uint64_t)tid * tiles + blockIdx.x] = s_c[tid];
}

// stable partition of a tile of OW_TILE partials: the tile is loaded lane-interleaved (coalesced) into
// LDS; thread t then owns rows [16t, 16t + 16) for the per-owner ranks (a block scan over threads per
// owner, as the order within an owner must stay ascending); the rows' tile-local order by owner goes to
// an LDS permutation, and the tile is written out lane-interleaved from it, so each owner's run of the
// tile lands in consecutive addresses (the round-2 version read and wrote each thread's 16 consecutive
// rows straight from / to HBM: 64 lanes, 64 cache lines per instruction; 459 us for the 7.4 M partials of
// a C2 window, now a fraction of that)
//
// PACK (the exchange of gs_window_*_dist): the rows go out as the exchange's packed rows instead --
// key (1 word, 2 when k_owner_count found a key outside [0, 2^32) on this rank), value, [maximum] --
// into `rows`; no separate pack pass over the partitioned partials
template <typename V, int MAXP, bool TWO, bool PACK>
__global__ __launch_bounds__(OW_BLOCK) void k_owner_scatter(const int64_t* __restrict__ keys, const V* __restrict__ vals,
                                                            const int64_t* __restrict__ vals2, uint64_t U,
                                                            uint32_t nparts, uint32_t tiles,
                                                            const uint32_t* __restrict__ off, int64_t* __restrict__ okeys,
                                                            V* __restrict__ ovals, int64_t* __restrict__ ovals2,
                                                            uint32_t* __restrict__ rows,
                                                            const unsigned long long* __restrict__ wide) {
  constexpr uint32_t PADN = OW_TILE + OW_TILE / OW_ITEMS;   // row i at i + i / 16: thread t's rows off bank 0
  __shared__ int64_t s_k[PADN];
  __shared__ V s_v[OW_TILE];
  __shared__ int64_t s_v2[TWO ? OW_TILE : 1];
  __shared__ uint16_t s_r[MAXP][OW_BLOCK];   // (MAXP 8: one node's ranks in 4 KiB; 64 otherwise)
  __shared__ uint16_t s_perm[OW_TILE];   // tile-local order by owner -> row
  __shared__ uint8_t s_own[OW_TILE];
  __shared__ uint32_t s_w[OW_BLOCK / WAVE];
  __shared__ uint32_t s_lo[MAXP + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * OW_TILE;
  const uint32_t nt = (uint32_t)min<uint64_t>(OW_TILE, U - base);
#pragma unroll
  for (int j = 0; j < OW_ITEMS; ++j) {   // coalesced loads
    const uint32_t r = (uint32_t)j * OW_BLOCK + tid;
    if (r < nt) {
      s_k[r + r / OW_ITEMS] = keys[base + r];
      s_v[r] = vals[base + r];
      if constexpr (TWO) s_v2[r] = vals2[base + r];
    }
  }
  for (uint32_t o = 0; o < nparts; ++o) s_r[o][tid] = 0;
  __syncthreads();
  uint32_t own[OW_ITEMS];
  const uint32_t i0 = (uint32_t)tid * OW_ITEMS;
#pragma unroll
  for (int j = 0; j < OW_ITEMS; ++j) {
    const uint32_t r = i0 + j;
    own[j] = r < nt ? owner_of(s_k[r + r / OW_ITEMS], nparts) : OW_MAXP;
    if (own[j] < OW_MAXP) {
      s_r[own[j]][tid]++;
      s_own[r] = (uint8_t)own[j];
    }
  }
  if (tid == 0) s_lo[0] = 0;
  for (uint32_t o = 0; o < nparts; ++o) {   // exclusive scan of owner o's counts over threads; its tile total
    const uint32_t x = s_r[o][tid];
    const uint32_t inc = wave_inclusive_sum(x);
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int k = 0; k < OW_BLOCK / WAVE; ++k) {
      pre += k < w ? s_w[k] : 0u;
      tot += s_w[k];
    }
    s_r[o][tid] = (uint16_t)(pre + inc - x);
    if (tid == 0) s_lo[o + 1] = tot;   // (turned into starts below)
    __syncthreads();
  }
  if (tid == 0)
    for (uint32_t o = 0; o < nparts; ++o) s_lo[o + 1] += s_lo[o];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < OW_ITEMS; ++j) {
    if (own[j] >= OW_MAXP) continue;
    s_perm[s_lo[own[j]] + s_r[own[j]][tid]++] = (uint16_t)(i0 + j);
  }
  __syncthreads();
  constexpr uint32_t VW = sizeof(V) / 4, MW = TWO ? 2 : 0;
  uint32_t kw = 1;
  if constexpr (PACK) kw = (*wide & 1ull) ? 2u : 1u;
#pragma unroll
  for (int j = 0; j < OW_ITEMS; ++j) {   // coalesced stores: consecutive q of one owner -> consecutive addresses
    const uint32_t q = (uint32_t)j * OW_BLOCK + tid;
    if (q >= nt) continue;
    const uint32_t r = s_perm[q], o = s_own[r];
    const uint32_t pos = off[(uint64_t)o * tiles + blockIdx.x] + (q - s_lo[o]);
    if constexpr (PACK) {
      uint32_t* w = rows + (uint64_t)pos * (kw + VW + MW);
      const uint64_t k = (uint64_t)s_k[r + r / OW_ITEMS];
      w[0] = (uint32_t)k;
      if (kw == 2) w[1] = (uint32_t)(k >> 32);
      const uint64_t v = (uint64_t)s_v[r];
      w[kw] = (uint32_t)v;
      if constexpr (VW == 2) w[kw + 1] = (uint32_t)(v >> 32);
      if constexpr (TWO) {
        const uint64_t m = (uint64_t)s_v2[r];
        w[kw + VW] = (uint32_t)m;
        w[kw + VW + 1] = (uint32_t)(m >> 32);
      }
    } else {
      okeys[pos] = s_k[r + r / OW_ITEMS];
      ovals[pos] = s_v[r];
      if constexpr (TWO) ovals2[pos] = s_v2[r];
    }
  }
}

// The owner partition on the device: rows grouped by owner (ascending keys within an owner), the
// per-owner totals in dist_cnt[0, nparts) (u64) and, with `wide`, the key-width flag.  With `rows` the
// partition writes the exchange's packed rows (k_owner_scatter PACK; needs `wide`) instead of okeys /
// ovals / ovals2.  No host wait.
gs_status owner_partition_dev(gs_ctx* c, const int64_t* keys, const void* vals, size_t vb, const int64_t* vals2,
                              uint64_t U, uint32_t nparts, int64_t* okeys, void* ovals, int64_t* ovals2,
                              unsigned long long* wide, uint32_t* rows = nullptr) {
  if (rows && !wide) return set_error(c, GS_EINVAL, "packed owner partition without the key-width flag");
  const uint32_t tiles = (uint32_t)std::max<uint64_t>(1, (U + OW_TILE - 1) / OW_TILE);
  // dist_cnt: [0, 1 KiB) per-call scalars (owner totals, exchange counts), then the tile counts
  GS_TRY(ensure(c, c->dist_cnt, 1024 + (size_t)tiles * nparts * 4));
  auto* totals = c->dist_cnt.as<unsigned long long>();
  uint32_t* cnt = (uint32_t*)(c->dist_cnt.as<char>() + 1024);
  if (!U) {
    GS_HIP(hipMemsetAsync(totals, 0, nparts * 8, c->stream));
    return GS_OK;
  }
  if (nparts <= 8)
    hipLaunchKernelGGL(k_owner_count<8>, dim3(tiles), dim3(OW_BLOCK), 0, c->stream, keys, U, nparts, tiles, cnt, wide);
  else
    hipLaunchKernelGGL(k_owner_count<OW_MAXP>, dim3(tiles), dim3(OW_BLOCK), 0, c->stream, keys, U, nparts, tiles, cnt, wide);
  hipLaunchKernelGGL(k_owner_scan, dim3(1), dim3(1024), 0, c->stream, cnt, tiles * nparts, tiles, nparts, totals,
                     nullptr);
  auto launch = [&](auto vtag, auto ptag, auto ttag) {
    using V = decltype(vtag);
    constexpr int MP = decltype(ptag)::value;
    constexpr bool TW = decltype(ttag)::value;
    if (rows)
      hipLaunchKernelGGL((k_owner_scatter<V, MP, TW, true>), dim3(tiles), dim3(OW_BLOCK), 0, c->stream, keys,
                         (const V*)vals, vals2, U, nparts, tiles, cnt, nullptr, nullptr, nullptr, rows,
                         (const unsigned long long*)wide);
    else
      hipLaunchKernelGGL((k_owner_scatter<V, MP, TW, false>), dim3(tiles), dim3(OW_BLOCK), 0, c->stream, keys,
                         (const V*)vals, vals2, U, nparts, tiles, cnt, okeys, (V*)ovals, ovals2, nullptr, nullptr);
  };
  using P8 = std::integral_constant<int, 8>;
  using P64 = std::integral_constant<int, OW_MAXP>;
  using T1 = std::true_type;
  using T0 = std::false_type;
  const bool small = nparts <= 8, two = vals2 != nullptr;
  if (vb == 8) {
    if (small) two ? launch(uint64_t{}, P8{}, T1{}) : launch(uint64_t{}, P8{}, T0{});
    else two ? launch(uint64_t{}, P64{}, T1{}) : launch(uint64_t{}, P64{}, T0{});
  } else {
    if (small) two ? launch(uint32_t{}, P8{}, T1{}) : launch(uint32_t{}, P8{}, T0{});
    else two ? launch(uint32_t{}, P64{}, T1{}) : launch(uint32_t{}, P64{}, T0{});
  }
  return hip_check(c, hipGetLastError(), "owner partition");
}

// ... with the per-owner totals read back (gs_window_reduce_partials: the caller runs the exchange)
gs_status owner_partition(gs_ctx* c, const int64_t* keys, const void* vals, size_t vb, const int64_t* vals2, uint64_t U,
                          uint32_t nparts, int64_t* okeys, void* ovals, int64_t* ovals2, uint64_t* counts_host) {
  GS_TRY(owner_partition_dev(c, keys, vals, vb, vals2, U, nparts, okeys, ovals, ovals2, nullptr));
  GS_HIP(hipMemcpyAsync(c->host_small + 8, c->dist_cnt.p, nparts * 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  memcpy(counts_host, c->host_small + 8, nparts * 8);
  return GS_OK;
}

// Exchange rows: key (1 u32 word when the sender's keys lie in [0, 2^32), else 2), value (vb / 4 words),
// [maximum (2 words)]: one row of u32 words, so the whole exchange is one grouped send / recv per peer.
// The receiver unpacks them by sender: segment q = rows [row0[q], row0[q + 1]) of the merge's input, from
// src[q] with sender q's key width (this rank's own segment straight from its send buffer: it does not
// travel)
struct RowSegs {
  const uint32_t* src[OW_MAXP];
  uint64_t row0[OW_MAXP + 1];
  uint32_t kw[OW_MAXP];
  uint32_t nseg;
};

__global__ __launch_bounds__(256) void k_unpack_rows(RowSegs segs, uint64_t n, int vw, int mw, int64_t* __restrict__ keys,
                                                     uint32_t* __restrict__ vals, int64_t* __restrict__ vals2) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t lo = 0, hi = segs.nseg - 1;   // the last segment q with row0[q] <= i
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (segs.row0[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  const uint32_t kw = segs.kw[lo];
  const uint32_t* r = segs.src[lo] + (i - segs.row0[lo]) * (kw + vw + mw);
  keys[i] = kw == 2 ? (int64_t)(((uint64_t)r[1] << 32) | r[0]) : (int64_t)(uint64_t)r[0];
  for (int j = 0; j < vw; ++j) vals[i * vw + j] = r[kw + j];
  if (mw) vals2[i] = (int64_t)(((uint64_t)r[kw + vw + 1] << 32) | r[kw + vw]);
}

}  // namespace gs

using namespace gs;

extern "C" {

uint32_t gs_owner_of(int64_t v, uint32_t nparts) { return nparts ? owner_of(v, nparts) : 0u; }

static gs_status check_partials_out(gs_ctx* c, const gs_partials_out* out, uint32_t nparts, bool two) {
  if (!out || !out->n_out || !out->owner_counts) return set_error(c, GS_EINVAL, "bad gs_partials_out");
  if (out->capacity && (!out->keys || !out->vals || (two && !out->vals2)))
    return set_error(c, GS_EINVAL, "bad gs_partials_out buffers");
  if (nparts < 1 || nparts > (uint32_t)OW_MAXP) return set_error(c, GS_EINVAL, "nparts %u outside [1, 64]", nparts);
  return GS_OK;
}

// local reduce into ctx staging, then the owner partition into the caller's buffers
static gs_status partials_impl(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, bool degmax, int64_t init_max,
                               uint32_t nparts, gs_partials_out* out) {
  GS_TRY(check_batch(c, b, dir));
  GS_TRY(check_partials_out(c, out, nparts, degmax));
  const uint64_t R = dir == GS_DIR_ALL ? 2 * b->n : b->n;
  if (nparts == 1) {   // one owner: the window's own output, in place (no partition pass)
    if (degmax) {
      gs_degree_out o{out->keys, (int64_t*)out->vals, out->vals2, out->capacity, out->n_out, out->mem, 0};
      GS_TRY(gs_window_fold_degree_max(c, b, dir, init_max, &o));
    } else {
      gs_vertex_out o{out->keys, out->vals, out->capacity, out->n_out, out->mem, 0};
      GS_TRY(gs_window_reduce(c, b, dir, op, &o));
    }
    out->owner_counts[0] = *out->n_out;
    return GS_OK;
  }
  GS_TRY(ensure(c, c->dist_k, R * 8 + 8));
  GS_TRY(ensure(c, c->dist_v, R * 8 + 8));
  if (degmax) GS_TRY(ensure(c, c->dist_v2, R * 8 + 8));
  uint64_t U = 0;
  size_t vb = 8;
  if (degmax) {
    gs_degree_out o{c->dist_k.as<int64_t>(), c->dist_v.as<int64_t>(), c->dist_v2.as<int64_t>(), R, &U, GS_MEM_DEVICE, 0};
    GS_TRY(gs_window_fold_degree_max(c, b, dir, init_max, &o));
  } else {
    vb = op == GS_OP_COUNT ? 8 : dtype_bytes(b->val_dtype);
    gs_vertex_out o{c->dist_k.as<int64_t>(), c->dist_v.p, R, &U, GS_MEM_DEVICE, 0};
    GS_TRY(gs_window_reduce(c, b, dir, op, &o));
  }
  const gs_stage_times keep = c->times;   // the window's own pipeline (the partition is not part of it)
  *out->n_out = U;
  const bool direct = out->mem == GS_MEM_DEVICE && out->capacity >= U;
  int64_t *ok = out->keys, *ov2 = out->vals2;
  void* ov = out->vals;
  if (!direct) {
    GS_TRY(ensure(c, c->dist_k2, U * 8 + 8));
    GS_TRY(ensure(c, c->dist_v3, U * 8 + 8));
    if (degmax) GS_TRY(ensure(c, c->dist_v4, U * 8 + 8));
    ok = c->dist_k2.as<int64_t>();
    ov = c->dist_v3.p;
    ov2 = degmax ? c->dist_v4.as<int64_t>() : nullptr;
  }
  GS_TRY(owner_partition(c, c->dist_k.as<int64_t>(), c->dist_v.p, vb, degmax ? c->dist_v2.as<int64_t>() : nullptr, U,
                         nparts, ok, ov, ov2, out->owner_counts));
  c->times = keep;
  if (U > out->capacity) return set_error(c, GS_ECAPACITY, "partials need %llu rows", (unsigned long long)U);
  if (!direct) {
    GS_TRY(deliver(c, out->keys, ok, U * 8, out->mem));
    GS_TRY(deliver(c, out->vals, ov, U * vb, out->mem));
    if (degmax) GS_TRY(deliver(c, out->vals2, ov2, U * 8, out->mem));
    GS_TRY(host_wait(c));
  }
  return GS_OK;
}

gs_status gs_window_reduce_partials(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, uint32_t nparts,
                                    gs_partials_out* out) {
  if (!c) return GS_EINVAL;
  if (op < GS_OP_SUM || op > GS_OP_COUNT) return set_error(c, GS_EINVAL, "bad op %d", op);
  return partials_impl(c, b, dir, op, false, 0, nparts, out);
}

gs_status gs_window_fold_degree_max_partials(gs_ctx* c, const gs_edge_batch* b, int32_t dir, uint32_t nparts,
                                             gs_partials_out* out) {
  if (!c) return GS_EINVAL;
  return partials_impl(c, b, dir, 0, true, INT64_MIN, nparts, out);
}

// the merges run the bucket path on received rows: their own speculative-partition slot (gs_internal.hpp)
struct SpMergeSlot {
  gs_ctx* c;
  explicit SpMergeSlot(gs_ctx* cc) : c(cc) { c->sp_slot = 1; }
  ~SpMergeSlot() { c->sp_slot = 0; }
};

gs_status gs_merge_partials(gs_ctx* c, const gs_partial_batch* p, int32_t op, const void* init, gs_vertex_out* out) {
  if (!c) return GS_EINVAL;
  SpMergeSlot slot(c);
  if (!p || (p->n && (!p->keys || !p->vals))) return set_error(c, GS_EINVAL, "bad gs_partial_batch");
  if (op < GS_OP_SUM || op > GS_OP_COUNT) return set_error(c, GS_EINVAL, "bad op %d", op);
  const int32_t mop = op == GS_OP_COUNT ? GS_OP_SUM : op;            // counts merge by SUM
  const int32_t dt = op == GS_OP_COUNT ? GS_I64 : p->val_dtype;
  const gs_edge_batch b{p->keys, p->keys, p->vals, p->n, dt, p->mem, 0};
  return init ? gs_window_fold(c, &b, GS_DIR_OUT, mop, init, out) : gs_window_reduce(c, &b, GS_DIR_OUT, mop, out);
}

gs_status gs_merge_degree_max_partials(gs_ctx* c, const gs_partial_batch* p, int64_t init_max, gs_degree_out* out) {
  if (!c) return GS_EINVAL;
  SpMergeSlot slot(c);
  if (!p || (p->n && (!p->keys || !p->vals || !p->vals2))) return set_error(c, GS_EINVAL, "bad gs_partial_batch");
  if (!out || !out->n_out || (out->capacity && (!out->keys || !out->degree || !out->max_neighbor)))
    return set_error(c, GS_EINVAL, "bad gs_degree_out");
  // both merges write the ctx's output staging (device), then the rows go to the caller
  const uint64_t n = p->n;
  GS_TRY(ensure(c, c->out_keys, n * 8 + 8));
  GS_TRY(ensure(c, c->out_a, n * 8 + 8));
  GS_TRY(ensure(c, c->out_b, n * 8 + 8));
  const gs_edge_batch bd{p->keys, p->keys, p->vals, n, GS_I64, p->mem, 0};
  const gs_edge_batch bm{p->keys, p->keys, p->vals2, n, GS_I64, p->mem, 0};
  uint64_t U = 0;
  gs_vertex_out od{c->out_keys.as<int64_t>(), c->out_a.p, n, &U, GS_MEM_DEVICE, 0};
  GS_TRY(gs_window_reduce(c, &bd, GS_DIR_OUT, GS_OP_SUM, &od));            // degrees add
  gs_vertex_out om{c->out_keys.as<int64_t>(), c->out_b.p, n, &U, GS_MEM_DEVICE, 0};
  GS_TRY(gs_window_fold(c, &bm, GS_DIR_OUT, GS_OP_MAX, &init_max, &om));   // maxima, then the fold's init
  *out->n_out = U;
  c->last_U = U;
  c->last_ob = 8;
  c->last_kind = 2;
  if (U > out->capacity) return set_error(c, GS_ECAPACITY, "output needs %llu vertices", (unsigned long long)U);
  GS_TRY(deliver(c, out->keys, c->out_keys.as<int64_t>(), U * 8, out->mem));
  GS_TRY(deliver(c, out->degree, c->out_a.p, U * 8, out->mem));
  GS_TRY(deliver(c, out->max_neighbor, c->out_b.p, U * 8, out->mem));
  return host_wait(c);
}

// A/B switch: GS_DIST_NO_DEFER=1 waits for the local window's read-back before the counts exchange
static bool dist_no_defer() {
  static const bool v = getenv("GS_DIST_NO_DEFER") && getenv("GS_DIST_NO_DEFER")[0] == '1';
  return v;
}

// partials of this rank's slice -> all-to-all over the ctx's communicator -> the merge of what this
// rank owns.  Per window: the local reduce (the bucket path's own read-back), the owner partition on the
// device straight into packed rows, ONE all-to-all of [rows, flags] per peer read back together (the only
// host wait of the exchange: sizes, each sender's key width, and every rank's status -- a rank whose local
// step failed still joins it with the failure flag, so all ranks return an error together instead of
// the others blocking in a collective), one packed all-to-all of the rows (4-byte keys from a sender whose
// keys all fit; a rank's own rows stay in place), the unpack by sender, then the merge.  One rank: the
// window's own output (no exchange, no merge).
static gs_status dist_body(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, const void* init, bool degmax,
                           int64_t init_max, gs_vertex_out* vout, gs_degree_out* dout);
static gs_status dist_impl(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, const void* init, bool degmax,
                           int64_t init_max, gs_vertex_out* vout, gs_degree_out* dout) {
  // The owner-grouped emit (c->oe) is set for this call's local window only: whatever way the call leaves
  // (a failed counts exchange with a deferred window still pending included), the next plain window of
  // this ctx must not find it set and write exchange rows instead of its output.
  struct OeReset {
    gs_ctx* c;
    ~OeReset() { c->oe = OwnerEmit{}; }
  } guard{c};
  return dist_body(c, b, dir, op, init, degmax, init_max, vout, dout);
}
static gs_status dist_body(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, const void* init, bool degmax,
                           int64_t init_max, gs_vertex_out* vout, gs_degree_out* dout) {
  if (!c->comm) return set_error(c, GS_EINVAL, "no communicator (gs_comm_init)");
  const uint32_t P = (uint32_t)c->comm_size;
  if (P == 1 && !(c->flags & GS_FLAG_TEST_FORCE_EXCHANGE)) {   // the only rank owns every vertex
    if (degmax) return gs_window_fold_degree_max(c, b, dir, init_max, dout);
    return init ? gs_window_fold(c, b, dir, op, init, vout) : gs_window_reduce(c, b, dir, op, vout);
  }
  const uint64_t R = dir == GS_DIR_ALL ? 2 * b->n : b->n;
  const size_t vb = degmax ? 8 : (op == GS_OP_COUNT ? 8 : dtype_bytes(b->val_dtype));
  GS_TRY(ensure(c, c->dist_x, 64 + (size_t)P * 32, true));   // (zeroed when allocated: the key-width flag)
  auto* wide = c->dist_x.as<unsigned long long>();
  auto* sendc = wide + 8;
  auto* recvc = sendc + 2 * P;
  // 1. local partials, written by the bucket path's last stage straight as the exchange's rows grouped by
  //    owner (OwnerEmit); a window that takes another path (sort path, chunks) leaves the ascending output,
  //    which the owner partition turns into the rows.  A failure is carried into the counts exchange.
  uint64_t U = 0;
  gs_status local = GS_OK;
  std::string local_err;
  const int vw = (int)(vb / 4), mw = degmax ? 2 : 0;
  bool emitted = false, pending = false;
  auto run_local = [&]() -> gs_status {
    if (degmax) {
      gs_degree_out o{c->dist_k.as<int64_t>(), c->dist_v.as<int64_t>(), c->dist_v2.as<int64_t>(), R, &U, GS_MEM_DEVICE, 0};
      return gs_window_fold_degree_max(c, b, dir, INT64_MIN, &o);
    }
    gs_vertex_out o{c->dist_k.as<int64_t>(), c->dist_v.p, R, &U, GS_MEM_DEVICE, 0};
    return gs_window_reduce(c, b, dir, op, &o);
  };
  {
    local = ensure(c, c->dist_k, R * 8 + 8);
    if (local == GS_OK) local = ensure(c, c->dist_v, R * 8 + 8);
    if (local == GS_OK && degmax) local = ensure(c, c->dist_v2, R * 8 + 8);
    // the packed rows this rank sends (room for 2-word keys: the width is picked on the device)
    if (local == GS_OK) local = ensure(c, c->dist_k2, R * (size_t)(2 + vw + mw) * 4 + 16);
    if (local == GS_OK) local = ensure(c, c->dist_cnt, 1024 + (size_t)OW_MAXP * BK_MAXB_DIST * BK_OE_SLICES_DIST * 4);
    if (local == GS_OK) {
      c->oe = OwnerEmit{};
      c->oe.nparts = P;
      c->oe.rows = c->dist_k2.as<uint32_t>();
      c->oe.cnt = (uint32_t*)(c->dist_cnt.as<char>() + 1024);
      c->oe.totals = c->dist_cnt.as<unsigned long long>();
      c->oe.wide = wide;
      c->oe.vw = vw;
      c->oe.mw = mw;
      c->oe.send = sendc;
      // a speculative window's read-back is left to the counts exchange's wait (device columns only: a
      // resumed call must not stage host columns again); its miss and timeout words ride in the flags
      c->oe.defer = b->mem == GS_MEM_DEVICE && !dist_no_defer();
      local = run_local();
      if (local == GS_PENDING_LOCAL) {
        pending = true;
        local = GS_OK;
      }
    }
    emitted = c->oe.done;
    if (!pending) c->oe = OwnerEmit{};
  }
  gs_stage_times keep = c->times;   // the local window's (a deferred one's after its resume, below)
  // the send rows (owner partition of the ascending output when the window did not emit rows itself), or
  // zero rows for everyone with the failure flag
  auto prepare_send = [&]() -> gs_status {
    if (local == GS_OK && !emitted)
      local = owner_partition_dev(c, c->dist_k.as<int64_t>(), c->dist_v.p, vb, degmax ? c->dist_v2.as<int64_t>() : nullptr,
                                  U, P, nullptr, nullptr, nullptr, wide, c->dist_k2.as<uint32_t>());
    if (local == GS_OK && !emitted) {   // (the owner-grouped emit launched it already)
      hipLaunchKernelGGL(k_send_rows, dim3(1), dim3(64), 0, c->stream, (const unsigned long long*)c->dist_cnt.as<unsigned long long>(),
                         wide, P, sendc, (const unsigned long long*)nullptr, (const uint32_t*)nullptr);
      local = hip_check(c, hipGetLastError(), "k_send_rows");
    }
    if (local != GS_OK) {
      local_err = c->err;
      for (uint32_t p = 0; p < P; ++p) {
        c->host_small[8 + 2 * p] = 0;
        c->host_small[9 + 2 * p] = 2;
      }
      GS_HIP(hipMemcpyAsync(sendc, c->host_small + 8, (size_t)P * 16, hipMemcpyHostToDevice, c->stream));
    }
    return GS_OK;
  };
  // the exchange of sizes + flags; read back with this rank's own send counts (with a deferred window, this
  // wait also brings back its read-back block)
  auto exchange_counts = [&]() -> gs_status {
    GS_TRY(comm_alltoall(c, sendc, recvc, 2, NCCL_T_U64));
    GS_HIP(hipMemcpyAsync(c->host_small + 8, sendc, (size_t)P * 32, hipMemcpyDeviceToHost, c->stream));
    return host_wait(c);
  };
  // 2. the counts exchange
  GS_TRY(prepare_send());
  GS_TRY(exchange_counts());
  if (pending) {   // the deferred window: its checks now (a missed speculation reruns it, which waits inside)
    c->oe.resume = true;
    local = run_local();
    emitted = c->oe.done;
    c->oe = OwnerEmit{};
    keep = c->times;
  }
  bool redo = false;
  for (uint32_t p = 0; p < P; ++p) redo |= (c->host_small[8 + 2 * P + 2 * p + 1] & 4) != 0;
  if (redo) {   // some rank's window missed its speculation: every rank sends its counts again
    const bool mine_missed = (c->host_small[9] & 4) != 0;
    if (mine_missed || local != GS_OK) GS_TRY(prepare_send());   // (the others' send rows stand)
    GS_TRY(exchange_counts());
  }
  const uint32_t me = (uint32_t)c->comm_rank;
  std::vector<uint64_t> send_b(P), recv_b(P);
  RowSegs segs{};
  segs.nseg = P;
  int failed = -1;
  uint64_t nrecv = 0, so = 0, ro = 0;
  const uint32_t kw_me = (c->host_small[9] & 1) ? 2u : 1u;   // (every send flag carries this rank's width)
  if (local != GS_OK && local_err.empty()) local_err = c->err;
  for (uint32_t p = 0; p < P; ++p) {
    const uint64_t fl = c->host_small[8 + 2 * P + 2 * p + 1];
    if ((fl & 2) && failed < 0) failed = (int)p;
  }
  if (local != GS_OK) return set_error(c, local, "%s", local_err.c_str());
  if (failed >= 0) return set_error(c, GS_ECOMM, "rank %d failed its local step of the window", failed);
  const uint32_t* sendrows = c->dist_k2.as<uint32_t>();
  for (uint32_t p = 0; p < P; ++p) {
    const uint64_t sn = c->host_small[8 + 2 * p], rn = c->host_small[8 + 2 * P + 2 * p];
    const uint32_t kw = (c->host_small[8 + 2 * P + 2 * p + 1] & 1) ? 2u : 1u;
    segs.row0[p] = nrecv;
    segs.kw[p] = kw;
    if (p == me) segs.src[p] = sendrows + so * (kw_me + vw + mw);   // own rows: read where the partition wrote them
    send_b[p] = sn * (kw_me + vw + mw) * 4;
    recv_b[p] = rn * (kw + vw + mw) * 4;
    so += sn;
    nrecv += rn;
  }
  segs.row0[P] = nrecv;
  uint64_t recv_bytes = 0;
  for (uint32_t p = 0; p < P; ++p) recv_bytes += p == me ? 0 : recv_b[p];
  // 3. one exchange of the packed rows (bytes; nothing to or from this rank itself)
  GS_TRY(ensure(c, c->dist_x2, recv_bytes + 16));
  GS_TRY(exchange_rows(c, c->dist_k2.as<char>(), send_b.data(), c->dist_x2.as<char>(), recv_b.data(), 1, true));
  for (uint32_t p = 0; p < P; ++p) {
    if (p == me) continue;
    segs.src[p] = c->dist_x2.as<uint32_t>() + ro / 4;
    ro += recv_b[p];
  }
  // unpacked merge input: the local partials are consumed, their buffers take it
  GS_TRY(ensure(c, c->dist_k, nrecv * 8 + 8));
  GS_TRY(ensure(c, c->dist_v, nrecv * vb + 8));
  if (degmax) GS_TRY(ensure(c, c->dist_v2, nrecv * 8 + 8));
  if (nrecv) {
    hipLaunchKernelGGL(k_unpack_rows, dim3((unsigned)((nrecv + 255) / 256)), dim3(256), 0, c->stream, segs, nrecv, vw, mw,
                       c->dist_k.as<int64_t>(), c->dist_v.as<uint32_t>(), degmax ? c->dist_v2.as<int64_t>() : nullptr);
    GS_HIP(hipGetLastError());
  }
  // 4. the merge of what this rank owns
  const int32_t pdt = degmax || op == GS_OP_COUNT ? GS_I64 : b->val_dtype;
  const gs_partial_batch pb{c->dist_k.as<int64_t>(), c->dist_v.p, degmax ? c->dist_v2.as<int64_t>() : nullptr, nrecv,
                            pdt, GS_MEM_DEVICE};
  const int timing = c->timing;   // the merge's stage times are not reported (the window's are): no events
  c->timing = GS_TIMING_OFF;
  gs_status st = degmax ? gs_merge_degree_max_partials(c, &pb, init_max, dout) : gs_merge_partials(c, &pb, op, init, vout);
  c->timing = timing;
  c->times = keep;
  return st;
}

gs_status gs_window_reduce_dist(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int32_t op, const void* init,
                                gs_vertex_out* out) {
  if (!c) return GS_EINVAL;
  if (op < GS_OP_SUM || op > GS_OP_COUNT) return set_error(c, GS_EINVAL, "bad op %d", op);
  GS_TRY(check_batch(c, b, dir));
  return dist_impl(c, b, dir, op, init, false, 0, out, nullptr);
}

gs_status gs_window_fold_degree_max_dist(gs_ctx* c, const gs_edge_batch* b, int32_t dir, int64_t init_max,
                                         gs_degree_out* out) {
  if (!c) return GS_EINVAL;
  GS_TRY(check_batch(c, b, dir));
  return dist_impl(c, b, dir, 0, nullptr, true, init_max, nullptr, out);
}

}  // extern "C"
