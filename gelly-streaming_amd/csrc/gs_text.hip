// gs_text.hip — the examples' edge text input on the device:
//   env.readTextFile(path).map(s -> { fields = s.split("\\s"); Long.parseLong(fields[0..2]) })
//   (example/WindowTriangles.java:175-185; ConnectedComponentsExample.java:113-115)
// Record rules (Flink 1.0.3 TextInputFormat + Java String.split / Long.parseLong) are restated in
// oracle/gs_oracle.c (gso_parse_edges_text), the checker of this file.
//
// HBM-bound passes over the bytes, no sort:
//   k_tx_count   newlines per 16 KiB tile (16-byte loads, one tile per 256-thread block)
//   k_tx_scan    exclusive scan of the tile counts (one block, coalesced 1024-wide chunks)
//   k_tx_starts  record start offsets (u32): tile offset + in-tile rank of each newline
//   k_tx_parse   256 records per block: their text span staged in LDS with coalesced word loads,
//                one record per thread: three fields, Java parseLong overflow rules; the first
//                malformed record index goes to an atomicMin
#include "gs_ops.hpp"

using namespace gs;

namespace {

constexpr int TX_BLOCK = 256;
constexpr int TX_VEC = 4;                              // 16-byte loads per thread per tile
constexpr uint32_t TX_TILE = TX_BLOCK * 16 * TX_VEC;   // 16 KiB per block
constexpr uint32_t TX_LDS_WORDS = 4096;                // 16 KiB of record text per 256 records

__device__ __forceinline__ uint32_t nl_mask16(uint4 v, uint64_t valid) {
  // bit j set when byte j of the 16 is '\n' and j < valid
  uint32_t m = 0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int b = 0; b < 4; ++b) m |= (((w[k] >> (8 * b)) & 0xFFu) == '\n' ? 1u : 0u) << (4 * k + b);
  }
  return valid >= 16 ? m : (m & ((1u << valid) - 1u));
}

// newline masks of this thread's 4 x 16 bytes of the tile (bytes past the end are masked out; the
// base is 16-byte aligned, so a load never leaves the text's last 16-byte granule)
__device__ __forceinline__ void tile_masks(const uint8_t* t, uint64_t bytes, uint64_t tile0, uint32_t (&m)[TX_VEC]) {
  uint4 v[TX_VEC];
#pragma unroll
  for (int u = 0; u < TX_VEC; ++u) {
    const uint64_t off = min(tile0 + ((uint64_t)u * TX_BLOCK + threadIdx.x) * 16, (bytes - 1) & ~15ull);
    v[u] = *reinterpret_cast<const uint4*>(t + off);
  }
#pragma unroll
  for (int u = 0; u < TX_VEC; ++u) {
    const uint64_t off = tile0 + ((uint64_t)u * TX_BLOCK + threadIdx.x) * 16;
    m[u] = off < bytes ? nl_mask16(v[u], bytes - off) : 0u;
  }
}

__global__ __launch_bounds__(TX_BLOCK) void k_tx_count(const uint8_t* __restrict__ t, uint64_t bytes,
                                                       uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s[TX_BLOCK / 64];
  uint32_t m[TX_VEC];
  tile_masks(t, bytes, (uint64_t)blockIdx.x * TX_TILE, m);
  uint32_t c = 0;
#pragma unroll
  for (int u = 0; u < TX_VEC; ++u) c += __popc(m[u]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// inclusive scan of one value per thread over a 1024-thread block (wave shuffles + 16 wave totals)
__device__ __forceinline__ uint32_t block_incl_scan1024(uint32_t v, uint32_t* sw, uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) sw[w] = v;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t x = sw[i];
    before += i < w ? x : 0u;
    total += x;
  }
  __syncthreads();
  return v + before;
}

// exclusive scan in place over nt tile counts (coalesced 1024-wide chunks with a carry); total at cnt[nt]
__global__ __launch_bounds__(1024) void k_tx_scan(uint32_t* __restrict__ cnt, uint32_t nt) {
  __shared__ uint32_t sw[16];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nt; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < nt ? cnt[i] : 0u;
    uint32_t total;
    const uint32_t incl = block_incl_scan1024(v, sw, total);
    if (i < nt) cnt[i] = carry + incl - v;
    carry += total;
  }
  if (threadIdx.x == 0) cnt[nt] = carry;
}

// starts[k + 1] = (byte offset of the k-th newline) + 1
__global__ __launch_bounds__(TX_BLOCK) void k_tx_starts(const uint8_t* __restrict__ t, uint64_t bytes,
                                                        const uint32_t* __restrict__ cnt,
                                                        uint32_t* __restrict__ starts) {
  __shared__ uint32_t sw[TX_BLOCK / 64];
  const uint64_t tile0 = (uint64_t)blockIdx.x * TX_TILE;
  uint32_t m[TX_VEC];
  tile_masks(t, bytes, tile0, m);
  // rank order = byte order: u-major (all threads' u = 0 bytes precede u = 1), so scan per u
  uint32_t k = cnt[blockIdx.x];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < TX_VEC; ++u) {
    const uint32_t c = __popc(m[u]);
    uint32_t v = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    if (lane == 63) sw[w] = v;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int i = 0; i < TX_BLOCK / 64; ++i) {
      before += i < w ? sw[i] : 0u;
      total += sw[i];
    }
    __syncthreads();
    uint32_t r = k + before + v - c;
    uint32_t mm = m[u];
    const uint64_t off = tile0 + ((uint64_t)u * TX_BLOCK + threadIdx.x) * 16;
    while (mm) {
      const int j = __ffs(mm) - 1;
      mm &= mm - 1;
      starts[r + 1] = (uint32_t)(off + j + 1);
      ++r;
    }
    k += total;
  }
}

__device__ __forceinline__ bool tx_ws(uint32_t ch) {
  return ch == ' ' || ch == '\t' || ch == '\n' || ch == 0x0B || ch == '\f' || ch == '\r';
}

// One record as a branch-free state machine over its bytes: the byte loop's trip count is the only
// divergent control flow.  (Nested per-field loops with a word cache ran 750 us for 2^24 lines, bound
// by the scalar unit: ~1600 SALU instructions per wave for exec-mask bookkeeping.)
// Field k (< 3) ends at a whitespace byte or at the record end; a sign is allowed only as its first
// byte; an empty field, a non-digit or a value outside [-2^63, 2^63) fails (Long.parseLong).
template <typename ByteAt>
__device__ __forceinline__ bool parse_record(ByteAt at, uint32_t p0, uint32_t q, int64_t (&f)[3]) {
  if (q > p0 && at(q - 1) == '\r') --q;
  uint32_t k = 0;                 // current field
  uint64_t v = 0;
  bool neg = false, any = false, first = true, ok = true;
  int64_t f0 = 0, f1 = 0, f2 = 0;
  for (uint32_t p = p0; p < q; ++p) {
    const uint32_t ch = at(p);
    const bool live = k < 3;
    const bool ws = tx_ws(ch);
    const bool sign = first && (ch == '-' || ch == '+');
    const uint32_t d = ch - '0';
    // v * 10 + d must stay <= 2^63 - 1 (2^63 after '-'); compared against lim / 10 and lim % 10
    const bool over = v > 922337203685477580ull || (v == 922337203685477580ull && d > (neg ? 8u : 7u));
    const bool digit_ok = d <= 9 && !over;
    const int64_t val = neg ? (int64_t)(0 - v) : (int64_t)v;
    if (live && ws) {             // end of field k (predicated: straight-line selects)
      ok = ok && any;
      f0 = k == 0 ? val : f0;
      f1 = k == 1 ? val : f1;
      f2 = k == 2 ? val : f2;
    }
    if (live && !ws && !sign) ok = ok && digit_ok;
    const bool dig = live && !ws && !sign;
    v = ws ? 0 : (dig ? v * 10 + d : v);
    neg = ws ? false : (sign ? ch == '-' : neg);
    any = ws ? false : (any || dig);
    first = ws;
    k += (live && ws) ? 1u : 0u;
  }
  if (k < 3) {                    // the record ended inside field k
    ok = ok && any && k == 2;
    f2 = neg ? (int64_t)(0 - v) : (int64_t)v;
  }
  f[0] = f0;
  f[1] = f1;
  f[2] = f2;
  return ok;
}

// 256 records per block: their text span is copied into LDS with coalesced word loads (when it fits
// 16 KiB), then each thread parses its record from LDS
__global__ __launch_bounds__(TX_BLOCK) void k_tx_parse(const uint8_t* __restrict__ t, uint64_t bytes,
                                                       const uint32_t* __restrict__ starts, uint32_t nl,
                                                       uint32_t nrec, int64_t* __restrict__ src,
                                                       int64_t* __restrict__ dst, int64_t* __restrict__ ts,
                                                       unsigned long long* __restrict__ bad) {
  __shared__ uint32_t tx_lds[TX_LDS_WORDS];
  uint32_t* lds = tx_lds;
  const uint32_t r0 = blockIdx.x * TX_BLOCK, i = r0 + threadIdx.x;
  const uint32_t rl = min(nrec, r0 + TX_BLOCK);            // records [r0, rl)
  const uint64_t span0 = starts[r0], span1 = rl <= nl ? (uint64_t)starts[rl] : bytes;
  const uint64_t w0 = span0 >> 2, w1 = (span1 + 3) >> 2;
  const uint32_t* gw = reinterpret_cast<const uint32_t*>(t);
  const bool staged = w1 - w0 <= TX_LDS_WORDS;
  if (staged && w1 > w0) {
    // all loads first (clamped, unconditional), then the LDS stores: a load inside the guarded
    // loop would be waited for before the next one is issued
    constexpr int U = TX_LDS_WORDS / TX_BLOCK;
    uint32_t x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = gw[min(w0 + (uint64_t)u * TX_BLOCK + threadIdx.x, w1 - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = (uint32_t)u * TX_BLOCK + threadIdx.x;
      if (k < w1 - w0) lds[k] = x[u];
    }
  }
  __syncthreads();
  if (i >= nrec) return;
  const uint64_t p0 = starts[i];
  const uint64_t q = i < nl ? (uint64_t)starts[i + 1] - 1 : bytes;   // record excludes its '\n'
  int64_t f[3];
  bool ok;
  if (staged) {   // uniform over the block
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(tx_lds) - (w0 << 2);
    ok = parse_record([lb](uint32_t p) { return (uint32_t)lb[p]; }, (uint32_t)p0, (uint32_t)q, f);
  } else {
    ok = parse_record([t](uint32_t p) { return (uint32_t)t[p]; }, (uint32_t)p0, (uint32_t)q, f);
  }
  if (!ok) {
    atomicMin(bad, (unsigned long long)i);
    return;
  }
  src[i] = f[0];
  dst[i] = f[1];
  ts[i] = f[2];
}

}  // namespace

extern "C" gs_status gs_parse_edges_text(gs_ctx* c, const char* text, uint64_t bytes, int32_t in_mem,
                                         int64_t* src, int64_t* dst, int64_t* ts, uint64_t capacity,
                                         int32_t out_mem, uint64_t* n_out, uint64_t* bad_record) {
  if (!c) return GS_EINVAL;
  if (!n_out || !bad_record || (bytes && !text) || (capacity && (!src || !dst || !ts)))
    return set_error(c, GS_EINVAL, "parse_edges_text: null argument");
  if ((in_mem != GS_MEM_HOST && in_mem != GS_MEM_DEVICE) || (out_mem != GS_MEM_HOST && out_mem != GS_MEM_DEVICE))
    return set_error(c, GS_EINVAL, "parse_edges_text: bad mem");
  if (bytes >= (1ull << 32) - 16) return set_error(c, GS_EINVAL, "parse_edges_text: text of 4 GiB or more");
  *n_out = 0;
  *bad_record = ~0ull;
  GS_HIP(hipSetDevice(c->device));
  GS_TRY(begin_call(c));
  if (bytes == 0) return GS_OK;
  // device text with a 16-byte aligned base is read in place (16-byte and word loads never leave its
  // last 16-byte granule); host or unaligned text is staged into an aligned buffer first
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  if (in_mem == GS_MEM_HOST || (reinterpret_cast<uintptr_t>(text) & 15)) {
    GS_TRY(ensure(c, c->tx_text, bytes + 32));
    GS_HIP(hipMemcpyAsync(c->tx_text.p, text, bytes, in_mem == GS_MEM_HOST ? hipMemcpyHostToDevice
                                                                            : hipMemcpyDeviceToDevice, c->stream));
    t = c->tx_text.as<uint8_t>();
  }
  const uint32_t nt = (uint32_t)((bytes + TX_TILE - 1) / TX_TILE);
  GS_TRY(ensure(c, c->tx_cnt, ((uint64_t)nt + 1) * 4));
  uint32_t* cnt = c->tx_cnt.as<uint32_t>();
  hipLaunchKernelGGL(k_tx_count, dim3(nt), dim3(TX_BLOCK), 0, c->stream, t, bytes, cnt);
  GS_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_tx_scan, dim3(1), dim3(1024), 0, c->stream, cnt, nt);
  GS_HIP(hipGetLastError());
  uint32_t h[2] = {0, 0};
  uint8_t last = 0;
  GS_HIP(hipMemcpyAsync(h, cnt + nt, 4, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipMemcpyAsync(&last, t + bytes - 1, 1, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  const uint32_t nl = h[0];
  const uint64_t nrec = (uint64_t)nl + (last != '\n' ? 1 : 0);
  *n_out = nrec;
  if (nrec > capacity) return set_error(c, GS_ECAPACITY, "parse_edges_text: %llu records", (unsigned long long)nrec);
  GS_TRY(ensure(c, c->tx_starts, ((uint64_t)nl + 2) * 4));
  uint32_t* starts = c->tx_starts.as<uint32_t>();
  GS_HIP(hipMemsetAsync(starts, 0, 4, c->stream));
  hipLaunchKernelGGL(k_tx_starts, dim3(nt), dim3(TX_BLOCK), 0, c->stream, t, bytes, cnt, starts);
  GS_HIP(hipGetLastError());
  int64_t *s = src, *d = dst, *w = ts;
  if (out_mem == GS_MEM_HOST) {
    GS_TRY(ensure(c, c->out_keys, nrec * 8));
    GS_TRY(ensure(c, c->out_a, nrec * 8));
    GS_TRY(ensure(c, c->out_b, nrec * 8));
    s = c->out_keys.as<int64_t>();
    d = c->out_a.as<int64_t>();
    w = c->out_b.as<int64_t>();
  }
  GS_TRY(ensure(c, c->pr_small, 64));
  unsigned long long* bad = c->pr_small.as<unsigned long long>();
  GS_HIP(hipMemsetAsync(bad, 0xFF, 8, c->stream));
  hipLaunchKernelGGL(k_tx_parse, dim3((uint32_t)((nrec + TX_BLOCK - 1) / TX_BLOCK)), dim3(TX_BLOCK), 0,
                     c->stream, t,
                     bytes, starts, nl, (uint32_t)nrec, s, d, w, bad);
  GS_HIP(hipGetLastError());
  uint64_t hb = 0;
  GS_HIP(hipMemcpyAsync(&hb, bad, 8, hipMemcpyDeviceToHost, c->stream));
  GS_TRY(host_wait(c));
  if (hb != ~0ull) {
    *bad_record = hb;
    return set_error(c, GS_EINVAL, "parse_edges_text: malformed edge record %llu (Long.parseLong would throw)",
                     (unsigned long long)hb);
  }
  if (out_mem == GS_MEM_HOST) {
    GS_HIP(hipMemcpyAsync(src, s, nrec * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(dst, d, nrec * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(ts, w, nrec * 8, hipMemcpyDeviceToHost, c->stream));
    GS_TRY(host_wait(c));
  }
  return GS_OK;
}
