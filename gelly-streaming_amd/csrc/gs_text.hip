// gs_text.hip — the examples' edge text input on the device:
//   env.readTextFile(path).map(s -> { fields = s.split("\\s"); Long.parseLong(fields[0..2]) })
//   (example/WindowTriangles.java:175-185; ConnectedComponentsExample.java:113-115)
// Record rules (Flink 1.0.3 TextInputFormat + Java String.split / Long.parseLong) are restated in
// oracle/gs_oracle.c (gso_parse_edges_text), the checker of this file.
//
// Three HBM-bound passes over the bytes, no sort:
//   k_tx_count   newlines per 4 KiB tile (16-byte loads, one tile per 256-thread block)
//   k_tx_scan    exclusive scan of the tile counts (one block)
//   k_tx_starts  record start offsets (u32): tile offset + in-tile rank of each newline
//   k_tx_parse   one record per thread: three fields, Java parseLong overflow rules; the first
//                malformed record index goes to an atomicMin
#include "gs_ops.hpp"

using namespace gs;

namespace {

constexpr int TX_BLOCK = 256;
constexpr uint32_t TX_TILE = TX_BLOCK * 16;   // bytes per block

__device__ __forceinline__ uint32_t nl_mask16(uint4 v, uint32_t valid) {
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

__device__ __forceinline__ uint4 load16(const uint8_t* t, uint64_t bytes, uint64_t off) {
  // bytes past the end read as 0 (the buffer is staged with 16 bytes of padding)
  return *reinterpret_cast<const uint4*>(t + off);
}

__global__ __launch_bounds__(TX_BLOCK) void k_tx_count(const uint8_t* __restrict__ t, uint64_t bytes,
                                                       uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s[TX_BLOCK / 64];
  const uint64_t off = (uint64_t)blockIdx.x * TX_TILE + threadIdx.x * 16;
  uint32_t c = 0;
  if (off < bytes) c = __popc(nl_mask16(load16(t, bytes, off), (uint32_t)min<uint64_t>(16, bytes - off)));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// exclusive scan in place over nt tile counts; total at cnt[nt]
__global__ __launch_bounds__(1024) void k_tx_scan(uint32_t* __restrict__ cnt, uint32_t nt) {
  __shared__ uint32_t s[1024];
  const uint32_t per = (nt + 1023) / 1024, i0 = min(nt, threadIdx.x * per), i1 = min(nt, i0 + per);
  uint32_t sum = 0;
  for (uint32_t i = i0; i < i1; ++i) sum += cnt[i];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t v = threadIdx.x >= (uint32_t)o ? s[threadIdx.x - o] : 0u;
    __syncthreads();
    s[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - sum;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t v = cnt[i];
    cnt[i] = run;
    run += v;
  }
  if (threadIdx.x == 1023) cnt[nt] = s[1023];
}

// starts[k + 1] = (byte offset of the k-th newline) + 1
__global__ __launch_bounds__(TX_BLOCK) void k_tx_starts(const uint8_t* __restrict__ t, uint64_t bytes,
                                                        const uint32_t* __restrict__ cnt,
                                                        uint32_t* __restrict__ starts) {
  __shared__ uint32_t s[TX_BLOCK];
  const uint64_t off = (uint64_t)blockIdx.x * TX_TILE + threadIdx.x * 16;
  uint32_t m = 0;
  if (off < bytes) m = nl_mask16(load16(t, bytes, off), (uint32_t)min<uint64_t>(16, bytes - off));
  const uint32_t c = __popc(m);
  s[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < TX_BLOCK; o <<= 1) {
    const uint32_t v = threadIdx.x >= (uint32_t)o ? s[threadIdx.x - o] : 0u;
    __syncthreads();
    s[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t k = cnt[blockIdx.x] + s[threadIdx.x] - c;
  while (m) {
    const int j = __ffs(m) - 1;
    m &= m - 1;
    starts[k + 1] = (uint32_t)(off + j + 1);
    ++k;
  }
}

__device__ __forceinline__ bool tx_ws(uint32_t ch) {
  return ch == ' ' || ch == '\t' || ch == '\n' || ch == 0x0B || ch == '\f' || ch == '\r';
}

// byte reader over one record with a one-word cache: ~1 dword load per 4 bytes
struct ByteReader {
  const uint32_t* w;
  uint64_t cur = ~0ull;
  uint32_t word = 0;
  __device__ uint32_t operator()(uint64_t p) {
    const uint64_t wi = p >> 2;
    if (wi != cur) {
      cur = wi;
      word = w[wi];
    }
    return (word >> (8 * (p & 3))) & 0xFFu;
  }
};

__global__ __launch_bounds__(TX_BLOCK) void k_tx_parse(const uint8_t* __restrict__ t, uint64_t bytes,
                                                       const uint32_t* __restrict__ starts, uint32_t nl,
                                                       uint32_t nrec, int64_t* __restrict__ src,
                                                       int64_t* __restrict__ dst, int64_t* __restrict__ ts,
                                                       unsigned long long* __restrict__ bad) {
  const uint32_t i = blockIdx.x * TX_BLOCK + threadIdx.x;
  if (i >= nrec) return;
  const uint64_t p0 = starts[i];
  uint64_t q = i < nl ? (uint64_t)starts[i + 1] - 1 : bytes;   // record excludes its '\n'
  ByteReader rd{reinterpret_cast<const uint32_t*>(t)};
  if (q > p0 && rd(q - 1) == '\r') --q;
  int64_t f[3] = {0, 0, 0};
  bool ok = true;
  uint64_t at = p0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    uint64_t p = at;
    bool neg = false, any = false;
    uint64_t v = 0;
    if (p < q) {
      const uint32_t ch = rd(p);
      if (ch == '-' || ch == '+') {
        neg = ch == '-';
        ++p;
      }
    }
    const uint64_t lim = neg ? (1ull << 63) : (1ull << 63) - 1;
    for (; p < q; ++p) {
      const uint32_t ch = rd(p);
      if (tx_ws(ch)) break;
      const uint32_t d = ch - '0';
      if (d > 9 || v > (lim - d) / 10) ok = false;
      v = v * 10 + d;
      any = true;
    }
    ok = ok && any;
    f[k] = neg ? (int64_t)(0 - v) : (int64_t)v;
    at = p + 1;
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
  // staged copy: 16-byte aligned, zero padding after the text (the tile loads read whole 16 bytes)
  GS_TRY(ensure(c, c->tx_text, bytes + 32));
  GS_HIP(hipMemsetAsync(c->tx_text.as<uint8_t>() + (bytes & ~15ull), 0, 32, c->stream));
  GS_HIP(hipMemcpyAsync(c->tx_text.p, text, bytes, in_mem == GS_MEM_HOST ? hipMemcpyHostToDevice
                                                                          : hipMemcpyDeviceToDevice, c->stream));
  const uint8_t* t = c->tx_text.as<uint8_t>();
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
  GS_HIP(hipStreamSynchronize(c->stream));
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
  hipLaunchKernelGGL(k_tx_parse, dim3((uint32_t)((nrec + TX_BLOCK - 1) / TX_BLOCK)), dim3(TX_BLOCK), 0, c->stream, t,
                     bytes, starts, nl, (uint32_t)nrec, s, d, w, bad);
  GS_HIP(hipGetLastError());
  uint64_t hb = 0;
  GS_HIP(hipMemcpyAsync(&hb, bad, 8, hipMemcpyDeviceToHost, c->stream));
  GS_HIP(hipStreamSynchronize(c->stream));
  if (hb != ~0ull) {
    *bad_record = hb;
    return set_error(c, GS_EINVAL, "parse_edges_text: malformed edge record %llu (Long.parseLong would throw)",
                     (unsigned long long)hb);
  }
  if (out_mem == GS_MEM_HOST) {
    GS_HIP(hipMemcpyAsync(src, s, nrec * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(dst, d, nrec * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipMemcpyAsync(ts, w, nrec * 8, hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipStreamSynchronize(c->stream));
  }
  return GS_OK;
}
