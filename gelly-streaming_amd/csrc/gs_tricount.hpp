// gs_tricount.hpp — the counting step of WindowTriangles (gs_graph.hip):
//   T = sum over u of sum over v in N+(u) of |N+(v) ∩ N+(u)|
// on the (degree, id)-oriented CSR: u's out-neighbours are onbr[pos[rowstart[u]] .. pos[rowstart[u] +
// deg[u]]), sorted, deduplicated.
//
// Vertex-centric and work-balanced: a wave takes a vertex u, puts N+(u) into an LDS hash set, then
// spreads the concatenation of N+(v) over v in N+(u) across its 64 lanes (prefix of |N+(v)| in LDS,
// a binary search per item) and probes each w: coalesced list reads, O(1) membership.  Vertices with
// more than TH_DMAX out-neighbours go to k_tri_heavy (a block each, sorted N+(u) in LDS, binary
// search).  Only vertices whose list starts in [q0, q1) count (the multi-GPU split).  This replaced
// a thread-per-oriented-edge merge intersection (load-imbalanced, latency-bound: 70.8 ms on an
// R-MAT scale-20 window, 95 % of the pipeline).
#pragma once
#include "gs_device.hpp"

namespace gs {

constexpr int TH_BLOCK = 256, TH_WPB = TH_BLOCK / WAVE;
constexpr uint32_t TH_DMAX = 512, TH_H = 1024, TH_EMPTY = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t th_hash(uint32_t x, uint32_t mask) { return ((x * 0x9E3779B1u) >> 7) & mask; }
// LDS written by some lanes of a wave, then read by others
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// out-list range [start, end) of every vertex in onbr (absent vertices: empty): one 8-byte load
// per lookup instead of the deg -> rowstart -> pos chain
__global__ __launch_bounds__(256) void k_tri_rows(const uint32_t* __restrict__ deg, const uint32_t* __restrict__ rowstart,
                                                  const uint32_t* __restrict__ pos, uint32_t nv,
                                                  uint2* __restrict__ range) {
  for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < nv; u += gridDim.x * 256u) {
    const uint32_t dg = deg[u];
    uint2 r = make_uint2(0, 0);
    if (dg) {
      const uint32_t rs = rowstart[u];
      r = make_uint2(pos[rs], pos[rs + dg]);
    }
    range[u] = r;
  }
}

constexpr int TH_ILP = 4;   // consecutive items per lane: one search, TH_ILP probes in flight

// N+(u) as an LDS hash set of 4-slot buckets (one 16-byte read answers almost every probe)
__device__ __forceinline__ void th_insert(uint32_t* hs, uint32_t x, uint32_t bmask) {
  for (uint32_t b = th_hash(x, bmask);; b = (b + 1) & bmask) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (atomicCAS(&hs[b * 4 + j], TH_EMPTY, x) == TH_EMPTY) return;
  }
}

__global__ __launch_bounds__(TH_BLOCK) void k_tri_light(const uint32_t* __restrict__ onbr,
                                                        const uint2* __restrict__ range, uint32_t nv, uint32_t q0,
                                                        uint32_t q1, uint32_t* __restrict__ heavy,
                                                        uint32_t* __restrict__ n_heavy,
                                                        unsigned long long* __restrict__ total) {
  // 8 KiB per wave, 32 KiB per block: five blocks per CU
  __shared__ uint4 s_hash[TH_WPB][TH_H / 4];
  __shared__ uint32_t s_off[TH_WPB][TH_DMAX];   // exclusive prefix of |N+(v)| over the non-empty v of N+(u)
  __shared__ uint32_t s_st[TH_WPB][TH_DMAX];    // start of that N+(v) in onbr
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint4* hb = s_hash[w];
  uint32_t* hs = reinterpret_cast<uint32_t*>(hb);
  uint32_t* po = s_off[w];
  uint32_t* ps = s_st[w];
  const uint32_t nw = gridDim.x * TH_WPB;
  uint64_t cnt = 0;
  for (uint32_t u = blockIdx.x * TH_WPB + w; u < nv; u += nw) {   // interleaved: no claim counter
    const uint2 ru = range[u];
    const uint32_t s = ru.x, d = ru.y - ru.x;
    if (d < 2 || s < q0 || s >= q1) continue;
    if (d > TH_DMAX) {
      if (lane == 0) heavy[atomicAdd(n_heavy, 1u)] = u;
      continue;
    }
    uint32_t nb = 16;
    while (nb < d && nb < TH_H / 4) nb <<= 1;
    const uint32_t bmask = nb - 1;
    for (uint32_t i = lane; i < nb * 4; i += WAVE) hs[i] = TH_EMPTY;
    wave_lds_sync();
    uint32_t run = 0, dn = 0;
    for (uint32_t i0 = 0; i0 < d; i0 += WAVE) {
      const uint32_t i = i0 + lane;
      uint32_t dv = 0, sv = 0;
      if (i < d) {
        const uint32_t x = onbr[s + i];
        th_insert(hs, x, bmask);
        const uint2 rv = range[x];
        dv = rv.y - rv.x;
        sv = rv.x;
      }
      // keep only the v with a non-empty out-list: every kept list spans >= 1 item
      const uint64_t ne = __ballot(dv != 0);
      const uint32_t at = dn + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(ne >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)ne, 0u));
      const uint32_t inc = wave_inclusive_sum(dv);
      if (dv) {
        po[at] = run + inc - dv;
        ps[at] = sv;
      }
      run += __shfl(inc, WAVE - 1, WAVE);
      dn += (uint32_t)__popcll(ne);
    }
    wave_lds_sync();
    uint32_t top = 1;
    while (2 * top < dn) top <<= 1;
    for (uint32_t k0 = 0; k0 < run; k0 += WAVE * TH_ILP) {
      const uint32_t kb = k0 + lane * TH_ILP;
      const uint32_t kk = min(kb, run - 1);
      // last kept v with po <= kk (po[dn] reads as run, above every item)
      uint32_t lo = 0;
      for (uint32_t st = top; st; st >>= 1) {
        const uint32_t t = lo + st;
        const uint32_t pv = t < dn ? po[min(t, dn - 1)] : run;
        lo = pv <= kk ? t : lo;
      }
      // the next TH_ILP-1 boundaries (each list >= 1 item: at most that many crossed)
      uint32_t bo[TH_ILP], bs[TH_ILP];
#pragma unroll
      for (int t = 0; t < TH_ILP; ++t) {
        const uint32_t q = lo + t;
        bo[t] = q < dn ? po[min(q, dn - 1)] : run;
        bs[t] = ps[min(q, dn - 1)];
      }
      uint32_t x[TH_ILP];
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) {
        const uint32_t kj = min(kb + j, run - 1);
        uint32_t o = bo[0], st = bs[0];
#pragma unroll
        for (int t = 1; t < TH_ILP; ++t) {
          o = bo[t] <= kj ? bo[t] : o;
          st = bo[t] <= kj ? bs[t] : st;
        }
        x[j] = onbr[st + (kj - o)];
      }
      uint32_t b[TH_ILP], pend = 0;
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) {
        b[j] = th_hash(x[j], bmask);
        pend |= (kb + j < run ? 1u : 0u) << j;
      }
      while (pend) {   // all pending probes of the lane read their bucket together
        uint4 y[TH_ILP];
#pragma unroll
        for (int j = 0; j < TH_ILP; ++j) y[j] = hb[b[j]];
#pragma unroll
        for (int j = 0; j < TH_ILP; ++j) {
          if (!(pend >> j & 1)) continue;
          const bool hit = y[j].x == x[j] || y[j].y == x[j] || y[j].z == x[j] || y[j].w == x[j];
          const bool open = y[j].w == TH_EMPTY;   // slots fill in order: a free last slot ends the chain
          if (hit || open) {
            cnt += hit ? 1u : 0u;
            pend &= ~(1u << j);
          }
          b[j] = (b[j] + 1) & bmask;
        }
      }
    }
    wave_lds_sync();
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, WAVE);
  if (lane == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

// one block per heavy vertex: N+(u) (sorted) in LDS when it fits, the v lists in chunks of TH_VCH
constexpr int TH_HBLOCK = 1024;
constexpr uint32_t TH_NU = 16384, TH_VCH = 4096;
__global__ __launch_bounds__(TH_HBLOCK) void k_tri_heavy(const uint32_t* __restrict__ onbr,
                                                         const uint2* __restrict__ range,
                                                         const uint32_t* __restrict__ heavy,
                                                         const uint32_t* __restrict__ n_heavy,
                                                         unsigned long long* __restrict__ total) {
  __shared__ uint32_t s_nu[TH_NU];
  __shared__ uint32_t s_off[TH_VCH + 1];
  __shared__ uint32_t s_st[TH_VCH];
  __shared__ uint32_t s_w[TH_HBLOCK / WAVE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint64_t cnt = 0;
  const uint32_t nh = *n_heavy;
  for (uint32_t hi = blockIdx.x; hi < nh; hi += gridDim.x) {
    const uint32_t u = heavy[hi];
    const uint2 ru = range[u];
    const uint32_t s = ru.x, d = ru.y - ru.x;
    const bool in_lds = d <= TH_NU;
    if (in_lds)
      for (uint32_t i = tid; i < d; i += TH_HBLOCK) s_nu[i] = onbr[s + i];
    const uint32_t* nu = in_lds ? s_nu : onbr + s;
    for (uint32_t c0 = 0; c0 < d; c0 += TH_VCH) {
      const uint32_t cn = min(TH_VCH, d - c0);
      __syncthreads();
      // prefix of |N+(v)| over this chunk of v (4 per thread, block scan)
      uint32_t dv[4], sv[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t i = tid * 4 + j;
        dv[j] = 0;
        sv[j] = 0;
        if (i < cn) {
          const uint2 rv = range[onbr[s + c0 + i]];
          sv[j] = rv.x;
          dv[j] = rv.y - rv.x;
        }
        sum += dv[j];
      }
      const uint32_t inc = wave_inclusive_sum(sum);
      if (lane == 63) s_w[w] = inc;
      __syncthreads();
      uint32_t base = 0, tot = 0;
      for (int i = 0; i < TH_HBLOCK / WAVE; ++i) {
        base += i < w ? s_w[i] : 0u;
        tot += s_w[i];
      }
      uint32_t run = base + inc - sum;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t i = tid * 4 + j;
        if (i < cn) {
          s_off[i] = run;
          s_st[i] = sv[j];
        }
        run += dv[j];
      }
      if (tid == 0) s_off[cn] = tot;
      __syncthreads();
      for (uint32_t k = tid; k < tot; k += TH_HBLOCK) {
        uint32_t lo = 0, hi2 = cn - 1;
        while (lo < hi2) {
          const uint32_t mid = (lo + hi2 + 1) >> 1;
          if (s_off[mid] <= k) lo = mid;
          else hi2 = mid - 1;
        }
        const uint32_t x = onbr[s_st[lo] + (k - s_off[lo])];
        uint32_t a = 0, b = d;   // lower bound of x in N+(u)
        while (a < b) {
          const uint32_t mid = (a + b) >> 1;
          if (nu[mid] < x) a = mid + 1;
          else b = mid;
        }
        cnt += (a < d && nu[a] == x) ? 1u : 0u;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, WAVE);
  if (lane == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
}

}  // namespace gs
