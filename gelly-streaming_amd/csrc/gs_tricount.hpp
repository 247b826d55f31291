// gs_tricount.hpp — the counting step of WindowTriangles (gs_graph.hip) on the degree-renumbered graph
// (u -> v iff u < v, out-lists sorted): every triangle is u -> v, u -> w, v -> w for exactly one
// (u, v, w), and w > v, so
//   T = sum over v of sum over u in N-(v) of |N+(u) after v  ∩  N+(v)|.
// Row x of the adjacency is [in-list | out-list] in one array (onbr); k_tri_sfx gives every in-entry
// u of v the range of N+(u) past v (sfx), so a chunk's lists come from one coalesced read.
//
// Middle-vertex order: a wave takes v, puts N+(v) into an LDS hash set of 4-slot buckets, spreads the
// concatenation of the suffixes over a chunk of TH_LCH in-neighbours u across its lanes (prefix of
// the lengths in LDS, one search per TH_ILP consecutive items) and probes each w with one 16-byte LDS
// read.  Probes: sum over u of d+(u)(d+(u)-1)/2 (R-MAT scale 20: 1.23 G; whole lists 2.47 G, first-
// vertex order 4.42 G).  In-lists longer than a chunk queue their further chunks for a second pass (a
// hub's work spreads over many waves); vertices with more than TH_DMAX out-neighbours (or TH_HMIN when
// the heavy bitmap covers their span) go to
// k_tri_heavy (a block each, N+(v) in a 64 KiB LDS hash set).  Only vertices whose out-list starts in
// [q0, q1) count (the multi-GPU split).
#pragma once
#include "gs_device.hpp"
#include "gs_internal.hpp"

namespace gs {

constexpr int TH_BLOCK = 256, TH_WPB = TH_BLOCK / WAVE;
// k_tri_heavy: 512 threads, three blocks per CU, N+(v) of up to TH_NU entries in LDS, in-entries in
// chunks of TH_VCH (history: one 1024-thread block per CU with a 16384-entry table, s22 70.9 -> 67.8
// ms; one 512-thread block per CU instead of two: 11.4 -> 17.9 ms; chunks of 512 / 1024 / 2048: equal)
#ifndef GS_TH_HBLOCK
#define GS_TH_HBLOCK 512
#endif
#ifndef GS_TH_NU
#define GS_TH_NU 4096   // heavy N+(v) up to 4096 in a 32 KiB LDS table (longer: HBM search)
#endif
#ifndef GS_TH_HGRID
#define GS_TH_HGRID 768   // heavy blocks in the grid: three per CU (49 KiB LDS each)
#endif
constexpr int TH_HBLOCK = GS_TH_HBLOCK;
#ifndef GS_TH_VCH
#define GS_TH_VCH 1024
#endif
constexpr uint32_t TH_NU = GS_TH_NU, TH_HB = TH_NU / 2, TH_VCH = GS_TH_VCH;   // TH_HB 4-slot buckets: load <= 1/2
#ifndef GS_TH_BITMAP
#define GS_TH_BITMAP 1   // k_tri_heavy: N+(v) as a bitmap over (v, last] when the span fits the table
#endif
constexpr bool TH_BITMAP = GS_TH_BITMAP;
// the heavy table's bits (TH_HB 16-byte buckets) less one word: the bitmap of a span of up to TH_BSPAN bits
// keeps a zero word after its last, which items past the span index (k_tri_heavy's branch-free probe)
constexpr uint32_t TH_BSPAN = TH_NU / 2 * 128u - 32u;
#ifndef GS_TH_LBITMAP
#define GS_TH_LBITMAP 0  // k_tri_light: the same for a wave's table (spans up to TH_H·32 bits); A/B: light count s24 7.08 vs 6.92 ms hash, off
#endif
constexpr bool TH_LBITMAP = GS_TH_LBITMAP;
static_assert(TH_VCH % TH_HBLOCK == 0, "TH_VCH must be a multiple of TH_HBLOCK");
#ifndef GS_TH_DMAX
#define GS_TH_DMAX 512   // light capacity (out-list of a light vertex, in-entries per light chunk); with the heavy bitmaps: s26 455 -> 376 ms
#endif
#ifndef GS_TH_HMIN
#define GS_TH_HMIN 256   // out-lists longer than this go to k_tri_heavy when its bitmap covers their span (the rest up to TH_DMAX stay light)
#endif
#ifndef GS_TH_H
#define GS_TH_H 1024
#endif
constexpr uint32_t TH_DMAX = GS_TH_DMAX, TH_HMIN = GS_TH_HMIN, TH_H = GS_TH_H, TH_EMPTY = 0xFFFFFFFFu;
static_assert(TH_HMIN <= TH_DMAX, "TH_HMIN must be <= TH_DMAX");
#ifndef GS_TH_LCH
#define GS_TH_LCH 256    // k_tri_light: in-entries per chunk (the wave's list prefix arrays: 2 KiB)
#endif
constexpr uint32_t TH_LCH = GS_TH_LCH;
// a light vertex's N+(v) (<= TH_DMAX entries) must leave the TH_H-slot table at most half full: insert
// and probe chains end at a free slot, so a full table would never end them
static_assert(TH_DMAX * 2 <= TH_H, "TH_DMAX must be <= TH_H / 2");
#ifndef GS_TH_ILP
#define GS_TH_ILP 8    // R-MAT s22 (DMAX 512): 2 -> 93.9 ms, 4 -> 70.2, 6 -> 62.6, 8 -> 62.0, 12 -> 64.5, 16 -> 137.8; DMAX 256: 6 -> 55.3, 8 -> 55.8, 10 -> 54.5 (s24 291.9, 289.6, 279.7); 6 waves/SIMD: 6 -> 23.8, 8 -> 23.7, 10 -> 23.8 (spills)
#endif
constexpr int TH_ILP = GS_TH_ILP;   // items per lane: TH_ILP probes in flight
#ifndef GS_TH_LONG
#define GS_TH_LONG 64    // light kernel: out-lists of >= TH_LONG items are gathered lane-interleaved (64 per load)
#endif
constexpr uint32_t TH_LONG = GS_TH_LONG;
#ifndef GS_TH_LWAVES
#define GS_TH_LWAVES 6   // k_tri_light waves per SIMD the registers are capped for (4 -> 6: s22 3.03 -> 2.38 ms)
#endif
#ifndef GS_TH_WALK
#define GS_TH_WALK 1     // k_tri_heavy: branch-free list walk (A/B, s26 heavy 144.5 -> 140.7 ms; 0 = a branch and an
                         // LDS round trip per item, in series)
#endif
#ifndef GS_TH_LWALK
#define GS_TH_LWALK 0    // k_tri_light: the same (A/B: light 39.6 -> 40.2 ms at s26, not kept)
#endif
#ifndef GS_TH_LPIPE
#define GS_TH_LPIPE 0    // k_tri_light: the same (A/B)
#endif
#ifndef GS_TH_PIPE
#define GS_TH_PIPE 0     // k_tri_heavy: gathers of the next step issued before this step's probes (A/B)
#endif
#ifndef GS_TH_HWAVES
#define GS_TH_HWAVES 6   // k_tri_heavy: three 512-thread blocks per CU (4 -> 6: s22 11.4 -> 9.8 ms, s24 72.3 -> 62.5)
#endif
static_assert(TH_LONG >= 64, "a 64-item segment must not span more than two long lists");

__device__ __forceinline__ uint32_t th_hash(uint32_t x, uint32_t mask) { return ((x * 0x9E3779B1u) >> 7) & mask; }
// a value the code keeps equal on every lane of the wave (LDS broadcast reads, per-wave bounds): into
// an SGPR, so loops over it compile to scalar branches instead of exec-masked per-lane loops
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// LDS written by some lanes of a wave, then read by others
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Every insert and probe chain is bounded by the table's bucket count: a full table (which the
// sizing rules exclude: TH_DMAX <= TH_H / 2, d <= TH_NU at <= half load) sets GS_DERR_TABLE_FULL in
// *err and gives up, and the host returns GS_EDEVICE, instead of a chain that never ends.
// (GS_FLAG_TEST_TINY_TABLES forces one-bucket tables so the tests can see that error.)
__device__ __forceinline__ void th_fail(uint32_t* err) { atomicOr(err, GS_DERR_TABLE_FULL); }

// N+(v) as an LDS hash set of 4-slot buckets; slots of a bucket fill in order
__device__ __forceinline__ void th_insert(uint32_t* hs, uint32_t x, uint32_t bmask, uint32_t* err) {
  uint32_t b = th_hash(x, bmask);
  for (uint32_t step = 0; step <= bmask; ++step, b = (b + 1) & bmask) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (atomicCAS(&hs[b * 4 + j], TH_EMPTY, x) == TH_EMPTY) return;
  }
  th_fail(err);
}

// members among x[0 .. nv) (the lane's valid items are always a prefix).  At <= half load nearly every
// probe ends in its first bucket (a hit, or a free last slot), so one branch-free round reads every
// item's bucket (one 16-byte LDS read each) and only items whose first bucket was full without a hit
// walk on.  The hit test is arithmetic (min of the XORs with the 4 slots == 0): written as compares
// the compiler built a 4-bit mask per item through 16-bit ops (~20 VALU per probe, PMC at s22).
__device__ __forceinline__ uint32_t slot_xor_min(const uint4& y, uint32_t x) {
  return min(min(y.x ^ x, y.y ^ x), min(y.z ^ x, y.w ^ x));
}

__device__ __forceinline__ uint32_t th_probe(const uint4* hb, uint32_t bmask, const uint32_t (&x)[TH_ILP],
                                             uint32_t nv, uint32_t* err) {
  uint32_t b[TH_ILP], cnt = 0, walk = 0;
#pragma unroll
  for (int j = 0; j < TH_ILP; ++j) b[j] = th_hash(x[j], bmask);
  uint4 y[TH_ILP];
#pragma unroll
  for (int j = 0; j < TH_ILP; ++j) y[j] = hb[b[j]];
#pragma unroll
  for (int j = 0; j < TH_ILP; ++j) {
    const uint32_t m = slot_xor_min(y[j], x[j]);
    const uint32_t on = (uint32_t)j < nv ? 1u : 0u;
    cnt += (m == 0u) ? on : 0u;
    walk |= (((m != 0u) & (y[j].w != TH_EMPTY)) ? on : 0u) << j;
  }
  if (walk) {   // rare: chains that continue past their first bucket
#pragma unroll
    for (int j = 0; j < TH_ILP; ++j) b[j] = (b[j] + 1) & bmask;
    for (uint32_t step = 1; walk; ++step) {
      if (step > bmask) {   // no free last slot on a whole sweep: the table is full
        th_fail(err);
        break;
      }
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) {
        if (!(walk >> j & 1)) continue;
        const uint4 z = hb[b[j]];
        const bool hit = slot_xor_min(z, x[j]) == 0u;
        if (hit || z.w == TH_EMPTY) {
          cnt += hit ? 1u : 0u;
          walk &= ~(1u << j);
        }
        b[j] = (b[j] + 1) & bmask;
      }
    }
  }
  return cnt;
}

// cnt += probe(items of step k0) for k0 = a, a + step, .. < b, the items from gather(k0, x) -> valid count.
// PIPE: software-pipelined -- step k0 + step's gathers (and the list search that places them) issue before
// step k0's probes, so the search's LDS chain and the gathers' memory latency of consecutive steps overlap
// (the loop bound is uniform over the caller's wave or block)
template <int PIPE, class C, class Gather, class Probe>
__device__ __forceinline__ void th_pipelined(uint32_t a, uint32_t b, uint32_t step, Gather&& gather, Probe&& probe,
                                             C& cnt) {
  if constexpr (PIPE) {
    if (a >= b) return;
    uint32_t xa[TH_ILP];
    uint32_t nva = gather(a, xa);
    for (uint32_t k0 = a; k0 < b; k0 += step) {
      uint32_t xb[TH_ILP], nvb = 0;
      if (k0 + step < b) {
        nvb = gather(k0 + step, xb);
      } else {
#pragma unroll
        for (int j = 0; j < TH_ILP; ++j) xb[j] = 0u;
      }
      cnt += probe(xa, nva);
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) xa[j] = xb[j];
      nva = nvb;
    }
  } else {
    for (uint32_t k0 = a; k0 < b; k0 += step) {
      uint32_t x[TH_ILP];
      const uint32_t nv = gather(k0, x);
      cnt += probe(x, nv);
    }
  }
}

// one wave: |suffix of N+(u) ∩ N+(v)| summed over the in-entries c0 .. c1 (<= CAP) of v, N+(v)
// behind probe(x, nv) (an LDS hash set, or a search in HBM)
// lists of >= TH_LONG items ("long") are gathered lane-interleaved (64 consecutive items per load:
// 2 cache lines); the short ones TH_ILP consecutive items per lane.  Short lists fill po / ps from the
// front (po = prefix of their lengths), long ones from the back (po = prefix over long lists)
template <uint32_t CAP, class Probe>
__device__ __forceinline__ uint32_t th_wave_probe(const uint32_t* __restrict__ onbr, const uint2* __restrict__ sfx,
                                                  uint32_t c0, uint32_t c1, int lane, uint32_t* po, uint32_t* ps,
                                                  uint64_t& probes, Probe probe) {
  uint32_t run = 0, dn = 0, lrun = 0, nl = 0;
  for (uint32_t i0 = c0; i0 < c1; i0 += WAVE) {
    const uint32_t i = i0 + lane;
    uint32_t du = 0, su = 0;
    if (i < c1) {
      const uint2 ru = sfx[i];
      du = ru.y - ru.x;
      su = ru.x;
    }
    const bool lg = du >= TH_LONG, sh = du != 0 && !lg;
    const uint64_t ms = __ballot(sh), ml = __ballot(lg);
    const uint32_t ds = sh ? du : 0u, dl = lg ? du : 0u;
    const uint32_t inc = wave_inclusive_sum(ds), incl = wave_inclusive_sum(dl);
    if (sh) {
      const uint32_t at = dn + mbcnt(ms);
      po[at] = run + inc - ds;
      ps[at] = GS_TH_LWALK ? su - (run + inc - ds) : su;   // (walk: item k of list at is onbr[k + ps[at]])
    }
    if (lg) {
      const uint32_t at = CAP - 1 - (nl + mbcnt(ml));
      po[at] = lrun + incl - dl;
      ps[at] = su;
    }
    run += uni(__shfl(inc, WAVE - 1, WAVE));
    lrun += uni(__shfl(incl, WAVE - 1, WAVE));
    dn += (uint32_t)__popcll(ms);
    nl += (uint32_t)__popcll(ml);
  }
  wave_lds_sync();
  probes += run + lrun;
  uint32_t cnt = 0;
  if (nl) {   // long lists: segment k of 64 items lies in list q or q + 1 (every long list >= 64 items)
    uint32_t q = 0;
    uint32_t qo = uni(po[CAP - 1]), qs = uni(ps[CAP - 1]);
    uint32_t qe = nl > 1 ? uni(po[CAP - 2]) : lrun, q1s = nl > 1 ? uni(ps[CAP - 2]) : 0u;
    auto gather_long = [&](uint32_t k0, uint32_t (&x)[TH_ILP]) -> uint32_t {
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) {
        const uint32_t seg = k0 + (uint32_t)j * WAVE;   // wave-uniform
        while (qe <= seg && q + 1 < nl) {                // advance to the list holding item seg
          ++q;
          qo = qe;
          qs = q1s;
          qe = q + 1 < nl ? uni(po[CAP - 2 - q]) : lrun;
          q1s = q + 1 < nl ? uni(ps[CAP - 2 - q]) : 0u;
        }
        const uint32_t k = min(seg + (uint32_t)lane, lrun - 1);
        x[j] = onbr[k < qe ? qs + (k - qo) : q1s + (k - qe)];
      }
      // valid items of this lane: segments j with k0 + 64 j + lane < lrun (a prefix of j)
      const uint32_t rem = lrun - k0;
      return rem > (uint32_t)lane ? min((uint32_t)TH_ILP, (rem - lane + WAVE - 1) / WAVE) : 0u;
    };
    th_pipelined<GS_TH_LPIPE>(0u, lrun, (uint32_t)(WAVE * TH_ILP), gather_long, probe, cnt);
  }
  uint32_t top = 1;
  while (2 * top < dn) top <<= 1;
  auto gather_short = [&](uint32_t k0, uint32_t (&x)[TH_ILP]) -> uint32_t {
    const uint32_t kb = k0 + lane * TH_ILP;
    const uint32_t kk = min(kb, run - 1);
    // last kept u with po <= kk (po[dn] reads as run, above every item)
    uint32_t lo = 0;
    for (uint32_t st = top; st; st >>= 1) {
      const uint32_t t = lo + st;
      const uint32_t pv = t < dn ? po[min(t, dn - 1)] : run;
      lo = pv <= kk ? t : lo;
    }
#if GS_TH_LWALK
    // branch-free, as k_tri_heavy's walk: the next TH_ILP - 1 list starts as a mask of the items that start one
    uint32_t m = 0;
#pragma unroll
    for (int i = 1; i < TH_ILP; ++i) {
      const uint32_t t = lo + (uint32_t)i;
      const uint32_t d = (t < dn ? po[min(t, dn - 1)] : run) - kb;
      m |= d < (uint32_t)TH_ILP ? 1u << d : 0u;
    }
#pragma unroll
    for (int j = 0; j < TH_ILP; ++j) {
      const uint32_t ql = min(lo + (uint32_t)__builtin_popcount(m & ((2u << j) - 1u)), dn - 1);
      x[j] = onbr[min(kb + j, run - 1) + ps[ql]];
    }
    return kb < run ? min((uint32_t)TH_ILP, run - kb) : 0u;
#endif
    // consecutive items cross at most one list boundary per step (every kept list has >= 1 item)
    uint32_t o = po[lo], st = ps[lo], q = lo;
    uint32_t nx = q + 1 < dn ? po[min(q + 1, dn - 1)] : run;
#pragma unroll
    for (int j = 0; j < TH_ILP; ++j) {
      const uint32_t kj = min(kb + j, run - 1);
      if (kj >= nx) {
        ++q;
        o = nx;
        st = ps[q];
        nx = q + 1 < dn ? po[q + 1] : run;
      }
      x[j] = onbr[st + (kj - o)];
    }
    return kb < run ? min((uint32_t)TH_ILP, run - kb) : 0u;
  };
  th_pipelined<GS_TH_LPIPE>(0u, run, (uint32_t)(WAVE * TH_ILP), gather_short, probe, cnt);
  wave_lds_sync();   // po / ps are reused by the next chunk
  return cnt;
}

// one wave: N+(v) into the wave's own LDS hash set, then the in-entries c0 .. c1 (<= TH_LCH) of v
__device__ __forceinline__ uint32_t th_wave_chunk(const uint32_t* __restrict__ onbr, const uint2* __restrict__ sfx,
                                                  uint32_t v_id, uint2 ro, uint32_t c0,
                                                  uint32_t c1, int lane, uint4* hb, uint32_t* po, uint32_t* ps,
                                                  uint64_t& probes, uint32_t nb_cap, uint32_t* err) {
  uint32_t* hs = reinterpret_cast<uint32_t*>(hb);
  const uint32_t d = ro.y - ro.x;
  // a bitmap over (v, last] when the span fits the table's TH_H·32 bits (k_tri_heavy): the high-rank
  // light vertices (hubs with few higher neighbours)
  const uint32_t v = uni(v_id), span = uni(onbr[ro.y - 1] - v);
  if (TH_LBITMAP && nb_cap > 1 && span <= TH_H * 32u) {
    const uint32_t nw = (span + 31) / 32;
    for (uint32_t i = lane; i < nw; i += WAVE) hs[i] = 0u;
    wave_lds_sync();
    for (uint32_t i = lane; i < d; i += WAVE) {
      const uint32_t o = onbr[ro.x + i] - v - 1;
      atomicOr(&hs[o >> 5], 1u << (o & 31));
    }
    wave_lds_sync();
    return th_wave_probe<TH_LCH>(onbr, sfx, c0, c1, lane, po, ps, probes,
                                  [&](const uint32_t (&x)[TH_ILP], uint32_t nv) {
                                    uint32_t c = 0;
#pragma unroll
                                    for (int j = 0; j < TH_ILP; ++j) {
                                      const uint32_t o = x[j] - v - 1;
                                      const uint32_t wv = hs[min(o, span - 1) >> 5];
                                      c += ((uint32_t)j < nv && o < span) ? (wv >> (o & 31)) & 1u : 0u;
                                    }
                                    return c;
                                  });
  }
  uint32_t nb = 16;
  while (nb < d && nb < TH_H / 4) nb <<= 1;
  nb = min(nb, nb_cap);
  const uint32_t bmask = nb - 1;
  for (uint32_t i = lane; i < nb * 4; i += WAVE) hs[i] = TH_EMPTY;
  wave_lds_sync();
  for (uint32_t i = lane; i < d; i += WAVE) th_insert(hs, onbr[ro.x + i], bmask, err);
  wave_lds_sync();
  return th_wave_probe<TH_LCH>(onbr, sfx, c0, c1, lane, po, ps, probes,
                                [&](const uint32_t (&x)[TH_ILP], uint32_t nv) { return th_probe(hb, bmask, x, nv, err); });
}

// The light chunks k_tri_lclass queued, (v, in-chunk of TH_LCH), a wave each: N+(v) into the wave's LDS
// hash set, then the chunk's in-entries (th_wave_chunk).  Interleaved over the queue (no claim counter);
// n_probes counts the hash probes (bench bytes).
// 24 KiB of LDS per block -> six blocks (24 waves) per CU: registers capped to match (80 VGPRs)
__global__ __launch_bounds__(TH_BLOCK) __attribute__((amdgpu_waves_per_eu(GS_TH_LWAVES, GS_TH_LWAVES))) void k_tri_light(const uint32_t* __restrict__ onbr,
                                                        const uint2* __restrict__ sfx,
                                                        const uint2* __restrict__ out_range,
                                                        const uint2* __restrict__ in_range,
                                                        const uint2* __restrict__ queue,
                                                        const uint32_t* __restrict__ n_queue,
                                                        unsigned long long* __restrict__ total,
                                                        unsigned long long* __restrict__ n_probes, uint32_t nb_cap,
                                                        uint32_t* __restrict__ err) {
  // 6 KiB per wave (4 KiB table + 2 KiB list prefix), 24 KiB per block
  __shared__ uint4 s_hash[TH_WPB][TH_H / 4];
  __shared__ uint32_t s_off[TH_WPB][TH_LCH];   // exclusive prefix of |N+(u)| over the non-empty u
  __shared__ uint32_t s_st[TH_WPB][TH_LCH];    // start of that N+(u) in onbr
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * TH_WPB;
  uint64_t cnt = 0, probes = 0;
  const uint32_t n_items = *n_queue;
  for (uint32_t it = blockIdx.x * TH_WPB + w; it < n_items; it += nw) {
    const uint2 q = queue[it];
    const uint32_t v = q.x;
    const uint2 ri = in_range[v];
    const uint32_t c0 = ri.x + q.y * TH_LCH, c1 = min(ri.y, c0 + TH_LCH);
    cnt += th_wave_chunk(onbr, sfx, v, out_range[v], c0, c1, lane, s_hash[w], s_off[w], s_st[w], probes,
                         nb_cap, err);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, WAVE);
  if (lane == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
  if (lane == 0 && probes) atomicAdd(n_probes, (unsigned long long)probes);   // wave-uniform
}

// The count's vertex pass, one lane per vertex: every vertex with in- and out-entries whose out-list
// starts in [q0, q1) becomes heavy items (its in-chunks of TH_VCH) or light queue entries (its in-chunks
// of TH_LCH).  Heavy: too long for a wave's table, or long enough to gain from the heavy kernel's bitmap
// (the span of N+(v) within its table's bits; history: the split at 256 alone, s26 455 ms, at 512 alone
// s24 72 -> 78 ms).  (Round 4: this pass ran inside k_tri_light, a wave per id in rank order, a dependent
// load per id, 2^26 ids at s26, most without work: light count 41.9 -> 39.0 ms.)  Appends are
// block-aggregated (one atomic per block and list: round 5 took one per wave).
#ifndef GS_TH_LCBLOCK
#define GS_TH_LCBLOCK 1024   // k_tri_lclass block: its appends are aggregated per block (one atomic per list per block)
#endif
constexpr int TH_LCBLOCK = GS_TH_LCBLOCK, TH_LCNW = TH_LCBLOCK / WAVE;
__global__ __launch_bounds__(TH_LCBLOCK) void k_tri_lclass(const uint32_t* __restrict__ onbr, const uint2* __restrict__ out_range,
                                                    const uint2* __restrict__ in_range, uint32_t nv, uint32_t q0,
                                                    uint32_t q1, uint32_t nb_cap, uint2* __restrict__ queue,
                                                    uint32_t* __restrict__ n_queue, uint2* __restrict__ heavy,
                                                    uint32_t* __restrict__ n_heavy,
                                                    unsigned long long* __restrict__ n_active,
                                                    unsigned long long* __restrict__ merge) {
  __shared__ uint32_t s_h[TH_LCNW], s_l[TH_LCNW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t act = 0;   // this lane's ranks with an out- or in-entry (n_active, when asked for)
  // sum over the oriented edges u -> v counted here of d+(u) + d+(v) (the list entries a merge
  // intersection per edge would read; bench's roofline): per vertex x, d+(x) (d+(x) + d-(x))
  unsigned long long mg = 0;
  for (uint32_t v0 = blockIdx.x * (uint32_t)TH_LCBLOCK; v0 < nv; v0 += gridDim.x * (uint32_t)TH_LCBLOCK) {   // block-uniform
    const uint32_t v = v0 + threadIdx.x;
    uint32_t nh = 0, nl = 0;
    if (v < nv) {
      const uint2 ro = out_range[v], ri = in_range[v];
      if (n_active) act += (ro.y != ro.x || ri.y != ri.x) ? 1u : 0u;
      if (ro.x >= q0 && ro.x < q1)
        mg += (unsigned long long)(ro.y - ro.x) * ((ro.y - ro.x) + (ri.y - ri.x));
      if (ro.y != ro.x && ri.y != ri.x && ro.x >= q0 && ro.x < q1) {
        const uint32_t dv = ro.y - ro.x;
        const bool heavy_v = dv > TH_DMAX ||
                             (TH_BITMAP && nb_cap > 1 && dv > TH_HMIN && onbr[ro.y - 1] - v <= TH_BSPAN);
        if (heavy_v) nh = (ri.y - ri.x + TH_VCH - 1) / TH_VCH;
        else nl = (ri.y - ri.x + TH_LCH - 1) / TH_LCH;
      }
    }
    // appends aggregated per block: the waves' totals, one atomic per list (R-MAT s26: 2^26 ids, most waves
    // with an append -- one atomic per wave on the same two counters serialized)
    const uint32_t ih = wave_inclusive_sum(nh), il = wave_inclusive_sum(nl);
    if (lane == 63) {
      s_h[w] = ih;
      s_l[w] = il;
    }
    __syncthreads();
    if (threadIdx.x < 2) {   // thread 0: heavy, thread 1: light -- exclusive prefix over the waves + the block's base
      uint32_t* t = threadIdx.x == 0 ? s_h : s_l;
      uint32_t run = 0;
      for (int x = 0; x < TH_LCNW; ++x) {
        const uint32_t c = t[x];
        t[x] = run;
        run += c;
      }
      const uint32_t base = run ? atomicAdd(threadIdx.x == 0 ? n_heavy : n_queue, run) : 0u;
      for (int x = 0; x < TH_LCNW; ++x) t[x] += base;
    }
    __syncthreads();
    const uint32_t bh = s_h[w] + ih - nh, bl = s_l[w] + il - nl;
    for (uint32_t j = 0; j < nh; ++j) heavy[bh + j] = make_uint2(v, j);
    for (uint32_t j = 0; j < nl; ++j) queue[bl + j] = make_uint2(v, j);
    __syncthreads();   // (the next round's totals)
  }
  if (n_active) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) act += __shfl_xor(act, o, WAVE);
    if (lane == 0 && act) atomicAdd(n_active, (unsigned long long)act);
  }
  if (merge) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mg += __shfl_xor(mg, o, WAVE);
    if (lane == 0 && mg) atomicAdd(merge, mg);
  }
}

// ... plus the ids whose only edges are self-loops (loops: the id-indexed self-loop bitmap; their ranks
// have no out- or in-entries), so n_active = the window's vertices with an edge
__global__ __launch_bounds__(256) void k_tri_loop_only(const uint32_t* __restrict__ loops, uint32_t words,
                                                       const uint32_t* __restrict__ rank, const uint2* __restrict__ out_range,
                                                       const uint2* __restrict__ in_range,
                                                       unsigned long long* __restrict__ n_active) {
  uint32_t cnt = 0;
  for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < words; w += gridDim.x * 256u) {
    for (uint32_t bits = loops[w]; bits; bits &= bits - 1) {
      const uint32_t r = rank[w * 32u + (uint32_t)__builtin_ctz(bits)];
      const uint2 ro = out_range[r], ri = in_range[r];
      cnt += (ro.y == ro.x && ri.y == ri.x) ? 1u : 0u;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, WAVE);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(n_active, (unsigned long long)cnt);
}

// work of each heavy item (v, chunk of TH_VCH in-entries): its probes (the suffix lengths) plus a
// fixed cost per in-entry; one wave per item
__global__ __launch_bounds__(256) void k_tri_hwork(const uint2* __restrict__ sfx, const uint2* __restrict__ in_range,
                                                   const uint2* __restrict__ heavy, uint32_t nh,
                                                   unsigned long long* __restrict__ work) {
  const int lane = threadIdx.x & 63;
  for (uint32_t h = (blockIdx.x * 256u + threadIdx.x) / WAVE; h < nh; h += gridDim.x * (256u / WAVE)) {
    const uint2 item = heavy[h];
    const uint2 ri = in_range[item.x];
    const uint32_t c0 = ri.x + item.y * TH_VCH, c1 = min(ri.y, c0 + TH_VCH);
    uint32_t w = 0;
    for (uint32_t i = c0 + lane; i < c1; i += WAVE) {
      const uint2 r = sfx[i];
      w += r.y - r.x + 4u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, WAVE);
    if (lane == 0) work[h] = w;
  }
}

// Phased order of the heavy items (GS_TH_PHASED): an item (v, in-chunk) gathers the suffixes of N+(u) for
// the chunk's in-neighbours u, whose out-lists lie in one stretch of onbr (in-lists are in u order).  The
// heavy vertices' items run at once, so in equal-work order the chip gathers from all of onbr (4 GB at
// R-MAT s26: HBM, 7 % L2 hits).  Ordered by that stretch (TH_PHASES phases of onbr) and claimed in order,
// the items in flight gather from a few phases' out-lists, which the Infinity Cache / L2 keep.
#ifndef GS_TH_PHASED
#define GS_TH_PHASED 1
#endif
#ifndef GS_TH_PHASES
#define GS_TH_PHASES 16384   // s26 heavy count (ms): 256 phases 149, 1024 146.5, 4096 143.3, 16384 142.0, 65536 141.2
#endif
constexpr uint32_t TH_PHASES = GS_TH_PHASES;
// (CH: in-entries per item, TH_VCH)
template <uint32_t CH>
__device__ __forceinline__ uint32_t th_phase(const uint2* __restrict__ sfx, const uint2* __restrict__ in_range, uint2 item,
                                             uint32_t M) {
  const uint32_t c0 = in_range[item.x].x + item.y * CH;
  return (uint32_t)((uint64_t)sfx[c0].x * TH_PHASES / (M ? M : 1u));
}
template <uint32_t CH>
__global__ __launch_bounds__(256) void k_tri_hphase_count(const uint2* __restrict__ sfx, const uint2* __restrict__ in_range,
                                                          const uint2* __restrict__ heavy, uint32_t nh, uint32_t M,
                                                          uint32_t* __restrict__ hist) {
  for (uint32_t h = blockIdx.x * 256u + threadIdx.x; h < nh; h += gridDim.x * 256u)
    atomicAdd(&hist[min(th_phase<CH>(sfx, in_range, heavy[h], M), TH_PHASES - 1)], 1u);
}
__global__ __launch_bounds__(256) void k_tri_hphase_scan(uint32_t* __restrict__ hist) {   // one block, in place
  static_assert(TH_PHASES % 256 == 0, "phases per thread");
  constexpr uint32_t PT = TH_PHASES / 256;
  __shared__ uint32_t s_w[256 / WAVE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t v[PT], x = 0;
#pragma unroll
  for (uint32_t j = 0; j < PT; ++j) x += (v[j] = hist[tid * PT + j]);
  const uint32_t inc = wave_inclusive_sum(x);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t off = 0;
  for (int i = 0; i < w; ++i) off += s_w[i];
  off += inc - x;
#pragma unroll
  for (uint32_t j = 0; j < PT; ++j) {
    hist[tid * PT + j] = off;
    off += v[j];
  }
}
template <uint32_t CH>
__global__ __launch_bounds__(256) void k_tri_hphase_place(const uint2* __restrict__ sfx, const uint2* __restrict__ in_range,
                                                          const uint2* __restrict__ heavy, uint32_t nh, uint32_t M,
                                                          uint32_t* __restrict__ off, uint32_t* __restrict__ order) {
  for (uint32_t h = blockIdx.x * 256u + threadIdx.x; h < nh; h += gridDim.x * 256u)
    order[atomicAdd(&off[min(th_phase<CH>(sfx, in_range, heavy[h], M), TH_PHASES - 1)], 1u)] = h;
}

// one block per heavy item (v, chunk of TH_VCH in-neighbours): N+(v) as an LDS hash set (up to TH_NU
// entries; longer lists are binary-searched in HBM; rebuilt only when the block's item changes v),
// the chunk's lists TH_ILP items per thread with one search.  One item per in-chunk spreads a hub over
// many blocks (one block per heavy vertex left the hubs' blocks running long after the rest).
// three 512-thread blocks per CU (49 KiB of LDS each): registers capped to match (80 VGPRs)
__global__ __launch_bounds__(TH_HBLOCK) __attribute__((amdgpu_waves_per_eu(GS_TH_HWAVES, GS_TH_HWAVES))) void k_tri_heavy(const uint32_t* __restrict__ onbr,
                                                         const uint2* __restrict__ sfx,
                                                         const uint2* __restrict__ out_range,
                                                         const uint2* __restrict__ in_range,
                                                         const uint2* __restrict__ heavy,
                                                         const uint32_t* __restrict__ n_heavy,
                                                         const unsigned long long* __restrict__ pre,
                                                         const uint32_t* __restrict__ order,
                                                         uint32_t* __restrict__ claim,
                                                         unsigned long long* __restrict__ total,
                                                         unsigned long long* __restrict__ n_probes, uint32_t nb_cap,
                                                         uint32_t* __restrict__ err) {
  __shared__ uint4 s_hash[TH_HB];               // TH_NU / 2 buckets (64 KiB): N+(v) as a hash set of 4-slot buckets
  __shared__ uint32_t s_off[TH_VCH + 1];        // short lists of the chunk (compacted): prefix of |N+(u)|, [ns] = total
  __shared__ uint32_t s_st[TH_VCH];             // start of that N+(u) in onbr
  __shared__ uint32_t s_loff[TH_VCH + 1];       // long lists (>= TH_LONG items), compacted the same way
  __shared__ uint32_t s_lst[TH_VCH];
  __shared__ uint4 s_w4[TH_HBLOCK / WAVE];
  __shared__ uint32_t s_claim;
  constexpr int PER = TH_VCH / TH_HBLOCK;
  constexpr int NW = TH_HBLOCK / WAVE;
  uint32_t* hs = reinterpret_cast<uint32_t*>(s_hash);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint64_t cnt = 0, probes = 0;
  const uint32_t nh = *n_heavy;
  uint32_t table_v = TH_EMPTY;   // the vertex whose N+ the LDS table holds (block-uniform)
  // a contiguous run of items per block, cut at equal shares of the items' work (k_tri_hwork +
  // exclusive scan: pre[h] = work before item h, pre[nh] = total): the chunks of one heavy vertex are
  // consecutive items, so a block rebuilds its table only when its run moves to the next vertex
  uint32_t h0 = 0, h1 = 0;
  if (!order) {   // equal-work runs (phased: items claimed one at a time in phase order)
    const unsigned long long W = pre[nh];
    auto lower = [&](unsigned long long t) {   // first h with pre[h] >= t
      uint32_t a = 0, b = nh;
      while (a < b) {
        const uint32_t m = (a + b) >> 1;
        if (pre[m] < t) a = m + 1;
        else b = m;
      }
      return a;
    };
    const unsigned long long lo = frac_share(W, blockIdx.x, gridDim.x), hi = frac_share(W, blockIdx.x + 1, gridDim.x);
    h0 = uni(lower(lo));
    h1 = blockIdx.x + 1 == gridDim.x ? nh : uni(lower(hi));
  }
  for (uint32_t k = 0;; ++k) {
    uint32_t hi;
    if (order) {
      if (tid == 0) s_claim = atomicAdd(claim, 1u);
      __syncthreads();
      hi = uni(s_claim);
      if (hi >= nh) break;
      hi = order[hi];
    } else {
      hi = h0 + k;
      if (hi >= h1) break;
    }
    const uint2 item = heavy[hi];   // (v, in-chunk)
    const uint32_t v = item.x;
    const uint2 ro = out_range[v], ri = in_range[v];
    const uint32_t d = ro.y - ro.x;
    // N+(v) lies in (v, last]: when that span fits the table's bits, a bitmap over it (one 4-byte LDS
    // read and a bit test per probe, no hash and no chain); else the hash set, or for lists longer than
    // the table a binary search in HBM.  Degree-class ranks put every heavy vertex near the top of the
    // order, so the span is short (R-MAT s22: < 2^16 for all of the heavy work).
    const uint32_t span = uni(d ? onbr[ro.y - 1] - v : 0u);
    const bool bitmap = TH_BITMAP && span <= TH_BSPAN && nb_cap > 1;   // (tiny test tables: hash only)
    const bool in_lds = bitmap || d <= TH_NU;
    uint32_t nb = 16;
    while (nb * 2 < d && nb < TH_HB) nb <<= 1;
    nb = min(nb, nb_cap);
    const uint32_t bmask = nb - 1;
    __syncthreads();   // the previous item is done with the table and the list arrays
    if (in_lds && table_v != v) {
      if (bitmap) {   // bit (w - v - 1) for w in N+(v); word nw stays zero
        const uint32_t nw = (span + 31) / 32;
        for (uint32_t i = tid; i <= nw; i += TH_HBLOCK) hs[i] = 0u;
        __syncthreads();
        for (uint32_t i = tid; i < d; i += TH_HBLOCK) {
          const uint32_t o = onbr[ro.x + i] - v - 1;
          atomicOr(&hs[o >> 5], 1u << (o & 31));
        }
      } else {
        for (uint32_t i = tid; i < nb * 4; i += TH_HBLOCK) hs[i] = TH_EMPTY;
        __syncthreads();
        for (uint32_t i = tid; i < d; i += TH_HBLOCK) th_insert(hs, onbr[ro.x + i], bmask, err);
      }
      table_v = v;
    }
    const uint32_t* nvl = onbr + ro.x;
    auto probe = [&](const uint32_t (&x)[TH_ILP], uint32_t nv) -> uint32_t {
      if (bitmap) {
        // items lie past v (suffixes of N+(u) after v): bit o = w - v - 1.  Branch-free, so the TH_ILP LDS
        // reads issue together: an item past the span reads a zero bit (its word's bits past the span,
        // or the zero word nw), and the lane's invalid items are masked arithmetically.  (Written with
        // a conditional per item, the compiler put each item's LDS read in its own branch and waited
        // for it there: eight LDS round trips in series per step.)
        const uint32_t nw = (span + 31) / 32;
        uint32_t o[TH_ILP], wv[TH_ILP];
#pragma unroll
        for (int j = 0; j < TH_ILP; ++j) {
          o[j] = x[j] - v - 1;
          wv[j] = hs[min(o[j] >> 5, nw)];
        }
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < TH_ILP; ++j) c += (wv[j] >> (o[j] & 31)) & ((uint32_t)j < nv ? 1u : 0u);
        return c;
      }
      if (in_lds) return th_probe(s_hash, bmask, x, nv, err);
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) {
        uint32_t a = 0, b = d;   // lower bound of x in N+(v)
        while (a < b) {
          const uint32_t mid = (a + b) >> 1;
          if (nvl[mid] < x[j]) a = mid + 1;
          else b = mid;
        }
        c += ((uint32_t)j < nv && a < d && nvl[a] == x[j]) ? 1u : 0u;
      }
      return c;
    };
    const uint32_t c0 = ri.x + item.y * TH_VCH;
    const uint32_t cn = min(TH_VCH, ri.y - c0);
    // the chunk's lists, split into short and long and compacted: one block scan of (short lists,
    // short items, long lists, long items)
    uint32_t du[PER], su[PER];
    uint4 mine = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t i = tid * PER + j;
      const uint2 ru = sfx[c0 + min(i, cn - 1)];
      su[j] = ru.x;
      du[j] = i < cn ? ru.y - ru.x : 0u;
      if (du[j] >= TH_LONG) { mine.z += 1; mine.w += du[j]; }
      else if (du[j]) { mine.x += 1; mine.y += du[j]; }
    }
    uint4 inc = make_uint4(wave_inclusive_sum(mine.x), wave_inclusive_sum(mine.y), wave_inclusive_sum(mine.z),
                           wave_inclusive_sum(mine.w));
    if (lane == 63) s_w4[w] = inc;
    __syncthreads();
    uint4 base = make_uint4(0, 0, 0, 0), tot = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const uint4 x = s_w4[i];
      if (i < w) { base.x += x.x; base.y += x.y; base.z += x.z; base.w += x.w; }
      tot.x += x.x; tot.y += x.y; tot.z += x.z; tot.w += x.w;
    }
    uint32_t si = base.x + inc.x - mine.x, so = base.y + inc.y - mine.y;
    uint32_t li = base.z + inc.z - mine.z, lo_ = base.w + inc.w - mine.w;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (du[j] >= TH_LONG) {
        s_loff[li] = lo_;
        s_lst[li] = su[j];
        ++li;
        lo_ += du[j];
      } else if (du[j]) {
        s_off[si] = so;
        s_st[si] = GS_TH_WALK ? su[j] - so : su[j];   // (walk: item k of list si is onbr[k + s_st[si]])
        ++si;
        so += du[j];
      }
    }
    const uint32_t ns = uni(tot.x), srun = uni(tot.y), nl = uni(tot.z), lrun = uni(tot.w);
    if (tid == 0) {
      s_off[ns] = srun;
      s_loff[nl] = lrun;
    }
    probes += srun + lrun;   // block-uniform
    __syncthreads();
    // short lists: TH_ILP consecutive items per thread, at most one list boundary per step
    uint32_t top = 1;
    while (2 * top < ns) top <<= 1;
    auto gather_short = [&](uint32_t k0, uint32_t (&x)[TH_ILP]) -> uint32_t {
      const uint32_t kb = k0 + tid * TH_ILP;
      const uint32_t kk = min(kb, srun - 1);
      uint32_t q = 0;
      for (uint32_t st = top; st; st >>= 1) {
        const uint32_t t = q + st;
        q = (t < ns && s_off[min(t, ns - 1)] <= kk) ? t : q;
      }
#if GS_TH_WALK
      // (round 6) branch-free: the next TH_ILP - 1 list starts in one batch of LDS reads, as a mask of the
      // items that start a list (s_off[ns] = srun lies past every item); item j lies in list q + (starts at
      // or before j), whose base is one more batch of reads -- instead of a branch and an LDS round trip
      // per item, in series
      uint32_t m = 0;
#pragma unroll
      for (int i = 1; i < TH_ILP; ++i) {
        const uint32_t d = s_off[min(q + (uint32_t)i, ns)] - kb;
        m |= d < (uint32_t)TH_ILP ? 1u << d : 0u;
      }
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) {
        const uint32_t ql = min(q + (uint32_t)__builtin_popcount(m & ((2u << j) - 1u)), ns - 1);
        x[j] = onbr[min(kb + j, srun - 1) + s_st[ql]];
      }
      return kb < srun ? min((uint32_t)TH_ILP, srun - kb) : 0u;
#endif
      uint32_t nx = s_off[q + 1], base = s_st[q] - s_off[q];   // item kj of list q: onbr[kj + base]
#pragma unroll
      for (int j = 0; j < TH_ILP; ++j) {
        const uint32_t kj = min(kb + j, srun - 1);
        if (kj >= nx) {
          ++q;
          base = s_st[q] - nx;
          nx = s_off[q + 1];
        }
        x[j] = onbr[kj + base];
      }
      return kb < srun ? min((uint32_t)TH_ILP, srun - kb) : 0u;
    };
    constexpr uint32_t SSTEP = TH_HBLOCK * TH_ILP, LSTEP = WAVE * TH_ILP;
    th_pipelined<GS_TH_PIPE>(0u, srun, SSTEP, gather_short, probe, cnt);
    // long lists: wave w walks items [w, w + 1) * lrun / NW in 64-item segments (one load of 64
    // consecutive items); a segment spans at most two lists (every long list >= 64 items)
    if (lrun) {
      const uint32_t wu = uni((uint32_t)w);
      const uint32_t a0 = uni((uint32_t)((uint64_t)lrun * wu / NW)), a1 = uni((uint32_t)((uint64_t)lrun * (wu + 1) / NW));
      uint32_t q = 0;
      {
        uint32_t t2 = 1;
        while (2 * t2 < nl) t2 <<= 1;
        for (uint32_t st = t2; st; st >>= 1) {
          const uint32_t t = q + st;
          q = (t < nl && uni(s_loff[min(t, nl - 1)]) <= a0) ? t : q;
        }
      }
      // item k of list q: onbr[k + dq]; of list q + 1: onbr[k + dq1] (wave-uniform offsets)
      uint32_t qe = uni(s_loff[q + 1]), q1s = q + 1 < nl ? uni(s_lst[q + 1]) : 0u;
      uint32_t dq = uni(s_lst[q]) - uni(s_loff[q]), dq1 = q1s - qe;
      auto gather_long = [&](uint32_t k0, uint32_t (&x)[TH_ILP]) -> uint32_t {
#pragma unroll
        for (int j = 0; j < TH_ILP; ++j) {
          const uint32_t seg = k0 + (uint32_t)j * WAVE;   // wave-uniform
          while (qe <= seg && q + 1 < nl) {
            ++q;
            dq = dq1;
            qe = uni(s_loff[q + 1]);
            q1s = q + 1 < nl ? uni(s_lst[q + 1]) : 0u;
            dq1 = q1s - qe;
          }
          const uint32_t k = min(seg + (uint32_t)lane, a1 - 1);
          x[j] = onbr[k + (k < qe ? dq : dq1)];
        }
        const uint32_t rem = a1 - k0;
        return rem > (uint32_t)lane ? min((uint32_t)TH_ILP, (rem - lane + WAVE - 1) / WAVE) : 0u;
      };
      th_pipelined<GS_TH_PIPE>(a0, a1, LSTEP, gather_long, probe, cnt);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, WAVE);
  if (lane == 0 && cnt) atomicAdd(total, (unsigned long long)cnt);
  if (tid == 0 && probes) atomicAdd(n_probes, (unsigned long long)probes);
}

}  // namespace gs
