"""Boundary-adjacency volume of the split-window triangle count (analysis, not a test).

For an R-MAT window (the oracle's generator: test infrastructure) split over N ranks, restates the
gs_tri_dist_* geometry of gs_triangles.hip in numpy -- raw degrees, degree-class ranks (2 classes per
octave, stable by id), oriented unique edges u -> v, route ranges owner(u) = u * N >> B, equal-work count
ranges C (work d+(d+1)/2) -- and reports per rank the row elements it receives in step 4:
  * boundary: the rows of C it did not build, then the non-empty rows of their targets it holds in
    neither C nor R (gs_tri_dist_plan / _need), and
  * all-gather: every row other ranks built (what step 4 did before round 4).
Bytes = 4 per element.  python tests/analysis_tri_boundary.py 24 [26]
"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import oracle.oracle as orc  # noqa: E402


def deg_class(d):
    d = d.astype(np.int64)
    lz = np.floor(np.log2(np.maximum(d, 1))).astype(np.int64)
    half = np.where(lz > 0, (d >> np.maximum(lz - 1, 0)) & 1, 0)
    return np.where(d == 0, 0, np.minimum(63, 1 + 2 * lz + half))


def geometry(scale, seed=0x5EED04):
    E = 16 << scale
    t = time.time()
    src, dst = orc.gen_rmat(scale, E, seed, no_self_loops=True)
    V = 1 << scale
    deg = np.bincount(src, minlength=V) + np.bincount(dst, minlength=V)
    rank = np.empty(V, np.int64)
    rank[np.argsort(deg_class(deg), kind="stable")] = np.arange(V)
    del deg
    a, b = rank[src], rank[dst]
    del src, dst
    key = np.minimum(a, b) << scale
    key |= np.maximum(a, b)
    del a, b
    draw = np.bincount(key >> scale, minlength=V).astype(np.int64)   # oriented out-degree with duplicates
    key = np.unique(key)
    u, v = key >> scale, key & (V - 1)
    del key
    dplus = np.bincount(u, minlength=V).astype(np.int64)
    print(f"s{scale}: E = {E}, unique oriented edges M = {len(u)} ({4 * len(u) / 1e9:.2f} GB of rows), "
          f"{time.time() - t:.0f} s", flush=True)
    return V, u, v, dplus, draw


def split(pre, V, N):
    W = int(pre[V])
    return [0 if q == 0 else V if q == N else int(np.searchsorted(pre[:V], W * q // N, side="left")) for q in range(N + 1)]


def volumes_routed(V, u, v, dplus, draw, N):
    """gs_tri_dist_route / _plan / _need as built: route ranges R at equal shares of the raw work
    draw(draw+1)/2, count ranges C at equal shares of the exact work d+(d+1)/2; per rank (elements of
    the rows of C it did not build + the non-empty rows of targets in neither range, elements an
    all-gather delivers)"""
    pre = np.concatenate([[0], np.cumsum(dplus)])
    rq = split(np.concatenate([[0], np.cumsum(draw * (draw + 1) // 2)]), V, N)
    cq = split(np.concatenate([[0], np.cumsum(dplus * (dplus + 1) // 2)]), V, N)
    out = []
    for r in range(N):
        c0, c1, r0, r1 = cq[r], cq[r + 1], rq[r], rq[r + 1]
        lo, hi = max(c0, r0), min(c1, r1)
        crows = int(pre[c1] - pre[c0]) - (int(pre[hi] - pre[lo]) if lo < hi else 0)
        tg = v[int(pre[c0]):int(pre[c1])]
        tg = np.unique(tg[((tg < c0) | (tg >= c1)) & ((tg < r0) | (tg >= r1))])
        out.append((crows + int(dplus[tg].sum()), int(pre[V] - (pre[r1] - pre[r0]))))
    return out


def volumes(V, B, u, v, dplus, N):
    pre = np.concatenate([[0], np.cumsum(dplus)])
    prew = np.concatenate([[0], np.cumsum(dplus * (dplus + 1) // 2)])
    W = int(prew[V])
    cq = [0 if q == 0 else V if q == N else int(np.searchsorted(prew[:V], W * q // N, side="left")) for q in range(N + 1)]
    rq = [min(V, -(-(q << B) // N)) for q in range(N + 1)]
    out = []
    for r in range(N):
        c0, c1, r0, r1 = cq[r], cq[r + 1], rq[r], rq[r + 1]
        lo, hi = max(c0, r0), min(c1, r1)
        own_c = int(pre[hi] - pre[lo]) if lo < hi else 0
        crows = int(pre[c1] - pre[c0]) - own_c
        tg = v[int(pre[c0]):int(pre[c1])]
        tg = np.unique(tg[((tg < c0) | (tg >= c1)) & ((tg < r0) | (tg >= r1))])
        req = int(dplus[tg].sum())
        allg = int(pre[V] - (pre[r1] - pre[r0]))
        out.append((crows + req, allg))
    return out


if __name__ == "__main__":
    for scale in [int(x) for x in sys.argv[1:]] or [22]:
        V, u, v, dplus, draw = geometry(scale)
        print("| window | N | boundary recv per rank, max / mean (MB) | all-gather recv per rank, max / mean (MB) "
              "| max ratio | sum ratio |")
        for N in (2, 4, 8):
            vol = volumes_routed(V, u, v, dplus, draw, N)
            b = [x[0] * 4 / 1e6 for x in vol]
            g = [x[1] * 4 / 1e6 for x in vol]
            print(f"| R-MAT s{scale} | {N} | {max(b):.0f} / {np.mean(b):.0f} | {max(g):.0f} / {np.mean(g):.0f} | "
                  f"{max(b) / max(g):.2f} | {sum(b) / sum(g):.2f} |", flush=True)
