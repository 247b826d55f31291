"""Where the triangle count's probes go, and three ways to cut them that do not pay (analysis,
not a test).

For an R-MAT window (the oracle's generator: test infrastructure), restated in numpy as in
analysis_tri_boundary.geometry (degree-class ranks, oriented unique edges u -> v with u < v):
  * probes: the count's work, sum over u of d+(u)(d+(u)-1)/2 (every in-entry u of v probes the suffix of
    N+(u) past v against N+(v));
  * smaller side: probing min(|suffix of N+(u) past v|, d+(v)) per edge instead;
  * range cut: probing only the suffix items inside [min N+(v), max N+(v)] (a binary search each end);
  * narrow items: the share of the probes whose v lies in the top 2^k ranks, so that every item of the
    suffixes it reads does too and fits 2 bytes relative to the top range (k_tri_heavy's onbr16, k = 16);
  * dense core: the share of the probes whose three vertices all lie among the top K ranks (where a
    dense K x K 0/1 product on the matrix cores, 2K^3 int8 operations, could count them instead).
python tests/analysis_tri_core.py 22 [24]
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
from analysis_tri_boundary import geometry  # noqa: E402


def report(scale):
    V, u, v, dplus, _ = geometry(scale)
    pre = np.concatenate([[0], np.cumsum(dplus)])
    M = len(u)
    pos = np.arange(M)
    suf_lo, suf_hi = pos + 1, pre[u + 1]
    suf = suf_hi - suf_lo
    total = int(suf.sum())
    print(f"probes: {total / 1e9:.2f} G")
    smaller = int(np.minimum(suf, dplus[v]).sum())
    print(f"smaller side per edge: {smaller / 1e9:.2f} G ({smaller / total:.3f})")
    has = dplus > 0
    lo = np.zeros(V, np.int64)
    hi = np.full(V, -1, np.int64)
    lo[has] = v[pre[:-1][has]]
    hi[has] = v[pre[1:][has] - 1]
    key = u * V + v
    a = np.maximum(np.searchsorted(key, u * V + lo[v], "left"), suf_lo)
    b = np.minimum(np.searchsorted(key, u * V + hi[v], "right"), suf_hi)
    cut = np.where(dplus[v] > 0, np.maximum(b - a, 0), 0)
    print(f"range cut: {cut.sum() / 1e9:.2f} G ({cut.sum() / total:.3f})")
    for k in (14, 15, 16, 17, 18):
        m = v >= V - (1 << k) - 1
        print(f"v in the top 2^{k} ranks: {suf[m].sum() / 1e9:.2f} G probes ({suf[m].sum() / total:.3f})")
    for K in (4096, 8192, 16384, 32768, 65536):
        c = V - K
        core = int((dplus[c:] * (dplus[c:] - 1) // 2).sum())
        print(f"dense core K = {K}: {core / 1e9:.2f} G probes ({core / total:.3f}), 2K^3 = {2 * K ** 3 / 1e12:.1f} T int8 ops")


if __name__ == "__main__":
    for s in [int(x) for x in sys.argv[1:]] or [22]:
        report(s)
