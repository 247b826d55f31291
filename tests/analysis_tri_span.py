"""Heavy-vertex span analysis for the k_tri_heavy bitmap: the degree-class renumbering
restated in numpy on an R-MAT window, then the share of heavy work whose N+(v) span fits 2^k bits.
    python tests/analysis_tri_span.py SCALE   (s24 needs ~20 GB of host memory)"""
import sys, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / 'tests'))
import __graft_entry__ as ge
orc = ge.load_oracle()
from test_distributed_gloo import OracleTriEngine
scale = int(sys.argv[1])
n = 16 << scale
s, d = orc.gen_rmat(scale, n, 0x5EED04, no_self_loops=True)
V = 1 << scale
deg = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
cls = OracleTriEngine.deg_class(deg)
rank = np.empty(V, np.int64); rank[np.argsort(cls, kind="stable")] = np.arange(V)
a, b = rank[s], rank[d]
u, v = np.minimum(a, b), np.maximum(a, b)
k = np.unique(u * V + v); u, v = k // V, k % V
dp = np.bincount(u, minlength=V)
start = np.concatenate([[0], np.cumsum(dp)])
# work per middle vertex m (as v in the kernel): sum over in-neighbours x of |N+(x) after m| = for edge (x->m): end(x) - (pos of m in N+(x)) - 1
pos = np.arange(len(u)) - start[u]
suffix = dp[u] - pos - 1            # items of N+(u) after v, for edge u->v
work = np.bincount(v, weights=suffix, minlength=V)
mx = np.zeros(V, np.int64); np.maximum.at(mx, u, v)
span = np.where(dp > 0, mx - np.arange(V), 0)
heavy = dp > 256
tot = work.sum(); hw = work[heavy].sum()
print("scale", scale, "V", V, "unique", len(u), "probes", tot, "heavy work frac", hw / tot, "heavy vertices", heavy.sum())
for bits in (15, 16, 17, 18, 19, 20, 21):
    m = heavy & (span < (1 << bits))
    print(f"  span < 2^{bits}: heavy work frac {work[m].sum()/max(hw,1):.3f}, vertices {m.sum()}")
print("heavy d+ max", dp[heavy].max() if heavy.any() else 0, "heavy rank min", np.arange(V)[heavy].min() if heavy.any() else 0)
