"""GPU: the triangle count's degree classes from a sample of the window (gs_triangles.hip triangles_impl).

The orientation needs only some total order of the ids -- every triangle is counted once, at its
lowest-ranked vertex, whatever the order (WindowTriangles.java:83-140 emits each candidate pair once per
vertex; the count does not depend on which vertex) -- and the degree classes only keep the out-lists
short.  Windows of >= 2^26 edges take their classes from the degrees of n / 4 of their edges by
default (16 slices spread over the window); GS_TRI_DEG_SAMPLE = 1 restores the exact degrees (read once per process, so each setting runs
in its own interpreter).  On an R-MAT scale-22 window (2^26 edges, self-loops kept) both settings must
give the same count, and the stage times' "vertices with edges" must equal the window's distinct ids
in both (with sampled classes it comes from the count's vertex pass, k_tri_lclass).  The same window
sorted by source (a replayed edge list) must count as with exact classes, at about the exact-degree time.
Both orders are also checked against the oracle: the count less the order's self-pair term is the
window's triangle count from the oracle's forward algorithm on the self-loop-free edges.
"""
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent

SCRIPT = textwrap.dedent("""
    import os
    import sys
    import time
    os.environ["GS_TRI_DEG_SAMPLE"] = "{k}"
    import torch
    sys.path.insert(0, {root!r})
    import __graft_entry__ as ge
    pkg = ge.load_package()
    eng = pkg.Engine(0)
    s, d = eng.generate_rmat(22, 1 << 26, 0x5EED07)
    exact, wrapped, has = eng.triangles(s, d)
    t = eng.stage_times()
    distinct = int(torch.unique(torch.cat([s, d])).numel())
    # the same window with its records sorted by source (a replayed edge list): the sample (slices
    # spread over the window) still finds the hubs, so the window costs about what exact classes cost
    o = torch.sort(s, stable=True).indices
    ss, sd = s[o].contiguous(), d[o].contiguous()
    def best(a, b):
        ms = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = eng.triangles(a, b)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
        return r[0], min(ms)
    c_shuf, ms_shuf = best(s, d)
    c_sort, ms_sort = best(ss, sd)
    # the independent check (first run only): each order's count less its self-pair term (the reference's
    # HashSet-order quirk for self-loops) is the window's triangle count, which the oracle's forward
    # algorithm gives on the self-loop-free edges (oracle/gs_oracle.c gso_triangles_fwd_mt)
    sp, sp_sort, T = eng.triangles_selfpair(s, d), eng.triangles_selfpair(ss, sd), -1
    if {k} == 4:
        orc = ge.load_oracle()
        sn, dn = s.cpu().numpy(), d.cpu().numpy()
        keep = sn != dn
        T = orc.triangles_fwd_mt(sn[keep], dn[keep])
    print("RESULT", exact, t.vertices, distinct, c_sort, int(ms_shuf * 1000), int(ms_sort * 1000), sp, sp_sort, T)
    eng.close()
""")


def _run(k):
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=str(ROOT), k=k)], capture_output=True, text=True,
                       timeout=190)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT")][-1]
    return tuple(int(x) for x in line.split()[1:])


@pytest.mark.timeout(400)   # two interpreters, each a 2^26-edge window seven times; the first also runs the oracle
def test_sampled_degree_classes_same_count_and_vertices():
    count_s, verts_s, distinct, sorted_s, us_shuf, us_sort, sp, sp_sort, T = _run(4)
    count_e, verts_e, distinct_e, sorted_e, us_shuf_e, us_sort_e = _run(1)[:6]
    # both orders against the oracle: count = triangles + the order's self-pair term
    assert count_s - sp == T and sorted_s - sp_sort == T, (count_s, sp, sorted_s, sp_sort, T)
    assert distinct == distinct_e
    # (the window keeps its self-loops, so the reference's count depends on the record order -- the
    # self-pair term follows HashSet order, which follows insertion order -- and the sorted window may
    # count differently; each order must count the same with sampled and exact classes)
    assert count_s == count_e and sorted_s == sorted_e, (count_s, count_e, sorted_s, sorted_e)
    assert verts_e == distinct, (verts_e, distinct)
    assert verts_s == distinct, (verts_s, distinct)
    print(f"shuffled / source-sorted window: sampled {us_shuf / 1e3:.2f} / {us_sort / 1e3:.2f} ms, "
          f"exact {us_shuf_e / 1e3:.2f} / {us_sort_e / 1e3:.2f} ms")
    # a source-sorted window keeps the sampled classes' work bound (a prefix sample lost it)
    assert us_sort < 1.5 * us_sort_e, (us_sort, us_sort_e)
