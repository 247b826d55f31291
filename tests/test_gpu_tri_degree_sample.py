"""GPU: the triangle count's degree classes from a sample of the window (gs_triangles.hip triangles_impl).

The orientation needs only some total order of the ids -- every triangle is counted once, at its
lowest-ranked vertex, whatever the order (WindowTriangles.java:83-140 emits each candidate pair once per
vertex; the count does not depend on which vertex) -- and the degree classes only keep the out-lists
short.  Windows of >= 2^26 edges take their classes from the degrees of their first n / 4 edges by
default; GS_TRI_DEG_SAMPLE = 1 restores the exact degrees (read once per process, so each setting runs
in its own interpreter).  On an R-MAT scale-22 window (2^26 edges, self-loops kept) both settings must
give the same count, and the stage times' "vertices with edges" must equal the window's distinct ids
in both (with sampled classes it comes from the count's vertex pass, k_tri_lclass).
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
    print("RESULT", exact, t.vertices, distinct)
    eng.close()
""")


def _run(k):
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=str(ROOT), k=k)], capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT")][-1]
    return tuple(int(x) for x in line.split()[1:])


def test_sampled_degree_classes_same_count_and_vertices():
    count_s, verts_s, distinct = _run(4)
    count_e, verts_e, distinct_e = _run(1)
    assert distinct == distinct_e
    assert count_s == count_e, (count_s, count_e)
    assert verts_e == distinct, (verts_e, distinct)
    assert verts_s == distinct, (verts_s, distinct)
