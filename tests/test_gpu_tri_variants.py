"""GPU: the oriented-key variants of the triangle count (gs_triangles.hip tri_okeys) on the same window.

The key step has a one-pass form (k_tri_okeys: the whole rank table) and a two-pass form for rank
tables past the Infinity Cache (k_tri_okeys_lo / _hi), each with U = 1, 2 or 4 edges per lane per step,
and (round 6, chosen when V > 2^25) the partitioned form: the records partitioned by each endpoint's top
id bits in turn, so each rank gather hits an L2-resident slice of the table (TriPartA / TriPartB,
k_tri_okeys_part).  The default picks one form per window size; GS_TRI_OKEYS_PART, GS_TRI_OKEYS_SPLIT
and GS_TRI_OKEYS_UNROLL force the others (read once per process, so every case runs in its own
interpreter).  Every combination must give the forward algorithm's count (WindowTriangles.java:83-140
restated in oracle/gs_oracle.c) on a self-loop-free R-MAT scale-18 window; the partitioned form also on
a window that keeps its self-loops (the count less the self-pair term), where its pass 2 marks them.
The partitioned form sorts the keys by u alone and each out-list in LDS (k_tri_segsort, round 6;
GS_TRI_SEGSORT=0: the full LSD sort instead); GS_TRI_SEGSORT_CAP=64 shrinks the LDS chunk so that every
out-list longer than 64 keys takes k_tri_segsort_long's stable passes over HBM.  The transposed sort's first
pass reads the out-lists directly (TriTpaySrc, histograms from k_tri_uo_write); GS_TRI_TPAY_FUSED=0 restores
k_tri_tpay's copy.
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
    os.environ.update(GS_TRI_OKEYS_SPLIT="{split}", GS_TRI_OKEYS_UNROLL="{unroll}", GS_TRI_OKEYS_PART="{part}",
                      GS_TRI_SEGSORT="{seg}", GS_TRI_SEGSORT_CAP="{cap}", GS_TRI_TPAY_FUSED="{tfuse}")
    import numpy as np
    sys.path.insert(0, {root!r})
    import __graft_entry__ as ge
    pkg, orc = ge.load_package(), ge.load_oracle()
    eng = pkg.Engine(0)
    s, d = orc.gen_rmat(18, 16 << 18, 0x5EED04, no_self_loops=True)
    exact, wrapped, has = eng.triangles(s, d)
    want = orc.triangles_fwd_mt(s, d)
    assert exact == want, (exact, want)
    if {loops}:   # R-MAT with its self-loops: count = triangles of the loop-free edges + the self-pair term
        s, d = orc.gen_rmat(18, 16 << 18, 0x5EED05)
        keep = s != d
        assert (~keep).any()
        exact, wrapped, has = eng.triangles(s, d)
        sp = eng.triangles_selfpair(s, d)
        want = orc.triangles_fwd_mt(s[keep], d[keep])
        assert exact - sp == want, (exact, sp, want)
    eng.close()
    print("triangles", exact)
""")


@pytest.mark.parametrize("split,unroll,part,seg,cap,tfuse", [
    (0, 1, 0, 1, 4096, 1), (0, 2, 0, 1, 4096, 1), (1, 1, 0, 1, 4096, 1), (1, 2, 0, 1, 4096, 1), (1, 4, 0, 1, 4096, 1),
    (0, 4, 1, 0, 4096, 1), (0, 4, 1, 1, 4096, 1), (0, 4, 1, 1, 64, 1), (0, 4, 1, 1, 4096, 0)])
def test_okeys_variants_same_count(split, unroll, part, seg, cap, tfuse):
    # (the knobs are set inside the child, before the library reads them: the child inherits this
    # process's environment unchanged)
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=str(ROOT), split=split, unroll=unroll,
                                                                part=part, loops=part, seg=seg, cap=cap,
                                                                tfuse=tfuse)],
                       capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "triangles" in r.stdout


def test_partition_histograms_guessed_from_the_previous_window(pkg, oracle):
    """Windows after the first count the partitioned keys' histograms in their id scan at the previous window's id
    width (tri_geometry); a window of another width misses and counts them itself.  Widths 24, 24, 20, 24 (R-MAT
    scale 24 ids and 20), each window against the forward algorithm."""
    eng = pkg.Engine(0)
    try:
        for scale, seed in [(24, 0x5EED21), (24, 0x5EED22), (20, 0x5EED23), (24, 0x5EED24)]:
            s, d = oracle.gen_rmat(scale, 1 << 21, seed, no_self_loops=True)
            exact, wrapped, has = eng.triangles(s, d)
            assert exact == oracle.triangles_fwd_mt(s, d), (scale, seed)
    finally:
        eng.close()
