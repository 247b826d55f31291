"""GPU: ConnectedComponents (gs_window_components; library/ConnectedComponents.java on
WindowGraphAggregation) against the oracle's DisjointSet restatement (oracle/gs_oracle.c gso_components,
pinned to ConnectedComponentsTest / DisjointSetTest in tests/test_oracle_golden.py): the partition of the
vertices seen so far, labelled by the smallest vertex of each component."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
FIX = json.loads((Path(__file__).parent / "golden" / "reference_fixtures.json").read_text())


def _same(got, want):
    gk, gl = (x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x) for x in got)
    assert np.array_equal(gk, want[0]) and np.array_equal(gl, want[1])


def test_connected_components_itcase_through_the_api(pkg):
    """ConnectedComponentsTest.java: graph.aggregate(new ConnectedComponents(5)) -> 3 components."""
    cc = FIX["connected_components"]
    e = np.array(cc["edges"], dtype=np.int64)
    env = pkg.StreamExecutionEnvironment.getExecutionEnvironment()
    g = pkg.SimpleEdgeStream(pkg.EdgeColumns(e[:, 0], e[:, 1]), env)
    out = g.aggregate(pkg.ConnectedComponents(cc["merge_window_ms"])).collect()
    comps = {}
    for v, lab in out:
        comps.setdefault(lab, []).append(v)
    assert sorted(sorted(c) for c in comps.values()) == sorted(cc["expected"])


@pytest.mark.parametrize("kind", ["rmat", "sparse_ids", "sparse_ids_large", "chains", "loops"])
def test_components_vs_oracle(engine, oracle, kind):
    rng = np.random.default_rng(3)
    if kind == "rmat":
        s, d = oracle.gen_rmat(16, 60_000, 0x5EED09)           # many small components + a giant one
    elif kind == "sparse_ids":                                  # negative and 64-bit spread ids
        s, d = oracle.gen_rmat(12, 5_000, 0x5EED0A)
        s, d = s * 7_919_000_003 - (1 << 61), d * 7_919_000_003 - (1 << 61)
    elif kind == "sparse_ids_large":                            # the relabel path's two-phase unions (>= 65536 records)
        s, d = oracle.gen_rmat(16, 300_000, 0x5EED0E)
        s, d = s * 7_919_000_003 - (1 << 61), d * 7_919_000_003 - (1 << 61)
    elif kind == "chains":                                      # long paths: deep union chains
        p = rng.permutation(200_000).astype(np.int64)
        s, d = p[:-1].copy(), p[1:].copy()
        o = rng.permutation(len(s))
        s, d = s[o], d[o]
    else:                                                       # self-loops make singleton components
        s = rng.integers(0, 5000, 20_000).astype(np.int64)
        d = np.where(rng.random(20_000) < 0.3, s, rng.integers(0, 5000, 20_000)).astype(np.int64)
    want = oracle.components(s, d)
    _same(engine.components(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()), want)
    _same(engine.components(s, d), want)                        # host columns


def test_components_accumulate_over_windows(engine, oracle):
    """transientState = false: window k's state = window k-1's state merged with window k's edges."""
    s, d = oracle.gen_rmat(15, 80_000, 0x5EED0B)
    state_g, state_o = None, None
    for w in range(4):
        ws, wd = s[w * 20_000:(w + 1) * 20_000], d[w * 20_000:(w + 1) * 20_000]
        state_o = oracle.components(ws, wd, state_o)
        state_g = engine.components(torch.from_numpy(ws).cuda(), torch.from_numpy(wd).cuda(), state_g)
        _same(state_g, state_o)
    _same(state_g, oracle.components(s, d))                    # = the components of all the edges


def test_components_config_size(engine, oracle):
    """A large window (R-MAT s20, 2^24 edges): the partition equals the oracle's."""
    s, d = oracle.gen_rmat(20, 1 << 24, 0x5EED0C)
    want = oracle.components(s, d)
    _same(engine.components(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()), want)


def test_components_partials_at_parallelism(pkg, oracle):
    """Environment parallelism 4 (GraphAggregation.java:103-116): one running state per non-empty
    partition's partial, through gs_window_components, each against the oracle's DisjointSet over the
    previous state and that partition's records (arrival index mod 4)."""
    s, d = oracle.gen_rmat(12, 20_000, 0x5EED0D)
    ts = (np.arange(len(s)) * 2).astype(np.int64)             # windows of 500 records (1000 ms)
    env = pkg.StreamExecutionEnvironment()
    env.setParallelism(4)
    out = pkg.SimpleEdgeStream(pkg.EdgeColumns(s, d, None, ts), env).aggregate(pkg.ConnectedComponents(1000))
    assert len(out.windows) == 4 * (len(s) // 500)
    state, i = None, 0
    for w0 in range(0, len(s), 500):
        for k in range(4):
            sel = np.arange(w0, w0 + 500)
            sel = sel[sel % 4 == k]
            state = oracle.components(s[sel], d[sel], state)
            _same(out.windows[i].columns, state)
            i += 1
    _same(out.windows[-1].columns, oracle.components(s, d))   # the last state = every edge's components
