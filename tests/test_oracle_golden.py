"""Pin the CPU oracle against the reference's own golden vectors (tests/golden/reference_fixtures.json,
extracted from TestSlice / TestReverse / TestUndirected / WindowTrianglesITCase by
tests/golden/extract_reference_fixtures.py).  CPU only."""
import json
from collections import defaultdict
from pathlib import Path

import numpy as np
import pytest

FIX = json.loads((Path(__file__).parent / "golden" / "reference_fixtures.json").read_text())
DIRS = {"IN": 0, "OUT": 1, "ALL": 2}


def _graph():
    e = np.array(FIX["slice_graph"]["edges"], dtype=np.int64)
    return e[:, 0].copy(), e[:, 1].copy(), e[:, 2].copy()


@pytest.mark.parametrize("case", FIX["slice_cases"], ids=lambda c: c["name"])
def test_testslice_goldens(oracle, case):
    s, d, v = _graph()
    direction = DIRS[case["direction"]]
    if case["kind"] == "reduce":       # SumEdgeValuesReduce, TestSlice.java:242-249
        k, r = oracle.window_reduce(s, d, v, direction, oracle.OP_SUM)
        got = {(str(a), str(b)) for a, b in zip(k, r)}
    elif case["kind"] == "fold":       # SumEdgeValues from Tuple2(0, 0), TestSlice.java:233-240
        k, r = oracle.window_fold(s, d, v, direction, oracle.OP_SUM, 0)
        got = {(str(a), str(b)) for a, b in zip(k, r)}
    else:                              # SumEdgeValuesApply: sum > 50 ? big : small, TestSlice.java:251-268
        k, off, nb, vals = oracle.window_csr(s, d, v, direction)
        got = set()
        for u in range(len(k)):
            tot = int(vals[off[u]:off[u + 1]].sum())
            got.add((str(k[u]), "big" if tot > 50 else "small"))
    assert got == {tuple(x) for x in case["expected"]}   # compareResultsByLinesInMemory: unordered


def test_reverse_and_undirected_expansion(oracle):
    s, d, v = _graph()
    # IN-keyed records == reverse(): group the golden reverse() edge list by f0 in arrival order
    for direction, golden in ((0, FIX["reverse_expected"]), (2, FIX["undirected_expected"])):
        k, off, nb, vals = oracle.window_csr(s, d, v, direction)
        want = defaultdict(list)
        for a, b, w in golden:
            want[a].append((b, w))
        got = {int(k[u]): [(int(nb[j]), int(vals[j])) for j in range(off[u], off[u + 1])] for u in range(len(k))}
        if direction == 2:
            # the golden lists e, e.reverse() per edge; per-key arrival order must match exactly
            assert got == {a: lst for a, lst in want.items()}
        else:
            assert got == dict(want)


def test_window_triangles_itcase(oracle):
    t = FIX["triangles"]
    e = np.array(t["edges_src_trg_ts"], dtype=np.int64)
    out = []
    for start, idx in oracle.split_windows(e[:, 2], t["window_ms"]):
        w_ref, ex_ref, has_ref, tree = oracle.window_triangles_ref(e[idx, 0], e[idx, 1])
        w_fwd, ex_fwd, has_fwd = oracle.window_triangles_fwd(e[idx, 0], e[idx, 1])
        assert (w_ref, ex_ref, has_ref) == (w_fwd, ex_fwd, has_fwd) and not tree
        if has_ref:
            out.append([w_ref, start + t["window_ms"] - 1])
    assert sorted(out) == sorted(t["expected"])


def test_triangle_algorithms_agree_random(oracle):
    """The reference candidate rule and the forward algorithm agree (incl. multi-edges, self-loops)."""
    rng = np.random.default_rng(5)
    for trial in range(30):
        V = int(rng.integers(3, 60))
        n = int(rng.integers(1, 400))
        s = rng.integers(0, V, n).astype(np.int64)
        d = rng.integers(0, V, n).astype(np.int64)
        if trial % 3 == 0:
            s, d = s * 1_000_003 + 7, d * 1_000_003 + 7   # sparse large IDs -> non-trivial HashSet order
        w_ref, ex_ref, has_ref, tree = oracle.window_triangles_ref(s, d)
        w_fwd, ex_fwd, has_fwd = oracle.window_triangles_fwd(s, d)
        assert (w_ref, ex_ref, has_ref) == (w_fwd, ex_fwd, has_fwd), trial


def test_hashset_order_model(oracle):
    """java.util.HashSet<Long> sizing used by the candidate rule: 16 buckets up to 12 entries, x2 after."""
    assert [oracle.java_hashset_cap(k) for k in (0, 1, 12, 13, 24, 25, 48, 49)] == [16, 16, 16, 32, 32, 64, 64, 128]


def test_hashset_exact_known_answers(oracle):
    """Known answers of the exact JDK HashMap restatement, derived by hand from HashMap.putVal /
    treeifyBin / resize / TreeNode.treeify (JDK 8+; no JVM in this image, so these pin it):
     - 16, 32, .., 144 all hash to bucket 0 of 16; the 9th add makes treeifyBin resize (capacity 16 < 64)
       to 32, where evens (bucket 0) precede odds (bucket 16), each in insertion order;
     - eight of them stay one plain bin;
     - 64, .., 704: the 9th and 10th adds resize to 32 and 64 (all still bucket 0), the 11th treeifies:
       ascending inserts give the red-black root 256 (4th key), moveRootToFront puts it first."""
    ex, pl, f = oracle.hashset_order([16 * j for j in range(1, 10)])
    assert ex.tolist() == [32, 64, 96, 128, 16, 48, 80, 112, 144] and f == 2
    assert pl.tolist() == [16 * j for j in range(1, 10)]
    ex, pl, f = oracle.hashset_order([16 * j for j in range(1, 9)])
    assert ex.tolist() == pl.tolist() == [16 * j for j in range(1, 9)] and f == 0
    ex, pl, f = oracle.hashset_order([64 * j for j in range(1, 12)])
    assert ex.tolist() == [256, 64, 128, 192] + [64 * j for j in range(5, 12)] and f == 3


def test_hashset_exact_matches_plain_without_collisions(oracle):
    """Random Long ids never fill a bin to 9 at these sizes: the exact simulation equals the plain-bin
    model (capacity from the size, buckets ascending, insertion order inside a bin)."""
    rng = np.random.default_rng(17)
    for k in (1, 12, 13, 100, 1000, 5000):
        ids = np.unique(rng.integers(-(1 << 62), 1 << 62, k))
        ids = rng.permutation(ids)
        ex, pl, f = oracle.hashset_order(ids)
        assert f == 0 and np.array_equal(ex, pl) and sorted(ex.tolist()) == sorted(ids.tolist())


def test_hashset_exact_tree_bins_split(oracle):
    """Ids j << 20 crowd few buckets at every capacity: bins treeify at 64, and the later resizes split
    tree bins (untreeify at <= 6, re-treeify above).  The order is always a permutation of the set."""
    for k in (20, 200, 2000, 6000):
        ids = np.arange(1, k + 1, dtype=np.int64) << 20
        ex, pl, f = oracle.hashset_order(ids)
        assert f == (2 if k == 20 else 3) and sorted(ex.tolist()) == ids.tolist() and not np.array_equal(ex, pl)


def test_generators_deterministic(oracle):
    a = oracle.gen_rmat(10, 1000, 1)
    b = oracle.gen_rmat(10, 1000, 1)
    c = oracle.gen_rmat(10, 500, 1, first_edge=500)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[0][500:], c[0]) and np.array_equal(a[1][500:], c[1])
    s, d = oracle.gen_rmat(10, 5000, 2, no_self_loops=True)
    assert not np.any(s == d)
    s, d = oracle.gen_uniform(100, 5000, 3)
    assert not np.any(s == d) and s.max() < 100 and d.min() >= 0


def test_reduce_java_arithmetic(oracle):
    s = np.zeros(3, np.int64)
    d = np.ones(3, np.int64)
    v = np.array([2**62, 2**62, 2**62], dtype=np.int64)
    k, r = oracle.window_reduce(s, d, v, 1, 0)
    assert int(r[0]) == -(2**62)  # 3 * 2^62 wraps (Long addition)
    v32 = np.array([2**30, 2**30, 2**30], dtype=np.int32)
    k, r = oracle.window_reduce(s, d, v32, 1, 0)
    assert r[0] == np.int32(-(2**30))  # 3 * 2^30 wraps to -2^30
    f = np.array([0.0, -0.0, np.nan], dtype=np.float64)
    k, r = oracle.window_reduce(s[:2], d[:2], f[:2], 1, 1)
    assert np.signbit(r[0])  # Math.min(0.0, -0.0) = -0.0
    k, r = oracle.window_reduce(s, d, f, 1, 2)
    assert np.isnan(r[0])


def test_count_candidates_itcase_windows(oracle):
    """Stage 2 (CountTriangles + sum) over the reference's own candidate records of each ITCase window
    gives the ITCase outputs: (2,399) (3,799) (2,1199)."""
    t = FIX["triangles"]
    e = np.array(t["edges_src_trg_ts"], dtype=np.int64)
    starts = e[:, 2] - e[:, 2] % t["window_ms"]
    got = []
    for st in np.unique(starts):
        idx = starts == st
        a, b, f, tree = oracle.window_candidates(e[idx, 0], e[idx, 1])
        w, ex, has, groups = oracle.count_candidates(a, b, f)
        w_ref, ex_ref, has_ref, _ = oracle.window_triangles_ref(e[idx, 0], e[idx, 1])
        assert (w, ex, has) == (w_ref, ex_ref, has_ref)
        if has:
            got.append([w, int(st + t["window_ms"] - 1)])
    assert sorted(got) == sorted(t["expected"])


def test_count_candidates_rules(oracle):
    """Groups without an edge record emit nothing; an edge-only group emits 0 (has_output, no count)."""
    a = np.array([1, 1, 1, 2, 2, 3], np.int64)
    b = np.array([5, 5, 5, 7, 7, 9], np.int64)
    f = np.array([1, 1, 0, 1, 1, 0], np.uint8)
    assert oracle.count_candidates(a, b, f) == (2, 2, True, 2)
    assert oracle.count_candidates(a[3:5], b[3:5], f[3:5]) == (0, 0, False, 0)
    assert oracle.count_candidates(a[:0], b[:0], f[:0]) == (0, 0, False, 0)


BAD_RECORDS = [b"1  2 3", b" 1 2 3", b"1 2", b"1 2 ", b"1 2 3x", b"1 2 9223372036854775808", b"", b"1 2 -",
               b"1\t2\t+", b"1,2,3", b"1 2 -9223372036854775809", b"0x1 2 3"]


def test_parse_edges_text_itcase_file(oracle):
    """The ITCase input file ("src trg ts" lines, ExamplesTestData.java:21-34) parses to its edges."""
    e = np.array(FIX["triangles"]["edges_src_trg_ts"], dtype=np.int64)
    text = "\n".join(" ".join(str(x) for x in r) for r in e).encode()
    s, d, t = oracle.parse_edges_text(text)
    assert np.array_equal(np.stack([s, d, t], 1), e)


def test_parse_edges_text_rules(oracle):
    """split("\\s") + Long.parseLong: CRLF, tabs, a '+' sign, extreme values, extra fields, no final newline."""
    s, d, t = oracle.parse_edges_text(b"1 2 3\r\n-4\t+5 6 extra fields\n9223372036854775807 "
                                      b"-9223372036854775808 0\f\n7 8 9")
    assert s.tolist() == [1, -4, 9223372036854775807, 7]
    assert d.tolist() == [2, 5, -9223372036854775808, 8]
    assert t.tolist() == [3, 6, 0, 9]
    assert [len(x) for x in oracle.parse_edges_text(b"")] == [0, 0, 0]
    for bad in BAD_RECORDS:
        with pytest.raises(ValueError, match="record 1"):
            oracle.parse_edges_text(b"1 2 3\n" + bad + b"\n4 5 6\n")


def test_connected_components_fixture(oracle):
    """ConnectedComponentsTest.java:19-38: edges 1-2 1-3 2-3 1-5 6-7 8-9 -> {1,2,3,5} {6,7} {8,9}."""
    cc = FIX["connected_components"]
    e = np.array(cc["edges"], dtype=np.int64)
    v, lab = oracle.components(e[:, 0], e[:, 1])
    comps = {}
    for x, l in zip(v.tolist(), lab.tolist()):
        comps.setdefault(l, []).append(x)
    assert sorted(sorted(c) for c in comps.values()) == sorted(cc["expected"])
    assert all(l == min(c) for l, c in comps.items())


def test_disjoint_set_fixture(oracle):
    """DisjointSetTest.java: union(i, i + 2), i < 8 -> 10 elements in 2 sets (evens, odds); merged into
    a set of union(i, i + 100), i < 8 -> 18 elements in 2 sets."""
    ds = FIX["disjoint_set"]
    u = np.array(ds["unions"], dtype=np.int64)
    v, lab = oracle.components(u[:, 0], u[:, 1])
    assert len(v) == ds["size"] and len(set(lab.tolist())) == ds["roots"]
    assert all(l == x % 2 for x, l in zip(v.tolist(), lab.tolist()))
    m = np.array(ds["merge_unions"], dtype=np.int64)
    v2, l2 = oracle.components(m[:, 0], m[:, 1])
    vm, lm = oracle.components(u[:, 0], u[:, 1], prev=(v2, l2))   # ds2.merge(ds)
    assert len(vm) == ds["merged_size"] and len(set(lm.tolist())) == ds["merged_roots"]
