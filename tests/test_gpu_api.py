"""GPU: the reference's own tests, re-run through the host mirror of the Java API (stream.py) and
libgellyhip.so — TestSlice (9 cases), WindowTrianglesITCase — plus triangle parity vs the oracle."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FIX = json.loads((Path(__file__).parent / "golden" / "reference_fixtures.json").read_text())


class SumEdgeValuesApply:
    """TestSlice.java:251-268 — user EdgesApply (host-side, after GPU grouping)."""

    def applyOnEdges(self, vertexID, neighbors, out):
        s = sum(v for _, v in neighbors)
        out.collect((vertexID, "big" if s > 50 else "small"))


@pytest.mark.parametrize("case", FIX["slice_cases"], ids=lambda c: c["name"])
def test_testslice_through_api(pkg, case):
    env = pkg.StreamExecutionEnvironment.getExecutionEnvironment()
    graph = pkg.SimpleEdgeStream(env.fromCollection([tuple(e) for e in FIX["slice_graph"]["edges"]]), env)
    w = graph.slice(pkg.Time.of(1, pkg.TimeUnit.SECONDS), pkg.EdgeDirection[case["direction"]])
    if case["kind"] == "fold":
        res = w.foldNeighbors((0, 0), pkg.SumValuesFold())
    elif case["kind"] == "reduce":
        res = w.reduceOnEdges(pkg.SumReduce())
    else:
        apply_fn = type("A", (pkg.EdgesApply,), {"applyOnEdges": SumEdgeValuesApply.applyOnEdges})()
        res = w.applyOnNeighbors(apply_fn)
    got = {(str(a), str(b)) for a, b in res.collect()}
    assert got == {tuple(x) for x in case["expected"]}


def test_user_lambdas_match_builtins(pkg):
    """A user EdgesReduce / EdgesFold (host after GPU grouping) agrees with the GPU built-ins."""
    env = pkg.StreamExecutionEnvironment.getExecutionEnvironment()
    rng = np.random.default_rng(3)
    edges = [(int(a), int(b), int(c)) for a, b, c in zip(rng.integers(0, 50, 400), rng.integers(0, 50, 400),
                                                          rng.integers(-99, 99, 400))]
    g = pkg.SimpleEdgeStream(env.fromCollection(edges), env)

    class UserSum(pkg.EdgesReduce):
        def reduceEdges(self, a, b):
            return a + b

    class UserFold(pkg.EdgesFold):
        def foldEdges(self, acc, vid, nid, val):
            return (vid, acc[1] + val)

    for d in (pkg.EdgeDirection.OUT, pkg.EdgeDirection.IN, pkg.EdgeDirection.ALL):
        w = g.slice(pkg.Time.seconds(1), d)
        assert sorted(w.reduceOnEdges(UserSum()).collect()) == sorted(w.reduceOnEdges(pkg.SumReduce()).collect())
        assert sorted(w.foldNeighbors((0, 5), UserFold()).collect()) == \
            sorted(w.foldNeighbors((0, 5), pkg.SumValuesFold()).collect())


def test_window_triangles_itcase(pkg, tmp_path):
    """WindowTrianglesITCase: WindowTriangles.main(<edges file>, <out>, "400") -> (2,399) (3,799) (2,1199)."""
    from gelly_streaming_amd import triangles

    t = FIX["triangles"]
    f = tmp_path / "edges.txt"
    f.write_text("\n".join(" ".join(str(x) for x in e) for e in t["edges_src_trg_ts"]))
    out = tmp_path / "result"
    lines = triangles.main([str(f), str(out), str(t["window_ms"])])
    got = sorted(tuple(int(x) for x in ln.strip("()").split(",")) for ln in lines)
    assert got == sorted(tuple(x) for x in t["expected"])
    assert out.read_text().strip().splitlines() == lines


def test_windowing_event_time(pkg, oracle):
    """Several tumbling windows from ascending timestamps: per-window results == oracle per window."""
    n = 20000
    s, d = oracle.gen_rmat(10, n, 41)
    v = oracle.gen_values(n, 42, oracle.DT_I64)
    ts = np.sort(np.random.default_rng(1).integers(0, 5000, n)).astype(np.int64)
    env = pkg.StreamExecutionEnvironment.getExecutionEnvironment()
    cols = pkg.EdgeColumns(s, d, v, ts)
    g = pkg.SimpleEdgeStream(cols, env)
    res = g.slice(pkg.Time.milliseconds(700), pkg.EdgeDirection.ALL).reduceOnEdges(pkg.SumReduce())
    got = res.collectWithTimestamps()
    want = []
    for start, idx in oracle.split_windows(ts, 700):
        k, r = oracle.window_reduce(s[idx], d[idx], v[idx], 2, 0)
        want += [((int(a), int(b)), start + 699) for a, b in zip(k, r)]
    assert got == want


@pytest.mark.parametrize("kind", ["uniform_c1", "rmat", "dense_small", "multi_edges", "heavy"])
def test_triangles_vs_oracle(engine, oracle, kind):
    if kind == "uniform_c1":      # BASELINE C1 shape: uniform V=2^16, 1M edges, no self-loops
        s, d = oracle.gen_uniform(1 << 16, 1_000_000, 0x5EED01)
    elif kind == "rmat":
        s, d = oracle.gen_rmat(14, 200_000, 0x5EED04, no_self_loops=True)
    elif kind == "dense_small":
        s, d = oracle.gen_uniform(40, 2000, 9)
    elif kind == "heavy":         # dense: oriented out-degrees > TH_DMAX (512) take k_tri_heavy
        rng = np.random.default_rng(11)
        a, b = rng.integers(0, 1500, 900_000), rng.integers(0, 1500, 900_000)
        keep = a != b
        s, d = a[keep].astype(np.int64), b[keep].astype(np.int64)
    else:
        s0, d0 = oracle.gen_uniform(300, 5000, 10)
        s, d = np.concatenate([s0, d0, s0]), np.concatenate([d0, s0, d0])   # duplicates + reversed copies
    w_fwd, ex_fwd, has = oracle.window_triangles_fwd(s, d)
    ex, wrapped, has_g = engine.triangles(*[torch.from_numpy(x).cuda() for x in (s, d)])
    assert (ex, wrapped, has_g) == (ex_fwd, w_fwd, has)


def _clique(n, shuffle_seed):
    iu = np.triu_indices(n, 1)
    s, d = iu[0].astype(np.int64) * 31 + 5, iu[1].astype(np.int64) * 31 + 5
    p = np.random.default_rng(shuffle_seed).permutation(len(s))
    return s[p], d[p]


def test_triangles_clique_hub_chunks(engine, oracle):
    """K_n has C(n, 3) triangles (pinned on K_30 by the oracle).  On K_4200 the (degree, id) orientation
    gives out-lists up to 4199 > TH_VCH: k_tri_heavy's several in-entry chunks."""
    from math import comb
    s, d = _clique(30, 1)
    w, ex, has = oracle.window_triangles_fwd(s, d)
    assert (ex, has) == (comb(30, 3), True)
    n = 4200
    s, d = _clique(n, 2)
    ex, wrapped, has = engine.triangles(*[torch.from_numpy(x).cuda() for x in (s, d)])
    want = comb(n, 3)
    w32 = want & 0xFFFFFFFF
    assert (ex, wrapped, has) == (want, w32 - (1 << 32) if w32 >= (1 << 31) else w32, True)


def test_triangles_matches_reference_rule(engine, oracle):
    """Small windows: the GPU count equals the reference candidate rule (GenerateCandidateEdges +
    CountTriangles + sum) computed literally by the oracle."""
    rng = np.random.default_rng(8)
    for trial in range(20):
        V = int(rng.integers(3, 80))
        n = int(rng.integers(1, 600))
        s = rng.integers(0, V, n).astype(np.int64)
        d = rng.integers(0, V, n).astype(np.int64)
        keep = s != d
        s, d = s[keep], d[keep]
        if len(s) == 0:
            continue
        w_ref, ex_ref, has_ref, _ = oracle.window_triangles_ref(s, d)
        ex, wrapped, has_g = engine.triangles(s, d)
        assert (ex, wrapped, has_g) == (ex_ref, w_ref, has_ref), trial


def test_triangles_empty_window(engine):
    ex, wrapped, has = engine.triangles(np.empty(0, np.int64), np.empty(0, np.int64))
    assert (ex, wrapped, has) == (0, 0, False)


def _cand_case(oracle, rng, kind):
    if kind == "small_ids":
        V, n = int(rng.integers(3, 60)), int(rng.integers(1, 500))
        s, d = rng.integers(0, V, n), rng.integers(0, V, n)
    elif kind == "sparse_ids":      # IDs >> table size: non-trivial HashSet order, multi-entry bins
        V, n = int(rng.integers(5, 200)), int(rng.integers(50, 2000))
        s, d = rng.integers(0, V, n) * 1_000_003 + 17, rng.integers(0, V, n) * 1_000_003 + 17
    elif kind == "negative_ids":    # Long.hashCode of negative IDs, signed order of the > v filter
        V, n = int(rng.integers(5, 100)), int(rng.integers(50, 1500))
        s, d = rng.integers(-V, V, n) * 65537, rng.integers(-V, V, n) * 65537
    else:                           # R-MAT with hubs
        s, d = oracle.gen_rmat(10, 3000, int(rng.integers(1, 1 << 30)))
    return np.asarray(s, np.int64), np.asarray(d, np.int64)


@pytest.mark.parametrize("kind", ["small_ids", "sparse_ids", "negative_ids", "rmat"])
def test_candidates_match_reference_rule(engine, oracle, kind):
    """gs_window_candidates == GenerateCandidateEdges record-for-record (same per-vertex sequence,
    including the JDK HashSet iteration order of the candidate pairs and the self pairs)."""
    rng = np.random.default_rng({"small_ids": 1, "sparse_ids": 2, "negative_ids": 3, "rmat": 4}[kind])
    for trial in range(6):
        s, d = _cand_case(oracle, rng, kind)
        ra, rb, rf, flags = oracle.window_candidates(s, d)
        ga, gb, gf = engine.candidates(*[torch.from_numpy(x).cuda() for x in (s, d)])
        assert engine.last_candidates_jdk_flags == flags, (kind, trial)
        assert np.array_equal(ga.cpu().numpy(), ra), (kind, trial)
        assert np.array_equal(gb.cpu().numpy(), rb), (kind, trial)
        assert np.array_equal(gf.cpu().numpy(), rf), (kind, trial)


def test_candidates_through_api_and_host_buffers(pkg, engine, oracle):
    s, d = _cand_case(oracle, np.random.default_rng(9), "sparse_ids")
    ra, rb, rf, _ = oracle.window_candidates(s, d)
    ga, gb, gf = engine.candidates(s, d)          # host columns
    assert np.array_equal(ga, ra) and np.array_equal(gb, rb) and np.array_equal(gf, rf)
    env = pkg.StreamExecutionEnvironment.getExecutionEnvironment()
    g = pkg.SimpleEdgeStream(pkg.EdgeColumns(s, d), env)
    recs = g.slice(pkg.Time.seconds(1), pkg.EdgeDirection.ALL).applyOnNeighbors(pkg.GenerateCandidateEdges()).collect()
    assert recs == [(int(a), int(b), int(f)) for a, b, f in zip(ra, rb, rf)]


def test_triangles_with_self_loops(engine, oracle):
    """Windows with self-loops: the reference's self-pair quirk (j = i) counts (x, x) candidates when
    x has a self-loop, except for the last HashSet element — reproduced exactly."""
    rng = np.random.default_rng(12)
    for trial in range(25):
        V = int(rng.integers(2, 50))
        n = int(rng.integers(1, 500))
        s = rng.integers(0, V, n).astype(np.int64)
        d = np.where(rng.random(n) < 0.15, s, rng.integers(0, V, n)).astype(np.int64)
        if trial % 2:
            s, d = s * 7919 + 3, d * 7919 + 3
        w_ref, ex_ref, has_ref, _ = oracle.window_triangles_ref(s, d)
        ex, wrapped, has = engine.triangles(s, d)
        assert (ex, wrapped, has) == (ex_ref, w_ref, has_ref), trial


@pytest.mark.parametrize("flags", [0, 1, 2])
def test_triangles_degree_paths(pkg, oracle, flags):
    """The renumbering's raw degrees come from the bucket path (COUNT over both endpoints); a ctx
    that refuses it (GS_FLAG_SORT_ONLY) or an id range too wide for its buckets takes the global-
    atomic fallback (k_tri_deg).  Every path gives the exact count (any vertex order does)."""
    from gelly_streaming_amd import _lib as L
    s, d = oracle.gen_rmat(13, 150_000, 0x5EED07, no_self_loops=True)
    if flags == 2:   # spread the ids over 2^27: beyond the bucket path's range, within 28 key bits
        s, d = s * 13_001 + 5, d * 13_001 + 5
        flags = 0
    w, ex, has = oracle.window_triangles_fwd(s, d)
    with pkg.Engine(0, flags=L.GS_FLAG_SORT_ONLY if flags else 0) as e:
        got = e.triangles(*[torch.from_numpy(x).cuda() for x in (s, d)])
    assert got == (ex, w, has)


def test_triangles_parts_sum_to_whole(engine, oracle):
    """gs_window_triangles_part over nparts (the multi-GPU split) sums to the whole-window count."""
    s, d = oracle.gen_rmat(13, 120_000, 0x5EED04, no_self_loops=True)
    S, D = [torch.from_numpy(x).cuda() for x in (s, d)]
    whole, wrapped, _ = engine.triangles(S, D)
    for nparts in (1, 2, 3, 8):
        assert sum(engine.triangles_part(S, D, p, nparts) for p in range(nparts)) == whole


@pytest.mark.parametrize("kind", ["small_ids", "sparse_ids", "negative_ids", "rmat"])
def test_count_candidates_matches_reference(engine, oracle, kind):
    """gs_window_count_candidates (stage 2: keyBy(0,1) CountTriangles + sum(0)) over the window's
    GenerateCandidateEdges records equals the oracle's restatement and the window's triangle count."""
    rng = np.random.default_rng({"small_ids": 11, "sparse_ids": 12, "negative_ids": 13, "rmat": 14}[kind])
    for trial in range(4):
        s, d = _cand_case(oracle, rng, kind)
        ra, rb, rf, _ = oracle.window_candidates(s, d)
        want = oracle.count_candidates(ra, rb, rf)
        got = engine.count_candidates(*[torch.from_numpy(x).cuda() for x in (ra, rb, rf)])
        assert got == (want[1], want[0], want[2], want[3]), (kind, trial)
        w_ref, ex_ref, has_ref, _ = oracle.window_triangles_ref(s, d)
        assert (got[0], got[1], got[2]) == (ex_ref, w_ref, has_ref)


def test_count_candidates_edge_cases(engine, oracle):
    rng = np.random.default_rng(21)
    # random records: candidate-only groups, edge-only groups, mixed; host columns
    n = 200_000
    a = rng.integers(-50, 50, n) * 1_000_003
    b = rng.integers(0, 300, n)
    f = (rng.random(n) < 0.8).astype(np.uint8)
    want = oracle.count_candidates(a, b, f)
    assert engine.count_candidates(a, b, f) == (want[1], want[0], want[2], want[3])
    # all candidates -> no output; empty window -> no output
    assert engine.count_candidates(a, b, np.ones(n, np.uint8))[2] is False
    assert engine.count_candidates(a[:0], b[:0], f[:0]) == (0, 0, False, 0)
    # IDs spanning 2^32 or more go through relabeled IDs (host columns)
    a2, b2, f2 = np.array([0, 1 << 40, 0, 1 << 40]), np.array([0, 1, 0, 1]), np.array([0, 1, 1, 0], np.uint8)
    want = oracle.count_candidates(a2, b2, f2)
    assert engine.count_candidates(a2, b2, f2) == (want[1], want[0], want[2], want[3])


def test_count_candidates_large_window(engine, oracle):
    """Full emission + stage 2 on a 2^16-edge R-MAT window equals the direct triangle count."""
    s, d = oracle.gen_rmat(14, 1 << 16, 0x5EED04, no_self_loops=True)
    ts, td = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    a, b, f = engine.candidates(ts, td)
    got = engine.count_candidates(a, b, f)
    ex, w, has = engine.triangles(ts, td)
    assert (got[0], got[1], got[2]) == (ex, w, has)


def test_two_stage_pipeline_itcase(pkg):
    """WindowTriangles written as the reference writes it — applyOnNeighbors(GenerateCandidateEdges)
    then keyBy(0,1) CountTriangles + sum(0) (here triangles.count_triangles) — gives the ITCase output."""
    from gelly_streaming_amd import triangles

    t = FIX["triangles"]
    e = np.array(t["edges_src_trg_ts"], dtype=np.int64)
    env = pkg.StreamExecutionEnvironment.getExecutionEnvironment()
    g = pkg.SimpleEdgeStream(pkg.EdgeColumns(e[:, 0].copy(), e[:, 1].copy(), e[:, 2].copy()), env,
                             pkg.EdgeValueTimestampExtractor())
    ws = g.slice(pkg.Time.milliseconds(t["window_ms"]), pkg.EdgeDirection.ALL)
    cands = ws.applyOnNeighbors(triangles.GenerateCandidateEdges())
    got = triangles.count_triangles(cands, ws.engine).collect()
    assert sorted(got) == sorted(tuple(x) for x in t["expected"])


def _edge_text(rng, n, crlf=False, extra=False):
    from gelly_streaming_amd.textio import format_edges_text

    cols = [rng.integers(-(1 << 40), 1 << 40, n), rng.integers(0, 1 << 62, n), rng.integers(-(1 << 63), (1 << 63) - 1, n)]
    cols[0][: n // 4] = rng.integers(0, 100, n // 4)     # short lines too
    t = format_edges_text(*cols, eol=b"\r\n" if crlf else b"\n")
    if extra:
        t = t.replace(b"\n", b" 17 junk\n", n // 2)    # fields after the third are ignored
    return t, cols


@pytest.mark.parametrize("case", ["plain", "crlf_extra", "no_final_newline", "device_text", "host_out"])
def test_parse_edges_text_matches_oracle(engine, oracle, case):
    rng = np.random.default_rng(["plain", "crlf_extra", "no_final_newline", "device_text", "host_out"].index(case))
    n = 1 << 18
    text, cols = _edge_text(rng, n, crlf=case == "crlf_extra", extra=case == "crlf_extra")
    if case == "no_final_newline":
        text = text[:-1]
    want = oracle.parse_edges_text(text)
    arg = torch.from_numpy(np.frombuffer(text, np.uint8).copy()).cuda() if case == "device_text" else text
    got = engine.parse_edges_text(arg, out_device=case != "host_out")
    for g, w, c in zip(got, want, cols):
        g = g.cpu().numpy() if hasattr(g, "cpu") else g
        assert np.array_equal(g, w) and np.array_equal(w, c)


def test_parse_edges_text_errors_and_edges(engine, oracle):
    from gelly_streaming_amd import GsError
    from test_oracle_golden import BAD_RECORDS

    rng = np.random.default_rng(5)
    good, _ = _edge_text(rng, 5000)
    lines = good.split(b"\n")
    for bad in BAD_RECORDS:
        at = int(rng.integers(0, 5000))
        text = b"\n".join(lines[:at] + [bad] + lines[at:])
        with pytest.raises(ValueError, match=f"record {at}$"):
            oracle.parse_edges_text(text)
        with pytest.raises(GsError, match=f"record {at} "):
            engine.parse_edges_text(text)
    assert [len(x) for x in engine.parse_edges_text(b"")] == [0, 0, 0]
    for small in (b"1 2 3", b"1 2 3\n", b"1 2 3\r\n", b"-1\t-2\t-3 x"):
        got = [x.cpu().numpy() for x in engine.parse_edges_text(small)]
        want = oracle.parse_edges_text(small)
        assert all(np.array_equal(g, w) for g, w in zip(got, want)), small


@pytest.mark.parametrize("kind", ["small_ids", "sparse_ids", "rmat"])
def test_candidate_count_sizing(engine, oracle, kind):
    """The sizing call (capacity 0) of gs_window_candidates returns exactly the oracle's record count."""
    rng = np.random.default_rng({"small_ids": 31, "sparse_ids": 32, "rmat": 33}[kind])
    for _ in range(3):
        s, d = _cand_case(oracle, rng, kind)
        assert engine.candidate_count(s, d) == oracle.candidate_count(s, d)


def test_text_to_window_reduce(engine, oracle):
    """Input path end to end: edge text parsed on the GPU, then slice(OUT).reduceOnEdges(SUM) over the
    third column as the value, equals the oracle on the oracle-parsed columns."""
    from gelly_streaming_amd.textio import format_edges_text

    s, d = oracle.gen_rmat(14, 1 << 17, 0x5EED07)
    v = oracle.gen_values(1 << 17, 7, oracle.DT_I64)
    text = format_edges_text(s, d, v)
    gs, gd, gv = engine.parse_edges_text(text)
    k, r = engine.reduce(gs, gd, gv, 1, 0)
    os_, od, ov = oracle.parse_edges_text(text)
    wk, wv = oracle.window_reduce(os_, od, ov, 1, 0)
    assert np.array_equal(k.cpu().numpy(), wk) and np.array_equal(r.cpu().numpy(), wv)


def test_triangle_table_overflow_is_an_error_not_a_hang(pkg, oracle):
    """Every LDS hash-set insert / probe chain is bounded: with GS_FLAG_TEST_TINY_TABLES (one-bucket
    sets) the sets overflow, the kernels give up and the call returns GS_EDEVICE instead of hanging."""
    from gelly_streaming_amd import _lib as L
    s, d = oracle.gen_rmat(14, 200_000, 0x5EED04, no_self_loops=True)
    S, D = (torch.from_numpy(x).cuda() for x in (s, d))
    with pkg.Engine(0, flags=L.GS_FLAG_TEST_TINY_TABLES) as e:
        with pytest.raises(pkg.GsError) as ei:
            e.triangles(S, D)
        assert ei.value.status == L.GS_EDEVICE and "hash set" in str(ei.value)
    with pkg.Engine(0) as e:   # the normal engine on the same window
        assert e.triangles(S, D)[0] == oracle.window_triangles_fwd(s, d)[1]


@pytest.mark.parametrize("loops", [False, True])
def test_triangles_arbitrary_long_ids(engine, oracle, loops):
    """IDs spanning the whole Long range (sparse, negative): the window is relabeled (order-preserving
    compact IDs) and the count equals the reference rule on the ORIGINAL IDs — with self-loops too, where
    the self-pair term depends on the JDK HashSet order of the original Longs (WindowTriangles.java:95-105)."""
    rng = np.random.default_rng(7 + loops)
    s, d = oracle.gen_rmat(11, 60_000, 0x5EED04, no_self_loops=not loops)
    ids = np.unique(rng.integers(-(1 << 62), 1 << 62, 5000))
    ids = rng.permutation(ids)[: 1 << 11]
    S_, D_ = ids[s], ids[d]
    w, ex, has, tree = oracle.window_triangles_ref(S_, D_)
    assert not tree
    got = engine.triangles(*(torch.from_numpy(x).cuda() for x in (S_, D_)))
    assert got == (ex, w, has)
    if not loops:   # relabeling is order-preserving: the same count as the dense window
        assert got[0] == engine.triangles(*(torch.from_numpy(x).cuda() for x in (s, d)))[0]


def test_count_candidates_ids_spanning_2_pow_32(engine, oracle):
    """Stage 2 over candidate records whose IDs span more than 2^32: grouped through relabeled IDs."""
    s, d = oracle.gen_rmat(10, 20_000, 5, no_self_loops=True)
    ids = np.random.default_rng(3).integers(-(1 << 60), 1 << 60, 1 << 10)
    a, b, f, _ = oracle.window_candidates(ids[s], ids[d])
    want = oracle.count_candidates(a, b, f)
    got = engine.count_candidates(*(torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (a, b, f)))
    assert (got[1], got[0], got[2], got[3]) == want


def _jdk_case(oracle, case):
    rng = np.random.default_rng(sum(map(ord, case)))
    if case == "resize16":            # a bin of 9 below capacity 64: treeifyBin resizes instead
        s, d = np.zeros(20, np.int64), np.arange(1, 21, dtype=np.int64) * 16
    elif case == "tree24":            # one tree bin at capacity 256
        s, d = np.zeros(200, np.int64), np.arange(1, 201, dtype=np.int64) << 24
    elif case == "tree20_split":      # tree bins split and re-treeified by later resizes
        s, d = np.zeros(3000, np.int64), np.arange(1, 3001, dtype=np.int64) << 20
    elif case == "hub_groups":        # large sets mixing tree bins and plain ones, well past capacity 256:
        ids = np.concatenate([np.arange(1, 4_001, dtype=np.int64) << 24,                   # bins of many
                              rng.integers(1, 1 << 40, 6_000).astype(np.int64)])          # spread
        ids = np.unique(ids)
        rng.shuffle(ids)
        s = np.concatenate([np.zeros(len(ids), np.int64), np.full(len(ids) // 2, 7, np.int64)])
        d = np.concatenate([ids, ids[: len(ids) // 2]])
    elif case == "many_vertices":     # hundreds of complex sets in one window, plus plain ones
        V = 400
        s = np.repeat(-np.arange(1, V + 1, dtype=np.int64), 20)
        d = 16 * (np.tile(np.arange(1, 21, dtype=np.int64), V) + 20 * np.repeat(np.arange(V), 20))
        d[: 20 * (V // 2)] += 3       # half the sets spread over buckets: plain
    else:                             # R-MAT window over ids j << 20: complex sets of many sizes
        s, d = oracle.gen_rmat(10, 20_000, 0x5EED31)
        s, d = (np.asarray(s, np.int64) + 1) << 20, (np.asarray(d, np.int64) + 1) << 20
    p = rng.permutation(len(s))
    return np.ascontiguousarray(s[p]), np.ascontiguousarray(d[p])


@pytest.mark.parametrize("case", ["resize16", "tree24", "tree20_split", "hub_groups", "many_vertices", "rmat_shifted"])
def test_candidates_exact_jdk_order(engine, oracle, case):
    """Neighbour sets whose java.util.HashMap leaves the plain-bin model -- a bin of 9 that makes
    treeifyBin resize below capacity 64, red-black tree bins, tree bins split by later resizes, hub sets of
    10^4 ids simulated by 256 bin groups past capacity 256, many such sets in one window -- are simulated
    exactly on the GPU (k_hs_detect finds them, k_hs_jdk_prefix / _group replay putVal): the records equal
    the oracle's exact JDK restatement, and the reported flags agree."""
    s, d = _jdk_case(oracle, case)
    ra, rb, rf, flags = oracle.window_candidates(s, d)
    assert flags
    ga, gb, gf = engine.candidates(*(torch.from_numpy(x).cuda() for x in (s, d)))
    assert engine.last_candidates_jdk_flags == flags
    assert np.array_equal(ga.cpu().numpy(), ra) and np.array_equal(gb.cpu().numpy(), rb)
    assert np.array_equal(gf.cpu().numpy(), rf)


def test_triangles_self_pairs_exact_jdk_order(engine, oracle):
    """The self-pair term (self-loops) skips each set's LAST HashSet element, so it depends on the exact
    JDK order: windows over ids j << 20 (tree bins and collision resizes) match the oracle."""
    s, d = oracle.gen_rmat(10, 20_000, 0x5EED32)
    s, d = np.asarray(s, np.int64), np.asarray(d, np.int64)
    d[::7] = s[::7]                   # self-loops
    s, d = (s + 1) << 20, (d + 1) << 20
    w, ex, has = oracle.window_triangles_fwd(s, d)
    assert engine.triangles(*(torch.from_numpy(x).cuda() for x in (s, d))) == (ex, w, has)
    w2, ex2, has2, flags = oracle.window_triangles_ref(s[:4000], d[:4000])
    assert flags and engine.triangles(s[:4000], d[:4000]) == (ex2, w2, has2)
