"""GPU: the bucket path (gs_bucket.hpp) — reduceOnEdges / foldNeighbors built-ins through the high-bit
partition + LDS accumulation — against the CPU oracle, at every pipeline shape it takes:

  direct partition    (default, path 2): per-tile histograms -> offsets -> one scatter pass
  onesweep partition  (GS_FLAG_BK_ONESWEEP, path 1): 1 pass (<= 2^(S+8) vertices) or 2 passes
  no partition        (vertex range <= 2^S: one bucket, records read straight from the columns)
  multi-item buckets  (a bucket with more than 2^17 records: LDS slabs merged by k_bk_merge)
  mispredicted base   (IDs far from 0 / negative: the info kernel reruns with base = min)
  out of range        (vertex range > 2048 buckets: falls back to the LSD sort path, path 0)

Integer results bit-exact; float sums within 1e-5 relative (north star)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FLOAT_RTOL = 1e-5
BUCKET = (1, 2)   # stage_times().path of the bucket path (onesweep / direct partition)


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _check(got_k, got_v, want_k, want_v, dtype, op):
    assert np.array_equal(got_k.cpu().numpy(), want_k)
    g = got_v.cpu().numpy()
    if np.issubdtype(np.dtype(dtype), np.floating) and op == 0:
        tol = FLOAT_RTOL * np.maximum(np.abs(want_v.astype(np.float64)), 1e-30)
        assert not (np.abs(g.astype(np.float64) - want_v.astype(np.float64)) > tol).any()
    else:
        assert np.array_equal(g.view(np.uint8), want_v.view(np.uint8))


def _window(rng, n, span, offset=0, hub_frac=0.0):
    s = rng.integers(0, span, n).astype(np.int64) + offset
    d = rng.integers(0, span, n).astype(np.int64) + offset
    if hub_frac:
        hub = rng.random(n) < hub_frac
        s[hub] = offset + span // 3
    return s, d


# spans per accumulator width: S = 14 (8-byte), 15 (4-byte / count), 13 (degree)
SPANS = {"one_bucket": 1 << 13, "one_pass": 1 << 19, "two_passes": 1 << 24}


@pytest.mark.parametrize("shape", list(SPANS))
@pytest.mark.parametrize("direction", [0, 1, 2])
@pytest.mark.parametrize("dtype,op", [(np.int64, 0), (np.int64, 1), (np.int64, 2), (np.int32, 0), (np.int32, 1),
                                      (np.int32, 2), (np.float64, 0), (np.float32, 0), (np.int64, 3)])
def test_bucket_reduce_shapes(engine, oracle, shape, direction, dtype, op):
    rng = np.random.default_rng(hash((shape, direction, op)) & 0xFFFF)
    n = 60000
    s, d = _window(rng, n, SPANS[shape])
    v = oracle.gen_values(n, 11 + op, oracle.DT_OF_NP[np.dtype(dtype)])
    rk, rv = oracle.window_reduce(s, d, v, direction, op)
    gk, gv = engine.reduce(*_dev(s, d, v), direction, op)
    assert engine.stage_times().path in BUCKET
    _check(gk, gv, rk, rv, dtype, op)


def test_bucket_pass_counts(pkg, oracle):
    """The pipeline shape follows the vertex range (S = 14 for Long sums): the direct partition is one
    scatter pass; the onesweep partition takes 1-2 LSD passes.  A fresh engine per span, so the
    direct path's predicted bucket count starts from the default."""
    rng = np.random.default_rng(5)
    for span, passes in ((1 << 14, 0), (1 << 18, 1), (1 << 22, 1), (1 << 23, 2), (1 << 25, 2)):
        s, d = _window(rng, 20000, span)
        s[0], d[0] = 0, span - 1
        v = oracle.gen_values(20000, 1, oracle.DT_I64)
        rk, rv = oracle.window_reduce(s, d, v, 2, 0)
        with pkg.Engine(0, bk_onesweep=True) as eo:
            gk, gv = eo.reduce(*_dev(s, d, v), 2, 0)
            t = eo.stage_times()
            assert (t.path, t.sort_passes) == (1, passes), span
            _check(gk, gv, rk, rv, np.int64, 0)
        with pkg.Engine(0) as ed:
            for rep in range(2):   # the second window runs on the learned prediction (one bucket: no scatter)
                gk, gv = ed.reduce(*_dev(s, d, v), 2, 0)
                t = ed.stage_times()
                assert t.path == 2 and t.sort_passes == (0 if rep and span <= 1 << 14 else 1), span
                _check(gk, gv, rk, rv, np.int64, 0)


@pytest.mark.parametrize("direction", [0, 1, 2])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_direct_matches_onesweep(pkg, oracle, direction, op):
    """The two partition front ends feed the same accumulation: integer results are identical."""
    rng = np.random.default_rng(40 + op)
    s, d = _window(rng, 150_001, 1 << 23, hub_frac=0.05)
    v = oracle.gen_values(150_001, 8, oracle.DT_I64)
    with pkg.Engine(0) as ed, pkg.Engine(0, bk_onesweep=True) as eo:
        kd, vd = ed.reduce(*_dev(s, d, v), direction, op)
        ko, vo = eo.reduce(*_dev(s, d, v), direction, op)
        assert (ed.stage_times().path, eo.stage_times().path) == (2, 1)
        assert torch.equal(kd, ko) and torch.equal(vd, vo)
    rk, rv = oracle.window_reduce(s, d, v, direction, op)
    _check(kd, vd, rk, rv, np.int64, op)


def test_direct_prediction_shrinks_and_grows(engine, oracle):
    """The direct path predicts the next window's base and bucket count; windows that need more
    buckets (or sit elsewhere) recount, windows that need fewer run on the wider table."""
    rng = np.random.default_rng(17)
    for span, off in ((1 << 24, 0), (1 << 16, 0), (1 << 16, 0), (1 << 24, 0), (1 << 20, -(1 << 33)),
                      (1 << 24, 1 << 40), (1 << 24, 0)):
        s, d = _window(rng, 30011, span, off)
        v = oracle.gen_values(30011, 5, oracle.DT_I64)
        rk, rv = oracle.window_reduce(s, d, v, 1, 0)
        gk, gv = engine.reduce(*_dev(s, d, v), 1, 0)
        assert engine.stage_times().path in BUCKET
        _check(gk, gv, rk, rv, np.int64, 0)


@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_bucket_multi_item_hub(engine, oracle, op):
    """A hub with 400k records in one bucket: several work items, LDS slabs merged in k_bk_merge."""
    rng = np.random.default_rng(21 + op)
    n = 700_000
    s, d = _window(rng, n, 1 << 20, hub_frac=0.6)
    v = oracle.gen_values(n, 3, oracle.DT_I64)
    for direction in (1, 2):
        rk, rv = oracle.window_reduce(s, d, v, direction, op)
        gk, gv = engine.reduce(*_dev(s, d, v), direction, op)
        t = engine.stage_times()
        buckets = (1 << 20) >> (15 if op == 3 else 14)
        assert t.path in BUCKET and t.partials > buckets      # the hub's bucket took several items
        _check(gk, gv, rk, rv, np.int64, op)


@pytest.mark.parametrize("offset", [-(1 << 40), -5000, 123_456_789_012, (1 << 62)])
def test_bucket_base_prediction(engine, oracle, offset):
    """IDs away from 0 (and a window after one at another offset): the predicted base misses, the info
    kernel reruns with base = min, results stay exact; the next window at the same offset hits."""
    rng = np.random.default_rng(abs(offset) % 1000)
    for span in (1 << 12, 1 << 20, 1 << 20):
        s, d = _window(rng, 40000, span, offset)
        v = oracle.gen_values(40000, 9, oracle.DT_I64)
        rk, rv = oracle.window_reduce(s, d, v, 2, 0)
        gk, gv = engine.reduce(*_dev(s, d, v), 2, 0)
        assert engine.stage_times().path in BUCKET
        _check(gk, gv, rk, rv, np.int64, 0)


def test_bucket_out_of_range_falls_back(engine, oracle):
    rng = np.random.default_rng(3)
    s, d = _window(rng, 30000, 1 << 30)
    v = oracle.gen_values(30000, 2, oracle.DT_I64)
    rk, rv = oracle.window_reduce(s, d, v, 1, 0)
    gk, gv = engine.reduce(*_dev(s, d, v), 1, 0)
    assert engine.stage_times().path == 0
    _check(gk, gv, rk, rv, np.int64, 0)


@pytest.mark.parametrize("dtype,op,init", [(np.int64, 0, -77), (np.int64, 1, 5), (np.int64, 2, 40000),
                                           (np.int32, 0, 2**31 - 5), (np.float64, 0, 0.25), (np.int64, 3, 1000)])
def test_bucket_fold_init(engine, oracle, dtype, op, init):
    rng = np.random.default_rng(op + 100)
    n = 50000
    s, d = _window(rng, n, 1 << 21)
    v = oracle.gen_values(n, 4, oracle.DT_OF_NP[np.dtype(dtype)])
    rk, rv = oracle.window_fold(s, d, v, 0, op, init)
    gk, gv = engine.fold(*_dev(s, d, v), 0, op, init)
    assert engine.stage_times().path in BUCKET
    _check(gk, gv, rk, rv, dtype, op)


@pytest.mark.parametrize("span", [1 << 10, 1 << 17, 1 << 24])
def test_bucket_degree_max(engine, oracle, span):
    rng = np.random.default_rng(span % 97)
    s, d = _window(rng, 80000, span, hub_frac=0.3)
    for direction in (0, 1, 2):
        for init_max in (np.iinfo(np.int64).min, span // 2):
            rk, rd, rm = oracle.window_fold_degree_max(s, d, direction, init_max)
            gk, gd, gm = engine.fold_degree_max(*_dev(s, d), direction, init_max)
            assert engine.stage_times().path in BUCKET
            assert np.array_equal(gk.cpu().numpy(), rk)
            assert np.array_equal(gd.cpu().numpy(), rd) and np.array_equal(gm.cpu().numpy(), rm)


def test_sort_only_engine_matches(pkg, oracle):
    """GS_FLAG_SORT_ONLY: the same window through the LSD sort path gives the same integer results."""
    rng = np.random.default_rng(8)
    s, d = _window(rng, 100000, 1 << 22, hub_frac=0.1)
    v = oracle.gen_values(100000, 6, oracle.DT_I64)
    with pkg.Engine(0) as eb, pkg.Engine(0, sort_only=True) as es:
        kb, vb = eb.reduce(*_dev(s, d, v), 2, 0)
        assert eb.stage_times().path in BUCKET
        ks, vs = es.reduce(*_dev(s, d, v), 2, 0)
        assert es.stage_times().path == 0
        assert torch.equal(kb, ks) and torch.equal(vb, vs)


def test_bucket_large_rmat_properties(engine):
    """R-MAT scale 22 (4M vertices, 64M edges): sum of per-vertex sums == sum of values, counts sum
    to the records, keys strictly ascending — size-independent checks at a size the oracle skips."""
    n = 1 << 26
    s, d = engine.generate_rmat(22, n, 77)
    v = engine.generate_values(n, 78, 1)
    k, x = engine.reduce(s, d, v, 2, 0)
    assert engine.stage_times().path in BUCKET
    assert bool((k[1:] > k[:-1]).all())
    assert int(x.sum()) == 2 * int(v.sum())
    k2, c = engine.reduce(s, d, v, 2, 3)
    assert torch.equal(k, k2) and int(c.sum()) == 2 * n


@pytest.mark.parametrize("direction", [0, 1, 2])
def test_degree_max_far_neighbours(engine, oracle, direction):
    """Keys in a small range, neighbours 2^40 away: the 32-bit neighbour offsets of the compact
    degree/max policy do not fit, the scatter flags it and the window reruns with 64-bit maxima."""
    rng = np.random.default_rng(31 + direction)
    n = 90000
    s = rng.integers(0, 1 << 20, n).astype(np.int64)
    d = rng.integers(0, 1 << 20, n).astype(np.int64)
    d[::7] += 1 << 40
    for init_max in (np.iinfo(np.int64).min, 1 << 41):
        rk, rd, rm = oracle.window_fold_degree_max(s, d, direction, init_max)
        gk, gd, gm = engine.fold_degree_max(*_dev(s, d), direction, init_max)
        assert np.array_equal(gk.cpu().numpy(), rk)
        assert np.array_equal(gd.cpu().numpy(), rd) and np.array_equal(gm.cpu().numpy(), rm)


VALUE_MIXES = {
    "narrow": lambda rng, n: rng.integers(0, 0xFFFF, n),                       # every value packs
    "boundary": lambda rng, n: rng.choice([0, 1, 0xFFFE, 0xFFFF, 0x10000, -1], n),   # escapes at 0xFFFF and up
    "sparse_wide": lambda rng, n: np.where(rng.random(n) < 0.01, rng.integers(-(1 << 31), 1 << 31, n),
                                           rng.integers(0, 0xFFFF, n)),
    "all_wide": lambda rng, n: rng.integers(-(1 << 30), -1, n),                 # every value escapes
}


@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("op", [0, 1, 2])
def test_packed_records_escapes(pkg, oracle, dtype, op):
    """k_dp_scatter_pack: values in [0, 0xFFFF) travel in 16 bits, others escape (0xFFFF + the full value
    beside the record).  Bit-exact against the oracle and against the unpacked scatter (GS_FLAG_NO_PACK),
    for every mix of values; after a window where escapes are common the engine stores 8-byte values."""
    rng = np.random.default_rng(1000 + op)
    n = 200_003
    s, d = _window(rng, n, 1 << 22, hub_frac=0.02)
    with pkg.Engine(0) as ep, pkg.Engine(0, no_pack=True) as eu:
        for w, mix in enumerate(("narrow", "sparse_wide", "boundary", "all_wide", "narrow")):
            v = VALUE_MIXES[mix](rng, n).astype(dtype)
            rk, rv = oracle.window_reduce(s, d, v, 1, op)
            kp, vp = ep.reduce(*_dev(s, d, v), 1, op)
            tp = ep.stage_times()
            ku, vu = eu.reduce(*_dev(s, d, v), 1, op)
            assert not eu.stage_times().packed
            _check(kp, vp, rk, rv, dtype, op)
            assert torch.equal(kp, ku) and torch.equal(vp, vu), mix
            if mix == "narrow" and w == 0:
                assert tp.packed and tp.escapes == 0
            if mix == "sparse_wide":
                assert tp.packed and 0 < tp.escapes < n // 8
            if mix == "boundary":   # about half the values escape: the following windows store 8-byte values
                assert tp.packed and tp.escapes > n // 8
            if mix == "all_wide" or w == 4:
                assert not tp.packed


def test_packed_prediction_miss_reruns(pkg, oracle):
    """No host round trip inside a window: a window whose IDs leave the predicted range is detected by
    the histogram, every later launch exits, and the window reruns with the measured range."""
    rng = np.random.default_rng(77)
    with pkg.Engine(0) as e:
        for span, off in ((1 << 20, 0), (1 << 23, 0), (1 << 20, 1 << 35), (1 << 16, -(1 << 50)), (1 << 24, 0)):
            s, d = _window(rng, 123_457, span, off)
            v = rng.integers(0, 0xFFFF, 123_457).astype(np.int64)
            rk, rv = oracle.window_reduce(s, d, v, 1, 0)
            gk, gv = e.reduce(*_dev(s, d, v), 1, 0)
            assert e.stage_times().path == 2
            _check(gk, gv, rk, rv, np.int64, 0)


@pytest.mark.parametrize("direction,dtype,op", [(1, np.int64, 0), (0, np.int64, 0), (2, np.int64, 0),
                                                (1, np.int32, 1), (2, np.int64, 2), (1, np.float64, 0),
                                                (2, np.float32, 0), (0, np.int64, 3)])
def test_speculative_partition(pkg, oracle, direction, dtype, op):
    """k_sp_scatter_pack: a packed window whose bucket counts the ctx's previous packed window measured in
    the same geometry (base, S, direction) sizes one region per bucket from them and reserves each tile's
    runs with atomics on per-bucket cursors -- no histogram pass.  Hits (incl. a hub bucket of several
    work items, escaped values, a larger window), a window crowding half its records into one bucket
    (regions overflow) and a key outside the predicted range all end bit-exact against the oracle and
    the histogram path (GS_FLAG_NO_SPEC); a miss reruns the window through the histogram
    (speculative == 2) and the next 8 windows do not speculate."""
    rng = np.random.default_rng(4242 + 10 * direction + op)
    n = 300_001

    flt = np.issubdtype(np.dtype(dtype), np.floating)
    packed = not flt and op != 3   # integer SUM / MIN / MAX: k_sp_scatter_pack; others: k_sp_scatter

    def win(m, span=1 << 22):
        s, d = _window(rng, m, span, hub_frac=0.1)
        v = rng.integers(0, 0xFFFF, m)
        v[rng.random(m) < 0.001] = -(1 << 40) if dtype == np.int64 else -(1 << 30)   # escapes
        return s, d, (rng.random(m) * 100 if flt else v).astype(dtype)

    with pkg.Engine(0) as e, pkg.Engine(0, no_spec=True) as ex:
        def run(s, d, v, expect):
            rk, rv = oracle.window_reduce(s, d, v, direction, op)
            gk, gv = e.reduce(*_dev(s, d, v), direction, op)
            t = e.stage_times()
            assert t.path == 2 and t.packed == packed
            _check(gk, gv, rk, rv, dtype, op)
            xk, xv = ex.reduce(*_dev(s, d, v), direction, op)
            assert ex.stage_times().speculative == 0
            assert torch.equal(gk, xk) and (flt or torch.equal(gv, xv))   # float sums: LDS-atomic order
            assert t.speculative == expect, (t.speculative, expect)

        run(*win(n), 0)            # first window: histogram (nothing to predict from)
        for _ in range(4):
            run(*win(n), 1)
        run(*win(n * 3 // 2), 1)   # regions scale with the record count
        s, d, v = win(n)
        (s if direction != 0 else d)[: n // 2] = 12345   # half the records in bucket 0: regions overflow
        if direction == 2:
            d[: n // 2] = 12345
        run(s, d, v, 2)
        for _ in range(8):
            run(*win(n), 0)
        run(*win(n), 1)
        s, d, v = win(n)
        s[n // 3] = d[n // 3] = (1 << 23) + 5   # outside the predicted bucket count
        run(s, d, v, 2)


@pytest.mark.parametrize("direction", [0, 1, 2])
def test_speculative_degree_max(pkg, oracle, direction):
    """foldNeighbors(degree, max neighbour) on k_sp_scatter: neighbours as 32-bit offsets from the window
    base (BkDeg32); a window whose neighbours leave base + 2^32 retries wide (BkDeg) and stays exact."""
    rng = np.random.default_rng(77 + direction)
    n = 250_001
    with pkg.Engine(0) as e:
        spec = []
        for w in range(6):
            s, d = _window(rng, n, 1 << 21, hub_frac=0.05)
            if w == 4:
                d[::1000] += 1 << 40   # far neighbours (keys stay in range for OUT)
            want = oracle.window_fold_degree_max(s, d, direction)
            got = e.fold_degree_max(*_dev(s, d), direction)
            for g, x in zip(got, want):
                assert np.array_equal(g.cpu().numpy(), x), w
            spec.append(e.stage_times().speculative)
        assert spec[1] == spec[2] == spec[3] == 1, spec


@pytest.mark.parametrize("spec", [False, True])
def test_packed_integer_sum_wraps_to_zero(pkg, oracle, spec):
    """Integer SUM on packed records: a vertex whose narrow values total exactly 2^32 (2^17 records of
    32768) has a 32-bit accumulator back at its identity 0; the reference still emits it, with the
    wrapped value 0.  Presence is marked per record for 4-byte sums, so the vertex is not dropped
    (both the histogram and the speculative partition)."""
    rng = np.random.default_rng(99)
    n_hub, n_rest = 1 << 17, 70_000
    with pkg.Engine(0, no_spec=not spec) as e:
        for w in range(3):
            s = np.concatenate([np.full(n_hub, 4242, np.int64), rng.integers(5000, 1 << 20, n_rest)])
            d = rng.integers(0, 1 << 20, n_hub + n_rest).astype(np.int64)
            v = np.concatenate([np.full(n_hub, 32768), rng.integers(0, 0xFFFF, n_rest)]).astype(np.int32)
            perm = rng.permutation(len(s))
            s, d, v = s[perm], d[perm], v[perm]
            rk, rv = oracle.window_reduce(s, d, v, 1, 0)   # OUT: key = src
            assert rv[np.searchsorted(rk, 4242)] == 0
            gk, gv = e.reduce(*_dev(s, d, v), 1, 0)
            t = e.stage_times()
            assert t.path == 2 and t.packed
            _check(gk, gv, rk, rv, np.int32, 0)


@pytest.mark.parametrize("op", [0, 1, 2])
def test_packed_presence_of_zero_and_escaped_only_vertices(pkg, oracle, op):
    """k_bk_accum's packed fast path takes 4 narrow, non-zero records with LDS atomics alone; a vertex
    seen only through zero values (SUM: the accumulator stays at its identity) or only through escaped
    values must still be emitted -- isolated, and mixed into groups of 4 with common records, through the
    histogram path and the speculative partition."""
    rng = np.random.default_rng(555 + op)
    n = 200_000
    with pkg.Engine(0) as e:
        for w in range(4):
            s, d = _window(rng, n, 1 << 16)   # ~3 records per vertex
            v = rng.integers(1, 0xFFFF, n).astype(np.int64)
            zero_v = rng.choice(1 << 16, 300, replace=False)
            for j, x in enumerate(zero_v):   # vertices whose every record is 0 (first 150) or escaped
                m = s == x
                v[m] = 0 if j < 150 else -(1 << 40) - j
            v[rng.random(n) < 0.0005] = 0      # and scattered zeros / escapes among common records
            v[rng.random(n) < 0.0005] = 1 << 33
            rk, rv = oracle.window_reduce(s, d, v, 1, op)
            gk, gv = e.reduce(*_dev(s, d, v), 1, op)
            t = e.stage_times()
            assert t.path == 2 and t.packed
            assert t.speculative == (0 if w == 0 else 1)
            _check(gk, gv, rk, rv, np.int64, op)


def test_timing_levels_same_results(pkg, oracle):
    """gs_set_timing: the stage events a window records change nothing but the stage times.  STAGES times
    every stage; DOMINANT only the direct path's scatter and accumulate (pass_ms[1], [2]); OFF none.  The
    speculative partition (windows after the first) runs at every level."""
    L = pkg._lib
    rng = np.random.default_rng(77)
    n = 1 << 20
    s, d = _window(rng, n, 1 << 22)
    v = oracle.gen_values(n, 5, oracle.DT_I64)
    rk, rv = oracle.window_reduce(s, d, v, 1, 0)
    e = pkg.Engine(0)
    try:
        with pytest.raises(pkg.GsError):
            e.set_timing(7)
        cols = _dev(s, d, v)
        for level in (L.GS_TIMING_STAGES, L.GS_TIMING_DOMINANT, L.GS_TIMING_OFF, L.GS_TIMING_STAGES):
            e.set_timing(level)
            for _ in range(2):
                gk, gv = e.reduce(*cols, 1, 0)
                _check(gk, gv, rk, rv, np.int64, 0)
                t = e.stage_times()
                assert t.path == 2
            pm = list(t.pass_ms)
            if level == L.GS_TIMING_STAGES:
                assert pm[1] > 0 and pm[2] > 0 and pm[4] > 0 and t.total_ms > 0
            elif level == L.GS_TIMING_DOMINANT:
                assert pm[1] > 0 and pm[2] > 0 and pm[3] == 0 and pm[4] == 0 and t.total_ms == 0
            else:
                assert not any(pm) and t.total_ms == 0
            assert t.speculative == 1   # the second window of each level
    finally:
        e.close()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_float_sum_presence_with_signed_zeros(engine, oracle, dtype):
    """Float SUM starts its accumulators at -0.0 (gs_bucket.hpp BkVal::FLOAT_SUM): a vertex whose values
    are all -0.0 sums to -0.0 as the reference's reduce does (it starts from the first value; from a +0.0
    start the bucket path returned +0.0 -- this test found it), a sum that cancels ends at +0.0, and
    presence is inferred from the accumulator except for -0.0 values.  Vertices whose records are all +0.0,
    all -0.0, cancel exactly, or mix -0.0 with others must all be present with the reference's signed
    zeros, including across the slabs of a multi-item hub bucket."""
    rng = np.random.default_rng(2024)
    n = 1 << 20
    hub = 5000
    s = rng.integers(0, 1 << 20, n).astype(np.int64)
    s[: n // 2] = hub                                   # a hub bucket of many items (slabs)
    v = rng.standard_normal(n).astype(dtype)
    special = {hub + 1: [0.0] * 40, hub + 2: [-0.0] * 40, hub + 3: [1.5, -1.5] * 20, hub + 4: [-0.0, 2.0] * 20,
               hub + 5: [-0.0] * 3, 700001: [0.0], 700002: [-0.0]}
    pos = rng.permutation(n)[: sum(len(x) for x in special.values())]
    at = 0
    for vid, vals in special.items():
        for x in vals:
            s[pos[at]], v[pos[at]] = vid, x
            at += 1
    d = rng.integers(0, 1 << 20, n).astype(np.int64)
    rk, rv = oracle.window_reduce(s, d, v, 1, 0)
    gk, gv = engine.reduce(*_dev(s, d, v), 1, 0)
    gk, gv = gk.cpu().numpy(), gv.cpu().numpy()
    assert np.array_equal(gk, rk)
    for vid in special:
        i = int(np.searchsorted(rk, vid))
        assert rk[i] == vid
        if rv[i] == 0:   # exact zeros: the same sign as the reference's sequential sum
            assert gv[i] == 0 and np.signbit(gv[i]) == np.signbit(rv[i]), (vid, gv[i], rv[i])
    # against the exact per-vertex sums (f64 over the values; the hub's 2^19 normal values cancel, so the
    # reference's own sequential f32 fold drifts past 1e-5 of its small sum there -- the f32 config-size test
    # bounds that drift)
    idx = np.searchsorted(rk, s)
    exact = np.bincount(idx, weights=v.astype(np.float64), minlength=len(rk))
    mag = np.bincount(idx, weights=np.abs(v.astype(np.float64)), minlength=len(rk))
    assert not (np.abs(gv.astype(np.float64) - exact) > 1e-6 * mag + 1e-300).any()


def test_reused_output_buffers(engine, oracle):
    """reduce / fold_degree_max with out=: one set of output tensors reused over windows of different sizes
    and shapes (a streaming operator's buffers, as bench.py's C2 line holds them) gives the same rows as
    fresh outputs; a buffer shorter than the window's records is refused before any launch."""
    rng = np.random.default_rng(0x0B0F)
    cap = 2 * 90000
    kv = (torch.empty(cap, dtype=torch.int64, device="cuda"), torch.empty(cap, dtype=torch.int64, device="cuda"))
    kdm = tuple(torch.empty(cap, dtype=torch.int64, device="cuda") for _ in range(3))
    for n, span in ((90000, 1 << 19), (20000, 1 << 13), (60000, 1 << 24)):
        s, d = _window(rng, n, span)
        v = oracle.gen_values(n, 0x0B1, oracle.DT_I64)
        gk, gv = engine.reduce(*_dev(s, d, v), 2, 0, out=kv)
        assert gk.data_ptr() == kv[0].data_ptr()
        _check(gk, gv, *oracle.window_reduce(s, d, v, 2, 0), np.int64, 0)
        gk, gdeg, gmx = engine.fold_degree_max(*_dev(s, d), 1, -5, out=kdm)
        wk, wdeg, wmx = oracle.window_fold_degree_max(s, d, 1, -5)
        assert np.array_equal(gk.cpu().numpy(), wk)
        assert np.array_equal(gdeg.cpu().numpy(), wdeg) and np.array_equal(gmx.cpu().numpy(), wmx)
    s, d = _window(rng, 1000, 1 << 13)
    short = (kv[0][:1999], kv[1][:1999])
    with pytest.raises(ValueError):
        engine.reduce(*_dev(s, d, s), 2, 0, out=short)
