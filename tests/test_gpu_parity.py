"""GPU parity: libgellyhip.so (through the C ABI) vs the CPU oracle on identical seeded windows.

Bar: bit-exact for integer sums/min/max/count, degree/max-neighbour and the CSR; float sums within
1e-5 relative of the arrival-order fold (north star), float min/max bit-exact.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DIRS = {"IN": 0, "OUT": 1, "ALL": 2}
FLOAT_RTOL = 1e-5  # north_star: float weight sums within 1e-5 relative


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _np(t):
    return t.cpu().numpy()


def _check_values(got, want, dtype, op):
    if np.issubdtype(dtype, np.floating) and op == 0:
        tol = FLOAT_RTOL * np.maximum(np.abs(want), 1e-30)
        bad = np.abs(got.astype(np.float64) - want.astype(np.float64)) > tol
        assert not bad.any(), f"{bad.sum()} float sums outside 1e-5 rel"
    else:
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), "values differ (bit-exact required)"


@pytest.mark.parametrize("direction", ["OUT", "IN", "ALL"])
@pytest.mark.parametrize("dtype", [np.int64, np.int32, np.float64, np.float32])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_reduce_rmat_small(engine, oracle, direction, dtype, op):
    n = 30000
    s, d = oracle.gen_rmat(14, n, 0x5EED02 + op)
    v = oracle.gen_values(n, 7 + op, oracle.DT_OF_NP[np.dtype(dtype)])
    rk, rv = oracle.window_reduce(s, d, v, DIRS[direction], op)
    gk, gv = engine.reduce(*_dev(s, d, v), DIRS[direction], op)
    assert np.array_equal(_np(gk), rk)
    _check_values(_np(gv), rv, dtype, op)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 4095, 4096, 4097, 5120, 10239, 10240, 10241, 12345, 20481, 200003])
def test_reduce_sizes_ragged(engine, oracle, n):
    s, d = oracle.gen_uniform(1 << 12, n, 99 + n)
    v = oracle.gen_values(n, 5, oracle.DT_I64)
    for direction in (0, 1, 2):
        rk, rv = oracle.window_reduce(s, d, v, direction, 0)
        gk, gv = engine.reduce(*_dev(s, d, v), direction, 0)
        assert np.array_equal(_np(gk), rk) and np.array_equal(_np(gv), rv)


def test_reduce_host_buffers(engine, oracle):
    n = 50000
    s, d = oracle.gen_rmat(16, n, 3)
    v = oracle.gen_values(n, 4, oracle.DT_I64)
    rk, rv = oracle.window_reduce(s, d, v, 1, 0)
    gk, gv = engine.reduce(s, d, v, 1, 0)   # numpy -> GS_MEM_HOST
    assert np.array_equal(gk, rk) and np.array_equal(gv, rv)


@pytest.mark.parametrize("keys", ["hub", "wide", "negative", "huge_ids", "all_equal"])
def test_reduce_key_shapes(engine, oracle, keys):
    rng = np.random.default_rng(11)
    n = 100000
    if keys == "hub":        # one vertex with most records: spans many tiles (look-back carry)
        s = np.where(rng.random(n) < 0.9, 7, rng.integers(0, 1000, n)).astype(np.int64)
    elif keys == "wide":     # > 32 varying bits -> 64-bit key path
        s = rng.integers(0, 1 << 40, n, dtype=np.int64)
    elif keys == "negative":  # sign bit varies
        s = rng.integers(-(1 << 20), 1 << 20, n, dtype=np.int64)
    elif keys == "huge_ids":  # shared high half, varying low bits
        s = (np.int64(0x7ABC) << 32) + rng.integers(0, 1 << 20, n, dtype=np.int64)
    else:
        s = np.full(n, 42, np.int64)
    d = rng.integers(0, 1 << 30, n, dtype=np.int64)
    v = rng.integers(-(1 << 62), 1 << 62, n, dtype=np.int64)   # wraps
    for op in (0, 1, 2, 3):
        rk, rv = oracle.window_reduce(s, d, v, 1, op)
        gk, gv = engine.reduce(*_dev(s, d, v), 1, op)
        assert np.array_equal(_np(gk), rk), (keys, op)
        assert np.array_equal(_np(gv), rv), (keys, op)


@pytest.mark.parametrize("direction", ["OUT", "IN", "ALL"])
def test_fold_with_init(engine, oracle, direction):
    n = 40000
    s, d = oracle.gen_rmat(13, n, 21)
    for dtype, init in ((np.int64, 1000), (np.float64, 0.5), (np.int32, -3)):
        v = oracle.gen_values(n, 22, oracle.DT_OF_NP[np.dtype(dtype)])
        for op in (0, 1, 2):
            rk, rv = oracle.window_fold(s, d, v, DIRS[direction], op, init)
            gk, gv = engine.fold(*_dev(s, d, v), DIRS[direction], op, init)
            assert np.array_equal(_np(gk), rk)
            _check_values(_np(gv), rv, dtype, op)
    rk, rv = oracle.window_fold(s, d, v, DIRS[direction], 3, 10)
    gk, gv = engine.fold(*_dev(s, d, v), DIRS[direction], 3, 10)
    assert np.array_equal(_np(gk), rk) and np.array_equal(_np(gv), rv)


@pytest.mark.parametrize("direction", ["OUT", "IN", "ALL"])
def test_fold_degree_max_skewed(engine, oracle, direction):
    # BASELINE C3 shape: skewed R-MAT (.65/.15/.15/.05), no permutation -> hubs at low IDs
    n = 300000
    s, d = oracle.gen_rmat(16, n, 0x5EED03, a=0.65, b=0.15, c=0.15, permute=False)
    rk, rd, rm = oracle.window_fold_degree_max(s, d, DIRS[direction])
    gk, gd, gm = engine.fold_degree_max(*_dev(s, d), DIRS[direction])
    assert np.array_equal(_np(gk), rk) and np.array_equal(_np(gd), rd) and np.array_equal(_np(gm), rm)


@pytest.mark.parametrize("direction", ["OUT", "IN", "ALL"])
def test_csr_arrival_order(engine, oracle, direction):
    n = 60000
    s, d = oracle.gen_rmat(12, n, 31)
    v = oracle.gen_values(n, 32, oracle.DT_F64)
    rk, ro, rn, rv = oracle.window_csr(s, d, v, DIRS[direction])
    gk, go, gn, gv = engine.csr(*_dev(s, d, v), DIRS[direction])
    assert np.array_equal(_np(gk), rk) and np.array_equal(_np(go), ro)
    assert np.array_equal(_np(gn), rn) and np.array_equal(_np(gv), rv)


def test_generators_match_oracle(engine, oracle):
    n = 1 << 18
    for kw in ({}, {"permute": False}, {"no_self_loops": True}, {"a": 0.65, "b": 0.15, "c": 0.15}):
        gs_, gd_ = engine.generate_rmat(18, n, 0x5EED04, first_edge=12345, **kw)
        os_, od_ = oracle.gen_rmat(18, n, 0x5EED04, first_edge=12345, **kw)
        assert np.array_equal(_np(gs_), os_) and np.array_equal(_np(gd_), od_)
    gs_, gd_ = engine.generate_uniform(1 << 16, n, 0x5EED01)
    os_, od_ = oracle.gen_uniform(1 << 16, n, 0x5EED01)
    assert np.array_equal(_np(gs_), os_) and np.array_equal(_np(gd_), od_)
    for dt in (0, 1, 2, 3):
        assert np.array_equal(_np(engine.generate_values(n, 9, dt)), oracle.gen_values(n, 9, dt))


def test_reduce_large_rmat_properties(engine):
    """At 2^26 edges (no oracle): sum of per-vertex sums == sum of values, counts sum to E,
    keys strictly ascending, result reproducible run to run."""
    n = 1 << 26
    s, d = engine.generate_rmat(22, n, 0x5EED02)
    v = engine.generate_values(n, 0x5EED02)
    k1, v1 = engine.reduce(s, d, v, 1, 0)
    assert int(v1.sum()) == int(v.sum())
    assert bool((k1[1:] > k1[:-1]).all())
    kc, vc = engine.reduce(s, d, v, 1, 3)
    assert int(vc.sum()) == n and torch.equal(kc, k1)
    k2, v2 = engine.reduce(s, d, v, 1, 0)
    assert torch.equal(k1, k2) and torch.equal(v1, v2)


def test_reduce_unaligned_device_slices(engine, oracle):
    """Columns that are views at an odd offset (8-byte aligned only) take the scalar key-scan path."""
    n = 70001
    s, d = oracle.gen_rmat(15, n + 1, 77)
    v = oracle.gen_values(n + 1, 78, oracle.DT_I64)
    S, D, Vv = _dev(s, d, v)
    for direction in (0, 1, 2):
        rk, rv = oracle.window_reduce(s[1:], d[1:], v[1:], direction, 0)
        gk, gv = engine.reduce(S[1:], D[1:], Vv[1:], direction, 0)
        assert np.array_equal(_np(gk), rk) and np.array_equal(_np(gv), rv)


def test_speculative_window_unaligned_device_slices(engine, oracle):
    """The speculative scatter reads two records per lane with 16-byte loads only from 16-byte aligned
    columns (k_sp_scatter_pack, GS_SPK_VEC): a second window of the same geometry (it speculates) over views
    at an odd offset -- keys only, values only, both -- takes the 8-byte path and gives the same output."""
    n = 1 << 18
    s, d = oracle.gen_rmat(16, n + 2, 79)
    v = oracle.gen_values(n + 2, 80, oracle.DT_I64)
    S, D, Vv = _dev(s, d, v)
    for direction in (0, 1):
        for ko, vo in ((0, 0), (1, 1), (1, 0), (0, 1)):
            ks, kd, vv = S[ko:ko + n], D[ko:ko + n], Vv[vo:vo + n]
            want = oracle.window_reduce(s[ko:ko + n], d[ko:ko + n], v[vo:vo + n], direction, 0)
            for w in range(2):   # the second window speculates
                gk, gv = engine.reduce(ks, kd, vv, direction, 0)
                assert np.array_equal(_np(gk), want[0]) and np.array_equal(_np(gv), want[1]), (direction, ko, vo, w)
