"""GPU: windows above one engine pass's record cap (gs_set_max_window_records; SimpleEdgeStream.java
:159-167 puts no cap on a window).  With a small cap the window runs in chunks of whole edges: each
chunk's per-vertex partials are merged into the running partials (gs_merge_partials /
gs_merge_degree_max_partials), foldNeighbors' init applied once at the end.  Integer results must equal
the one-pass window's and the oracle's bit for bit; float sums within 1e-5 relative.  Host and device
batches, every direction; COUNT, folds with init, the degree / max-neighbour fold."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FLOAT_RTOL = 1e-5


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def _np(x):
    return x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


def _check(got_k, got_v, want_k, want_v, dtype, op):
    assert np.array_equal(_np(got_k), want_k)
    g = _np(got_v)
    if np.issubdtype(np.dtype(dtype), np.floating) and op == 0:
        tol = FLOAT_RTOL * np.maximum(np.abs(want_v.astype(np.float64)), 1e-30)
        assert not (np.abs(g.astype(np.float64) - want_v.astype(np.float64)) > tol).any()
    else:
        assert np.array_equal(g.view(np.uint8), want_v.view(np.uint8))


@pytest.fixture()
def chunked(pkg):
    with pkg.Engine(0) as e:
        e.set_max_window_records(40_000)
        yield e


def _window(oracle, n, seed, span_scale=16):
    return oracle.gen_rmat(span_scale, n, seed, a=0.6, b=0.15, c=0.15, permute=False)


@pytest.mark.parametrize("direction", [0, 1, 2])
@pytest.mark.parametrize("dtype,op", [(np.int64, 0), (np.int64, 1), (np.int64, 2), (np.int64, 3), (np.int32, 0),
                                      (np.float64, 0), (np.float32, 0)])
@pytest.mark.parametrize("host", [False, True])
def test_chunked_reduce(chunked, oracle, direction, dtype, op, host):
    n = 230_003   # 6-12 chunks of 40k records, the last one ragged
    s, d = _window(oracle, n, 700 + op)
    v = oracle.gen_values(n, 9 + op, oracle.DT_OF_NP[np.dtype(dtype)])
    rk, rv = oracle.window_reduce(s, d, v, direction, op)
    args = (s, d, v) if host else _dev(s, d, v)
    gk, gv = chunked.reduce(*args, direction, op)
    _check(gk, gv, rk, rv, dtype, op)


@pytest.mark.parametrize("dtype,op,init", [(np.int64, 0, -77), (np.int64, 2, 1 << 40), (np.int64, 3, 1000),
                                           (np.float64, 0, 0.5)])
def test_chunked_fold_init_applied_once(chunked, oracle, dtype, op, init):
    n = 180_001
    s, d = _window(oracle, n, 800 + op)
    v = oracle.gen_values(n, 19 + op, oracle.DT_OF_NP[np.dtype(dtype)])
    for direction in (1, 2):
        rk, rv = oracle.window_fold(s, d, v, direction, op, init)
        gk, gv = chunked.fold(*_dev(s, d, v), direction, op, init)
        _check(gk, gv, rk, rv, dtype, op)


@pytest.mark.parametrize("direction", [0, 1, 2])
def test_chunked_degree_max(chunked, oracle, direction):
    n = 200_000
    s, d = _window(oracle, n, 900 + direction)
    for init_max in (np.iinfo(np.int64).min, 1 << 15):
        want = oracle.window_fold_degree_max(s, d, direction, init_max)
        for args in ((s, d), _dev(s, d)):
            got = chunked.fold_degree_max(*args, direction, init_max)
            for g, w in zip(got, want):
                assert np.array_equal(_np(g), w)


def test_chunked_equals_one_pass_and_cap_resets(pkg, oracle):
    """The same windows chunked and in one pass give identical integer results; cap 0 restores one pass;
    a window just under the cap is not chunked."""
    n = 300_000
    s, d = _window(oracle, n, 1234, span_scale=20)
    v = oracle.gen_values(n, 5, oracle.DT_I64)
    S, D, V = _dev(s, d, v)
    with pkg.Engine(0) as e:
        k1, v1 = e.reduce(S, D, V, 2, 0)
        e.set_max_window_records(2 * n - 1)   # ALL: 2n records, two chunks
        k2, v2 = e.reduce(S, D, V, 2, 0)
        assert torch.equal(k1, k2) and torch.equal(v1, v2)
        e.set_max_window_records(2 * n)        # fits: one pass
        k3, v3 = e.reduce(S, D, V, 2, 0)
        assert torch.equal(k1, k3) and torch.equal(v1, v3)
        e.set_max_window_records(0)
        k4, v4 = e.reduce(S, D, V, 2, 3)
        wk, wv = oracle.window_reduce(s, d, v, 2, 3)
        assert np.array_equal(_np(k4), wk) and np.array_equal(_np(v4), wv)
