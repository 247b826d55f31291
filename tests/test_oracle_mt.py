"""CPU: the multi-threaded oracle variants that carry the config-size GPU tests (test_gpu_config_size.py)
are tied here to their sequential twins, which the reference's own fixtures pin
(tests/test_oracle_golden.py: TestSlice x9, WindowTrianglesITCase):

  window_reduce_mt / window_reduce_mt(init)  ==  window_reduce / window_fold
  window_fold_degree_max_mt                  ==  window_fold_degree_max
  triangles_fwd_mt                           ==  window_triangles_fwd  ==  window_triangles_ref (reference rule)

on skewed R-MAT windows of 2^21-2^22 edges (hubs spread over many threads' key ranges).  Every
comparison is bit-exact, Double sums included: the multi-threaded fold routes each key to one thread
(keyBy), so every vertex's values are still added in arrival order (GraphWindowStream.java:107-121)."""
import numpy as np
import pytest

N = 1 << 21


@pytest.fixture(scope="module")
def window(oracle):
    s, d = oracle.gen_rmat(18, N, 0x5EED31, a=0.65, b=0.15, c=0.15, permute=False)
    return s, d


@pytest.mark.parametrize("direction", [0, 1, 2])
@pytest.mark.parametrize("dtype,op", [(np.int64, 0), (np.int64, 1), (np.int64, 2), (np.int64, 3), (np.float64, 0),
                                      (np.int32, 0), (np.float32, 0)])
def test_reduce_mt_matches_sequential(oracle, window, direction, dtype, op):
    s, d = window
    v = oracle.gen_values(N, 40 + op, oracle.DT_OF_NP[np.dtype(dtype)])
    wk, wv = oracle.window_reduce(s, d, v, direction, op)
    for threads in (3, 16):
        gk, gv = oracle.window_reduce_mt(s, d, v, direction, op, threads=threads)
        assert np.array_equal(gk, wk)
        assert np.array_equal(gv.view(np.uint8), wv.view(np.uint8)), threads


@pytest.mark.parametrize("dtype,op,init", [(np.int64, 0, -77), (np.int64, 2, 1 << 20), (np.float64, 0, 0.25),
                                           (np.int64, 3, 1000)])
def test_fold_mt_matches_sequential(oracle, window, dtype, op, init):
    s, d = window
    v = oracle.gen_values(N, 50 + op, oracle.DT_OF_NP[np.dtype(dtype)])
    for direction in (0, 2):
        wk, wv = oracle.window_fold(s, d, v, direction, op, init)
        gk, gv = oracle.window_reduce_mt(s, d, v, direction, op, threads=7, init=init)
        assert np.array_equal(gk, wk) and np.array_equal(gv.view(np.uint8), wv.view(np.uint8))


def test_reduce_mt_large_window(oracle):
    """2^22 edges, 2^22-vertex range, Long and Double sums (C2's value shape)."""
    n = 1 << 22
    s, d = oracle.gen_rmat(22, n, 0x5EED02)
    for dt in (oracle.DT_I64, oracle.DT_F64):
        v = oracle.gen_values(n, 0x5EED02, dt)
        wk, wv = oracle.window_reduce(s, d, v, 0, 0)
        gk, gv = oracle.window_reduce_mt(s, d, v, 0, 0)
        assert np.array_equal(gk, wk) and np.array_equal(gv.view(np.uint8), wv.view(np.uint8))


@pytest.mark.parametrize("direction", [0, 1, 2])
def test_degree_max_mt_matches_sequential(oracle, window, direction):
    s, d = window
    for init_max in (np.iinfo(np.int64).min, 1 << 17):
        want = oracle.window_fold_degree_max(s, d, direction, init_max)
        for threads in (2, 16):
            got = oracle.window_fold_degree_max_mt(s, d, direction, init_max, threads=threads)
            for g, w in zip(got, want):
                assert np.array_equal(g, w)


def test_triangles_mt_matches_sequential(oracle):
    """Forward algorithm, threaded vs sequential, on a 2^21-edge window; and the sequential forward count
    vs the reference's candidate rule (GenerateCandidateEdges + CountTriangles, WindowTriangles.java
    :83-140) on a 2^16-edge window, both self-loop-free."""
    s, d = oracle.gen_rmat(17, N, 0x5EED32, no_self_loops=True)
    w, ex, has = oracle.window_triangles_fwd(s, d)
    assert has and ex > 0
    for threads in (5, 16):
        assert oracle.triangles_fwd_mt(s, d, threads=threads) == ex
    s2, d2 = oracle.gen_rmat(12, 1 << 16, 0x5EED33, no_self_loops=True)
    rw, rex, rhas, tree = oracle.window_triangles_ref(s2, d2)
    fw, fex, fhas = oracle.window_triangles_fwd(s2, d2)
    assert (rw, rex, rhas) == (fw, fex, fhas) and rex > 0
    assert oracle.triangles_fwd_mt(s2, d2) == rex
