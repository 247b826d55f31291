"""GPU: the ABI's own multi-rank orchestration at P = 2, 3, 4 and 8 ranks on ONE GPU.

gs_window_reduce_dist / gs_window_fold_degree_max_dist (gs_dist.hip: local partials -> owner partition
-> all-to-all of counts and flags -> packed row exchange -> merge) and gs_window_triangles_dist
(gs_triangles.hip: range, degrees, orientation, route, out-lists, boundary adjacency plan / need /
serve / assemble, count, self-pair gather) are the code the driver's multi-GPU run takes over RCCL.  RCCL
refuses two ranks on one device, so here the same C++ orchestration runs over the in-process comm group
(gs_comm_group_create / gs_comm_init_group, gs_comm.hip): P ctxs on device 0, one host thread per rank,
the collectives done by device copies between the ranks' buffers.  The group also checks that every rank
enters the same collective with matching sizes, which RCCL cannot.

Every rank holds a ragged slice of an R-MAT s16 window (2^20 edges; one rank's slice empty in one case);
the union of the ranks' outputs must equal the whole-window oracle (reference keyBy semantics,
SimpleEdgeStream.java:159-167), each rank holding exactly the vertices gs_owner_of gives it; the
triangle count equals the oracle's count of the whole window on every rank (WindowTriangles.java:64-66),
with self-loops (the reference's self-pair rule), with ids far from 0, and with sparse Long ids spanning
more than 2^56 values (the split window relabels to the whole window's compact ids: tri_dist_relabel;
so does a window whose id space is far sparser than its records, whose per-id tables would be
all-reduced)."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RANKS = (2, 3, 4, 8)
SCALE, N = 16, 1 << 20


def run_group(pkg, P, fn, timeout=240):
    """fn(rank, engine) on P threads, each rank an Engine on device 0 joined to one CommGroup."""
    grp = pkg.CommGroup(P)
    engines = [pkg.Engine(0, torch_stream=False) for _ in range(P)]
    for r, e in enumerate(engines):
        e.comm_init_group(grp, r)
    grp.close()   # the ctxs keep the group alive
    res, errs = [None] * P, []

    def run(r):
        try:
            res[r] = fn(r, engines[r])
        except BaseException as ex:   # reported by the main thread
            errs.append((r, ex))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=timeout)
    assert not any(th.is_alive() for th in ths), "a rank hung"
    for e in engines:
        e.close()
    return res, errs


def slices(n, P, empty_rank=None):
    """ragged contiguous slices of the window, rank r's share ~ (r + 1); empty_rank gets none"""
    w = np.arange(1, P + 1, dtype=np.float64)
    if empty_rank is not None:
        w[empty_rank] = 0
    b = np.concatenate([[0], np.round(np.cumsum(w) / w.sum() * n)]).astype(np.int64)
    b[-1] = n
    return [(int(b[r]), int(b[r + 1])) for r in range(P)]


def owner_np(keys, nparts):
    x = keys.astype(np.uint64)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xFF51AFD7ED558CCD)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xC4CEB9FE1A85EC53)
        x ^= x >> np.uint64(33)
    return (((x >> np.uint64(32)) * np.uint64(nparts)) >> np.uint64(32)).astype(np.int64)


def check_union(parts, want, P, rtol=None):
    """rank outputs -> the whole window: disjoint, each rank's keys ascending and owned by it"""
    keys = []
    for r, (k, *vals) in enumerate(parts):
        k = np.asarray(k)
        assert (np.diff(k) > 0).all(), r
        assert (owner_np(k, P) == r).all(), r
        keys.append(k)
    k = np.concatenate(keys)
    o = np.argsort(k, kind="stable")
    assert np.array_equal(k[o], want[0])
    for j in range(1, len(want)):
        got = np.concatenate([np.asarray(p[j]) for p in parts])[o]
        if rtol is not None and got.dtype.kind == "f":
            assert np.allclose(got, want[j], rtol=rtol, atol=0)
        else:
            assert np.array_equal(got, want[j])


@pytest.fixture(scope="module")
def window(oracle):
    s, d = oracle.gen_rmat(SCALE, N, 0x5EED0A)   # R-MAT keeps its self-loops
    return s, d


@pytest.mark.parametrize("P", RANKS)
def test_reduce_and_fold_dist(pkg, oracle, window, P):
    s, d = window
    empty = 1 if P == 3 else None
    sl = slices(N, P, empty)
    cases = []
    for dt in (oracle.DT_I64, oracle.DT_I32, oracle.DT_F64):
        v = oracle.gen_values(N, 0x5EED0A + dt, dt)
        for direction, op in ((1, 0), (0, 1), (2, 2), (2, 3), (2, 0)):
            if dt == oracle.DT_F64 and op in (1, 2):
                continue
            cases.append((v, direction, op, None))
    v64 = oracle.gen_values(N, 77, oracle.DT_I64)
    cases.append((v64, 1, 0, -7))   # foldNeighbors SUM with an init, applied once per vertex

    def fn(r, e):
        a, b = sl[r]
        out = []
        for v, direction, op, init in cases:
            out.append(e.reduce_dist(s[a:b], d[a:b], v[a:b], direction, op, init=init))
        for direction in (1, 2):
            out.append(e.fold_degree_max_dist(s[a:b], d[a:b], direction, -5))
        return out

    res, errs = run_group(pkg, P, fn)
    assert not errs, errs
    for i, (v, direction, op, init) in enumerate(cases):
        want = oracle.window_reduce(s, d, v, direction, op) if init is None else \
            oracle.window_fold(s, d, v, direction, op, init)
        check_union([res[r][i] for r in range(P)], want, P, rtol=1e-5 if v.dtype == np.float64 else None)
    for j, direction in enumerate((1, 2)):
        want = oracle.window_fold_degree_max(s, d, direction, -5)
        check_union([res[r][len(cases) + j] for r in range(P)], want, P)


@pytest.mark.parametrize("P", (2, 3))
def test_reduce_dist_mixed_key_widths(pkg, oracle, window, P):
    """Each sender picks its own key width for the packed rows (1 word when its partials' keys lie in
    [0, 2^32), else 2): here the last rank's slice holds ids past 2^32, the others' do not, so every
    owner unpacks segments of both widths (its own segment straight from its send buffer)."""
    s, d = window
    s, d = s.copy(), d.copy()
    sl = slices(N, P)
    a, b = sl[-1]
    s[a:b] += 3 << 33
    d[a:b] += 3 << 33
    v = oracle.gen_values(N, 0x5EED0C, oracle.DT_I64)

    def fn(r, e):
        a, b = sl[r]
        return [e.reduce_dist(s[a:b], d[a:b], v[a:b], 2, 0), e.fold_degree_max_dist(s[a:b], d[a:b], 1, -5)]

    res, errs = run_group(pkg, P, fn)
    assert not errs, errs
    check_union([res[r][0] for r in range(P)], oracle.window_reduce(s, d, v, 2, 0), P)
    check_union([res[r][1] for r in range(P)], oracle.window_fold_degree_max(s, d, 1, -5), P)


@pytest.mark.parametrize("P", (2, 3))
def test_reduce_dist_speculation_miss_on_one_rank(pkg, oracle, window, P):
    """A rank's speculative window is not waited for before the counts exchange: its miss word rides in
    the flags, and when one rank missed (its window's records fell into other buckets than its previous
    window's), every rank sends its counts again after that rank reran.  Three windows per rank: two of the
    same shape (the second speculates and hits), then the last rank alone gets a window whose records all
    land in one bucket (its speculation misses, the others' hits)."""
    s, d = window
    sl = slices(N, P)
    v = oracle.gen_values(N, 0x5EED0D, oracle.DT_I64)
    skew = (s % 97).astype(np.int64)   # every source in the first bucket

    def src_of(r, w):
        a, b = sl[r]
        return (skew if (w == 2 and r == P - 1) else s)[a:b]

    def fn(r, e):
        a, b = sl[r]
        out, spec = [], []
        for w in range(3):
            out.append(e.reduce_dist(src_of(r, w), d[a:b], v[a:b], 1, 0))
            spec.append(e.stage_times().speculative)
        return out, spec

    res, errs = run_group(pkg, P, fn)
    assert not errs, errs
    for w in range(3):
        ss = np.concatenate([src_of(r, w) for r in range(P)])
        check_union([res[r][0][w] for r in range(P)], oracle.window_reduce(ss, d, v, 1, 0), P)
    for r in range(P):   # window 1 speculates everywhere; window 2 misses (2) on the last rank only
        assert res[r][1][1] == 1, (r, res[r][1])
        assert res[r][1][2] == (2 if r == P - 1 else 1), (r, res[r][1])


def _tri_windows(oracle):
    s, d = oracle.gen_rmat(SCALE, N, 0x5EED0B, no_self_loops=True)
    ls, ld = oracle.gen_rmat(11, 30_000, 0x5EED0C)           # self-loops kept: the reference's rule
    assert (ls == ld).any()
    ws, wd = s * 3 + (5 << 40), d * 3 + (5 << 40)            # ids far from 0, a dense 18-bit span (no relabel)
    sparse = lambda x: x * ((1 << 40) + 12345) - (1 << 60)   # Long ids spanning > 2^56: relabeled
    return {"rmat": (s, d), "loops": (ls, ld), "far": (ws, wd), "sparse": (sparse(s), sparse(d)),
            "sparse_loops": (sparse(ls), sparse(ld))}


@pytest.fixture(scope="module")
def tri_windows(oracle):
    wins = _tri_windows(oracle)
    want = {}
    for k, (s, d) in wins.items():
        if k.endswith("loops"):
            w, ex, has, tree = oracle.window_triangles_ref(s, d)
            assert not tree
        else:
            w, ex, has = oracle.window_triangles_fwd(s, d)
        want[k] = (ex, w, has)
    return wins, want


@pytest.mark.parametrize("P", RANKS)
def test_triangles_dist(pkg, tri_windows, P):
    wins, want = tri_windows
    empty = P - 1 if P == 4 else None

    def fn(r, e):
        out = {}
        for k, (s, d) in wins.items():
            a, b = slices(len(s), P, empty)[r]
            out[k] = e.triangles_dist(s[a:b], d[a:b])
        return out

    res, errs = run_group(pkg, P, fn)
    assert not errs, errs
    for k in wins:
        for r in range(P):
            assert res[r][k] == want[k], (k, r, res[r][k], want[k])


def test_single_gpu_and_group_of_one_agree(pkg, tri_windows):
    """P = 1 over the group: the dist entry points are the single-GPU window (no exchange)."""
    wins, want = tri_windows
    res, errs = run_group(pkg, 1, lambda r, e: {k: e.triangles_dist(*w) for k, w in wins.items()})
    assert not errs, errs
    assert res[0] == want


def test_group_detects_mismatched_collectives(pkg, oracle):
    """Rank 0 runs reduceOnEdges while rank 1 runs WindowTriangles: the ranks enter different
    collectives, and both calls fail with GS_ECOMM instead of hanging (RCCL would deadlock here)."""
    s, d = oracle.gen_rmat(10, 20_000, 0x5EED0D, no_self_loops=True)
    v = oracle.gen_values(len(s), 1, oracle.DT_I64)

    def fn(r, e):
        return e.reduce_dist(s, d, v, 1, 0) if r == 0 else e.triangles_dist(s, d)

    res, errs = run_group(pkg, 2, fn, timeout=60)
    assert len(errs) == 2, (res, errs)
    for r, ex in errs:
        assert isinstance(ex, pkg.GsError) and ex.status == -4, (r, ex)


def test_group_rejects_a_rank_twice(pkg):
    grp = pkg.CommGroup(2)
    with pkg.Engine(0, torch_stream=False) as a, pkg.Engine(0, torch_stream=False) as b:
        a.comm_init_group(grp, 0)
        with pytest.raises(pkg.GsError):
            b.comm_init_group(grp, 0)
        with pytest.raises(pkg.GsError):
            b.comm_init_group(grp, 2)
        b.comm_init_group(grp, 1)
    grp.close()


def test_split_window_s20_four_ranks(pkg, oracle):
    """A larger split window (R-MAT s20, 2^24 edges, Graph500 skew) over 4 ranks: reduceOnEdges Long SUM
    (ALL) and the degree / max-neighbour fold against the whole-window oracle, WindowTriangles against the
    oracle's forward count."""
    P, n = 4, 1 << 24
    s, d = oracle.gen_rmat(20, n, 0x5EED10, no_self_loops=True)
    v = oracle.gen_values(n, 0x5EED10, oracle.DT_I64)
    sl = slices(n, P)

    def fn(r, e):
        a, b = sl[r]
        return (e.reduce_dist(s[a:b], d[a:b], v[a:b], 2, 0), e.fold_degree_max_dist(s[a:b], d[a:b], 1),
                e.triangles_dist(s[a:b], d[a:b]))

    res, errs = run_group(pkg, P, fn)
    assert not errs, errs
    check_union([res[r][0] for r in range(P)], oracle.window_reduce_mt(s, d, v, 2, 0), P)
    check_union([res[r][1] for r in range(P)], oracle.window_fold_degree_max(s, d, 1), P)
    w, ex, has = oracle.window_triangles_fwd(s, d)
    for r in range(P):
        assert res[r][2] == (ex, w, has), (r, res[r][2], ex)


@pytest.mark.parametrize("P", (2,))
def test_reduce_dist_reused_outputs(pkg, oracle, window, P):
    """reduce_dist with out=: each rank keeps one (keys, values) pair over three windows (the second
    speculates); the owned rows land in the same tensors and match the oracle's union every window."""
    s, d = window
    sl = slices(N, P)
    v = oracle.gen_values(N, 0x5EED0E, oracle.DT_I64)

    def fn(r, e):
        a, b = sl[r]
        cap = 2 * (b - a) + 1024
        buf = (torch.empty(cap, dtype=torch.int64, device="cuda"), torch.empty(cap, dtype=torch.int64, device="cuda"))
        ds, dd, dv = (torch.from_numpy(np.ascontiguousarray(x[a:b])).cuda() for x in (s, d, v))
        out = []
        for w in range(3):
            k, val = e.reduce_dist(ds, dd, dv, 2, 0, out=buf)
            assert k.data_ptr() == buf[0].data_ptr()
            out.append((k.cpu().numpy(), val.cpu().numpy()))
        with pytest.raises(ValueError):   # device outputs for host inputs: refused
            e.reduce_dist(s[a:b], d[a:b], v[a:b], 2, 0, out=buf)
        return out

    res, errs = run_group(pkg, P, fn)
    assert not errs, errs
    want = oracle.window_reduce(s, d, v, 2, 0)
    for w in range(3):
        check_union([res[r][w] for r in range(P)], want, P)


def test_failed_reduce_dist_leaves_plain_reduce_intact(pkg, oracle, window):
    """A reduce_dist whose counts exchange fails while its local window is deferred (device columns, a
    speculative second window) must not leave the owner-grouped emit set on the ctx: the next plain
    reduceOnEdges of that ctx returns its own output (gs_dist.hip dist_impl's reset on every exit).  Rank 1
    enters WindowTriangles in the second window, so the comm group sees a collective mismatch and both
    ranks' calls fail with GS_ECOMM; rank 0 then runs a plain window on the same ctx."""
    s, d = window
    v = oracle.gen_values(N, 0x5EED0F, oracle.DT_I64)
    sl = slices(N, 2)

    def fn(r, e):
        a, b = sl[r]
        ds, dd, dv = (torch.from_numpy(np.ascontiguousarray(x[a:b])).cuda() for x in (s, d, v))
        e.reduce_dist(ds, dd, dv, 1, 0)   # window 0: histogram path, measures the buckets
        with pytest.raises(pkg.GsError) as ei:
            if r == 0:
                e.reduce_dist(ds, dd, dv, 1, 0)   # window 1: speculative, deferred read-back
            else:
                e.triangles_dist(ds.cpu().numpy(), dd.cpu().numpy())
        assert ei.value.status == -4
        if r == 0:
            k, val = e.reduce(ds, dd, dv, 1, 0)
            return k.cpu().numpy(), val.cpu().numpy()
        return None

    res, errs = run_group(pkg, 2, fn, timeout=120)
    assert not errs, errs
    a, b = sl[0]
    want = oracle.window_reduce(s[a:b], d[a:b], v[a:b], 1, 0)
    assert np.array_equal(res[0][0], want[0])
    assert np.array_equal(res[0][1], want[1])


def test_split_window_s22_eight_ranks(pkg, oracle):
    """The memory-scaling case: eight ranks on one GPU, each with 1/8 of an R-MAT s22 window (2^26 edges).
    WindowTriangles over the split window against the oracle's forward count of the whole window, and the
    C3-shaped degree / max-neighbour fold (skewed R-MAT, hubs at low ids, no permutation) against the
    whole-window fold (WindowTriangles.java:64-66; GraphWindowStream.java:62-87)."""
    P, n = 8, 1 << 26
    s, d = oracle.gen_rmat(22, n, 0x5EED11, no_self_loops=True)
    sl = slices(n, P)

    def fn_tri(r, e):
        a, b = sl[r]
        return e.triangles_dist(s[a:b], d[a:b])

    res, errs = run_group(pkg, P, fn_tri, timeout=600)
    assert not errs, errs
    T = oracle.triangles_fwd_mt(s, d)
    want = (T, ((T + (1 << 31)) % (1 << 32)) - (1 << 31), True)   # Integer sum(0) wraps (WindowTriangles.java:66)
    for r in range(P):
        assert res[r] == want, (r, res[r], want)
    del s, d
    fs, fd = oracle.gen_rmat(22, n, 0x5EED12, a=0.65, b=0.15, c=0.15, permute=False)

    def fn_fold(r, e):
        a, b = sl[r]
        return e.fold_degree_max_dist(fs[a:b], fd[a:b], 1, -5)

    res, errs = run_group(pkg, P, fn_fold, timeout=600)
    assert not errs, errs
    check_union(res, oracle.window_fold_degree_max_mt(fs, fd, 1, -5), P)
