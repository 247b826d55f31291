"""CPU, world_size 2 (gloo): the keyBy exchange of distributed.py — per-rank partials grouped by a hash
owner, all_to_all of [count, key-width flag], all_to_all of packed rows, merge — equals the
single-window oracle on the whole window.  The two halves (partials / merge) are the oracle here (test
infrastructure, owner split restated in numpy); on GPUs they are the C ABI's gs_window_reduce_partials /
gs_merge_partials (tests/test_gpu_dist.py runs this same exchange through them)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent
M = np.uint64(0xFFFFFFFFFFFFFFFF)


def owner_np(keys, nparts):
    """gs_owner_of restated: murmur3 fmix64 of the vertex, multiply-high by nparts."""
    with np.errstate(over="ignore"):
        x = keys.astype(np.int64).view(np.uint64)
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xFF51AFD7ED558CCD)
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xC4CEB9FE1A85EC53)
        x = x ^ (x >> np.uint64(33))
        return (((x >> np.uint64(32)) * np.uint64(nparts)) >> np.uint64(32)).astype(np.int64)


def oracle_halves(orc):
    tn = lambda t: t.numpy() if isinstance(t, torch.Tensor) else t
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))

    def group(k, cols, nparts):
        own = owner_np(k, nparts)
        order = np.argsort(own, kind="stable")
        return [t(k[order])] + [t(c[order]) for c in cols] + [np.bincount(own, minlength=nparts).tolist()]

    def partials(src, dst, val, direction, op, nparts):
        k, r = orc.window_reduce(tn(src), tn(dst), tn(val), direction, op)
        return tuple(group(k, [r], nparts))

    def merge(keys, vals, op, init):
        mop = 0 if op == 3 else op
        k, v = (orc.window_reduce(tn(keys), tn(keys), tn(vals), 1, mop) if init is None else
                orc.window_fold(tn(keys), tn(keys), tn(vals), 1, mop, init))
        return t(k), t(v)

    def fold_partials(src, dst, direction, nparts):
        k, dg, mx = orc.window_fold_degree_max(tn(src), tn(dst), direction)
        return tuple(group(k, [dg, mx], nparts))

    def fold_merge(keys, deg, mx, init_max):
        k, d = orc.window_reduce(tn(keys), tn(keys), tn(deg), 1, 0)
        _, m = orc.window_fold(tn(keys), tn(keys), tn(mx), 1, 2, init_max)
        return t(k), t(d), t(m)

    return partials, merge, fold_partials, fold_merge


class OracleTriEngine:
    """The gs_tri_dist_* steps restated in numpy (test infrastructure, CPU): the same id geometry,
    degree-class renumbering, owner(u) ranges, out-lists and equal-work parts as gs_triangles.hip, so
    distributed.triangles_window's exchanges run on gloo here; the self-pair term comes from the oracle
    (reference rule minus the simple graph's triangles)."""

    def __init__(self, orc):
        self.orc = orc

    @staticmethod
    def _np(t):
        return t.numpy() if isinstance(t, torch.Tensor) else np.asarray(t)

    def tri_dist_range(self, src, dst):
        s, d = self._np(src), self._np(dst)
        if len(s) == 0:
            return np.iinfo(np.int64).max, np.iinfo(np.int64).min
        return int(min(s.min(), d.min())), int(max(s.max(), d.max()))

    def _geom(self, gmin, gmax):
        x = (gmin ^ gmax) & ((1 << 64) - 1)
        B = max(1, x.bit_length())
        assert B <= 28
        return B, gmin & ~((1 << B) - 1)

    def tri_dist_degrees(self, src, dst, gmin, gmax):
        self.B, self.xor = self._geom(gmin, gmax)
        V = 1 << self.B
        s, d = self._np(src) ^ self.xor, self._np(dst) ^ self.xor
        return torch.from_numpy((np.bincount(s, minlength=V) + np.bincount(d, minlength=V)).astype(np.int32))

    @staticmethod
    def deg_class(d):
        d = d.astype(np.int64)
        lz = np.floor(np.log2(np.maximum(d, 1))).astype(np.int64)
        half = np.where(lz > 0, (d >> np.maximum(lz - 1, 0)) & 1, 0)
        return np.where(d == 0, 0, np.minimum(63, 1 + 2 * lz + half))

    def tri_dist_orient(self, src, dst, deg):
        B, V = self.B, 1 << self.B
        cls = self.deg_class(self._np(deg))
        rank = np.empty(V, np.int64)
        rank[np.argsort(cls, kind="stable")] = np.arange(V)
        a, b = self._np(src) ^ self.xor, self._np(dst) ^ self.xor
        keep = a != b
        ra, rb = rank[a[keep]], rank[b[keep]]
        u, v = np.minimum(ra, rb), np.maximum(ra, rb)
        self.okeys = (u << B) | v
        return torch.from_numpy(np.bincount(u, minlength=V).astype(np.int32)), int((~keep).sum())

    def tri_dist_route(self, dout, nparts):
        """owner ranges at equal shares of the raw work dout(dout+1)/2 (gs_tri_dist_route)"""
        B, V = self.B, 1 << self.B
        d = self._np(dout).astype(np.int64)
        pre = np.concatenate([[0], np.cumsum(d * (d + 1) // 2)])
        W = int(pre[V])
        self.split = [0 if q == 0 else V if q == nparts else int(np.searchsorted(pre[:V], W * q // nparts, side="left"))
                      for q in range(nparts + 1)]
        own = np.searchsorted(np.array(self.split[1:nparts]), self.okeys >> B, side="right")
        order = np.argsort(own, kind="stable")
        return torch.from_numpy(self.okeys[order]), np.bincount(own, minlength=nparts).tolist()

    def tri_dist_build(self, keys, V):
        k = np.unique(self._np(keys))
        u, v = k >> self.B, k & ((1 << self.B) - 1)
        return torch.from_numpy(v.astype(np.int32)), torch.from_numpy(np.bincount(u, minlength=V).astype(np.int32))

    def tri_dist_plan(self, dplus, part, nparts):
        """gs_tri_dist_plan: count ranges C_q (equal work), route ranges R_q (owner(u) = u * P >> B), and
        the elements of C_q ∩ R_part / C_part ∩ R_q"""
        dp = self._np(dplus).astype(np.int64)
        V, B, P = len(dp), self.B, nparts
        pre = np.concatenate([[0], np.cumsum(dp)])
        prew = np.concatenate([[0], np.cumsum(dp * (dp + 1) // 2)])
        W = int(prew[V])
        lower = lambda t: int(np.searchsorted(prew[:V], t, side="left"))
        cq = [0 if q == 0 else V if q == P else lower(W * q // P) for q in range(P + 1)]
        rq = self.split   # the route's owner ranges

        def inter(a, b):
            u0, u1 = max(cq[a], rq[b]), min(cq[a + 1], rq[b + 1])
            return int(pre[u1] - pre[u0]) if u0 < u1 else 0

        self.bd = dict(dp=dp, pre=pre, c=(cq[part], cq[part + 1]), r=(rq[part], rq[part + 1]), P=P)
        recv = [inter(part, q) for q in range(P)]
        # what an all-gather would have received vs the boundary exchange (rows of C, then requested rows)
        self.allgather_elems = int(pre[V] - (pre[rq[part + 1]] - pre[rq[part]]))
        self.boundary_elems = sum(recv) - inter(part, part)
        return [inter(q, part) for q in range(P)], recv, int(pre[V])

    def tri_dist_need(self, crows, nparts, V):
        bd, cr = self.bd, self._np(crows).astype(np.int64)
        (c0, c1), (r0, r1), dp = bd["c"], bd["r"], bd["dp"]
        v = cr[((cr < c0) | (cr >= c1)) & ((cr < r0) | (cr >= r1))]
        ids = np.unique(v[dp[v] > 0])
        own = np.searchsorted(np.array(self.split[1:nparts]), ids, side="right")
        self.req = ids
        counts = np.bincount(own, minlength=nparts).tolist()
        elems = np.bincount(own, weights=dp[ids], minlength=nparts).astype(np.int64).tolist()
        self.boundary_elems += sum(elems)
        return torch.from_numpy(ids.astype(np.int32)), counts, elems

    def tri_dist_serve(self, nbr, req_in, counts_in, elems_in):
        bd, nb, ids = self.bd, self._np(nbr), self._np(req_in).astype(np.int64)
        pre, dp, r0 = bd["pre"], bd["dp"], bd["r"][0]
        assert all(bd["r"][0] <= v < bd["r"][1] for v in ids)
        rows = [nb[pre[v] - pre[r0]: pre[v] - pre[r0] + dp[v]] for v in ids]
        bounds = np.concatenate([[0], np.cumsum(counts_in)]).astype(np.int64)
        send = [int(sum(dp[v] for v in ids[bounds[q]:bounds[q + 1]])) for q in range(len(counts_in))]
        out = np.concatenate(rows).astype(np.int32) if rows else np.zeros(0, np.int32)
        return torch.from_numpy(out), send

    def tri_dist_assemble(self, nbr, crows, rows_in, M):
        bd = self.bd
        pre, dp = bd["pre"], bd["dp"]
        full = np.zeros(M, np.int32)
        (c0, c1), (r0, r1) = bd["c"], bd["r"]
        full[pre[r0]:pre[r1]] = self._np(nbr)
        full[pre[c0]:pre[c1]] = self._np(crows)
        ri, at = self._np(rows_in), 0
        for v in self.req:
            full[pre[v]:pre[v] + dp[v]] = ri[at:at + dp[v]]
            at += dp[v]
        return torch.from_numpy(full)

    def tri_dist_count(self, nbr, dplus, part, nparts):
        nbr, dp = self._np(nbr).astype(np.int64), self._np(dplus).astype(np.int64)
        V = len(dp)
        start = np.concatenate([[0], np.cumsum(dp)])
        work = dp * (dp + 1) // 2
        pre = np.concatenate([[0], np.cumsum(work)])   # pre[u] = work before u, pre[V] = total
        W = int(pre[V])
        lower = lambda t: int(np.searchsorted(pre[:V], t, side="left"))
        u0 = 0 if part == 0 else lower(W * part // nparts)
        u1 = V if part + 1 == nparts else lower(W * (part + 1) // nparts)
        T = 0
        for u in range(u0, u1):
            L = nbr[start[u]:start[u + 1]]
            for i, v in enumerate(L[:-1]):
                T += len(np.intersect1d(L[i + 1:], nbr[start[v]:start[v + 1]], assume_unique=True))
        return T

    def triangles_selfpair(self, src, dst):
        """reference rule minus the simple graph's triangles (this pipeline on the whole window)"""
        s, d = self._np(src), self._np(dst)
        keep = s != d
        return self.orc.window_triangles_ref(s, d)[1] - self.orc.window_triangles_fwd(s[keep], d[keep])[1]


def candidate_groups(a, b, f):
    """GenerateCandidateEdges output split per emitting vertex: a vertex's rows start with its
    (v, neighbour, false) records, so row i belongs to a[last false row <= i]."""
    a, b, f = (np.asarray(x) for x in (a, b, f))
    idx = np.maximum.accumulate(np.where(f == 0, np.arange(len(f)), -1))
    v = a[idx]
    starts = np.flatnonzero(np.r_[True, v[1:] != v[:-1]])
    ends = np.r_[starts[1:], len(v)]
    return {int(v[s0]): (a[s0:e0], b[s0:e0], f[s0:e0]) for s0, e0 in zip(starts, ends)}


def oracle_candidates_part(orc):
    """gs_window_candidates_part restated: the oracle's window output, rows of owned vertices only."""
    def part_fn(src, dst, nparts, part):
        a, b, f, _ = orc.window_candidates(src.numpy(), dst.numpy())
        idx = np.maximum.accumulate(np.where(f == 0, np.arange(len(f)), -1))
        keep = owner_np(a[idx], nparts) == part
        return a[keep], b[keep], f[keep]
    return part_fn


def check_candidates_split(outs, full):
    """Every vertex's rows come from exactly one rank and equal the whole window's rows for it."""
    want = candidate_groups(*full)
    seen = set()
    for a, b, f in outs:
        for v, rows in candidate_groups(a, b, f).items():
            assert v not in seen, v
            seen.add(v)
            for g, w in zip(rows, want[v]):
                assert np.array_equal(g, w), v
    assert seen == set(want)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CASES = [("reduce", dr, op, None) for dr in (0, 1, 2) for op in (0, 1, 2, 3)] + \
        [("fold", 1, 0, 1000), ("fold", 2, 1, 5), ("fold", 0, 3, 7), ("deg", 0, None, None), ("deg", 1, None, None),
         ("deg", 2, None, 1 << 11)]
SHIFTS = (("rel32", 1 << 20, 0), ("wide", 1 << 30, -(1 << 50)))


def run_cases(D, halves, s, d, v, to_dev=lambda a: torch.from_numpy(a)):
    partials, merge, fold_partials, fold_merge = halves
    res = {}
    S, Dd, V = to_dev(s), to_dev(d), to_dev(v)
    for kind, direction, op, init in CASES:
        if kind == "deg":
            k, dg, mx = D.fold_degree_max_window(fold_partials, fold_merge, S, Dd, direction,
                                                 -(1 << 63) if init is None else init)
            res[(kind, direction, op, init)] = (k.cpu().numpy(), dg.cpu().numpy(), mx.cpu().numpy())
        else:
            k, r = D.reduce_window(partials, merge, S, Dd, V, direction, op, init)
            res[(kind, direction, op, init)] = (k.cpu().numpy(), r.cpu().numpy())
    # keys past 2^32 (the 64-bit row encoding) and negative keys
    for tag, mul, off in SHIFTS:
        k, r = D.reduce_window(partials, merge, to_dev(s * mul + off), to_dev(d * mul + off), V, 1, 0)
        res[tag] = (k.cpu().numpy(), r.cpu().numpy())
    return res


def check_cases(oracle, out, world, s, d, v):
    for kind, direction, op, init in CASES:
        key = (kind, direction, op, init)
        parts = [out[r][key] for r in range(world)]
        cat = [np.concatenate([p[i] for p in parts]) for i in range(len(parts[0]))]
        order = np.argsort(cat[0], kind="stable")   # owners hold interleaved vertex sets
        cat = [c[order] for c in cat]
        if kind == "deg":
            want = oracle.window_fold_degree_max(s, d, direction, -(1 << 63) if init is None else init)
        elif init is None:
            want = oracle.window_reduce(s, d, v, direction, op)
        else:
            want = oracle.window_fold(s, d, v, direction, op, init)
        for g, w in zip(cat, want):
            assert np.array_equal(g, w), key
    for tag, mul, off in SHIFTS:
        k = np.concatenate([out[r][tag][0] for r in range(world)])
        r_ = np.concatenate([out[r][tag][1] for r in range(world)])
        o = np.argsort(k)
        wk, wv = oracle.window_reduce(s * mul + off, d * mul + off, v, 1, 0)
        assert np.array_equal(k[o], wk) and np.array_equal(r_[o], wv), tag


def _worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as ge
    ge.load_package()
    from gelly_streaming_amd import distributed as D
    orc = ge.load_oracle()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 40000
    s, d = orc.gen_rmat(12, n, 0x5EED03, a=0.65, b=0.15, c=0.15, permute=False, first_edge=rank * n)
    v = orc.gen_values(n, 5, orc.DT_I64, first_edge=rank * n)
    res = run_cases(D, oracle_halves(orc), s, d, v)
    fs, fd = D.gather_window(torch.from_numpy(s), torch.from_numpy(d))
    res["gathered"] = (fs.numpy(), fd.numpy())
    # WindowTriangles over the split window: the real exchanges (ranges, degrees, routed oriented edges, the
    # boundary adjacency rows, equal-work parts) with the steps restated in numpy; plus a small window
    # with self-loops (the gathered self-pair term)
    te = OracleTriEngine(orc)
    ts, td = orc.gen_rmat(11, 20000, 0x5EED05, no_self_loops=True, first_edge=rank * 20000)
    res["tri"] = D.triangles_window(te, torch.from_numpy(ts), torch.from_numpy(td))
    ls, ld = orc.gen_rmat(6, 1500, 0x5EED06, first_edge=rank * 1500)
    res["tri_loops"] = D.triangles_window(te, torch.from_numpy(ls), torch.from_numpy(ld))
    # a rank with an empty slice (rank 1 holds nothing) and a window with fewer records than ranks
    es, ed = orc.gen_rmat(9, 5000, 0x5EED08, no_self_loops=True)
    if rank:
        es, ed = es[:0], ed[:0]
    res["tri_empty_rank"] = D.triangles_window(te, torch.from_numpy(es), torch.from_numpy(ed))
    one_s, one_d = (np.array([3], np.int64), np.array([7], np.int64)) if rank == 0 else \
        (np.zeros(0, np.int64), np.zeros(0, np.int64))
    res["tri_one_record"] = D.triangles_window(te, torch.from_numpy(one_s), torch.from_numpy(one_d))
    ev = orc.gen_values(len(es), 9, orc.DT_I64)
    ek, er = D.reduce_window(oracle_halves(orc)[0], oracle_halves(orc)[1], torch.from_numpy(es),
                             torch.from_numpy(ed), torch.from_numpy(ev), 2, 0)
    res["reduce_empty_rank"] = (ek.numpy(), er.numpy())
    # GenerateCandidateEdges over the split window: edges routed to their endpoints' owners (the real
    # all-to-all), each rank's owned vertices from the oracle
    cs, cd = orc.gen_rmat(8, 3000, 0x5EED07, first_edge=rank * 3000)
    res["cand"] = D.candidates_window(oracle_candidates_part(orc), torch.from_numpy(cs), torch.from_numpy(cd))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_window_two_ranks(oracle):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 40000
    s, d = oracle.gen_rmat(12, 2 * n, 0x5EED03, a=0.65, b=0.15, c=0.15, permute=False)
    v = oracle.gen_values(2 * n, 5, oracle.DT_I64)
    check_cases(oracle, out, world, s, d, v)
    ts, td = oracle.gen_rmat(11, 40000, 0x5EED05, no_self_loops=True)
    w, ex, _ = oracle.window_triangles_fwd(ts, td)
    ls, ld = oracle.gen_rmat(6, 3000, 0x5EED06)
    assert (ls == ld).any()                       # the self-pair term is exercised
    lw, lex, _, tree = oracle.window_triangles_ref(ls, ld)
    assert not tree
    cs, cd = oracle.gen_rmat(8, 6000, 0x5EED07)
    assert (cs == cd).any()                       # self-loops (two records for their vertex) included
    check_candidates_split([out[r]["cand"] for r in range(world)], oracle.window_candidates(cs, cd)[:3])
    es, ed = oracle.gen_rmat(9, 5000, 0x5EED08, no_self_loops=True)
    ew, eex, _ = oracle.window_triangles_fwd(es, ed)
    ev = oracle.gen_values(len(es), 9, oracle.DT_I64)
    rk = np.concatenate([out[r]["reduce_empty_rank"][0] for r in range(world)])
    rv = np.concatenate([out[r]["reduce_empty_rank"][1] for r in range(world)])
    o = np.argsort(rk)
    wk, wv = oracle.window_reduce(es, ed, ev, 2, 0)
    assert np.array_equal(rk[o], wk) and np.array_equal(rv[o], wv)
    for r in range(world):
        assert np.array_equal(out[r]["gathered"][0], s) and np.array_equal(out[r]["gathered"][1], d)
        assert out[r]["tri"] == (ex, w, True)
        assert out[r]["tri_loops"] == (lex, lw, True)
        assert out[r]["tri_empty_rank"] == (eex, ew, True)
        assert out[r]["tri_one_record"] == (0, 0, True)


def test_owner_split_is_balanced():
    """The hash owner spreads a skewed window's vertices evenly (keyBy's purpose)."""
    keys = np.arange(1 << 20, dtype=np.int64)
    c = np.bincount(owner_np(keys, 8), minlength=8)
    assert c.min() > 0.98 * c.max()


def _tri_worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as ge
    ge.load_package()
    from gelly_streaming_amd import distributed as D
    orc = ge.load_oracle()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    te = OracleTriEngine(orc)
    n = 12000
    ts, td = orc.gen_rmat(12, n, 0x5EED09, no_self_loops=True, first_edge=rank * n)
    got = D.triangles_window(te, torch.from_numpy(ts), torch.from_numpy(td))
    q.put((rank, (got, te.boundary_elems, te.allgather_elems)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 4])
def test_split_window_triangles_boundary_exchange(oracle, world):
    """WindowTriangles over a window split across 3 / 4 gloo ranks: the boundary adjacency (rows of each
    rank's count range, then the rows of their targets it holds in neither range) gives the whole
    window's count on every rank; no rank receives more row elements than an all-gather of every other
    rank's out-lists would deliver, and the ranks together receive well under it."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tri_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ts, td = oracle.gen_rmat(12, 12000 * world, 0x5EED09, no_self_loops=True)
    w, ex, _ = oracle.window_triangles_fwd(ts, td)
    assert ex > 0
    for r in range(world):
        got, bnd, full = out[r]
        assert got == (ex, w, True), (r, got, ex)
        assert bnd <= full, (r, bnd, full)
    # over the ranks, far less than every rank receiving every other rank's rows
    assert sum(out[r][1] for r in range(world)) < 0.8 * sum(out[r][2] for r in range(world)), out


def _sparse(x):
    """an order-preserving injective map of small ids onto Long ids spanning more than 2^52 values"""
    return x * ((1 << 40) + 12345) - (1 << 60)


def _tri_sparse_worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as ge
    ge.load_package()
    from gelly_streaming_amd import distributed as D
    orc = ge.load_oracle()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    te = OracleTriEngine(orc)
    out = {}
    n = 9000
    ts, td = orc.gen_rmat(12, n, 0x5EED0E, no_self_loops=True, first_edge=rank * n)
    out["sparse"] = D.triangles_window(te, torch.from_numpy(_sparse(ts)), torch.from_numpy(_sparse(td)))
    ls, ld = orc.gen_rmat(9, 3000, 0x5EED0F, first_edge=rank * 3000)
    out["sparse_loops"] = D.triangles_window(te, torch.from_numpy(_sparse(ls)), torch.from_numpy(_sparse(ld)))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_split_window_triangles_sparse_long_ids():
    """Split-window WindowTriangles over Long ids spanning more than 2^52 values (SimpleEdgeStream.java
    :173-183 keys any Long): the ranks relabel to the whole window's compact ids (relabel_window: distinct
    ids all-gathered) and count the whole window's triangles; with self-loops the self-pair term keeps
    the original ids (its HashSet order)."""
    import __graft_entry__ as ge
    orc = ge.load_oracle()
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tri_sparse_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ts, td = orc.gen_rmat(12, 9000 * world, 0x5EED0E, no_self_loops=True)
    w, ex, _ = orc.window_triangles_fwd(_sparse(ts), _sparse(td))
    assert ex > 0 and (w, ex) == orc.window_triangles_fwd(ts, td)[:2]
    ls, ld = orc.gen_rmat(9, 3000 * world, 0x5EED0F)
    assert (ls == ld).any()
    lw, lex, _, tree = orc.window_triangles_ref(_sparse(ls), _sparse(ld))
    for r in range(world):
        assert out[r]["sparse"] == (ex, w, True), (r, out[r]["sparse"], ex)
        assert out[r]["sparse_loops"] == (lex, lw, True), (r, out[r]["sparse_loops"], lex)
