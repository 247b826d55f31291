"""GPU: the multi-GPU keyBy halves of the C ABI (gs_dist.hip) and the ctx-owned RCCL communicator.

  - gs_window_reduce_partials / gs_window_fold_degree_max_partials: rows grouped by gs_owner_of (the
    device split equals the numpy restatement), ascending within an owner, counts per owner;
  - world 2 over gloo between two processes sharing this GPU: distributed.reduce_window /
    fold_degree_max_window through the ENGINE's halves (partials on the device, rows exchanged on the
    host, merge on the device) equal the whole-window oracle for every op, direction and init;
  - world 1 over RCCL through the library's own communicator: gs_window_reduce_dist /
    gs_window_fold_degree_max_dist equal the single-GPU window, gs_comm_allreduce_sum_u64 sums."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
from test_distributed_gloo import _free_port, check_cases, check_candidates_split, owner_np, run_cases  # noqa: E402


@pytest.mark.parametrize("nparts", [1, 2, 3, 8, 64])
def test_partials_grouped_by_owner(engine, oracle, nparts):
    n = 300_001
    s, d = oracle.gen_rmat(16, n, 0x5EED02)
    v = oracle.gen_values(n, 3, oracle.DT_I64)
    S, D, V = (torch.from_numpy(x).cuda() for x in (s, d, v))
    for direction in (1, 2):
        k, p, counts = engine.reduce_partials(S, D, V, direction, 0, nparts)
        k, p = k.cpu().numpy(), p.cpu().numpy()
        rk, rv = oracle.window_reduce(s, d, v, direction, 0)
        assert sum(counts) == len(rk) == len(k)
        own = owner_np(k, nparts)
        bounds = np.concatenate([[0], np.cumsum(counts)])
        for o in range(nparts):
            seg = slice(bounds[o], bounds[o + 1])
            assert (own[seg] == o).all() and (np.diff(k[seg]) > 0).all()
        o = np.argsort(k)
        assert np.array_equal(k[o], rk) and np.array_equal(p[o], rv)
        assert all(engine.owner_of(int(x), nparts) == int(y) for x, y in zip(k[:50], own[:50]))
    kd, dg, mx, counts = engine.fold_degree_max_partials(S, D, 0, nparts)
    o = np.argsort(kd.cpu().numpy())
    want = oracle.window_fold_degree_max(s, d, 0)
    for g, w in zip((kd, dg, mx), want):
        assert np.array_equal(g.cpu().numpy()[o], w)


def test_merge_partials_ops(engine, oracle):
    """The owner half alone: rows of several ranks for the same vertices merge by op (COUNT by SUM)."""
    rng = np.random.default_rng(5)
    k = rng.integers(0, 1 << 18, 200_000).astype(np.int64)
    v = rng.integers(-(1 << 40), 1 << 40, 200_000).astype(np.int64)
    K, Vv = torch.from_numpy(k).cuda(), torch.from_numpy(v).cuda()
    for op, mop in ((0, 0), (1, 1), (2, 2), (3, 0)):
        gk, gv = engine.merge_partials(K, Vv, op)
        wk, wv = oracle.window_reduce(k, k, v, 1, mop)
        assert np.array_equal(gk.cpu().numpy(), wk) and np.array_equal(gv.cpu().numpy(), wv)
    gk, gv = engine.merge_partials(K, Vv, 1, init=-5)
    wk, wv = oracle.window_fold(k, k, v, 1, 1, -5)
    assert np.array_equal(gv.cpu().numpy(), wv)


def _worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from gelly_streaming_amd import distributed as D
    orc = ge.load_oracle()
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 40000
    s, d = orc.gen_rmat(12, n, 0x5EED03, a=0.65, b=0.15, c=0.15, permute=False, first_edge=rank * n)
    v = orc.gen_values(n, 5, orc.DT_I64, first_edge=rank * n)
    eng = pkg.Engine(0)
    res = run_cases(D, D.engine_halves(eng), s, d, v, to_dev=lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda())
    # GenerateCandidateEdges over the split window: routed edges, gs_window_candidates_part per rank
    cs, cd = orc.gen_rmat(10, 20000, 0x5EED07, first_edge=rank * 20000)
    a, b, f = D.candidates_window(eng.candidates, torch.from_numpy(cs).cuda(), torch.from_numpy(cd).cuda())
    res["cand"] = (a.cpu().numpy(), b.cpu().numpy(), f.cpu().numpy())
    eng.close()
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_engine_halves_two_ranks_gloo(oracle):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 40000
    s, d = oracle.gen_rmat(12, 2 * n, 0x5EED03, a=0.65, b=0.15, c=0.15, permute=False)
    v = oracle.gen_values(2 * n, 5, oracle.DT_I64)
    check_cases(oracle, out, world, s, d, v)
    cs, cd = oracle.gen_rmat(10, 40000, 0x5EED07)
    check_candidates_split([out[r]["cand"] for r in range(world)], oracle.window_candidates(cs, cd)[:3])


@pytest.mark.parametrize("nparts", [2, 3, 8])
def test_candidates_part(pkg, engine, oracle, nparts):
    """gs_window_candidates_part: part p, given the edges incident to its vertices in stream order, emits
    exactly the whole window's records of the vertices it owns (exact JDK HashSet order included: the
    ids are multiples of 16, so large neighbour sets collide into bins of 9 and take the simulation)."""
    s, d = oracle.gen_rmat(12, 120_000, 0x5EED08)
    for mul in (1, 16):
        S, D_ = s * mul, d * mul
        full = [x.cpu().numpy() for x in engine.candidates(torch.from_numpy(S).cuda(), torch.from_numpy(D_).cuda())]
        w = oracle.window_candidates(S, D_)
        assert all(np.array_equal(g, x) for g, x in zip(full, w[:3]))
        oa, ob = owner_np(S, nparts), owner_np(D_, nparts)
        outs = []
        for part in range(nparts):
            keep = (oa == part) | (ob == part)
            ps, pd = (torch.from_numpy(np.ascontiguousarray(x[keep])).cuda() for x in (S, D_))
            outs.append([x.cpu().numpy() for x in engine.candidates(ps, pd, nparts, part)])
            # the chunked part session (gs_candidates_begin_part, GpuCandidatesOperator at parallelism P):
            # the same records in the same order, in chunks
            total = engine.candidates_begin(ps, pd, nparts, part)
            assert total == len(outs[-1][0])
            got, done = [], total == 0
            while not done:
                a, b, f, first, done = engine.candidates_next(50_000)
                assert first == sum(len(g[0]) for g in got)
                got.append((a.cpu().numpy(), b.cpu().numpy(), f.cpu().numpy()))
            if total:
                for j in range(3):
                    assert np.array_equal(np.concatenate([g[j] for g in got]), outs[-1][j]), (mul, part, j)
                with pytest.raises(pkg.GsError):
                    engine.candidates_vertex_range(int(ps[0]))   # not offered on a part session
        check_candidates_split(outs, full)


def test_device_count(pkg):
    assert pkg.Engine.device_count() >= 1


def test_rccl_world_one_through_the_abi(pkg, oracle):
    n = 250_000
    s, d = oracle.gen_rmat(15, n, 0x5EED02)
    v = oracle.gen_values(n, 8, oracle.DT_I64)
    S, D, V = (torch.from_numpy(x).cuda() for x in (s, d, v))
    with pkg.Engine(0) as e:
        e.comm_init(1, 0, pkg.Engine.comm_unique_id())
        for direction in (0, 1, 2):
            for op in (0, 1, 2, 3):
                gk, gv = e.reduce_dist(S, D, V, direction, op)
                wk, wv = oracle.window_reduce(s, d, v, direction, op)
                assert np.array_equal(gk.cpu().numpy(), wk) and np.array_equal(gv.cpu().numpy(), wv)
        gk, gv = e.reduce_dist(S, D, V, 1, 0, init=10)
        assert np.array_equal(gv.cpu().numpy(), oracle.window_fold(s, d, v, 1, 0, 10)[1])
        got = e.fold_degree_max_dist(S, D, 2)
        for g, w in zip(got, oracle.window_fold_degree_max(s, d, 2)):
            assert np.array_equal(g.cpu().numpy(), w)
        assert e.comm_allreduce_sum(12345) == 12345
        e.comm_destroy()


@pytest.mark.parametrize("keys", ["narrow", "wide"])
def test_rccl_exchange_forced_at_world_one(pkg, oracle, keys):
    """gs_window_reduce_dist's exchange itself on a one-rank communicator (GS_FLAG_TEST_FORCE_EXCHANGE):
    local partials -> owner partition -> one all-to-all of [rows, flags] -> one packed all-to-all of rows
    (4-byte keys; 8-byte keys when a key lies outside [0, 2^32)) -> merge.  Every op, dtype and the degree
    fold, against the oracle."""
    n = 200_003
    s, d = oracle.gen_rmat(15, n, 0x5EED09)
    if keys == "wide":
        s, d = s * 7919 - (3 << 40), d * 7919 - (3 << 40)
    s, d = np.ascontiguousarray(s), np.ascontiguousarray(d)
    with pkg.Engine(0, flags=pkg._lib.GS_FLAG_TEST_FORCE_EXCHANGE) as e:
        e.comm_init(1, 0, pkg.Engine.comm_unique_id())
        for dt in (oracle.DT_I64, oracle.DT_I32, oracle.DT_F64):
            v = oracle.gen_values(n, 8 + dt, dt)
            S, D, V = (torch.from_numpy(x).cuda() for x in (s, d, v))
            for direction, op in ((1, 0), (2, 1), (0, 2), (2, 3)):
                if dt == oracle.DT_F64 and op in (1, 2):
                    continue
                gk, gv = e.reduce_dist(S, D, V, direction, op)
                wk, wv = oracle.window_reduce(s, d, v, direction, op)
                assert np.array_equal(gk.cpu().numpy(), wk)
                g = gv.cpu().numpy()
                if dt == oracle.DT_F64 and op == 0:
                    assert np.allclose(g, wv, rtol=1e-5, atol=0)
                else:
                    assert np.array_equal(g, wv), (dt, direction, op)
        gk, gv = e.reduce_dist(S, D, V, 1, 3, init=10)
        assert np.array_equal(gv.cpu().numpy(), oracle.window_fold(s, d, v, 1, 3, 10)[1])
        for direction in (1, 2):
            got = e.fold_degree_max_dist(S, D, direction, -5)
            for g, w in zip(got, oracle.window_fold_degree_max(s, d, direction, -5)):
                assert np.array_equal(g.cpu().numpy(), w)
        e.comm_destroy()


# ---- WindowTriangles over a split window (gs_tri_dist_*) -------------------------------------------
TRI_CASES = (("rmat", 14, 120_000, True), ("loops", 8, 6_000, False), ("wide", 13, 60_000, True))


def _tri_case(orc, kind, scale, n, no_loops, rank):
    s, d = orc.gen_rmat(scale, n, 0x5EED07, no_self_loops=no_loops, first_edge=rank * n)
    if kind == "wide":   # ids spread over 2^27 (still one 28-bit geometry) and shifted far from 0
        s, d = s * 13_001 + (5 << 40), d * 13_001 + (5 << 40)
    return np.ascontiguousarray(s), np.ascontiguousarray(d)


def _tri_worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from gelly_streaming_amd import distributed as D
    orc = ge.load_oracle()
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = pkg.Engine(0)
    res = {}
    for kind, scale, n, no_loops in TRI_CASES:
        s, d = _tri_case(orc, kind, scale, n, no_loops, rank)
        res[kind] = D.triangles_window(eng, torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda())
    eng.close()
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_split_window_triangles_two_ranks_gloo(oracle):
    """Two processes sharing this GPU, gloo between them: every rank holds half of the window's records;
    degrees all-reduced, oriented edges routed to owner(u), the boundary adjacency exchanged (rows of the
    rank's count range, then the rows of their targets it holds in neither range), each rank counts its
    equal-work share -> the whole window's count (forward algorithm; the reference rule with loops)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tri_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for kind, scale, n, no_loops in TRI_CASES:
        parts = [_tri_case(oracle, kind, scale, n, no_loops, r) for r in range(world)]
        s = np.concatenate([p[0] for p in parts])
        d = np.concatenate([p[1] for p in parts])
        if no_loops:
            w, ex, _ = oracle.window_triangles_fwd(s, d)
        else:
            assert (s == d).any()
            w, ex, _, tree = oracle.window_triangles_ref(s, d)
            assert not tree
        for r in range(world):
            assert out[r][kind] == (ex, w, True), (kind, r)


def test_split_window_steps_and_rccl_world_one(pkg, oracle):
    """The steps on one rank (nparts 1 and a 3-way split of the count summed) and gs_window_triangles_dist
    over a world-1 RCCL communicator equal gs_window_triangles."""
    s, d = oracle.gen_rmat(15, 300_000, 0x5EED08)
    S, Dd = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    with pkg.Engine(0) as e:
        whole = e.triangles(S, Dd)
        lo, hi = e.tri_dist_range(S, Dd)
        assert (lo, hi) == (int(min(s.min(), d.min())), int(max(s.max(), d.max())))
        deg = e.tri_dist_degrees(S, Dd, lo, hi)
        dout, loops = e.tri_dist_orient(S, Dd, deg)
        assert loops == int((s == d).sum()) and int(dout.sum()) == len(s) - loops
        keys, counts = e.tri_dist_route(dout, 1)
        assert counts == [keys.numel()] == [len(s) - loops]
        nbr, dplus = e.tri_dist_build(keys, deg.numel())
        assert int(dplus.sum()) == nbr.numel()
        T = sum(e.tri_dist_count(nbr, dplus, p, 3) for p in range(3))
        S_ = e.triangles_selfpair(S, Dd) if loops else 0
        assert T + S_ == whole[0] == e.tri_dist_count(nbr, dplus, 0, 1) + S_
        e.comm_init(1, 0, pkg.Engine.comm_unique_id())
        assert e.triangles_dist(S, Dd) == whole
        e.comm_destroy()


def test_merges_keep_their_own_speculative_counts(pkg, oracle):
    """keyBy on one ctx alternates a window's partials and a merge of received rows: the merge's rows
    spread over the buckets unlike the window's and arrive as sorted sender runs, so merges run in their
    own slot (slot 1: their own bucket counts, one segment per bucket, their own packing state) and the
    windows keep speculating from their own counts (a shared slot made every window miss).  Each merge
    here gets two sender runs with common vertices: owner 0's partials of windows w and w + 1."""
    def win(w):
        s, d = oracle.gen_rmat(18, 1 << 21, 0x5EED02, first_edge=w << 21)
        v = oracle.gen_values(1 << 21, 0x5EED02, oracle.DT_I64, first_edge=w << 21)
        return s, d, v

    with pkg.Engine(0) as e:
        spec, mspec = [], []
        nxt = win(0)
        for w in range(6):
            (s, d, v), nxt = nxt, win(w + 1)
            runs_k, runs_v = [], []
            for j, (a, b, c) in enumerate(((s, d, v), nxt)):
                S, D_, V = (torch.from_numpy(x).cuda() for x in (a, b, c))
                k, p, counts = e.reduce_partials(S, D_, V, 1, 0, 2)
                if j == 0:
                    spec.append(e.stage_times().speculative)
                runs_k.append(k[:counts[0]].clone())
                runs_v.append(p[:counts[0]].clone())
            mk, mv = e.merge_partials(torch.cat(runs_k), torch.cat(runs_v), 0)
            mspec.append(e.stage_times().speculative)
            rk, rv = oracle.window_reduce(np.concatenate([s, nxt[0]]), np.concatenate([d, nxt[1]]),
                                          np.concatenate([v, nxt[2]]), 1, 0)
            own = owner_np(rk, 2) == 0
            assert np.array_equal(mk.cpu().numpy(), rk[own]) and np.array_equal(mv.cpu().numpy(), rv[own])
        assert spec[0] == 0 and spec[1:] == [1] * 5, spec
        assert mspec[0] == 0 and mspec[1:] == [1] * 5, mspec
