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
    # WindowTriangles across ranks: all-gathered adjacency must be the whole window in stream order;
    # each rank contributes its part (here: rank 0 counts everything) and the all-reduce sums them
    fs, fd = D.gather_window(torch.from_numpy(s), torch.from_numpy(d))
    res["gathered"] = (fs.numpy(), fd.numpy())
    part = lambda a, b, r, w: (orc.window_triangles_fwd(a.numpy(), b.numpy())[1] if r == 0 else 0)
    res["tri"] = D.triangles_window(part, torch.from_numpy(s), torch.from_numpy(d))
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
    for r in range(world):
        assert np.array_equal(out[r]["gathered"][0], s) and np.array_equal(out[r]["gathered"][1], d)
        w, ex, _ = oracle.window_triangles_fwd(s, d)
        assert out[r]["tri"] == (ex, w)


def test_owner_split_is_balanced():
    """The hash owner spreads a skewed window's vertices evenly (keyBy's purpose)."""
    keys = np.arange(1 << 20, dtype=np.int64)
    c = np.bincount(owner_np(keys, 8), minlength=8)
    assert c.min() > 0.98 * c.max()
