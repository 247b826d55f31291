"""Multi-GPU window: keyBy(vertex) across ranks, one process per GPU.

The reference partitions each window by `keyBy(NeighborKeySelector)` (SimpleEdgeStream.java:159-167):
every record travels to the subtask that owns its key, which folds it.  Here every rank pre-reduces its
own slice of the window on its GPU and only the per-vertex partials travel, through the two halves of
the C ABI (include/gelly_hip.h, gs_dist.hip) around one exchange:

  1. partials: gs_window_reduce_partials -> this slice's (vertex, partial) rows grouped by
               owner(v) = gs_owner_of(v, world) (a hash of the vertex, as keyBy is), with the
               per-owner row counts; the owner split is computed on the device
  2. exchange: all_to_all_single of [row count, key-width flag] per peer, then ONE all_to_all_single of
               packed rows (RCCL over xGMI with the "nccl" backend; gloo in the CPU tests).  Keys travel
               as 32-bit values when every rank's keys are non-negative and below 2^32 (12-byte rows
               for a Long partial instead of 16)
  3. merge:    gs_merge_partials -> the vertices this rank owns (COUNT partials add up; foldNeighbors'
               init is applied once, here)

Which rank owns a vertex is not observable in the reference's output (per-vertex records compared as
unordered sets).  Integer results stay bit-exact (the ops are associative and commutative); float
sums move within the 1e-5 tolerance.  The halves are injectable callables so the exchange logic also
runs on CPU with gloo in tests (tests/test_distributed_gloo.py); on GPUs they are Engine methods.
The library also owns an RCCL communicator itself (Engine.comm_init + Engine.reduce_dist): the same
three steps with the exchange inside gs_window_reduce_dist, for callers without torch.distributed.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

SUM, MIN, MAX, COUNT = 0, 1, 2, 3


def merge_op(op: int) -> int:
    return SUM if op == COUNT else op


def _comm_device(group, like: torch.Tensor) -> torch.device:
    """nccl exchanges device tensors; gloo host tensors."""
    return like.device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def exchange_partials(keys: torch.Tensor, cols: list, counts: list, group=None):
    """Send rows [sum(counts[:p]), sum(counts[:p+1])) of (keys, *cols) to rank p (rows grouped by owner).
    Returns the received (keys, cols) on keys' device."""
    world = dist.get_world_size(group)
    home = keys.device
    cdev = _comm_device(group, keys)
    if keys.numel():
        wide = (keys.min() < 0) | (keys.max() >= (1 << 32))
    else:
        wide = torch.zeros((), dtype=torch.bool, device=home)
    send = torch.stack([torch.tensor(counts, dtype=torch.int64, device=home),
                        wide.to(torch.int64).expand(world)], dim=1).to(cdev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    rl = recv.tolist()                                   # the exchange's one host read
    recv_counts = [r[0] for r in rl]
    wide_any = any(r[1] for r in rl)
    kpart = keys.contiguous() if wide_any else keys.to(torch.int32)
    parts = [kpart] + [c.contiguous() for c in cols]
    widths = [p.element_size() for p in parts]
    row = sum(widths)
    # an empty slice may come as a stride-0 tensor, which cannot be viewed as bytes
    as_bytes = lambda p, w: p.view(torch.uint8).view(-1, w) if p.numel() else \
        torch.empty((0, w), dtype=torch.uint8, device=p.device)
    packed = torch.cat([as_bytes(p, w) for p, w in zip(parts, widths)], dim=1).to(cdev)
    rp = torch.empty((sum(recv_counts), row), dtype=torch.uint8, device=cdev)
    dist.all_to_all_single(rp, packed, recv_counts, list(counts), group=group)
    rp = rp.to(home)
    out, at = [], 0
    for p, w in zip(parts, widths):
        out.append(rp[:, at:at + w].contiguous().view(p.dtype).view(-1))
        at += w
    rk = out[0] if wide_any else (out[0].to(torch.int64) & 0xFFFFFFFF)
    return rk, out[1:]


def reduce_window(partials, merge, src, dst, val, direction: int, op: int, init=None, group=None):
    """reduceOnEdges (init None) / foldNeighbors over a window whose edges are spread over the ranks of
    `group`.  partials(src, dst, val, direction, op, nparts) -> (keys, vals, counts);
    merge(keys, vals, op, init) -> (keys, vals).  Returns this rank's owned (vertex, value) pairs,
    vertices ascending."""
    world = dist.get_world_size(group)
    k, v, counts = partials(src, dst, val, direction, op, world)
    if world == 1 and init is None:   # the only rank owns every vertex: nothing to exchange or merge
        return k, v
    rk, (rv,) = exchange_partials(k, [v], counts, group)
    return merge(rk, rv, op, init)


def fold_degree_max_window(partials, merge, src, dst, direction: int, init_max: int, group=None):
    """foldNeighbors(degree, max neighbour) across ranks: degrees merge by SUM, maxima by MAX, then the
    fold's init.  partials(src, dst, direction, nparts) -> (keys, deg, mx, counts);
    merge(keys, deg, mx, init_max) -> (keys, deg, mx)."""
    world = dist.get_world_size(group)
    k, d, m, counts = partials(src, dst, direction, world)
    if world == 1:
        return merge(k, d, m, init_max) if init_max != -(1 << 63) else (k, d, m)
    rk, (rd, rm) = exchange_partials(k, [d, m], counts, group)
    return merge(rk, rd, rm, init_max)


def owner_of(v: torch.Tensor, nparts: int) -> torch.Tensor:
    """gs_owner_of on a tensor (murmur3 fmix64 of the vertex, multiply-high by nparts) in int64
    arithmetic: products wrap mod 2^64, right shifts are masked to logical shifts."""
    m31, m32 = (1 << 31) - 1, (1 << 32) - 1
    c1, c2 = 0xFF51AFD7ED558CCD - (1 << 64), 0xC4CEB9FE1A85EC53 - (1 << 64)
    x = v.to(torch.int64)
    x = x ^ ((x >> 33) & m31)
    x = x * c1
    x = x ^ ((x >> 33) & m31)
    x = x * c2
    x = x ^ ((x >> 33) & m31)
    return (((x >> 32) & m32) * nparts) >> 32


def route_edges_to_owners(src: torch.Tensor, dst: torch.Tensor, group=None):
    """Every edge (a, b) of this rank's slice goes to owner(a) and to owner(b) (once when they are the
    same rank), local order kept; each rank receives its edges concatenated in rank order (= stream
    order when rank r holds the r-th slice of the window).  Returns (src, dst) on src's device."""
    world = dist.get_world_size(group)
    home = src.device
    n = src.numel()
    oa, ob = owner_of(src, world), owner_of(dst, world)
    e = torch.arange(n, device=home)
    two = ob != oa
    dest = torch.cat([oa, ob[two]])
    idx = torch.cat([e, e[two]])
    order = torch.argsort(dest * max(n, 1) + idx)   # by destination, then by position in the slice
    idx = idx[order]
    counts = torch.bincount(dest, minlength=world)
    cdev = _comm_device(group, src)
    recv_counts = torch.empty_like(counts, device=cdev)
    dist.all_to_all_single(recv_counts, counts.to(cdev), group=group)
    sc, rc = counts.tolist(), recv_counts.tolist()
    rows = torch.stack([src[idx], dst[idx]], dim=1).contiguous().to(cdev)
    got = torch.empty((sum(rc), 2), dtype=src.dtype, device=cdev)
    dist.all_to_all_single(got, rows, rc, sc, group=group)
    got = got.to(home)
    return got[:, 0].contiguous(), got[:, 1].contiguous()


def candidates_window(candidates_part, src, dst, group=None):
    """applyOnNeighbors(GenerateCandidateEdges) over a window spread over the ranks:
    edges routed to the owners of their endpoints, then each rank emits the candidate records of the
    vertices it owns -- candidates_part(src, dst, nparts, part) -> (a, b, is_candidate), e.g.
    Engine.candidates (gs_window_candidates_part).  The union over ranks is the whole window's output;
    no candidate pair crosses ranks."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    rs, rd = route_edges_to_owners(src, dst, group) if world > 1 else (src, dst)
    return candidates_part(rs, rd, world, rank)


def engine_halves(eng):
    """The Engine's partials / merge entry points in the shape reduce_window / fold_degree_max_window take."""
    return (eng.reduce_partials, eng.merge_partials, eng.fold_degree_max_partials, eng.merge_degree_max_partials)


def gather_window(src: torch.Tensor, dst: torch.Tensor, group=None):
    """All-gather every rank's slice of the window, in rank order (= stream order when rank r holds the
    r-th slice).  Variable slice sizes: gather the sizes, pad to the largest, trim after."""
    world = dist.get_world_size(group)
    n = torch.tensor([src.numel()], dtype=torch.int64, device=src.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x) for x in sizes]
    mx = max(sizes)
    pad = lambda t: torch.cat([t, t.new_zeros(mx - t.numel())]) if t.numel() < mx else t
    outs = []
    for col in (src, dst):
        buf = [col.new_empty(mx) for _ in range(world)]
        dist.all_gather(buf, pad(col.contiguous()), group=group)
        outs.append(torch.cat([b[:k] for b, k in zip(buf, sizes)]))
    return outs[0], outs[1]


def _exchange(t, send, recv, cdev, home, group):
    """all-to-all of a 1-D tensor: send[p] elements to rank p (in rank order), recv[p] from it"""
    out = torch.empty(sum(recv), dtype=t.dtype, device=cdev)
    dist.all_to_all_single(out, t[:sum(send)].contiguous().to(cdev), recv, send, group=group)
    return out.to(home)


TRI_MAX_BITS = 28   # gs_triangles.hip: the composite-key budget of one id


def relabel_window(src, dst, group=None):
    """Ids spanning more than 2^TRI_MAX_BITS values (any Long key, SimpleEdgeStream.java:173-183): the
    order-preserving compact ids of the WHOLE window -- every rank's distinct ids all-gathered, the
    sorted union G the same on every rank, each endpoint replaced by its rank in G (what
    gs_window_triangles_dist does inside the library).  Returns (src, dst, |G| - 1)."""
    mine = torch.unique(torch.cat([src, dst]))
    a, _ = gather_window(mine, mine, group)
    G = torch.unique(a)
    return torch.searchsorted(G, src), torch.searchsorted(G, dst), int(G.numel()) - 1


def triangles_window(eng, src, dst, group=None):
    """WindowTriangles over a window whose records are split across the ranks of `group` (SURVEY.md §8e,
    WindowTriangles.java:61-66).  The six steps of include/gelly_hip.h's gs_tri_dist_* with the
    collectives in torch.distributed: nothing of the raw window travels (unless it has self-loops):
      1. id range          all-reduce MIN / MAX
      2. raw degrees       all-reduce SUM of an int32[V]          (every rank renumbers identically)
      3. oriented edges    all-reduce SUM of their raw out-degrees int32[V]; all-to-all of 8-byte keys to
                           owner(u) (ranges of the degree order at equal shares of the raw work)
      4. out-lists         all-reduce SUM of d+ int32[V]; then the boundary adjacency: the rows of this
                           rank's equal-work count range (all-to-all, sizes from d+), the rows of their
                           targets it holds in neither range (all-to-all of ids, then of rows)
      5. count             each rank its equal-work share of the middle-vertex intersections; all-reduce
      6. self-pair term    only when the window has self-loops: gather the records, rank 0 adds it
    eng: an Engine on this rank's GPU; src, dst: this rank's records (device tensors).
    Returns (exact, Integer-wrapped, has_output), the same on every rank."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    home = src.device
    cdev = _comm_device(group, src)
    # an empty slice reports (INT64_MAX, INT64_MIN): reduce lo by MIN and hi by MAX directly (negating
    # INT64_MIN would overflow), so a rank with no records joins every collective like the others
    lo, hi = eng.tri_dist_range(src, dst)
    lo_t = torch.tensor([lo], dtype=torch.int64, device=cdev)
    hi_t = torch.tensor([hi], dtype=torch.int64, device=cdev)
    nt = torch.tensor([src.numel()], dtype=torch.int64, device=cdev)
    dist.all_reduce(lo_t, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi_t, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(nt, op=dist.ReduceOp.SUM, group=group)
    gmin, gmax, total = int(lo_t[0]), int(hi_t[0]), int(nt[0])
    if total == 0:
        return 0, 0, False
    osrc, odst = src, dst   # the self-pair term (step 6) needs the original ids: their HashSet order
    span_bits = max(1, ((gmin ^ gmax) & ((1 << 64) - 1)).bit_length())
    if span_bits > TRI_MAX_BITS or (span_bits > 20 and (1 << span_bits) > 8 * total):
        # (also when the id space is far sparser than the window: the per-id tables are all-reduced)
        src, dst, gmax = relabel_window(src, dst, group)
        gmin = 0
    deg = eng.tri_dist_degrees(src, dst, gmin, gmax)
    d = deg.to(cdev)
    dist.all_reduce(d, op=dist.ReduceOp.SUM, group=group)
    dout, loops = eng.tri_dist_orient(src, dst, d.to(home))
    do = dout.to(cdev)
    dist.all_reduce(do, op=dist.ReduceOp.SUM, group=group)
    keys, counts = eng.tri_dist_route(do.to(home), world)
    send = torch.tensor(counts, dtype=torch.int64, device=cdev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    rc = recv.tolist()
    rk = torch.empty(sum(rc), dtype=torch.int64, device=cdev)
    dist.all_to_all_single(rk, keys.to(cdev), rc, counts, group=group)
    lt = torch.tensor([loops], dtype=torch.int64, device=cdev)
    dist.all_reduce(lt, op=dist.ReduceOp.SUM, group=group)
    nbr, dplus = eng.tri_dist_build(rk.to(home), deg.numel())
    dp = dplus.to(cdev)
    dist.all_reduce(dp, op=dist.ReduceOp.SUM, group=group)
    dph = dp.to(home)
    # 4. boundary adjacency: the rows of this rank's count range, then the rows of their targets it holds
    #    in neither range (requested by id) -- not every rank's out-lists
    s1, r1, M = eng.tri_dist_plan(dph, rank, world)
    crows = _exchange(nbr, s1, r1, cdev, home, group)
    req, rc, re = eng.tri_dist_need(crows, world, deg.numel())
    mine = torch.tensor([x for pair in zip(rc, re) for x in pair], dtype=torch.int64, device=cdev)
    theirs = torch.empty_like(mine)
    dist.all_to_all_single(theirs, mine, group=group)
    qc, qe = theirs.view(-1, 2)[:, 0].tolist(), theirs.view(-1, 2)[:, 1].tolist()
    req_in = _exchange(req, rc, qc, cdev, home, group)
    rows, se = eng.tri_dist_serve(nbr, req_in, qc, qe)
    rows_in = _exchange(rows, se, re, cdev, home, group)
    full = eng.tri_dist_assemble(nbr, crows, rows_in, M)
    T = eng.tri_dist_count(full, dph, rank, world)
    if int(lt[0]):
        fs, fd = gather_window(osrc, odst, group)
        if rank == 0:
            T += eng.triangles_selfpair(fs, fd)
    t = torch.tensor([T], dtype=torch.int64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    total_t = int(t.item()) & ((1 << 64) - 1)
    wrapped = total_t & 0xFFFFFFFF
    return total_t, wrapped - (1 << 32) if wrapped >= (1 << 31) else wrapped, True
