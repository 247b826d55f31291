"""Multi-GPU window: keyBy(vertex) across ranks with one RCCL all-to-all.

The reference partitions each window by `keyBy(NeighborKeySelector)` (SimpleEdgeStream.java:159-167):
every record travels to the subtask that owns its key, which folds it.  Here every rank first
pre-reduces its own slice of the window on its GPU (sort + segmented reduce, associative ops only),
then the per-vertex partials — far fewer than records — are exchanged once:

  1. local:   (keys, partials) = engine.reduce(slice)            keys ascending
  2. owners:  vertex-range partition of [global min, global max] (all_reduce of 2 int64)
              -> each owner's partials are a contiguous slice of the sorted local output
  3. shuffle: all_to_all_single of counts, then of keys and partials (RCCL over xGMI)
  4. merge:   engine.reduce(received keys, partials) with the merge op (COUNT merges by SUM)

Which rank owns a vertex is not observable in the reference's output (per-vertex records compared
as unordered sets), so the range owner replaces Flink's hash owner.  Integer results stay bit-exact
(the ops are associative and commutative); float sums move within the 1e-5 tolerance.
`local_reduce` is injectable so the same exchange logic is exercised on CPU with gloo in tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

SUM, MIN, MAX, COUNT = 0, 1, 2, 3


def merge_op(op: int) -> int:
    return SUM if op == COUNT else op


def owner_bounds(kmin: int, kmax: int, world: int) -> list:
    """Split [kmin, kmax] into `world` contiguous vertex ranges; returns world-1 interior bounds."""
    span = kmax - kmin + 1
    return [kmin + (span * r) // world for r in range(1, world)]


def exchange_sorted(keys: torch.Tensor, cols: list, group=None):
    """Send each owner its slice of (keys, *cols); keys must be ascending.  Returns received tensors."""
    world = dist.get_world_size(group)
    dev = keys.device
    if keys.numel():
        mm = torch.stack([keys[-1], -keys[0]]).to(torch.int64)
    else:
        mm = torch.tensor([-(1 << 63), -(1 << 63)], dtype=torch.int64, device=dev)
    dist.all_reduce(mm, op=dist.ReduceOp.MAX, group=group)
    mx = mm.tolist()
    kmax, kmin = mx[0], -mx[1]
    if kmax < kmin:   # no rank has a vertex in this window
        return keys[:0], [c[:0] for c in cols]
    bounds = torch.tensor(owner_bounds(kmin, kmax, world), dtype=torch.int64, device=dev)
    cuts = torch.searchsorted(keys, bounds, right=False) if world > 1 else bounds
    edges = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), cuts,
                       torch.full((1,), keys.numel(), dtype=torch.int64, device=dev)])
    send = (edges[1:] - edges[:-1]).to(torch.int64)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    sr = torch.cat([send, recv]).tolist()   # one host read for both
    send_l, recv_l = sr[:world], sr[world:]
    total = sum(recv_l)
    # keys travel as 32-bit offsets from the global minimum when the window's span allows (12-byte
    # instead of 16-byte rows for a Long partial)
    narrow = kmax - kmin < (1 << 32)
    kpart = (keys - kmin).to(torch.int32) if narrow else keys.contiguous()
    # one all-to-all of packed rows (key bytes, then each column's bytes) instead of one per column:
    # fewer collective launches and one rendezvous per window
    parts = [kpart] + [c.contiguous() for c in cols]
    widths = [p.element_size() for p in parts]
    row = sum(widths)
    packed = torch.cat([p.view(torch.uint8).view(-1, w) for p, w in zip(parts, widths)], dim=1)
    rp = torch.empty((total, row), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(rp, packed, recv_l, send_l, group=group)
    out, at = [], 0
    for p, w in zip(parts, widths):
        out.append(rp[:, at:at + w].contiguous().view(p.dtype).view(-1))
        at += w
    rk = ((out[0].to(torch.int64) & 0xFFFFFFFF) + kmin) if narrow else out[0]
    return rk, out[1:]


def reduce_window(local_reduce, src, dst, val, direction: int, op: int, group=None):
    """reduceOnEdges over a window whose edges are spread over the ranks of `group`.
    Returns this rank's owned (vertex, value) pairs, vertices ascending."""
    k, v = local_reduce(src, dst, val, direction, op)
    if dist.get_world_size(group) == 1:   # the only rank owns every vertex: no exchange, no merge
        return k, v
    rk, (rv,) = exchange_sorted(k, [v], group)
    if rk.numel() == 0:
        return rk, rv
    return local_reduce(rk, rk, rv, 1, merge_op(op))


def fold_degree_max_window(local_fold, local_reduce, src, dst, direction: int, init_max: int, group=None):
    """foldNeighbors(degree, max-neighbour) across ranks: degrees merge by SUM, maxima by MAX."""
    k, d, m = local_fold(src, dst, direction, init_max)
    if dist.get_world_size(group) == 1:
        return k, d, m
    rk, (rd, rm) = exchange_sorted(k, [d, m], group)
    if rk.numel() == 0:
        return rk, rd, rm
    k1, d1 = local_reduce(rk, rk, rd, 1, SUM)
    _, m1 = local_reduce(rk, rk, rm, 1, MAX)
    return k1, d1, m1


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


def triangles_window(local_part_count, src, dst, group=None):
    """WindowTriangles over a window spread across ranks: all-gather the adjacency,
    count this rank's share of the oriented edges, all-reduce(SUM).  Returns (exact, Integer-wrapped)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    fs, fd = gather_window(src, dst, group)
    part = local_part_count(fs, fd, rank, world)
    t = torch.tensor([part], dtype=torch.int64, device=src.device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    total = int(t.item()) & ((1 << 64) - 1)
    wrapped = total & 0xFFFFFFFF
    return total, wrapped - (1 << 32) if wrapped >= (1 << 31) else wrapped
