"""ctypes wrapper of oracle/liboracle.so — the CPU restatement of gelly-streaming's window path.

TEST INFRASTRUCTURE ONLY (see gs_oracle.c).  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product package gelly-streaming_amd.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"

DIR_IN, DIR_OUT, DIR_ALL = 0, 1, 2
OP_SUM, OP_MIN, OP_MAX, OP_COUNT = 0, 1, 2, 3
DT_I32, DT_I64, DT_F32, DT_F64, DT_NONE = 0, 1, 2, 3, 4
NP_OF_DT = {DT_I32: np.int32, DT_I64: np.int64, DT_F32: np.float32, DT_F64: np.float64}
DT_OF_NP = {np.dtype(v): k for k, v in NP_OF_DT.items()}

_lib = None


def build() -> Path:
    import subprocess

    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        P = ctypes.c_void_p
        u64, i64, i32, u32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
        sig = {
            "gso_splitmix64": (u64, [u64, u64]),
            "gso_gen_rmat": (None, [i32, u64, u64, u32, u32, u32, i32, i32, u64, P, P]),
            "gso_gen_uniform": (None, [u64, u64, u64, u64, P, P]),
            "gso_gen_values": (None, [u64, u64, u64, i32, P]),
            "gso_window_reduce": (i64, [P, P, P, u64, i32, i32, i32, P, P, u64]),
            "gso_window_fold": (i64, [P, P, P, u64, i32, i32, i32, P, P, P, u64]),
            "gso_window_fold_degree_max": (i64, [P, P, u64, i32, i64, P, P, P, u64]),
            "gso_window_csr": (i64, [P, P, P, u64, i32, i32, P, P, P, P, u64]),
            "gso_window_candidates": (i64, [P, P, u64, P, P, P, u64, P]),
            "gso_candidates_mt": (i64, [P, P, u64, i32, u64, P]),
            "gso_window_triangles_ref": (ctypes.c_int32, [P, P, u64, P, P, P]),
            "gso_window_triangles_fwd": (ctypes.c_int32, [P, P, u64, P, P]),
            "gso_baseline_reduce": (u64, [P, P, P, u64, i32, i32, i32, i32]),
            "gso_java_hashset_cap": (u64, [u64]),
            "gso_hashset_order": (i32, [P, u64, P, P]),
            "gso_parse_edges_text": (i64, [ctypes.c_char_p, u64, P, P, P, u64]),
            "gso_java_long_bucket": (u32, [i64, u64]),
            "gso_zipf_cdf": (None, [u64, ctypes.c_double, P]),
            "gso_gen_zipf": (i32, [u64, ctypes.c_double, u64, u64, u64, P, P]),
            "gso_window_fold_mt": (i64, [P, P, P, u64, i32, i32, i32, i32, P, i64, i32, P, P, P, u64]),
            "gso_triangles_fwd_mt": (i32, [P, P, u64, i32, ctypes.POINTER(u64)]),
            "gso_components": (i64, [P, P, u64, P, P, u64, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


# ---- generators --------------------------------------------------------------------------
def fx32(p: float) -> int:
    return int(p * 4294967296.0)


def gen_rmat(scale, n, seed, a=0.57, b=0.19, c=0.19, permute=True, no_self_loops=False, first_edge=0):
    src = np.empty(n, np.int64)
    dst = np.empty(n, np.int64)
    lib().gso_gen_rmat(scale, n, seed, fx32(a), fx32(b), fx32(c), int(permute), int(no_self_loops),
                       first_edge, _p(src), _p(dst))
    return src, dst


def gen_uniform(num_vertices, n, seed, first_edge=0):
    src = np.empty(n, np.int64)
    dst = np.empty(n, np.int64)
    lib().gso_gen_uniform(num_vertices, n, seed, first_edge, _p(src), _p(dst))
    return src, dst


def gen_values(n, seed, dtype=DT_I64, first_edge=0):
    v = np.empty(n, NP_OF_DT[dtype])
    lib().gso_gen_values(n, seed, first_edge, dtype, _p(v))
    return v


def gen_zipf(num_vertices, n, seed, exponent=1.1, first_edge=0):
    """Zipf(exponent) sources over [0, num_vertices) (hubs at the lowest IDs), uniform destinations."""
    src = np.empty(n, np.int64)
    dst = np.empty(n, np.int64)
    assert lib().gso_gen_zipf(num_vertices, exponent, n, seed, first_edge, _p(src), _p(dst)) == 0
    return src, dst


def zipf_cdf(num_vertices, exponent=1.1):
    cdf = np.empty(num_vertices, np.uint64)
    lib().gso_zipf_cdf(num_vertices, exponent, _p(cdf))
    return cdf


# ---- window operators ----------------------------------------------------------------------
def _nrec(n, d):
    return 2 * n if d == DIR_ALL else n


def window_reduce(src, dst, val, direction, op):
    src, dst = _i64(src), _i64(dst)
    val = np.ascontiguousarray(val)
    dt = DT_OF_NP[val.dtype]
    cap = _nrec(len(src), direction) + 1
    keys = np.empty(cap, np.int64)
    out = np.empty(cap, np.int64 if op == OP_COUNT else val.dtype)
    u = lib().gso_window_reduce(_p(src), _p(dst), _p(val), len(src), dt, direction, op, _p(keys), _p(out), cap)
    assert u >= 0
    return keys[:u], out[:u]


def window_fold(src, dst, val, direction, op, init):
    src, dst = _i64(src), _i64(dst)
    val = np.ascontiguousarray(val)
    dt = DT_OF_NP[val.dtype]
    cap = _nrec(len(src), direction) + 1
    keys = np.empty(cap, np.int64)
    odt = np.int64 if op == OP_COUNT else val.dtype
    out = np.empty(cap, odt)
    init_a = np.array([init], dtype=odt)
    u = lib().gso_window_fold(_p(src), _p(dst), _p(val), len(src), dt, direction, op, _p(init_a), _p(keys),
                              _p(out), cap)
    assert u >= 0
    return keys[:u], out[:u]


def window_fold_degree_max(src, dst, direction, init_max=np.iinfo(np.int64).min):
    src, dst = _i64(src), _i64(dst)
    cap = _nrec(len(src), direction) + 1
    keys, deg, mx = (np.empty(cap, np.int64) for _ in range(3))
    u = lib().gso_window_fold_degree_max(_p(src), _p(dst), len(src), direction, init_max, _p(keys), _p(deg),
                                         _p(mx), cap)
    assert u >= 0
    return keys[:u], deg[:u], mx[:u]


def window_csr(src, dst, val, direction):
    src, dst = _i64(src), _i64(dst)
    R = _nrec(len(src), direction)
    dt = DT_NONE if val is None else DT_OF_NP[np.asarray(val).dtype]
    val = None if val is None else np.ascontiguousarray(val)
    keys = np.empty(R + 1, np.int64)
    offs = np.empty(R + 2, np.uint64)
    nbrs = np.empty(R + 1, np.int64)
    vals = None if val is None else np.empty(R + 1, val.dtype)
    u = lib().gso_window_csr(_p(src), _p(dst), _p(val), len(src), dt, direction, _p(keys), _p(offs), _p(nbrs),
                             _p(vals), R + 1)
    assert u >= 0
    return keys[:u], offs[: u + 1].astype(np.int64), nbrs[:R], (None if vals is None else vals[:R])


def window_candidates(src, dst):
    src, dst = _i64(src), _i64(dst)
    tree = ctypes.c_int(0)
    need = lib().gso_window_candidates(_p(src), _p(dst), len(src), None, None, None, 0, ctypes.byref(tree))
    P = -1 - need if need < 0 else need
    a, b = np.empty(P, np.int64), np.empty(P, np.int64)
    f = np.empty(P, np.uint8)
    got = lib().gso_window_candidates(_p(src), _p(dst), len(src), _p(a), _p(b), _p(f), P, ctypes.byref(tree))
    assert got == P
    return a, b, f, int(tree.value)   # JDK flags of hashset_order (nonzero: some set left the plain model)


def candidates_mt(src, dst, threads=None, chunk=1 << 20):
    """GenerateCandidateEdges over `threads` threads with a consumer that reads every chunk of `chunk`
    records back (column sums): (records, [sum a, sum b, sum flags]) -- bench.py's C5 cpu_baseline."""
    src, dst = _i64(src), _i64(dst)
    sums = np.zeros(3, np.uint64)
    n = lib().gso_candidates_mt(_p(src), _p(dst), len(src), threads or default_threads(), chunk, _p(sums))
    if n < 0:
        raise ValueError("gso_candidates_mt failed")
    return int(n), [int(x) for x in sums]


def candidate_count(src, dst):
    """Number of GenerateCandidateEdges records the window emits (the size query of gso_window_candidates)."""
    src, dst = _i64(src), _i64(dst)
    tree = ctypes.c_int(0)
    need = lib().gso_window_candidates(_p(src), _p(dst), len(src), None, None, None, 0, ctypes.byref(tree))
    return -1 - need if need < 0 else need


def parse_edges_text(text: bytes):
    """"src trg ts" records (example/WindowTriangles.java:175-185, gso_parse_edges_text) -> int64 columns.
    Raises ValueError(index of the first malformed record) where the reference's map throws."""
    n = lib().gso_parse_edges_text(text, len(text), None, None, None, 0)
    if n < 0:
        raise ValueError(f"malformed edge record {-1 - n}")
    s, d, t = np.empty(n, np.int64), np.empty(n, np.int64), np.empty(n, np.int64)
    assert lib().gso_parse_edges_text(text, len(text), _p(s), _p(d), _p(t), n) == n
    return s, d, t


def count_candidates(a, b, is_candidate):
    """Stage 2 of WindowTriangles over one window's candidate records (example/WindowTriangles.java:64-66):
    keyBy(0, 1) groups by the ordered pair (a, b); CountTriangles.apply (:119-140) counts candidate
    (true) and edge (false) records and emits the candidate count iff edges > 0; timeWindowAll(..).sum(0)
    adds the emitted Integers (wrapping).  Returns (Integer sum, exact sum, has_output, emitted records)."""
    a, b = _i64(a), _i64(b)
    f = np.asarray(is_candidate) != 0
    if len(a) == 0:
        return 0, 0, False, 0
    pairs = np.stack([a, b], axis=1)
    _, inv = np.unique(pairs, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    cand = np.bincount(inv, weights=f.astype(np.int64)).astype(np.int64)
    edges = np.bincount(inv, weights=(~f).astype(np.int64)).astype(np.int64)
    emit = edges > 0
    exact = int(cand[emit].sum())
    w = exact & 0xFFFFFFFF
    return (w - (1 << 32) if w >= (1 << 31) else w), exact, bool(emit.any()), int(emit.sum())


def window_triangles_ref(src, dst):
    src, dst = _i64(src), _i64(dst)
    ex, has, tree = ctypes.c_uint64(0), ctypes.c_int(0), ctypes.c_int(0)
    w = lib().gso_window_triangles_ref(_p(src), _p(dst), len(src), ctypes.byref(ex), ctypes.byref(has),
                                       ctypes.byref(tree))
    return int(w), int(ex.value), bool(has.value), int(tree.value)


def window_triangles_fwd(src, dst):
    src, dst = _i64(src), _i64(dst)
    ex, has = ctypes.c_uint64(0), ctypes.c_int(0)
    w = lib().gso_window_triangles_fwd(_p(src), _p(dst), len(src), ctypes.byref(ex), ctypes.byref(has))
    return int(w), int(ex.value), bool(has.value)


def default_threads():
    """worker threads for the large-window restatements: this host's CPUs, at most 16 (the GPU box's
    CPU share per GPU)"""
    return max(1, min(16, os.cpu_count() or 1))


def window_reduce_mt(src, dst, val, direction, op, threads=None, init=None):
    """gso_window_fold_mt: the same results as window_reduce (init None) / window_fold, over threads
    (keyBy-style routing keeps every key's arrival order)."""
    src, dst = _i64(src), _i64(dst)
    val = np.ascontiguousarray(val)
    dt = DT_OF_NP[val.dtype]
    cap = _nrec(len(src), direction) + 1
    keys = np.empty(cap, np.int64)
    odt = np.int64 if op == OP_COUNT else val.dtype
    out = np.empty(cap, odt)
    mode, ia = (0, None) if init is None else (1, np.array([init], dtype=odt))
    u = lib().gso_window_fold_mt(_p(src), _p(dst), _p(val), len(src), dt, direction, op, mode, _p(ia), 0,
                                 threads or default_threads(), _p(keys), _p(out), None, cap)
    assert u >= 0, u
    return keys[:u], out[:u]


def window_fold_degree_max_mt(src, dst, direction, init_max=np.iinfo(np.int64).min, threads=None):
    src, dst = _i64(src), _i64(dst)
    cap = _nrec(len(src), direction) + 1
    keys, deg, mx = (np.empty(cap, np.int64) for _ in range(3))
    dummy = np.zeros(1, np.int64)
    u = lib().gso_window_fold_mt(_p(src), _p(dst), _p(dummy), len(src), DT_I64, direction, OP_COUNT, 2, None,
                                 int(init_max), threads or default_threads(), _p(keys), _p(deg), _p(mx), cap)
    assert u >= 0, u
    return keys[:u], deg[:u], mx[:u]


def triangles_fwd_mt(src, dst, threads=None):
    """Exact triangle count of a self-loop-free window (forward algorithm over compacted IDs)."""
    src, dst = _i64(src), _i64(dst)
    t = ctypes.c_uint64(0)
    rc = lib().gso_triangles_fwd_mt(_p(src), _p(dst), len(src), threads or default_threads(), ctypes.byref(t))
    if rc != 0:
        raise ValueError("triangles_fwd_mt: the window has a self-loop")
    return int(t.value)


def baseline_reduce(src, dst, val, direction, op, threads):
    src, dst = _i64(src), _i64(dst)
    val = np.ascontiguousarray(val)
    return int(lib().gso_baseline_reduce(_p(src), _p(dst), _p(val), len(src), DT_OF_NP[val.dtype], direction, op,
                                         threads))


# ---- stream helpers: tumbling event-time windows (Flink 1.0.3 TumblingEventTimeWindows) -------
def window_start(ts, size):
    """start = ts - ts % size with Java's truncated remainder."""
    ts = np.asarray(ts, dtype=np.int64)
    return ts - np.fmod(ts, size)


def split_windows(ts, size):
    """[(start, index array)] in ascending window order; records keep their arrival order."""
    st = window_start(ts, size)
    order = np.argsort(st, kind="stable")
    starts, first = np.unique(st[order], return_index=True)
    bounds = list(first) + [len(order)]
    return [(int(s), order[bounds[i]:bounds[i + 1]]) for i, s in enumerate(starts)]


def java_hashset_cap(k):
    return int(lib().gso_java_hashset_cap(k))


def components(src, dst, prev=None):
    """ConnectedComponents after one window (gso_components): the running state `prev` = (vertices,
    labels) or None, merged with the window's edges -> (vertices ascending, smallest vertex of each one's
    component)."""
    src, dst = _i64(src), _i64(dst)
    pv, pl = (np.empty(0, np.int64), np.empty(0, np.int64)) if prev is None else (_i64(prev[0]), _i64(prev[1]))
    cap = 2 * len(src) + 2 * len(pv) + 1
    ov, ol = np.empty(cap, np.int64), np.empty(cap, np.int64)
    u = lib().gso_components(_p(src), _p(dst), len(src), _p(pv), _p(pl), len(pv), _p(ov), _p(ol))
    return ov[:u].copy(), ol[:u].copy()


def hashset_order(ids):
    """java.util.HashSet<Long> built by add() of `ids` (distinct, arrival order) -> (iteration order of the
    exact JDK 8+ HashMap simulation, the plain-bin model's order, flags: 1 = a bin treeified,
    2 = a collision resize below capacity 64)."""
    ids = _i64(ids)
    ex, pl = np.empty(len(ids) + 1, np.int64), np.empty(len(ids) + 1, np.int64)
    f = lib().gso_hashset_order(_p(ids), len(ids), _p(ex), _p(pl))
    return ex[:len(ids)].copy(), pl[:len(ids)].copy(), int(f)
