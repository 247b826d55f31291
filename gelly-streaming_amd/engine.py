"""Engine: one gs_ctx (one HIP stream + workspace) driving the per-window operators.

Inputs are either device tensors (torch, on the ctx's GPU: zero-copy, results stay in HBM) or host
numpy arrays (copied in by the library, results copied back).  One Engine per thread, like one
gs_ctx per Flink subtask (include/gelly_hip.h, "Conventions").
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from ._lib import GsError


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _ptr(x):
    if x is None:
        return None
    if _is_torch(x):
        return ctypes.c_void_p(x.data_ptr())
    return ctypes.c_void_p(x.ctypes.data)


def _gs_dtype(x) -> int:
    if x is None:
        return L.GS_NONE
    if _is_torch(x):
        import torch

        return {torch.int32: L.GS_I32, torch.int64: L.GS_I64, torch.float32: L.GS_F32,
                torch.float64: L.GS_F64}[x.dtype]
    return L.GS_DTYPE_OF[np.dtype(x.dtype)]


def fx32(p: float) -> int:
    """probability -> 32-bit fixed point, as gs_generate_rmat / oracle take it"""
    return int(p * 4294967296.0)


@dataclass
class StageTimes:
    keyinfo_ms: float
    sort_ms: float
    reduce_ms: float
    total_ms: float
    sort_passes: int
    key_bits: int
    records: int
    vertices: int
    pass_ms: list
    key_bytes: int
    payload_bytes: int
    partials: int
    fused_last: bool
    path: int = 0          # 0: LSD sort + reduce-by-key; 1: bucket path, onesweep partition (pass_ms = passes,
                           # accumulate, merge, emit); 2: bucket path, direct partition (pass_ms = offset scans,
                           # scatter, accumulate, merge, emit; keyinfo_ms = per-tile histogram); 3: triangles
                           # (ranks + keys + sort, unique, out-lists + transposed sort, light, heavy); 4: connected
                           # components (compact IDs, union-find, labels)
    packed: bool = False   # path 2: 4-byte packed partition records (k_dp_scatter_pack)
    escapes: int = 0       # path 2, packed: values stored in full
    speculative: int = 0   # path 2: 1 = regions from the previous window's counts, 2 = that missed


class CommGroup:
    """gs_comm_group: P ranks in this process (one Engine per rank, e.g. P ranks on one GPU); the
    gs_window_*_dist orchestration runs over it exactly as over RCCL (include/gelly_hip.h)."""

    def __init__(self, nranks: int):
        self._L = L.load()
        h = ctypes.c_void_p()
        st = self._L.gs_comm_group_create(int(nranks), ctypes.byref(h))
        if st != L.GS_OK:
            raise GsError(st, f"gs_comm_group_create({nranks}) failed")
        self.handle = h
        self.nranks = nranks

    def close(self):
        if getattr(self, "handle", None):
            self._L.gs_comm_group_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_OUT_DTYPES = None


def _out_dtypes():
    """numpy -> torch dtype of the out= buffers (built once: Engine._check_out runs between windows)"""
    global _OUT_DTYPES
    if _OUT_DTYPES is None:
        import torch

        _OUT_DTYPES = {np.int64: torch.int64, np.int32: torch.int32, np.float32: torch.float32,
                       np.float64: torch.float64}
    return _OUT_DTYPES


class Engine:
    def __init__(self, device: int = 0, reserve_edges: int = 0, torch_stream: bool = True, sort_only: bool = False,
                 bk_onesweep: bool = False, no_pack: bool = False, no_spec: bool = False, flags: int = 0,
                 async_outputs: bool = True):
        """torch_stream: the library runs on torch's current stream (its tensors are ordered with our kernels).
        async_outputs (with torch_stream): reduce / fold / fold_degree_max into device tensors return as soon
        as the window's sizes are known; the last kernel may still be writing the outputs, which torch work on
        the same stream sees complete (GS_FLAG_ASYNC_OUTPUT) -- switch torch streams only after synchronizing."""
        self._L = L.load()
        flags |= (L.GS_FLAG_SORT_ONLY if sort_only else 0) | (L.GS_FLAG_BK_ONESWEEP if bk_onesweep else 0) | \
            (L.GS_FLAG_NO_PACK if no_pack else 0) | (L.GS_FLAG_NO_SPEC if no_spec else 0) | \
            (L.GS_FLAG_ASYNC_OUTPUT if (torch_stream and async_outputs) else 0)
        cfg = L.GsConfig(device, flags, reserve_edges)
        ctx = ctypes.c_void_p()
        st = self._L.gs_create(ctypes.byref(cfg), ctypes.byref(ctx))
        if st != L.GS_OK:
            raise GsError(st, f"gs_create(device={device}) failed — a HIP device is required")
        self.ctx = ctx
        self.device = device
        if torch_stream:
            # share torch's current stream so tensors allocated by torch are ordered with our kernels
            self.use_torch_stream()

    # -- lifecycle -------------------------------------------------------------------------------
    def close(self):
        if getattr(self, "ctx", None):
            self._L.gs_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st: int):
        if st != L.GS_OK:
            raise GsError(st, self._L.gs_last_error(self.ctx).decode())

    def set_stream(self, hip_stream_ptr: int):
        """Run on an existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream; 0 = default stream)."""
        self._check(self._L.gs_set_stream(self.ctx, ctypes.c_void_p(hip_stream_ptr) if hip_stream_ptr else None))

    def set_timing(self, level: int):
        """gs_set_timing: which stage-time events a window records (L.GS_TIMING_OFF / _DOMINANT / _STAGES)."""
        self._check(self._L.gs_set_timing(self.ctx, int(level)))

    def use_torch_stream(self):
        import torch

        with torch.cuda.device(self.device):
            self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def set_max_window_records(self, max_records: int):
        """gs_set_max_window_records: records per engine pass; larger reduce / fold windows run in chunks
        merged through the partials halves (0 = the default, 2^32 - 1)."""
        self._check(self._L.gs_set_max_window_records(self.ctx, int(max_records)))

    def synchronize(self):
        self._check(self._L.gs_synchronize(self.ctx))

    def stage_times(self) -> StageTimes:
        return self.stage_times_of(self.stage_times_raw())

    def stage_times_raw(self):
        """The last window's gs_stage_times as the raw ctypes struct (a copy): cheap enough for a timed loop
        between windows; stage_times_of() turns it into StageTimes afterwards."""
        t = L.GsStageTimes()
        self._check(self._L.gs_last_stage_times(self.ctx, ctypes.byref(t)))
        return t

    @staticmethod
    def stage_times_of(t) -> StageTimes:
        if isinstance(t, StageTimes):
            return t
        launched = 5 if t.path in (2, 3) else 3 if t.path == 4 else \
            t.sort_passes + (3 if t.path == 1 else 1 if t.fused_last else 0)
        return StageTimes(t.keyinfo_ms, t.sort_ms, t.reduce_ms, t.total_ms, t.sort_passes, t.key_bits, t.records,
                          t.vertices, list(t.pass_ms)[:launched], t.key_bytes, t.payload_bytes,
                          t.partials, bool(t.fused_last), t.path, bool(t.packed), t.escapes, t.speculative)

    # -- helpers ---------------------------------------------------------------------------------
    def _batch(self, src, dst, val):
        dev = _is_torch(src)
        if dev:
            assert src.is_cuda and dst.is_cuda and (val is None or val.is_cuda), "mixed host/device columns"
            assert src.is_contiguous() and dst.is_contiguous() and (val is None or val.is_contiguous())
        else:
            src = np.ascontiguousarray(src, dtype=np.int64)
            dst = np.ascontiguousarray(dst, dtype=np.int64)
            if val is not None:
                val = np.ascontiguousarray(val)
        if len(src) != len(dst) or (val is not None and len(val) != len(src)):
            raise ValueError("src, dst and val must have the same length")
        b = L.GsEdgeBatch(_ptr(src), _ptr(dst), _ptr(val), len(src), _gs_dtype(val),
                          L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        return b, (src, dst, val), dev

    def _empty(self, like_dev: bool, n: int, np_dtype):
        if like_dev:
            import torch

            tdt = {np.int64: torch.int64, np.int32: torch.int32, np.float32: torch.float32,
                   np.float64: torch.float64, np.uint64: torch.int64, np.uint8: torch.uint8,
                   np.uint32: torch.uint32}[np_dtype]
            return torch.empty(max(n, 1), dtype=tdt, device=f"cuda:{self.device}")
        return np.empty(max(n, 1), dtype=np_dtype)

    @staticmethod
    def _records(n, direction):
        return 2 * n if int(direction) == 2 else n

    def _check_out(self, out, dev: bool, np_dtypes, min_records=None):
        """out= buffers: device tensors (with device inputs), contiguous, of the dtypes the library writes
        (it writes 8-byte keys and the op's value width at raw addresses: a narrower or strided tensor
        would take out-of-bounds or misplaced writes), and at least min_records long when given."""
        tdt = _out_dtypes()
        if len(out) != len(np_dtypes):
            raise ValueError(f"out: {len(np_dtypes)} tensors expected")
        for t, want in zip(out, np_dtypes):
            if not (dev and _is_torch(t) and t.is_cuda):
                raise ValueError("out: device tensors, with device inputs")
            if t.dtype != tdt[want]:
                raise ValueError(f"out: dtype {t.dtype}, the library writes {tdt[want]}")
            if not t.is_contiguous():
                raise ValueError("out: contiguous tensors")
            if min_records is not None and t.numel() < min_records:
                raise ValueError("out: device tensors of at least the window's records")

    # -- operators ------------------------------------------------------------------------------
    def reduce(self, src, dst, val, direction, op, out=None):
        """gs_window_reduce: reduceOnEdges with a built-in op. Returns (keys, values) trimmed to U.
        out: optional (keys, values) device tensors of at least the window's record count, reused across
        windows (a streaming operator's output buffers) instead of allocating per call."""
        return self._fold(src, dst, val, direction, op, None, out)

    def fold(self, src, dst, val, direction, op, init):
        """gs_window_fold: foldNeighbors(init, op). Returns (keys, values)."""
        return self._fold(src, dst, val, direction, op, init)

    # A streaming operator calls reduce with the same device columns and out= buffers window after window
    # (the bench cycles its windows): the ctypes arguments built for such a call are kept, keyed by the
    # tensors' identities and checked against their data pointers, so the next call goes straight to the
    # library -- the Python between two windows is GPU idle time.
    _ARGS_KEEP = 8

    def _fold(self, src, dst, val, direction, op, init, out=None):
        if init is None and out is not None and _is_torch(src):
            v = None if op == L.GS_OP_COUNT else val
            key = (id(src), id(dst), id(v), int(direction), int(op), id(out[0]), id(out[1]))
            ptrs = (src.data_ptr(), dst.data_ptr(), v.data_ptr() if v is not None else 0, out[0].data_ptr(),
                    out[1].data_ptr(), src.numel())
            args = getattr(self, "_args", None)
            if args is None:
                args = self._args = {}
            hit = args.get(key)
            if hit is None or hit[0] != ptrs:
                b, _, dev = self._batch(src, dst, v)
                R = self._records(b.n, direction)
                odt = np.int64 if op == L.GS_OP_COUNT else L.NP_DTYPE[b.val_dtype]
                self._check_out(out, dev, (np.int64, odt), R)
                n_out = ctypes.c_uint64(0)
                vo = L.GsVertexOut(_ptr(out[0]), _ptr(out[1]), R, ctypes.pointer(n_out), L.GS_MEM_DEVICE, 0)
                if len(args) >= self._ARGS_KEEP:
                    args.pop(next(iter(args)))
                # (the tensors are held: their ids stay theirs while the entry lives)
                hit = args[key] = (ptrs, ctypes.byref(b), ctypes.byref(vo), n_out, (b, vo, src, dst, v, out))
            self._check(self._L.gs_window_reduce(self.ctx, hit[1], int(direction), int(op), hit[2]))
            U = hit[3].value
            return out[0][:U], out[1][:U]
        b, keep, dev = self._batch(src, dst, None if op == L.GS_OP_COUNT else val)
        R = self._records(b.n, direction)
        odt = np.int64 if op == L.GS_OP_COUNT else L.NP_DTYPE[b.val_dtype]
        if out is not None:
            self._check_out(out, dev, (np.int64, odt), R)
            keys, vals = out
        else:
            keys = self._empty(dev, R, np.int64)
            vals = self._empty(dev, R, odt)
        n_out = ctypes.c_uint64(0)
        out = L.GsVertexOut(_ptr(keys), _ptr(vals), R, ctypes.pointer(n_out),
                            L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        if init is None:
            st = self._L.gs_window_reduce(self.ctx, ctypes.byref(b), int(direction), int(op), ctypes.byref(out))
        else:
            ia = np.array([init], dtype=odt)
            st = self._L.gs_window_fold(self.ctx, ctypes.byref(b), int(direction), int(op),
                                        ia.ctypes.data_as(ctypes.c_void_p), ctypes.byref(out))
        self._check(st)
        U = n_out.value
        return keys[:U], vals[:U]

    def fold_degree_max(self, src, dst, direction, init_max: int = -(1 << 63), out=None):
        """gs_window_fold_degree_max: (keys, degrees, max neighbours).  out: optional (keys, degrees, maxima)
        device tensors of at least the window's records, reused across windows."""
        b, keep, dev = self._batch(src, dst, None)
        R = self._records(b.n, direction)
        if out is not None:
            self._check_out(out, dev, (np.int64, np.int64, np.int64), R)
            keys, deg, mx = out
        else:
            keys, deg, mx = (self._empty(dev, R, np.int64) for _ in range(3))
        n_out = ctypes.c_uint64(0)
        out = L.GsDegreeOut(_ptr(keys), _ptr(deg), _ptr(mx), R, ctypes.pointer(n_out),
                            L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_window_fold_degree_max(self.ctx, ctypes.byref(b), int(direction), int(init_max),
                                                      ctypes.byref(out)))
        U = n_out.value
        return keys[:U], deg[:U], mx[:U]

    def csr(self, src, dst, val, direction):
        """gs_window_csr: (keys, offsets[U+1], neighbours[R], values[R] or None), arrival order per vertex."""
        b, keep, dev = self._batch(src, dst, val)
        R = self._records(b.n, direction)
        keys = self._empty(dev, R, np.int64)
        offs = self._empty(dev, R + 1, np.int64)
        nbrs = self._empty(dev, R, np.int64)
        vals = None if val is None else self._empty(dev, R, L.NP_DTYPE[b.val_dtype])
        nv, nr = ctypes.c_uint64(0), ctypes.c_uint64(0)
        out = L.GsCsrOut(_ptr(keys), _ptr(offs), _ptr(nbrs), _ptr(vals), R, R, ctypes.pointer(nv),
                         ctypes.pointer(nr), L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_window_csr(self.ctx, ctypes.byref(b), int(direction), ctypes.byref(out)))
        U, RR = nv.value, nr.value
        return keys[:U], offs[:U + 1], nbrs[:RR], (None if vals is None else vals[:RR])

    def candidates(self, src, dst, nparts: int = 1, part: int = 0):
        """gs_window_candidates: GenerateCandidateEdges records (a, b, is_candidate), ids in exact JDK
        HashSet order.  self.last_candidates_jdk_flags: bit 0 = some neighbour set used a treeified
        HashMap bin, bit 1 = a bin of 9 forced a resize below capacity 64 (both simulated exactly).
        nparts > 1: gs_window_candidates_part, only the vertices gs_owner_of assigns to `part`."""
        b, keep, dev = self._batch(src, dst, None)
        n_out = ctypes.c_uint64(0)
        call = lambda o: self._L.gs_window_candidates_part(self.ctx, ctypes.byref(b), nparts, part, ctypes.byref(o))
        probe = L.GsPairOut(None, None, None, 0, ctypes.pointer(n_out), L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        st = call(probe)
        if st not in (L.GS_OK, L.GS_ECAPACITY):
            self._check(st)
        P = n_out.value
        a, bb = self._empty(dev, P, np.int64), self._empty(dev, P, np.int64)
        f = self._empty(dev, P, np.uint8)
        out = L.GsPairOut(_ptr(a), _ptr(bb), _ptr(f), P, ctypes.pointer(n_out),
                          L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(call(out))
        self.last_candidates_jdk_flags = int(out.reserved)
        return a[:P], bb[:P], f[:P]

    def candidates_begin(self, src, dst, nparts: int = 1, part: int = 0) -> int:
        """gs_candidates_begin (gs_candidates_begin_part with nparts > 1: only part's vertices emit): build
        the window's HashSet-ordered sets once; returns the record count.  The columns must stay alive (and
        unchanged) until the session's last candidates_next."""
        b, keep, dev = self._batch(src, dst, None)
        total, fl = ctypes.c_uint64(0), ctypes.c_uint32(0)
        if nparts == 1:
            st = self._L.gs_candidates_begin(self.ctx, ctypes.byref(b), ctypes.byref(total), ctypes.byref(fl))
        else:
            st = self._L.gs_candidates_begin_part(self.ctx, ctypes.byref(b), int(nparts), int(part), ctypes.byref(total),
                                                  ctypes.byref(fl))
        self._check(st)
        self._cand_dev = dev
        self.last_candidates_jdk_flags = int(fl.value)
        return total.value

    def candidates_next(self, capacity: int, out=None):
        """gs_candidates_next: the next <= capacity records (a, b, is_candidate) of the session, the global
        position of the first and whether the session is done.  out: optional (a, b, f) buffers to fill."""
        dev = self._cand_dev
        if out is None:
            out = (self._empty(dev, capacity, np.int64), self._empty(dev, capacity, np.int64),
                   self._empty(dev, capacity, np.uint8))
        a, bb, f = out
        n_out, first, done = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_int32(0)
        o = L.GsPairOut(_ptr(a), _ptr(bb), _ptr(f), capacity, ctypes.pointer(n_out),
                        L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_candidates_next(self.ctx, ctypes.byref(o), ctypes.byref(first), ctypes.byref(done)))
        n = n_out.value
        return a[:n], bb[:n], f[:n], first.value, bool(done.value)

    def candidates_next_u32(self, capacity: int, out=None):
        """gs_candidates_next_u32: the next <= capacity records with the ids as uint32 columns relative to the
        window's smallest id.  Returns (a32, b32, is_candidate, first position, done, id_base): a = id_base +
        a32.  Raises GsError (GS_EUNSUPPORTED) when the window's ids span more than 2^32 values."""
        dev = self._cand_dev
        if out is None:
            out = (self._empty(dev, capacity, np.uint32), self._empty(dev, capacity, np.uint32),
                   self._empty(dev, capacity, np.uint8))
        a, bb, f = out
        n_out, first, done, base = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_int32(0), ctypes.c_int64(0)
        o = L.GsPairOutU32(_ptr(a), _ptr(bb), _ptr(f), capacity, ctypes.pointer(n_out),
                           L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_candidates_next_u32(self.ctx, ctypes.byref(o), ctypes.byref(base), ctypes.byref(first),
                                                   ctypes.byref(done)))
        n = n_out.value
        return a[:n], bb[:n], f[:n], first.value, bool(done.value), base.value

    def candidates_seek(self, record: int):
        """gs_candidates_seek: the session's next chunk starts at output position `record`."""
        self._check(self._L.gs_candidates_seek(self.ctx, int(record)))

    def candidates_vertex_range(self, vertex: int):
        """gs_candidates_vertex_range: (first position, record count) of one vertex's block in the session."""
        first, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._check(self._L.gs_candidates_vertex_range(self.ctx, int(vertex), ctypes.byref(first), ctypes.byref(n)))
        return first.value, n.value

    def candidate_count(self, src, dst) -> int:
        """Sizing call of gs_window_candidates (capacity 0): the number of records the window emits."""
        b, keep, dev = self._batch(src, dst, None)
        n_out = ctypes.c_uint64(0)
        probe = L.GsPairOut(None, None, None, 0, ctypes.pointer(n_out), L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        st = self._L.gs_window_candidates(self.ctx, ctypes.byref(b), ctypes.byref(probe))
        if st not in (L.GS_OK, L.GS_ECAPACITY):
            self._check(st)
        return n_out.value

    def count_candidates(self, a, b, is_candidate):
        """gs_window_count_candidates: WindowTriangles stage 2 (keyBy(0, 1) CountTriangles + sum(0)) over
        one window's candidate records.  Returns (exact, the Integer the reference emits, has_output,
        records CountTriangles emits)."""
        dev = _is_torch(a)
        if dev:
            import torch

            assert a.is_cuda and b.is_cuda and is_candidate.is_cuda, "mixed host/device columns"
            a, b = a.contiguous(), b.contiguous()
            f = (is_candidate != 0).to(torch.uint8)
        else:
            a = np.ascontiguousarray(a, dtype=np.int64)
            b = np.ascontiguousarray(b, dtype=np.int64)
            f = np.ascontiguousarray(np.asarray(is_candidate) != 0, dtype=np.uint8)
        if len(a) != len(b) or len(f) != len(a):
            raise ValueError("a, b and is_candidate must have the same length")
        pb = L.GsPairBatch(_ptr(a), _ptr(b), _ptr(f), len(a), L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        cnt, wrapped, has, groups = ctypes.c_uint64(0), ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_uint64(0)
        self._check(self._L.gs_window_count_candidates(self.ctx, ctypes.byref(pb), ctypes.byref(cnt),
                                                       ctypes.byref(wrapped), ctypes.byref(has), ctypes.byref(groups)))
        return cnt.value, wrapped.value, bool(has.value), groups.value

    def parse_edges_text(self, text, out_device: bool = True):
        """gs_parse_edges_text: "src trg ts" records -> (src, dst, ts) int64 columns (WindowTriangles.java:175-185).
        `text`: bytes / numpy uint8 (host) or a uint8 CUDA tensor.  Malformed records raise GsError."""
        dev_in = _is_torch(text)
        if dev_in:
            assert text.is_cuda and text.dtype.itemsize == 1, "text must be a uint8 CUDA tensor"
            text = text.contiguous()
            ptr, nbytes = text.data_ptr(), text.numel()
        else:
            buf = np.frombuffer(text, dtype=np.uint8) if isinstance(text, (bytes, bytearray)) else \
                np.ascontiguousarray(text, dtype=np.uint8)
            text = buf
            ptr, nbytes = (buf.ctypes.data if buf.size else None), buf.size
        in_mem = L.GS_MEM_DEVICE if dev_in else L.GS_MEM_HOST
        n_out, bad = ctypes.c_uint64(0), ctypes.c_uint64(0)
        cap = nbytes // 6 + 1          # a record takes at least 6 bytes ("0 0 0\n"), the last one 5
        cols = [self._empty(out_device, cap, np.int64) for _ in range(3)]
        self._check(self._L.gs_parse_edges_text(self.ctx, ptr, nbytes, in_mem, _ptr(cols[0]), _ptr(cols[1]),
                                                _ptr(cols[2]), cap, L.GS_MEM_DEVICE if out_device else L.GS_MEM_HOST,
                                                ctypes.pointer(n_out), ctypes.pointer(bad)))
        n = n_out.value
        return tuple(c[:n] for c in cols)

    def triangles(self, src, dst):
        """gs_window_triangles: (exact count, the Integer the reference emits, has_output)."""
        b, keep, dev = self._batch(src, dst, None)
        cnt, wrapped, has = ctypes.c_uint64(0), ctypes.c_int32(0), ctypes.c_int32(0)
        self._check(self._L.gs_window_triangles(self.ctx, ctypes.byref(b), ctypes.byref(cnt), ctypes.byref(wrapped),
                                                ctypes.byref(has)))
        return cnt.value, wrapped.value, bool(has.value)

    def triangles_part(self, src, dst, part: int, nparts: int) -> int:
        """gs_window_triangles_part: this part's share of the window's triangle count (multi-GPU)."""
        b, keep, dev = self._batch(src, dst, None)
        cnt = ctypes.c_uint64(0)
        self._check(self._L.gs_window_triangles_part(self.ctx, ctypes.byref(b), part, nparts, ctypes.byref(cnt)))
        return cnt.value

    # -- WindowTriangles over a split window (gs_tri_dist_*, include/gelly_hip.h) -----------------------
    # Device tensors in and out; the caller runs the collective after each step (distributed.py).
    def tri_dist_range(self, src, dst):
        """Step 1: this rank's (min, max) id (all-reduce MIN / MAX across ranks)."""
        b, keep, dev = self._batch(src, dst, None)
        mm = (ctypes.c_int64 * 2)()
        self._check(self._L.gs_tri_dist_range(self.ctx, ctypes.byref(b), mm))
        return int(mm[0]), int(mm[1])

    def tri_dist_degrees(self, src, dst, gmin: int, gmax: int):
        """Step 2: this rank's raw degrees over the common id range, an int32 tensor [V] (all-reduce SUM)."""
        import torch

        b, keep, dev = self._batch(src, dst, None)
        V = ctypes.c_uint64(0)
        self._check(self._L.gs_tri_dist_degrees(self.ctx, ctypes.byref(b), int(gmin), int(gmax), None, ctypes.byref(V)))
        deg = torch.empty(V.value, dtype=torch.int32, device=f"cuda:{self.device}")
        self._check(self._L.gs_tri_dist_degrees(self.ctx, ctypes.byref(b), int(gmin), int(gmax), _ptr(deg),
                                                ctypes.byref(V)))
        return deg

    def tri_dist_orient(self, src, dst, deg):
        """Step 3a: this rank's oriented edges (kept for step 3b) -> (int32 raw out-degrees dout [V], local
        self-loops); all-reduce SUM of both."""
        import torch

        b, keep, dev = self._batch(src, dst, None)
        dout = torch.empty(deg.numel(), dtype=torch.int32, device=f"cuda:{self.device}")
        loops = ctypes.c_uint64(0)
        self._check(self._L.gs_tri_dist_orient(self.ctx, ctypes.byref(b), _ptr(deg.contiguous()), _ptr(dout),
                                               ctypes.byref(loops)))
        self._route_n = b.n
        return dout, loops.value

    def tri_dist_route(self, dout, nparts: int):
        """Step 3b: the oriented edges grouped by owner(u) (ranges at equal shares of the raw work of the
        summed dout): (int64 keys tensor, rows per owner)."""
        import torch

        keys = torch.empty(max(self._route_n, 1), dtype=torch.int64, device=f"cuda:{self.device}")
        counts = (ctypes.c_uint64 * nparts)()
        self._check(self._L.gs_tri_dist_route(self.ctx, _ptr(dout.contiguous()), nparts, _ptr(keys), counts))
        counts = [int(x) for x in counts]
        return keys[:sum(counts)], counts

    def tri_dist_build(self, keys, V: int):
        """Step 4: the received rows -> this rank's out-lists: (int32 targets [m], int32 d+ [V])."""
        import torch

        keys = keys.contiguous()
        nbr = torch.empty(max(keys.numel(), 1), dtype=torch.int32, device=f"cuda:{self.device}")
        dplus = torch.empty(V, dtype=torch.int32, device=f"cuda:{self.device}")
        m = ctypes.c_uint64(0)
        self._check(self._L.gs_tri_dist_build(self.ctx, _ptr(keys), keys.numel(), _ptr(nbr), _ptr(dplus),
                                              ctypes.byref(m)))
        return nbr[:m.value], dplus

    def tri_dist_plan(self, dplus, part: int, nparts: int):
        """Step 4a: from the global d+, the boundary exchange's first all-to-all: (elements of this rank's
        rows each rank counts, elements each rank built of the rows this rank counts, unique edges M)."""
        send, recv, M = (ctypes.c_uint64 * nparts)(), (ctypes.c_uint64 * nparts)(), ctypes.c_uint64(0)
        self._check(self._L.gs_tri_dist_plan(self.ctx, _ptr(dplus.contiguous()), part, nparts, send, recv, ctypes.byref(M)))
        return [int(x) for x in send], [int(x) for x in recv], M.value

    def tri_dist_need(self, crows, nparts: int, V: int):
        """Step 4b: the rows this rank's count share reads but holds in neither of its ranges: (int32 ids
        ascending, ids per owner, row elements per owner)."""
        import torch

        crows = crows.contiguous()
        req = torch.empty(max(V, 1), dtype=torch.int32, device=f"cuda:{self.device}")
        rc, re, n = (ctypes.c_uint64 * nparts)(), (ctypes.c_uint64 * nparts)(), ctypes.c_uint64(0)
        self._check(self._L.gs_tri_dist_need(self.ctx, _ptr(crows), _ptr(req), V, rc, re, ctypes.byref(n)))
        return req[:n.value], [int(x) for x in rc], [int(x) for x in re]

    def tri_dist_serve(self, nbr, req_in, counts_in, elems_in):
        """Step 4c: the rows other ranks requested (req_in grouped by requester, counts_in ids each, elems_in
        row elements each) -> (int32 packed rows, elements per requester)."""
        import torch

        P = len(counts_in)
        rows = torch.empty(max(sum(elems_in), 1), dtype=torch.int32, device=f"cuda:{self.device}")
        cin, se = (ctypes.c_uint64 * P)(*[int(x) for x in counts_in]), (ctypes.c_uint64 * P)()
        self._check(self._L.gs_tri_dist_serve(self.ctx, _ptr(nbr.contiguous()), _ptr(req_in.contiguous()), cin,
                                              _ptr(rows), sum(elems_in), se))
        return rows[:sum(elems_in)], [int(x) for x in se]

    def tri_dist_assemble(self, nbr, crows, rows_in, M: int):
        """Step 4d: every row this rank's count share reads, at its window position (int32 [M])."""
        import torch

        full = torch.empty(max(M, 1), dtype=torch.int32, device=f"cuda:{self.device}")
        self._check(self._L.gs_tri_dist_assemble(self.ctx, _ptr(nbr.contiguous()), _ptr(crows.contiguous()),
                                                 _ptr(rows_in.contiguous()), _ptr(full)))
        return full[:M]

    def tri_dist_count(self, nbr, dplus, part: int, nparts: int) -> int:
        """Step 5: this rank's share of the count over the assembled rows (all-reduce SUM)."""
        cnt = ctypes.c_uint64(0)
        nbr = nbr.contiguous()
        self._check(self._L.gs_tri_dist_count(self.ctx, _ptr(nbr), nbr.numel(), _ptr(dplus.contiguous()), part, nparts,
                                              ctypes.byref(cnt)))
        return cnt.value

    def triangles_selfpair(self, src, dst) -> int:
        """gs_window_triangles_selfpair: the self-pair term of a whole window."""
        b, keep, dev = self._batch(src, dst, None)
        S = ctypes.c_uint64(0)
        self._check(self._L.gs_window_triangles_selfpair(self.ctx, ctypes.byref(b), ctypes.byref(S)))
        return S.value

    def triangles_dist(self, src, dst):
        """gs_window_triangles_dist: this rank's records of the window, the ctx communicator's ranks
        together -> (exact count, the reference's Integer, has_output), the same on every rank."""
        b, keep, dev = self._batch(src, dst, None)
        cnt, wrapped, has = ctypes.c_uint64(0), ctypes.c_int32(0), ctypes.c_int32(0)
        self._check(self._L.gs_window_triangles_dist(self.ctx, ctypes.byref(b), ctypes.byref(cnt), ctypes.byref(wrapped),
                                                     ctypes.byref(has)))
        return cnt.value, wrapped.value, bool(has.value)

    # -- ConnectedComponents (gs_components.hip) -------------------------------------------------------
    def components(self, src, dst, prev=None):
        """gs_window_components: the running components after this window's edges; prev = (vertices,
        labels) of the previous window's state or None.  Returns (vertices ascending, smallest vertex of
        each one's component), on the columns' side (device tensors / numpy)."""
        b, keep, dev = self._batch(src, dst, None)
        pk = pv = None
        pb = None
        if prev is not None and len(prev[0]):
            pk, pv = prev
            if dev:
                pk, pv = pk.contiguous(), pv.contiguous()
            else:
                pk, pv = np.ascontiguousarray(pk, np.int64), np.ascontiguousarray(pv, np.int64)
            pb = L.GsPartialBatch(_ptr(pk), _ptr(pv), None, len(pk), L.GS_I64, L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST)
        cap = 2 * (b.n + (len(pk) if pk is not None else 0)) + 1
        keys, labels = self._empty(dev, cap, np.int64), self._empty(dev, cap, np.int64)
        n_out = ctypes.c_uint64(0)
        out = L.GsVertexOut(_ptr(keys), _ptr(labels), cap, ctypes.pointer(n_out), L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_window_components(self.ctx, ctypes.byref(b), ctypes.byref(pb) if pb is not None else None,
                                                 ctypes.byref(out)))
        U = n_out.value
        return keys[:U], labels[:U]

    # -- multi-GPU keyBy halves (gs_dist.hip) --------------------------------------------------------
    def reduce_partials(self, src, dst, val, direction, op, nparts: int):
        """gs_window_reduce_partials: this slice's per-vertex partials grouped by owner (gs_owner_of).
        Returns (keys, partials, owner_counts: list of nparts ints)."""
        b, keep, dev = self._batch(src, dst, None if op == L.GS_OP_COUNT else val)
        R = self._records(b.n, direction)
        odt = np.int64 if op == L.GS_OP_COUNT else L.NP_DTYPE[b.val_dtype]
        keys, vals = self._empty(dev, R, np.int64), self._empty(dev, R, odt)
        n_out, counts = ctypes.c_uint64(0), (ctypes.c_uint64 * nparts)()
        out = L.GsPartialsOut(_ptr(keys), _ptr(vals), None, R, ctypes.pointer(n_out), counts,
                              L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_window_reduce_partials(self.ctx, ctypes.byref(b), int(direction), int(op), nparts,
                                                      ctypes.byref(out)))
        U = n_out.value
        return keys[:U], vals[:U], list(counts)

    def fold_degree_max_partials(self, src, dst, direction, nparts: int):
        """gs_window_fold_degree_max_partials: (keys, degrees, maxima, owner_counts), grouped by owner."""
        b, keep, dev = self._batch(src, dst, None)
        R = self._records(b.n, direction)
        keys, deg, mx = (self._empty(dev, R, np.int64) for _ in range(3))
        n_out, counts = ctypes.c_uint64(0), (ctypes.c_uint64 * nparts)()
        out = L.GsPartialsOut(_ptr(keys), _ptr(deg), _ptr(mx), R, ctypes.pointer(n_out), counts,
                              L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_window_fold_degree_max_partials(self.ctx, ctypes.byref(b), int(direction), nparts,
                                                               ctypes.byref(out)))
        U = n_out.value
        return keys[:U], deg[:U], mx[:U], list(counts)

    def _partial_batch(self, keys, vals, vals2=None):
        dev = _is_torch(keys)
        if not dev:
            keys = np.ascontiguousarray(keys, dtype=np.int64)
            vals = np.ascontiguousarray(vals)
            vals2 = None if vals2 is None else np.ascontiguousarray(vals2, dtype=np.int64)
        else:
            keys, vals = keys.contiguous(), vals.contiguous()
            vals2 = None if vals2 is None else vals2.contiguous()
        pb = L.GsPartialBatch(_ptr(keys), _ptr(vals), _ptr(vals2), len(keys), _gs_dtype(vals),
                              L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST)
        return pb, (keys, vals, vals2), dev

    def merge_partials(self, keys, vals, op, init=None):
        """gs_merge_partials: an owner's received partials -> (keys, values), keys ascending."""
        pb, keep, dev = self._partial_batch(keys, vals)
        n = pb.n
        odt = np.int64 if op == L.GS_OP_COUNT else L.NP_DTYPE[pb.val_dtype]
        ko, vo = self._empty(dev, n, np.int64), self._empty(dev, n, odt)
        n_out = ctypes.c_uint64(0)
        out = L.GsVertexOut(_ptr(ko), _ptr(vo), n, ctypes.pointer(n_out), L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        ia = None if init is None else np.array([init], dtype=odt)
        self._check(self._L.gs_merge_partials(self.ctx, ctypes.byref(pb), int(op),
                                              None if ia is None else ia.ctypes.data_as(ctypes.c_void_p),
                                              ctypes.byref(out)))
        U = n_out.value
        return ko[:U], vo[:U]

    def merge_degree_max_partials(self, keys, deg, mx, init_max=-(1 << 63)):
        pb, keep, dev = self._partial_batch(keys, deg, mx)
        n = pb.n
        ko, do, mo = (self._empty(dev, n, np.int64) for _ in range(3))
        n_out = ctypes.c_uint64(0)
        out = L.GsDegreeOut(_ptr(ko), _ptr(do), _ptr(mo), n, ctypes.pointer(n_out),
                            L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        self._check(self._L.gs_merge_degree_max_partials(self.ctx, ctypes.byref(pb), int(init_max), ctypes.byref(out)))
        U = n_out.value
        return ko[:U], do[:U], mo[:U]

    def owner_of(self, vertex: int, nparts: int) -> int:
        return int(self._L.gs_owner_of(int(vertex), nparts))

    # -- the ctx communicator: RCCL (one rank per process) or an in-process CommGroup ---------------------
    @staticmethod
    def device_count() -> int:
        n = ctypes.c_int32(0)
        st = L.load().gs_device_count(ctypes.byref(n))
        if st != L.GS_OK:
            raise GsError(st, "gs_device_count failed")
        return n.value

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        st = L.load().gs_comm_unique_id(buf)
        if st != L.GS_OK:
            raise GsError(st, "gs_comm_unique_id failed (RCCL not found?)")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, unique_id: bytes):
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        self._check(self._L.gs_comm_init(self.ctx, nranks, rank, buf))

    def comm_init_group(self, group: "CommGroup", rank: int):
        """gs_comm_init_group: this ctx becomes rank `rank` of an in-process thread group; every rank's
        calls then come from its own thread (ctypes releases the GIL for the call)."""
        self._check(self._L.gs_comm_init_group(self.ctx, group.handle, int(rank)))

    def comm_destroy(self):
        self._check(self._L.gs_comm_destroy(self.ctx))

    def comm_allreduce_sum(self, value: int) -> int:
        v = ctypes.c_uint64(value & ((1 << 64) - 1))
        self._check(self._L.gs_comm_allreduce_sum_u64(self.ctx, ctypes.byref(v)))
        return v.value

    def reduce_dist(self, src, dst, val, direction, op, init=None, out=None):
        """gs_window_reduce_dist: this rank's slice through partials -> RCCL all-to-all -> merge; returns
        the (keys, values) this rank owns.  out: optional (keys, values) device tensors reused across
        windows (their length is the capacity)."""
        b, keep, dev = self._batch(src, dst, None if op == L.GS_OP_COUNT else val)
        odt = np.int64 if op == L.GS_OP_COUNT else L.NP_DTYPE[b.val_dtype]
        if out is not None:
            self._check_out(out, dev, (np.int64, odt))
            keys, vals = out
            cap = min(keys.numel(), vals.numel())
        else:
            cap = self._records(b.n, direction) + 1024   # a guess; more owned vertices: gs_fetch_last_output
            keys, vals = self._empty(dev, cap, np.int64), self._empty(dev, cap, odt)
        n_out = ctypes.c_uint64(0)
        out = L.GsVertexOut(_ptr(keys), _ptr(vals), cap, ctypes.pointer(n_out), L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        ia = None if init is None else np.array([init], dtype=odt)
        st = self._L.gs_window_reduce_dist(self.ctx, ctypes.byref(b), int(direction), int(op),
                                          None if ia is None else ia.ctypes.data_as(ctypes.c_void_p), ctypes.byref(out))
        if st == L.GS_ECAPACITY:   # more owned vertices than this guess: fetch the staged rows (no recompute)
            U = n_out.value
            keys, vals = self._empty(dev, U, np.int64), self._empty(dev, U, odt)
            out = L.GsVertexOut(_ptr(keys), _ptr(vals), U, ctypes.pointer(n_out),
                                L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
            st = self._L.gs_fetch_last_output(self.ctx, ctypes.byref(out))
        self._check(st)
        U = n_out.value
        return keys[:U], vals[:U]

    def fold_degree_max_dist(self, src, dst, direction, init_max=-(1 << 63)):
        b, keep, dev = self._batch(src, dst, None)
        cap = self._records(b.n, direction) + 1024
        keys, deg, mx = (self._empty(dev, cap, np.int64) for _ in range(3))
        n_out = ctypes.c_uint64(0)
        out = L.GsDegreeOut(_ptr(keys), _ptr(deg), _ptr(mx), cap, ctypes.pointer(n_out),
                            L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
        st = self._L.gs_window_fold_degree_max_dist(self.ctx, ctypes.byref(b), int(direction), int(init_max),
                                                    ctypes.byref(out))
        if st == L.GS_ECAPACITY:
            U = n_out.value
            keys, deg, mx = (self._empty(dev, U, np.int64) for _ in range(3))
            out = L.GsDegreeOut(_ptr(keys), _ptr(deg), _ptr(mx), U, ctypes.pointer(n_out),
                                L.GS_MEM_DEVICE if dev else L.GS_MEM_HOST, 0)
            st = self._L.gs_fetch_last_degree_output(self.ctx, ctypes.byref(out))
        self._check(st)
        U = n_out.value
        return keys[:U], deg[:U], mx[:U]

    # -- synthetic streams (device) ----------------------------------------------------------------
    def generate_rmat(self, scale, n, seed, a=0.57, b=0.19, c=0.19, permute=True, no_self_loops=False,
                      first_edge=0, out=None):
        import torch

        src, dst = out if out is not None else (torch.empty(n, dtype=torch.int64, device=f"cuda:{self.device}"),
                                                torch.empty(n, dtype=torch.int64, device=f"cuda:{self.device}"))
        self._check(self._L.gs_generate_rmat(self.ctx, scale, n, seed, fx32(a), fx32(b), fx32(c), int(permute),
                                             int(no_self_loops), first_edge, _ptr(src), _ptr(dst)))
        return src, dst

    def generate_uniform(self, num_vertices, n, seed, first_edge=0):
        import torch

        src = torch.empty(n, dtype=torch.int64, device=f"cuda:{self.device}")
        dst = torch.empty(n, dtype=torch.int64, device=f"cuda:{self.device}")
        self._check(self._L.gs_generate_uniform(self.ctx, num_vertices, n, seed, first_edge, _ptr(src), _ptr(dst)))
        return src, dst

    def generate_zipf(self, num_vertices, n, seed, exponent=1.1, first_edge=0):
        """Zipf(exponent) sources over [0, num_vertices) (hubs at the lowest IDs), uniform destinations."""
        import torch

        src = torch.empty(n, dtype=torch.int64, device=f"cuda:{self.device}")
        dst = torch.empty(n, dtype=torch.int64, device=f"cuda:{self.device}")
        self._check(self._L.gs_generate_zipf(self.ctx, num_vertices, float(exponent), n, seed, first_edge, _ptr(src),
                                             _ptr(dst)))
        return src, dst

    def generate_values(self, n, seed, dtype=L.GS_I64, first_edge=0):
        import torch

        tdt = {L.GS_I32: torch.int32, L.GS_I64: torch.int64, L.GS_F32: torch.float32, L.GS_F64: torch.float64}[dtype]
        v = torch.empty(n, dtype=tdt, device=f"cuda:{self.device}")
        self._check(self._L.gs_generate_values(self.ctx, n, seed, first_edge, dtype, _ptr(v)))
        return v
