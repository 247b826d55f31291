"""WindowOperator: the columnar event-time window-buffer operator of libgellyhip.so (gs_stream_*).

It replaces what Flink does between slice() and the window function for the built-in operators
(SimpleEdgeStream.java:153-171 keyBy(...).timeWindow(size); GraphWindowStream.java:49-53; Flink 1.0.3
TumblingEventTimeWindows + EventTimeTrigger): records are appended with their event timestamps, buffered
per window in pinned host memory (start = ts - ts % size, Java remainder), and a window fires when the
watermark reaches end - 1.  Its columns are copied to HBM on the operator's copy stream (overlapping the
previous window's kernels) and its result — stamped end - 1 — comes back from poll() in firing order.
Watermarks are explicit (watermark()) or ascending (max timestamp seen - 1 after every append, the
AscendingTimestampExtractor of SimpleEdgeStream.java:90-94); flush() ends a finite source.  Records of a
window that already fired open a fresh pane that fires at the next watermark (late_mode GS_LATE_REFIRE,
Flink 1.0.3's WindowOperator) or are dropped (GS_LATE_DROP); both are counted in stats()["late_records"].
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from ._lib import GsError


@dataclass
class WindowResult:
    start: int
    end: int
    max_timestamp: int        # end - 1: the timestamp of every record the window emits
    edges: int
    columns: tuple            # (keys, values) | (keys, degrees, maxima) | (exact, Integer) for triangles
    has_output: bool
    latency_ms: float


class WindowOperator:
    def __init__(self, engine, window_ms: int, kind: int = L.GS_STREAM_REDUCE, direction: int = 1, op: int = 0,
                 val_dtype=np.int64, watermarks: int = L.GS_WATERMARK_ASCENDING, init=None,
                 init_max: int = -(1 << 63), max_window_edges: int = 0, staging: int = L.GS_STAGE_PINNED,
                 late_mode: int = L.GS_LATE_REFIRE):
        self._L, self.engine = engine._L, engine
        self.kind = kind
        self.op = op
        self.np_dtype = None if val_dtype is None else np.dtype(val_dtype)
        gdt = L.GS_NONE if val_dtype is None else L.GS_DTYPE_OF[np.dtype(val_dtype)]
        self._init = None
        if init is not None:
            self._init = np.array([init], dtype=np.int64 if op == L.GS_OP_COUNT else val_dtype)
        cfg = L.GsStreamConfig(int(window_ms), kind, int(direction), int(op), gdt, watermarks, int(staging),
                               None if self._init is None else self._init.ctypes.data_as(ctypes.c_void_p),
                               int(init_max), int(max_window_edges), int(late_mode), 0)
        h = ctypes.c_void_p()
        st = self._L.gs_stream_create(engine.ctx, ctypes.byref(cfg), ctypes.byref(h))
        if st != L.GS_OK:
            raise GsError(st, self._L.gs_last_error(engine.ctx).decode())
        self.h = h

    def _check(self, st):
        if st != L.GS_OK:
            raise GsError(st, self._L.gs_last_error(self.engine.ctx).decode())

    def close(self):
        if getattr(self, "h", None):
            self._L.gs_stream_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def append(self, src, dst, val, ts):
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        if val is not None and self.np_dtype is not None:
            val = np.ascontiguousarray(val, dtype=self.np_dtype)
        else:
            val = None
        if not (len(src) == len(dst) == len(ts)) or (val is not None and len(val) != len(src)):
            raise ValueError("columns must have the same length")
        p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)
        self._check(self._L.gs_stream_append(self.h, p(src), p(dst), p(val), p(ts), len(src)))

    def watermark(self, wm: int):
        self._check(self._L.gs_stream_watermark(self.h, int(wm)))

    def flush(self):
        self._check(self._L.gs_stream_flush(self.h))

    def poll(self, wait: bool = True):
        """The next window result in firing order (None when none is ready and wait is False, or when
        nothing has fired)."""
        r = L.GsWindowResult()
        st = self._L.gs_stream_poll(self.h, 1 if wait else 0, ctypes.byref(r))
        if st == L.GS_EAGAIN:
            return None
        self._check(st)
        U = r.n_vertices
        if self.kind == L.GS_STREAM_TRIANGLES:
            cols = (r.triangles, r.triangles_ref)
        else:
            keys = np.ctypeslib.as_array(ctypes.cast(r.keys, ctypes.POINTER(ctypes.c_int64)), (U,)).copy() if U else \
                np.empty(0, np.int64)
            vdt = np.int64 if (self.kind == L.GS_STREAM_DEGREE_MAX or self.op == L.GS_OP_COUNT) else self.np_dtype
            vals = (np.frombuffer((ctypes.c_char * (U * np.dtype(vdt).itemsize)).from_address(r.vals), dtype=vdt).copy()
                    if U else np.empty(0, vdt))
            cols = (keys, vals)
            if self.kind == L.GS_STREAM_DEGREE_MAX:
                mx = np.ctypeslib.as_array(ctypes.cast(r.vals2, ctypes.POINTER(ctypes.c_int64)), (U,)).copy() if U else \
                    np.empty(0, np.int64)
                cols = (keys, vals, mx)
        return WindowResult(r.window_start, r.window_end, r.max_timestamp, r.edges, cols, bool(r.has_output),
                            r.latency_ms)

    def drain(self):
        """Every result that has fired, in order."""
        out = []
        while True:
            st = self.stats()
            if st["pending_windows"] == 0:
                return out
            out.append(self.poll(True))

    def stats(self) -> dict:
        s = L.GsStreamStats()
        self._check(self._L.gs_stream_stats(self.h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in L.GsStreamStats._fields_}
