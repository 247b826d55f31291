"""Host-side mirror of the reference's windowed graph-stream API, backed by libgellyhip.so.

  SimpleEdgeStream   <- streaming/SimpleEdgeStream.java:59-540 (constructors :73-94, slice :139-171,
                        reverse :332-341, undirected :354-365)
  GraphWindowStream  <- streaming/GraphWindowStream.java:47-183 (foldNeighbors :62, reduceOnEdges :101,
                        applyOnNeighbors :130)

Same names, argument meaning and error behaviour as the Java API (camelCase kept on purpose so a
reference test reads the same here).  Windowing follows Flink 1.0.3 tumbling windows: a record with
timestamp ts belongs to [ts - ts % size, ... + size) (Java remainder), a window's results carry
timestamp end - 1.  A stream built without a time extractor behaves like the reference's
ingestion-time tests (TestSlice): every record lands in the first window.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from enum import IntEnum

import numpy as np

from . import _lib as L
from .engine import Engine, _is_torch
from .functions import (Collector, EdgesApply, EdgesFold, EdgesReduce, DegreeMaxNeighborFold, _BuiltinFold,
                        _BuiltinReduce)


class EdgeDirection(IntEnum):
    """org.apache.flink.graph.EdgeDirection (ordinals IN, OUT, ALL)."""
    IN = 0
    OUT = 1
    ALL = 2


class TimeUnit(IntEnum):
    MILLISECONDS = 1
    SECONDS = 1000
    MINUTES = 60000


@dataclass(frozen=True)
class Time:
    """org.apache.flink.streaming.api.windowing.time.Time."""
    ms: int

    @staticmethod
    def of(size: int, unit: TimeUnit = TimeUnit.MILLISECONDS) -> "Time":
        return Time(int(size) * int(unit))

    @staticmethod
    def milliseconds(n: int) -> "Time":
        return Time(int(n))

    @staticmethod
    def seconds(n: int) -> "Time":
        return Time(int(n) * 1000)

    def toMilliseconds(self) -> int:
        return self.ms


@dataclass
class EdgeColumns:
    """A DataStream<Edge<Long, EV>> laid out as columns (Tuple3 f0 = src, f1 = dst, f2 = value) plus an
    optional event-time column.  Columns are numpy (host) or torch CUDA tensors (device)."""
    src: object
    dst: object
    val: object = None
    ts: object = None

    def __len__(self):
        return len(self.src)


class StreamExecutionEnvironment:
    """Holds the engine (one gs_ctx) — the role of the Flink environment for this path."""
    _default = None

    def __init__(self, device: int = 0):
        self.device = device
        self._engine = None
        self._parallelism = 1

    def setParallelism(self, parallelism: int) -> "StreamExecutionEnvironment":
        """env.setParallelism: the operators' parallelism; on this path it changes what the windowed
        graph aggregation emits (one running state per partition's partial, aggregation.py)."""
        if int(parallelism) < 1:
            raise ValueError("parallelism must be at least 1")
        self._parallelism = int(parallelism)
        return self

    def getParallelism(self) -> int:
        return self._parallelism

    @classmethod
    def getExecutionEnvironment(cls) -> "StreamExecutionEnvironment":
        if cls._default is None:
            cls._default = cls()
        return cls._default

    @property
    def engine(self) -> Engine:
        if self._engine is None:
            self._engine = Engine(self.device)
        return self._engine

    def fromCollection(self, edges, value_dtype=np.int64) -> EdgeColumns:
        """env.fromCollection(List<Edge<Long, EV>>): tuples (src, dst[, value[, ts]])."""
        edges = list(edges)
        src = np.array([e[0] for e in edges], dtype=np.int64)
        dst = np.array([e[1] for e in edges], dtype=np.int64)
        val = np.array([e[2] for e in edges], dtype=value_dtype) if edges and len(edges[0]) > 2 else None
        ts = np.array([e[3] for e in edges], dtype=np.int64) if edges and len(edges[0]) > 3 else None
        return EdgeColumns(src, dst, val, ts)


class AscendingTimestampExtractor:
    """Marks a stream as event-time (SimpleEdgeStream.java:90-94).  extract(cols) -> int64 timestamps."""

    def extractAscendingTimestamp(self, cols: EdgeColumns):
        raise NotImplementedError


class EdgeValueTimestampExtractor(AscendingTimestampExtractor):
    """WindowTriangles.EdgeValueTimestampExtractor (WindowTriangles.java:224-230): ts = edge value."""

    def extractAscendingTimestamp(self, cols: EdgeColumns):
        v = cols.val
        return v.cpu().numpy().astype(np.int64) if _is_torch(v) else np.asarray(v, dtype=np.int64)


@dataclass
class WindowOutput:
    start: int
    end: int
    columns: tuple            # columnar results (keys, values...) or ('records', list)

    @property
    def max_timestamp(self) -> int:
        return self.end - 1


@dataclass
class DataStream:
    """Result stream: per window, the records emitted at window end (timestamp end - 1)."""
    windows: list = field(default_factory=list)

    def collect(self) -> list:
        """All records as Python tuples, window by window (vertices ascending inside a window)."""
        out = []
        for w in self.windows:
            out.extend(_rows(w.columns))
        return out

    def collectWithTimestamps(self) -> list:
        out = []
        for w in self.windows:
            out.extend((r, w.max_timestamp) for r in _rows(w.columns))
        return out


def _to_np(x):
    if x is None:
        return None
    return x.cpu().numpy() if _is_torch(x) else np.asarray(x)


def _rows(cols):
    if cols and isinstance(cols[0], str) and cols[0] == "records":
        return list(cols[1])
    arrs = [_to_np(c) for c in cols]
    return [tuple(v.item() for v in row) for row in zip(*arrs)]


def _take(x, idx):
    if x is None:
        return None
    if _is_torch(x):
        import torch

        return x.index_select(0, torch.as_tensor(idx, device=x.device))
    return np.asarray(x)[idx]


class SimpleEdgeStream:
    """streaming/SimpleEdgeStream.java — the windowed-neighbourhood part of it."""

    def __init__(self, edges: EdgeColumns, context: StreamExecutionEnvironment = None,
                 timeExtractor: AscendingTimestampExtractor = None):
        self.context = context or StreamExecutionEnvironment.getExecutionEnvironment()
        self.edges = edges
        if timeExtractor is not None:   # :90-94 event time
            self.edges = EdgeColumns(edges.src, edges.dst, edges.val,
                                     np.asarray(timeExtractor.extractAscendingTimestamp(edges), dtype=np.int64))

    def getEdges(self) -> EdgeColumns:
        return self.edges

    def getContext(self) -> StreamExecutionEnvironment:
        return self.context

    def mapEdges(self, mapper) -> "SimpleEdgeStream":
        """mapEdges (SimpleEdgeStream.java:221-226) for the value-dropping mapper of WindowTriangles
        (RemoveEdgeValue -> NullValue): mapper(values) returns the new value column or None."""
        e = self.edges
        return SimpleEdgeStream(EdgeColumns(e.src, e.dst, mapper(e.val), e.ts), self.context)

    def reverse(self) -> "SimpleEdgeStream":
        """:332-341 Edge.reverse() = (f1, f0, f2)."""
        e = self.edges
        return SimpleEdgeStream(EdgeColumns(e.dst, e.src, e.val, e.ts), self.context)

    def undirected(self) -> "SimpleEdgeStream":
        """:354-365 emits e then e.reverse() for every edge."""
        e = self.edges
        n = len(e)
        if _is_torch(e.src):
            import torch

            src = torch.stack([e.src, e.dst], 1).reshape(-1)
            dst = torch.stack([e.dst, e.src], 1).reshape(-1)
            val = None if e.val is None else torch.repeat_interleave(e.val, 2)
        else:
            src = np.empty(2 * n, np.int64); src[0::2] = e.src; src[1::2] = e.dst
            dst = np.empty(2 * n, np.int64); dst[0::2] = e.dst; dst[1::2] = e.src
            val = None if e.val is None else np.repeat(np.asarray(e.val), 2)
        ts = None if e.ts is None else np.repeat(np.asarray(e.ts), 2)
        return SimpleEdgeStream(EdgeColumns(src, dst, val, ts), self.context)

    def aggregate(self, graphAggregation) -> "DataStream":
        """GraphStream.aggregate (SimpleEdgeStream.java:104-106): e.g. ConnectedComponents(mergeWindowTime)."""
        return graphAggregation.run(self)

    def slice(self, size: Time, direction: EdgeDirection = EdgeDirection.OUT) -> "GraphWindowStream":
        """:139-171 tumbling windows keyed by the neighbour-key vertex."""
        if not isinstance(direction, EdgeDirection) and direction not in (0, 1, 2):
            raise ValueError("Illegal edge direction")   # IllegalArgumentException :168-169
        return GraphWindowStream(self, size.toMilliseconds(), EdgeDirection(direction))

    # tumbling windows of this stream: [(start, end, columns of that window in arrival order)]
    def _windows(self, size_ms: int, with_index: bool = False):
        """with_index: each window also carries its records' positions in the stream (arrival order)."""
        e = self.edges
        if e.ts is None:
            return [(0, size_ms, e, np.arange(len(e)))] if with_index else [(0, size_ms, e)]
        ts = np.asarray(e.ts, dtype=np.int64)
        start = ts - np.fmod(ts, size_ms)
        order = np.argsort(start, kind="stable")
        starts, first = np.unique(start[order], return_index=True)
        bounds = list(first) + [len(order)]
        out = []
        for i, s in enumerate(starts):
            idx = order[bounds[i]:bounds[i + 1]]
            contiguous = len(idx) == 0 or (idx[-1] - idx[0] + 1 == len(idx) and np.all(np.diff(idx) == 1))
            if contiguous and len(idx):
                sl = slice(int(idx[0]), int(idx[-1]) + 1)
                cols = EdgeColumns(e.src[sl], e.dst[sl], None if e.val is None else e.val[sl], ts[sl])
            else:
                cols = EdgeColumns(_take(e.src, idx), _take(e.dst, idx), _take(e.val, idx), ts[idx])
            out.append((int(s), int(s) + size_ms, cols, idx) if with_index else (int(s), int(s) + size_ms, cols))
        return out


class GraphWindowStream:
    """streaming/GraphWindowStream.java:47-183."""

    def __init__(self, stream: SimpleEdgeStream, size_ms: int, direction: EdgeDirection):
        self.stream = stream
        self.size_ms = size_ms
        self.direction = direction

    @property
    def engine(self) -> Engine:
        return self.stream.context.engine

    def _each(self):
        return self.stream._windows(self.size_ms)

    def reduceOnEdges(self, reduceFunction: EdgesReduce) -> DataStream:
        """:101-104 -> Tuple2<K, EV>(vertex, reduced value) per vertex and window."""
        out = DataStream()
        for s, t, w in self._each():
            if len(w) == 0:
                continue
            if isinstance(reduceFunction, _BuiltinReduce):
                if reduceFunction.op != L.GS_OP_COUNT and w.val is None:
                    raise ValueError("reduceOnEdges needs edge values")
                k, v = self.engine.reduce(w.src, w.dst, w.val, self.direction, reduceFunction.op)
                out.windows.append(WindowOutput(s, t, (k, v)))
            else:
                recs = []
                for key, nbrs, vals in self._groups(w):
                    acc = vals[0]
                    for x in vals[1:]:
                        acc = reduceFunction.reduceEdges(acc, x)   # EdgesReduceFunction.reduce :116-120
                    recs.append((key, acc))
                out.windows.append(WindowOutput(s, t, ("records", recs)))
        return out

    def foldNeighbors(self, initialValue, foldFunction: EdgesFold) -> DataStream:
        """:62-64 -> one accumulator per vertex and window, folded from a copy of initialValue."""
        out = DataStream()
        for s, t, w in self._each():
            if len(w) == 0:
                continue
            if isinstance(foldFunction, DegreeMaxNeighborFold):
                init_max = int(initialValue[2]) if len(initialValue) > 2 else -(1 << 63)
                k, d, m = self.engine.fold_degree_max(w.src, w.dst, self.direction, init_max)
                if int(initialValue[1]) != 0:
                    d = d + int(initialValue[1])
                out.windows.append(WindowOutput(s, t, (k, d, m)))
            elif isinstance(foldFunction, _BuiltinFold):
                if foldFunction.op != L.GS_OP_COUNT and w.val is None:
                    raise ValueError("foldNeighbors needs edge values")
                k, v = self.engine.fold(w.src, w.dst, w.val, self.direction, foldFunction.op, initialValue[1])
                out.windows.append(WindowOutput(s, t, (k, v)))
            else:
                recs = []
                for key, nbrs, vals in self._groups(w):
                    acc = copy.deepcopy(initialValue)
                    for nb, x in zip(nbrs, vals if vals is not None else [None] * len(nbrs)):
                        acc = foldFunction.foldEdges(acc, key, nb, x)   # EdgesFoldFunction.fold :78-80
                    recs.append(acc)
                out.windows.append(WindowOutput(s, t, ("records", recs)))
        return out

    def applyOnNeighbors(self, applyFunction: EdgesApply) -> DataStream:
        """:130-131 -> 0..n records per vertex from its (neighbour, value) list in arrival order."""
        from .triangles import GenerateCandidateEdges

        out = DataStream()
        for s, t, w in self._each():
            if len(w) == 0:
                continue
            if isinstance(applyFunction, GenerateCandidateEdges) and self.direction == EdgeDirection.ALL:
                a, b, f = self.engine.candidates(w.src, w.dst)
                out.windows.append(WindowOutput(s, t, (a, b, f)))
                continue
            col = Collector()
            for key, nbrs, vals in self._groups(w):
                vv = vals if vals is not None else [None] * len(nbrs)
                applyFunction.applyOnEdges(key, [(nb, x) for nb, x in zip(nbrs, vv)], col)   # :144-175
            out.windows.append(WindowOutput(s, t, ("records", col.records)))
        return out

    # GPU grouping for host-side user functions: (key, neighbours, values) in arrival order
    def _groups(self, w: EdgeColumns):
        keys, offs, nbrs, vals = self.engine.csr(w.src, w.dst, w.val, self.direction)
        keys, offs, nbrs = _to_np(keys), _to_np(offs), _to_np(nbrs)
        vals = _to_np(vals)
        for u in range(len(keys)):
            lo, hi = int(offs[u]), int(offs[u + 1])
            yield (int(keys[u]), [int(x) for x in nbrs[lo:hi]],
                   None if vals is None else [x.item() for x in vals[lo:hi]])
