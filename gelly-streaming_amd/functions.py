"""The reference's user-function interfaces and the built-ins the engine runs on the GPU.

  EdgesReduce  <- streaming/EdgesReduce.java:31-44   reduceEdges(firstEdgeValue, secondEdgeValue)
  EdgesFold    <- streaming/EdgesFold.java:33-48     foldEdges(accum, vertexID, neighborID, edgeValue)
  EdgesApply   <- streaming/EdgesApply.java:35-48    applyOnEdges(vertexID, neighbors, out)

Dispatch rule: an instance of a *built-in* class below is executed by
libgellyhip.so (sort + segmented reduce on the GPU).  Any other subclass is user code: the GPU still
groups the window (gs_window_csr, arrival order kept) and the user function is then called per
vertex on the host exactly as Flink's window function would call it.
"""
from __future__ import annotations

from . import _lib as L


class EdgesReduce:
    """Interface: combine two edge values of one vertex into one (GraphWindowStream.java:101-121)."""

    def reduceEdges(self, firstEdgeValue, secondEdgeValue):
        raise NotImplementedError


class EdgesFold:
    """Interface: fold one neighbour edge into the accumulator (GraphWindowStream.java:62-87)."""

    def foldEdges(self, accum, vertexID, neighborID, edgeValue):
        raise NotImplementedError


class EdgesApply:
    """Interface: compute 0..n outputs from a vertex neighbourhood (GraphWindowStream.java:130-175)."""

    def applyOnEdges(self, vertexID, neighbors, out):
        raise NotImplementedError


class Collector:
    """org.apache.flink.util.Collector: out.collect(record)."""

    def __init__(self):
        self.records = []

    def collect(self, record):
        self.records.append(tuple(record) if isinstance(record, (list, tuple)) else record)


# ---- built-in reducers (GPU) ----------------------------------------------------------------------
class _BuiltinReduce(EdgesReduce):
    op: int = -1


class SumReduce(_BuiltinReduce):
    """reduceEdges(a, b) = a + b  (Integer/Long wrap, Float/Double IEEE) — TestSlice.java:242-249."""
    op = L.GS_OP_SUM

    def reduceEdges(self, a, b):
        return a + b


class MinReduce(_BuiltinReduce):
    """reduceEdges(a, b) = Math.min(a, b)."""
    op = L.GS_OP_MIN

    def reduceEdges(self, a, b):
        return min(a, b)


class MaxReduce(_BuiltinReduce):
    """reduceEdges(a, b) = Math.max(a, b)."""
    op = L.GS_OP_MAX

    def reduceEdges(self, a, b):
        return max(a, b)


class CountReduce(_BuiltinReduce):
    """Number of edge records of the vertex in the window (Long)."""
    op = L.GS_OP_COUNT


# ---- built-in folds (GPU) -------------------------------------------------------------------------
class _BuiltinFold(EdgesFold):
    op: int = -1


class SumValuesFold(_BuiltinFold):
    """acc.f0 = vertexID; acc.f1 += edgeValue, from init (k, v0) -> (vertex, v0 + sum).  TestSlice.java:233-240."""
    op = L.GS_OP_SUM

    def foldEdges(self, accum, vertexID, neighborID, edgeValue):
        return (vertexID, accum[1] + edgeValue)


class MinValuesFold(_BuiltinFold):
    op = L.GS_OP_MIN

    def foldEdges(self, accum, vertexID, neighborID, edgeValue):
        return (vertexID, min(accum[1], edgeValue))


class MaxValuesFold(_BuiltinFold):
    op = L.GS_OP_MAX

    def foldEdges(self, accum, vertexID, neighborID, edgeValue):
        return (vertexID, max(accum[1], edgeValue))


class CountFold(_BuiltinFold):
    """acc = (vertex, acc.f1 + 1)."""
    op = L.GS_OP_COUNT

    def foldEdges(self, accum, vertexID, neighborID, edgeValue):
        return (vertexID, accum[1] + 1)


class DegreeMaxNeighborFold(_BuiltinFold):
    """acc = (vertex, degree + 1, max(maxNeighbor, neighborID)) from init (k, 0, m0) (BASELINE config C3)."""
    op = -2

    def foldEdges(self, accum, vertexID, neighborID, edgeValue):
        return (vertexID, accum[1] + 1, max(accum[2], neighborID))


def is_builtin(f) -> bool:
    return isinstance(f, (_BuiltinReduce, _BuiltinFold))
