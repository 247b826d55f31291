"""WindowTriangles (example/WindowTriangles.java:49-244) on the engine.

The reference pipeline is
    edges.slice(windowTime, ALL).applyOnNeighbors(GenerateCandidateEdges)
         .keyBy(0, 1).timeWindow(windowTime).apply(CountTriangles)
         .timeWindowAll(windowTime).sum(0)                               (:61-66)
Here each window goes to gs_window_triangles, which computes the same Integer (count of matched
candidates, mod 2^32 as signed) without materialising the O(sum d^2) candidate stream.
`GenerateCandidateEdges` stays available as an EdgesApply: on slice(ALL) it runs on the GPU
(gs_window_candidates) and emits exactly the reference's records.
"""
from __future__ import annotations

import sys

import numpy as np

from .functions import EdgesApply
from .stream import (DataStream, EdgeColumns, EdgeDirection, EdgeValueTimestampExtractor, SimpleEdgeStream,
                     StreamExecutionEnvironment, Time, WindowOutput)


class GenerateCandidateEdges(EdgesApply):
    """WindowTriangles.java:83-116 — routed to gs_window_candidates on slice(ALL)."""

    def applyOnEdges(self, vertexID, neighbors, out):
        raise RuntimeError("GenerateCandidateEdges runs in the engine (slice(..., EdgeDirection.ALL))")


class CountTriangles:
    """WindowTriangles.java:119-140: per (a, b) group, emit (#candidates, window.maxTimestamp) iff edges > 0.
    Runs in the engine through `count_triangles` (gs_window_count_candidates)."""


def count_triangles(candidates: DataStream, engine) -> DataStream:
    """Stage 2 of WindowTriangles over materialised candidate records (WindowTriangles.java:64-66):
    .keyBy(0, 1).timeWindow(w).apply(CountTriangles()).timeWindowAll(w).sum(0).  Stage-1 records carry
    ts = end - 1, so each stage-1 window is one stage-2 window; it yields one (Integer, end - 1) record
    when any pair group emits."""
    out = DataStream()
    for w in candidates.windows:
        a, b, f = w.columns
        exact, wrapped, has, groups = engine.count_candidates(a, b, f)
        if has:
            out.windows.append(WindowOutput(w.start, w.end, ("records", [(wrapped, w.end - 1)])))
    return out


class RemoveEdgeValue:
    """WindowTriangles.java:232-238: value -> NullValue."""

    def __call__(self, values):
        return None


def window_triangles(edges: SimpleEdgeStream, window: Time) -> DataStream:
    """The whole WindowTriangles pipeline: one (Integer count, window end - 1) record per non-empty window."""
    ws = edges.slice(window, EdgeDirection.ALL)
    eng = ws.engine
    out = DataStream()
    for s, t, w in ws._each():
        if len(w) == 0:
            continue
        exact, wrapped, has = eng.triangles(w.src, w.dst)
        if has:
            out.windows.append(WindowOutput(s, t, ("records", [(wrapped, t - 1)])))
    return out


def parse_edges_text(path: str, engine):
    """"src trg ts" per line (WindowTriangles.java:175-185) -> int64 host columns, parsed on the GPU
    (gs_parse_edges_text: the reference's split("\\s") + Long.parseLong rules; a malformed line raises
    GsError, as the reference's map throws)."""
    with open(path, "rb") as f:
        text = f.read()
    return engine.parse_edges_text(text, out_device=False)


def default_edges():
    """WindowTriangles.java:188-197: generateSequence(1, 10) -> (k, k+i, k*100 + (i-1)*50), i = 1, 2."""
    rows = [(k, k + i, k * 100 + (i - 1) * 50) for k in range(1, 11) for i in (1, 2)]
    a = np.array(rows, dtype=np.int64)
    return a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy()


def main(args=None, env: StreamExecutionEnvironment = None) -> list:
    """WindowTriangles.main: <input edges path> <output path> <window time (ms)>; returns the output lines."""
    args = list(sys.argv[1:] if args is None else args)
    window = Time.milliseconds(300)   # :145
    if args:
        if len(args) != 3:
            print("Usage: WindowTriangles <input edges path> <output path> <window time (ms)>", file=sys.stderr)
            return []
        env = env or StreamExecutionEnvironment.getExecutionEnvironment()
        src, dst, ts = parse_edges_text(args[0], env.engine)
        window = Time.milliseconds(int(args[2]))
    else:
        src, dst, ts = default_edges()
    env = env or StreamExecutionEnvironment.getExecutionEnvironment()
    stream = SimpleEdgeStream(EdgeColumns(src, dst, ts), env, EdgeValueTimestampExtractor()).mapEdges(RemoveEdgeValue())
    result = window_triangles(stream, window)
    lines = [f"({c},{t})" for (c, t) in result.collect()]
    if args:
        with open(args[1], "w") as f:
            f.write("\n".join(lines) + ("\n" if lines else ""))
    else:
        print("\n".join(lines))
    return lines
