"""GraphStream.aggregate(...) for the one aggregation the reference's library ships: ConnectedComponents
(library/ConnectedComponents.java:43-131 on WindowGraphAggregation.java:30-65 and GraphAggregation.java's
Merger).

Per tumbling window of `mergeWindowTime` ms the reference folds the window's edges into a DisjointSet
(UpdateCC -> union) and the parallelism-1 Merger combines it into its running state (CombineCC ->
DisjointSet.merge; transientState = false, so the state accumulates over windows) and emits the state.
Here each window is one gs_window_components call on the GPU with the previous state as input: the
emitted record per vertex is (vertex, smallest vertex of its component) -- the partition DisjointSet
holds (its toString groups by root; which vertex is the root depends on HashMap order).

Parallelism (GraphAggregation.java:103-116, WindowGraphAggregation.java:54-58): the reference keys the
edges by the partition index of the map subtask that saw them (InitialMapper), folds each partition's
window separately, and its parallelism-1 Merger emits the running state after EVERY partial it receives.
At environment parallelism P a window therefore emits one state per non-empty partition, the last of
them the state after the whole window (the only one ConnectedComponentsTest reads: its parser takes the
last line).  The mirror deals the edges to the P partitions as Flink's rebalance from a parallelism-1
source does (round robin over the stream's arrival order) and emits the states after partials 0, 1, ...
in partition order -- one of the orders the reference's merger can see (the partials race to it)."""
from __future__ import annotations

import numpy as np

from .stream import DataStream, WindowOutput, _take


class WindowGraphAggregation:
    """WindowGraphAggregation.java:30-65: windowed fold + merge of a graph property."""

    def __init__(self, mergeWindowTime: int):
        self.mergeWindowTime = int(mergeWindowTime)

    def run(self, stream) -> DataStream:
        raise NotImplementedError


class ConnectedComponents(WindowGraphAggregation):
    """library/ConnectedComponents.java: weakly connected components, merged across windows."""

    def run(self, stream) -> DataStream:
        env = stream.getContext()
        eng = env.engine
        P = env.getParallelism()
        out = DataStream()
        state = None
        for start, end, w, idx in stream._windows(self.mergeWindowTime, with_index=True):
            if P == 1:
                state = eng.components(w.src, w.dst, state)
                out.windows.append(WindowOutput(start, end, state))
                continue
            part = np.asarray(idx) % P   # rebalance: record i of the stream to map subtask i mod P
            for k in range(P):
                sel = np.flatnonzero(part == k)
                if len(sel) == 0:   # no fold window for a partition without records: no partial, no emission
                    continue
                state = eng.components(_take(w.src, sel), _take(w.dst, sel), state)
                out.windows.append(WindowOutput(start, end, state))
        return out
