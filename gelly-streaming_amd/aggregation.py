"""GraphStream.aggregate(...) for the one aggregation the reference's library ships: ConnectedComponents
(library/ConnectedComponents.java:43-131 on WindowGraphAggregation.java:30-65 and GraphAggregation.java's
Merger).

Per tumbling window of `mergeWindowTime` ms the reference folds the window's edges into a DisjointSet
(UpdateCC -> union) and the parallelism-1 Merger combines it into its running state (CombineCC ->
DisjointSet.merge; transientState = false, so the state accumulates over windows) and emits the state.
Here each window is one gs_window_components call on the GPU with the previous state as input: the
emitted record per vertex is (vertex, smallest vertex of its component) -- the partition DisjointSet
holds (its toString groups by root; which vertex is the root depends on HashMap order)."""
from __future__ import annotations

from .stream import DataStream, WindowOutput


class WindowGraphAggregation:
    """WindowGraphAggregation.java:30-65: windowed fold + merge of a graph property."""

    def __init__(self, mergeWindowTime: int):
        self.mergeWindowTime = int(mergeWindowTime)

    def run(self, stream) -> DataStream:
        raise NotImplementedError


class ConnectedComponents(WindowGraphAggregation):
    """library/ConnectedComponents.java: weakly connected components, merged across windows."""

    def run(self, stream) -> DataStream:
        eng = stream.getContext().engine
        out = DataStream()
        state = None
        for start, end, w in stream._windows(self.mergeWindowTime):
            state = eng.components(w.src, w.dst, state)
            out.windows.append(WindowOutput(start, end, state))
        return out
