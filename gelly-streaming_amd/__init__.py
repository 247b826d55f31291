"""gelly-streaming_amd — MI355X-native engine for gelly-streaming's per-window neighbourhood path.

The drop-in boundary is the C ABI of libgellyhip.so (include/gelly_hip.h).  This package is the
host-side mirror of the reference's Java API for that path (SimpleEdgeStream.slice ->
GraphWindowStream.reduceOnEdges / foldNeighbors / applyOnNeighbors, WindowTriangles), the engine
binding, and the multi-GPU window shuffle.

The directory name contains a hyphen, so it is loaded by path:
    import importlib.util, sys
    spec = importlib.util.spec_from_file_location("gelly_streaming_amd", ".../gelly-streaming_amd/__init__.py")
or with ``load_package()`` from __graft_entry__.py.
"""
from ._lib import GsError, load as load_library  # noqa: F401
from .engine import CommGroup, Engine, StageTimes  # noqa: F401
from .functions import (Collector, CountFold, CountReduce, DegreeMaxNeighborFold, EdgesApply, EdgesFold,  # noqa: F401
                        EdgesReduce, MaxReduce, MaxValuesFold, MinReduce, MinValuesFold, SumReduce, SumValuesFold)
from .stream import (AscendingTimestampExtractor, DataStream, EdgeColumns, EdgeDirection,  # noqa: F401
                     EdgeValueTimestampExtractor, GraphWindowStream, SimpleEdgeStream, StreamExecutionEnvironment,
                     Time, TimeUnit)
from .triangles import CountTriangles, GenerateCandidateEdges, window_triangles  # noqa: F401
from .aggregation import ConnectedComponents, WindowGraphAggregation  # noqa: F401

__all__ = [n for n in dir() if not n.startswith("_")]
