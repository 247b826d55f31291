/*
 * Built-in neighbourhood functions the engine runs (SURVEY.md §8(b) dispatch rule).  They are ordinary
 * EdgesReduce / EdgesFold implementations -- on the unchanged Flink path they compute exactly what
 * they name -- and GraphWindowStream routes an instance of them to GpuWindowOperator instead.  Any
 * other lambda stays on Flink's window functions (GraphWindowStream.java:63, 102, 131).
 */
package org.apache.flink.graph.streaming.gpu;

import org.apache.flink.api.common.functions.FlatMapFunction;
import org.apache.flink.api.common.functions.Partitioner;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.graph.Edge;
import org.apache.flink.graph.streaming.EdgesFold;
import org.apache.flink.graph.streaming.EdgesReduce;
import org.apache.flink.util.Collector;

public final class GpuBuiltins {

	private GpuBuiltins() {
	}

	/** A reducer the engine implements: gs_op of the reduction. */
	public interface Builtin {
		int op();
	}

	/** A fold the engine implements: gs_op (or -2 for the degree / max-neighbour fold). */
	public interface BuiltinFold {
		int op();
	}

	/**
	 * An apply function the engine implements: the records of WindowTriangles.GenerateCandidateEdges
	 * (WindowTriangles.java:83-116), which the dispatch patch marks with this interface.  Routed to
	 * GpuCandidatesOperator (gs_candidates_begin / gs_candidates_next).
	 */
	public interface BuiltinApply {
	}

	/** Whether the dispatch is on: -Dgelly.gpu=false keeps every call on the Flink path. */
	public static boolean enabled() {
		return System.getProperty("gelly.gpu", "true").equals("true");
	}

	/**
	 * Whether the engine takes these edges: Long vertex IDs (GpuWindowOperator reads Edge<Long, EV>) and
	 * Integer / Long / Float / Double values, or none (NullValue) when the op needs no values.  Anything
	 * else stays on Flink instead of failing with a ClassCastException in the operator.
	 */
	public static boolean supports(Class<?> keyClass, Class<?> valueClass, boolean needsValues) {
		if (keyClass != Long.class) return false;
		return dtypeOf(valueClass) != GellyHip.GS_NONE || !needsValues;
	}

	/** Long / Integer / Float / Double sum (Java wrapping for the integers). */
	@SuppressWarnings({"serial", "unchecked"})
	public static final class SumReduce<EV extends Number> implements EdgesReduce<EV>, Builtin {
		public int op() { return GellyHip.GS_OP_SUM; }

		public EV reduceEdges(EV a, EV b) {
			if (a instanceof Long) return (EV) Long.valueOf(a.longValue() + b.longValue());
			if (a instanceof Integer) return (EV) Integer.valueOf(a.intValue() + b.intValue());
			if (a instanceof Float) return (EV) Float.valueOf(a.floatValue() + b.floatValue());
			return (EV) Double.valueOf(a.doubleValue() + b.doubleValue());
		}
	}

	@SuppressWarnings({"serial", "unchecked"})
	public static final class MinReduce<EV extends Number> implements EdgesReduce<EV>, Builtin {
		public int op() { return GellyHip.GS_OP_MIN; }

		public EV reduceEdges(EV a, EV b) {
			if (a instanceof Long) return (EV) Long.valueOf(Math.min(a.longValue(), b.longValue()));
			if (a instanceof Integer) return (EV) Integer.valueOf(Math.min(a.intValue(), b.intValue()));
			if (a instanceof Float) return (EV) Float.valueOf(Math.min(a.floatValue(), b.floatValue()));
			return (EV) Double.valueOf(Math.min(a.doubleValue(), b.doubleValue()));
		}
	}

	@SuppressWarnings({"serial", "unchecked"})
	public static final class MaxReduce<EV extends Number> implements EdgesReduce<EV>, Builtin {
		public int op() { return GellyHip.GS_OP_MAX; }

		public EV reduceEdges(EV a, EV b) {
			if (a instanceof Long) return (EV) Long.valueOf(Math.max(a.longValue(), b.longValue()));
			if (a instanceof Integer) return (EV) Integer.valueOf(Math.max(a.intValue(), b.intValue()));
			if (a instanceof Float) return (EV) Float.valueOf(Math.max(a.floatValue(), b.floatValue()));
			return (EV) Double.valueOf(Math.max(a.doubleValue(), b.doubleValue()));
		}
	}

	/** foldNeighbors(new Tuple2<>(k, v0), new SumValuesFold()): (vertex, v0 + sum of values), TestSlice's shape. */
	@SuppressWarnings("serial")
	public static final class SumValuesFold implements EdgesFold<Long, Long, Tuple2<Long, Long>>, BuiltinFold {
		public int op() { return GellyHip.GS_OP_SUM; }

		public Tuple2<Long, Long> foldEdges(Tuple2<Long, Long> acc, Long id, Long neighbor, Long value) {
			acc.setField(id, 0);
			acc.setField(acc.f1 + value, 1);
			return acc;
		}
	}

	/** foldNeighbors(new Tuple2<>(k, v0), new MinValuesFold()): (vertex, min(v0, values)). */
	@SuppressWarnings("serial")
	public static final class MinValuesFold implements EdgesFold<Long, Long, Tuple2<Long, Long>>, BuiltinFold {
		public int op() { return GellyHip.GS_OP_MIN; }

		public Tuple2<Long, Long> foldEdges(Tuple2<Long, Long> acc, Long id, Long neighbor, Long value) {
			acc.setField(id, 0);
			acc.setField(Math.min(acc.f1, value), 1);
			return acc;
		}
	}

	/** foldNeighbors(new Tuple2<>(k, v0), new MaxValuesFold()): (vertex, max(v0, values)). */
	@SuppressWarnings("serial")
	public static final class MaxValuesFold implements EdgesFold<Long, Long, Tuple2<Long, Long>>, BuiltinFold {
		public int op() { return GellyHip.GS_OP_MAX; }

		public Tuple2<Long, Long> foldEdges(Tuple2<Long, Long> acc, Long id, Long neighbor, Long value) {
			acc.setField(id, 0);
			acc.setField(Math.max(acc.f1, value), 1);
			return acc;
		}
	}

	/**
	 * foldNeighbors(new Tuple2<>(k, c0), new CountFold()): (vertex, c0 + the vertex's neighbour records), the
	 * COUNT built-in.  COUNT is a fold, not an EdgesReduce: reduceEdges(EV, EV) combines two edge values and
	 * Flink's reduce starts from the first value, so a reducer cannot count (GraphWindowStream.java:107-121).
	 */
	@SuppressWarnings("serial")
	public static final class CountFold<EV> implements EdgesFold<Long, EV, Tuple2<Long, Long>>, BuiltinFold {
		public int op() { return GellyHip.GS_OP_COUNT; }

		public Tuple2<Long, Long> foldEdges(Tuple2<Long, Long> acc, Long id, Long neighbor, EV value) {
			acc.setField(id, 0);
			acc.setField(acc.f1 + 1, 1);
			return acc;
		}
	}

	/** (vertex, degree, max neighbour) from init (k, 0, m0): BASELINE config C3's fold. */
	@SuppressWarnings("serial")
	public static final class DegreeMaxNeighborFold<EV>
			implements EdgesFold<Long, EV, Tuple3<Long, Long, Long>>, BuiltinFold {
		public int op() { return -2; }

		public Tuple3<Long, Long, Long> foldEdges(Tuple3<Long, Long, Long> acc, Long id, Long neighbor, EV value) {
			acc.setField(id, 0);
			acc.setField(acc.f1 + 1, 1);
			acc.setField(Math.max(acc.f2, neighbor), 2);
			return acc;
		}
	}

	/* ---- parallelism: one operator subtask per GPU ------------------------------------------------------
	 * Flink runs a window operator at the environment's parallelism (local env: the host's cores), and
	 * keyBy(NeighborKeySelector) (SimpleEdgeStream.java:159-167) gives every record of a vertex to one
	 * subtask.  The GPU operators keep that contract: at parallelism 1 one subtask takes the whole stream;
	 * at P > 1 the records go through partitionCustom(OwnerPartitioner) on their key (reduce / folds), or
	 * every edge to the owners of both endpoints (RouteToOwners -> TargetPartitioner, candidates), and
	 * subtask i runs on device i % deviceCount() with its own gs_ctx. */

	/**
	 * The GPU operators' parallelism: min(the environment's parallelism, visible HIP devices), at least 1;
	 * -Dgelly.gpu.parallelism=N overrides it (e.g. several subtasks per device).
	 */
	public static int parallelism(int envParallelism) {
		final String forced = System.getProperty("gelly.gpu.parallelism");
		if (forced != null) return Math.max(1, Integer.parseInt(forced));
		final int devices = Math.max(1, GellyHip.deviceCount());
		return Math.max(1, Math.min(envParallelism > 0 ? envParallelism : devices, devices));
	}

	/** The device a subtask's gs_ctx lives on. */
	public static int deviceFor(int subtaskIndex) {
		return subtaskIndex % Math.max(1, GellyHip.deviceCount());
	}

	/**
	 * gs_owner_of (gs_ops.hpp owner_of): murmur3's 64-bit finaliser of the vertex, scaled to nparts by a
	 * multiply-high -- the same function the library's part entry points (gs_candidates_begin_part) filter
	 * by, so the routing and the emission agree (tests/test_abi.py compares the constants).
	 */
	public static int ownerOf(long v, int nparts) {
		long x = v;
		x ^= x >>> 33;
		x *= 0xff51afd7ed558ccdL;
		x ^= x >>> 33;
		x *= 0xc4ceb9fe1a85ec53L;
		x ^= x >>> 33;
		return (int) (((x >>> 32) * (long) nparts) >>> 32);
	}

	/** keyBy on a Long vertex key: the record goes to subtask ownerOf(key, P). */
	@SuppressWarnings("serial")
	public static final class OwnerPartitioner implements Partitioner<Long> {
		@Override
		public int partition(Long key, int numPartitions) {
			return ownerOf(key, numPartitions);
		}
	}

	/** Records already tagged with their target subtask (RouteToOwners' f0). */
	@SuppressWarnings("serial")
	public static final class TargetPartitioner implements Partitioner<Integer> {
		@Override
		public int partition(Integer target, int numPartitions) {
			return target;
		}
	}

	/**
	 * Every edge to the owners of both its endpoints (once when they are the same subtask), stream order
	 * kept per channel: the subtask that owns v then holds every edge incident to v, which
	 * GenerateCandidateEdges needs (its HashSet is built from all of v's neighbour records).
	 */
	@SuppressWarnings("serial")
	public static final class RouteToOwners<EV> implements FlatMapFunction<Edge<Long, EV>, Tuple2<Integer, Edge<Long, EV>>> {
		private final int parts;

		public RouteToOwners(int parts) {
			this.parts = parts;
		}

		@Override
		public void flatMap(Edge<Long, EV> e, Collector<Tuple2<Integer, Edge<Long, EV>>> out) {
			final int a = ownerOf(e.f0, parts), b = ownerOf(e.f1, parts);
			out.collect(new Tuple2<Integer, Edge<Long, EV>>(a, e));
			if (b != a) out.collect(new Tuple2<Integer, Edge<Long, EV>>(b, e));
		}
	}

	/** gs_dtype of an edge value class (NullValue / anything else: GS_NONE). */
	public static int dtypeOf(Class<?> c) {
		if (c == Integer.class) return GellyHip.GS_I32;
		if (c == Long.class) return GellyHip.GS_I64;
		if (c == Float.class) return GellyHip.GS_F32;
		if (c == Double.class) return GellyHip.GS_F64;
		return GellyHip.GS_NONE;
	}
}
