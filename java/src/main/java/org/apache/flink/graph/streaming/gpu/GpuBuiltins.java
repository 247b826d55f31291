/*
 * Built-in neighbourhood functions the engine runs (SURVEY.md §8(b) dispatch rule).  They are ordinary
 * EdgesReduce / EdgesFold implementations -- on the unchanged Flink path they compute exactly what
 * they name -- and GraphWindowStream routes an instance of them to GpuWindowOperator instead.  Any
 * other lambda stays on Flink's window functions (GraphWindowStream.java:63, 102, 131).
 */
package org.apache.flink.graph.streaming.gpu;

import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.graph.streaming.EdgesFold;
import org.apache.flink.graph.streaming.EdgesReduce;

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

	/** gs_dtype of an edge value class (NullValue / anything else: GS_NONE). */
	public static int dtypeOf(Class<?> c) {
		if (c == Integer.class) return GellyHip.GS_I32;
		if (c == Long.class) return GellyHip.GS_I64;
		if (c == Float.class) return GellyHip.GS_F32;
		if (c == Double.class) return GellyHip.GS_F64;
		return GellyHip.GS_NONE;
	}
}
