/*
 * applyOnNeighbors(GenerateCandidateEdges) on the engine (GraphWindowStream.java:130-182 with
 * WindowTriangles.java:83-116): the operator that replaces slice(ALL)'s keyBy(vertex).timeWindow(size) +
 * EdgesWindowFunction for the built-in apply.  It buffers each event-time window's edges as columns
 * (start = ts - ts % size, Flink 1.0.3 TumblingEventTimeWindows), and when a watermark passes a window's
 * end - 1 it streams that window's Tuple3<Long, Long, Boolean>(a, b, isCandidate) records out of one
 * gs_candidates session (gs_candidates_begin, then gs_candidates_next in chunks: a window's output is
 * O(sum d^2), 1.6e11 records for a 1e8-edge R-MAT window), stamped end - 1, in the record order of
 * gs_window_candidates (vertex by vertex, each vertex's records exactly as GenerateCandidateEdges emits
 * them, JDK HashSet order included), all before the watermark is forwarded.
 *
 * A record for a window that already fired (late) opens that window again and fires it at the next
 * watermark with only the late records, as Flink 1.0.3's WindowOperator does without allowed lateness.
 * One operator subtask owns one gs_ctx on device subtask % devices.  applyOnNeighbors() builds it the way
 * slice(ALL)'s keyBy would (SimpleEdgeStream.java:163-167): one subtask over the whole stream, or P
 * subtasks each fed every edge incident to the vertices it owns (GpuBuiltins.RouteToOwners ->
 * partitionCustom), each emitting only those vertices' records (gs_candidates_begin_part).  The input is
 * the edge itself (P = 1) or the routed Tuple2(target subtask, edge).
 */
package org.apache.flink.graph.streaming.gpu;

import java.nio.ByteBuffer;
import java.util.Map;
import java.util.TreeMap;

import org.apache.flink.api.common.typeinfo.BasicTypeInfo;
import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.java.tuple.Tuple;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.api.java.typeutils.TupleTypeInfo;
import org.apache.flink.graph.Edge;
import org.apache.flink.streaming.api.datastream.DataStream;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;

@SuppressWarnings("serial")
public class GpuCandidatesOperator<EV> extends AbstractStreamOperator<Tuple3<Long, Long, Boolean>>
		implements OneInputStreamOperator<Tuple, Tuple3<Long, Long, Boolean>> {

	private static final int CHUNK = 1 << 20;   // records per gs_candidates_next

	private final long windowMs;
	private final int parts;

	private transient long ctx;
	private transient int part;
	private transient TreeMap<Long, WindowColumns> open;   // window start -> its edges, in arrival order
	private transient ByteBuffer a, b, f;

	/** parts: the operator's parallelism (1: every vertex on one subtask) */
	public GpuCandidatesOperator(long windowMs, int parts) {
		this.windowMs = windowMs;
		this.parts = parts;
	}

	/** applyOnNeighbors(GenerateCandidateEdges) over slice(ALL) on the engine (GraphWindowStream.java:130-182). */
	@SuppressWarnings({"unchecked", "rawtypes"})
	public static <EV, T> DataStream<T> applyOnNeighbors(DataStream<Edge<Long, EV>> edges, long windowMs,
			TypeInformation<T> type) {
		final int p = GpuBuiltins.parallelism(edges.getExecutionEnvironment().getParallelism());
		if (p == 1)
			return ((DataStream) edges).transform("gpu-applyOnNeighbors", type, new GpuCandidatesOperator<EV>(windowMs, 1))
					.setParallelism(1);
		final TypeInformation<Tuple2<Integer, Edge<Long, EV>>> routed = new TupleTypeInfo<Tuple2<Integer, Edge<Long, EV>>>(
				BasicTypeInfo.INT_TYPE_INFO, edges.getType());
		return ((DataStream) edges.flatMap(new GpuBuiltins.RouteToOwners<EV>(p)).returns(routed)
				.partitionCustom(new GpuBuiltins.TargetPartitioner(), 0))
				.transform("gpu-applyOnNeighbors", type, new GpuCandidatesOperator<EV>(windowMs, p)).setParallelism(p);
	}

	@Override
	public void open() throws Exception {
		super.open();
		part = getRuntimeContext().getIndexOfThisSubtask();
		if (part >= parts) throw new IllegalStateException("subtask " + part + " of an operator built for " + parts);
		ctx = GellyHip.create(GpuBuiltins.deviceFor(part), 0, 0);
		GellyHip.setTiming(ctx, GellyHip.GS_TIMING_OFF);   // no stage-time events in production
		open = new TreeMap<Long, WindowColumns>();
		a = GellyHip.direct(8L * CHUNK);
		b = GellyHip.direct(8L * CHUNK);
		f = GellyHip.direct(CHUNK);
	}

	@Override
	@SuppressWarnings("unchecked")
	public void processElement(StreamRecord<Tuple> element) throws Exception {
		final long ts = element.getTimestamp();
		final long start = ts - ts % windowMs;   // Java remainder, as TumblingEventTimeWindows
		WindowColumns w = open.get(start);
		if (w == null) open.put(start, w = new WindowColumns());
		final Tuple v = element.getValue();
		final Edge<Long, EV> e = v instanceof Edge ? (Edge<Long, EV>) v : ((Tuple2<Integer, Edge<Long, EV>>) v).f1;
		w.add(e.f0, e.f1);
	}

	@Override
	public void processWatermark(Watermark mark) throws Exception {
		fireUpTo(mark.getTimestamp());
		output.emitWatermark(mark);
	}

	@Override
	public void close() throws Exception {
		fireUpTo(Long.MAX_VALUE);   // end of a finite source: every open window fires
		super.close();
	}

	@Override
	public void dispose() {
		if (ctx != 0) GellyHip.destroy(ctx);
		ctx = 0;
	}

	/** fires, in window order, every buffered window with end - 1 <= watermark */
	private void fireUpTo(long watermark) {
		while (!open.isEmpty()) {
			final Map.Entry<Long, WindowColumns> first = open.firstEntry();
			final long stamp = first.getKey() + windowMs - 1;
			if (stamp > watermark) return;
			open.remove(first.getKey());
			emitWindow(first.getValue(), stamp);
		}
	}

	private void emitWindow(WindowColumns w, long stamp) {
		final long total = GellyHip.candidatesBegin(ctx, w.src, w.dst, w.n, parts, part)[0];
		final StreamRecord<Tuple3<Long, Long, Boolean>> rec = new StreamRecord<Tuple3<Long, Long, Boolean>>(null, stamp);
		long got = 0;
		while (got < total) {
			final long[] r = GellyHip.candidatesNext(ctx, a, b, f, CHUNK);   // {records, first, done}
			final int n = (int) r[0];
			for (int i = 0; i < n; ++i)
				output.collect(rec.replace(new Tuple3<Long, Long, Boolean>(a.getLong(i * 8), b.getLong(i * 8),
						f.get(i) != 0), stamp));
			got += n;
			if (r[2] != 0) break;
		}
	}
}
