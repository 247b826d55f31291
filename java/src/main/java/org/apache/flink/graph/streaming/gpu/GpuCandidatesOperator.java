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
 * One operator subtask owns one gs_ctx; the window's edges must all reach it (parallelism 1, or one
 * subtask per owner partition fed through GellyHip's owner routing and gs_window_candidates_part).
 */
package org.apache.flink.graph.streaming.gpu;

import java.nio.ByteBuffer;
import java.util.Map;
import java.util.TreeMap;

import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.graph.Edge;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;

@SuppressWarnings("serial")
public class GpuCandidatesOperator<EV> extends AbstractStreamOperator<Tuple3<Long, Long, Boolean>>
		implements OneInputStreamOperator<Edge<Long, EV>, Tuple3<Long, Long, Boolean>> {

	private static final int CHUNK = 1 << 20;   // records per gs_candidates_next

	private final long windowMs;
	private final int device;

	private transient long ctx;
	private transient TreeMap<Long, Columns> open;   // window start -> its edges, in arrival order
	private transient ByteBuffer a, b, f;

	/** one window's edges as growable direct columns (what gs_candidates_begin reads, no copy) */
	private static final class Columns {
		ByteBuffer src = GellyHip.direct(8L * 1024), dst = GellyHip.direct(8L * 1024);
		int n;

		void add(long s, long d) {
			if ((long) (n + 1) * 8 > src.capacity()) {   // a direct buffer holds < 2^31 bytes: 2^28 edges per window
				src = grow(src);
				dst = grow(dst);
			}
			src.putLong(n * 8, s);
			dst.putLong(n * 8, d);
			++n;
		}

		private static ByteBuffer grow(ByteBuffer old) {
			final ByteBuffer nb = GellyHip.direct(2L * old.capacity());
			old.clear();
			nb.put(old);
			nb.clear();
			return nb;
		}
	}

	public GpuCandidatesOperator(long windowMs, int device) {
		this.windowMs = windowMs;
		this.device = device;
	}

	@Override
	public void open() throws Exception {
		super.open();
		ctx = GellyHip.create(device, 0, 0);
		GellyHip.setTiming(ctx, GellyHip.GS_TIMING_OFF);   // no stage-time events in production
		open = new TreeMap<Long, Columns>();
		a = GellyHip.direct(8L * CHUNK);
		b = GellyHip.direct(8L * CHUNK);
		f = GellyHip.direct(CHUNK);
	}

	@Override
	public void processElement(StreamRecord<Edge<Long, EV>> element) throws Exception {
		final long ts = element.getTimestamp();
		final long start = ts - ts % windowMs;   // Java remainder, as TumblingEventTimeWindows
		Columns w = open.get(start);
		if (w == null) open.put(start, w = new Columns());
		final Edge<Long, EV> e = element.getValue();
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
			final Map.Entry<Long, Columns> first = open.firstEntry();
			final long stamp = first.getKey() + windowMs - 1;
			if (stamp > watermark) return;
			open.remove(first.getKey());
			emitWindow(first.getValue(), stamp);
		}
	}

	private void emitWindow(Columns w, long stamp) {
		final long total = GellyHip.candidatesBegin(ctx, w.src, w.dst, w.n)[0];
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
