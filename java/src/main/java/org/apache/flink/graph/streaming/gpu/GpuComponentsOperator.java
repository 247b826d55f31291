/*
 * ConnectedComponents on the engine (SURVEY.md §8(f)#4): the operator that replaces
 * WindowGraphAggregation.run (WindowGraphAggregation.java:47-65) for library/ConnectedComponents
 * (:56-131).  The reference folds each window's edges into a DisjointSet per partition (UpdateCC:
 * union(src, dst)), and a parallelism-1 Merger combines every partial into the running state with
 * CombineCC (DisjointSet.merge; transientState = false) and emits that state.
 *
 * Here one subtask buffers each event-time window's edges as columns (start = ts - ts % size, Flink 1.0.3
 * TumblingEventTimeWindows) and, when a watermark passes the window's end - 1, runs gs_window_components
 * over the window and the running state (the previous window's (vertex, label) rows): the state after the
 * window, every vertex seen so far labelled by the smallest vertex of its component.  It emits that state
 * as a DisjointSet<Long> stamped end - 1 -- the same partition the reference's merger holds after the
 * window's partials (which vertex DisjointSet keeps as root depends on HashMap iteration order and is not
 * observable: ConnectedComponentsTest compares the components), before the watermark is forwarded.  The
 * reference's merger runs at parallelism 1; so does this operator (the whole window on one GPU).
 *
 * Parallelism (GraphAggregation.java:103-116, WindowGraphAggregation.java:54-58): at environment
 * parallelism P the reference folds each of P partitions separately (InitialMapper keys every edge by the
 * index of the map subtask that saw it) and the Merger emits the running state after EVERY partial, so a
 * window emits one state per non-empty partition, the last one the state after the whole window.  This
 * operator keeps that record stream: it deals the edges to P partitions as Flink's rebalance from a
 * parallelism-1 source does (round robin over arrival order), runs gs_window_components once per non-empty
 * partition in partition order (one of the orders the partials can reach the merger in) and emits the
 * state after each.  P = 1: one call and one state per window.
 */
package org.apache.flink.graph.streaming.gpu;

import java.nio.ByteBuffer;
import java.util.Map;
import java.util.TreeMap;

import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.java.typeutils.TypeExtractor;
import org.apache.flink.graph.Edge;
import org.apache.flink.graph.streaming.example.util.DisjointSet;
import org.apache.flink.streaming.api.datastream.DataStream;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;

@SuppressWarnings("serial")
public class GpuComponentsOperator<EV> extends AbstractStreamOperator<DisjointSet<Long>>
		implements OneInputStreamOperator<Edge<Long, EV>, DisjointSet<Long>> {

	private final long windowMs;
	private final int partitions;   // the reference's fold parallelism: states emitted per window, at most

	private transient long ctx;
	private transient long seq;                              // records seen: record i -> partition i % partitions
	private transient TreeMap<Long, WindowColumns[]> open;   // window start -> its edges per partition, in arrival order
	private transient ByteBuffer keys, labels;             // the running state: m (vertex, label) rows
	private transient long m;

	public GpuComponentsOperator(long windowMs, int partitions) {
		if (partitions < 1) throw new IllegalArgumentException("partitions must be at least 1");
		this.windowMs = windowMs;
		this.partitions = partitions;
	}

	/** SimpleEdgeStream.aggregate(new ConnectedComponents(windowMs)) on the engine. */
	@SuppressWarnings({"unchecked", "rawtypes"})
	public static <EV> DataStream<DisjointSet<Long>> connectedComponents(DataStream<Edge<Long, EV>> edges,
			long windowMs) {
		final TypeInformation<DisjointSet<Long>> type = (TypeInformation) TypeExtractor.getForClass(DisjointSet.class);
		final int p = Math.max(1, edges.getExecutionEnvironment().getParallelism());
		return edges.transform("gpu-connected-components", type, new GpuComponentsOperator<EV>(windowMs, p))
				.setParallelism(1);
	}

	@Override
	public void open() throws Exception {
		super.open();
		ctx = GellyHip.create(GpuBuiltins.deviceFor(getRuntimeContext().getIndexOfThisSubtask()), 0, 0);
		GellyHip.setTiming(ctx, GellyHip.GS_TIMING_OFF);   // no stage-time events in production
		open = new TreeMap<Long, WindowColumns[]>();
		seq = 0;
		keys = GellyHip.direct(8);
		labels = GellyHip.direct(8);
		m = 0;
	}

	@Override
	public void processElement(StreamRecord<Edge<Long, EV>> element) throws Exception {
		final long ts = element.getTimestamp();
		final long start = ts - ts % windowMs;   // Java remainder, as TumblingEventTimeWindows
		WindowColumns[] w = open.get(start);
		if (w == null) open.put(start, w = new WindowColumns[partitions]);
		final int k = (int) (seq++ % partitions);
		if (w[k] == null) w[k] = new WindowColumns();
		final Edge<Long, EV> e = element.getValue();
		w[k].add(e.f0, e.f1);
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

	private void fireUpTo(long watermark) {
		while (!open.isEmpty()) {
			final Map.Entry<Long, WindowColumns[]> first = open.firstEntry();
			final long stamp = first.getKey() + windowMs - 1;
			if (stamp > watermark) return;
			open.remove(first.getKey());
			for (WindowColumns part : first.getValue()) {   // a partition without records has no partial
				if (part != null && part.n > 0) fire(part, stamp);
			}
		}
	}

	/** the state after one partial (CombineCC of the running state and one partition's UpdateCC fold) */
	private void fire(WindowColumns w, long stamp) {
		final long cap = m + 2L * w.n;   // every vertex seen so far at most
		final ByteBuffer ok = GellyHip.direct(8 * cap), ol = GellyHip.direct(8 * cap);
		final long rows = GellyHip.windowComponents(ctx, w.src, w.dst, w.n, keys, labels, m, ok, ol, cap);
		if (rows < 0) throw new IllegalStateException("gs_window_components needs " + (-rows) + " rows of " + cap);
		keys = ok;
		labels = ol;
		m = rows;
		final DisjointSet<Long> ds = new DisjointSet<Long>();
		for (int i = 0; i < m; ++i) ds.makeSet(keys.getLong(i * 8));
		for (int i = 0; i < m; ++i) {   // a label is its component's smallest vertex, itself a row
			final long v = keys.getLong(i * 8), l = labels.getLong(i * 8);
			if (v != l) ds.getMatches().put(v, l);
		}
		output.collect(new StreamRecord<DisjointSet<Long>>(ds, stamp));
	}
}
