/*
 * The window-buffer operator that replaces keyBy(vertex).timeWindow(size) + the window function for the
 * built-ins (SimpleEdgeStream.java:153-171, GraphWindowStream.java:49-53, 62-182).  Records are batched
 * into direct column buffers and appended to the library's event-time window buffer (gs_stream_*:
 * start = ts - ts % size, Flink 1.0.3 TumblingEventTimeWindows); a watermark fires every window with
 * end - 1 <= watermark, and each fired window's rows are emitted with the timestamp end - 1
 * (window.maxTimestamp(), what Flink stamps window results with) before the watermark is forwarded: the
 * operator waits for every window the watermark fired (their H2D copies and kernels are in flight when
 * gs_stream_watermark returns), as Flink 1.0.3's WindowOperator emits results before the watermark.
 * Emitting after it would stamp rows end - 1 <= a watermark already sent: late downstream, where e.g.
 * WindowTriangles.java:66's timeWindowAll(..).sum(0) would split one window's count over two panes.
 *
 * One operator subtask owns one gs_ctx (one HIP stream + workspace: gelly_hip.h "Conventions") on device
 * subtask % devices.  neighborhood() builds it the way keyBy would (SimpleEdgeStream.java:159-167): one
 * subtask over the whole stream, or P subtasks behind partitionCustom(OwnerPartitioner) on the
 * direction-expanded records, so every record of a vertex reaches the subtask that owns it.  Flink 1.0.3
 * operator API.
 */
package org.apache.flink.graph.streaming.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

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
import org.apache.flink.streaming.api.windowing.time.Time;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;

@SuppressWarnings("serial")
public class GpuWindowOperator<EV, OUT extends Tuple> extends AbstractStreamOperator<OUT>
		implements OneInputStreamOperator<Edge<Long, EV>, OUT> {

	private static final int BATCH = 1 << 16;   // records per gs_stream_append

	private final long windowMs;
	private final int kind, direction, op, valDtype;
	private final Object init;                  // FOLD: the fold's initial value (its f1); DEGREE_MAX: Long
	private final long maxWindowEdges;

	private transient long ctx, stream;
	private transient ByteBuffer src, dst, val, ts;
	private transient int buffered;
	private transient long[] meta;
	private transient ByteBuffer[] rows;

	/**
	 * @param kind GellyHip.GS_STREAM_REDUCE / _FOLD / _DEGREE_MAX / _TRIANGLES
	 * @param init FOLD: the initial value (Long / Integer / Float / Double); DEGREE_MAX: the initial maximum
	 */
	public GpuWindowOperator(long windowMs, int kind, int direction, int op, int valDtype, Object init,
			long maxWindowEdges) {
		this.windowMs = windowMs;
		this.kind = kind;
		this.direction = direction;
		this.op = op;
		this.valDtype = valDtype;
		this.init = init;
		this.maxWindowEdges = maxWindowEdges;
	}

	/**
	 * reduceOnEdges / foldNeighbors with a built-in on the engine (GraphWindowStream.java:62-121).
	 * edges: the stream before keyBy; keyed: the direction-expanded records keyBy sees (getEdges(),
	 * reverse() or undirected(): SimpleEdgeStream.java:153-171).  At parallelism 1 the operator expands the
	 * direction itself on the original edges; at P > 1 the keyed records are partitioned by their key's
	 * owner and every subtask reduces its share as OUT (each vertex's records all on one subtask).
	 */
	@SuppressWarnings({"unchecked", "rawtypes"})
	public static <EV, OUT extends Tuple> DataStream<OUT> neighborhood(String name, DataStream<Edge<Long, EV>> edges,
			DataStream<Edge<Long, EV>> keyed, long windowMs, int kind, int direction, int op, int valDtype, Object init,
			TypeInformation<OUT> type) {
		final int p = GpuBuiltins.parallelism(edges.getExecutionEnvironment().getParallelism());
		if (p == 1)
			return edges.transform(name, type, new GpuWindowOperator<EV, OUT>(windowMs, kind, direction, op, valDtype,
					init, 0)).setParallelism(1);
		return keyed.partitionCustom(new GpuBuiltins.OwnerPartitioner(), 0).transform(name, type,
				new GpuWindowOperator<EV, OUT>(windowMs, kind, GellyHip.GS_DIR_OUT, op, valDtype, init, 0))
				.setParallelism(p);
	}

	@Override
	public void open() throws Exception {
		super.open();
		final int device = GpuBuiltins.deviceFor(getRuntimeContext().getIndexOfThisSubtask());
		ctx = GellyHip.create(device, 0, maxWindowEdges);
		GellyHip.setTiming(ctx, GellyHip.GS_TIMING_OFF);   // no stage-time events in production
		ByteBuffer initBuf = null;
		long initMax = Long.MIN_VALUE;
		if (kind == GellyHip.GS_STREAM_FOLD) {
			initBuf = GellyHip.direct(8);
			if (op == GellyHip.GS_OP_COUNT) initBuf.putLong(0, ((Number) init).longValue());   // I64 for COUNT
			else putValue(initBuf, 0, init);
		} else if (kind == GellyHip.GS_STREAM_DEGREE_MAX && init != null) {
			initMax = (Long) init;
		}
		stream = GellyHip.streamCreate(ctx, windowMs, kind, direction, op, valDtype, GellyHip.GS_WATERMARK_EXPLICIT,
				GellyHip.GS_STAGE_PINNED, initBuf, initMax, maxWindowEdges, GellyHip.GS_LATE_REFIRE);
		src = GellyHip.direct(8L * BATCH);
		dst = GellyHip.direct(8L * BATCH);
		val = valDtype == GellyHip.GS_NONE ? null : GellyHip.direct(8L * BATCH);
		ts = GellyHip.direct(8L * BATCH);
		meta = new long[8];
		rows = new ByteBuffer[3];
	}

	@Override
	public void processElement(StreamRecord<Edge<Long, EV>> element) throws Exception {
		final Edge<Long, EV> e = element.getValue();
		final int at = buffered * 8;
		src.putLong(at, e.f0);
		dst.putLong(at, e.f1);
		if (val != null) putValue(val, buffered, e.f2);
		ts.putLong(at, element.getTimestamp());
		if (++buffered == BATCH) appendBatch();
	}

	@Override
	public void processWatermark(Watermark mark) throws Exception {
		appendBatch();
		GellyHip.streamWatermark(stream, mark.getTimestamp());
		emitFired(true);   // every window this watermark fired, before the watermark goes downstream
		output.emitWatermark(mark);
	}

	@Override
	public void close() throws Exception {
		appendBatch();
		GellyHip.streamFlush(stream);   // end of a finite source: every open window fires
		emitFired(true);
		super.close();
	}

	@Override
	public void dispose() {
		if (stream != 0) GellyHip.streamDestroy(stream);
		if (ctx != 0) GellyHip.destroy(ctx);
		stream = ctx = 0;
	}

	private void appendBatch() {
		if (buffered == 0) return;
		GellyHip.streamAppend(stream, src, dst, val, ts, buffered);
		buffered = 0;
	}

	/** every fired window's rows, stamped end - 1; drain: wait until the stream has none pending */
	@SuppressWarnings("unchecked")
	private void emitFired(boolean drain) {
		while (GellyHip.streamPoll(stream, drain && pending() > 0, meta, rows)) {
			for (int k = 0; k < rows.length; ++k)   // views of native rows: the platform's byte order
				if (rows[k] != null) rows[k].order(ByteOrder.nativeOrder());
			final long stamp = meta[2];
			final int n = (int) meta[4];
			final StreamRecord<OUT> rec = new StreamRecord<OUT>(null, stamp);
			if (kind == GellyHip.GS_STREAM_TRIANGLES) {
				if (meta[7] != 0)   // Tuple2<Integer, Long>(candidates sum, window end - 1): WindowTriangles.java:66
					output.collect(rec.replace((OUT) new Tuple2<Integer, Long>((int) meta[6], stamp), stamp));
				continue;
			}
			for (int i = 0; i < n; ++i) {
				final long key = rows[0].getLong(i * 8);
				final OUT t;
				if (kind == GellyHip.GS_STREAM_DEGREE_MAX)
					t = (OUT) new Tuple3<Long, Long, Long>(key, rows[1].getLong(i * 8), rows[2].getLong(i * 8));
				else
					t = (OUT) new Tuple2<Long, Object>(key, getValue(rows[1], i));
				output.collect(rec.replace(t, stamp));
			}
		}
	}

	/**
	 * WindowTriangles.java:61-66 in one operator: slice(ALL) -> GenerateCandidateEdges -> keyBy(0, 1)
	 * CountTriangles -> timeWindowAll(size).sum(0), i.e. one Tuple2<Integer, Long>(count as Integer, end - 1)
	 * per window with output (gs_stream TRIANGLES).  Parallelism 1, as the reference's timeWindowAll.
	 */
	@SuppressWarnings({"unchecked", "rawtypes"})
	public static <EV> DataStream<Tuple2<Integer, Long>> windowTriangles(DataStream<Edge<Long, EV>> edges, Time size) {
		final TypeInformation<Tuple2<Integer, Long>> type = new TupleTypeInfo<Tuple2<Integer, Long>>(
				BasicTypeInfo.INT_TYPE_INFO, BasicTypeInfo.LONG_TYPE_INFO);
		return edges.transform("gpu-window-triangles", type,
				new GpuWindowOperator<EV, Tuple2<Integer, Long>>(size.toMilliseconds(), GellyHip.GS_STREAM_TRIANGLES,
						GellyHip.GS_DIR_ALL, 0, GellyHip.GS_NONE, null, 0)).setParallelism(1);
	}

	private long pending() {
		return GellyHip.streamStats(stream)[3];
	}

	private Object getValue(ByteBuffer b, int i) {
		if (op == GellyHip.GS_OP_COUNT) return b.getLong(i * 8);
		switch (valDtype) {
			case GellyHip.GS_I32: return b.getInt(i * 4);
			case GellyHip.GS_F32: return b.getFloat(i * 4);
			case GellyHip.GS_F64: return b.getDouble(i * 8);
			default: return b.getLong(i * 8);
		}
	}

	private void putValue(ByteBuffer b, int i, Object v) {
		switch (valDtype) {
			case GellyHip.GS_I32: b.putInt(i * 4, ((Number) v).intValue()); break;
			case GellyHip.GS_F32: b.putFloat(i * 4, ((Number) v).floatValue()); break;
			case GellyHip.GS_F64: b.putDouble(i * 8, ((Number) v).doubleValue()); break;
			default: b.putLong(i * 8, ((Number) v).longValue());
		}
	}
}
