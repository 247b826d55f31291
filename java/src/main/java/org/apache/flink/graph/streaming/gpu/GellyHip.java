/*
 * JNI binding of libgellyhip.so (include/gelly_hip.h), the MI355X engine behind gelly-streaming's
 * per-window neighbourhood path.  Java 7 compatible (the reference targets 1.7, pom.xml:61-64).
 *
 * Every native method wraps one C entry point (java/src/main/c/gellyhip_jni.c).  Columns cross as
 * direct ByteBuffers (host memory: gs_mem GS_MEM_HOST); a non-zero gs_status is thrown as a
 * RuntimeException carrying gs_last_error(ctx), the `throws Exception` of EdgesReduce.java:43 /
 * EdgesFold.java:47 / EdgesApply.java:47.  The constants below must equal the header's enums
 * (tests/test_abi.py parses both files and compares them).
 */
package org.apache.flink.graph.streaming.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

public final class GellyHip {

	static {
		System.loadLibrary("gellyhip_jni");   // java/Makefile: links libgellyhip.so
		// the shim was compiled against one gelly_hip.h: refuse a library of another ABI (struct layouts and
		// entry point signatures change with GS_ABI_VERSION) instead of passing it wrong arguments
		final int abi = abiVersion();
		if (abi != GS_ABI_VERSION)
			throw new UnsatisfiedLinkError("libgellyhip.so has ABI " + abi + ", this binding needs " + GS_ABI_VERSION);
	}

	private GellyHip() {
	}

	public static final int GS_ABI_VERSION = 2;

	/* gs_status */
	public static final int GS_OK = 0;
	public static final int GS_EINVAL = -1;
	public static final int GS_ECAPACITY = -2;
	public static final int GS_EDEVICE = -3;
	public static final int GS_ECOMM = -4;
	public static final int GS_ENOMEM = -5;
	public static final int GS_EUNSUPPORTED = -6;
	public static final int GS_EAGAIN = -7;

	/* gs_dir: org.apache.flink.graph.EdgeDirection's ordinals (IN, OUT, ALL) */
	public static final int GS_DIR_IN = 0;
	public static final int GS_DIR_OUT = 1;
	public static final int GS_DIR_ALL = 2;

	/* gs_op: the built-in reducers / folds */
	public static final int GS_OP_SUM = 0;
	public static final int GS_OP_MIN = 1;
	public static final int GS_OP_MAX = 2;
	public static final int GS_OP_COUNT = 3;

	/* gs_dtype: Integer, Long, Float, Double, NullValue */
	public static final int GS_I32 = 0;
	public static final int GS_I64 = 1;
	public static final int GS_F32 = 2;
	public static final int GS_F64 = 3;
	public static final int GS_NONE = 4;

	/* gs_mem */
	public static final int GS_MEM_HOST = 0;
	public static final int GS_MEM_DEVICE = 1;

	/* gs_stream_config.kind / watermark_mode / staging */
	public static final int GS_STREAM_REDUCE = 0;
	public static final int GS_STREAM_FOLD = 1;
	public static final int GS_STREAM_DEGREE_MAX = 2;
	public static final int GS_STREAM_TRIANGLES = 3;
	public static final int GS_WATERMARK_EXPLICIT = 0;
	public static final int GS_WATERMARK_ASCENDING = 1;
	public static final int GS_STAGE_PINNED = 0;
	public static final int GS_STAGE_DIRECT = 1;
	public static final int GS_LATE_REFIRE = 0;   // Flink 1.0.3 WindowOperator: a late record re-fires its window
	public static final int GS_LATE_DROP = 1;

	/* gs_set_timing levels */
	public static final int GS_TIMING_OFF = 0;
	public static final int GS_TIMING_DOMINANT = 1;
	public static final int GS_TIMING_STAGES = 2;

	/* ---- lifecycle: gs_abi_version, gs_create / gs_destroy ---------------------------------------- */
	static native int abiVersion();

	/** gs_create: one ctx (HIP stream + workspace) per Flink subtask thread; returns the gs_ctx*. */
	static native long create(int device, int flags, long reserveEdges);

	static native void destroy(long ctx);

	/** gs_device_count: HIP devices visible to this JVM (the GPU operators' parallelism, GpuBuiltins). */
	static native int deviceCount();

	/** gs_set_timing: which stage-time events a window records (GS_TIMING_*; the operators run OFF). */
	static native void setTiming(long ctx, int level);

	/** gs_set_max_window_records: records per engine pass (larger reduce / fold windows run in chunks). */
	static native void setMaxWindowRecords(long ctx, long maxRecords);

	/* ---- per-window operators (one tumbling window as SoA columns) ------------------------------------
	 * Each returns the rows written, or -(rows needed) when the output buffers are too small (GS_ECAPACITY:
	 * grow them and call fetchLastOutput / fetchLastDegreeOutput, which deliver without recomputing). */

	/** gs_window_reduce: reduceOnEdges with a built-in op (GraphWindowStream.java:101-121). */
	static native long windowReduce(long ctx, ByteBuffer src, ByteBuffer dst, ByteBuffer val, long n, int valDtype,
			int direction, int op, ByteBuffer outKeys, ByteBuffer outVals, long capacity);

	/** gs_window_fold: foldNeighbors(init, built-in op) (GraphWindowStream.java:62-87); init = one value. */
	static native long windowFold(long ctx, ByteBuffer src, ByteBuffer dst, ByteBuffer val, long n, int valDtype,
			int direction, int op, ByteBuffer init, ByteBuffer outKeys, ByteBuffer outVals, long capacity);

	/** gs_window_fold_degree_max: the (vertex, degree, max neighbour) fold. */
	static native long windowFoldDegreeMax(long ctx, ByteBuffer src, ByteBuffer dst, long n, int direction,
			long initMax, ByteBuffer outKeys, ByteBuffer outDeg, ByteBuffer outMax, long capacity);

	static native long fetchLastOutput(long ctx, ByteBuffer outKeys, ByteBuffer outVals, long capacity);

	static native long fetchLastDegreeOutput(long ctx, ByteBuffer outKeys, ByteBuffer outDeg, ByteBuffer outMax,
			long capacity);

	/** gs_window_triangles: WindowTriangles.java:61-66 for one window -> {exact, Integer emitted, hasOutput}. */
	static native long[] windowTriangles(long ctx, ByteBuffer src, ByteBuffer dst, long n);

	/**
	 * gs_candidates_begin_part: GenerateCandidateEdges (WindowTriangles.java:83-116) over one window's
	 * columns, emitting the vertices v with owner(v, nparts) == part (nparts 1: every vertex; the columns
	 * hold every edge incident to them, GpuBuiltins.RouteToOwners); returns {record count, JDK flags}
	 * (flags bit 0: a neighbour set used a treeified HashMap bin, bit 1: a bin of 9 forced a resize below
	 * capacity 64 -- both simulated exactly).
	 */
	static native long[] candidatesBegin(long ctx, ByteBuffer src, ByteBuffer dst, long n, int nparts, int part);

	/**
	 * gs_candidates_next: the next records of the session into (a, b, isCandidate); returns {records
	 * written, global position of the first, done (1 after the last record)}.
	 */
	static native long[] candidatesNext(long ctx, ByteBuffer a, ByteBuffer b, ByteBuffer isCandidate, long capacity);

	/** gs_candidates_seek: the next candidatesNext starts at output position `record`. */
	static native void candidatesSeek(long ctx, long record);

	/** gs_candidates_vertex_range: {first position, records} of one vertex's block in the session. */
	static native long[] candidatesVertexRange(long ctx, long vertex);

	/**
	 * gs_window_components: ConnectedComponents (library/ConnectedComponents.java:56-131) over one window:
	 * the previous state's m (vertex, label) rows merged with the window's n edges into out (every vertex
	 * seen so far, ascending, labelled by its component's smallest vertex).  Returns the rows written, or
	 * -(rows needed) when capacity is short (m + 2n always suffices).
	 */
	static native long windowComponents(long ctx, ByteBuffer src, ByteBuffer dst, long n, ByteBuffer prevKeys,
			ByteBuffer prevLabels, long m, ByteBuffer outKeys, ByteBuffer outLabels, long capacity);

	/* ---- the window-buffer operator (gs_stream_*): event-time tumbling windows ------------------------ */
	static native long streamCreate(long ctx, long windowMs, int kind, int direction, int op, int valDtype,
			int watermarkMode, int staging, ByteBuffer init, long initMax, long maxWindowEdges, int lateMode);

	static native void streamDestroy(long stream);

	/** gs_stream_append: n records (columns of direct buffers; val null for NullValue edges). */
	static native void streamAppend(long stream, ByteBuffer src, ByteBuffer dst, ByteBuffer val, ByteBuffer ts,
			long n);

	/** gs_stream_watermark: fires every window with end - 1 <= watermark. */
	static native void streamWatermark(long stream, long watermark);

	/** gs_stream_flush: end of a finite source (watermark Long.MAX_VALUE). */
	static native void streamFlush(long stream);

	/**
	 * gs_stream_poll: the next fired window, or false (GS_EAGAIN) when none is ready and !wait.
	 * meta = {window_start, window_end, max_timestamp, edges, n_vertices, triangles, triangles_ref, has_output};
	 * rows[0..2] = views of the pinned result rows (keys, vals, vals2), valid until the next poll.
	 */
	static native boolean streamPoll(long stream, boolean wait, long[] meta, ByteBuffer[] rows);

	/** gs_stream_stats -> {watermark, open, fired, pending, late records, edges fired}. */
	static native long[] streamStats(long stream);

	/** A direct buffer in the platform's byte order (the C side reads int64 / double natively). */
	static ByteBuffer direct(long bytes) {
		return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
	}
}
