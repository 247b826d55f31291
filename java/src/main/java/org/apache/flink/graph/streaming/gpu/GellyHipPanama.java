/*
 * The same binding through the Foreign Function & Memory API (JDK 22+, java.lang.foreign): no native
 * shim, libgellyhip.so's C ABI (include/gelly_hip.h) called directly.  An alternative to GellyHip
 * (JNI, Java 7) for a JVM new enough; the operators can use either.  Columns live in MemorySegments
 * (an Arena's, or gs_alloc_pinned memory for zero-copy DMA); a non-zero gs_status is thrown as a
 * RuntimeException with gs_last_error(ctx), the `throws Exception` of EdgesReduce.java:43 /
 * EdgesFold.java:47 / EdgesApply.java:47.  Struct layouts follow the header (tests/test_abi.py checks
 * every entry point this class looks up against it; no JDK exists in the build image, so it is not
 * compiled here).
 */
package org.apache.flink.graph.streaming.gpu;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;

public final class GellyHipPanama implements AutoCloseable {

	/* gs_config, gs_edge_batch, gs_vertex_out, gs_degree_out, gs_pair_out (gelly_hip.h) */
	static final StructLayout CONFIG = MemoryLayout.structLayout(
			JAVA_INT.withName("device"), JAVA_INT.withName("flags"), JAVA_LONG.withName("reserve_edges"));
	static final StructLayout EDGE_BATCH = MemoryLayout.structLayout(
			ADDRESS.withName("src"), ADDRESS.withName("dst"), ADDRESS.withName("val"), JAVA_LONG.withName("n"),
			JAVA_INT.withName("val_dtype"), JAVA_INT.withName("mem"), JAVA_LONG.withName("window_end_ms"));
	static final StructLayout VERTEX_OUT = MemoryLayout.structLayout(
			ADDRESS.withName("keys"), ADDRESS.withName("vals"), JAVA_LONG.withName("capacity"),
			ADDRESS.withName("n_out"), JAVA_INT.withName("mem"), JAVA_INT.withName("reserved"));
	static final StructLayout DEGREE_OUT = MemoryLayout.structLayout(
			ADDRESS.withName("keys"), ADDRESS.withName("degree"), ADDRESS.withName("max_neighbor"),
			JAVA_LONG.withName("capacity"), ADDRESS.withName("n_out"), JAVA_INT.withName("mem"),
			JAVA_INT.withName("reserved"));
	static final StructLayout PAIR_OUT = MemoryLayout.structLayout(
			ADDRESS.withName("a"), ADDRESS.withName("b"), ADDRESS.withName("is_candidate"),
			JAVA_LONG.withName("capacity"), ADDRESS.withName("n_out"), JAVA_INT.withName("mem"),
			JAVA_INT.withName("reserved"));

	private static final Linker LINKER = Linker.nativeLinker();
	private static final SymbolLookup LIB = SymbolLookup.libraryLookup("libgellyhip.so", Arena.global());

	private static MethodHandle fn(String name, FunctionDescriptor d) {
		return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
	}

	private static final MethodHandle CREATE = fn("gs_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
	private static final MethodHandle DESTROY = fn("gs_destroy", FunctionDescriptor.ofVoid(ADDRESS));
	private static final MethodHandle LAST_ERROR = fn("gs_last_error", FunctionDescriptor.of(ADDRESS, ADDRESS));
	private static final MethodHandle WINDOW_REDUCE = fn("gs_window_reduce",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS));
	private static final MethodHandle WINDOW_FOLD_DEGREE_MAX = fn("gs_window_fold_degree_max",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, JAVA_LONG, ADDRESS));
	private static final MethodHandle WINDOW_TRIANGLES = fn("gs_window_triangles",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS, ADDRESS));
	private static final MethodHandle CANDIDATES_BEGIN = fn("gs_candidates_begin_part",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS, ADDRESS));
	private static final MethodHandle DEVICE_COUNT = fn("gs_device_count", FunctionDescriptor.of(JAVA_INT, ADDRESS));
	private static final MethodHandle ABI_VERSION = fn("gs_abi_version", FunctionDescriptor.of(JAVA_INT));
	private static final MethodHandle CANDIDATES_NEXT = fn("gs_candidates_next",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS));
	private static final MethodHandle FETCH_LAST_OUTPUT = fn("gs_fetch_last_output",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
	private static final MethodHandle SET_TIMING = fn("gs_set_timing", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));

	private final Arena arena = Arena.ofConfined();
	private final MemorySegment ctx;

	/** gs_device_count: HIP devices visible to this process. */
	public static int deviceCount() throws Throwable {
		try (Arena a = Arena.ofConfined()) {
			final MemorySegment n = a.allocate(JAVA_INT);
			final int st = (int) DEVICE_COUNT.invokeExact(n);
			if (st != GellyHip.GS_OK) throw new RuntimeException("gs_device_count: status " + st);
			return n.get(JAVA_INT, 0);
		}
	}

	/** gs_create on `device`: one ctx (HIP stream + workspace) per operator subtask thread. */
	public GellyHipPanama(int device) throws Throwable {
		final int abi = (int) ABI_VERSION.invokeExact();
		if (abi != GellyHip.GS_ABI_VERSION)
			throw new UnsatisfiedLinkError("libgellyhip.so has ABI " + abi + ", this binding needs " + GellyHip.GS_ABI_VERSION);
		final MemorySegment cfg = arena.allocate(CONFIG);
		cfg.set(JAVA_INT, 0, device);
		final MemorySegment out = arena.allocate(ADDRESS);
		final int st = (int) CREATE.invokeExact(cfg, out);
		if (st != GellyHip.GS_OK) throw new RuntimeException("gs_create: status " + st + " (a HIP device is required)");
		ctx = out.get(ADDRESS, 0);
		// no stage events inside operator windows (each hipEventRecord costs the stream a few microseconds)
		check((int) SET_TIMING.invokeExact(ctx, GellyHip.GS_TIMING_OFF), "gs_set_timing");
	}

	@Override
	public void close() throws Throwable {
		DESTROY.invokeExact(ctx);
		arena.close();
	}

	private void check(int st, String what) throws Throwable {
		if (st == GellyHip.GS_OK) return;
		final MemorySegment msg = (MemorySegment) LAST_ERROR.invokeExact(ctx);
		throw new RuntimeException(what + ": status " + st + ": " + msg.reinterpret(4096).getString(0));
	}

	private MemorySegment batch(MemorySegment src, MemorySegment dst, MemorySegment val, long n, int dtype) {
		final MemorySegment b = arena.allocate(EDGE_BATCH);
		b.set(ADDRESS, 0, src);
		b.set(ADDRESS, 8, dst);
		b.set(ADDRESS, 16, val == null ? MemorySegment.NULL : val);
		b.set(JAVA_LONG, 24, n);
		b.set(JAVA_INT, 32, val == null ? GellyHip.GS_NONE : dtype);
		b.set(JAVA_INT, 36, GellyHip.GS_MEM_HOST);
		return b;
	}

	/**
	 * gs_window_reduce (reduceOnEdges with a built-in op, GraphWindowStream.java:101-121): the rows written,
	 * or -(rows needed) when keys / vals hold fewer (grow them and call fetchLastOutput).
	 */
	public long windowReduce(MemorySegment src, MemorySegment dst, MemorySegment val, long n, int dtype, int dir,
			int op, MemorySegment keys, MemorySegment vals, long capacity) throws Throwable {
		final MemorySegment nOut = arena.allocate(JAVA_LONG);
		final MemorySegment o = arena.allocate(VERTEX_OUT);
		o.set(ADDRESS, 0, keys);
		o.set(ADDRESS, 8, vals);
		o.set(JAVA_LONG, 16, capacity);
		o.set(ADDRESS, 24, nOut);
		o.set(JAVA_INT, 32, GellyHip.GS_MEM_HOST);
		final int st = (int) WINDOW_REDUCE.invokeExact(ctx, batch(src, dst, val, n, dtype), dir, op, o);
		if (st == GellyHip.GS_ECAPACITY) return -nOut.get(JAVA_LONG, 0);
		check(st, "gs_window_reduce");
		return nOut.get(JAVA_LONG, 0);
	}

	/** gs_fetch_last_output: the rows a GS_ECAPACITY reduce left staged, without recomputing the window. */
	public long fetchLastOutput(MemorySegment keys, MemorySegment vals, long capacity) throws Throwable {
		final MemorySegment nOut = arena.allocate(JAVA_LONG);
		final MemorySegment o = arena.allocate(VERTEX_OUT);
		o.set(ADDRESS, 0, keys);
		o.set(ADDRESS, 8, vals);
		o.set(JAVA_LONG, 16, capacity);
		o.set(ADDRESS, 24, nOut);
		o.set(JAVA_INT, 32, GellyHip.GS_MEM_HOST);
		check((int) FETCH_LAST_OUTPUT.invokeExact(ctx, o), "gs_fetch_last_output");
		return nOut.get(JAVA_LONG, 0);
	}

	/** gs_window_fold_degree_max (foldNeighbors(degree, max neighbour), BASELINE C3). */
	public long windowFoldDegreeMax(MemorySegment src, MemorySegment dst, long n, int dir, long initMax,
			MemorySegment keys, MemorySegment degree, MemorySegment maxNeighbor, long capacity) throws Throwable {
		final MemorySegment nOut = arena.allocate(JAVA_LONG);
		final MemorySegment o = arena.allocate(DEGREE_OUT);
		o.set(ADDRESS, 0, keys);
		o.set(ADDRESS, 8, degree);
		o.set(ADDRESS, 16, maxNeighbor);
		o.set(JAVA_LONG, 24, capacity);
		o.set(ADDRESS, 32, nOut);
		o.set(JAVA_INT, 40, GellyHip.GS_MEM_HOST);
		final int st = (int) WINDOW_FOLD_DEGREE_MAX.invokeExact(ctx, batch(src, dst, null, n, GellyHip.GS_NONE), dir,
				initMax, o);
		if (st == GellyHip.GS_ECAPACITY) return -nOut.get(JAVA_LONG, 0);
		check(st, "gs_window_fold_degree_max");
		return nOut.get(JAVA_LONG, 0);
	}

	/** gs_window_triangles (WindowTriangles.java:61-66): {exact count, the Integer emitted, has output}. */
	public long[] windowTriangles(MemorySegment src, MemorySegment dst, long n) throws Throwable {
		final MemorySegment count = arena.allocate(JAVA_LONG), wrapped = arena.allocate(JAVA_INT),
				has = arena.allocate(JAVA_INT);
		check((int) WINDOW_TRIANGLES.invokeExact(ctx, batch(src, dst, null, n, GellyHip.GS_NONE), count, wrapped, has),
				"gs_window_triangles");
		return new long[] {count.get(JAVA_LONG, 0), wrapped.get(JAVA_INT, 0), has.get(JAVA_INT, 0)};
	}

	/**
	 * gs_candidates_begin_part (GenerateCandidateEdges, WindowTriangles.java:83-116; nparts 1 = the whole
	 * window): {records, JDK flags}.
	 */
	public long[] candidatesBegin(MemorySegment src, MemorySegment dst, long n, int nparts, int part) throws Throwable {
		final MemorySegment total = arena.allocate(JAVA_LONG), flags = arena.allocate(JAVA_INT);
		check((int) CANDIDATES_BEGIN.invokeExact(ctx, batch(src, dst, null, n, GellyHip.GS_NONE), nparts, part, total,
				flags), "gs_candidates_begin_part");
		return new long[] {total.get(JAVA_LONG, 0), flags.get(JAVA_INT, 0)};
	}

	/** gs_candidates_next: the next records into (a, b, isCandidate): {records, first position, done}. */
	public long[] candidatesNext(MemorySegment a, MemorySegment b, MemorySegment isCandidate, long capacity)
			throws Throwable {
		final MemorySegment nOut = arena.allocate(JAVA_LONG), first = arena.allocate(JAVA_LONG),
				done = arena.allocate(JAVA_INT);
		final MemorySegment o = arena.allocate(PAIR_OUT);
		o.set(ADDRESS, 0, a);
		o.set(ADDRESS, 8, b);
		o.set(ADDRESS, 16, isCandidate);
		o.set(JAVA_LONG, 24, capacity);
		o.set(ADDRESS, 32, nOut);
		o.set(JAVA_INT, 40, GellyHip.GS_MEM_HOST);
		check((int) CANDIDATES_NEXT.invokeExact(ctx, o, first, done), "gs_candidates_next");
		return new long[] {nOut.get(JAVA_LONG, 0), first.get(JAVA_LONG, 0), done.get(JAVA_INT, 0)};
	}
}
