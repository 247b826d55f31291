/*
 * One event-time window's edges as growable direct columns (src, dst int64, arrival order): what
 * gs_candidates_begin_part / gs_window_components read without a copy.  Used by GpuCandidatesOperator and
 * GpuComponentsOperator, which buffer whole windows (start = ts - ts % size, Flink 1.0.3
 * TumblingEventTimeWindows) and fire them on the watermark.
 */
package org.apache.flink.graph.streaming.gpu;

import java.nio.ByteBuffer;

final class WindowColumns {
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
