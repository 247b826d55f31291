/*
 * gellyhip_jni.c — the JNI shim between org.apache.flink.graph.streaming.gpu.GellyHip and libgellyhip.so
 * (include/gelly_hip.h).  Each function fills the ABI's structs from direct ByteBuffers
 * (GetDirectBufferAddress: host memory, GS_MEM_HOST), calls one entry point and maps a non-zero
 * gs_status to a RuntimeException with gs_last_error(ctx) -- the `throws Exception` of the reference's
 * SAM interfaces (EdgesReduce.java:43, EdgesFold.java:47, EdgesApply.java:47).  GS_ECAPACITY is not
 * thrown: the row count needed comes back negated so the caller grows its buffers and fetches the staged
 * rows (gs_fetch_last_output) without recomputing the window.
 *
 * Build (needs a JDK for jni.h; none exists in this image): java/Makefile.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gelly_hip.h"

#define JNI_FN(name) JNICALL Java_org_apache_flink_graph_streaming_gpu_GellyHip_##name

static void* addr(JNIEnv* env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }

static void throw_status(JNIEnv* env, gs_ctx* ctx, gs_status s, const char* what) {
  char msg[512];
  snprintf(msg, sizeof msg, "%s: status %d: %s", what, (int)s, ctx ? gs_last_error(ctx) : "");
  (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/RuntimeException"), msg);
}

/* rows written, -(rows needed) on GS_ECAPACITY, 0 after a thrown error */
static jlong rows_or_throw(JNIEnv* env, gs_ctx* ctx, gs_status s, uint64_t n_out, const char* what) {
  if (s == GS_OK) return (jlong)n_out;
  if (s == GS_ECAPACITY) return -(jlong)n_out;
  throw_status(env, ctx, s, what);
  return 0;
}

static gs_edge_batch batch(JNIEnv* env, jobject src, jobject dst, jobject val, jlong n, jint dt) {
  gs_edge_batch b;
  memset(&b, 0, sizeof b);
  b.src = (const int64_t*)addr(env, src);
  b.dst = (const int64_t*)addr(env, dst);
  b.val = val ? addr(env, val) : NULL;
  b.n = (uint64_t)n;
  b.val_dtype = val ? dt : GS_NONE;
  b.mem = GS_MEM_HOST;
  return b;
}

JNIEXPORT jint JNI_FN(abiVersion)(JNIEnv* env, jclass cls) { return gs_abi_version(); }

JNIEXPORT jlong JNI_FN(create)(JNIEnv* env, jclass cls, jint device, jint flags, jlong reserve) {
  gs_config cfg = {device, (uint32_t)flags, (uint64_t)reserve};
  gs_ctx* ctx = NULL;
  gs_status s = gs_create(&cfg, &ctx);
  if (s != GS_OK) {
    throw_status(env, NULL, s, "gs_create (a HIP device is required)");
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNI_FN(destroy)(JNIEnv* env, jclass cls, jlong ctx) { gs_destroy((gs_ctx*)(intptr_t)ctx); }

JNIEXPORT jint JNI_FN(deviceCount)(JNIEnv* env, jclass cls) {
  int32_t n = 0;
  gs_status s = gs_device_count(&n);
  if (s != GS_OK) throw_status(env, NULL, s, "gs_device_count");
  return (jint)n;
}

JNIEXPORT void JNI_FN(setTiming)(JNIEnv* env, jclass cls, jlong ctx, jint level) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_status s = gs_set_timing(c, (int32_t)level);
  if (s != GS_OK) throw_status(env, c, s, "gs_set_timing");
}

JNIEXPORT void JNI_FN(setMaxWindowRecords)(JNIEnv* env, jclass cls, jlong ctx, jlong max_records) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_status s = gs_set_max_window_records(c, (uint64_t)max_records);
  if (s != GS_OK) throw_status(env, c, s, "gs_set_max_window_records");
}

JNIEXPORT jlong JNI_FN(windowReduce)(JNIEnv* env, jclass cls, jlong ctx, jobject src, jobject dst, jobject val, jlong n,
                                     jint dt, jint dir, jint op, jobject ok, jobject ov, jlong cap) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_edge_batch b = batch(env, src, dst, val, n, dt);
  uint64_t n_out = 0;
  gs_vertex_out o = {(int64_t*)addr(env, ok), addr(env, ov), (uint64_t)cap, &n_out, GS_MEM_HOST, 0};
  return rows_or_throw(env, c, gs_window_reduce(c, &b, dir, op, &o), n_out, "gs_window_reduce");
}

JNIEXPORT jlong JNI_FN(windowFold)(JNIEnv* env, jclass cls, jlong ctx, jobject src, jobject dst, jobject val, jlong n,
                                   jint dt, jint dir, jint op, jobject init, jobject ok, jobject ov, jlong cap) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_edge_batch b = batch(env, src, dst, val, n, dt);
  uint64_t n_out = 0;
  gs_vertex_out o = {(int64_t*)addr(env, ok), addr(env, ov), (uint64_t)cap, &n_out, GS_MEM_HOST, 0};
  return rows_or_throw(env, c, gs_window_fold(c, &b, dir, op, addr(env, init), &o), n_out, "gs_window_fold");
}

JNIEXPORT jlong JNI_FN(windowFoldDegreeMax)(JNIEnv* env, jclass cls, jlong ctx, jobject src, jobject dst, jlong n,
                                            jint dir, jlong init_max, jobject ok, jobject od, jobject om, jlong cap) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_edge_batch b = batch(env, src, dst, NULL, n, GS_NONE);
  uint64_t n_out = 0;
  gs_degree_out o = {(int64_t*)addr(env, ok), (int64_t*)addr(env, od), (int64_t*)addr(env, om), (uint64_t)cap, &n_out,
                     GS_MEM_HOST, 0};
  return rows_or_throw(env, c, gs_window_fold_degree_max(c, &b, dir, init_max, &o), n_out, "gs_window_fold_degree_max");
}

JNIEXPORT jlong JNI_FN(fetchLastOutput)(JNIEnv* env, jclass cls, jlong ctx, jobject ok, jobject ov, jlong cap) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  uint64_t n_out = 0;
  gs_vertex_out o = {(int64_t*)addr(env, ok), addr(env, ov), (uint64_t)cap, &n_out, GS_MEM_HOST, 0};
  return rows_or_throw(env, c, gs_fetch_last_output(c, &o), n_out, "gs_fetch_last_output");
}

JNIEXPORT jlong JNI_FN(fetchLastDegreeOutput)(JNIEnv* env, jclass cls, jlong ctx, jobject ok, jobject od, jobject om,
                                              jlong cap) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  uint64_t n_out = 0;
  gs_degree_out o = {(int64_t*)addr(env, ok), (int64_t*)addr(env, od), (int64_t*)addr(env, om), (uint64_t)cap, &n_out,
                     GS_MEM_HOST, 0};
  return rows_or_throw(env, c, gs_fetch_last_degree_output(c, &o), n_out, "gs_fetch_last_degree_output");
}

JNIEXPORT jlongArray JNI_FN(windowTriangles)(JNIEnv* env, jclass cls, jlong ctx, jobject src, jobject dst, jlong n) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_edge_batch b = batch(env, src, dst, NULL, n, GS_NONE);
  uint64_t count = 0;
  int32_t wrapped = 0, has = 0;
  gs_status s = gs_window_triangles(c, &b, &count, &wrapped, &has);
  if (s != GS_OK) {
    throw_status(env, c, s, "gs_window_triangles");
    return NULL;
  }
  jlong r[3] = {(jlong)count, (jlong)wrapped, (jlong)has};
  jlongArray out = (*env)->NewLongArray(env, 3);
  (*env)->SetLongArrayRegion(env, out, 0, 3, r);
  return out;
}

static jlongArray long_array(JNIEnv* env, const jlong* v, jsize n) {
  jlongArray out = (*env)->NewLongArray(env, n);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, n, v);
  return out;
}

JNIEXPORT jlongArray JNI_FN(candidatesBegin)(JNIEnv* env, jclass cls, jlong ctx, jobject src, jobject dst, jlong n,
                                             jint nparts, jint part) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_edge_batch b = batch(env, src, dst, NULL, n, GS_NONE);
  uint64_t total = 0;
  uint32_t flags = 0;
  gs_status s = gs_candidates_begin_part(c, &b, (uint32_t)nparts, (uint32_t)part, &total, &flags);
  if (s != GS_OK) {
    throw_status(env, c, s, "gs_candidates_begin_part");
    return NULL;
  }
  const jlong r[2] = {(jlong)total, (jlong)flags};
  return long_array(env, r, 2);
}

JNIEXPORT jlongArray JNI_FN(candidatesNext)(JNIEnv* env, jclass cls, jlong ctx, jobject a, jobject b, jobject f,
                                            jlong cap) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  uint64_t n_out = 0, first = 0;
  int32_t done = 0;
  gs_pair_out o = {(int64_t*)addr(env, a), (int64_t*)addr(env, b), (uint8_t*)addr(env, f), (uint64_t)cap, &n_out,
                   GS_MEM_HOST, 0};
  gs_status s = gs_candidates_next(c, &o, &first, &done);
  if (s != GS_OK) {
    throw_status(env, c, s, "gs_candidates_next");
    return NULL;
  }
  const jlong r[3] = {(jlong)n_out, (jlong)first, (jlong)done};
  return long_array(env, r, 3);
}

JNIEXPORT void JNI_FN(candidatesSeek)(JNIEnv* env, jclass cls, jlong ctx, jlong record) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_status s = gs_candidates_seek(c, (uint64_t)record);
  if (s != GS_OK) throw_status(env, c, s, "gs_candidates_seek");
}

JNIEXPORT jlongArray JNI_FN(candidatesVertexRange)(JNIEnv* env, jclass cls, jlong ctx, jlong vertex) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  uint64_t first = 0, n = 0;
  gs_status s = gs_candidates_vertex_range(c, (int64_t)vertex, &first, &n);
  if (s != GS_OK) {
    throw_status(env, c, s, "gs_candidates_vertex_range");
    return NULL;
  }
  const jlong r[2] = {(jlong)first, (jlong)n};
  return long_array(env, r, 2);
}

JNIEXPORT jlong JNI_FN(windowComponents)(JNIEnv* env, jclass cls, jlong ctx, jobject src, jobject dst, jlong n,
                                         jobject pk, jobject pl, jlong m, jobject ok, jobject ol, jlong cap) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_edge_batch b = batch(env, src, dst, NULL, n, GS_NONE);
  gs_partial_batch prev;
  memset(&prev, 0, sizeof prev);
  prev.keys = (const int64_t*)addr(env, pk);
  prev.vals = addr(env, pl);
  prev.n = (uint64_t)m;
  prev.val_dtype = GS_I64;
  prev.mem = GS_MEM_HOST;
  uint64_t n_out = 0;
  gs_vertex_out o = {(int64_t*)addr(env, ok), addr(env, ol), (uint64_t)cap, &n_out, GS_MEM_HOST, 0};
  return rows_or_throw(env, c, gs_window_components(c, &b, m ? &prev : NULL, &o), n_out, "gs_window_components");
}

/* ---- gs_stream_*: the stream keeps its ctx (one per operator subtask) -------------------------------- */
typedef struct {
  gs_ctx* ctx;
  gs_stream* stream;
  jlong vbytes;   /* bytes per result value: 4 for Integer / Float REDUCE / FOLD results, else 8 */
} jstream;

JNIEXPORT jlong JNI_FN(streamCreate)(JNIEnv* env, jclass cls, jlong ctx, jlong window_ms, jint kind, jint dir, jint op,
                                     jint dt, jint wm_mode, jint staging, jobject init, jlong init_max,
                                     jlong max_edges, jint late_mode) {
  gs_ctx* c = (gs_ctx*)(intptr_t)ctx;
  gs_stream_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.window_ms = window_ms;
  cfg.kind = kind;
  cfg.dir = dir;
  cfg.op = op;
  cfg.val_dtype = dt;
  cfg.watermark_mode = wm_mode;
  cfg.staging = staging;
  cfg.init = addr(env, init);
  cfg.init_max = init_max;
  cfg.max_window_edges = (uint64_t)max_edges;
  cfg.late_mode = late_mode;
  gs_stream* st = NULL;
  gs_status s = gs_stream_create(c, &cfg, &st);
  if (s != GS_OK) {
    throw_status(env, c, s, "gs_stream_create");
    return 0;
  }
  jstream* js = (jstream*)malloc(sizeof(jstream));
  js->ctx = c;
  js->stream = st;
  js->vbytes = (kind == GS_STREAM_REDUCE || kind == GS_STREAM_FOLD) && op != GS_OP_COUNT &&
                       (dt == GS_I32 || dt == GS_F32) ? 4 : 8;
  return (jlong)(intptr_t)js;
}

JNIEXPORT void JNI_FN(streamDestroy)(JNIEnv* env, jclass cls, jlong h) {
  jstream* js = (jstream*)(intptr_t)h;
  if (!js) return;
  gs_stream_destroy(js->stream);
  free(js);
}

JNIEXPORT void JNI_FN(streamAppend)(JNIEnv* env, jclass cls, jlong h, jobject src, jobject dst, jobject val, jobject ts,
                                    jlong n) {
  jstream* js = (jstream*)(intptr_t)h;
  gs_status s = gs_stream_append(js->stream, (const int64_t*)addr(env, src), (const int64_t*)addr(env, dst),
                                 addr(env, val), (const int64_t*)addr(env, ts), (uint64_t)n);
  if (s != GS_OK) throw_status(env, js->ctx, s, "gs_stream_append");
}

JNIEXPORT void JNI_FN(streamWatermark)(JNIEnv* env, jclass cls, jlong h, jlong wm) {
  jstream* js = (jstream*)(intptr_t)h;
  gs_status s = gs_stream_watermark(js->stream, wm);
  if (s != GS_OK) throw_status(env, js->ctx, s, "gs_stream_watermark");
}

JNIEXPORT void JNI_FN(streamFlush)(JNIEnv* env, jclass cls, jlong h) {
  jstream* js = (jstream*)(intptr_t)h;
  gs_status s = gs_stream_flush(js->stream);
  if (s != GS_OK) throw_status(env, js->ctx, s, "gs_stream_flush");
}

JNIEXPORT jboolean JNI_FN(streamPoll)(JNIEnv* env, jclass cls, jlong h, jboolean wait, jlongArray meta,
                                      jobjectArray rows) {
  jstream* js = (jstream*)(intptr_t)h;
  gs_window_result r;
  memset(&r, 0, sizeof r);
  gs_status s = gs_stream_poll(js->stream, wait ? 1 : 0, &r);
  if (s == GS_EAGAIN) return JNI_FALSE;
  if (s != GS_OK) {
    throw_status(env, js->ctx, s, "gs_stream_poll");
    return JNI_FALSE;
  }
  jlong m[8] = {r.window_start, r.window_end, r.max_timestamp, (jlong)r.edges, (jlong)r.n_vertices,
                (jlong)r.triangles, (jlong)r.triangles_ref, (jlong)r.has_output};
  (*env)->SetLongArrayRegion(env, meta, 0, 8, m);
  /* views of the pinned rows, valid until the next poll */
  const jlong n8 = (jlong)r.n_vertices * 8, nv = (jlong)r.n_vertices * js->vbytes;
  (*env)->SetObjectArrayElement(env, rows, 0, r.keys ? (*env)->NewDirectByteBuffer(env, (void*)r.keys, n8) : NULL);
  (*env)->SetObjectArrayElement(env, rows, 1, r.vals ? (*env)->NewDirectByteBuffer(env, (void*)r.vals, nv) : NULL);
  (*env)->SetObjectArrayElement(env, rows, 2, r.vals2 ? (*env)->NewDirectByteBuffer(env, (void*)r.vals2, n8) : NULL);
  return JNI_TRUE;
}

JNIEXPORT jlongArray JNI_FN(streamStats)(JNIEnv* env, jclass cls, jlong h) {
  jstream* js = (jstream*)(intptr_t)h;
  gs_stream_stats_t st;
  gs_status s = gs_stream_stats(js->stream, &st);
  if (s != GS_OK) {
    throw_status(env, js->ctx, s, "gs_stream_stats");
    return NULL;
  }
  jlong r[6] = {st.watermark, (jlong)st.open_windows, (jlong)st.fired_windows, (jlong)st.pending_windows,
                (jlong)st.late_records, (jlong)st.edges_fired};
  jlongArray out = (*env)->NewLongArray(env, 6);
  (*env)->SetLongArrayRegion(env, out, 0, 6, r);
  return out;
}
