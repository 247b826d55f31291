"""ctypes binding of libgellyhip.so (include/gelly_hip.h).

The product path: every operator of this package runs through these entry points.  If the
library is missing or no HIP device is present, :func:`load` / :class:`Engine` raise — there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
# GELLY_HIP_LIB selects a tuning build (csrc/Makefile `variant`); default is the in-tree library
LIB_PATH = Path(os.environ.get("GELLY_HIP_LIB", PKG / "libgellyhip.so"))

GS_OK, GS_EINVAL, GS_ECAPACITY, GS_EDEVICE, GS_ECOMM, GS_ENOMEM, GS_EUNSUPPORTED, GS_EAGAIN = 0, -1, -2, -3, -4, -5, -6, -7
GS_STREAM_REDUCE, GS_STREAM_FOLD, GS_STREAM_DEGREE_MAX, GS_STREAM_TRIANGLES = 0, 1, 2, 3
GS_WATERMARK_EXPLICIT, GS_WATERMARK_ASCENDING = 0, 1
GS_STAGE_PINNED, GS_STAGE_DIRECT = 0, 1
GS_MEM_HOST, GS_MEM_DEVICE = 0, 1
GS_TIMING_OFF, GS_TIMING_DOMINANT, GS_TIMING_STAGES = 0, 1, 2   # gs_set_timing
GS_I32, GS_I64, GS_F32, GS_F64, GS_NONE = 0, 1, 2, 3, 4
GS_OP_SUM, GS_OP_MIN, GS_OP_MAX, GS_OP_COUNT = 0, 1, 2, 3
STATUS_NAMES = {0: "GS_OK", -1: "GS_EINVAL", -2: "GS_ECAPACITY", -3: "GS_EDEVICE", -4: "GS_ECOMM",
                -5: "GS_ENOMEM", -6: "GS_EUNSUPPORTED", -7: "GS_EAGAIN"}

NP_DTYPE = {GS_I32: np.int32, GS_I64: np.int64, GS_F32: np.float32, GS_F64: np.float64}
GS_DTYPE_OF = {np.dtype(np.int32): GS_I32, np.dtype(np.int64): GS_I64, np.dtype(np.float32): GS_F32,
               np.dtype(np.float64): GS_F64}

# every symbol include/gelly_hip.h declares (checked by tests/test_abi.py)
EXPORTS = ("gs_abi_version", "gs_device_count", "gs_create", "gs_destroy", "gs_last_error", "gs_set_stream", "gs_set_timing", "gs_synchronize",
           "gs_alloc_pinned", "gs_free_pinned", "gs_window_reduce", "gs_window_fold",
           "gs_window_fold_degree_max", "gs_window_csr", "gs_window_candidates", "gs_window_candidates_part",
           "gs_window_triangles",
           "gs_window_triangles_part", "gs_window_count_candidates", "gs_tri_dist_range", "gs_tri_dist_degrees",
           "gs_tri_dist_orient", "gs_tri_dist_route", "gs_tri_dist_build", "gs_tri_dist_plan", "gs_tri_dist_need", "gs_tri_dist_serve",
           "gs_tri_dist_assemble", "gs_tri_dist_count", "gs_window_triangles_selfpair",
           "gs_window_triangles_dist", "gs_window_components",
           "gs_parse_edges_text", "gs_fetch_last_output", "gs_fetch_last_degree_output", "gs_owner_of", "gs_window_reduce_partials", "gs_window_fold_degree_max_partials",
           "gs_merge_partials", "gs_merge_degree_max_partials", "gs_comm_unique_id", "gs_comm_init", "gs_comm_destroy",
           "gs_comm_group_create", "gs_comm_group_destroy", "gs_comm_init_group",
           "gs_comm_allreduce_sum_u64", "gs_window_reduce_dist", "gs_window_fold_degree_max_dist",
           "gs_stream_create", "gs_stream_destroy", "gs_stream_append", "gs_stream_watermark", "gs_stream_flush",
           "gs_stream_poll", "gs_stream_stats", "gs_generate_rmat", "gs_generate_uniform", "gs_generate_zipf", "gs_generate_values", "gs_last_stage_times",
           "gs_set_max_window_records", "gs_candidates_begin", "gs_candidates_begin_part", "gs_candidates_next", "gs_candidates_next_u32", "gs_candidates_seek",
           "gs_candidates_vertex_range")

P = ctypes.c_void_p
u64, i64, i32, u32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32


GS_FLAG_SORT_ONLY = 1   # include/gelly_hip.h: reduce / fold always take the LSD sort path
GS_FLAG_BK_ONESWEEP = 2   # bucket path: 1-2 LSD partition passes instead of the direct scatter (A/B)
GS_FLAG_NO_PACK = 4       # bucket path: integer SUM/MIN/MAX keep 8-byte partitioned values (A/B)
GS_FLAG_NO_SPEC = 16      # bucket path: no speculative partition (per-tile histograms first; A/B)
GS_FLAG_TEST_TINY_TABLES = 8   # TEST ONLY: triangle hash sets of one bucket -> must fail with GS_EDEVICE
GS_LATE_REFIRE, GS_LATE_DROP = 0, 1   # gs_stream_config.late_mode
GS_FLAG_TEST_FORCE_EXCHANGE = 32   # TEST ONLY: *_dist on one rank still partitions, exchanges and merges
GS_FLAG_ASYNC_OUTPUT = 64   # device outputs of reduce / fold complete in the ctx stream's order (no wait for them)


class GsConfig(ctypes.Structure):
    _fields_ = [("device", i32), ("flags", u32), ("reserve_edges", u64)]


class GsEdgeBatch(ctypes.Structure):
    _fields_ = [("src", P), ("dst", P), ("val", P), ("n", u64), ("val_dtype", i32), ("mem", i32),
                ("window_end_ms", i64)]


class GsVertexOut(ctypes.Structure):
    _fields_ = [("keys", P), ("vals", P), ("capacity", u64), ("n_out", ctypes.POINTER(u64)), ("mem", i32),
                ("reserved", i32)]


class GsDegreeOut(ctypes.Structure):
    _fields_ = [("keys", P), ("degree", P), ("max_neighbor", P), ("capacity", u64),
                ("n_out", ctypes.POINTER(u64)), ("mem", i32), ("reserved", i32)]


class GsCsrOut(ctypes.Structure):
    _fields_ = [("keys", P), ("offsets", P), ("neighbors", P), ("vals", P), ("capacity_vertices", u64),
                ("capacity_records", u64), ("n_vertices", ctypes.POINTER(u64)), ("n_records", ctypes.POINTER(u64)),
                ("mem", i32), ("reserved", i32)]


class GsPairOut(ctypes.Structure):
    _fields_ = [("a", P), ("b", P), ("is_candidate", P), ("capacity", u64), ("n_out", ctypes.POINTER(u64)),
                ("mem", i32), ("reserved", i32)]


class GsPairOutU32(ctypes.Structure):   # gs_pair_out_u32: the same fields, uint32_t id columns
    _fields_ = [("a", P), ("b", P), ("is_candidate", P), ("capacity", u64), ("n_out", ctypes.POINTER(u64)),
                ("mem", i32), ("reserved", i32)]


class GsPairBatch(ctypes.Structure):
    _fields_ = [("a", P), ("b", P), ("is_candidate", P), ("n", u64), ("mem", i32), ("reserved", i32)]


class GsPartialsOut(ctypes.Structure):
    _fields_ = [("keys", P), ("vals", P), ("vals2", P), ("capacity", u64), ("n_out", ctypes.POINTER(u64)),
                ("owner_counts", ctypes.POINTER(u64)), ("mem", i32), ("reserved", i32)]


class GsPartialBatch(ctypes.Structure):
    _fields_ = [("keys", P), ("vals", P), ("vals2", P), ("n", u64), ("val_dtype", i32), ("mem", i32)]


class GsStreamConfig(ctypes.Structure):
    _fields_ = [("window_ms", i64), ("kind", i32), ("dir", i32), ("op", i32), ("val_dtype", i32),
                ("watermark_mode", i32), ("staging", i32), ("init", P), ("init_max", i64), ("max_window_edges", u64),
                ("late_mode", i32), ("reserved", i32)]


class GsWindowResult(ctypes.Structure):
    _fields_ = [("window_start", i64), ("window_end", i64), ("max_timestamp", i64), ("edges", u64),
                ("n_vertices", u64), ("keys", P), ("vals", P), ("vals2", P), ("triangles", u64),
                ("triangles_ref", i32), ("has_output", i32), ("latency_ms", ctypes.c_double)]


class GsStreamStats(ctypes.Structure):
    _fields_ = [("watermark", i64), ("open_windows", u64), ("fired_windows", u64), ("pending_windows", u64),
                ("late_records", u64), ("edges_fired", u64)]


class GsStageTimes(ctypes.Structure):
    _fields_ = [("keyinfo_ms", ctypes.c_float), ("sort_ms", ctypes.c_float), ("reduce_ms", ctypes.c_float),
                ("total_ms", ctypes.c_float), ("sort_passes", u32), ("key_bits", u32), ("records", u64),
                ("vertices", u64), ("pass_ms", ctypes.c_float * 8), ("key_bytes", u32), ("payload_bytes", u32),
                ("partials", u64), ("fused_last", u32), ("path", u32), ("packed", u32), ("speculative", u32),
                ("escapes", u64)]


class GsError(RuntimeError):
    """A non-zero gs_status — the Java wrapper maps these to an Exception (EdgesReduce.java:43 `throws Exception`)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


_lib = None


def load() -> ctypes.CDLL:
    """Load libgellyhip.so (build it first with __graft_entry__.build() or `make -C csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} is missing: the HIP engine is not built (run __graft_entry__.build())")
    # torch before the library: torch ships its own libamdhip64.so.7 (the soname of /opt/rocm's), and
    # whichever loads first serves the process.  Loaded after ours, torch ran on a runtime it was not
    # built with and found no GPU ("No HIP GPUs are available" in a process that made the library's
    # calls before touching torch); loaded first, both share torch's (tests/test_gpu_fresh_process.py).
    import torch  # noqa: F401
    L = ctypes.CDLL(str(LIB_PATH))
    st = ctypes.c_int32
    sigs = {
        "gs_abi_version": (i32, []),
        "gs_device_count": (st, [ctypes.POINTER(i32)]),
        "gs_create": (st, [ctypes.POINTER(GsConfig), ctypes.POINTER(P)]),
        "gs_destroy": (None, [P]),
        "gs_last_error": (ctypes.c_char_p, [P]),
        "gs_set_stream": (st, [P, P]),
        "gs_set_timing": (st, [P, i32]),
        "gs_synchronize": (st, [P]),
        "gs_alloc_pinned": (P, [ctypes.c_size_t]),
        "gs_free_pinned": (None, [P]),
        "gs_window_reduce": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, i32, ctypes.POINTER(GsVertexOut)]),
        "gs_window_fold": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, i32, P, ctypes.POINTER(GsVertexOut)]),
        "gs_window_fold_degree_max": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, i64, ctypes.POINTER(GsDegreeOut)]),
        "gs_window_csr": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, ctypes.POINTER(GsCsrOut)]),
        "gs_window_candidates": (st, [P, ctypes.POINTER(GsEdgeBatch), ctypes.POINTER(GsPairOut)]),
        "gs_window_candidates_part": (st, [P, ctypes.POINTER(GsEdgeBatch), u32, u32, ctypes.POINTER(GsPairOut)]),
        "gs_window_triangles": (st, [P, ctypes.POINTER(GsEdgeBatch), ctypes.POINTER(u64), ctypes.POINTER(i32),
                                     ctypes.POINTER(i32)]),
        "gs_window_triangles_part": (st, [P, ctypes.POINTER(GsEdgeBatch), u32, u32, ctypes.POINTER(u64)]),
        "gs_tri_dist_range": (st, [P, ctypes.POINTER(GsEdgeBatch), ctypes.POINTER(i64)]),
        "gs_tri_dist_degrees": (st, [P, ctypes.POINTER(GsEdgeBatch), i64, i64, P, ctypes.POINTER(u64)]),
        "gs_tri_dist_orient": (st, [P, ctypes.POINTER(GsEdgeBatch), P, P, ctypes.POINTER(u64)]),
        "gs_tri_dist_route": (st, [P, P, u32, P, P]),
        "gs_tri_dist_build": (st, [P, P, u64, P, P, ctypes.POINTER(u64)]),
        "gs_tri_dist_plan": (st, [P, P, u32, u32, P, P, ctypes.POINTER(u64)]),
        "gs_tri_dist_need": (st, [P, P, P, u64, P, P, ctypes.POINTER(u64)]),
        "gs_tri_dist_serve": (st, [P, P, P, P, P, u64, P]),
        "gs_tri_dist_assemble": (st, [P, P, P, P, P]),
        "gs_tri_dist_count": (st, [P, P, u64, P, u32, u32, ctypes.POINTER(u64)]),
        "gs_window_triangles_selfpair": (st, [P, ctypes.POINTER(GsEdgeBatch), ctypes.POINTER(u64)]),
        "gs_window_components": (st, [P, ctypes.POINTER(GsEdgeBatch), ctypes.POINTER(GsPartialBatch),
                                      ctypes.POINTER(GsVertexOut)]),
        "gs_window_triangles_dist": (st, [P, ctypes.POINTER(GsEdgeBatch), ctypes.POINTER(u64), ctypes.POINTER(i32),
                                          ctypes.POINTER(i32)]),
        "gs_window_count_candidates": (st, [P, ctypes.POINTER(GsPairBatch), ctypes.POINTER(u64), ctypes.POINTER(i32),
                                            ctypes.POINTER(i32), ctypes.POINTER(u64)]),
        "gs_parse_edges_text": (st, [P, P, u64, i32, P, P, P, u64, i32, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "gs_fetch_last_output": (st, [P, ctypes.POINTER(GsVertexOut)]),
        "gs_fetch_last_degree_output": (st, [P, ctypes.POINTER(GsDegreeOut)]),
        "gs_owner_of": (u32, [i64, u32]),
        "gs_stream_create": (st, [P, ctypes.POINTER(GsStreamConfig), ctypes.POINTER(P)]),
        "gs_stream_destroy": (None, [P]),
        "gs_stream_append": (st, [P, P, P, P, P, u64]),
        "gs_stream_watermark": (st, [P, i64]),
        "gs_stream_flush": (st, [P]),
        "gs_stream_poll": (st, [P, i32, ctypes.POINTER(GsWindowResult)]),
        "gs_stream_stats": (st, [P, ctypes.POINTER(GsStreamStats)]),
        "gs_window_reduce_partials": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, i32, u32, ctypes.POINTER(GsPartialsOut)]),
        "gs_window_fold_degree_max_partials": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, u32,
                                                    ctypes.POINTER(GsPartialsOut)]),
        "gs_merge_partials": (st, [P, ctypes.POINTER(GsPartialBatch), i32, P, ctypes.POINTER(GsVertexOut)]),
        "gs_merge_degree_max_partials": (st, [P, ctypes.POINTER(GsPartialBatch), i64, ctypes.POINTER(GsDegreeOut)]),
        "gs_comm_unique_id": (st, [P]),
        "gs_comm_init": (st, [P, i32, i32, P]),
        "gs_comm_destroy": (st, [P]),
        "gs_comm_group_create": (st, [i32, ctypes.POINTER(P)]),
        "gs_comm_group_destroy": (None, [P]),
        "gs_comm_init_group": (st, [P, P, i32]),
        "gs_comm_allreduce_sum_u64": (st, [P, ctypes.POINTER(u64)]),
        "gs_window_reduce_dist": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, i32, P, ctypes.POINTER(GsVertexOut)]),
        "gs_window_fold_degree_max_dist": (st, [P, ctypes.POINTER(GsEdgeBatch), i32, i64, ctypes.POINTER(GsDegreeOut)]),
        "gs_generate_rmat": (st, [P, i32, u64, u64, u32, u32, u32, i32, i32, u64, P, P]),
        "gs_generate_uniform": (st, [P, u64, u64, u64, u64, P, P]),
        "gs_generate_zipf": (st, [P, u64, ctypes.c_double, u64, u64, u64, P, P]),
        "gs_generate_values": (st, [P, u64, u64, u64, i32, P]),
        "gs_last_stage_times": (st, [P, ctypes.POINTER(GsStageTimes)]),
        "gs_set_max_window_records": (st, [P, u64]),
        "gs_candidates_begin": (st, [P, ctypes.POINTER(GsEdgeBatch), ctypes.POINTER(u64), ctypes.POINTER(u32)]),
        "gs_candidates_begin_part": (st, [P, ctypes.POINTER(GsEdgeBatch), u32, u32, ctypes.POINTER(u64),
                                          ctypes.POINTER(u32)]),
        "gs_candidates_next": (st, [P, ctypes.POINTER(GsPairOut), ctypes.POINTER(u64), ctypes.POINTER(i32)]),
        "gs_candidates_next_u32": (st, [P, ctypes.POINTER(GsPairOutU32), ctypes.POINTER(i64), ctypes.POINTER(u64),
                                        ctypes.POINTER(i32)]),
        "gs_candidates_seek": (st, [P, u64]),
        "gs_candidates_vertex_range": (st, [P, i64, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L
