"""bench.py — edges/sec per tumbling slice for reduceOnEdges on the BASELINE C2 window.

    python bench.py [--gpus N] [--steps K] [--warmup W]

Workload (BASELINE.json configs[1]): one tumbling window of an R-MAT scale-24
stream (Graph500 a,b,c,d = .57,.19,.19,.05, edge factor 16 -> E = 2^28 edges, seeded vertex
permutation, seed 0x5EED02), Long edge values splitmix64 & 0xFFFF, slice(OUT).reduceOnEdges(SUM).
A step = the whole window through the engine with the edge columns already resident in HBM:
key scan -> LSD radix passes -> segmented reduce -> per-vertex (vertex, sum) in HBM.
N > 1 (torchrun, one rank per GPU): each rank holds its own 2^28-edge slice of the stream
(weak scaling); the step adds the RCCL keyBy exchange of per-vertex partials and the merge.
Rank 0 prints one JSON line (roofline of the dominant kernel + the CPU baseline at N = 1).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "edges/sec per tumbling slice (reduceOnEdges, window triangles) at 1/2/4/8 GPUs"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--scale", type=int, default=24)
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED02)
    p.add_argument("--dtype", default="int64", choices=["int64", "float64"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--alloc-outputs", action="store_true",
                   help="reduce / fold: allocate the output tensors per window (A/B; default: reused across windows, as a streaming operator keeps its buffers)")
    p.add_argument("--cpu-sample-log2", type=int, default=30,
                   help="triangles: the CPU baseline counts windows up to 2^this many edges (larger windows: their "
                        "first 2^this); 30 = the whole C4 (s26) window (~65 s of 16-thread CPU)")
    p.add_argument("--cpu-reps", type=int, default=None,
                   help="triangles: CPU baseline windows timed (median); default 5, 1 for windows over 2^28 edges")
    p.add_argument("--timing", default="dominant", choices=["dominant", "stages"],
                   help="reduce / fold: stage events inside the timed region -- the dominant kernels only "
                        "(default) or every stage (each record costs the stream a few microseconds)")
    p.add_argument("--windows", type=int, default=2, help="distinct windows of the stream the timed steps cycle through")
    p.add_argument("--stream", default="rmat", choices=["rmat", "zipf"],
                   help="fold (C3): skewed R-MAT (default) or the Zipf(1.1) source stream")
    p.add_argument("--staging", default="direct", choices=["direct", "pinned", "buffered"],
                   help="e2e: host columns in pageable memory, appended with direct staging (direct); in caller-"
                        "pinned memory (gs_alloc_pinned, as a Java operator's direct buffers), DMA'd straight to HBM "
                        "(pinned); or copied into the operator's own pinned window buffers, H2D at firing (buffered)")
    p.add_argument("--e2e-kind", default="reduce", choices=["reduce", "triangles"],
                   help="e2e: reduceOnEdges(SUM) on C2 windows, or WindowTriangles on C5-size windows "
                        "(--windows-edges edges of an R-MAT --scale stream per 1000 ms window)")
    p.add_argument("--no-pack", action="store_true",
                   help="ablation: integer SUM keeps 8-byte partitioned values instead of 4-byte packed records")
    p.add_argument("--no-spec", action="store_true",
                   help="ablation: packed windows count per-tile bucket histograms before the scatter instead of "
                        "sizing bucket regions from the previous window's counts")
    p.add_argument("--sort-only", action="store_true",
                   help="ablation: reduce / fold through the full LSD sort + reduce-by-key path")
    p.add_argument("--bk-onesweep", action="store_true",
                   help="ablation: bucket path partitions with 1-2 LSD passes instead of the direct scatter")
    p.add_argument("--exchange", default="abi", choices=["abi", "torch"],
                   help="N > 1: the library's own RCCL communicator (gs_window_*_dist, what the Java side binds; "
                        "default) or torch.distributed around the partials / merge halves (A/B)")
    p.add_argument("--force-exchange", action="store_true",
                   help="rehearsal: at world size 1 the ABI path still partitions by owner, exchanges through RCCL "
                        "and merges (what each rank pays at N > 1, minus the link transfer)")
    p.add_argument("--sync-outputs", action="store_true",
                   help="reduce / fold: every call waits for its outputs (A/B; default GS_FLAG_ASYNC_OUTPUT: a call "
                        "returns once the window's sizes are known, its outputs complete in the stream's order)")
    p.add_argument("--check", action="store_true",
                   help="after timing: sum(per-vertex sums) == sum(values) and ascending keys on each window")
    p.add_argument("--chunk-records", type=float, default=2 ** 28,
                   help="cand_stream: records per gs_candidates_next chunk")
    p.add_argument("--cand-overlap", action="store_true",
                   help="cand_stream: run the consumer on a second stream, overlapping the next chunk's emission "
                        "(default: on the emission stream right after its chunk -- the mixed read/write traffic of "
                        "the overlap ran slower than the two in turn)")
    p.add_argument("--cand-consumer", default="sum", choices=["sum", "none"],
                   help="cand_stream: a device consumer reads every record (column sums), or none (emission alone)")
    p.add_argument("--cand-ids", default="i64", choices=["i64", "u32"],
                   help="cand_stream: id columns as int64 (gs_candidates_next: 17-byte records) or as uint32 relative "
                        "to the window's smallest id (gs_candidates_next_u32: 9-byte records, the same records)")
    p.add_argument("--cand-windows", type=int, default=2,
                   help="cand_stream: consecutive windows streamed (the next window's sets built while the current "
                        "one's chunks drain)")
    p.add_argument("--cand-cadence-ms", type=float, default=0,
                   help="cand_stream: fire window w at w x this many ms (the stream's window cadence, e.g. 1000) "
                        "instead of back to back; the window latency is measured from each fire")
    p.add_argument("--max-chunks", type=int, default=0,
                   help="cand_stream: stop after this many chunks (profiling passes; 0 = the whole window)")
    p.add_argument("--windows-edges", type=float, default=1e8,
                   help="apply (C5): edges per 1000 ms window of the continuous stream")
    p.add_argument("--workload", default="reduce",
                   choices=["reduce", "fold", "triangles", "cc", "c1", "apply", "candidates", "cand_stream", "parse",
                            "e2e"],
                   help="reduce = C2 (default, the headline); fold = C3 degree/max on skewed R-MAT; "
                        "triangles = WindowTriangles on an R-MAT window without self-loops (C4 shape); "
                        "cc = ConnectedComponents of an R-MAT window (SURVEY.md §8f#4)")
    return p.parse_args()


def algorithmic_bytes(workload, E, U, vb=8):
    """SURVEY.md §8(d) algorithmic bytes of one window (E input edges, U output vertices):
    reduce OUT/IN 16E + 16U (8-byte values; 4-byte: 12E + 12U), fold degree/max 16E + 24U."""
    if workload == "fold":
        return 16 * E + 24 * U
    return (8 + vb) * E + (8 + vb) * U


def kernel_table(times_list, E, U_avg, stage_list=None, nbr_payload=False):
    """Average per-launch durations (device events inside the library, same stream) and each kernel's
    own algorithmic bytes.  times_list: the timed windows (GS_TIMING_DOMINANT: the direct
    path's scatter and accumulate only); stage_list: windows after them with every stage event.
    nbr_payload: the records' payload is the neighbour id (the degree / max-neighbour fold), read from
    the int64 neighbour column and stored in payload_bytes."""
    t0 = times_list[0]
    if t0.path == 2:
        return direct_kernel_table(times_list, E, U_avg, stage_list or times_list, nbr_payload)
    times_list = stage_list or times_list   # other paths: every stage from the stage-timed windows
    t0 = times_list[0]
    if t0.path == 1:
        return bucket_kernel_table(times_list, E, U_avg, nbr_payload)
    kb, vb = t0.key_bytes, t0.payload_bytes
    ab = 8                      # partial accumulator of a Long sum
    passes = t0.sort_passes
    P = statistics.mean(t.partials for t in times_list)
    rows = {}
    for p in range(passes):
        ms = statistics.mean(t.pass_ms[p] for t in times_list)
        if t0.fused_last and p == passes - 1:
            rows["onesweep_combine(last pass)"] = {"ms": ms, "bytes": E * (kb + vb) + P * (kb + ab)}
        else:
            # pass 0 reads the int64 key column + values, later passes the compact keys; all write compact
            rd = (8 + vb) if p == 0 else (kb + vb)
            rows[f"onesweep_pass{p}"] = {"ms": ms, "bytes": E * (rd + kb + vb)}
    ms = statistics.mean(t.reduce_ms - (t.pass_ms[passes - 1] if t0.fused_last else 0.0) for t in times_list)
    if t0.fused_last:   # region table + compaction of the partials + reduce_by_key merge
        rows["merge(compact+reduce_by_key)"] = {"ms": ms, "bytes": 3 * P * (kb + ab) + U_avg * 16}
    else:
        rows["reduce_by_key"] = {"ms": ms, "bytes": E * (kb + vb) + U_avg * 16}
    ms = statistics.mean(t.keyinfo_ms for t in times_list)
    rows["keyinfo(+host sync)"] = {"ms": ms, "bytes": E * 8}
    return rows, P


def bucket_kernel_table(times_list, E, U_avg, nbr_payload=False):
    """Bucket path (gs_bucket.hpp): bk_info, 1-2 partition passes over the bucket index, LDS accumulate,
    merge of multi-item buckets, emit.  Algorithmic bytes per launch as in DESIGN.md."""
    t0 = times_list[0]
    vb = t0.payload_bytes
    ab = 8 if vb else 4          # staged accumulator (i64 sum / u32 count)
    passes = t0.sort_passes
    mean = lambda f: statistics.mean(f(t) for t in times_list)
    rows = {}
    for p in range(passes):
        rd = (8 + (8 if nbr_payload else vb)) if p == 0 else (4 + vb)
        wr = (2 if p == passes - 1 else 4) + vb
        rows[f"bucket_partition{p}"] = {"ms": mean(lambda t: t.pass_ms[p]), "bytes": E * (rd + wr)}
    rd = (2 + vb) if passes else (8 + (8 if nbr_payload else vb))
    rows["bucket_accumulate"] = {"ms": mean(lambda t: t.pass_ms[passes]), "bytes": E * rd + U_avg * (4 + ab)}
    rows["bucket_merge"] = {"ms": mean(lambda t: t.pass_ms[passes + 1]), "bytes": 0}
    rows["bucket_emit"] = {"ms": mean(lambda t: t.pass_ms[passes + 2]), "bytes": U_avg * (4 + ab + 16)}
    rows["keyinfo(+host sync)"] = {"ms": mean(lambda t: t.keyinfo_ms), "bytes": E * 8}
    return rows, mean(lambda t: t.partials)


def direct_kernel_table(times_list, E, U_avg, stage_list, nbr_payload=False):
    """Direct bucket path (gs_bucket.hpp k_dp_*): per-tile histogram, offset scans, ONE scatter, LDS
    accumulate, merge, emit.  Each kernel's own bytes (E = records): the packed scatter
    writes 4-byte records (2-byte key + 2-byte value), the plain one a 2-byte key + the payload."""
    t0 = times_list[0]
    vb = t0.payload_bytes        # packed: 2
    lb = 8 if (t0.packed or nbr_payload) else vb  # loaded value bytes (the int64 neighbour column for a fold)
    ab = 8 if (vb or t0.packed) else 4   # staged accumulator (i64 sum / u32 count)
    mean = lambda f: statistics.mean(f(t) for t in times_list)
    smean = lambda f: statistics.mean(f(t) for t in stage_list)   # the stages the timed windows did not time
    rows = {}
    spec = t0.speculative == 1   # regions from the previous window's counts: no histogram, no offset scans
    name = ("sp_scatter_pack" if spec else "dp_scatter_pack") if t0.packed else ("sp_scatter" if spec else "dp_scatter")
    rows[name] = {"ms": mean(lambda t: t.pass_ms[1]), "bytes": E * ((8 + lb) + (2 + vb))}
    acc_ms = mean(lambda t: t.pass_ms[2])   # (0: the timed windows bracketed the scatter only)
    rows["bucket_accumulate"] = {"ms": acc_ms if acc_ms > 0 else smean(lambda t: t.pass_ms[2]),
                                 "bytes": E * (2 + vb) + U_avg * (4 + ab)}
    rows["bucket_merge"] = {"ms": smean(lambda t: t.pass_ms[3]), "bytes": 0}
    rows["bucket_emit"] = {"ms": smean(lambda t: t.pass_ms[4]), "bytes": U_avg * (4 + ab + 16)}
    if spec:
        rows["sp_regions"] = {"ms": smean(lambda t: t.keyinfo_ms), "bytes": 0}
    else:
        rows["dp_offsets(up+spine+plan+down)"] = {"ms": smean(lambda t: t.pass_ms[0]), "bytes": 0}
        rows["dp_hist"] = {"ms": smean(lambda t: t.keyinfo_ms), "bytes": E * 8}
    return rows, mean(lambda t: t.partials)


def triangle_kernel_table(times_list, n):
    """WindowTriangles (stage_times path 3): algorithmic bytes per stage as in DESIGN.md §4 —
    n input edges, M unique (oriented) edges, P hash probes, V id range."""
    mean = lambda f: statistics.mean(f(t) for t in times_list)
    M, P = mean(lambda t: t.records), mean(lambda t: t.partials)
    V = 2 ** statistics.mean(t.key_bits for t in times_list)
    rows = {
        # raw degrees (edge list in), degree-class ranks (2 reads + 1 write of V), oriented keys of the
        # ranks (edge list in, 2 rank gathers, n keys out), one read + write of the n keys
        "tri_rank+keys+sort": {"ms": mean(lambda t: t.pass_ms[0]),
                               "bytes": 16 * n + 12 * V + 16 * n + 8 * n + 8 * n + 16 * n},
        "tri_unique": {"ms": mean(lambda t: t.pass_ms[1]), "bytes": 8 * n + 8 * M},
        # out-lists (keys in; neighbour ids, transposed keys + payload out), list ends, the transposed
        # sort (one read + write of 8 B per edge), in-lists + suffix ranges (8 B in, 4 B gathered, 8 B out)
        "tri_out+transpose+in": {"ms": mean(lambda t: t.pass_ms[2]),
                                 "bytes": 8 * M + 16 * M + 8 * M + 4 * M + 16 * M + 20 * M + 16 * V},
        # N+(v) (4 B per out-entry), one suffix range per in-entry (8 B), one 4-byte list item per probe
        "tri_count(light+heavy)": {"ms": mean(lambda t: t.pass_ms[3] + t.pass_ms[4]), "bytes": 12 * M + 4 * P},
        "tri_count_light": {"ms": mean(lambda t: t.pass_ms[3]), "bytes": 0},
        "tri_count_heavy": {"ms": mean(lambda t: t.pass_ms[4]), "bytes": 0},
    }
    return rows, P


def finish_rows(rows, B):
    """GB/s and HBM fraction of each kernel on its own bytes; on the window's §8(d) bytes B only for the
    kernel that reads the window's columns (B over a small kernel's time is no fraction of anything)."""
    for r in rows.values():
        r["GB/s"] = r["bytes"] / (r["ms"] * 1e-3) / 1e9 if r["ms"] > 0 else 0.0
        r["frac"] = r["GB/s"] / HBM_PEAK_GBS
        r["frac_on_B"] = (B / (r["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS) if r["ms"] > 0 else 0.0
    return rows


def lib_sha16():
    """sha256 prefix of the library this process runs (GELLY_HIP_LIB or the in-tree build)."""
    import hashlib

    p = Path(os.environ.get("GELLY_HIP_LIB", ROOT / "gelly-streaming_amd" / "libgellyhip.so"))
    return hashlib.sha256(p.read_bytes()).hexdigest()[:16] if p.exists() else None


def pmc_table():
    """profiles/pmc_traffic.json: per-kernel HBM bytes per launch from separate rocprofv3 --pmc passes
    (tools/pmc_traffic.py, gfx950 FETCH_SIZE correction)."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return {}
    try:
        return json.loads(f.read_text())
    except Exception:
        return {}


def host_cpu():
    """The CPU the baseline ran on: model name, nproc (every hardware thread the OS reports) and the
    threads the baseline used.  On the GPU box the pool allots 16 CPUs per GPU (its rules cap worker
    pools there), so the baseline runs min(16, nproc) threads; nproc is recorded beside it."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    # the worker-pool caps the GPU box exports (16 per GPU there), as they were when the baseline ran
    env = {k: os.environ[k] for k in ("OMP_NUM_THREADS", "MAX_JOBS", "CMAKE_BUILD_PARALLEL_LEVEL") if k in os.environ}
    return {"cpu_model": model, "nproc": nproc, "affinity_cpus": affinity, "pool_env": env or None}


def cpu_baseline(wins, workload, threads, reps=5):
    """BASELINE.md CPU baseline: the oracle's keyBy + per-subtask arrival-order hash-map fold
    (gso_baseline_reduce; Flink's keyBy at local-env parallelism = threads) over WHOLE windows of the
    same stream, cycling the bench's windows: 1 warm-up window, then the median of `reps`; plus a
    one-thread figure on the first 1/8 of a window."""
    orc = ge.load_oracle()
    host = [tuple(x.cpu().numpy() if x is not None else None for x in w) for w in wins]
    op = 4 if workload == "fold" else 0      # 4 = the degree / max-neighbour fold
    run = lambda h, th, k=None: orc.baseline_reduce(h[0][:k], h[1][:k], (h[2] if h[2] is not None else h[0])[:k],
                                                   1, op, th)
    run(host[0], threads)
    ts = []
    for r in range(reps):
        h = host[r % len(host)]
        t = time.perf_counter()
        run(h, threads)
        ts.append(time.perf_counter() - t)
    tmed = statistics.median(ts)
    E = len(host[0][0])
    k1 = E // 8
    t = time.perf_counter()
    run(host[0], 1, k1)
    t1 = time.perf_counter() - t
    what = "degree/max-neighbour fold" if workload == "fold" else "reduceOnEdges(SUM) fold"
    return {"value": E / tmed, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"whole {E}-edge windows of the same stream ({len(host)} distinct, cycled), keyBy over "
                      f"{threads} threads + per-subtask arrival-order hash-map {what} (oracle/gs_oracle.c "
                      f"gso_baseline_reduce), 1 warm-up + median of {reps}",
            "window_s_median": tmed, "single_core_value": k1 / t1,
            "single_core_sample": f"first {k1} edges of window 0, one thread"}


def cc_kernel_table(times_list, E):
    """ConnectedComponents (stage_times path 4): compact IDs (sort of the 2E endpoints with positions),
    union-find over the E edges, labels out."""
    mean = lambda f: statistics.mean(f(t) for t in times_list)
    U = mean(lambda t: t.vertices)
    return {
        # ids spanning <= 2^28 values (the bench windows): range scan + parent init; wider: the relabel sort
        "cc_ids": {"ms": mean(lambda t: t.pass_ms[0]), "bytes": 16 * E + 4 * 2 ** statistics.mean(t.key_bits for t in times_list)},
        "cc_union_find": {"ms": mean(lambda t: t.pass_ms[1]), "bytes": 16 * E + 8 * U},
        "cc_labels": {"ms": mean(lambda t: t.pass_ms[2]), "bytes": 4 * U + 8 * U + 16 * U},
    }, U


def cpu_baseline_cc(src, dst, sample_log2=23):
    """ConnectedComponents on the host: the oracle's DisjointSet restatement (one thread, as the
    reference's parallelism-1 merger) on the first 2^sample_log2 edges, 1 warm-up + median of 3."""
    orc = ge.load_oracle()
    S = min(1 << sample_log2, src.numel())
    s, d = src[:S].cpu().numpy(), dst[:S].cpu().numpy()
    orc.components(s[: S // 16], d[: S // 16])
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        v, _ = orc.components(s, d)
        ts.append(time.perf_counter() - t)
    dt = statistics.median(ts)
    return {"value": S / dt, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"first 2^{sample_log2} edges of the window, union-find by rank with path compression "
                      f"(oracle/gs_oracle.c gso_components, one thread), median of 3: {dt:.2f} s, {len(v)} vertices"}


def cpu_baseline_triangles(wins, threads, sample_log2=30, reps=None):
    """BASELINE.md C4 CPU baseline: the forward algorithm (the reference's O(sum d^2) candidate rule is
    infeasible at this scale) over `threads` threads (oracle gso_triangles_fwd_mt) on whole windows up to
    2^sample_log2 edges (default 2^30: the whole C4 s26 window; larger windows: their first 2^sample_log2
    edges), cycling the bench's windows: 1 warm-up on a 1/16 sample, then the median of `reps` (default 5,
    1 above 2^28 edges: one s26 window is ~65 s of 16-thread CPU)."""
    orc = ge.load_oracle()
    S = min(1 << sample_log2, wins[0][0].numel())
    if reps is None:
        reps = 5 if S <= (1 << 28) else 1
    host = [(w[0][:S].cpu().numpy(), w[1][:S].cpu().numpy()) for w in wins[:max(1, min(reps, len(wins)))]]
    orc.triangles_fwd_mt(host[0][0][: S // 16], host[0][1][: S // 16], threads)
    ts = []
    for r in range(reps):
        s, d = host[r % len(host)]
        t = time.perf_counter()
        T = orc.triangles_fwd_mt(s, d, threads)
        ts.append(time.perf_counter() - t)
    dt = statistics.median(ts)
    whole = S == wins[0][0].numel()
    return {"value": S / dt, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": (f"whole {S}-edge windows" if whole else f"first {S} edges of each window") +
                      f" ({len(host)} distinct, cycled), forward-algorithm triangle count over {threads} threads "
                      f"(oracle/gs_oracle.c gso_triangles_fwd_mt), median of {reps}: {dt:.2f} s, {T} triangles"}


def window_stream_main(a):
    """Secondary single-GPU workloads, one JSON line each:

    c1          C1: WindowTriangles on the uniform 1M-edge stream (V = 2^16, self-loops rejected), one
                1000 ms window; the CPU baseline runs the reference's candidate rule on the WHOLE window.
    apply       C5: a continuous R-MAT scale-23 stream cut into 1000 ms windows of --windows-edges edges
                (1e8 = the 100M edges/s target).  Per window: slice(ALL).applyOnNeighbors grouping
                (gs_window_csr: every vertex's neighbour list in arrival order, what a user EdgesApply
                consumes) and the GenerateCandidateEdges sizing pass (HashSet order + per-vertex pair
                counts; emitting them is not possible at this size).  Reports sustained
                windows/s and p50/p99 latency from window close (columns in HBM) to results in HBM.
    candidates  GenerateCandidateEdges records emitted in full (gs_window_candidates) on R-MAT scale-23
                windows of 2^22 edges."""
    torch.cuda.set_device(0)
    pkg = ge.load_package()
    eng = pkg.Engine(0)
    orc_cpu = None
    lat, extra = [], {}
    if a.workload == "c1":
        E = 1_000_000
        src, dst = eng.generate_uniform(1 << 16, E, 0x5EED01)
        wins = [(src, dst)]
        run = lambda s_, d_: eng.triangles(s_, d_)
        bytes_per_window = 16 * E
        desc = "C1: WindowTriangles over the uniform 1M-edge window (V = 2^16, self-loops rejected, one 1000 ms slice)"
    else:
        E = int(a.windows_edges) if a.workload == "apply" else 1 << 22
        nwin = 2
        wins = [eng.generate_rmat(23, E, 0x5EED05, first_edge=w * E) for w in range(nwin)]
        if a.workload == "apply":
            def run(s_, d_):
                return eng.csr(s_, d_, None, 2), eng.candidate_count(s_, d_)
            desc = (f"C5: continuous R-MAT scale-23 stream, 1000 ms windows of {E:.3g} edges: slice(ALL) "
                    f"applyOnNeighbors grouping + GenerateCandidateEdges sizing")
        else:
            run = lambda s_, d_: eng.candidates(s_, d_)
            desc = "C5 emission: GenerateCandidateEdges records for R-MAT scale-23 windows of 2^22 edges"
    torch.cuda.synchronize()
    for w in range(a.warmup):
        r = run(*wins[w % len(wins)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for w in range(a.steps):
        t = time.perf_counter()
        r = run(*wins[w % len(wins)])
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t)
    elapsed = time.perf_counter() - t0
    if a.workload == "c1":
        extra["triangles"] = r[0]
        extra["reference_integer_output"] = r[1]
        algo = bytes_per_window
    elif a.workload == "apply":
        (keys, offs, nbrs, _), P = r
        extra.update(vertices=int(keys.numel()), csr_records=int(nbrs.numel()), candidate_records_needed=int(P),
                     candidate_bytes_needed=int(P) * 17)
        algo = 16 * E + 16 * keys.numel() + 8 * nbrs.numel()   # edges in; keys + offsets + neighbours out
    else:
        a_, b_, f_ = r
        P = int(a_.numel())
        extra.update(candidate_records=P, candidates_per_s=P * a.steps / elapsed)
        # stage 2 (keyBy(0,1) CountTriangles + sum(0)) on the emitted records, checked against the
        # direct triangle count of the same window
        t2 = []
        for _ in range(3):
            tt = time.perf_counter()
            c2 = eng.count_candidates(a_, b_, f_)
            torch.cuda.synchronize()
            t2.append(time.perf_counter() - tt)
        tri = eng.triangles(*wins[(a.steps - 1) % len(wins)])
        assert c2[0] == tri[0], "stage-2 count differs from the window's triangle count"
        extra.update(stage2_ms=statistics.median(t2) * 1e3, stage2_records_per_s=P / statistics.median(t2),
                     triangles=c2[0], stage2_emitting_groups=c2[3])
        algo = 16 * E + 17 * P
    ms = statistics.mean(lat) * 1e3
    cpu = None
    if a.workload == "c1" and not a.no_cpu_baseline:
        orc = ge.load_oracle()
        s, d = src.cpu().numpy(), dst.cpu().numpy()
        tt = time.perf_counter()
        ref = orc.window_triangles_ref(s, d)
        dt = time.perf_counter() - tt
        extra["cpu_reference_rule_result"] = ref[1]
        assert ref[1] == r[0] and ref[0] == r[1], "C1: GPU triangle count differs from the reference rule"
        cpu = {"value": E / dt, "unit": "edges/s", "cores": 1, "kind": "port",
               "sample": f"the whole C1 window (1M edges) through the reference's candidate rule "
                         f"(oracle gso_window_triangles_ref), one thread, {dt:.2f} s"}
    gbs = algo / (ms * 1e-3) / 1e9
    line = {"metric": METRIC, "value": E * a.steps / elapsed, "unit": "edges/s", "n_gpus": 1, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (uniform / R-MAT, seeded), generated on device",
            "config": {"workload": desc, "edges_per_window": E, "windows_per_s": 1e3 / ms,
                       "latency_ms_p50": float(np.percentile(np.array(lat) * 1e3, 50)),
                       "latency_ms_p99": float(np.percentile(np.array(lat) * 1e3, 99)),
                       # apply: grouping + candidate sizing only; emission is the cand_stream line
                       "sizing_sustains_target": (a.workload != "apply") or (E * 1e3 / ms >= a.windows_edges),
                       **extra, "parallelism": "1 GPU"},
            "roofline": {"bound": "hbm", "kernel": "whole window", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "algorithmic_bytes_per_launch": algo, "avg_launch_ms": round(ms, 4)},
            "cpu_baseline": cpu}
    emit(line)
    eng.close()


def cand_stream_main(a):
    """C5 emission at full size (WindowTriangles.java:91-114): every GenerateCandidateEdges
    record of a 1e8-edge R-MAT scale-23 window, streamed in chunks of --chunk-records through
    gs_candidates_begin / gs_candidates_next (a window has ~1.6e11 records, 2.7 TB, which no single buffer
    holds).  Each chunk is consumed on the device by the stand-in of a downstream operator: per-chunk sums
    of the a, b and is_candidate columns (three reductions, no temporaries), so every record is read once
    after it is written.  By default the consumer runs on the emission stream right after its chunk
    (--cand-overlap: on a second stream while the next chunk is emitted into the other of two buffers;
    no host round trip per chunk either way: gs_candidates_next only enqueues device output).  --cand-windows W > 1 streams W consecutive windows of
    the stream through two engines (sessions), the next window's gs_candidates_begin overlapping the
    current window's emission: the sustained window period.  Reports records/s, the window period, chunk
    latency p50 / p99 (device events, emission start to consumer end) and checks that the chunks add up to
    gs_candidates_begin's total."""
    torch.cuda.set_device(0)
    pkg = ge.load_package()
    W = max(1, int(a.cand_windows))
    E = int(a.windows_edges)
    cap = int(a.chunk_records)
    engines = [pkg.Engine(0, torch_stream=False) for _ in range(min(W, 2))]
    emit_streams = [torch.cuda.Stream() for _ in engines]
    for e, st in zip(engines, emit_streams):
        e.set_stream(st.cuda_stream)
    cons = torch.cuda.Stream()
    wins = []
    for w in range(W):   # consecutive windows of one stream: the generator's edge offset moves on
        with torch.cuda.stream(emit_streams[w % len(engines)]):
            wins.append(engines[w % len(engines)].generate_rmat(23, E, 0x5EED05, first_edge=w * E))
    torch.cuda.synchronize()
    u32 = a.cand_ids == "u32"
    idt = torch.uint32 if u32 else torch.int64
    rec_bytes = 9 if u32 else 17
    bufs = [(torch.empty(cap, dtype=idt, device="cuda"), torch.empty(cap, dtype=idt, device="cuda"),
             torch.empty(cap, dtype=torch.uint8, device="cuda")) for _ in range(2)]
    freed = [None, None]   # consumer events after which a buffer may be written again
    sums = []              # per chunk: a, b, flag-word sums (device scalars, read at the end)
    ev_pairs = []          # (emission start, consumer end) per chunk
    totals, begin_ms, win_end, fire = [], [], [], []
    cadence = float(a.cand_cadence_ms) / 1e3
    # host <-> device clock: an event recorded on an idle stream at a known host time maps every later
    # device event to the host clock (window latency = host fire time -> its last record consumed)
    ev_ref = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_ref.record(emit_streams[0])

    def begin(w):
        eng = engines[w % len(engines)]
        if cadence > 0:   # the stream's own cadence: window w fires at t0 + w * cadence
            time.sleep(max(0.0, t0 + w * cadence - time.perf_counter()))
        fire.append(time.perf_counter())
        tb = time.perf_counter()
        total = eng.candidates_begin(*wins[w])   # (returns after the sets are built: it reads back sizes)
        begin_ms.append((time.perf_counter() - tb) * 1e3)
        totals.append(total)

    begin(0)
    nchunk = 0
    for w in range(W):
        eng, est = engines[w % len(engines)], emit_streams[w % len(engines)]
        got = 0
        while got < totals[w]:
            k = nchunk % 2
            ev0 = torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(est):
                if freed[k] is not None:
                    est.wait_event(freed[k])
                ev0.record(est)
                if u32:
                    ca, cb, cf, first, done, idb = eng.candidates_next_u32(cap, bufs[k])   # enqueued, no wait
                else:
                    ca, cb, cf, first, done = eng.candidates_next(cap, bufs[k])   # enqueued, no wait
                emitted = torch.cuda.Event()
                emitted.record(est)
            assert first == got, (first, got)
            n = int(ca.numel())
            if a.cand_consumer == "none":   # emission alone: the result is available in HBM
                ev1 = emitted = torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(est):
                    ev1.record(est)
            else:
                cst = cons if a.cand_overlap else est   # the consumer's stream
                with torch.cuda.stream(cst):
                    if a.cand_overlap:
                        cons.wait_event(emitted)
                    n8 = (n // 8) * 8
                    if u32:   # the id columns read as 8-byte words (two ids each; a widening int32 sum ran 3x slower)
                        n2 = (n // 2) * 2
                        sums.append(torch.stack([ca[:n2].view(torch.int64).sum() + ca[n2:].view(torch.int32).sum(),
                                                 cb[:n2].view(torch.int64).sum() + cb[n2:].view(torch.int32).sum(),
                                                 cf[:n8].view(torch.int64).sum() + cf[n8:].sum()]))
                    else:
                        sums.append(torch.stack([ca.sum(), cb.sum(), cf[:n8].view(torch.int64).sum() + cf[n8:].sum()]))
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record(cst)
                    freed[k] = ev1 if a.cand_overlap else None
            ev_pairs.append((ev0, ev1))
            got += n
            nchunk += 1
            if a.max_chunks and nchunk >= a.max_chunks:
                break
            if got >= totals[w] and w + 1 < W:
                begin(w + 1)   # the next window's sets on the other engine while this one's chunks drain
        if a.max_chunks and nchunk >= a.max_chunks:
            break
        win_end.append(ev_pairs[-1][1])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if a.max_chunks and nchunk >= a.max_chunks:   # a profiling pass over the first chunks only: no bench line
        print(f"# cand_stream: {nchunk} chunks", file=sys.stderr)
        return
    total = sum(totals)
    lat_ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev_pairs])
    # window latency: from the window's fire (its gs_candidates_begin call) to its last
    # record consumed on the device
    wlat_ms = np.array([(ev_ref.elapsed_time(win_end[w]) / 1e3 + t0 - fire[w]) * 1e3 for w in range(len(win_end))])
    s = torch.stack(sums).sum(0).tolist() if sums else [0, 0, 0]
    chk = (s[0] * 31 + s[1] + s[2]) & ((1 << 63) - 1)
    cands = total - 2 * E * W   # every record past the 2E edge records (one per slice(ALL) record) is a candidate
    period = elapsed / W
    line = {"metric": "candidate records/s (GenerateCandidateEdges, chunked emission)", "value": total / elapsed,
            "unit": "records/s", "n_gpus": 1, "steps": W, "warmup": 0, "ms_per_step": period * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic R-MAT scale 23, seeded, generated on device",
            "config": {"workload": f"C5 emission: every GenerateCandidateEdges record of {W} consecutive "
                                   f"{E:.3g}-edge R-MAT scale-23 windows (slice(ALL)), in chunks of {cap} records, "
                                   + ("each consumed on the device (column sums) while the next is emitted"
                                      if a.cand_overlap else
                                      "each consumed on the device (column sums) right after it is emitted, on the "
                                      "same stream (the next window's sets built on a second stream meanwhile)"),
                       "edges_per_window": E, "windows": W, "records": total, "candidate_records": cands,
                       "chunks": nchunk, "chunk_records": cap, "begin_ms": begin_ms,
                       "chunk_latency_ms_p50": float(np.percentile(lat_ms, 50)),
                       "chunk_latency_ms_p99": float(np.percentile(lat_ms, 99)),
                       "window_latency_ms": [round(x, 1) for x in wlat_ms.tolist()],
                       "window_latency_ms_p50": float(np.percentile(wlat_ms, 50)),
                       "window_latency_ms_p99": float(np.percentile(wlat_ms, 99)),
                       "window_fire": (f"every {a.cand_cadence_ms:g} ms (the stream's window cadence)" if cadence > 0
                                       else "back to back (each window fires as soon as the previous one's chunks "
                                            "are enqueued)"),
                       "window_latency_definition": "window fire (gs_candidates_begin call, host clock) -> the "
                                                    "consumer's end event of its last chunk (device clock mapped "
                                                    "to the host's)",
                       "window_period_s": period, "sustained_edges_per_s": E / period,
                       "target_edges_per_s": 1e8, "checksum": int(chk), "consumer": a.cand_consumer,
                       "id_columns": ("uint32, id - the window's smallest id (gs_candidates_next_u32)" if u32
                                      else "int64 (gs_candidates_next)"), "record_bytes": rec_bytes,
                       "checksum_of": ("the columns' 8-byte words (u32: two ids a word; not comparable across "
                                       "--cand-ids)"),
                       "parallelism": "1 GPU"},
            "roofline": {"bound": "hbm", "kernel": "whole window (emission + consumer)",
                         "achieved": round(rec_bytes * total / elapsed / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(rec_bytes * total / elapsed / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                         "algorithmic_bytes_per_launch": rec_bytes * total, "avg_launch_ms": elapsed * 1e3},
            "cpu_baseline": None}
    if not a.no_cpu_baseline:
        cpu = cand_cpu_baseline(E)
        cpu["gpu_over_cpu"] = round(line["value"] / cpu["value"], 1)
        cpu["window_s_equivalent"] = round(total / W / cpu["value"], 1)   # this window's records at the CPU rate
        line["cpu_baseline"] = cpu
    emit(line)
    for e in engines:
        e.close()


def cand_cpu_baseline(E, sample_log2=25, threads=None):
    """The oracle's GenerateCandidateEdges (the reference's JDK HashSet order) over min(16, nproc) threads WITH
    a consumer that reads every record back (gso_candidates_mt: per-thread chunks of 2^20 records, each summed
    column by column before it is reused -- the GPU line's device consumer), on the largest sample that keeps
    the CPU leg within ~10-30 s: the first 2^sample_log2 edges of the same R-MAT scale-23 stream as one
    window (the whole 1e8-edge window emits 1.6e11 records, minutes of 16 CPU threads).  The CSR build inside
    it runs on one thread, as in gso_window_candidates."""
    orc = ge.load_oracle()
    threads = threads or max(1, min(16, os.cpu_count() or 1))
    n = min(E, 1 << sample_log2)
    s, d = orc.gen_rmat(23, n, 0x5EED05)
    orc.candidates_mt(s[: n // 16], d[: n // 16], threads)   # warm-up
    t = time.perf_counter()
    recs, _ = orc.candidates_mt(s, d, threads)
    dt = time.perf_counter() - t
    return {"value": recs / dt, "unit": "records/s", "cores": threads, "kind": "port",
            "sample": f"first 2^{sample_log2} edges of the R-MAT s23 stream as one window ({recs} records), "
                      f"oracle gso_candidates_mt (emission + a consumer summing every chunk's columns), "
                      f"{threads} threads, {dt:.1f} s",
            "window_s_equivalent": None, **host_cpu()}


def parse_main(a):
    """Input path: the examples' "src trg ts" edge text (WindowTriangles.java:175-185)
    parsed on the GPU (gs_parse_edges_text) from text resident in HBM: R-MAT scale-24 edges with
    ascending millisecond timestamps, 2^24 lines.  CPU baseline: the oracle's parser (same rules), one
    thread, on the whole text."""
    torch.cuda.set_device(0)
    pkg = ge.load_package()
    from gelly_streaming_amd.textio import format_edges_text

    eng = pkg.Engine(0)
    n = 1 << 24
    s, d = eng.generate_rmat(24, n, 0x5EED02)
    ts = np.arange(n, dtype=np.int64) * 1000 // n + 1_700_000_000_000
    text = format_edges_text(s.cpu().numpy(), d.cpu().numpy(), ts)
    dev = torch.from_numpy(np.frombuffer(text, np.uint8).copy()).cuda()
    for _ in range(a.warmup):
        r = eng.parse_edges_text(dev)
    torch.cuda.synchronize()
    lat = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t = time.perf_counter()
        r = eng.parse_edges_text(dev)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t)
    elapsed = time.perf_counter() - t0
    assert torch.equal(r[0], s) and torch.equal(r[1], d), "parsed columns differ from the generated edges"
    ms = statistics.mean(lat) * 1e3
    algo = len(text) + 24 * n      # text in, three int64 columns out (the staging copy is extra traffic)
    cpu = None
    if not a.no_cpu_baseline:
        orc = ge.load_oracle()
        tt = time.perf_counter()
        cs, cd, ct = orc.parse_edges_text(text)
        dt = time.perf_counter() - tt
        assert np.array_equal(cs, s.cpu().numpy()) and np.array_equal(ct, ts)
        cpu = {"value": n / dt, "unit": "edges/s", "cores": 1, "kind": "port",
               "sample": f"the whole text ({len(text) / 1e6:.0f} MB) through oracle gso_parse_edges_text, one thread, "
                         f"{dt:.2f} s"}
    gbs = algo / (ms * 1e-3) / 1e9
    emit({
        "metric": METRIC, "value": n * a.steps / elapsed, "unit": "edges/s", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic R-MAT scale-24 edge text, generated on the host",
        "config": {"workload": "input path: 'src trg ts' edge text -> int64 columns (gs_parse_edges_text)",
                   "records": n, "text_bytes": len(text), "latency_ms_p50": float(np.percentile(np.array(lat) * 1e3, 50)),
                   "parallelism": "1 GPU"},
        "roofline": {"bound": "hbm", "kernel": "parse call (stage + count + starts + parse)", "achieved": round(gbs, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                     "algorithmic_bytes_per_launch": algo, "avg_launch_ms": round(ms, 4)},
        "cpu_baseline": cpu})
    eng.close()


def e2e_main(a):
    """End-to-end windows (BASELINE.md "end-to-end incl. pinned H2D/D2H"): the C2 stream
    (C2: R-MAT scale-24 windows of 2^28 edges with Long values; C5 with --e2e-kind triangles: --windows-edges per window) arrives on the HOST with ascending event timestamps
    (window k: ts in [k*1000, k*1000 + 1000)) and goes through the window-buffer operator (gs_stream_*):
    host columns -> pinned window buffers -> the watermark fires the window -> H2D on the operator's copy
    stream (overlapping the previous window's kernels) -> reduceOnEdges(SUM) -> D2H of the per-vertex
    results.  value = edges / wall time over the timed windows; latency = window fire -> result on the
    host.  Not the headline: the headline keeps the window resident in HBM."""
    torch.cuda.set_device(0)
    pkg = ge.load_package()
    from gelly_streaming_amd import _lib as L
    from gelly_streaming_amd.window_operator import WindowOperator
    eng = pkg.Engine(0)
    tri = a.e2e_kind == "triangles"
    E = int(a.windows_edges) if tri else a.edge_factor << a.scale
    ndist = 2                       # distinct host windows, cycled
    host = []
    for w in range(ndist):
        if tri:   # C5: a continuous R-MAT stream cut into windows of E edges (self-loops removed)
            s_, d_ = eng.generate_rmat(a.scale, E, 0x5EED05, no_self_loops=True, first_edge=w * E)
            host.append((s_.cpu().numpy(), d_.cpu().numpy(), None))
        else:
            s_, d_ = eng.generate_rmat(a.scale, E, a.seed, first_edge=w * E)
            v_ = eng.generate_values(E, a.seed, 1, first_edge=w * E)
            host.append((s_.cpu().numpy(), d_.cpu().numpy(), v_.cpu().numpy()))
            del v_
        del s_, d_
    torch.cuda.empty_cache()
    pinned_bufs = []
    if a.staging == "pinned":   # the caller's columns in pinned host memory (gs_alloc_pinned)
        import ctypes
        lib = L.load()

        def pinned_like(x):
            p = lib.gs_alloc_pinned(x.nbytes)
            assert p, "gs_alloc_pinned failed"
            pinned_bufs.append(p)
            y = np.ctypeslib.as_array((ctypes.c_char * x.nbytes).from_address(p)).view(x.dtype)
            y[:] = x
            return y
        host = [tuple(None if x is None else pinned_like(x) for x in h) for h in host]
    ts0 = (np.arange(E, dtype=np.int64) * 1000) // E
    total = a.warmup + a.steps
    tss = [ts0 + k * 1000 for k in range(total)]   # window k's event times (prepared before timing)
    lat, results = [], []
    staging = L.GS_STAGE_PINNED if a.staging == "buffered" else L.GS_STAGE_DIRECT
    if tri:
        op = WindowOperator(eng, 1000, L.GS_STREAM_TRIANGLES, 2, 0, None, L.GS_WATERMARK_ASCENDING, max_window_edges=E,
                            staging=staging)
    else:
        op = WindowOperator(eng, 1000, L.GS_STREAM_REDUCE, 1, 0, np.int64, L.GS_WATERMARK_ASCENDING, max_window_edges=E,
                            staging=staging)
    t0 = None
    for k in range(total + 1):
        if k == a.warmup:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        if k < total:
            src, dst, val = host[k % ndist]
            op.append(src, dst, val, tss[k])   # fires window k-1 (watermark = max ts - 1)
        else:
            op.flush()
        while (r := op.poll(wait=(k == total))) is not None:
            results.append(r)
            if r.start >= a.warmup * 1000:
                lat.append(r.latency_ms)
            if k < total:
                break
    results += op.drain()
    elapsed = time.perf_counter() - t0
    timed = [r for r in results if r.start >= a.warmup * 1000]
    assert len(timed) == a.steps and all(r.edges == E for r in timed)
    lat = [r.latency_ms for r in timed]
    if a.check and not tri:
        for r in timed[:2]:
            v = host[(r.start // 1000) % ndist][2]
            assert int(r.columns[1].sum()) == int(v.sum()), "e2e window: sum of sums != sum of values"
    op.close()
    for p in pinned_bufs:
        L.load().gs_free_pinned(p)
    ms = elapsed / a.steps * 1e3
    h2d_bytes = (16 if tri else 24) * E
    emit({
        "metric": METRIC, "value": E * a.steps / elapsed, "unit": "edges/s", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int64", "data": f"synthetic R-MAT scale-{a.scale} windows generated on device, copied to host memory "
                                  "before timing; ascending event timestamps",
        "config": {"workload": (f"end-to-end C5 shape: host records of an R-MAT scale-{a.scale} stream, {E} edges per "
                                f"1000 ms window -> gs_stream window operator ({a.staging} staging) -> WindowTriangles"
                                if tri else
                                f"end-to-end C2: host records -> gs_stream window operator ({a.staging}: "
                                + {"buffered": "pageable columns copied into the operator's pinned window buffers, "
                                               "H2D at firing",
                                   "direct": "pageable columns, each append copied straight to HBM",
                                   "pinned": "caller-pinned columns (gs_alloc_pinned), each append DMA'd straight to "
                                             "HBM"}[a.staging] + ", reduceOnEdges(SUM) OUT, D2H of results)"),
                   "edges_per_window": E, "windows_timed": a.steps,
                   "latency_ms_p50": float(np.percentile(lat, 50)), "latency_ms_p99": float(np.percentile(lat, 99)),
                   "h2d_bytes_per_window": h2d_bytes, "h2d_GBps_effective": h2d_bytes / (ms * 1e-3) / 1e9,
                   "vertices_out_per_window": None if tri else int(timed[-1].columns[0].size),
                   "triangles_last_window": int(timed[-1].columns[0]) if tri else None, "parallelism": "1 GPU"},
        "roofline": None, "cpu_baseline": None})
    eng.close()


_JSON_OUT = None


def quiet_native_stdout():
    """The driver reads ONE JSON line from stdout.  RCCL (and other native libraries) print banners to file
    descriptor 1 at communicator init ("RCCL version : ..."), so fd 1 is pointed at stderr for the rest of
    the run and the JSON line goes to a duplicate of the original stdout."""
    global _JSON_OUT
    if _JSON_OUT is None:
        sys.stdout.flush()
        _JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


def emit(line):
    out = _JSON_OUT if _JSON_OUT is not None else sys.stdout
    out.write(json.dumps(line) + "\n")
    out.flush()


def main():
    a = parse()
    quiet_native_stdout()
    if a.workload == "e2e":
        return e2e_main(a)
    if a.workload in ("c1", "apply", "candidates"):
        return window_stream_main(a)
    if a.workload == "cand_stream":
        return cand_stream_main(a)
    if a.workload == "parse":
        return parse_main(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ:   # launched by torchrun: RCCL path (also at world size 1)
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        dist = None
        torch.cuda.set_device(0)
    pkg = ge.load_package()
    from importlib import import_module
    D = import_module("gelly_streaming_amd.distributed")

    eng = pkg.Engine(local, sort_only=a.sort_only, bk_onesweep=a.bk_onesweep, no_pack=a.no_pack, no_spec=a.no_spec,
                     flags=pkg._lib.GS_FLAG_TEST_FORCE_EXCHANGE if a.force_exchange else 0,
                     async_outputs=not a.sync_outputs)
    abi = dist is not None and a.exchange == "abi"
    if abi:   # the ctx-owned RCCL communicator: rank 0's unique id broadcast over torch.distributed
        uid = torch.zeros(128, dtype=torch.uint8, device=f"cuda:{local}")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(pkg.Engine.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        eng.comm_init(world, rank, bytes(uid.cpu().numpy().tobytes()))
    E = a.edge_factor << a.scale
    vdt = 1 if a.dtype == "int64" else 3
    # a.windows distinct windows of the stream (rank r holds windows r*W .. r*W+W-1), cycled by the
    # steps: every step is a different window than the one before it
    wins = []
    for w in range(a.windows):
        fe = (rank * a.windows + w) * E
        if a.workload == "fold" and a.stream == "zipf":   # C3: Zipf(1.1) sources over 2^scale IDs
            src, dst = eng.generate_zipf(1 << a.scale, E, 0x5EED03, 1.1, first_edge=fe)
        elif a.workload == "fold":   # C3: skewed R-MAT (.65/.15/.15/.05), no permutation -> hubs at low IDs
            src, dst = eng.generate_rmat(a.scale, E, 0x5EED03, a=0.65, b=0.15, c=0.15, permute=False, first_edge=fe)
        elif a.workload == "triangles":   # C4 shape: R-MAT, self-loops removed
            src, dst = eng.generate_rmat(a.scale, E, 0x5EED04, no_self_loops=True, first_edge=fe)
        elif a.workload == "cc":          # ConnectedComponents: R-MAT (permuted ids)
            src, dst = eng.generate_rmat(a.scale, E, 0x5EED05, first_edge=fe)
        else:                         # C2
            src, dst = eng.generate_rmat(a.scale, E, a.seed, first_edge=fe)
        val = eng.generate_values(E, a.seed, vdt, first_edge=fe) if a.workload == "reduce" else None
        wins.append((src, dst, val))
    torch.cuda.synchronize()

    local_times = []

    red_out = None   # the output buffers a streaming operator keeps across windows

    def local_reduce(s_, d_, v_, direction, op):
        nonlocal red_out
        R = s_.numel() * (2 if direction == 2 else 1)
        if red_out is None or red_out[0].numel() < R:
            red_out = (torch.empty(R, dtype=torch.int64, device=s_.device),
                       torch.empty(R, dtype=v_.dtype if v_ is not None else torch.int64, device=s_.device))
        r = eng.reduce(s_, d_, v_, direction, op, out=None if a.alloc_outputs else red_out)
        if not local_times:
            local_times.append(eng.stage_times_raw())   # the window's own pipeline, not the merge
        return r

    fold_out = None

    def local_fold(s_, d_, direction, init_max):
        nonlocal fold_out
        R = s_.numel() * (2 if direction == 2 else 1)
        if fold_out is None or fold_out[0].numel() < R:
            fold_out = tuple(torch.empty(R, dtype=torch.int64, device=s_.device) for _ in range(3))
        r = eng.fold_degree_max(s_, d_, direction, init_max, out=None if a.alloc_outputs else fold_out)
        if not local_times:
            local_times.append(eng.stage_times_raw())
        return r

    P_red, M_red, P_fold, M_fold = D.engine_halves(eng)

    def partials_timed(*args):   # the window's own pipeline runs inside the partials half
        r = P_red(*args)
        if not local_times:
            local_times.append(eng.stage_times_raw())
        return r

    def fold_partials_timed(*args):
        r = P_fold(*args)
        if not local_times:
            local_times.append(eng.stage_times_raw())
        return r

    def part_count(s_, d_, part, nparts):
        r = eng.triangles_part(s_, d_, part, nparts)
        local_times.append(eng.stage_times_raw())
        return r

    dist_out = None

    def step(i):
        src, dst, val = wins[i % len(wins)]
        local_times.clear()
        if a.workload == "triangles":
            if abi:    # the split window through gs_window_triangles_dist (RCCL inside the library)
                tot = eng.triangles_dist(src, dst)[0]
                local_times.append(eng.stage_times_raw())
            elif dist:   # the same steps with torch.distributed collectives
                tot = D.triangles_window(eng, src, dst)[0]
                local_times.append(eng.stage_times_raw())
            else:
                tot = part_count(src, dst, 0, 1)
            z = torch.zeros(1, dtype=torch.int64, device=src.device)
            return z + tot, z, local_times[0]
        if a.workload == "cc":   # per-window components (replicas only across GPUs: no exchange)
            r = eng.components(src, dst)
            return r[0], r[1], eng.stage_times()
        if a.workload == "fold":
            if abi:   # gs_window_fold_degree_max_dist: its stage times are the local window's pipeline
                r = eng.fold_degree_max_dist(src, dst, 1)
                local_times.append(eng.stage_times_raw())
            else:
                r = D.fold_degree_max_window(fold_partials_timed, M_fold, src, dst, 1, -(1 << 63)) if dist \
                    else local_fold(src, dst, 1, -(1 << 63))
            return r[0], r[1], local_times[0]
        if abi:       # gs_window_reduce_dist
            nonlocal dist_out
            if dist_out is None and not a.alloc_outputs:   # (kept across windows; 2x the slice's records)
                dist_out = (torch.empty(2 * src.numel() + 1024, dtype=torch.int64, device=src.device),
                            torch.empty(2 * src.numel() + 1024, dtype=val.dtype, device=src.device))
            r = eng.reduce_dist(src, dst, val, 1, 0, out=dist_out)
            local_times.append(eng.stage_times_raw())
        else:
            r = D.reduce_window(partials_timed, M_red, src, dst, val, 1, 0) if dist else local_reduce(src, dst, val, 1, 0)
        return r[0], r[1], local_times[0]

    for i in range(a.warmup):
        step(i)
    # the timed windows record only the dominant kernels' events (gs_set_timing: each event record costs
    # the stream a few microseconds); the other stages are timed on windows after the timed region
    lean = a.workload in ("reduce", "fold") and a.timing == "dominant"
    if lean:
        eng.set_timing(pkg._lib.GS_TIMING_DOMINANT)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    times, us = [], []
    t0 = time.perf_counter()
    for i in range(a.steps):
        k, v, st = step(a.warmup + i)
        times.append(st)
        us.append(int(k.numel()))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # (the timed loop kept each window's raw stage-time struct: StageTimes objects are built after it)
    times = [eng.stage_times_of(t) for t in times]
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    stage_times_after = None
    if lean:
        eng.set_timing(pkg._lib.GS_TIMING_STAGES)
        stage_times_after = [eng.stage_times_of(step(a.warmup + a.steps + i)[2]) for i in range(3)]
        torch.cuda.synchronize()

    checks = {}
    if a.check and world == 1 and a.workload == "reduce":
        for i in range(min(2, len(wins))):
            k, v, _ = step(i)
            val = wins[i][2]
            if a.dtype == "int64":
                assert int(v.sum()) == int(val.sum()), "bench window: sum of per-vertex sums != sum of values"
            assert bool((k[1:] > k[:-1]).all()), "bench window: keys not ascending"
        checks["sums_and_order"] = "ok"

    # local window only: the dominant kernel of the single-GPU pipeline
    E_rec = times[0].records
    U_avg = statistics.mean(t.vertices for t in times)
    if a.workload == "triangles":
        kt, partials = triangle_kernel_table(times, E * world)
        B = 16 * E       # §8(d): the edge-list term; the intersection term is per probe (kernels table)
    elif a.workload == "cc":
        kt, U_cc = cc_kernel_table(times, E)
        partials = 0
        B = 16 * E + 16 * U_cc
    else:
        kt, partials = kernel_table(times, E_rec, U_avg, stage_times_after, nbr_payload=a.workload == "fold")
        B = algorithmic_bytes(a.workload, E, U_avg, 8)
    finish_rows(kt, B)
    dom_name = max((n for n in kt if n not in ("tri_count_light", "tri_count_heavy")), key=lambda n: kt[n]["ms"])
    dom = kt[dom_name]
    ms_step = elapsed / a.steps * 1e3
    pmc = pmc_table()
    pmc_dom = pmc.get(dom_name, {}).get("bytes_per_launch") if a.workload == "reduce" and world == 1 else None
    pmc_window = None
    if a.workload == "reduce" and world == 1 and all(n in pmc for n in kt if kt[n]["bytes"]):
        pmc_window = sum(pmc[n]["bytes_per_launch"] for n in kt if n in pmc)
        if "bucket_merge" in kt:   # the merge stage's time covers k_bk_merge_slices + k_bk_merge
            pmc_window += pmc.get("k_bk_merge_slices", {}).get("bytes_per_launch", 0)
    window_gbs = B / (ms_step * 1e-3) / 1e9 / world
    roofline = {"bound": "hbm", "kernel": dom_name,
                "achieved": round(B / (dom["ms"] * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dom["frac_on_B"], 4), "traffic": pmc_dom,
                "algorithmic_bytes_per_launch": B,
                "algorithmic_bytes_formula": {"reduce": "16E + 16U (SURVEY.md §8d, reduce OUT, 8-byte values)",
                                              "fold": "16E + 24U (SURVEY.md §8d, fold degree/max)",
                                              "triangles": "16E (SURVEY.md §8d edge-list term)",
                                              "cc": "16E + 16U (edge list in, (vertex, label) out)"}[a.workload],
                "avg_launch_ms": round(dom["ms"], 4),
                "kernel_own_bytes_per_launch": dom["bytes"], "kernel_own_frac": round(dom["frac"], 4),
                "whole_window": {"achieved": round(window_gbs, 1), "frac": round(window_gbs / HBM_PEAK_GBS, 4),
                                 "ms": round(ms_step, 4)},
                "window_traffic_pmc": pmc_window,
                "window_traffic_over_B": round(pmc_window / B, 3) if pmc_window else None,
                "traffic_source": ({"file": "profiles/pmc_traffic.json", **pmc.get("_meta", {}),
                                    "running_lib_sha16": lib_sha16(),
                                    "same_build": pmc.get("_meta", {}).get("lib_sha16") == lib_sha16()}
                                   if pmc_dom is not None or pmc_window else None),
                "timing": ("device events on the library's stream (gs_last_stage_times) around the scatter and the "
                           "accumulate inside the timed region (gs_set_timing DOMINANT); the other stages on 3 "
                           "windows after it with every stage event") if lean else
                          "device events on the library's stream around each launch (gs_last_stage_times)"}

    if a.workload == "reduce" and "bucket_accumulate" in kt and dom_name in ("sp_scatter_pack", "sp_scatter",
                                                                            "dp_scatter_pack", "dp_scatter"):
        # north_star's segmented reduce = the partition scatter + the LDS accumulate: B over both kernels'
        # time; and the accumulate alone on its own bytes (the PMC bytes when the table has them)
        acc = kt["bucket_accumulate"]
        t_seg = (dom["ms"] + acc["ms"]) * 1e-3
        acc_b = pmc.get("bucket_accumulate", {}).get("bytes_per_launch") or acc["bytes"]
        roofline["segmented_reduce"] = {
            "kernels": f"{dom_name} + bucket_accumulate", "ms": round(t_seg * 1e3, 4),
            "achieved": round(B / t_seg / 1e9, 1), "frac": round(B / t_seg / 1e9 / HBM_PEAK_GBS, 4),
            "formula": "B / (scatter + accumulate device time)",
            "accumulate": {"ms": round(acc["ms"], 4), "bytes": acc_b,
                           "bytes_source": "PMC" if pmc.get("bucket_accumulate") else "algorithmic",
                           "achieved": round(acc_b / (acc["ms"] * 1e-3) / 1e9, 1) if acc["ms"] > 0 else 0.0,
                           "frac": round(acc_b / (acc["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if acc["ms"] > 0 else 0.0}}
    if a.workload == "triangles":
        # the count step is bound by LDS reads, not HBM: one 16-byte bucket read per hash probe ->
        # 128 B/clk/CU x 256 CUs x 2.4 GHz / 16 B = 4.9 T probes/s (MI355X_MICROARCH.md LDS bandwidth)
        t_cnt = kt["tri_count(light+heavy)"]["ms"] * 1e-3
        peak = 128 * 256 * 2.4e9 / 16 / 1e9
        ach = partials / t_cnt / 1e9 if t_cnt > 0 else 0.0
        roofline["probe_roofline"] = {"bound": "lds", "kernel": "tri_count(light+heavy)", "achieved": round(ach, 1),
                                      "peak": round(peak, 1), "unit": "G probes/s", "frac": round(ach / peak, 4),
                                      "probes_per_window": int(partials),
                                      "peak_formula": "LDS 128 B/clk/CU x 256 CUs x 2.4 GHz / 16 B per bucket read"}
        # SURVEY.md §8(d)'s intersection term beside 16E: a per-edge merge intersection reads both out-lists,
        # 4 B per entry, sum over the oriented edges u -> v of d+(u) + d+(v) (gs_stage_times.escapes, path 3)
        ment = statistics.mean(t.escapes for t in times)
        mb = 4 * ment
        # The count is bound by its LDS probes, not by HBM: the probe roofline governs the line.  The HBM
        # figures of the edge-list term stay beside it; the merge-intersection term is reported as bytes only
        # (the count does not read those bytes -- it probes hash sets / bitmaps -- so bytes over its time would
        # be no fraction of anything: above 1 on every window)
        hbm = {k: roofline.pop(k) for k in list(roofline) if k not in ("probe_roofline",)}
        pr = roofline.pop("probe_roofline")
        roofline.update({"bound": "lds", "kernel": pr["kernel"], "achieved": pr["achieved"], "peak": pr["peak"],
                         "unit": pr["unit"], "frac": pr["frac"], "traffic": None,
                         "probes_per_window": pr["probes_per_window"], "peak_formula": pr["peak_formula"],
                         "hbm_edge_list_term": hbm,
                         "merge_intersection_term": {
                             "bytes_per_window": int(mb), "formula": "4 * sum over oriented edges u->v of (d+(u) + d+(v))",
                             "over_16E": round(mb / B, 2),
                             "note": "what a per-edge merge intersection would read; the count reads one 4-byte list "
                                     "item per probe instead (probes_per_window)"}})

    cpu = None
    threads = max(1, min(16, os.cpu_count() or 1))
    if world == 1 and rank == 0 and not a.no_cpu_baseline:
        if a.workload in ("reduce", "fold"):
            cpu = cpu_baseline(wins, a.workload, threads)
        elif a.workload == "triangles":
            cpu = cpu_baseline_triangles(wins, threads, a.cpu_sample_log2, a.cpu_reps)
        elif a.workload == "cc":
            cpu = cpu_baseline_cc(wins[0][0], wins[0][1])
    value = E * world * a.steps / elapsed
    if cpu:
        cpu["gpu_over_cpu"] = round(value / cpu["value"], 1)
        cpu.update(host_cpu())
        if cpu["cores"] > 1 and cpu["nproc"] > cpu["cores"]:
            # P = nproc; the box allots 16 CPUs per GPU, so the nproc-thread figure is the
            # measured rate scaled linearly (an upper bound for the CPU), labelled as such
            cpu["value_at_nproc_linear"] = cpu["value"] * cpu["nproc"] / cpu["cores"]
            cpu["gpu_over_cpu_at_nproc_linear"] = round(value / cpu["value_at_nproc_linear"], 1)

    if rank == 0:
        t0s = times[0]
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype if a.workload == "reduce" else "int64",
            "data": ("synthetic " + ("Zipf(1.1) sources / uniform destinations" if a.stream == "zipf" and
                                     a.workload == "fold" else "R-MAT") +
                     f", seeded, generated on device; {a.windows} distinct windows per rank cycled by the steps"),
            "config": {"workload": {"reduce": f"C2: slice(OUT).reduceOnEdges(SUM) over R-MAT scale-{a.scale} windows",
                                    "fold": f"C3: slice(OUT).foldNeighbors(degree, max neighbour), skewed "
                                            f"{'Zipf(1.1)' if a.stream == 'zipf' else 'R-MAT'} scale-{a.scale}",
                                    "triangles": f"C4 shape: WindowTriangles over R-MAT scale-{a.scale} windows",
                                    "cc": f"ConnectedComponents of R-MAT scale-{a.scale} windows"}[a.workload],
                       "scale": a.scale, "edges_per_window_per_gpu": E, "windows_cycled": a.windows,
                       "direction": "ALL" if a.workload in ("triangles", "cc") else "OUT",
                       "op": {"reduce": "SUM", "fold": "DegreeMaxNeighbor", "triangles": "count",
                              "cc": "union-find"}[a.workload],
                       "value_dtype": a.dtype, "vertices_out": U_avg, "sort_passes": t0s.sort_passes,
                       "key_bits": t0s.key_bits, "partials_after_fused_pass": int(partials),
                       "pipeline": {0: "sort", 1: "bucket-onesweep", 2: "bucket-direct", 3: "triangles",
                                    4: "components"}[t0s.path],
                       "packed_records": bool(t0s.packed), "escaped_values": int(t0s.escapes),
                       "speculative_windows": sum(1 for t in times if getattr(t, "speculative", 0) == 1),
                       "speculative_misses": sum(1 for t in times if getattr(t, "speculative", 0) == 2),
                       "parallelism": ("1 GPU" if not dist else
                                       f"{world} replicas (per-window components, no exchange)" if a.workload == "cc" else
                                       f"split window over {world} GPUs: summed degrees, oriented edges to owner(u), "
                                       f"all-gathered out-lists, equal-work count shares (gs_tri_dist_*)"
                                       if a.workload == "triangles" else
                                       (f"hash keyBy over {world} GPU(s) through gs_window_*_dist: per-rank partials "
                                        f"-> owner partition -> RCCL all-to-all of sizes + one packed all-to-all of "
                                        f"rows (library communicator) -> merge" if abi else
                                        f"hash keyBy over {world} GPU(s): per-rank partials (gs_window_reduce_partials) "
                                        f"-> torch.distributed all-to-all -> gs_merge_partials")),
                       "exchange": (a.exchange if dist else None),
                       "cpu_baseline_sample": cpu["sample"] if cpu else None, **checks},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels": {n: {"avg_ms": round(r["ms"], 4), "own_bytes": r["bytes"], "GB/s": round(r["GB/s"], 1),
                            "frac": round(r["frac"], 4),
                            **({"frac_on_B": round(r["frac_on_B"], 4)} if n == dom_name else {})}
                        for n, r in kt.items()},
        }
        emit(line)
    if abi:
        eng.comm_destroy()
    if dist:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
