"""Per-item timeline of k_bk_accum on C2 windows (not a bench line).  Needs the GS_BK_TRACE tuning build
(GELLY_HIP_LIB=gelly-streaming_amd/variants/trace/libgellyhip.so): its accumulate records per item the
workgroup, the wall clock at start / end (100 MHz) and the records (gs_debug_bk_trace).  Runs 4 windows and
prints per window: the kernel's span, the workgroups' busy time, when they ran out of items, and the
largest items started last."""
import ctypes
import json

import numpy as np
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    eng = pkg.Engine(0)
    E = 1 << 28
    val = eng.generate_values(E, 0x5EED02)
    wins = [eng.generate_rmat(24, E, 0x5EED02, first_edge=w * E) for w in range(2)]
    torch.cuda.synchronize()
    eng.set_timing(pkg._lib.GS_TIMING_OFF)
    L = pkg._lib.load()
    buf = np.zeros((16384, 4), dtype=np.uint64)
    for rep in range(4):
        s, d = wins[rep % 2]
        eng.reduce(s, d, val, 1, 0)
        torch.cuda.synchronize()
        buf[:] = 0
        assert L.gs_debug_bk_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(16384)) == 0
        t = buf[buf[:, 2] > 0]
        wg, t0, t1, n = t[:, 0], t[:, 1].astype(np.int64), t[:, 2].astype(np.int64), t[:, 3]
        base = t0.min()
        span = (t1.max() - base) / 100.0   # us
        busy = np.zeros(int(wg.max()) + 1)
        last = np.zeros(int(wg.max()) + 1)
        np.add.at(busy, wg.astype(int), (t1 - t0) / 100.0)
        np.maximum.at(last, wg.astype(int), (t1 - base) / 100.0)
        dur = (t1 - t0) / 100.0
        print(json.dumps({"window": rep, "items": int(len(t)), "span_us": round(span, 1),
                          "busy_us_mean": round(float(busy.mean()), 1), "busy_us_max": round(float(busy.max()), 1),
                          "wg_done_us_p10_p50_p90": [round(float(x), 1) for x in np.percentile(last, [10, 50, 90])],
                          "item_us_mean": round(float(dur.mean()), 2), "us_per_M_records": round(float(dur.sum() / n.sum() * 1e6), 2),
                          "fit_us_per_item_us_per_M": [round(float(x), 2) for x in np.polyfit(n.astype(np.float64) / 1e6, dur, 1)[::-1]],
                          "first_starts_us_p50_max": [round(float(x), 1) for x in np.percentile(np.array([((t0[wg == g] - base).min()) / 100.0 for g in np.unique(wg)]), [50, 100])],
                          "item_start_gap_us_mean": round(float(((t0 - base) / 100.0)[np.argsort(t0)][1:].mean()), 1)}),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
