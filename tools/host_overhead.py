"""Host time per reduce call (not a bench line): engine.reduce (Python wrapper: output tensors, batch
struct, ctypes) against the bare ctypes call with preallocated outputs, on a small window whose kernels
take a few microseconds, and on C2 windows (GPU-bound: the difference is the host turnaround)."""
import ctypes
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    L = pkg._lib
    eng = pkg.Engine(0)
    eng.set_timing(L.GS_TIMING_OFF)
    out = {}
    for name, scale, E in (("small", 12, 1 << 16), ("c2", 24, 1 << 28)):
        s, d = eng.generate_rmat(scale, E, 0x5EED02)
        v = eng.generate_values(E, 0x5EED02)
        torch.cuda.synchronize()
        reps = 200 if name == "small" else 20
        for _ in range(5):
            eng.reduce(s, d, v, 1, 0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            eng.reduce(s, d, v, 1, 0)
        torch.cuda.synchronize()
        py = (time.perf_counter() - t) / reps * 1e6
        b, keep, dev = eng._batch(s, d, v)
        keys = torch.empty(E, dtype=torch.int64, device="cuda:0")
        vals = torch.empty(E, dtype=torch.int64, device="cuda:0")
        n_out = ctypes.c_uint64(0)
        o = L.GsVertexOut(keys.data_ptr(), vals.data_ptr(), E, ctypes.pointer(n_out), L.GS_MEM_DEVICE, 0)
        f = eng._L.gs_window_reduce
        for _ in range(5):
            f(eng.ctx, ctypes.byref(b), 1, 0, ctypes.byref(o))
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            f(eng.ctx, ctypes.byref(b), 1, 0, ctypes.byref(o))
        torch.cuda.synchronize()
        bare = (time.perf_counter() - t) / reps * 1e6
        out[name] = {"engine_reduce_us": round(py, 1), "bare_ctypes_us": round(bare, 1)}
        del s, d, v, keys, vals
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
