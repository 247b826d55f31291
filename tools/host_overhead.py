"""Per-call host + launch overhead of gs_window_reduce: tiny windows (the kernels take a few us), so the
wall time per call is what a window pays besides its kernels.  python tools/host_overhead.py"""
import sys, time
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as ge

pkg = ge.load_package()
eng = pkg.Engine(0)
for n in (1 << 10, 1 << 16):
    s, d = eng.generate_rmat(10, n, 1)
    v = eng.generate_values(n, 1)
    for _ in range(20):
        eng.reduce(s, d, v, 1, 0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    K = 200
    for _ in range(K):
        eng.reduce(s, d, v, 1, 0)
    torch.cuda.synchronize()
    print(f"{n} edges: {(time.perf_counter() - t) / K * 1e6:.1f} us per gs_window_reduce call", flush=True)
eng.close()
