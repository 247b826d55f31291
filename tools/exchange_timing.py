"""Per-phase timing of the multi-GPU keyBy exchange (distributed.py) on one C2 window.
Run under torchrun (any world size): local bucket reduce, exchange_sorted, merge reduce, each bracketed
by torch.cuda.synchronize().  At world 1 the exchange is forced (reduce_window skips it there)."""
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as ge  # noqa: E402

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
rank = dist.get_rank()
pkg = ge.load_package()
from gelly_streaming_amd import distributed as D  # noqa: E402

eng = pkg.Engine(local)
E = 1 << 28
src, dst = eng.generate_rmat(24, E, 0x5EED02, first_edge=rank * E)
val = eng.generate_values(E, 0x5EED02, 1, first_edge=rank * E)
ph = {"local": [], "exchange": [], "merge": []}
for it in range(8):
    torch.cuda.synchronize(); dist.barrier(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    k, v = eng.reduce(src, dst, val, 1, 0)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    rk, (rv,) = D.exchange_sorted(k, [v])
    torch.cuda.synchronize(); t2 = time.perf_counter()
    mk, mv = eng.reduce(rk, rk, rv, 1, 0)
    torch.cuda.synchronize(); t3 = time.perf_counter()
    if it >= 2:
        ph["local"].append((t1 - t0) * 1e3)
        ph["exchange"].append((t2 - t1) * 1e3)
        ph["merge"].append((t3 - t2) * 1e3)
if rank == 0:
    print({n: round(sum(x) / len(x), 3) for n, x in ph.items()}, "local U", k.numel(), "received", rk.numel(),
          "owned", mk.numel(), flush=True)
dist.destroy_process_group()
