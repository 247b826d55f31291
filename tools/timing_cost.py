"""Cost of the timed region's stage events (not a bench line): C2 windows at GS_TIMING_DOMINANT (the
scatter's and accumulate's events on their dispatches), OFF, and STAGES, alternating, same box."""
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
    E = 1 << 28
    wins = [eng.generate_rmat(24, E, 0x5EED02, first_edge=w * E) for w in range(2)]
    v = eng.generate_values(E, 0x5EED02)
    torch.cuda.synchronize()
    res = {}
    for rep in range(3):
        for name, lvl in (("dominant", L.GS_TIMING_DOMINANT), ("off", L.GS_TIMING_OFF), ("stages", L.GS_TIMING_STAGES)):
            eng.set_timing(lvl)
            for i in range(4):
                eng.reduce(wins[i % 2][0], wins[i % 2][1], v, 1, 0)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(30):
                eng.reduce(wins[i % 2][0], wins[i % 2][1], v, 1, 0)
            torch.cuda.synchronize()
            res.setdefault(name, []).append(round((time.perf_counter() - t) / 30 * 1e3, 4))
    print(json.dumps({"ms_per_window": res}), flush=True)


if __name__ == "__main__":
    main()
