"""Probe of the bucket path's stages on C2-size windows of different skew (not a bench line).

reduceOnEdges(SUM, OUT) over 2^28-edge windows of R-MAT scale 24 with the Graph500 skew (C2), a milder
skew and the uniform case (a = b = c = 0.25), two windows each, then the stage times of a few more
windows with every stage event on: whether the accumulate's time follows the hubs (same-address LDS
atomics) or not.  Prints one JSON line per stream.  GELLY_HIP_LIB selects a tuning build.
"""
import json
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
    for name, (a, b, c) in (("graph500", (0.57, 0.19, 0.19)), ("mild", (0.35, 0.22, 0.22)), ("uniform", (0.25, 0.25, 0.25))):
        wins = [eng.generate_rmat(24, E, 0x5EED02 + w, a=a, b=b, c=c) for w in range(2)]
        torch.cuda.synchronize()
        eng.set_timing(pkg._lib.GS_TIMING_STAGES)
        rows = []
        for rep in range(8):
            s, d = wins[rep % 2]
            k, v = eng.reduce(s, d, val, 1, 0)
            t = eng.stage_times()
            if rep >= 2:
                rows.append(t.pass_ms)
        avg = [round(sum(r[i] for r in rows) / len(rows), 4) for i in range(len(rows[0]))]
        deg = torch.bincount(wins[0][0]).max().item()
        print(json.dumps({"stream": name, "abc": [a, b, c], "max_out_degree": deg, "vertices_out": int(k.numel()),
                          "pass_ms(scans,scatter,accumulate,merge,emit)": avg}), flush=True)
        del wins
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
