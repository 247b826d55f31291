"""Does gs_merge_partials keep its own speculative partition across windows? (C2-sized partials)"""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as ge

pkg = ge.load_package()
eng = pkg.Engine(0)
E = 1 << 28
wins = []
for w in range(2):
    s, d = eng.generate_rmat(24, E, 0x5EED02, first_edge=w * E)
    v = eng.generate_values(E, 0x5EED02, first_edge=w * E)
    wins.append((s, d, v))
for i in range(8):
    s, d, v = wins[i % 2]
    k, p, cnt = eng.reduce_partials(s, d, v, 1, 0, 2)
    t0 = eng.stage_times()
    mk, mv = eng.merge_partials(k, p, 0)
    t = eng.stage_times()
    print(i, "local: spec", t0.speculative, "packed", t0.packed, "| merge: rows", int(k.numel()), "spec", t.speculative,
          "packed", t.packed, "escapes", t.escapes, "path", t.path, flush=True)
eng.close()
