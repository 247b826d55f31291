import sys, numpy as np, torch
sys.path.insert(0, '.')
import __graft_entry__ as ge
pkg = ge.load_package(); orc = ge.load_oracle()
rng = np.random.default_rng(5)
for span in (1 << 22, 1 << 23, 1 << 25):
    for direction in (1, 2):
        n = 20000
        s = rng.integers(0, span, n).astype(np.int64); d = rng.integers(0, span, n).astype(np.int64)
        s[0], d[0] = 0, span - 1
        v = orc.gen_values(n, 1, orc.DT_I64)
        rk, rv = orc.window_reduce(s, d, v, direction, 0)
        with pkg.Engine(0) as e:
            for rep in range(3):
                gk, gv = e.reduce(*[torch.from_numpy(a).cuda() for a in (s, d, v)], direction, 0)
                t = e.stage_times()
                ok = np.array_equal(gk.cpu().numpy(), rk) and np.array_equal(gv.cpu().numpy(), rv)
                print(span, direction, rep, "path", t.path, "spec", t.speculative, "packed", t.packed, "ok", ok, flush=True)
