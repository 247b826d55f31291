import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import __graft_entry__ as ge
pkg = ge.load_package(); orc = ge.load_oracle()
from test_gpu_bucket import VALUE_MIXES, _window
rng = np.random.default_rng(1000)
n = 200_003
s, d = _window(rng, n, 1 << 22, hub_frac=0.02)
dev = lambda *a: [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]
with pkg.Engine(0) as ep:
    for w, mix in enumerate(("narrow", "sparse_wide", "boundary", "all_wide", "narrow")):
        v = VALUE_MIXES[mix](rng, n).astype(np.int64)
        rk, rv = orc.window_reduce(s, d, v, 1, 0)
        kp, vp = ep.reduce(*dev(s, d, v), 1, 0)
        t = ep.stage_times()
        gk, gv = kp.cpu().numpy(), vp.cpu().numpy()
        ok = np.array_equal(gk, rk) and np.array_equal(gv, rv)
        print(mix, "packed", t.packed, "spec", t.speculative, "ok", ok, flush=True)
        if not ok and len(gk) == len(rk):
            bad = np.nonzero(gv != rv)[0]
            print("  bad", len(bad), "keys", gk[bad[:8]], "got", gv[bad[:8]], "want", rv[bad[:8]], "diff", (gv[bad[:8]] - rv[bad[:8]]))
            for kk in gk[bad[:3]]:
                m = s == kk
                print("   key", kk, "records", m.sum(), "vals", v[m][:10])
