"""GPU: the library's first call in a fresh process (SURVEY.md §8(b) "Errors").

Round 3 recorded `GS_EDEVICE: k_dp_hist: invalid resource handle` on the first gs_window_reduce of a
fresh process (profiles/r03/host_overhead.txt).  The launch checks read the thread's sticky HIP error,
so any earlier failed HIP call of the process -- hipEventElapsedTime on an event the call's path never
recorded (hipErrorInvalidHandle), or a failed call of torch's -- surfaced at the next launch.  The
library now drains that state at every entry point and reads stage times through event_ms(), and
gs_set_stream validates the handle it adopts.

Each case runs in its own interpreter: import torch, create an Engine on torch's current stream, and
reduce a tiny window as the process's first GPU call, bit-exact against the oracle; and the process maps
exactly one HIP runtime (torch bundles libamdhip64.so.7 with the same soname as /opt/rocm's, so the
library binds to whichever loaded first)."""
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent

SCRIPT = textwrap.dedent("""
    import sys
    import numpy as np
    import torch
    sys.path.insert(0, {root!r})
    import __graft_entry__ as ge
    pkg, orc = ge.load_package(), ge.load_oracle()
    eng = pkg.Engine(0)                       # adopts torch's current stream (gs_set_stream)
    s, d = orc.gen_rmat(10, {n}, 7)
    v = orc.gen_values({n}, 7, orc.DT_I64)
    for rep in range(3):
        # the first GPU call of the process: host columns, copied in by the library
        gk, gv = eng.reduce(s, d, v, 1, 0)
        rk, rv = orc.window_reduce(s, d, v, 1, 0)
        assert np.array_equal(np.asarray(gk), rk) and np.array_equal(np.asarray(gv), rv), rep
    side = torch.cuda.Stream()
    eng.set_stream(side.cuda_stream)          # a second live stream: accepted
    gk, gv = eng.reduce(s, d, v, 2, 3)
    rk, rv = orc.window_reduce(s, d, v, 2, 3)
    assert np.array_equal(np.asarray(gk), rk) and np.array_equal(np.asarray(gv), rv)
    eng.close()
    libs = sorted({{l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}})
    assert len(libs) == 1, libs
    print("HIP runtime:", libs[0])
""")


LIBRARY_FIRST = textwrap.dedent("""
    import sys
    import numpy as np
    sys.path.insert(0, {root!r})
    import __graft_entry__ as ge
    pkg, orc = ge.load_package(), ge.load_oracle()
    eng = pkg.Engine(0)                       # the library before any torch call of this script
    s, d = orc.gen_rmat(10, 4096, 7)
    v = orc.gen_values(4096, 7, orc.DT_I64)
    gk, gv = eng.reduce(s, d, v, 1, 0)
    rk, rv = orc.window_reduce(s, d, v, 1, 0)
    assert np.array_equal(np.asarray(gk), rk) and np.array_equal(np.asarray(gv), rv)
    import torch
    assert torch.cuda.is_available()
    x = torch.arange(1000, device="cuda:0").sum().item()
    assert x == 499500, x
    eng.close()
    libs = sorted({{l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}})
    assert len(libs) == 1, libs
    print("HIP runtime:", libs[0])
""")


def test_library_before_torch_in_fresh_process():
    """Loading the library first must not leave torch without a GPU (_lib.load imports torch first: the
    two HIP runtimes share a soname, and torch on the runtime of /opt/rocm found no device)."""
    r = subprocess.run([sys.executable, "-c", LIBRARY_FIRST.format(root=str(ROOT))], capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "HIP runtime:" in r.stdout


@pytest.mark.parametrize("n", [1024, 65536])
def test_first_call_in_fresh_process(n):
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=str(ROOT), n=n)], capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "HIP runtime:" in r.stdout
