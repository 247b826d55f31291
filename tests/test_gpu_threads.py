"""GPU: the threading contract of include/gelly_hip.h (SURVEY.md §8(b) "Threading"): Flink runs each
window-operator subtask on its own task thread (local-env parallelism = cores), so several subtasks
call the library at once, one gs_ctx each.  Here 4 host threads each drive their own ctx (own HIP
stream and workspace) through a sequence of windows concurrently -- reduce, fold, the degree fold and
WindowTriangles, host batches copied in by the library -- and every result must equal the oracle's
bit for bit.  ctypes releases the GIL around each C call, so the calls really overlap."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 4


def _jobs(oracle, t):
    """The windows thread t runs, with the oracle's answers."""
    jobs = []
    for w in range(3):
        seed = 1000 * t + w
        s, d = oracle.gen_rmat(16 + (w % 2) * 2, 150_000 + 7919 * t, seed, a=0.6, b=0.15, c=0.15)
        v = oracle.gen_values(len(s), seed, oracle.DT_I64)
        jobs.append(("reduce", (s, d, v, (t + w) % 3, w % 4), oracle.window_reduce(s, d, v, (t + w) % 3, w % 4)))
        jobs.append(("fold", (s, d, v, 1, 0, -5), oracle.window_fold(s, d, v, 1, 0, -5)))
        jobs.append(("deg", (s, d, 2), oracle.window_fold_degree_max(s, d, 2)))
        ts, td = oracle.gen_rmat(12, 40_000, seed, no_self_loops=True)
        w_, ex, has = oracle.window_triangles_fwd(ts, td)
        jobs.append(("tri", (ts, td), (ex, w_, has)))
    return jobs


def test_concurrent_contexts_bit_exact(pkg, oracle):
    work = [_jobs(oracle, t) for t in range(THREADS)]
    errors, done = [], [0] * THREADS
    start = threading.Barrier(THREADS)

    def run(t):
        try:
            with pkg.Engine(0, torch_stream=False) as e:
                start.wait()
                for rep in range(2):
                    for kind, args, want in work[t]:
                        if kind == "reduce":
                            got = e.reduce(*args)
                        elif kind == "fold":
                            got = e.fold(*args)
                        elif kind == "deg":
                            got = e.fold_degree_max(*args)
                        else:
                            got = e.triangles(*args)
                            assert got == want, (t, kind, got, want)
                            done[t] += 1
                            continue
                        for g, w in zip(got, want):
                            assert np.array_equal(np.asarray(g), w), (t, kind)
                        done[t] += 1
        except BaseException as ex:   # reported by the main thread
            errors.append((t, repr(ex)))

    ths = [threading.Thread(target=run, args=(t,)) for t in range(THREADS)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths), "a thread hung"
    assert not errors, errors
    assert done == [2 * len(w) for w in work]
