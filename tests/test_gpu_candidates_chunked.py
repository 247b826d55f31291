"""GPU: GenerateCandidateEdges emitted in chunks (gs_candidates_begin / gs_candidates_next;
WindowTriangles.java:91-114).  A window's output is O(sum d^2) -- 1.6e11 records for one C5 window --
so a consumer streams it: the concatenated chunks must equal gs_window_candidates (and the oracle's
GenerateCandidateEdges) record for record at every chunk size, with chunk boundaries inside a vertex's
edge records and inside one pair row, exact JDK HashSet orders included; device and host outputs; a
later call on the ctx ends the session."""
import numpy as np
import pytest
import torch

from test_gpu_api import _cand_case, _jdk_case

pytestmark = pytest.mark.gpu


def _stream(engine, s, d, cap, dev=True):
    args = (torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()) if dev else (s, d)
    total = engine.candidates_begin(*args)
    parts, at, done = [], 0, False
    while not done:
        a, b, f, first, done = engine.candidates_next(cap)
        assert first == at and (len(a) == cap or done)
        at += len(a)
        parts.append([x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x) for x in (a, b, f)])
    assert at == total
    return [np.concatenate([p[i] for p in parts]) for i in range(3)], total


@pytest.mark.parametrize("kind", ["small_ids", "sparse_ids", "negative_ids", "rmat"])
@pytest.mark.parametrize("cap", [1, 7, 1000, 1 << 20])
def test_chunks_concatenate_to_the_window(engine, oracle, kind, cap):
    rng = np.random.default_rng(hash((kind, cap)) & 0xFFFF)
    for trial in range(2 if cap == 1 else 3):
        s, d = _cand_case(oracle, rng, kind)
        ra, rb, rf, flags = oracle.window_candidates(s, d)
        (ga, gb, gf), total = _stream(engine, s, d, cap, dev=trial % 2 == 0)
        assert total == len(ra) == engine.candidate_count(s, d)
        assert np.array_equal(ga, ra) and np.array_equal(gb, rb) and np.array_equal(gf, rf), (kind, cap, trial)


@pytest.mark.parametrize("case", ["tree24", "many_vertices", "rmat_shifted"])
def test_chunks_exact_jdk_order(engine, oracle, case):
    s, d = _jdk_case(oracle, case)
    ra, rb, rf, flags = oracle.window_candidates(s, d)
    for cap in (333, 65536):
        (ga, gb, gf), total = _stream(engine, s, d, cap)
        assert engine.last_candidates_jdk_flags == flags
        assert np.array_equal(ga, ra) and np.array_equal(gb, rb) and np.array_equal(gf, rf)


def test_chunks_of_a_hub_window_equal_the_whole(engine, oracle):
    """A 600k-edge R-MAT window (hub rows of thousands of pairs): chunks of 2^20 records vs the whole
    window's gs_window_candidates on the device."""
    s, d = oracle.gen_rmat(14, 600_000, 0x5EED05)
    S, D = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    wa, wb, wf = engine.candidates(S, D)
    (ga, gb, gf), total = _stream(engine, s, d, 1 << 20)
    assert total == len(wa) > 10 ** 7
    assert np.array_equal(ga, wa.cpu().numpy()) and np.array_equal(gb, wb.cpu().numpy())
    assert np.array_equal(gf, wf.cpu().numpy())


def test_session_ends_at_the_next_call(pkg, engine, oracle):
    s, d = oracle.gen_rmat(8, 3000, 7)
    engine.candidates_begin(s, d)
    engine.candidates_next(10)
    engine.reduce(s, d, np.ones(len(s), np.int64), 1, 0)   # another entry point on the ctx
    with pytest.raises(pkg.GsError):
        engine.candidates_next(10)


def _stream_u32(engine, s, d, cap, dev=True):
    args = (torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()) if dev else (s, d)
    total = engine.candidates_begin(*args)
    parts, at, done, base = [], 0, False, None
    while not done:
        a, b, f, first, done, base = engine.candidates_next_u32(cap)
        assert first == at and (len(a) == cap or done)
        at += len(a)
        parts.append([x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x) for x in (a, b, f)])
    assert at == total
    a, b, f = (np.concatenate([p[i] for p in parts]) for i in range(3))
    assert a.dtype == np.uint32 and b.dtype == np.uint32
    return (a.astype(np.int64) + base, b.astype(np.int64) + base, f), base


@pytest.mark.parametrize("kind", ["small_ids", "sparse_ids", "negative_ids", "rmat"])
@pytest.mark.parametrize("cap", [7, 1 << 20])
def test_u32_chunks_equal_the_oracle(engine, oracle, kind, cap):
    """gs_candidates_next_u32: the same records as gs_candidates_next with every id as id - id_base in a
    uint32 column (id_base = the window's smallest id; negative and sparse ids included)."""
    rng = np.random.default_rng(hash(("u32", kind, cap)) & 0xFFFF)
    for trial in range(3):
        s, d = _cand_case(oracle, rng, kind)
        ra, rb, rf, flags = oracle.window_candidates(s, d)
        (ga, gb, gf), base = _stream_u32(engine, s, d, cap, dev=trial != 1)
        assert base == min(s.min(), d.min())
        assert np.array_equal(ga, ra) and np.array_equal(gb, rb) and np.array_equal(gf, rf), (kind, cap, trial)


def test_u32_chunks_of_a_hub_window(engine, oracle):
    s, d = oracle.gen_rmat(14, 600_000, 0x5EED06)
    s, d = s + (5 << 40), d + (5 << 40)   # ids far from 0, span < 2^32
    S, D = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    wa, wb, wf = engine.candidates(S, D)
    (ga, gb, gf), base = _stream_u32(engine, s, d, 1 << 20)
    assert len(ga) == len(wa) > 10 ** 7 and base == min(s.min(), d.min())
    assert np.array_equal(ga, wa.cpu().numpy()) and np.array_equal(gb, wb.cpu().numpy())
    assert np.array_equal(gf, wf.cpu().numpy())


def test_u32_refuses_a_span_past_2_32(pkg, engine, oracle):
    s, d = oracle.gen_rmat(8, 3000, 9)
    s = s.copy()
    s[0] = 1 << 33   # one id 2^33 away from the rest
    engine.candidates_begin(s, d)
    with pytest.raises(pkg.GsError):
        engine.candidates_next_u32(100)
    a, b, f, first, done = engine.candidates_next(1 << 20)   # the session stays usable with 64-bit ids
    ra, rb, rf, flags = oracle.window_candidates(s, d)
    assert first == 0 and done and np.array_equal(np.asarray(a), ra) and np.array_equal(np.asarray(b), rb)


@pytest.mark.parametrize("u32", [False, True])
def test_chunks_into_unaligned_columns(engine, oracle, u32):
    """Output columns that start off their natural 16-byte (ids) and 4-byte (flags) alignment: the emission's
    vector stores give way to per-record stores, with the same records."""
    s, d = oracle.gen_rmat(12, 40_000, 0x5EED07)
    ra, rb, rf, flags = oracle.window_candidates(s, d)
    cap = 1 << 18
    idt = torch.uint32 if u32 else torch.int64
    raw = [torch.zeros(cap + 3, dtype=idt, device="cuda") for _ in range(2)] + \
          [torch.zeros(cap + 5, dtype=torch.uint8, device="cuda")]
    bufs = (raw[0][1:cap + 1], raw[1][3:cap + 3], raw[2][1:cap + 1])   # a, b off 16-byte alignment, f off 4
    total = engine.candidates_begin(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda())
    got, done = [], False
    while not done:
        if u32:
            a, b, f, first, done, base = engine.candidates_next_u32(cap, bufs)
            a, b = a.cpu().numpy().astype(np.int64) + base, b.cpu().numpy().astype(np.int64) + base
        else:
            a, b, f, first, done = engine.candidates_next(cap, bufs)
            a, b = a.cpu().numpy(), b.cpu().numpy()
        got.append((a, b, f.cpu().numpy()))
    ga, gb, gf = (np.concatenate([g[i] for g in got]) for i in range(3))
    assert len(ga) == total == len(ra)
    assert np.array_equal(ga, ra) and np.array_equal(gb, rb) and np.array_equal(gf, rf)
