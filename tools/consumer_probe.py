"""Read bandwidth of candidate-chunk consumers made of torch reductions (not a bench line): three sums
(a, b, flags) vs one sum over a and b stored back to back, per 2^28-record chunk (4.56 GB)."""
import json

import torch


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    cap = 1 << 28
    ab = torch.randint(0, 1 << 40, (2 * cap,), dtype=torch.int64, device="cuda")
    fl = torch.randint(0, 2, (cap,), dtype=torch.uint8, device="cuda")
    a, b = ab[:cap], ab[cap:]
    res = {
        "three_sums_ms": t(lambda: torch.stack([a.sum(), b.sum(), fl.view(torch.int64).sum()])),
        "one_ab_sum_plus_flags_ms": t(lambda: torch.stack([ab.sum(), fl.view(torch.int64).sum()])),
        "a_sum_ms": t(lambda: a.sum()),
    }
    res["three_sums_TBps"] = round(17 * cap / res["three_sums_ms"] / 1e9, 2)
    res["one_ab_TBps"] = round(17 * cap / res["one_ab_sum_plus_flags_ms"] / 1e9, 2)
    res["a_sum_TBps"] = round(8 * cap / res["a_sum_ms"] / 1e9, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
