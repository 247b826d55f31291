"""Idle time inside and between C2 windows from a rocprofv3 kernel trace (not a bench line).

usage: window_gaps.py <run_kernel_trace.csv> [first kernel of a window, default k_sp_regions]
Per window (from one first kernel to the next): the span, the sum of kernel durations, the idle time
between consecutive kernels, and the gap from the previous window's last kernel to this one's first
(the host turnaround: read-back wait, bookkeeping, the next call's launches)."""
import csv
import statistics
import sys

r = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
mark = sys.argv[2] if len(sys.argv) > 2 else "k_sp_regions"
idx = [i for i, x in enumerate(r) if mark in x["Kernel_Name"]]
rows = []
for a, b in zip(idx, idx[1:]):
    ks = r[a:b]
    span = (int(r[b]["Start_Timestamp"]) - int(ks[0]["Start_Timestamp"])) / 1e3
    busy = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in ks) / 1e3
    inner = sum(max(0, int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) for x, y in zip(ks, ks[1:])) / 1e3
    turn = (int(r[b]["Start_Timestamp"]) - int(ks[-1]["End_Timestamp"])) / 1e3
    names = [x["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0] for x in ks]
    if not any("scatter" in n for n in names):
        continue
    rows.append((span, busy, inner, turn, len(ks)))
    print(f"window us {span:8.1f}  kernels {busy:8.1f}  gaps inside {inner:6.1f}  turnaround {turn:6.1f}  launches {len(ks)}")
if rows:
    med = lambda j: statistics.median(x[j] for x in rows)
    print(f"median: window {med(0):.1f} us, kernels {med(1):.1f}, gaps inside {med(2):.1f}, turnaround {med(3):.1f}")
