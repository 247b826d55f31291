"""Print the kernel timeline of one window from a rocprofv3 kernel trace (not a bench line).

usage: timeline.py <run_kernel_trace.csv> [marker kernel substring] [which occurrence from the end]
"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x['Start_Timestamp']))
mark = sys.argv[2] if len(sys.argv) > 2 else 'k_sp_scatter_pack'
k = int(sys.argv[3]) if len(sys.argv) > 3 else 3
idx = [i for i, x in enumerate(r) if mark in x['Kernel_Name']]
a, b = idx[-k], idx[-k + 1]
t0 = int(r[a]['Start_Timestamp'])
prev = None
for x in r[a:b]:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    gap = (s - prev) / 1000 if prev else 0
    print(f"{(s - t0) / 1000:8.1f} +{gap:6.1f} {(e - s) / 1000:7.1f} {x['Kernel_Name'][:80]}")
    prev = e
print('window us', (int(r[b]['Start_Timestamp']) - t0) / 1000)
