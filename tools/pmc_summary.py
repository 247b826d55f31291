"""Summarise rocprofv3 --pmc CSVs per kernel family (mean over dispatches)."""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def family(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    short = n.split("<")[0].replace("gs::", "")
    if "EdgeSrc" in name:
        short += "[edge-src]"
    return short


def load(d):
    rows = defaultdict(lambda: defaultdict(list))
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            rows[family(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return rows


if __name__ == "__main__":
    agg = defaultdict(dict)
    for d in sys.argv[1:]:
        for k, cs in load(d).items():
            for c, v in cs.items():
                agg[k][c] = sum(v) / len(v)
    for k, cs in sorted(agg.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:24s} {v:16.4g}")
