"""HBM traffic per launch from separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), per kernel family.

    python tools/pmc_traffic.py <prof dir with fetch/ and write/ runs> [-o profiles/pmc_traffic.json]

rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  MI355X_MICROARCH.md (HBM): on gfx950 FETCH_SIZE
counts half the bytes of a wide coalesced streaming read (128-B requests tallied at 64 B), so the
read side is doubled; WRITE_SIZE is taken as reported.  bench.py puts the corrected sum for the
dominant kernel in roofline.traffic, next to the algorithmic bytes."""
import argparse
import csv
import json
import re
from collections import defaultdict
from pathlib import Path

NAMES = {"k_dp_scatter": "dp_scatter", "k_dp_scatter_pack": "dp_scatter_pack", "k_bk_accum": "bucket_accumulate",
         "k_dp_hist": "dp_hist", "k_sp_scatter_pack": "sp_scatter_pack", "k_sp_scatter": "sp_scatter", "k_sp_regions": "sp_regions",
         "k_bk_merge": "bucket_merge", "k_bk_emit": "bucket_emit"}


def family(name: str) -> str:
    n = re.sub(r"^void ", "", re.sub(r"\(.*", "", name)).split("<")[0].replace("gs::", "")
    return NAMES.get(n, n)


def per_launch(d: Path, counter: str):
    vals = defaultdict(list)
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[family(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("-o", default="profiles/pmc_traffic.json")
    ap.add_argument("--lib", default=str(Path(__file__).resolve().parent.parent / "gelly-streaming_amd" / "libgellyhip.so"),
                    help="the library the passes ran (its sha256 goes into _meta: bench.py checks it)")
    a = ap.parse_args()
    d = Path(a.prof)
    fetch, write = per_launch(d / "fetch", "FETCH_SIZE"), per_launch(d / "write", "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        rd, wr = 2 * fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        out[k] = {"read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
                  "note": "2 x FETCH_SIZE (gfx950 wide-read tally) + WRITE_SIZE, KiB -> bytes, mean per launch"}
    import hashlib
    import subprocess

    lib = Path(a.lib)
    head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                          cwd=Path(__file__).resolve().parent.parent).stdout.strip() or None
    meta = {"lib_sha16": hashlib.sha256(lib.read_bytes()).hexdigest()[:16] if lib.exists() else None,
            "git_head": head, "passes": str(d)}
    Path(a.o).write_text(json.dumps({"_meta": meta, **out}, indent=1) + "\n")
    print(json.dumps({k: round(v["bytes_per_launch"] / 1e9, 3) for k, v in out.items()}))
