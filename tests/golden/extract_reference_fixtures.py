"""Extract the reference's own golden vectors into tests/golden/reference_fixtures.json.

Run in the build container (where /root/reference exists):
    python tests/golden/extract_reference_fixtures.py
The JSON it writes is committed; the GPU box never reads /root/reference.

It parses DATA out of the reference's test sources (read as text):
  - GraphStreamTestUtils.java:56-67   the 7-edge Long/Long graph  (new Edge<>(1L, 2L, 12L) ...)
  - TestSlice.java:70-229             9 goldens: {fold,reduce,apply} x {default=OUT, IN, ALL}
  - TestReverse.java / TestUndirected.java   expected edge lists of reverse() / undirected()
  - ExamplesTestData.java:21-34       TRIANGLES_DATA and TRIANGLES_RESULT; window 400 ms
                                       from WindowTrianglesITCase.java:43
  - ConnectedComponentsTest.java:19-38  the 6 edges, the expected components, the 5 ms merge window
  - DisjointSetTest.java:19-64          union(i, i + 2) for i < 8 -> 10 elements / 2 roots; merged with
                                       union(i, i + 100) for i < 8 -> 18 elements / 2 roots
Only inputs and expected outputs are written — no reference source text.
"""
from __future__ import annotations

import json
import re
import sys
from pathlib import Path

REF = Path("/root/reference/src/test/java/org/apache/flink/graph/streaming")
OUT = Path(__file__).resolve().parent / "reference_fixtures.json"


def _expected_blocks(text: str):
    """Map test method name -> expected lines ("a,b") in order of appearance."""
    out = {}
    for m in re.finditer(r"public void (test\w+)\(\)(.*?)(?=public void test|\Z)", text, re.S):
        name, body = m.group(1), m.group(2)
        em = re.search(r"expectedResult\s*=\s*((?:\"[^\"]*\"\s*\+?\s*)+);", body, re.S)
        if not em:
            continue
        s = "".join(re.findall(r"\"([^\"]*)\"", em.group(1)))
        lines = [ln for ln in s.replace("\\n", "\n").split("\n") if ln]
        direction = "ALL" if "EdgeDirection.ALL" in body else ("IN" if "EdgeDirection.IN" in body else "OUT")
        out[name] = {"direction": direction, "expected": lines}
    return out


def main() -> int:
    utils = (REF / "test" / "GraphStreamTestUtils.java").read_text()
    edges = [tuple(int(x) for x in m) for m in
             re.findall(r"new Edge<>\((\d+)L,\s*(\d+)L,\s*(\d+)L\)", utils)]
    slice_src = (REF / "test" / "operations" / "TestSlice.java").read_text()
    slice_cases = _expected_blocks(slice_src)
    # which op each test exercises (method-name prefix) and its golden
    cases = []
    for name, c in slice_cases.items():
        kind = ("fold" if name.startswith("testFold") else "reduce" if name.startswith("testReduce") else "apply")
        cases.append({"name": name, "kind": kind, "direction": c["direction"],
                      "expected": [ln.split(",") for ln in c["expected"]]})

    def edge_lines(path):
        t = path.read_text()
        em = re.search(r"expectedResult\s*=\s*((?:\"[^\"]*\"\s*\+?\s*)+);", t, re.S)
        s = "".join(re.findall(r"\"([^\"]*)\"", em.group(1))).replace("\\n", "\n")
        return [[int(x) for x in ln.split(",")] for ln in s.split("\n") if ln]

    reverse = edge_lines(REF / "test" / "operations" / "TestReverse.java")
    undirected = edge_lines(REF / "test" / "operations" / "TestUndirected.java")

    etd = (REF / "example" / "util" / "ExamplesTestData.java").read_text()
    tri_data = "".join(re.findall(r"\"([^\"]*)\"", re.search(r"TRIANGLES_DATA\s*=(.*?);", etd, re.S).group(1)))
    tri_edges = [[int(x) for x in ln.split()] for ln in tri_data.replace("\\n", "\n").split("\n") if ln.strip()]
    tri_res = "".join(re.findall(r"\"([^\"]*)\"", re.search(r"TRIANGLES_RESULT\s*=(.*?);", etd, re.S).group(1)))
    tri_out = [[int(x) for x in re.findall(r"-?\d+", ln)] for ln in tri_res.replace("\\n", "\n").split("\n") if ln]
    itcase = (REF / "example" / "test" / "WindowTrianglesITCase.java").read_text()
    window_ms = int(re.search(r"WindowTriangles\.main\(new String\[\]\{[^}]*\"(\d+)\"\}\)", itcase).group(1))

    cct = (REF / "example" / "test" / "ConnectedComponentsTest.java").read_text()
    cc_edges = [[int(a), int(b)] for a, b in re.findall(r"new Edge<>\((\d+)L,\s*(\d+)L,\s*NullValue", cct)]
    cc_res = "".join(re.findall(r"\"([^\"]*)\"", re.search(r"Connected_RESULT\s*=(.*?);", cct, re.S).group(1)))
    cc_comps = [sorted(int(x) for x in re.findall(r"\d+", ln)) for ln in cc_res.replace("\\n", "\n").split("\n") if ln.strip()]
    cc_ms = int(re.search(r"new ConnectedComponents<[^>]*>\((\d+)\)", cct).group(1))
    dst_ = (REF / "example" / "util" / "DisjointSetTest.java").read_text()
    setup = re.search(r"for \(int i = 0; i < (\d+); i\+\+\) \{\s*ds\.union\(i, i \+ (\d+)\);", dst_)
    merge = re.search(r"for \(int i = 0; i < (\d+); i\+\+\) \{\s*ds2\.union\(i, i \+ (\d+)\);", dst_)
    sizes = [int(x) for x in re.findall(r"assertEquals\((?:ds\.getMatches\(\)\.size\(\), )?(\d+)", dst_)]
    roots = [int(x) for x in re.findall(r"assertEquals\((\d+), treeRoots\.size\(\)\)", dst_)]
    ds = {"unions": [[i, i + int(setup.group(2))] for i in range(int(setup.group(1)))],
          "size": sizes[0], "roots": 2,   # testFind: find(0) != find(1), every i has the root of i % 2
          "merge_unions": [[i, i + int(merge.group(2))] for i in range(int(merge.group(1)))],
          "merged_size": sizes[1], "merged_roots": roots[0]}

    fixtures = {
        "source": "Ren91/gelly-streaming test sources (see extract_reference_fixtures.py docstring)",
        "slice_graph": {"edges": edges, "window_ms": 1000,
                        "note": "TestSlice uses 1 s ingestion-time windows; all 7 edges fall in one window"},
        "slice_cases": cases,
        "reverse_expected": reverse,
        "undirected_expected": undirected,
        "triangles": {"edges_src_trg_ts": tri_edges, "window_ms": window_ms, "expected": tri_out},
        "connected_components": {"edges": cc_edges, "merge_window_ms": cc_ms, "expected": cc_comps},
        "disjoint_set": ds,
    }
    OUT.write_text(json.dumps(fixtures, indent=1) + "\n")
    print(f"wrote {OUT} ({len(edges)} slice edges, {len(cases)} slice cases, {len(tri_edges)} triangle edges)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
