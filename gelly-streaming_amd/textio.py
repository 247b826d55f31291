"""Edge text files of the examples ("src trg ts" per line, WindowTriangles.java:175-185).

Reading goes through the engine (gs_parse_edges_text, a GPU parser with the reference's
String.split("\\\\s") + Long.parseLong rules).  `format_edges_text` writes such text from int64 columns
(vectorised numpy, used to build test and bench inputs)."""
from __future__ import annotations

import numpy as np

_POW10 = np.array([10 ** k for k in range(19)], dtype=np.uint64)


def _digits(mag: np.ndarray) -> np.ndarray:
    """Decimal digit count of each uint64 (0 -> 1)."""
    n = np.ones(mag.shape, dtype=np.int64)
    for k in range(1, 20):
        n += mag >= (_POW10[k] if k < 19 else np.uint64(10) ** np.uint64(19))
    return n


def format_edges_text(*cols, sep: bytes = b" ", eol: bytes = b"\n") -> bytes:
    """Columns of int64 -> b"c0 c1 c2\\n" lines (Long.toString of each value)."""
    cols = [np.ascontiguousarray(c, dtype=np.int64) for c in cols]
    n = len(cols[0])
    if n == 0:
        return b""
    neg = [c < 0 for c in cols]
    mag = [np.where(ng, (~c.view(np.uint64)) + np.uint64(1), c.view(np.uint64)) for c, ng in zip(cols, neg)]
    width = [_digits(m) + ng for m, ng in zip(mag, neg)]
    line = sum(width) + len(sep) * (len(cols) - 1) + len(eol)
    start = np.zeros(n, dtype=np.int64)
    np.cumsum(line[:-1], out=start[1:])
    buf = np.empty(int(start[-1] + line[-1]), dtype=np.uint8)
    at = start.copy()
    for k, (m, ng, w) in enumerate(zip(mag, neg, width)):
        buf[at[ng]] = ord("-")
        end = at + w - 1                       # position of the last digit
        rem = m.copy()
        for d in range(int(w.max())):
            live = w - ng > d
            buf[(end - d)[live]] = (rem[live] % np.uint64(10)).astype(np.uint8) + ord("0")
            rem //= np.uint64(10)
        at = at + w
        tail = sep if k < len(cols) - 1 else eol
        for j, ch in enumerate(tail):
            buf[at + j] = ch
        at = at + len(tail)
    return buf.tobytes()
