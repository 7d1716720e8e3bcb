"""Text tables as github.com/olekukonko/tablewriter v0.0.4 renders them for cyclonus.

Only the features the probe tables use (pkg/connectivity/probe/truthtable.go:101-117,
table.go:58-156): auto-formatted (upper-cased) centred headers, optional row lines, multi-line
cells, default alignment (numbers right, text left), 1-space padding and '+', '-', '|' borders.
Pinned by README.md:294-313.  Long-cell auto-wrapping (cells wider than 30 columns that contain
spaces) is not restated: probe cells never contain spaces.
"""
from __future__ import annotations

import re
import unicodedata

_DECIMAL = re.compile(r"^-?(?:\d{1,3}(?:,\d{3})*|\d+)(?:\.\d+)?$")
_PERCENT = re.compile(r"^-?\d+\.?\d*$%$")


def display_width(s: str) -> int:
    return sum(2 if unicodedata.east_asian_width(c) in ("W", "F") else 1 for c in s)


def title(name: str) -> str:
    """tablewriter util.go Title (v0.0.4): '_' and '.' become spaces, trimmed, upper-cased."""
    orig = len(name)
    name = name.replace("_", " ").replace(".", " ").strip()
    if not name and orig > 0:
        name = " "
    return name.upper()


def _pad_center(s: str, w: int) -> str:
    gap = w - display_width(s)
    if gap <= 0:
        return s
    left = gap // 2
    return " " * left + s + " " * (gap - left)


def _pad_right(s: str, w: int) -> str:
    return s + " " * max(0, w - display_width(s))


def _pad_left(s: str, w: int) -> str:
    return " " * max(0, w - display_width(s)) + s


def render(header, rows, row_line: bool = False) -> str:
    """Render like tablewriter.NewWriter + SetHeader + SetRowLine + Append... + Render."""
    headers = [h.split("\n") for h in header]
    cells = [[str(c).split("\n") for c in r] for r in rows]
    ncol = len(headers)
    widths = [0] * ncol
    for i, h in enumerate(headers):
        widths[i] = max(widths[i], max(display_width(x) for x in h))
    for r in cells:
        for i, c in enumerate(r):
            widths[i] = max(widths[i], max(display_width(x) for x in c))
    line = "+" + "+".join("-" * (w + 2) for w in widths) + "+\n"
    out = [line]
    hmax = max(len(h) for h in headers) if headers else 0
    for x in range(hmax):
        s = "|"
        for y in range(ncol):
            h = headers[y][x] if x < len(headers[y]) else ""
            s += " " + _pad_center(title(h), widths[y]) + " |"
        out.append(s + "\n")
    out.append(line)
    for r in cells:
        rmax = max(len(c) for c in r)
        r = [c + ["  "] * (rmax - len(c)) for c in r]
        for x in range(rmax):
            s = ""
            for y in range(len(r)):
                v = r[y][x]
                t = v.strip()
                pad = _pad_left if (_DECIMAL.match(t) or _PERCENT.match(t)) else _pad_right
                s += "| " + pad(v, widths[y]) + " "
            out.append(s + "|\n")
        if row_line:
            out.append(line)
    if not row_line:
        out.append(line)
    return "".join(out)
