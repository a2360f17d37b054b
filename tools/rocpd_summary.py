"""Summaries of a rocprofv3 ``--kernel-trace`` database (rocpd SQLite, the
default output format of rocprofv3 in ROCm 7).

    python tools/rocpd_summary.py DB [--match SUBSTR] [--window NAME_A:NAME_B:k]

* per-kernel table: calls, total / mean / min duration (us), sorted by total;
* ``--window A:B:k``: the k-th span that starts at a kernel whose name contains
  A and ends at the next kernel whose name contains B: every kernel in it with
  its duration and the idle gap before it (a launch-floor timeline).
"""
from __future__ import annotations

import argparse
import re
import sqlite3
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"<.*", "", n) if len(n) > 80 else n
    return n[-70:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--window", default="")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    if a.match:
        rows = [r for r in rows if a.match in r[0]]
    agg = {}
    for name, s, e, d in rows:
        k = short(name)
        t = agg.setdefault(k, [0, 0.0, 1e30])
        t[0] += 1
        t[1] += d / 1e3
        t[2] = min(t[2], d / 1e3)
    print(f"{'kernel':70s} {'calls':>7s} {'total us':>10s} {'mean us':>9s} {'min us':>8s}")
    for k, (n, tot, mn) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{k:70s} {n:7d} {tot:10.1f} {tot / n:9.2f} {mn:8.2f}")
    if a.window:
        A, B, kk = a.window.split(":")
        kk = int(kk)
        starts = [i for i, r in enumerate(rows) if A in r[0]]
        if kk >= len(starts):
            sys.exit(f"only {len(starts)} spans start with {A!r}")
        i0 = starts[kk]
        i1 = next((i for i in range(i0 + 1, len(rows)) if B in rows[i][0]), len(rows) - 1)
        print(f"\nspan {kk}: {i1 - i0 + 1} kernels, {(rows[i1][2] - rows[i0][1]) / 1e3:.1f} us wall")
        busy = 0.0
        for i in range(i0, i1 + 1):
            name, s, e, d = rows[i]
            gap = (s - rows[i - 1][2]) / 1e3 if i > i0 else 0.0
            busy += d / 1e3
            print(f"  +{gap:7.2f} gap  {d / 1e3:7.2f} us  {short(name)}")
        print(f"  busy {busy:.1f} us of {(rows[i1][2] - rows[i0][1]) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
