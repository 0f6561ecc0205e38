#!/usr/bin/env python3
"""Per-kernel totals and the device timeline of the last steps of a rocprofv3 --kernel-trace
database (run_results.db): which kernels a step launches, their durations, and the idle gaps
between them (host-bound stretches).  usage: tools/trace_steps.py <run_results.db> [kernel-substr]"""
import re
import sqlite3
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"<.*>", "", n)
    return n.split("::")[-1]


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, start, end, grid_x, grid_y from kernels order by start").fetchall()
    mark = sys.argv[2] if len(sys.argv) > 2 else "fas_pairs_kernel"
    tot = {}
    for n, s, e, gx, gy in rows:
        k = short(n)
        t = tot.setdefault(k, [0, 0.0])
        t[0] += 1
        t[1] += (e - s) / 1e3
    print("kernel totals (calls, us):")
    for k, (c, us) in sorted(tot.items(), key=lambda x: -x[1][1])[:14]:
        print(f"  {k:34s} {c:6d} {us:12.1f} {us / c:9.1f}/call")
    idx = [i for i, r in enumerate(rows) if mark in r[0]]
    if len(idx) < 4:
        return
    # the window between the 4th-last and the last marker launch: about three steps
    a, b = idx[-4], idx[-1]
    w = rows[a:b]
    busy = sum(e - s for _, s, e, _, _ in w) / 1e3
    span = (w[-1][2] - w[0][1]) / 1e3
    print(f"last 3 steps: span {span:.1f} us, kernels busy {busy:.1f} us ({100 * busy / span:.0f}%)")
    prev = w[0][1]
    for n, s, e, gx, gy in w:
        print(f"  gap {(s - prev) / 1e3:8.1f}  {short(n):30s} {(e - s) / 1e3:8.1f} us  grid {gx}x{gy}")
        prev = e


if __name__ == "__main__":
    main()
