#!/usr/bin/env python3
"""rocprofv3 --stats-style kernel summary (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, StdDev) from a rocprofv3 run_results.db (the SQLite output of --kernel-trace).
usage: tools/db_kernel_stats.py <run_results.db> > kernel_stats.csv"""
import math
import re
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, start, end from kernels").fetchall()
    by = {}
    for n, s, e in rows:
        k = re.sub(r"\(.*", "", n)
        k = re.sub(r"^void ", "", k).split("::")[-1]
        by.setdefault(k, []).append(e - s)
    tot = sum(sum(v) for v in by.values()) or 1
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
    for k, v in sorted(by.items(), key=lambda x: -sum(x[1])):
        m = sum(v) / len(v)
        sd = math.sqrt(sum((x - m) ** 2 for x in v) / len(v))
        print(f'"{k}",{len(v)},{sum(v)},{m:.6f},{100.0 * sum(v) / tot:.2f},{min(v)},{max(v)},{sd:.6f}')


if __name__ == "__main__":
    main()
