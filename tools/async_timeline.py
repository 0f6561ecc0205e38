#!/usr/bin/env python3
"""Device timeline of the asynchronous cfg-3 region of a rocprofv3 kernel-trace database: the
kernels of a few consecutive steps with their streams, and the pair kernel's start period
against its duration (the idle share of the step).  usage: tools/async_timeline.py <run_results.db>"""
import re
import sqlite3
import statistics
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    rows = con.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    short = lambda n: re.sub(r"\(.*", "", n).split("::")[-1][:24]
    idx = [i for i, r in enumerate(rows) if "fas_pairs" in r[0]]
    warm = 5
    sel = idx[warm + 5:warm + 9]
    t0 = rows[sel[0]][1]
    for i in range(sel[0] - 3, sel[-1] + 6):
        n, s, e, st = rows[i]
        print("%-26s stream %d start %8.1f dur %7.1f" % (short(n), st, (s - t0) / 1e3, (e - s) / 1e3))
    starts = [rows[i][1] for i in idx[warm:warm + 60]]
    per = [(b - a) / 1e3 for a, b in zip(starts, starts[1:])]
    dur = [(rows[i][2] - rows[i][1]) / 1e3 for i in idx[warm:warm + 60]]
    print("pair kernel start period median %.1f us, mean %.1f; its duration mean %.1f us" %
          (statistics.median(per), statistics.mean(per), statistics.mean(dur)))


if __name__ == "__main__":
    main()
