#!/usr/bin/env python3
"""K5 launch times from a rocprofv3 --kernel-trace of the default cfg-2 bench command (run_results.db):
the timed launches (overlapping on the scan lanes), their completion-to-completion interval (the
steady-state time per launch the bench line's roofline divides by), and the isolated launches after
the timed region.  usage: tools/k5_trace_summary.py <run_results.db> <warmup> <steps> [bench json]"""
import json
import sqlite3
import sys


def main():
    db, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    k5 = [(s, e) for n, s, e in rows if "fas_post_kernel" in n]
    timed = k5[warm:warm + steps]
    iso = k5[warm + steps:warm + steps + min(steps, 20)]
    ends = sorted(e for _, e in timed)
    out = {"k5_dispatches": len(k5),
           "timed_avg_us": sum(e - s for s, e in timed) / len(timed) / 1e3,
           "timed_completion_interval_us": (ends[-1] - ends[0]) / (len(ends) - 1) / 1e3,
           "timed_span_per_launch_us": (max(e for _, e in timed) - min(s for s, _ in timed)) / len(timed) / 1e3,
           "isolated_avg_us": sum(e - s for s, e in iso) / len(iso) / 1e3 if iso else None,
           "isolated_launches": len(iso)}
    if len(sys.argv) > 4:
        d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
        R = d["roofline"]
        out["bench_line"] = {"value": d["value"], "ms_per_step": d["ms_per_step"],
                             "roofline_avg_launch_ms": R["avg_launch_ms"],
                             "events_overlapped_ms": R.get("overlapped_launch", {}).get("avg_launch_ms"),
                             "events_isolated_ms": R.get("isolated_launch", {}).get("avg_launch_ms")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
