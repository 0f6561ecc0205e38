#!/usr/bin/env python3
"""Join tools/fetch_calib's known byte counts with the FETCH_SIZE rows of its rocprofv3 --pmc
pass: bytes / (FETCH_SIZE KiB x 1024) per kernel = the factor FETCH_SIZE undercounts by for
that load width and access shape on gfx950 (MI355X_MICROARCH.md HBM section asks for this
calibration before an absolute is trusted).

    python3 tools/fetch_calib.py <rocprof out dir> <fetch_calib stdout json> > profiles/fetch_calib_r2.json

k5_factor: the factor bench.py applies to fas_post_kernel's FETCH_SIZE -- the mean of the
4-B and 8-B widths' factors (entries and norms, the kernel's loads), reported next to
the 16-B factor the guide calibrated."""
import csv
import glob
import json
import os
import sys


def main():
    d, known_path = sys.argv[1], sys.argv[2]
    known = None
    with open(known_path) as f:
        for line in f:
            if line.strip().startswith("{"):
                known = json.loads(line)
    rows = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != "FETCH_SIZE":
                    continue
                name = r["Kernel_Name"]
                for k in ("w4_stream", "w8_stream", "w16_stream", "w4_runs", "w8_runs"):
                    if k in name:
                        rows.setdefault(k, []).append(float(r["Counter_Value"]))
    out = {}
    for k, vals in rows.items():
        vals = vals[1:] if len(vals) > 1 else vals  # the first launch of each runs cold (TLB)
        kib = sum(vals) / len(vals)
        b = known[k]["bytes"]
        out[k] = {"known_bytes": b, "fetch_size_kib": kib, "factor": b / (kib * 1024.0)}
        if "line_bytes" in known[k]:
            out[k]["line_bytes"] = known[k]["line_bytes"]
            out[k]["factor_vs_lines"] = known[k]["line_bytes"] / (kib * 1024.0)
    f4 = [out[k]["factor"] for k in ("w4_stream", "w4_runs", "w8_stream", "w8_runs") if k in out]
    out["k5_factor"] = sum(f4) / len(f4) if f4 else 2.0
    out["note"] = ("factor = known bytes / (FETCH_SIZE KiB * 1024); k5_factor = mean over the 4-B and 8-B widths "
                   "(list entries and norms); runs = 32-entry runs at scattered 128-B-aligned offsets")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
