#!/usr/bin/env python3
"""Per-launch means of every counter in the rocprofv3 --pmc passes under a directory
(tools/pmc_passes.sh output), for kernels matching a name fragment; the first quarter of
the launches (warmup) is dropped.   python3 tools/pmc_sq.py <dir> [kernel-fragment]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    frag = sys.argv[2] if len(sys.argv) > 2 else "fas_post_kernel"
    vals = defaultdict(list)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if frag in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, v in sorted(vals.items()):
        v = v[len(v) // 4:]
        out[k] = sum(v) / len(v)
    print(json.dumps({"kernel": frag, "counters": out}, indent=1))


if __name__ == "__main__":
    main()
