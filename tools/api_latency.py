"""B2 serving measurement: request latency of pokec_api_cli (the reference's stdin/JSON
protocol, src/api_cli.cpp:175-252) on a synthetic corpus written in the reference's formats.
Each `USER <uid>` request runs the four recommenders (graph, collaborative, interest, clubs;
topk 20, limit 5000) on the GPU and prints one JSON line.

    python tools/api_latency.py [--users N] [--requests R] [--dir DIR]

Prints one JSON line: start-up time to READY, per-request latency p50/p90/p99/max, requests/s.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1632803)
    ap.add_argument("--requests", type=int, default=300)
    ap.add_argument("--dir", default=None)
    args = ap.parse_args()
    import synth
    exe = os.path.join(ROOT, "recommendation-system-pokec_amd", "pokec_api_cli")
    if not os.path.exists(exe):
        sys.exit("build with make -C recommendation-system-pokec_amd")
    with tempfile.TemporaryDirectory(dir=args.dir) as d:
        c = synth.Corpus(n_users=args.users, seed=5, edge_cases=0, threads=16)
        c.write_reference_files(d)
        c.close()
        t0 = time.perf_counter()
        p = subprocess.Popen([exe, "--no-cap", "--root", d], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, text=True, bufsize=1)
        for line in p.stdout:
            if line.strip() == "READY":
                break
        ready_s = time.perf_counter() - t0
        rng = np.random.default_rng(9)
        uids = rng.integers(1, args.users + 1, args.requests)
        lat, found, nrec = [], 0, 0
        t1 = time.perf_counter()
        for u in uids:
            t = time.perf_counter()
            p.stdin.write(f"USER {int(u)}\n")
            p.stdin.flush()
            out = p.stdout.readline()
            lat.append(time.perf_counter() - t)
            j = json.loads(out)
            if "recommendations" in j:
                found += 1
                nrec += sum(len(v) for v in j["recommendations"].values())
        total = time.perf_counter() - t1
        p.stdin.write("EXIT\n")
        p.stdin.flush()
        p.wait(timeout=60)
    lat = np.array(lat) * 1e3
    print(json.dumps({"what": "pokec_api_cli USER requests (graph + collaborative + interest + clubs, topk 20, "
                              "limit 5000), one at a time over stdin/stdout",
                      "users": args.users, "requests": len(lat), "found": found, "recommendations": nrec,
                      "ready_s": round(ready_s, 2), "requests_per_s": len(lat) / total,
                      "latency_ms": {"p50": float(np.percentile(lat, 50)), "p90": float(np.percentile(lat, 90)),
                                     "p99": float(np.percentile(lat, 99)), "max": float(lat.max()),
                                     "mean": float(lat.mean())}}), flush=True)


if __name__ == "__main__":
    main()
