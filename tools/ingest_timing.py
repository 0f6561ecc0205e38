"""F2 measurement: time pf_dataset_load (users_encoded.csv + adjacency.csv at corpus scale)
with 1 thread and with the default thread count, on a synthetic corpus written in the
reference's formats (tools/synth.py; no Pokec data offline).  Host only, no GPU.

    python tools/ingest_timing.py [--users N] [--dir DIR] [--single]

Prints one JSON line; PF_DEBUG=host_prof=1 adds the loader's stage clocks on stderr.
"""
import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "recommendation-system-pokec_amd"))
sys.path.insert(0, HERE)


def timed_load(pf, root, threads):
    old = os.environ.get("PF_DEBUG")
    if threads:
        os.environ["PF_DEBUG"] = f"load_threads={threads}"
    else:
        os.environ.pop("PF_DEBUG", None)
    try:
        t = time.perf_counter()
        ds = pf.Dataset(root, -1)
        dt = time.perf_counter() - t
        n = ds.info().n_profiles
        ds.close()
    finally:
        if old is None:
            os.environ.pop("PF_DEBUG", None)
        else:
            os.environ["PF_DEBUG"] = old
    return dt, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1632803)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--single", action="store_true", help="also time one thread")
    args = ap.parse_args()
    import pokec_fas as pf
    import synth
    with tempfile.TemporaryDirectory(dir=args.dir) as d:
        t = time.perf_counter()
        c = synth.Corpus(n_users=args.users, seed=5, edge_cases=0, threads=16)
        c.write_reference_files(d)
        c.close()
        gen = time.perf_counter() - t
        size = sum(os.path.getsize(os.path.join(d, "data", f)) for f in os.listdir(os.path.join(d, "data")))
        dt, n = timed_load(pf, d, 0)
        out = {"what": "pf_dataset_load users_encoded.csv + adjacency.csv", "users": n, "csv_bytes": size,
               "threads": min(16, os.cpu_count() or 1), "load_s": round(dt, 3), "write_s": round(gen, 1)}
        if args.single:
            dt1, _ = timed_load(pf, d, 1)
            out["load_s_1thread"] = round(dt1, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
