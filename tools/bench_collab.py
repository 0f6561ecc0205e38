#!/usr/bin/env python3
"""BASELINE cfg 3: collaborative FoF propagation top-10 on the full 1,632,803-user synthetic
corpus, one MI355X (recommend_collaborative, recommender_graph.cpp:105-222).

A step scores a batch of seeded query users through pf_recommend_collab (the batched job
runner: one pair-kernel launch per chunk for every user's sim(u, f) and FAS(f, c) pairs, one
K4 launch for the friend-order sums).  Units: pair-FAS/s (|F| + |F|*|C| per
user) and candidates/s (|C|); the wall clock includes the host's 2-hop gathers and query
images.  CPU baseline: the oracle's recommend_collaborative on a bounded prefix of the corpus.
Prints one JSON line.

    python tools/bench_collab.py [--users N] [--queries Q] [--limit L] [--steps K]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "recommendation-system-pokec_amd"))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def adjacency(desc_ptr):
    import pokec_testlib as tl
    d = tl.PfCorpusDesc.from_address(desc_ptr)
    n = d.n_adj
    uid = np.ctypeslib.as_array(ctypes.cast(d.adj_uid, ctypes.POINTER(ctypes.c_int32)), shape=(n,)).copy()
    off = np.ctypeslib.as_array(ctypes.cast(d.adj_off, ctypes.POINTER(ctypes.c_int64)), shape=(n + 1,)).copy()
    nbr = np.ctypeslib.as_array(ctypes.cast(d.adj_nbr, ctypes.POINTER(ctypes.c_int32)), shape=(int(off[-1]),))
    return {int(u): nbr[off[i]:off[i + 1]] for i, u in enumerate(uid)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1632803)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--limit", type=int, default=10000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import synth
    import pokec_fas as pf
    c = synth.Corpus(n_users=args.users, seed=1, edge_cases=0, threads=16)
    desc = c.desc_ptr()
    eng = pf.FasEngine(desc, 0)
    rng = np.random.default_rng(4)
    q = rng.integers(1, args.users + 1, args.queries).astype(np.int32)
    adj = adjacency(desc)
    pairs = cands = 0
    for u in q:
        f = adj.get(int(u), np.zeros(0, np.int32))
        nf = len(set(int(x) for x in f))
        cand = eng.fof_candidates(int(u), args.limit, pf.PF_FOF_COLLAB)
        nc = int(np.count_nonzero(cand != u))
        pairs += nf + nf * nc
        cands += nc
    eng.recommend_collaborative(q, 10, args.limit)  # warmup
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = eng.recommend_collaborative(q, 10, args.limit)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    rec = {"metric": "collaborative FoF top-10 (cfg 3): pair-FAS/s and candidates/s", "workload":
           f"cfg3: {args.users} users, {args.queries} queries per step, limit {args.limit}",
           "pairs_per_step": pairs, "candidates_per_step": cands, "s_per_step": el,
           "pair_fas_per_s": pairs / el, "candidates_per_s": cands / el, "queries_per_s": args.queries / el,
           "nonempty_results": int(sum(len(x[0]) > 0 for x in out)), "data": "synthetic (tools/pokec_synth.cpp seed 1)"}
    if not args.no_cpu_baseline:
        import pokec_testlib as tl
        sample = 150000
        orc = tl.Oracle(None, max_users=sample, desc_ptr=desc)
        qs = [int(x) for x in rng.integers(1, sample + 1, 4)]
        t = time.perf_counter()
        orc.collab(qs, 10, args.limit)
        cel = time.perf_counter() - t
        # pairs of the oracle's queries on its own (prefix) graph: friends inside the sample
        cp = 0
        for u in qs:
            f = [int(x) for x in adj.get(u, []) if int(x) <= sample]
            cand = set()
            for x in f:
                for y in adj.get(x, []):
                    if int(y) != u and int(y) <= sample:
                        cand.add(int(y))
                        if len(cand) >= args.limit:
                            break
                if len(cand) >= args.limit:
                    break
            cp += len(set(f)) + len(set(f)) * len(cand)
        orc.close()
        rec["cpu_baseline"] = {"pair_fas_per_s": cp / cel if cel > 0 else None, "cores": 1, "kind": "port",
                               "sample": f"{len(qs)} collaborative queries over the first {sample} users "
                                         f"(oracle/refcpu.cpp, single thread, {cel:.2f}s)"}
        rec["speedup_pairs_vs_cpu"] = rec["pair_fas_per_s"] / rec["cpu_baseline"]["pair_fas_per_s"] if cp else None
    print(json.dumps(rec), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
