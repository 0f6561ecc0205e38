#!/usr/bin/env python3
"""BASELINE cfg 5 driver: the reference's hold-out evaluations (test.cpp:13-105 and
recommendation_tests.cpp:68-169) over a data directory in the reference's formats, batched on
the GPU and sharded over ranks (one process per GPU).  Each rank evaluates plan entries
i % world == rank; one all-gather collects them; rank 0 averages in plan order (bit-identical to
the sequential drivers) and prints one JSON line with the timings.

    python tools/eval_holdout.py --data DIR [--lines N] [--holdout S] [--rectests S] [--topk K]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/eval_holdout.py ...
    python tools/eval_holdout.py --make-data DIR --users N     (writes a synthetic corpus in reference formats)

--sequential also times the one-user-at-a-time drivers (rank 0) and checks equality.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "recommendation-system-pokec_amd"))
sys.path.insert(0, HERE)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data")
    ap.add_argument("--make-data")
    ap.add_argument("--users", type=int, default=200000)
    ap.add_argument("--lines", type=int, default=0, help="loader line cap (0: every line; the reference caps at 100000)")
    ap.add_argument("--holdout", type=int, default=2000)
    ap.add_argument("--rectests", type=int, default=1000)
    ap.add_argument("--topk", type=int, default=10)
    ap.add_argument("--batch", type=int, default=2048, help="users per device pass (large passes run as pipelined chunks)")
    ap.add_argument("--sequential", action="store_true")
    args = ap.parse_args()
    if args.make_data:
        import synth
        c = synth.Corpus(n_users=args.users, seed=5, edge_cases=0, threads=16)
        os.makedirs(args.make_data, exist_ok=True)
        c.write_reference_files(args.make_data)
        log(f"wrote {args.users} users to {args.make_data}")
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import pokec_fas as pf
    t0 = time.time()
    ds = pf.Dataset(args.data, args.lines if args.lines > 0 else 2**62)
    eng = pf.FasEngine(ds.desc_ptr(), local)
    t_open = time.time() - t0
    info = ds.info()

    def gather(a):
        if world == 1:
            return [a]
        t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        return [p.cpu().numpy() for p in parts]

    if dist:
        dist.barrier()
    t1 = time.time()
    ratios = ds.eval_holdout_friends(eng, args.holdout, rank, world, args.batch)
    ratios = pf.merge_shards(gather(ratios))
    t2 = time.time()
    hits, club = ds.eval_recommendation_tests(eng, args.rectests, args.topk, rank, world, args.batch)
    hits = pf.merge_shards(gather(hits))
    club = pf.merge_shards(gather(club))
    t3 = time.time()
    rec5 = pf.rec_tests_summary(hits, club)
    if dist:
        t = torch.tensor([t2 - t1, t3 - t2], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_hold, t_rec = float(t[0]), float(t[1])
    else:
        t_hold, t_rec = t2 - t1, t3 - t2
    rec = {"workload": "cfg5: hold-out evaluations (test.cpp friends hold-out + recommendation_tests.cpp)",
           "n_profiles": info.n_profiles, "n_gpus": world, "batch": args.batch,
           "holdout_users": int(len(ratios)), "holdout_avg_ratio": float(np.mean(ratios)) if len(ratios) else 0.0,
           "holdout_s": t_hold, "holdout_users_per_s": len(ratios) / t_hold if t_hold > 0 else None,
           "rectests_users": int(len(hits)), "rectests": [float(x) for x in rec5],
           "rectests_s": t_rec, "rectests_users_per_s": len(hits) / t_rec if t_rec > 0 else None,
           "open_s": t_open}
    if args.sequential and rank == 0:
        t4 = time.time()
        seq = ds.holdout_friends(eng, args.holdout)
        t5 = time.time()
        seq5 = ds.recommendation_tests(eng, args.rectests, args.topk)
        t6 = time.time()
        rec["sequential"] = {"holdout_s": t5 - t4, "rectests_s": t6 - t5,
                             "holdout_equal": bool(np.array_equal(seq.view(np.uint64), ratios.view(np.uint64))),
                             "rectests_equal": list(seq5) == list(rec5)}
    if rank == 0:
        print(json.dumps(rec), flush=True)
    eng.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
