#!/usr/bin/env python3
"""BASELINE cfg 5 driver: the reference's hold-out evaluations (test.cpp:13-105 and
recommendation_tests.cpp:68-169) over a data directory in the reference's formats, batched on
the GPU and sharded over ranks (one process per GPU).  Each rank evaluates plan entries
i % world == rank; one all-gather collects them; rank 0 averages in plan order (bit-identical to
the sequential drivers) and prints one JSON line with the timings.

    python tools/eval_holdout.py --data DIR [--lines N] [--holdout S] [--rectests S] [--topk K]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/eval_holdout.py ...
    python tools/eval_holdout.py --make-data DIR --users N     (writes a synthetic corpus in reference formats)
    python tools/eval_holdout.py --cfg5-corpus 1632803 --whole --check-prefix 64 --out F.json
        (BASELINE cfg 5 on the whole corpus: bench.py's seed-1 cfg-5 corpus, written if missing, and
         EVERY eligible user of both drivers -- degree >= 20 for test.cpp:20-26, degree >= 4 for
         recommendation_tests.cpp:79-90 -- with the batched drivers' first N users checked against
         the sequential drivers run over N users)

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
    ap.add_argument("--cfg5-corpus", type=int, default=0, help="use bench.py's cfg-5 corpus of this many users")
    ap.add_argument("--whole", action="store_true", help="every eligible user (sample sizes = the profile count)")
    ap.add_argument("--check-prefix", type=int, default=0,
                    help="rank 0: the sequential drivers over this many users against the batched run's prefix")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.cfg5_corpus:
        sys.path.insert(0, ROOT)
        import bench
        import synth
        args.data = bench.cfg5_dir(args.cfg5_corpus)
        marker = os.path.join(args.data, "written")
        if int(os.environ.get("RANK", "0")) == 0 and not os.path.exists(marker):
            c = synth.Corpus(n_users=args.cfg5_corpus, seed=1, edge_cases=0, threads=16)
            c.write_reference_files(args.data)
            del c
            with open(marker, "w") as f:
                f.write("ok\n")
        t = time.time()
        while not os.path.exists(marker):
            if time.time() - t > 900:
                raise RuntimeError("cfg5 corpus files not written")
            time.sleep(1.0)
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
    cache = os.path.join(args.data, f"parse_r{rank}.bin") if args.cfg5_corpus else None
    ds = pf.Dataset(args.data, args.lines if args.lines > 0 else 2**62, cache=cache)
    eng = pf.FasEngine(ds.desc_ptr(), local)
    t_open = time.time() - t0
    info = ds.info()
    if args.whole:
        args.holdout = args.rectests = int(info.n_profiles)

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
    if args.check_prefix and rank == 0:
        P = args.check_prefix
        seq = ds.holdout_friends(eng, P)
        seq5 = ds.recommendation_tests(eng, P, args.topk)
        rec["prefix_check"] = {
            "users": P,
            "holdout_equal": bool(np.array_equal(seq.view(np.uint64), ratios[:len(seq)].view(np.uint64))),
            "rectests_equal": [float(x) for x in seq5] == [float(x) for x in pf.rec_tests_summary(hits[:P], club[:P])]}
    if rank == 0:
        print(json.dumps(rec), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(rec, f, indent=1)
    eng.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
