#!/usr/bin/env python3
"""FAS all-candidates scan benchmark (BASELINE.json metric: "FAS candidates scored/sec
over 1.6M users, top-k=10; 1/2/4/8 GPU + %HBM peak").

Workload (BASELINE.json configs[1]): synthetic Pokec-shaped corpus of
1,632,803 users (seeded generator tools/pokec_synth.cpp, resident in HBM), interest FAS
top-10 over every candidate (A13).  One step = one all-candidates pass for a batch of
queries: at N GPUs the batch holds N distinct query users (1 at N=1, i.e. exactly
config 2), every rank scores its candidate shard (1/N of the corpus, split by stream
bytes) for the whole batch, the per-shard top-10 keys are exchanged with one RCCL
all-gather over xGMI and merged on device.  Per-GPU work is fixed (1.6M pairs/step):
weak scaling.  value = candidates scored / s over the whole job.  With --workload cfg4 a
step is a fixed batch of 1024 queries (SURVEY D1 cfg 4, seed 3) over the sharded candidates:
strong scaling.

Also reports the roofline of the dominant kernel (fas_post_kernel, the postings scan, by
default; fas_scan_kernel, the record-stream scan, with --scan-kernel stream; HIP events
around every launch) with both the algorithmic rate and the measured DRAM share, and the
CPU baseline (oracle/refcpu.cpp, the reference algorithm with its unordered_map data
structures, single thread, bounded sample of the same corpus).

    python bench.py [--gpus N --steps K --warmup W]        (cfg 2, the headline)
    python bench.py --workload cfg4 --steps 5 --warmup 1     (cfg 4: 1024 queries per step)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "recommendation-system-pokec_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

N_USERS = 1632803
TOPK = 10
CFG4_QUERIES = 1024  # cfg 4 = 1024 query uids (seed 3)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "FAS candidates scored/sec over 1.6M users, top-k=10; 1/2/4/8 GPU + %HBM peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(desc_ptr, seconds_budget=12.0):
    """Oracle (reference algorithm, unordered_map per profile/column) on one core over a
    bounded prefix of the same corpus: all-candidates interest top-10 per query."""
    import pokec_testlib as tl
    sample_users = 150000
    t0 = time.time()
    orc = tl.Oracle(None, max_users=sample_users, desc_ptr=desc_ptr)
    build_s = time.time() - t0
    rng = np.random.default_rng(123)
    done, cands, el = 0, 0, 0.0
    while el < seconds_budget and done < 64:
        q = int(rng.integers(1, sample_users + 1))
        t = time.perf_counter()
        orc.interest([q], TOPK, tl.PF_MODE_ALL, 0)
        el += time.perf_counter() - t
        cands += orc.L.ro_num_users(orc.h) - 1
        done += 1
    orc.close()
    return {"value": cands / el, "unit": "candidates/s", "cores": 1, "kind": "port",
            "sample": f"{done} all-candidates interest top-10 queries over the first {sample_users} users of the "
                      f"same synthetic corpus (oracle/refcpu.cpp, single thread, {el:.1f}s timed, "
                      f"{build_s:.1f}s map build untimed)"}


def pmc_traffic(workload, kernel):
    """HBM bytes per scan launch from the committed rocprofv3 PMC pass (profiles/pmc_traffic.json,
    written by tools/profile_round.sh), keyed by workload and kernel."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(f"{workload}:{kernel}")
        return None if e is None else float(e["bytes_per_launch"])
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--users", type=int, default=N_USERS)
    ap.add_argument("--queries-per-gpu", type=int, default=1)
    ap.add_argument("--workload", choices=["cfg2", "cfg4"], default="cfg2",
                    help="cfg2: N queries per step (1 per GPU, weak scaling; the default); "
                         "cfg4: a fixed batch of 1024 queries per step over the sharded candidates (strong scaling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--time-every", type=int, default=1,
                    help="HIP-event timing on every n-th scan launch of the timed region (1 = all)")
    ap.add_argument("--scan-kernel", choices=["auto", "stream", "postings"], default="auto",
                    help="all-candidates scan kernel (auto = postings when the corpus fits its encoding)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import synth
    import pokec_fas as pf

    t0 = time.time()
    corpus = synth.Corpus(n_users=args.users, seed=1, edge_cases=0, threads=16)
    desc = corpus.desc_ptr()
    t1 = time.time()
    eng = pf.FasEngine(desc, local)
    t2 = time.time()
    eng.set_shard(rank, world)
    eng.set_scan_kernel({"auto": pf.PF_SCAN_AUTO, "stream": pf.PF_SCAN_STREAM, "postings": pf.PF_SCAN_POSTINGS}
                        [args.scan_kernel])
    lay = eng.layout()
    kernel_name = "fas_post_kernel" if lay.scan_kernel == pf.PF_SCAN_POSTINGS else "fas_scan_kernel"
    log(f"[rank {rank}] corpus {t1 - t0:.1f}s, engine open {t2 - t1:.1f}s, stream {lay.stream_bytes / 1e9:.3f} GB, "
        f"alg {lay.alg_bytes / 1e9:.3f} GB, packed={lay.packed_tokens}")

    cfg4 = args.workload == "cfg4"
    Q = CFG4_QUERIES if cfg4 else world * args.queries_per_gpu
    k = TOPK
    steps, warm = args.steps, args.warmup
    rng = np.random.default_rng(3 if cfg4 else 2)  # same query stream on every rank (SURVEY D1 seeds)
    qstream = rng.integers(1, args.users + 1, size=(warm + steps, Q)).astype(np.int32)
    # a dedicated stream: the engine, the all-gather and the copies are all ordered on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    local_keys = torch.empty((Q, k), dtype=torch.int64, device="cuda")
    gathered = torch.empty((world, Q, k), dtype=torch.int64, device="cuda") if world > 1 else None
    final = torch.empty((Q, k), dtype=torch.int64, device="cuda")

    def step(i):
        if world == 1:  # the scan's fused merge already yields the final top-k
            eng.scan_keys_async(qstream[i], k, final.data_ptr(), sptr)
            return
        eng.scan_keys_async(qstream[i], k, local_keys.data_ptr(), sptr)
        dist.all_gather_into_tensor(gathered, local_keys)
        eng.merge_keys_async(gathered.data_ptr(), world, Q, k, final.data_ptr(), sptr)

    for i in range(warm):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on every scan launch of the timed region by default.  They cost ~9 us of
    # stream time per single-query step; --time-every 3 times launches 0, 3, 6, ... only
    # (r1p: +2 % candidates/s, but 17 sampled queries averaged 235 us against rocprof's 209 us
    # over all launches, so the default keeps every launch timed)
    eng.profile_sample(args.time_every)
    eng.profile_reset()
    t_start = time.perf_counter()
    for i in range(warm, warm + steps):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    scan_ms, launches = eng.profile_read()
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # sanity: the merged top-k of the last step rescored by the pair kernel
    last = final.cpu().numpy().view(np.uint64)
    uids, scores = pf.decode_keys(last[0])
    chk = eng.fas_pairs(np.full(len(uids), qstream[warm + steps - 1][0], np.int32), uids)
    consistent = bool(len(uids) == k and np.array_equal(chk.view(np.uint32), scores.view(np.uint32)))

    n_cand = eng.num_users - 1  # candidates per query: every profile but the query (minus adj[q])
    value = Q * n_cand * steps / elapsed
    avg_launch_ms = scan_ms / max(launches, 1)
    # algorithmic bytes per launch: SURVEY 8(d) D3 b_c summed over this rank's shard, x queries per launch
    shard_frac = 1.0 / world
    alg_bytes = lay.alg_bytes * shard_frac * Q
    achieved = alg_bytes / (avg_launch_ms * 1e-3) / 1e9
    workload = f"{args.workload}_all_candidates_top{k}_{args.users}users_q{Q}_shard1of{world}"
    if cfg4:
        wl_name = (f"cfg4: {Q}-query batch, interest FAS all-candidates top-10 over the full 1.6M-user corpus, "
                   f"candidates sharded over {world} GPU(s)" + ("" if world == 1 else ", RCCL all-gather of per-shard top-10"))
    else:
        wl_name = ("cfg2: full 1.6M-user single-query interest FAS all-candidates top-10"
                   + ("" if world == 1 else f"; {Q} queries/step, candidates sharded over {world} GPUs, "
                                            "RCCL all-gather of per-shard top-10"))
    traffic = pmc_traffic(workload, kernel_name)
    rec = {
        "metric": METRIC,
        "value": value,
        "unit": "candidates/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warm,
        "ms_per_step": elapsed * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "strong" if cfg4 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded Pokec-shaped corpus, tools/pokec_synth.cpp; no Pokec data offline)",
        "config": {"workload": wl_name,
                   "workload_key": workload, "n_users": args.users, "queries_per_step": Q, "topk": k,
                   "parallelism": f"candidate-shard x{world}" + (" + all_gather" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kernel_name, "avg_launch_ms": avg_launch_ms,
                     "timed_launches": launches, "timed_every": args.time_every,
                     "alg_bytes_per_launch": alg_bytes,
                     # what the kernel really moves: PMC FETCH_SIZE bytes over the same launch time
                     "dram_gbs": None if traffic is None else traffic / (avg_launch_ms * 1e-3) / 1e9,
                     "dram_frac": None if traffic is None else traffic / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "note": ("postings scan: reads only the query's candidate lists (~0.2 GB), so the "
                              "algorithmic rate of a full record pass exceeds the HBM peak; dram_frac is the "
                              "measured HBM share" if kernel_name == "fas_post_kernel" else
                              "record-stream scan: one pass over every candidate's record"),
                     "stream_bytes_per_launch": (lay.stream_bytes + lay.header_bytes) * shard_frac * Q},
        "topk_selfcheck": consistent,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(desc)
        rec["cpu_baseline"] = base
        rec["speedup_vs_cpu"] = value / base["value"]
    elif rank == 0:
        rec["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(rec), flush=True)
    eng.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
