#!/usr/bin/env python3
"""FAS all-candidates scan benchmark (BASELINE.json metric: "FAS candidates scored/sec
over 1.6M users, top-k=10; 1/2/4/8 GPU + %HBM peak").

Workload: synthetic Pokec-shaped corpus of 1,632,803 users (seeded
generator tools/pokec_synth.cpp, resident in HBM), interest FAS top-10 over every candidate
(A13).  Default by N:
  N = 1  cfg 2 (BASELINE.json configs[1], the metric's configuration): one query per step,
         every candidate scored.
  N > 1  cfg 4 (configs[3]): a fixed batch of 1024 queries per step (seed 3), candidates
         sharded over the N ranks by posting weight, each rank's per-shard top-10 keys
         exchanged with one RCCL all-gather over xGMI and merged on device.  Total work is
         fixed: strong scaling (the north-star ">= 6x at 8 GPUs" is defined on cfg 4).
--workload cfg2|cfg4 overrides the default (cfg2 at N > 1: N queries per step, one per GPU,
weak scaling).  value = candidates scored / s over the whole job.
--workload cfg3 (configs[2]): collaborative FoF top-10, 64 query users per step; value = pair-FAS/s;
one engine context, three asynchronous calls in flight (--contexts C: C contexts per GPU, steps
dealt round-robin to their host threads).
--workload cfg5 (configs[4]): the hold-out evaluation (recommendation_tests.cpp: interest + collab
+ clubs) of 2048 users per step, users split over the ranks, one engine context per GPU by
default; value = hold-out users/s.

Roofline of the dominant kernel (fas_post_kernel, the postings scan, by default;
fas_scan_kernel, the record-stream scan, with --scan-kernel stream), HIP events around every
launch on the kernel's stream:
  achieved  = the bytes the kernel reads by its access pattern (pf_scan_bytes: headers, cell
              words, the list entries of the query's lists, their norms)
              summed over the timed queries / the summed launch time;
  traffic   = HBM bytes per launch measured in this run by a rocprofv3 --pmc FETCH_SIZE pass
              of the same command (a child process started before this one touches the GPU;
              FETCH_SIZE KiB x 1024 x the gfx950 factor calibrated for the kernel's load widths,
              profiles/fetch_calib_*.json), null when rocprofv3 is absent or --no-pmc;
  d3_equiv_* = SURVEY D3's per-candidate record bytes (b_c, the metric's definition)
              over the same time: an *equivalent* rate, NOT an HBM fraction (the postings scan
              never reads those records, so d3_equiv_x_peak can exceed 1); roofline.frac is the
              kernel's HBM fraction.
CPU baseline: oracle/refcpu.cpp (the reference algorithm with its unordered_map data
structures), one core, bounded sample of the same corpus, median per query; plus an
all-cores context figure (one oracle per core).

    python bench.py [--gpus N --steps K --warmup W]
    python bench.py --workload cfg4 --steps 5 --warmup 1     (cfg 4 at N = 1)
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


SAMPLE_USERS = 150000


_DESC = None  # the parent's corpus descriptor, inherited by the forked oracle workers


def _oracle_worker(args):
    """One core's share of the all-cores context figure: queries for `seconds` on its own oracle
    (forked before any GPU use, so it shares the parent's corpus arrays copy-on-write)."""
    seed, seconds = args
    import pokec_testlib as tl
    orc = tl.Oracle(None, max_users=SAMPLE_USERS, desc_ptr=_DESC)
    rng = np.random.default_rng(seed)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        orc.interest([int(rng.integers(1, SAMPLE_USERS + 1))], TOPK, tl.PF_MODE_ALL, 0)
        done += 1
    el = time.perf_counter() - t0
    cands = (orc.L.ro_num_users(orc.h) - 1) * done
    orc.close()
    return cands, el


def _pinned_oracle_child(conn, desc_ptr, core, cfg2_queries, cfg3_users, cfg3_budget):
    """Forked child (no GPU): pinned to `core`, the oracle (the reference algorithm with its
    unordered_map data structures, oracle/refcpu.cpp -O3) on the FULL corpus: per-query times of
    all-candidates interest top-10 (cfg 2) and recommend_collaborative(u, 10, 10000) (cfg 3),
    then the former 150k-prefix figure; results through the pipe."""
    try:
        os.sched_setaffinity(0, {core})
        import pokec_testlib as tl
        out = {}
        t0 = time.time()
        orc = tl.Oracle(None, desc_ptr=desc_ptr)
        out["build_s"] = time.time() - t0
        out["n_users"] = int(orc.L.ro_num_users(orc.h))
        per = []
        for q in cfg2_queries:
            t = time.perf_counter()
            orc.interest([int(q)], TOPK, tl.PF_MODE_ALL, 0)
            per.append(time.perf_counter() - t)
        out["cfg2_query_s"] = per
        if cfg3_users is not None:
            calls, el, n = 0, 0.0, 0
            for q in cfg3_users:
                if n >= 16 and el >= cfg3_budget:
                    break
                orc.fas_calls(True)
                t = time.perf_counter()
                orc.collab([int(q)], TOPK, CFG3_LIMIT)
                dt = time.perf_counter() - t
                c = orc.fas_calls(True)
                if c == 0:
                    continue
                calls, el, n = calls + c, el + dt, n + 1
            out["cfg3"] = {"fas_calls": calls, "seconds": el, "queries": n}
        orc.close()
        # the former figure, kept for comparison: the median query over a 150k-user prefix
        orc = tl.Oracle(None, max_users=SAMPLE_USERS, desc_ptr=desc_ptr)
        npre = int(orc.L.ro_num_users(orc.h))
        rng = np.random.default_rng(123)
        per, el = [], 0.0
        while el < 6.0 and len(per) < 64:
            q = int(rng.integers(1, npre + 1))
            t = time.perf_counter()
            orc.interest([q], TOPK, tl.PF_MODE_ALL, 0)
            dt = time.perf_counter() - t
            per.append(dt)
            el += dt
        out["prefix_query_s"] = per
        out["prefix_n_users"] = npre
        orc.close()
        conn.send(out)
    except Exception as e:  # reported, never fatal to the bench
        conn.send({"error": repr(e)[:300]})
    finally:
        conn.close()


def cpu_baselines(desc_ptr, n_users, cfg3_users=None, cfg3_budget=10.0, all_cores_seconds=6.0):
    """the oracle timed on this box's host, one core pinned (os.sched_setaffinity in a
    forked child, before this process touches the GPU), on the FULL corpus the GPU line scores:
    cfg 2 = the median of 3 all-candidates interest top-10 queries (candidates / s); cfg 3 (when
    cfg3_users is given) = pair-FAS/s over >= 16 recommend_collaborative(u, 10, 10000) queries and
    about cfg3_budget seconds.  The former 150k-user-prefix median and an all-cores context figure
    (one oracle process per core on that prefix) ride along as second fields."""
    import multiprocessing as mp
    core = min(os.sched_getaffinity(0))
    rng = np.random.default_rng(123)
    q2 = [int(x) for x in rng.integers(1, n_users + 1, 3)]
    ctx = mp.get_context("fork")
    a, b = ctx.Pipe(duplex=False)
    p = ctx.Process(target=_pinned_oracle_child, args=(b, desc_ptr, core, q2, cfg3_users, cfg3_budget))
    t0 = time.time()
    p.start()
    b.close()
    res = a.recv()
    p.join()
    wall = time.time() - t0
    if "error" in res:
        return {"value": None, "error": res["error"]}, None
    n_cand = res["n_users"] - 1
    med = float(np.median(res["cfg2_query_s"]))
    pre = res["prefix_query_s"]
    pmed = float(np.median(pre))
    base2 = {"value": n_cand / med, "unit": "candidates/s", "cores": 1, "kind": "port", "pinned_core": core,
             "cpu_model": cpu_model(), "median_query_s": med, "query_s": res["cfg2_query_s"], "queries": len(q2),
             "sample": f"{len(q2)} all-candidates interest top-10 queries (seed 123) over the full {res['n_users']}-user "
                       f"corpus the GPU line scores (oracle/refcpu.cpp -O3, one thread pinned to core {core}, median of "
                       f"the per-query times; {res['build_s']:.1f}s map build untimed, {wall:.0f}s wall)",
             "prefix": {"value": (res["prefix_n_users"] - 1) / pmed, "median_query_s": pmed, "queries": len(pre),
                        "n_users": res["prefix_n_users"],
                        "note": "the round-2 figure: the same oracle on the first 150,000 users only"}}
    global _DESC
    _DESC = desc_ptr
    try:
        ncores = min(16, len(os.sched_getaffinity(0)))
        with ctx.Pool(ncores) as pool:
            r = pool.map(_oracle_worker, [(1000 + i, all_cores_seconds) for i in range(ncores)])
        base2["all_cores"] = {"value": sum(c for c, _ in r) / max(e for _, e in r), "cores": ncores,
                              "note": "one oracle process per core, each on the 150k-user prefix; context only"}
    except Exception as e:  # context figure only
        base2["all_cores"] = {"value": None, "error": str(e)[:200]}
    base3 = None
    if cfg3_users is not None and res.get("cfg3", {}).get("seconds"):
        c3 = res["cfg3"]
        base3 = {"value": c3["fas_calls"] / c3["seconds"], "unit": "pair-FAS/s", "cores": 1, "kind": "port",
                 "pinned_core": core, "cpu_model": cpu_model(), "queries": c3["queries"], "fas_calls": c3["fas_calls"],
                 "sample": f"{c3['queries']} recommend_collaborative(u, 10, {CFG3_LIMIT}) queries (the GPU line's first "
                           f"query users) over the full {res['n_users']}-user corpus (oracle/refcpu.cpp -O3, one thread "
                           f"pinned to core {core}; profile_similarity calls counted by the oracle, "
                           f"{c3['seconds']:.1f}s timed)"}
    return base2, base3


def pmc_pass(args, select):
    """HBM bytes per timed launch of each kernel in `select` (name -> a function picking the timed
    launches from that kernel's FETCH_SIZE values in dispatch order) from one rocprofv3 --pmc
    FETCH_SIZE pass of this same command, run as a child before this process touches the GPU.
    FETCH_SIZE (KiB) x 1024 x the gfx950 factor (profiles/fetch_calib_r2.json: the factor measured
    on known byte counts of the kernel's load widths; MI355X_MICROARCH.md HBM section).
    Returns {name: (info or None, error or None)}."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return {k: (None, "rocprofv3 not found") for k in select}
    # one calibration for every kernel (profiles/fetch_calib_r2.json, tools/fetch_calib.hip): the
    # postings scans' 4/8-B gathers take its k5_factor, the record-stream kernels (K1, K1': 16-B
    # steps) its w16_stream factor; 2.0 (MI355X_MICROARCH.md) only when the file is absent
    factors = {}
    cal = os.path.join(ROOT, "profiles", "fetch_calib_r2.json")
    calib = None
    if os.path.exists(cal):
        try:
            with open(cal) as f:
                calib = json.load(f)
        except Exception:
            calib = None
    for k in select:
        factor, fsrc = 2.0, "MI355X_MICROARCH.md (16-B/lane streams)"
        if calib is not None:
            if k in ("fas_post_kernel", "fas_slice_kernel"):
                factor, fsrc = float(calib["k5_factor"]), "profiles/fetch_calib_r2.json k5_factor"
            else:
                factor, fsrc = float(calib["w16_stream"]["factor"]), "profiles/fetch_calib_r2.json w16_stream"
        factors[k] = (factor, fsrc)
    d = tempfile.mkdtemp(prefix="pf_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [prof, "--pmc", "FETCH_SIZE", "--kernel-include-regex", "|".join(select), "-T", "--output-format", "csv",
           "-d", d, "-o", "run", "--", sys.executable, os.path.abspath(__file__), "--gpus", "1",
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--no-cpu-baseline", "--no-pmc",
           "--workload", args.workload, "--scan-kernel", args.scan_kernel, "--users", str(args.users),
           "--contexts", str(args.contexts), "--cfg5-batch", str(args.cfg5_batch),
           "--cfg3-steps", str(args.cfg3_steps)]
    if args.no_cfg3:
        cmd.append("--no-cfg3")
    if args.sync_calls:
        cmd.append("--sync-calls")
    if args.eval_sync:
        cmd.append("--eval-sync")
    try:
        r = subprocess.run(["timeout", "-s", "KILL", "240"] + cmd, capture_output=True, text=True,
                           env={**os.environ, "TMPDIR": os.environ.get("TMPDIR", "/tmp")})
        if r.returncode != 0:
            return {k: (None, f"rocprofv3 pass rc={r.returncode}: {r.stderr[-300:]}") for k in select}
        vals = {k: [] for k in select}
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for row in csv.DictReader(f):
                    if row.get("Counter_Name") != "FETCH_SIZE":
                        continue
                    for k in select:
                        if k in row.get("Kernel_Name", ""):
                            vals[k].append((int(row.get("Dispatch_Id", len(vals[k]))), float(row["Counter_Value"])))
        out = {}
        for k, pick in select.items():
            v = pick([x for _, x in sorted(vals[k])])
            if not v:
                out[k] = (None, "no FETCH_SIZE rows")
                continue
            mean = sum(v) / len(v)
            factor, fsrc = factors[k]
            # _raw: the picked per-dispatch values, for callers that group dispatches into stages
            # (pair_stage_traffic); never printed
            out[k] = ({"bytes_per_launch": mean * 1024 * factor, "fetch_size_kib_mean": mean, "launches": len(v),
                       "factor": factor, "factor_source": fsrc, "_raw": list(v)}, None)
        return out
    except Exception as e:
        return {k: (None, str(e)[:300]) for k in select}
    finally:
        shutil.rmtree(d, ignore_errors=True)


class Comm:
    """The collectives bench.py uses, named like torch.distributed's: RCCL ("nccl", one rank
    per GPU, device tensors) or gloo through host memory (--dist-backend gloo: N ranks may share
    one GPU, a correctness rehearsal of the N > 1 path on a one-GPU box; its timings are not
    scaling numbers)."""

    def __init__(self, backend, local):
        import torch
        import torch.distributed as dist
        self.dist, self.torch, self.gloo = dist, torch, backend == "gloo"
        self.ReduceOp = dist.ReduceOp
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if self.gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier(self):
        self.dist.barrier()

    def all_reduce(self, t, op):
        if self.gloo:
            h = t.cpu()
            self.dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            self.dist.all_reduce(t, op=op)

    def all_gather(self, parts, t):
        if self.gloo:
            hp = [self.torch.empty_like(t, device="cpu") for _ in parts]
            self.dist.all_gather(hp, t.cpu())
            for d, h in zip(parts, hp):
                d.copy_(h)
        else:
            self.dist.all_gather(parts, t)

    def all_gather_into_tensor(self, out, t):
        if self.gloo:
            self.all_gather(list(out.unbind(0)), t)
        else:
            self.dist.all_gather_into_tensor(out, t)

    def destroy_process_group(self):
        self.dist.destroy_process_group()


CFG3_QUERIES = 64      # cfg 3 step: a batch of seeded query users
CFG3_LIMIT = 10000     # recommend_collaborative's default candidate_limit (include/recommender.h)


def cfg3_queries(users, warm, steps, rank=0, world=1):
    """cfg 3's query users: per step a batch of CFG3_QUERIES seeded uids (seed 4), this rank's
    share of each at N > 1."""
    rng = np.random.default_rng(4)
    qstream = rng.integers(1, users + 1, size=(warm + steps, CFG3_QUERIES)).astype(np.int32)
    return [qs[rank::world] for qs in qstream]


ASYNC_DEPTH = 3  # asynchronous calls kept in flight (the engine's workspace slots, pf_ctx.h kJobSlots)


def measure_cfg3(engs, mine, warm, steps, dist=None, torch=None, use_async=True, depth=ASYNC_DEPTH):
    """cfg 3 (BASELINE configs[2]): collaborative FoF propagation top-10 on the full corpus.  A
    step = recommend_collaborative(u, 10, 10000) for a batch of 64 seeded users (this rank's share
    at N > 1), through the device job pipeline (K3 gather, K6 images, K1' pairs, K4' sums, K8
    top-k) and back to the host.  Returns the timing and counters: pair-FAS scored (SURVEY D3's
    cfg-3 unit, |F| + |F|.|C| per user) and the pair kernel's HIP-event time per launch (its
    roofline).  One context: the steps go through the asynchronous calls (pf_recommend_collab_async,
    three in flight), so steps i + 1 and i + 2 are planned on the host while step i runs on the device
    (use_async=False: the synchronous calls).  With C = len(engs) > 1 contexts, step i runs on
    context i % C from its own host thread (ctypes releases the GIL)."""
    eng = engs[0]
    C = len(engs)
    for i in range(warm):
        engs[i % C].recommend_collaborative(mine[i], TOPK, CFG3_LIMIT)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    # timed region: the pair kernel timed by HIP events (the launch roofline); the pair and byte
    # counts come from an untimed replay of the same steps (the counting kernel stays out of it)
    disp0 = sum(e.jobs_stats()["pair_dispatches"] for e in engs)  # K1' dispatches before the timed steps
    for e in engs:
        e.jobs_stats_reset(time_pairs=True, count=False)

    def run_steps(t):  # context t: steps warm + t, warm + t + C, ...
        n = 0
        e = engs[t]
        if use_async:
            pend = []
            for i in range(warm + t, warm + steps, C):
                pend.append(e.recommend_collaborative_async(mine[i], TOPK, CFG3_LIMIT))
                if len(pend) == depth:
                    n += sum(len(o[0]) for o in e.wait(pend.pop(0)))
            for p in pend:
                n += sum(len(o[0]) for o in e.wait(p))
            return n
        for i in range(warm + t, warm + steps, C):
            out = e.recommend_collaborative(mine[i], TOPK, CFG3_LIMIT)
            n += sum(len(o[0]) for o in out)
        return n

    t0 = time.perf_counter()
    if C == 1:
        nres = run_steps(0)
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(C) as ex:
            nres = sum(ex.map(run_steps, range(C)))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timing = {"pair_ms": 0.0, "pair_launches": 0, "disp1": 0}
    for e in engs:
        tm_ = e.jobs_stats()
        timing["pair_ms"] += tm_["pair_ms"]
        timing["pair_launches"] += tm_["pair_launches"]
        timing["disp1"] += tm_["pair_dispatches"]
        if e is not eng:
            e.jobs_stats_reset(time_pairs=False, count=False)
    eng.jobs_stats_reset(time_pairs=False, count=True)
    for i in range(warm, warm + steps):
        eng.recommend_collaborative(mine[i], TOPK, CFG3_LIMIT)
    st = eng.jobs_stats()
    eng.jobs_stats_reset(time_pairs=False, count=False)
    st["pair_ms"], st["pair_launches"] = timing["pair_ms"], timing["pair_launches"]
    st["disp0"], st["disp1"] = disp0, timing["disp1"]
    st["elapsed"], st["results"], st["async"] = elapsed, nres, use_async
    if dist:
        t = torch.tensor([st["pairs"], st["candidates"]], dtype=torch.float64, device="cuda")
        tm = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        st["pairs"], st["candidates"], st["elapsed"] = float(t[0]), float(t[1]), float(tm.item())
    return st


def pair_stage_traffic(pmc, st):
    """HBM bytes per pair STAGE of the timed region from the PMC child's per-dispatch FETCH_SIZE rows
    of fas_pairs_kernel (every dispatch, in order): a pair stage launches up to four K1' dispatches
    (one per image LDS class, plus the pre-walked pairs), so the rows are grouped by the engines'
    own dispatch counters (pf_jobs_stats.pair_dispatches before / after the timed region; the child
    runs the same deterministic command, so its dispatch sequence is the same).  Returns (bytes per
    stage or None, traffic_source)."""
    if not pmc or not pmc[0]:
        return None, (pmc[1] if pmc else "not run")
    info = {k: v for k, v in pmc[0].items() if k != "_raw"}
    raw, d0, d1, stages = pmc[0].get("_raw", []), st.get("disp0"), st.get("disp1"), st.get("pair_launches")
    if d0 is None or d1 is None or not stages or d1 > len(raw) or d1 <= d0:
        return None, {**info, "error": f"dispatch counts {d0}..{d1} do not fit the {len(raw)} PMC rows"}
    kib = sum(raw[d0:d1])
    per_stage = kib * 1024 * info["factor"] / stages
    info.update({"bytes_per_launch": per_stage, "unit_of_launch": "pair stage (all its K1' dispatches)",
                 "dispatches": d1 - d0, "stages": stages, "dispatch_range": [d0, d1],
                 "fetch_size_kib_per_stage": kib / stages})
    info.pop("fetch_size_kib_mean", None)
    info.pop("launches", None)
    return per_stage, info


def cfg3_fields(st, steps, pmc):
    """value + roofline fields of a cfg-3 measurement (measure_cfg3)."""
    elapsed = st["elapsed"]
    ms, launches = st["pair_ms"], st["pair_launches"]
    avg_ms = ms / launches if launches else None
    phys = (st["pair_record_bytes"] + st["pair_image_bytes"]) / launches if launches else None

    def rate(b):
        return None if (b is None or not avg_ms) else b / (avg_ms * 1e-3) / 1e9

    achieved = rate(phys)
    alg_pl = st["pair_alg_bytes"] / launches if launches else None
    traffic, tsrc = pair_stage_traffic(pmc, st)
    return {
        "value": st["pairs"] / elapsed, "unit": "pair-FAS/s", "ms_per_step": elapsed * 1e3 / steps,
        "candidates_per_s": st["candidates"] / elapsed, "queries_per_s": CFG3_QUERIES * steps / elapsed,
        "pairs_per_step": st["pairs"] / steps, "candidates_per_step": st["candidates"] / steps,
        "results": st["results"],
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": None if achieved is None else achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "fas_pairs_kernel", "avg_launch_ms": avg_ms, "timed_launches": launches,
                     "bytes_per_launch": phys,
                     "bytes_model": "pf_jobs_stats: per scored pair the candidate's 48-B tile-store headers + record "
                                    "words (K1' walks the record), per pair block the staged query image",
                     "dram_gbs": rate(traffic),
                     "dram_frac": None if traffic is None or not avg_ms else rate(traffic) / HBM_PEAK_GBS,
                     "traffic_source": tsrc,
                     "d3_equiv_gbs": rate(alg_pl),
                     "d3_equiv_x_peak": None if rate(alg_pl) is None else rate(alg_pl) / HBM_PEAK_GBS,
                     "alg_bytes_per_launch": alg_pl,
                     "pair_kernel_share_of_step": (ms / (elapsed * 1e3)) if elapsed > 0 else None},
    }


def run_cfg3(args, engs, pf, torch, dist, world, rank, base, pmc, open_s):
    """--workload cfg3: the cfg-3 measurement as the bench line (query users split over the ranks:
    strong scaling); value = FAS pairs scored / s."""
    steps, warm = args.steps, args.warmup
    mine = cfg3_queries(args.users, warm, steps, rank, world)
    st = measure_cfg3(engs, mine, warm, steps, dist, torch, use_async=not args.sync_calls, depth=args.async_depth)
    C = len(engs)
    f = cfg3_fields(st, steps, pmc)
    rec = {
        "metric": METRIC, "value": f.pop("value"), "unit": f.pop("unit"), "n_gpus": world, "steps": steps,
        "warmup": warm, "ms_per_step": f.pop("ms_per_step"), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded Pokec-shaped corpus, tools/pokec_synth.cpp; no Pokec data offline)",
        "config": {"workload": f"cfg3: collaborative FoF top-10 on the full {args.users}-user corpus, {CFG3_QUERIES} "
                               f"query users per step (limit {CFG3_LIMIT})" + (f", split over {world} GPUs" if world > 1 else ""),
                   "workload_key": f"cfg3_collab_top{TOPK}_{args.users}users_q{CFG3_QUERIES}_limit{CFG3_LIMIT}_world{world}",
                   "n_users": args.users, "queries_per_step": CFG3_QUERIES, "topk": TOPK, "limit": CFG3_LIMIT,
                   "parallelism": f"query-users x{world}" + (f", {C} engine contexts per GPU" if C > 1 else "")
                                  + (f", asynchronous calls ({args.async_depth} in flight)" if st["async"] else "")},
        **f, "open_s": open_s,
    }
    if rank == 0 and world == 1 and base is not None:
        rec["cpu_baseline"] = base
        rec["speedup_vs_cpu"] = rec["value"] / base["value"] if base.get("value") else None
    elif rank == 0:
        rec["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(rec), flush=True)
    for e in engs:
        e.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


CFG5_USERS = 2048      # cfg 5 step: one recommendation_tests evaluation of this many sampled users
CFG5_TOPK = 10


def cfg5_dir(users):
    """The cfg-5 corpus in the reference's on-disk formats (data/, config/; Appendix A), written
    once per box by rank 0 (the synthetic generator, seed 1) and parsed by every rank."""
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"pf_cfg5_{users}u_seed1")


def _pinned_call(fn, *a):
    """fn(*a) in a forked child pinned to one core (the CPU baseline single-threaded and
    pinned), before this process touches the GPU; returns (result, core)."""
    import multiprocessing as mp
    core = min(os.sched_getaffinity(0))
    ctx = mp.get_context("fork")
    rd, wr = ctx.Pipe(duplex=False)

    def child():
        try:
            os.sched_setaffinity(0, {core})
            wr.send(fn(*a))
        except Exception as e:
            wr.send({"value": None, "error": repr(e)[:300]})
        finally:
            wr.close()
    p = ctx.Process(target=child)
    p.start()
    wr.close()
    res = rd.recv()
    p.join()
    return res, core


def cpu_baseline_cfg5(ds_dir, users_timed=101):
    """Oracle run_recommendation_tests_sample (the reference algorithm and its O(N) adj_mod copy
    per user, recommendation_tests.cpp:68-169) on the SAME full corpus, one core: users/s =
    (S - 1) extra users / (t(S) - t(1)), the marginal per-user rate without the per-call sampling
    plan (which favours the CPU: the GPU step pays its plan), plus the whole-call rate."""
    res, core = _pinned_call(_cpu_baseline_cfg5, ds_dir, users_timed)
    if res.get("value") is not None:
        res["pinned_core"] = core
        res["sample"] += f"; pinned to core {core}"
    return res


def _cpu_baseline_cfg5(ds_dir, users_timed):
    import pokec_fas as pf
    import pokec_testlib as tl
    t0 = time.time()
    ds = pf.Dataset(ds_dir, 0, cache=os.path.join(ds_dir, "parse_r0.bin"))
    orc = tl.Oracle(None, desc_ptr=ds.desc_ptr())
    build_s = time.time() - t0
    t = time.perf_counter()
    orc.recommendation_tests(1, CFG5_TOPK)
    t1 = time.perf_counter() - t
    orc.fas_calls(True)
    t = time.perf_counter()
    orc.recommendation_tests(users_timed, CFG5_TOPK)
    tn = time.perf_counter() - t
    calls = orc.fas_calls(True)
    orc.close()
    ds.close()
    marg = (users_timed - 1) / (tn - t1) if tn > t1 else None
    return {"value": marg, "unit": "hold-out users/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
            "whole_call_users_per_s": users_timed / tn, "pair_fas_per_s": calls / tn, "fas_calls": calls,
            "sample": f"run_recommendation_tests_sample over {users_timed} users (graph, collaborative, interest, "
                      f"clubs at limit 5000, top-{CFG5_TOPK}) on the same full corpus, oracle/refcpu.cpp -O3, one "
                      f"core; value = {users_timed - 1} users / (t({users_timed}) - t(1)) = "
                      f"{users_timed - 1} / ({tn:.2f} - {t1:.2f}) s; {build_s:.1f}s load + map build untimed"}


def run_cfg5(args, world, rank, local):
    """cfg 5 (BASELINE configs[4]): the full pipeline's hold-out evaluation on the whole corpus.
    A step = run_recommendation_tests_sample over CFG5_USERS sampled users (recommendation_tests.cpp:
    68-169: graph = interest FoF, collaborative and clubs at limit 5000, top-10 each, the user's
    own friend row edited), batched through the device job pipeline (K3 gathers, K6 images, K1'
    pairs, K4' sums, K7 clubs, K8 top-k), plan entries split over the ranks (i % world == rank;
    strong scaling), the per-user hits all-gathered and averaged in plan order on rank 0 (the
    sequential driver's bits).  value = users evaluated / s."""
    import synth
    d = cfg5_dir(args.users)
    marker = os.path.join(d, "written")
    t0 = time.time()
    if rank == 0 and not os.path.exists(marker):
        c = synth.Corpus(n_users=args.users, seed=1, edge_cases=0, threads=16)
        c.write_reference_files(d)
        del c
        with open(marker, "w") as f:
            f.write("ok\n")
    while not os.path.exists(marker):  # the other ranks wait for rank 0's files
        if time.time() - t0 > 900:
            raise RuntimeError("cfg5 corpus files not written")
        time.sleep(1.0)
    write_s = time.time() - t0
    log(f"[rank {rank}] cfg5 corpus files ready after {write_s:.1f}s")
    base, pmc, pmc_err = None, None, "not run (N > 1 or --no-pmc)"
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            base = cpu_baseline_cfg5(d)
            log(f"cpu baseline: {base['value']} users/s ({base['sample']})")
        if not args.no_pmc:  # every pair launch (several per step, warmup steps of the same kind)
            pmc, pmc_err = pmc_pass(args, {"fas_pairs_kernel": lambda v: v})["fas_pairs_kernel"]
            if pmc_err:
                log(f"pmc pass: {pmc_err}")
    import torch
    local = local % max(1, torch.cuda.device_count())  # --dist-backend gloo: ranks may share a GPU
    torch.cuda.set_device(local)
    dist = Comm(args.dist_backend, local) if world > 1 else None
    import pokec_fas as pf
    t1 = time.time()
    ds = pf.Dataset(d, 0, cache=os.path.join(d, f"parse_r{rank}.bin"))
    C = max(1, args.contexts)  # engine contexts on this GPU, one host thread each
    engs = [pf.FasEngine(ds.desc_ptr(), local) for _ in range(C)]
    eng = engs[0]
    open_s = time.time() - t1
    log(f"[rank {rank}] dataset + {C} engine context(s) open {open_s:.1f}s")
    S, steps, warm = CFG5_USERS, args.steps, args.warmup
    nsh = world * C  # plan shards: entry i belongs to shard i % nsh = rank * C + context
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(C) if C > 1 else None

    def sum_stats(fn):
        tot = {}
        for e in engs:
            for key, v in fn(e).items():
                tot[key] = tot.get(key, 0) + v
        return tot

    def gather(a):
        if world == 1:
            return [a]
        t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        return [p.cpu().numpy() for p in parts]

    def summarize(parts):
        hs = gather(np.stack([h for h, _ in parts]))  # per rank [C, entries, 3]
        cs = gather(np.stack([c for _, c in parts]))
        hits = pf.merge_shards([h[t] for h in hs for t in range(C)])  # shard order rank * C + t
        club = pf.merge_shards([c[t] for c in cs for t in range(C)])
        return pf.rec_tests_summary(hits, club), len(hits)

    def step():
        def part(t):
            return ds.eval_recommendation_tests(engs[t], S, CFG5_TOPK, rank * C + t, nsh, args.cfg5_batch)
        return summarize([part(0)] if pool is None else list(pool.map(part, range(C))))

    # one context: the asynchronous driver call (pf_eval_recommendation_tests_async) leaves each
    # step's last chunk on the device; the next step plans and launches its first chunk before that
    # chunk is unpacked, so the host's planning hides behind the device (--eval-sync: the old form)
    use_async = C == 1 and not args.eval_sync

    def steps_async(n):
        prev, out = None, None
        for _ in range(n):
            cur = ds.eval_recommendation_tests_async(eng, S, CFG5_TOPK, rank, nsh, args.cfg5_batch)
            if prev is not None:
                out = summarize([ds.eval_wait(eng, prev)])
            prev = cur
        if prev is not None:
            out = summarize([ds.eval_wait(eng, prev)])
        return out

    if use_async:
        steps_async(warm)
    else:
        for _ in range(warm):
            step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    disp0 = sum_stats(lambda e: e.jobs_stats())["pair_dispatches"]  # K1' dispatches before the timed steps
    for e in engs:
        e.jobs_stats_reset(time_pairs=True, count=False)
    ts = time.perf_counter()
    if use_async:
        summary, n_eval = steps_async(steps)
    else:
        for _ in range(steps):
            summary, n_eval = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    timing = sum_stats(lambda e: e.jobs_stats())
    for e in engs:
        e.jobs_stats_reset(time_pairs=False, count=True)
    step()  # untimed replay: pair and byte counts of one step on this rank
    st = sum_stats(lambda e: e.jobs_stats())
    for e in engs:
        e.jobs_stats_reset(time_pairs=False, count=False)
    selfcheck = None
    if world == 1:  # the batched driver against the sequential one on a small sample (untimed)
        h, c = ds.eval_recommendation_tests(eng, 64, CFG5_TOPK, 0, 1, 128)
        selfcheck = list(pf.rec_tests_summary(h, c)) == list(ds.recommendation_tests(eng, 64, CFG5_TOPK))
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([st["pairs"]], dtype=torch.float64, device="cuda")
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        st["pairs"] = float(c.item())
    launches = timing["pair_launches"]
    avg_ms = timing["pair_ms"] / launches if launches else None
    launches_per_step = launches / steps if steps else 0
    phys = ((st["pair_record_bytes"] + st["pair_image_bytes"]) / launches_per_step
            if launches_per_step else None)
    alg_pl = st["pair_alg_bytes"] / launches_per_step if launches_per_step else None

    def rate(b):
        return None if (b is None or not avg_ms) else b / (avg_ms * 1e-3) / 1e9

    achieved = rate(phys)
    # HBM bytes per pair stage: the timed stages' K1' dispatches grouped by the dispatch counters
    traffic, tsrc = pair_stage_traffic((pmc, pmc_err), {"disp0": disp0, "disp1": timing["pair_dispatches"],
                                                        "pair_launches": launches})
    value = n_eval * steps / elapsed
    rec = {
        "metric": METRIC, "value": value, "unit": "hold-out users/s", "n_gpus": world, "steps": steps,
        "warmup": warm, "ms_per_step": elapsed * 1e3 / steps, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded Pokec-shaped corpus in the reference's CSV formats, tools/pokec_synth.cpp; "
                "no Pokec data offline)",
        "config": {"workload": f"cfg5: run_recommendation_tests_sample over {S} users per step (graph/interest + "
                               f"collaborative + clubs, limit 5000, top-{CFG5_TOPK}) on the full {args.users}-user "
                               f"corpus" + (f", users split over {world} GPUs" if world > 1 else ""),
                   "workload_key": f"cfg5_rectests_{args.users}users_s{S}_top{CFG5_TOPK}_world{world}",
                   "n_users": args.users, "users_per_step": S, "topk": CFG5_TOPK, "limit": 5000,
                   "parallelism": f"hold-out users x{world}" + (" + all_gather" if world > 1 else "")
                                  + (f", {C} engine contexts per GPU" if C > 1 else "")},
        "rectests_summary": [float(x) for x in summary], "pairs_per_step": st["pairs"],
        "pair_fas_per_s": st["pairs"] / (elapsed / steps) if elapsed > 0 else None,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": None if achieved is None else achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "fas_pairs_kernel", "avg_launch_ms": avg_ms, "timed_launches": launches,
                     "bytes_per_launch": phys,
                     "bytes_model": "pf_jobs_stats: per scored pair the candidate's 48-B tile-store headers + record "
                                    "words (K1' walks the record), per 256-pair block the staged query image",
                     "dram_gbs": rate(traffic),
                     "dram_frac": None if traffic is None or not avg_ms else rate(traffic) / HBM_PEAK_GBS,
                     "traffic_source": tsrc,
                     "d3_equiv_gbs": rate(alg_pl),
                     "alg_bytes_per_launch": alg_pl,
                     "pair_kernel_share_of_step": (timing["pair_ms"] / (elapsed * 1e3)) if elapsed > 0 else None},
        "selfcheck_vs_sequential_64_users": selfcheck, "files_s": write_s, "open_s": open_s,
        "driver_calls": "asynchronous (pf_eval_recommendation_tests_async: step i + 1 planned beside step i's "
                        "last device chunk)" if use_async else "synchronous",
    }
    if rank == 0 and world == 1 and base is not None:
        rec["cpu_baseline"] = base
        rec["speedup_vs_cpu"] = value / base["value"] if base.get("value") else None
    elif rank == 0:
        rec["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if pool is not None:
        pool.shutdown()
    for e in engs:
        e.close()
    ds.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def solo_shards(args, eng, pf, torch, qstream, warm, steps, Q, k, n_cand, stream, n1_ms):
    """A one-GPU projection of cfg 4's N-GPU strong scaling (no multi-GPU node needed): each of the
    S shards pf_set_shard(r, S) gives a rank, timed ALONE on this whole GPU over the same 1,024-query
    steps; the projected N = S step is the slowest shard + the cross-shard merge (timed here on S
    gathered key lists) + an all-gather estimate for S x Q x k x 8 B over xGMI.  What does not divide
    by S shows as sum(shard ms) - the N = 1 step: per-query costs every shard pays again (the query
    image staged per workgroup, the fused merge, the launch)."""
    S = args.solo_shards
    sptr = stream.cuda_stream
    out = torch.empty((Q, k), dtype=torch.int64, device="cuda")
    ns = max(1, min(steps, args.solo_steps))
    per = []
    for r in range(S):
        eng.set_shard(r, S)
        eng.scan_keys_async(qstream[0], k, out.data_ptr(), sptr)  # warm this shard's launch shape
        torch.cuda.synchronize()
        eng.profile_sample(1)
        eng.profile_reset()
        ta = time.perf_counter()
        for i in range(warm, warm + ns):
            eng.scan_keys_async(qstream[i], k, out.data_ptr(), sptr)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - ta) * 1e3 / ns
        kms, nl = eng.profile_read()
        eng.profile_sample(0)
        lay = eng.layout()
        per.append({"shard": r, "ms_per_step": wall, "kernel_ms": kms / nl if nl else None,
                    "shard_cands": int(lay.shard_cands), "shard_entries": int(lay.shard_entries)})
    eng.set_shard(0, 1)
    # the merge of S gathered lists (pf_merge_keys_async, the N = S step's last kernel), timed alone
    gathered = torch.full((S, Q, k), -1, dtype=torch.int64, device="cuda")
    for r in range(S):
        gathered[r].copy_(out)
    torch.cuda.synchronize()
    ta = time.perf_counter()
    reps = 20
    for _ in range(reps):
        eng.merge_keys_async(gathered.data_ptr(), S, Q, k, out.data_ptr(), sptr)
    torch.cuda.synchronize()
    merge_ms = (time.perf_counter() - ta) * 1e3 / reps
    # all-gather estimate: a ring moves (S - 1) / S of the S x Q x k x 8 B per rank over one xGMI link
    # (~50 GB/s achieved of 153 GB/s peak per direction), plus ~25 us of collective latency
    ag_bytes = S * Q * k * 8
    ag_ms = 0.025 + (S - 1) / S * ag_bytes / 50e9 * 1e3
    ms = [x["ms_per_step"] for x in per]
    proj = max(ms) + merge_ms + ag_ms
    return {"shards": S, "steps_per_shard": ns, "per_shard": per,
            "shard_ms_max_over_mean": max(ms) / (sum(ms) / S),
            "merge_ms": merge_ms, "allgather_ms_estimate": ag_ms, "allgather_bytes": ag_bytes,
            "n1_ms_per_step": n1_ms, "sum_shard_ms": sum(ms),
            "non_dividing_ms": sum(ms) - n1_ms,
            "projected_ms_per_step": proj, "projected_value": Q * n_cand / (proj * 1e-3),
            "projected_speedup_vs_n1": n1_ms / proj,
            "note": "each shard timed alone on one whole GPU (the rank's work at N = S); projected N = S step = "
                    "max shard + merge (timed) + all-gather (estimated); not a multi-GPU measurement"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: cfg2 200 single-query steps, ~30 ms; every other workload 50)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--users", type=int, default=N_USERS)
    ap.add_argument("--queries-per-gpu", type=int, default=1)
    ap.add_argument("--workload", choices=["cfg2", "cfg3", "cfg4", "cfg5"], default=None,
                    help="cfg2: N queries per step (1 per GPU, weak scaling; the default at N = 1); "
                         "cfg3: collaborative FoF top-10, 64 queries per step (limit 10000), query users "
                         "split over the ranks; "
                         "cfg4: a fixed batch of 1024 queries per step over the sharded candidates (strong "
                         "scaling; the default at N > 1); "
                         "cfg5: hold-out evaluation (recommendation_tests: interest + collab + clubs) of 2048 "
                         "users per step, users split over the ranks")
    ap.add_argument("--contexts", type=int, default=None,
                    help="cfg3 / cfg5: engine contexts per GPU, each a full replica driven by its own host "
                         "thread; default 1 (cfg3: the asynchronous calls overlap the host planning; cfg5: one "
                         "context 99.6k-113.4k users/s against 99.0k-121.2k with three on the round-4 boxes, "
                         "DESIGN.md section 5)")
    ap.add_argument("--eval-sync", action="store_true",
                    help="cfg5: the synchronous driver call per step instead of the asynchronous one")
    ap.add_argument("--sync-calls", action="store_true",
                    help="cfg3: the synchronous recommender calls instead of the asynchronous ones")
    ap.add_argument("--async-depth", type=int, default=ASYNC_DEPTH,
                    help="cfg3: asynchronous calls kept in flight (1..3, the engine's workspace slots)")
    ap.add_argument("--cfg5-batch", type=int, default=CFG5_USERS,
                    help="cfg5: users per device pass of the driver (r2o: 128 -> 15.1k, 512 -> 17.2k, 2048 -> "
                         "31.8k users/s; a 2048-user pass runs as three pipelined chunks)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1 collectives: nccl (RCCL over xGMI, one rank per GPU) or gloo through host memory "
                         "(ranks may share one GPU: a correctness rehearsal of the multi-GPU path)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 FETCH_SIZE pass (traffic = null)")
    ap.add_argument("--time-every", type=int, default=1,
                    help="HIP-event timing on every n-th scan launch of the timed region (1 = all).  A timed "
                         "launch costs ~4 us of stream time (r6q, one box: 182.2 us per cfg-2 step timing every "
                         "launch, 179.9 every 2nd, 177.5 every 4th, 178.0 none); the default times every launch "
                         "so the line's average is over the same launches as rocprof's")
    ap.add_argument("--scan-kernel", choices=["auto", "stream", "postings"], default="auto",
                    help="all-candidates scan kernel (auto = postings when the corpus fits its encoding)")
    ap.add_argument("--no-cfg3", action="store_true",
                    help="cfg2 at N = 1: skip the cfg-3 sub-record (collaborative FoF top-10, 64 users per step)")
    ap.add_argument("--cfg3-steps", type=int, default=50,
                    help="timed steps of the cfg-3 sub-record (with 5 warmup steps: the query stream of --workload cfg3)")
    ap.add_argument("--solo-shards", type=int, default=0,
                    help="cfg4 at N = 1: also time each of S shards alone on this GPU and project the N = S "
                         "step (solo_shards record)")
    ap.add_argument("--solo-steps", type=int, default=3, help="timed steps per shard of --solo-shards")
    ap.add_argument("--same-query", action="store_true",
                    help="cfg2/cfg4 analysis only (not the workload): every query of every step is the first "
                         "query of the stream, so a batch's lists are all shared (bounds what a query-tiled "
                         "batch could save; the line's config says so)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="analysis: hardware queues for this process (GPU_MAX_HW_QUEUES, set before HIP starts; 0 = "
                         "the environment's, HIP's default 4); pair with PF_DEBUG scan_lanes=N.  16 queues with 15 "
                         "lanes read +3-5 %% over 200 steps but degrade with the backlog of longer runs "
                         "(profiles/r9_ab.txt r9x-r9ze), so the default line keeps four")
    ap.add_argument("--force-dist", action="store_true",
                    help="cfg2/cfg4 at WORLD_SIZE=1: run the N > 1 step anyway (scan into the local keys, an RCCL "
                         "all_gather_into_tensor on the scan stream, pf_merge_keys_async), so the communicator, "
                         "the collective and its stream ordering execute on one GPU (not a scaling run)")
    ap.add_argument("--n1-steps", type=int, default=5,
                    help="N > 1: steps rank 0 times the same workload unsharded on its own GPU (n1_same_workload)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    if args.workload is None:
        args.workload = "cfg2" if world == 1 else "cfg4"
    if args.steps is None:
        args.steps = 200 if args.workload == "cfg2" else 50
    if args.contexts is None:
        args.contexts = 1
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(16, args.hw_queues))  # before any HIP call
    if args.workload == "cfg5":
        return run_cfg5(args, world, rank, local)
    import synth

    t0 = time.time()
    corpus = synth.Corpus(n_users=args.users, seed=1, edge_cases=0, threads=16)
    desc = corpus.desc_ptr()
    t1 = time.time()
    # the cfg-3 sub-record of the default N = 1 line (the north star's FoF half, BASELINE cfg 3)
    sub3 = args.workload == "cfg2" and world == 1 and not args.no_cfg3
    W3 = 5  # the sub-record's warmup: with --cfg3-steps 50 the same seeded users as --workload cfg3's defaults
    # rank 0 at N = 1, before this process touches the GPU: the CPU baselines (forked, pinned
    # children) and the rocprofv3 PMC pass (a child running this same command)
    want_kernel = "fas_scan_kernel" if args.scan_kernel == "stream" else "fas_post_kernel"
    base, base3, pmcs = None, None, {}
    if rank == 0 and world == 1:
        if args.workload == "cfg3" or sub3:
            steps3 = args.steps if args.workload == "cfg3" else args.cfg3_steps
            warm3 = args.warmup if args.workload == "cfg3" else W3
            users3 = [int(u) for qs in cfg3_queries(args.users, warm3, steps3)[warm3:] for u in qs]
        if not args.no_cpu_baseline:
            base, base3 = cpu_baselines(desc, args.users, users3 if (args.workload == "cfg3" or sub3) else None)
            if args.workload == "cfg3":
                base = base3
            log(f"cpu baseline: {base}")
        if not args.no_pmc:
            sel = {}
            if args.workload in ("cfg2", "cfg4"):
                # the timed launches: the last `steps` before the isolated-launch sample (cfg 2 at N = 1:
                # min(steps, 20) launches after the timed region)
                # cfg 2 at N = 1: the isolated launches, the ones the line's roofline divides by (the
                # counter pass serialises dispatches anyway); otherwise the timed launches
                iso = min(args.steps, 20) if (args.workload == "cfg2" and args.queries_per_gpu == 1) else 0
                sel[want_kernel] = ((lambda v, k=args.steps, i=iso: v[len(v) - i:] if len(v) >= k + i else [])
                                    if iso else (lambda v, k=args.steps: v[len(v) - k:] if len(v) >= k else []))
            if args.workload == "cfg3" or sub3:
                # every K1' dispatch; the timed stages' ones are picked later by the engines'
                # dispatch counters (pair_stage_traffic)
                sel["fas_pairs_kernel"] = lambda v: v
            pmcs = pmc_pass(args, sel)
            for k, (_, e) in pmcs.items():
                if e:
                    log(f"pmc pass {k}: {e}")

    import torch
    local = local % max(1, torch.cuda.device_count())  # --dist-backend gloo: ranks may share a GPU
    torch.cuda.set_device(local)
    # --force-dist: the collective path at world 1 (before any other GPU work of this process)
    use_dist = world > 1 or (args.force_dist and args.workload in ("cfg2", "cfg4"))
    if use_dist and world == 1:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 2000))
    dist = Comm(args.dist_backend, local) if use_dist else None
    import pokec_fas as pf

    t2 = time.time()
    eng = pf.FasEngine(desc, local)
    t3 = time.time()
    if args.workload == "cfg3":
        engs = [eng] + [pf.FasEngine(desc, local) for _ in range(max(1, args.contexts) - 1)]
        return run_cfg3(args, engs, pf, torch, dist, world, rank, base, pmcs.get("fas_pairs_kernel"),
                        time.time() - t2)
    eng.set_shard(rank, world)
    eng.set_scan_kernel({"auto": pf.PF_SCAN_AUTO, "stream": pf.PF_SCAN_STREAM, "postings": pf.PF_SCAN_POSTINGS}
                        [args.scan_kernel])
    lay = eng.layout()
    kernel_name = "fas_post_kernel" if lay.scan_kernel == pf.PF_SCAN_POSTINGS else "fas_scan_kernel"
    pmc, pmc_err = pmcs.get(kernel_name, (None, "not run (N > 1 or --no-pmc)"))
    if rank == 0 and world == 1 and not args.no_pmc and kernel_name != want_kernel:
        pmc, pmc_err = None, f"the pass profiled {want_kernel}, the engine runs {kernel_name}"
    log(f"[rank {rank}] corpus {t1 - t0:.1f}s, engine open {t3 - t2:.1f}s, stream {lay.stream_bytes / 1e9:.3f} GB, "
        f"alg {lay.alg_bytes / 1e9:.3f} GB, packed={lay.packed_tokens}")

    cfg4 = args.workload == "cfg4"
    Q = CFG4_QUERIES if cfg4 else world * args.queries_per_gpu
    k = TOPK
    steps, warm = args.steps, args.warmup
    rng = np.random.default_rng(3 if cfg4 else 2)  # same query stream on every rank (SURVEY D1 seeds)
    qstream = rng.integers(1, args.users + 1, size=(warm + steps, Q)).astype(np.int32)
    if args.same_query:  # analysis: perfect list sharing inside every batch (not the metric's workload)
        qstream[:] = qstream[0, 0]
    # a dedicated stream: the engine, the all-gather and the copies are all ordered on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    local_keys = torch.empty((Q, k), dtype=torch.int64, device="cuda")
    gathered = torch.empty((world, Q, k), dtype=torch.int64, device="cuda") if use_dist else None
    final = torch.empty((Q, k), dtype=torch.int64, device="cuda")

    def step(i):
        if not use_dist:  # the scan's fused merge already yields the final top-k
            eng.scan_keys_async(qstream[i], k, final.data_ptr(), sptr)
            return
        eng.scan_keys_async(qstream[i], k, local_keys.data_ptr(), sptr)
        dist.all_gather_into_tensor(gathered, local_keys)
        eng.merge_keys_async(gathered.data_ptr(), world, Q, k, final.data_ptr(), sptr)

    n_cand = eng.num_users - 1  # candidates per query: every profile but the query (minus adj[q])
    # N > 1: rank 0 first runs the same workload unsharded on its own GPU (the like-for-like N = 1
    # point of the driver's scaling curve); the other ranks wait at the barrier
    n1 = None
    if world > 1:
        if rank == 0:
            eng.set_shard(0, 1)
            for i in range(min(warm, 2)):
                eng.scan_keys_async(qstream[i], k, final.data_ptr(), sptr)
            torch.cuda.synchronize()
            ns = max(1, min(args.n1_steps, steps))
            ta = time.perf_counter()
            for i in range(warm, warm + ns):
                eng.scan_keys_async(qstream[i], k, final.data_ptr(), sptr)
            torch.cuda.synchronize()
            el1 = time.perf_counter() - ta
            n1 = {"value": Q * n_cand * ns / el1, "unit": "candidates/s", "steps": ns, "ms_per_step": el1 * 1e3 / ns,
                  "note": "rank 0 alone, the same queries over the whole corpus (unsharded, no collective), timed "
                          "before the sharded steps: the like-for-like N = 1 point for this line's value"}
            eng.set_shard(rank, world)
        dist.barrier()

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
    t_submitted = time.perf_counter() - t_start  # the host's enqueue time for the K steps
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    scan_ms, launches = eng.profile_read()
    eng.profile_sample(0)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # sanity: the merged top-k of the last step rescored by the pair kernel
    last = final.cpu().numpy().view(np.uint64)
    uids, scores = pf.decode_keys(last[0])
    chk = eng.fas_pairs(np.full(len(uids), qstream[warm + steps - 1][0], np.int32), uids)
    consistent = bool(len(uids) == k and np.array_equal(chk.view(np.uint32), scores.view(np.uint32)))

    # One query per step on a caller's stream runs on the engine's two scan lanes (pf_ctx.h
    # ScanLane): consecutive launches overlap, so a launch's HIP events span its neighbours' tails.
    # After the timed region, the same queries once more one at a time (synchronised, untimed by
    # the step clock) give the kernel's isolated launch time beside it.
    isolated = None
    if Q == 1 and not use_dist:
        eng.profile_sample(1)
        eng.profile_reset()
        n_iso = min(steps, 20)
        for i in range(warm, warm + n_iso):
            eng.scan_keys_async(qstream[i], k, final.data_ptr(), sptr)
            torch.cuda.synchronize()
        iso_ms, iso_n = eng.profile_read()
        eng.profile_sample(0)
        if iso_n:
            isolated = {"launches": iso_n, "avg_launch_ms": iso_ms / iso_n,
                        "note": "the first timed queries again, one at a time after the timed region (the same launch "
                                "shape: seven eighths of a resident round of workgroups); the roofline's avg_launch_ms is the "
                                "steady-state time per launch"}


    value = Q * n_cand * steps / elapsed
    # bytes per launch by the kernel's access pattern, over the queries timed (this rank's shard)
    # one call per step: the byte model counts the image staging of a launch of Q queries
    phys = np.concatenate([eng.scan_bytes(qstream[i]) for i in range(warm, warm + steps)])
    timed_steps = list(range(0, steps, max(args.time_every, 1)))[:launches] if launches else []
    phys_per_launch = (float(np.mean([phys[i * Q:(i + 1) * Q].sum() for i in timed_steps]))
                       if timed_steps else None)
    avg_launch_ms = scan_ms / launches if launches else None
    # N > 1: every rank's scan time and shard (pf_set_shard's static posting-weight split), so the
    # line shows the per-shard skew behind the max-over-ranks step time
    per_rank = None
    if dist:
        ls = eng.layout()
        t = torch.tensor([[avg_launch_ms or 0.0, float(ls.shard_cands), float(ls.shard_entries),
                           phys_per_launch or 0.0]], dtype=torch.float64, device="cuda")
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        rows = [p.cpu().numpy()[0] for p in parts]
        ms_r = [float(x[0]) for x in rows]
        cand_r = [float(x[1]) for x in rows]
        per_rank = {"ranks": [{"rank": r, "avg_launch_ms": ms_r[r], "shard_cands": int(cand_r[r]),
                               "shard_entries": int(rows[r][2]), "bytes_per_launch": float(rows[r][3])}
                              for r in range(world)],
                    "launch_ms_max_over_mean": max(ms_r) / (sum(ms_r) / world) if sum(ms_r) > 0 else None,
                    "shard_cands_max_over_mean": max(cand_r) / (sum(cand_r) / world) if sum(cand_r) > 0 else None}
    # SURVEY 8(d) D3 record bytes of this rank's shard x queries per launch (the metric's definition)
    shard_frac = 1.0 / world
    alg_bytes = lay.alg_bytes * shard_frac * Q

    def rate_ms(b, ms):  # GB/s of b bytes over ms
        return None if (b is None or not ms) else b / (ms * 1e-3) / 1e9

    def rate(b):  # GB/s over the average launch
        return rate_ms(b, avg_launch_ms)

    achieved = rate(phys_per_launch)
    alg_eff = rate(alg_bytes)
    traffic = pmc["bytes_per_launch"] if pmc else None
    workload = f"{args.workload}_all_candidates_top{k}_{args.users}users_q{Q}_shard1of{world}"
    if cfg4:
        wl_name = (f"cfg4: {Q}-query batch, interest FAS all-candidates top-10 over the full 1.6M-user corpus, "
                   f"candidates sharded over {world} GPU(s)" + ("" if world == 1 else ", RCCL all-gather of per-shard top-10"))
    else:
        wl_name = ("cfg2: full 1.6M-user single-query interest FAS all-candidates top-10"
                   + ("" if world == 1 else f"; {Q} queries/step, candidates sharded over {world} GPUs, "
                                            "RCCL all-gather of per-shard top-10"))
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
        "config": {"workload": wl_name + (" [ANALYSIS: --same-query, every query the same user]" if args.same_query else ""),
                   "workload_key": workload + ("_samequery" if args.same_query else ""), "n_users": args.users,
                   "queries_per_step": Q, "topk": k,
                   "parallelism": f"candidate-shard x{world}" + (" + all_gather" if use_dist else ""),
                   "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "4 (HIP default)"),
                   **({"force_dist": "the N > 1 step (local keys, RCCL all-gather, device merge) at world 1: a "
                                     "code-path check, not a scaling point"} if use_dist and world == 1 else {})},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": None if achieved is None else achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kernel_name, "avg_launch_ms": avg_launch_ms,
                     "timed_launches": launches, "timed_every": args.time_every,
                     "bytes_per_launch": phys_per_launch,
                     "bytes_model": ("pf_scan_bytes: per block 32-B headers, 2 cell words per query list, each list's "
                                     "cell-range entries (4 B; token entries + 8-B norm), exclusions; staged image "
                                     "per workgroup" if kernel_name == "fas_post_kernel" else
                                     "pf_scan_bytes: the shard's record stream + 48-B headers"),
                     "dram_gbs": rate(traffic),
                     "dram_frac": None if traffic is None or not avg_launch_ms else rate(traffic) / HBM_PEAK_GBS,
                     "traffic_source": ({k: v for k, v in pmc.items() if k != "_raw"} if pmc else pmc_err),
                     "d3_equiv_gbs": alg_eff,
                     "d3_equiv_x_peak": None if alg_eff is None else alg_eff / HBM_PEAK_GBS,
                     "alg_bytes_per_launch": alg_bytes,
                     "note": ("achieved/frac: the bytes this kernel reads by its access pattern; "
                              "d3_equiv_*: SURVEY D3 record bytes b_c of every candidate over the same time (the "
                              "postings scan reads only the query's lists, so that effective rate can pass the peak)")},
        "topk_selfcheck": consistent,
        "host_enqueue_ms_per_step": t_submitted * 1e3 / steps,
    }
    if isolated is not None and phys_per_launch:
        # One query per step: consecutive launches overlap on the scan lanes (up to three in flight),
        # so a timed launch's HIP events span its neighbours' work and no launch runs alone.  The
        # roofline divides a launch's bytes by the steady-state time per launch, ms_per_step (the
        # timed region's launch-to-launch interval; rocprofv3's trace of the same run gives the same
        # span over its K5 dispatches, profiles/r9*_k5_trace_summary.json), and keeps the overlapped
        # events and an isolated launch (the same queries once more, one at a time) as named fields
        iso_bytes = float(np.mean([phys[i * Q:(i + 1) * Q].sum() for i in range(isolated["launches"])]))
        iso_gbs = iso_bytes / (isolated["avg_launch_ms"] * 1e-3) / 1e9
        R = rec["roofline"]
        R["overlapped_launch"] = {"avg_launch_ms": avg_launch_ms, "timed_launches": launches,
                                  "bytes_per_launch": phys_per_launch, "achieved": achieved,
                                  "frac": None if achieved is None else achieved / HBM_PEAK_GBS,
                                  "note": "the timed region's launches, each overlapping its neighbours on the "
                                          "scan lanes (HIP events span the overlap)"}
        step_ms = rec["ms_per_step"]
        step_gbs = phys_per_launch / (step_ms * 1e-3) / 1e9
        R.update({"achieved": step_gbs, "frac": step_gbs / HBM_PEAK_GBS, "avg_launch_ms": step_ms,
                  "launch_basis": "steady state: the timed region's time per launch (ms_per_step; launches overlap "
                                  "on the scan lanes)",
                  "dram_gbs": rate_ms(traffic, step_ms),
                  "dram_frac": (None if traffic is None else rate_ms(traffic, step_ms) / HBM_PEAK_GBS),
                  "d3_equiv_gbs": rate_ms(alg_bytes, step_ms)})
        R["d3_equiv_x_peak"] = R["d3_equiv_gbs"] / HBM_PEAK_GBS
        isolated["bytes_per_launch"] = iso_bytes
        isolated["achieved_gbs"], isolated["frac"] = iso_gbs, iso_gbs / HBM_PEAK_GBS
        isolated["dram_frac"] = None if traffic is None else rate_ms(traffic, isolated["avg_launch_ms"]) / HBM_PEAK_GBS
        R["isolated_launch"] = isolated
    if n1 is not None:
        rec["n1_same_workload"] = n1
    if per_rank is not None:
        rec["per_rank"] = per_rank
    if rank == 0 and world == 1 and base is not None:
        rec["cpu_baseline"] = base
        rec["speedup_vs_cpu"] = value / base["value"] if base.get("value") else None
    elif rank == 0:
        rec["cpu_baseline"] = None
    if cfg4 and world == 1 and args.solo_shards > 1:
        rec["solo_shards"] = solo_shards(args, eng, pf, torch, qstream, warm, steps, Q, k, n_cand, stream,
                                         elapsed * 1e3 / steps)
    if sub3:
        # cfg 3 (BASELINE configs[2]) on the same engine: recommend_collaborative(u, 10, 10000) for
        # 64 seeded users per step, one engine context (the default line's own replica)
        ta = time.perf_counter()
        mine = cfg3_queries(args.users, W3, args.cfg3_steps)
        st = measure_cfg3([eng], mine, W3, args.cfg3_steps, None, torch)
        f3 = cfg3_fields(st, args.cfg3_steps, pmcs.get("fas_pairs_kernel"))
        f3.update({"steps": args.cfg3_steps, "warmup": W3, "contexts": 1,
                   "workload": f"cfg3: recommend_collaborative(u, {TOPK}, {CFG3_LIMIT}) for {CFG3_QUERIES} seeded users "
                               f"per step on the full {args.users}-user corpus, one engine context",
                   "cpu_baseline": base3,
                   "speedup_vs_cpu": f3["value"] / base3["value"] if base3 and base3.get("value") else None,
                   "wall_s": time.perf_counter() - ta})
        rec["cfg3"] = f3
    if rank == 0:
        print(json.dumps(rec), flush=True)
    eng.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
