"""Child process of test_gpu_parity.test_kernel_variants: the engine reads PF_DEBUG's
stage_limit, tile_steps, scan, k5_block, k5_wgs and resident_images once per process/context, so each
forced kernel variant (global-memory query tables, records split over lanes, postings block sizes,
few workgroups per one-query launch, per-call query images, a variant library via PF_LIB_PATH) runs
in its own process.  Besides the batched calls, every query is also scanned alone on a caller's
stream (pf_scan_keys_async, the cfg-2 step: the scan lanes, every block claimed per XCD group; with
k5_wgs=16 each workgroup claims several blocks).  Exits non-zero on any mismatch."""
import sys

import numpy as np

import pokec_testlib as tl


def main():
    c = tl.synth.Corpus(n_users=20000, seed=77, edge_cases=1)
    ptr = c.desc_ptr()
    eng, orc = tl.engine(ptr), tl.Oracle(None, desc_ptr=ptr)
    rng = np.random.default_rng(11)
    q = [int(x) for x in rng.integers(1, 20001, 6)] + [8, 1]
    for k in (10, 64):
        for rep in range(2):  # the second pass reuses the per-query rendezvous state
            got = eng.recommend_interest_all(q, k)
            ref = orc.interest(q, k, tl.PF_MODE_ALL, 0)
            for u, g, r in zip(q, got, ref):
                if list(g[0]) != list(r[0]) or not np.array_equal(g[1].view(np.uint32), r[1].view(np.uint32)):
                    print(f"mismatch uid={u} k={k} rep={rep}", file=sys.stderr)
                    return 1
    # one query per call on a caller's stream (bench.py's cfg-2 step), rows copied out in call order
    import torch
    pf = tl.product()
    st = torch.cuda.Stream()
    qs = q + [int(x) for x in rng.integers(1, 20001, 16)]
    outs = torch.empty((len(qs), 10), dtype=torch.int64, device="cuda")
    for i, u in enumerate(qs):
        eng.scan_keys_async(np.array([u], np.int32), 10, outs[i].data_ptr(), st.cuda_stream)
    st.synchronize()
    keys = outs.cpu().numpy().view(np.uint64)
    for u, kr, r in zip(qs, keys, orc.interest(qs, 10, tl.PF_MODE_ALL, 0)):
        uids, scores = pf.decode_keys(kr)
        if list(uids) != list(r[0]) or not np.array_equal(np.asarray(scores, np.float32).view(np.uint32),
                                                          np.asarray(r[1], np.float32).view(np.uint32)):
            print(f"single-query mismatch uid={u}", file=sys.stderr)
            return 1
    a = rng.integers(1, 20001, 20000).astype(np.int32)
    b = rng.integers(1, 20001, 20000).astype(np.int32)
    if np.count_nonzero(eng.fas_pairs(a, b).view(np.uint32) != orc.fas_pairs(a, b).view(np.uint32)):
        print("pair mismatch", file=sys.stderr)
        return 1
    # the collaborative recommender (per-call images: resident_images=0)
    qc = [3, 8, 1000, 15000, 19999]
    for u, g, r in zip(qc, eng.recommend_collaborative(qc, 10, 1000), orc.collab(qc, 10, 1000)):
        if list(g[0]) != list(r[0]) or not np.array_equal(g[1].view(np.uint32), r[1].view(np.uint32)):
            print(f"collab mismatch uid={u}", file=sys.stderr)
            return 1
    print("ok")
    return 0


if __name__ == "__main__":
    sys.exit(main())
