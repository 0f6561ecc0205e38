"""Child process of test_gpu_parity.test_kernel_variants: the engine reads PF_DEBUG's
stage_limit, tile_steps, scan, k5_block and resident_images once per process/context, so each forced
kernel variant (global-memory query tables, records split over lanes, postings block sizes, per-call
query images) runs in its own process.  Exits non-zero on any
mismatch."""
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
