import os, sys, numpy as np
sys.path.insert(0, "tests"); import pokec_testlib as tl
c = tl.synth.Corpus(n_users=20000, seed=77, edge_cases=1)
ptr = c.desc_ptr()
orc = tl.Oracle(None, desc_ptr=ptr)
eng = tl.engine(ptr)
q = [3, 8, 1000, 15000]
g = eng.recommend_interest_all(q, 10); r = orc.interest(q, 10, tl.PF_MODE_ALL, 0)
for u, a, b in zip(q, g, r):
    print(os.environ.get("PF_STAGE_LIMIT"), u, list(a[0]) == list(b[0]), np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)))
    if list(a[0]) != list(b[0]): print(" gpu", list(a[0]), a[1]); print(" orc", list(b[0]), b[1])
a = np.repeat(np.array(q, np.int32), 2000); b = np.random.default_rng(1).integers(1, 20001, len(a)).astype(np.int32)
d = eng.fas_pairs(a, b) - orc.fas_pairs(a, b)
print("pairs max diff", np.abs(d).max(), "nonzero", np.count_nonzero(d))
