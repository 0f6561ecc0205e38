import sys, numpy as np, torch
sys.path.insert(0, "recommendation-system-pokec_amd"); sys.path.insert(0, "tools"); sys.path.insert(0, "tests")
import synth, pokec_fas as pf, pokec_testlib as tl
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
c = synth.Corpus(n_users=n, seed=1, threads=16); d = c.desc_ptr()
eng = pf.FasEngine(d, 0)
torch.cuda.set_device(0)
s = torch.cuda.current_stream()
keys = torch.empty((1, 10), dtype=torch.int64, device="cuda")
for q in [5, 77, 123456 % n, 999]:
    eng.scan_keys_async(np.array([q], np.int32), 10, keys.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    u1, s1 = pf.decode_keys(keys.cpu().numpy().view(np.uint64)[0])
    (u2, s2), = eng.recommend_interest_all([q], 10)
    chk = eng.fas_pairs(np.full(len(u1), q, np.int32), u1)
    print(q, "scan==interest_all", list(u1) == list(u2), np.array_equal(s1, s2), "pairs==scan", np.array_equal(chk, s1))
    if not np.array_equal(chk, s1):
        print("  uids", list(u1)); print("  scan", s1); print("  pair", chk)
if n <= 300000:
    orc = tl.Oracle(None, desc_ptr=d)
    (u3, s3), = orc.interest([5], 10, tl.PF_MODE_ALL, 0)
    (u2, s2), = eng.recommend_interest_all([5], 10)
    print("oracle==gpu", list(u3) == list(u2), np.array_equal(s3, s2))
    print("oracle pairs vs gpu pairs", np.abs(orc.fas_pairs(np.full(10, 5, np.int32), u3) - eng.fas_pairs(np.full(10, 5, np.int32), u3)).max())
