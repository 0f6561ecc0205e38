"""Child process of test_gpu_parity.test_rccl_world1_merge: bench.py's N > 1 step with a real RCCL
communicator at world size 1 (one GPU).  Each step scans into the rank's local keys on a dedicated
stream, all-gathers them with torch.distributed's "nccl" backend (RCCL) on that stream
(all_gather_into_tensor, as bench.py `step` does), and merges the gathered lists with
pf_merge_keys_async on the same stream.  The merged keys must equal the unsharded scan (ids and score
bits), for a batch call and for one-query calls on the scan lanes.  Exits non-zero on any mismatch."""
import os
import socket
import sys

import numpy as np

import pokec_testlib as tl


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    import torch
    import torch.distributed as dist
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(free_port()), "RANK": "0", "WORLD_SIZE": "1"})
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    pf = tl.product()
    c = tl.synth.Corpus(n_users=20000, seed=77, edge_cases=1)
    eng = tl.engine(c.desc_ptr())
    world, k = dist.get_world_size(), 10
    eng.set_shard(dist.get_rank(), world)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    rng = np.random.default_rng(9)
    bad = 0
    for Q in (5, 1, 1, 1, 1):
        q = rng.integers(1, 20001, Q).astype(np.int32)
        local = torch.empty((Q, k), dtype=torch.int64, device="cuda")
        gathered = torch.empty((world, Q, k), dtype=torch.int64, device="cuda")
        final = torch.empty((Q, k), dtype=torch.int64, device="cuda")
        for rep in range(3):
            eng.scan_keys_async(q, k, local.data_ptr(), sptr)
            dist.all_gather_into_tensor(gathered, local)
            eng.merge_keys_async(gathered.data_ptr(), world, Q, k, final.data_ptr(), sptr)
        stream.synchronize()
        keys = final.cpu().numpy().view(np.uint64)
        ref = eng.recommend_interest_all([int(x) for x in q], k)
        for i in range(Q):
            uids, scores = pf.decode_keys(keys[i])
            if list(uids) != list(ref[i][0]) or not np.array_equal(np.asarray(scores, np.float32).view(np.uint32),
                                                                   ref[i][1].view(np.uint32)):
                print(f"mismatch Q={Q} uid={q[i]}", file=sys.stderr)
                bad += 1
    eng.close()
    dist.barrier()
    dist.destroy_process_group()
    if bad:
        return 1
    print(f"ok: world {world}, backend {dist.Backend.NCCL}, merged keys = unsharded scan")
    return 0


if __name__ == "__main__":
    sys.exit(main())
