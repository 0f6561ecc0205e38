"""How much of a cfg-4 batch's postings work is shared between its queries.

For the seeded cfg-4 batch (bench.py: 1024 query uids per step, rng seed 3, the D1 corpus), every
query's K5 lists are its (column, tid) token lists (tf > 0, weight != 0), its distinct clubs and its
distinct friends (the `friends` column).  A list of L entries costs a query L entries of walk.  This
reports, over the batch:
  - total entries walked by the 1024 queries separately (sum over queries of their lists' lengths),
  - entries of the DISTINCT lists of the batch (each list once),
  - the fraction of the walk in lists shared by >= 2, >= 8, >= 64 queries,
  - the same per query tile of Q consecutive queries (a workgroup holding Q queries' state would
    read a list once per tile): the walk the tiles would do for Q = 2, 4, 8, 16.
Usage: python tools/cfg4_sharing.py [--users 1632803] [--out profiles/r4_cfg4_sharing.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from collections import Counter

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import synth  # noqa: E402


class Desc(ctypes.Structure):
    _fields_ = [("n_users", ctypes.c_int32), ("n_cols", ctypes.c_int32),
                ("user_id", ctypes.c_void_p), ("public_flag", ctypes.c_void_p), ("completion", ctypes.c_void_p),
                ("gender", ctypes.c_void_p), ("age", ctypes.c_void_p), ("region", ctypes.c_void_p),
                ("club_off", ctypes.c_void_p), ("club_ids", ctypes.c_void_p),
                ("friend_off", ctypes.c_void_p), ("friend_ids", ctypes.c_void_p),
                ("tok_off", ctypes.c_void_p), ("tok_tid", ctypes.c_void_p), ("tok_tf", ctypes.c_void_p)]


def arr(ptr, n, dt):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1632803)
    ap.add_argument("--queries", type=int, default=1024)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t0 = time.time()
    c = synth.Corpus(n_users=a.users, seed=1, edge_cases=0, threads=16)
    d = Desc.from_address(c.desc_ptr())
    n, T = d.n_users, d.n_cols
    tok_off = arr(d.tok_off, n * T + 1, np.int64)
    tid = arr(d.tok_tid, int(tok_off[-1]), np.int32)
    tf = arr(d.tok_tf, int(tok_off[-1]), np.int32)
    club_off = arr(d.club_off, n + 1, np.int64)
    clubs = arr(d.club_ids, int(club_off[-1]), np.uint32)
    fr_off = arr(d.friend_off, n + 1, np.int64)
    friends = arr(d.friend_ids, int(fr_off[-1]), np.uint32)
    uid = arr(d.user_id, n, np.int32)
    # list lengths: token lists = df over tf > 0; set lists = users holding the id (distinct per user)
    row_col = np.repeat(np.tile(np.arange(T, dtype=np.int64), n), np.diff(tok_off))
    keep = tf > 0
    tkey = (row_col[keep] << 32) | tid[keep].astype(np.int64)
    tk, tcnt = np.unique(tkey, return_counts=True)
    tlen = dict(zip(tk.tolist(), tcnt.tolist()))

    def set_lens(off, ids):
        u = np.repeat(np.arange(n, dtype=np.int64), np.diff(off))
        pairs = np.unique((ids.astype(np.int64) << 32) | u)
        k, cnt = np.unique(pairs >> 32, return_counts=True)
        return dict(zip(k.tolist(), cnt.tolist()))

    clen, flen = set_lens(club_off, clubs), set_lens(fr_off, friends)
    t1 = time.time()
    rng = np.random.default_rng(3)
    q = rng.integers(1, a.users + 1, size=a.queries).astype(np.int32)  # bench.py's first cfg-4 step
    idx_of = {int(u): i for i, u in enumerate(uid)} if not np.array_equal(uid, np.arange(1, n + 1)) else None
    qlists = []
    for u in q:
        i = (idx_of[int(u)] if idx_of else int(u) - 1)
        L = set()
        for t in range(T):
            s, e = tok_off[i * T + t], tok_off[i * T + t + 1]
            for k in range(s, e):
                if tf[k] > 0:
                    L.add(("t", (t << 32) | int(tid[k])))
        for x in set(clubs[club_off[i]:club_off[i + 1]].tolist()):
            L.add(("c", x))
        for x in set(friends[fr_off[i]:fr_off[i + 1]].tolist()):
            L.add(("f", x))
        qlists.append(L)

    def length(key):
        kind, x = key
        return tlen[x] if kind == "t" else (clen if kind == "c" else flen).get(x, 0)

    share = Counter()
    for L in qlists:
        share.update(L)
    per_query = sum(length(k) for L in qlists for k in L)
    distinct = sum(length(k) for k in share)
    frac = {f">={m}": sum(length(k) * cnt for k, cnt in share.items() if cnt >= m) / per_query for m in (2, 8, 64)}
    tiles = {}
    for Q in (2, 4, 8, 16, 32):
        w = 0
        for b in range(0, len(qlists), Q):
            u = set().union(*qlists[b:b + Q])
            w += sum(length(k) for k in u)
        tiles[str(Q)] = {"entries": w, "vs_separate": w / per_query}
    tok_pq = sum(length(k) for L in qlists for k in L if k[0] == "t")
    rec = {
        "what": "cfg-4 batch list sharing (tools/cfg4_sharing.py; VERDICT r3 item 2)",
        "users": a.users, "queries": a.queries, "query_seed": 3,
        "entries_walked_separately": per_query, "token_entries_separately": tok_pq,
        "entries_distinct_lists": distinct, "distinct_vs_separate": distinct / per_query,
        "walk_fraction_in_lists_shared_by": frac,
        "query_tiles": tiles,
        "lists_per_query_mean": float(np.mean([len(L) for L in qlists])),
        "distinct_lists": len(share),
        "corpus_s": t1 - t0, "analysis_s": time.time() - t1,
    }
    print(json.dumps(rec, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
