"""Python binding of the MI355X FAS engine (ctypes over libpokec_fas.so, the C ABI
of include/pokec_fas.h).

Mirrors the reference's `Recommender` operator surface (include/recommender.h:17-71)
with the same names, argument meaning and error behaviour: an unknown user yields an
empty list (recommender_graph.cpp:36-40), results are [(id, score)] sorted by
(score desc, id asc).  The library is loaded from this directory (built in-tree by
`make -C recommendation-system-pokec_amd`); if it or a gfx950 GPU is missing, opening
an engine raises — there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PF_LIB_PATH") or os.path.join(HERE, "libpokec_fas.so")

PF_OK, PF_EINVAL, PF_ENODEV, PF_ENOMEM, PF_ENOTFOUND, PF_EUNSUPP = 0, -1, -2, -3, -4, -5
PF_MODE_FOF, PF_MODE_ALL = 0, 1
PF_FOF_GRAPH, PF_FOF_COLLAB = 0, 1
PF_SCAN_AUTO, PF_SCAN_STREAM, PF_SCAN_POSTINGS = 0, 1, 2
MAX_TOPK_DEVICE = 64

# every entry point of include/pokec_fas.h
EXPORTS = ["pf_abi_version", "pf_open", "pf_close", "pf_last_error", "pf_num_users", "pf_idf", "pf_fas_pairs",
           "pf_recommend_interest", "pf_recommend_collab", "pf_recommend_clubs", "pf_fof_candidates", "pf_set_adj",
           "pf_set_shard", "pf_scan_keys_async", "pf_merge_keys_async", "pf_decode_keys", "pf_layout",
           "pf_last_scan_ms", "pf_profile_reset", "pf_profile_read", "pf_profile_sample", "pf_set_scan_kernel",
           "pf_scan_bytes", "pf_jobs_stats_reset", "pf_jobs_stats_read", "pf_recommend_interest_async",
           "pf_recommend_collab_async", "pf_recommend_clubs_async", "pf_wait", "pf_completed_ticket"]
# include/pokec_io.h: loaders and hold-out drivers
IO_EXPORTS = ["pf_dataset_load", "pf_dataset_load_cached", "pf_dataset_free", "pf_dataset_desc", "pf_dataset_info_get", "pf_dataset_column",
              "pf_dataset_profile_order", "pf_dataset_adj_order", "pf_dataset_profile_json", "pf_dataset_club_name",
              "pf_compute_normalizers", "pf_holdout_friends", "pf_recommendation_tests",
              "pf_eval_holdout_friends", "pf_eval_recommendation_tests", "pf_holdout_friends_digest",
              "pf_recommendation_tests_digest", "pf_eval_holdout_friends_digest",
              "pf_eval_recommendation_tests_digest", "pf_eval_recommendation_tests_async"]
PF_LOAD_REFERENCE_CAP = 100000


class PfLayoutStats(ctypes.Structure):
    _fields_ = [("n_slots", ctypes.c_int64), ("stream_bytes", ctypes.c_int64), ("header_bytes", ctypes.c_int64),
                ("alg_bytes", ctypes.c_int64), ("packed_tokens", ctypes.c_int32), ("n_tiles", ctypes.c_int32),
                ("post_bytes", ctypes.c_int64), ("scan_kernel", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("shard_cands", ctypes.c_int64), ("shard_entries", ctypes.c_int64)]


class PfJobsStats(ctypes.Structure):
    _fields_ = [("jobs", ctypes.c_int64), ("candidates", ctypes.c_int64), ("pairs", ctypes.c_int64),
                ("pair_alg_bytes", ctypes.c_int64), ("pair_record_bytes", ctypes.c_int64),
                ("pair_image_bytes", ctypes.c_int64), ("pair_ms", ctypes.c_double), ("pair_launches", ctypes.c_int64),
                ("pair_dispatches", ctypes.c_int64)]


class PfDatasetInfo(ctypes.Structure):
    _fields_ = [("lines_read", ctypes.c_int64), ("n_profiles", ctypes.c_int32), ("n_cols", ctypes.c_int32),
                ("n_adj", ctypes.c_int32), ("median_age", ctypes.c_int32), ("median_loaded", ctypes.c_int32),
                ("ages_replaced", ctypes.c_int32), ("n_normalizers", ctypes.c_int32),
                ("vocab_loaded", ctypes.c_int32), ("n_club_names", ctypes.c_int32)]


class FasError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libpokec_fas.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FasError(f"{LIB_PATH} missing: build it with `make -C {HERE}` (no CPU fallback exists)")
        # One HIP runtime per process: torch's libraries ask for "libamdhip64.so" (its bundled
        # copy), this library for "libamdhip64.so.7".  Loaded in that order the engine binds to
        # torch's copy; the other way round the process ends up with two HIP/HSA runtimes and
        # whichever initialises second finds no device.  So torch, when present, goes first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        V, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.pf_abi_version.restype = ctypes.c_int
        L.pf_open.argtypes = [V, ctypes.c_int, ctypes.POINTER(V)]
        L.pf_close.argtypes = [V]
        L.pf_last_error.argtypes = [V]
        L.pf_last_error.restype = ctypes.c_char_p
        L.pf_num_users.argtypes = [V]
        L.pf_num_users.restype = I32
        L.pf_idf.argtypes = [V, I32, I32]
        L.pf_idf.restype = ctypes.c_float
        L.pf_fas_pairs.argtypes = [V, V, V, I64, V]
        L.pf_recommend_interest.argtypes = [V, V, I32, I32, I32, I32, V, V, V]
        L.pf_recommend_collab.argtypes = [V, V, I32, I32, I32, V, V, V]
        L.pf_recommend_clubs.argtypes = [V, V, I32, I32, I32, V, V, V]
        L.pf_fof_candidates.argtypes = [V, I32, I32, I32, V, I32, ctypes.POINTER(I32)]
        for fn in ("pf_recommend_interest_async", "pf_recommend_collab_async", "pf_recommend_clubs_async"):
            getattr(L, fn).argtypes = [V, V, I32, I32, I32, V, V, V, ctypes.POINTER(ctypes.c_uint64)]
        L.pf_wait.argtypes = [V, ctypes.c_uint64]
        L.pf_completed_ticket.argtypes = [V]
        L.pf_completed_ticket.restype = ctypes.c_uint64
        L.pf_set_adj.argtypes = [V, I32, V, I32]
        L.pf_set_shard.argtypes = [V, I32, I32]
        L.pf_set_scan_kernel.argtypes = [V, I32]
        L.pf_scan_keys_async.argtypes = [V, V, I32, I32, V, V]
        L.pf_merge_keys_async.argtypes = [V, V, I32, I32, I32, V, V]
        L.pf_decode_keys.argtypes = [V, I32, V, V, V]
        L.pf_decode_keys.restype = None
        L.pf_layout.argtypes = [V, ctypes.POINTER(PfLayoutStats)]
        L.pf_last_scan_ms.argtypes = [V]
        L.pf_last_scan_ms.restype = ctypes.c_float
        L.pf_profile_reset.argtypes = [V]
        L.pf_profile_sample.argtypes = [V, I32]
        L.pf_profile_read.argtypes = [V, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(I64)]
        L.pf_scan_bytes.argtypes = [V, V, I32, V]
        L.pf_jobs_stats_reset.argtypes = [V, I32]
        L.pf_jobs_stats_read.argtypes = [V, ctypes.POINTER(PfJobsStats)]
        L.pf_dataset_load.argtypes = [ctypes.c_char_p, I64, ctypes.POINTER(V)]
        L.pf_dataset_load_cached.argtypes = [ctypes.c_char_p, I64, ctypes.c_char_p, ctypes.POINTER(I32), ctypes.POINTER(V)]
        L.pf_dataset_free.argtypes = [V]
        L.pf_dataset_free.restype = None
        L.pf_dataset_desc.argtypes = [V]
        L.pf_dataset_desc.restype = V
        L.pf_dataset_info_get.argtypes = [V, ctypes.POINTER(PfDatasetInfo)]
        L.pf_dataset_column.argtypes = [V, I32]
        L.pf_dataset_column.restype = ctypes.c_char_p
        L.pf_dataset_profile_order.argtypes = [V, V, I32, ctypes.POINTER(I32)]
        L.pf_dataset_adj_order.argtypes = [V, V, I32, ctypes.POINTER(I32)]
        L.pf_dataset_profile_json.argtypes = [V, I32, V, I64, ctypes.POINTER(I64)]
        L.pf_dataset_club_name.argtypes = [V, I32]
        L.pf_dataset_club_name.restype = ctypes.c_char_p
        L.pf_compute_normalizers.argtypes = [V, I32, I32, ctypes.c_char_p, V, V]
        L.pf_holdout_friends.argtypes = [V, V, I32, V, I32, ctypes.POINTER(I32)]
        L.pf_recommendation_tests.argtypes = [V, V, I32, I32, V]
        L.pf_eval_holdout_friends.argtypes = [V, V, I32, I32, I32, I32, V, I32, ctypes.POINTER(I32)]
        L.pf_eval_recommendation_tests.argtypes = [V, V, I32, I32, I32, I32, I32, V, V, I32, ctypes.POINTER(I32)]
        L.pf_holdout_friends_digest.argtypes = [V, V, I32, V, I32, ctypes.POINTER(I32)]
        L.pf_recommendation_tests_digest.argtypes = [V, V, I32, I32, V, I32, ctypes.POINTER(I32)]
        L.pf_eval_holdout_friends_digest.argtypes = [V, V, I32, I32, I32, I32, V, I32, ctypes.POINTER(I32)]
        L.pf_eval_recommendation_tests_digest.argtypes = [V, V, I32, I32, I32, I32, I32, V, I32, ctypes.POINTER(I32)]
        L.pf_eval_recommendation_tests_async.argtypes = [V, V, I32, I32, I32, I32, I32, V, V, I32, ctypes.POINTER(I32),
                                                         ctypes.POINTER(ctypes.c_uint64)]
        _lib = L
    return _lib


def _i32(a):
    return np.ascontiguousarray(np.atleast_1d(np.asarray(a)), dtype=np.int32)


class FasEngine:
    """One device context (pf_ctx) over an in-memory corpus (a pf_corpus_desc pointer)."""

    def __init__(self, desc_ptr, device=0):
        L = lib()
        self._L = L
        self.h = ctypes.c_void_p()
        # in-flight asynchronous calls by ticket: the C side writes their outputs into these arrays
        # whenever the queue drains (pf_wait, or any synchronous call), so the engine, not the
        # caller's handle, keeps them alive until a wait covers them or the engine closes
        self._inflight = {}
        rc = L.pf_open(desc_ptr, device, ctypes.byref(self.h))
        if rc != PF_OK:
            raise FasError(f"pf_open failed ({rc}): {L.pf_last_error(None).decode()}")

    def close(self):
        if getattr(self, "h", None):
            self._L.pf_close(self.h)  # drops never-waited calls without writing their outputs
            self.h = None
        getattr(self, "_inflight", {}).clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != PF_OK:
            raise FasError(f"{what} failed ({rc}): {self._L.pf_last_error(self.h).decode()}")

    @property
    def num_users(self):
        return self._L.pf_num_users(self.h)

    def idf(self, col, tid):
        return self._L.pf_idf(self.h, col, tid)

    def layout(self):
        s = PfLayoutStats()
        self._check(self._L.pf_layout(self.h, ctypes.byref(s)), "pf_layout")
        return s

    # -- profile_similarity (recommender_similarity.cpp:10-124), batched
    def fas_pairs(self, a_uid, b_uid):
        a, b = _i32(a_uid), _i32(b_uid)
        out = np.empty(len(a), np.float32)
        self._check(self._L.pf_fas_pairs(self.h, a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data),
                    "pf_fas_pairs")
        return out

    def _topk(self, fn, users, topk, *extra):
        q = _i32(users)
        k = max(int(topk), 0)
        ou = np.zeros(max(len(q) * k, 1), np.int32)
        os_ = np.zeros(max(len(q) * k, 1), np.float32)
        oc = np.zeros(max(len(q), 1), np.int32)
        self._check(getattr(self._L, fn)(self.h, q.ctypes.data, len(q), k, *extra, ou.ctypes.data,
                                         os_.ctypes.data, oc.ctypes.data), fn)
        self._prune_inflight()
        return [(ou[i * k:i * k + oc[i]].copy(), os_[i * k:i * k + oc[i]].copy()) for i in range(len(q))]

    # -- asynchronous calls (pokec_fas.h): the handle keeps the output arrays alive until wait()
    class Pending:
        def __init__(self, q, k, ou, os_, oc, ticket):
            self.q, self.k, self.ou, self.os, self.oc, self.ticket = q, k, ou, os_, oc, ticket

    def _topk_async(self, fn, users, topk, limit):
        q = _i32(users)
        k = max(int(topk), 0)
        ou = np.zeros(max(len(q) * k, 1), np.int32)
        os_ = np.zeros(max(len(q) * k, 1), np.float32)
        oc = np.zeros(max(len(q), 1), np.int32)
        t = ctypes.c_uint64()
        self._check(getattr(self._L, fn)(self.h, q.ctypes.data, len(q), k, limit, ou.ctypes.data, os_.ctypes.data,
                                         oc.ctypes.data, ctypes.byref(t)), fn)
        p = FasEngine.Pending(q, k, ou, os_, oc, t.value)
        self._inflight[p.ticket] = p
        return p

    def recommend_interest_async(self, users, topk, candidate_limit=10000):
        return self._topk_async("pf_recommend_interest_async", users, topk, candidate_limit)

    def recommend_collaborative_async(self, users, topk, candidate_limit=10000):
        return self._topk_async("pf_recommend_collab_async", users, topk, candidate_limit)

    def recommend_clubs_collab_async(self, users, topk, candidate_limit=10000):
        return self._topk_async("pf_recommend_clubs_async", users, topk, candidate_limit)

    def _prune_inflight(self):
        """Drop the output arrays of calls the engine has completed (a synchronous call completes
        every pending one first), so callers that never wait() do not keep them alive."""
        if self._inflight:
            done = int(self._L.pf_completed_ticket(self.h))
            for t in [t for t in self._inflight if t <= done]:
                del self._inflight[t]

    def wait(self, p):
        """Results of an asynchronous call (and of every earlier one), as the synchronous form's."""
        self._check(self._L.pf_wait(self.h, p.ticket), "pf_wait")
        for t in [t for t in self._inflight if t <= p.ticket]:  # pf_wait finished every call up to p
            del self._inflight[t]
        k = p.k
        return [(p.ou[i * k:i * k + p.oc[i]].copy(), p.os[i * k:i * k + p.oc[i]].copy()) for i in range(len(p.q))]

    # -- Recommender surface (include/recommender.h:24-35); batched over users
    def recommend_interest(self, users, topk, mode=PF_MODE_FOF, candidate_limit=10000):
        return self._topk("pf_recommend_interest", users, topk, mode, candidate_limit)

    def recommend_collaborative(self, users, topk, candidate_limit=10000):
        return self._topk("pf_recommend_collab", users, topk, candidate_limit)

    def recommend_clubs_collab(self, users, topk, candidate_limit=10000):
        return self._topk("pf_recommend_clubs", users, topk, candidate_limit)

    def recommend_graph_registration(self, users, topk, candidate_limit=10000):
        return self.recommend_interest(users, topk, PF_MODE_FOF, candidate_limit)

    recommend_by_interest = recommend_graph_registration
    recommend_friends_graph = recommend_graph_registration
    recommend_friends_by_interest = recommend_graph_registration
    recommend_friends_collab = recommend_collaborative

    def recommend_interest_all(self, users, topk):
        """All-candidates interest scan."""
        return self.recommend_interest(users, topk, PF_MODE_ALL, 0)

    def fof_candidates(self, uid, limit, flavour=PF_FOF_GRAPH):
        cap = max(int(limit), 1) + 1
        out = np.zeros(cap, np.int32)
        n = ctypes.c_int32()
        self._check(self._L.pf_fof_candidates(self.h, uid, limit, flavour, out.ctypes.data, cap, ctypes.byref(n)),
                    "pf_fof_candidates")
        return out[:min(n.value, cap)].copy()

    def set_adj(self, uid, nbrs):
        if nbrs is None:
            self._check(self._L.pf_set_adj(self.h, uid, None, -1), "pf_set_adj")
        else:
            a = _i32(nbrs) if len(nbrs) else np.zeros(1, np.int32)
            self._check(self._L.pf_set_adj(self.h, uid, a.ctypes.data, len(nbrs)), "pf_set_adj")

    def set_shard(self, shard, nshards):
        self._check(self._L.pf_set_shard(self.h, shard, nshards), "pf_set_shard")

    def set_scan_kernel(self, kind):
        """PF_SCAN_AUTO / PF_SCAN_STREAM (record walk, K1) / PF_SCAN_POSTINGS (K5)."""
        self._check(self._L.pf_set_scan_kernel(self.h, kind), "pf_set_scan_kernel")

    # -- device-resident scan for multi-GPU benches (device pointers and a hipStream_t
    #    handle as ints; stream 0 is the HIP null stream, exactly as given)
    def scan_keys_async(self, users, topk, d_keys_ptr, stream_ptr):
        q = _i32(users)
        self._check(self._L.pf_scan_keys_async(self.h, q.ctypes.data, len(q), topk, ctypes.c_void_p(d_keys_ptr),
                                               ctypes.c_void_p(stream_ptr)), "pf_scan_keys_async")

    def merge_keys_async(self, d_parts_ptr, nparts, nq, topk, d_out_ptr, stream_ptr):
        self._check(self._L.pf_merge_keys_async(self.h, ctypes.c_void_p(d_parts_ptr), nparts, nq, topk,
                                                ctypes.c_void_p(d_out_ptr), ctypes.c_void_p(stream_ptr)),
                    "pf_merge_keys_async")

    @property
    def last_scan_ms(self):
        return self._L.pf_last_scan_ms(self.h)

    def profile_reset(self):
        self._check(self._L.pf_profile_reset(self.h), "pf_profile_reset")

    def profile_sample(self, every):
        """Time only every `every`-th scan launch after profile_reset() (1 = all)."""
        self._check(self._L.pf_profile_sample(self.h, int(every)), "pf_profile_sample")

    def profile_read(self):
        """(summed scan-kernel device ms, launches) since profile_reset()."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._check(self._L.pf_profile_read(self.h, ctypes.byref(ms), ctypes.byref(n)), "pf_profile_read")
        return ms.value, n.value

    def jobs_stats_reset(self, time_pairs=True, count=True):
        """Start (or stop) the recommenders' job-pipeline statistics (pf_jobs_stats): pair-kernel
        timing events and/or the pair / byte counters."""
        self._check(self._L.pf_jobs_stats_reset(self.h, (1 if time_pairs else 0) | (2 if count else 0)),
                    "pf_jobs_stats_reset")

    def jobs_stats(self):
        s = PfJobsStats()
        self._check(self._L.pf_jobs_stats_read(self.h, ctypes.byref(s)), "pf_jobs_stats_read")
        return {k: getattr(s, k) for k, _ in PfJobsStats._fields_}

    def scan_bytes(self, uids):
        """Bytes the all-candidates scan kernel reads per query over this shard (pf_scan_bytes)."""
        q = np.ascontiguousarray(np.atleast_1d(uids), np.int32)
        out = np.zeros(len(q), np.int64)
        self._check(self._L.pf_scan_bytes(self.h, q.ctypes.data, len(q), out.ctypes.data), "pf_scan_bytes")
        return out


def decode_keys(keys):
    """Packed 64-bit keys (numpy uint64, one query) -> (uids, scores)."""
    keys = np.ascontiguousarray(keys, np.uint64)
    ou = np.zeros(len(keys), np.int32)
    os_ = np.zeros(len(keys), np.float32)
    n = ctypes.c_int32()
    lib().pf_decode_keys(keys.ctypes.data, len(keys), ou.ctypes.data, os_.ctypes.data, ctypes.byref(n))
    return ou[:n.value], os_[:n.value]


class Dataset:
    """The reference's start-up loaders over a data directory (pf_dataset_load): the
    corpus the engine opens on, plus the reference's own iteration orders.  Host only."""

    def __init__(self, root, max_lines=PF_LOAD_REFERENCE_CAP, cache=None):
        """cache: path of a binary cache of the parse (pf_dataset_load_cached); None = none.
        self.from_cache tells whether the cache served."""
        L = lib()
        self._L = L
        self.h = ctypes.c_void_p()
        fc = ctypes.c_int32(0)
        rc = L.pf_dataset_load_cached(os.fsencode(root), max_lines, os.fsencode(cache) if cache else None,
                                      ctypes.byref(fc), ctypes.byref(self.h))
        self.from_cache = bool(fc.value)
        if rc != PF_OK:
            raise FasError(f"pf_dataset_load failed ({rc}): {L.pf_last_error(None).decode()}")

    def close(self):
        if getattr(self, "h", None):
            self._L.pf_dataset_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def desc_ptr(self):
        return self._L.pf_dataset_desc(self.h)

    def info(self):
        s = PfDatasetInfo()
        self._L.pf_dataset_info_get(self.h, ctypes.byref(s))
        return s

    def columns(self):
        out, t = [], 0
        while True:
            c = self._L.pf_dataset_column(self.h, t)
            if c is None:
                return out
            out.append(c.decode())
            t += 1

    def _order(self, fn):
        n = ctypes.c_int32()
        fn(self.h, None, 0, ctypes.byref(n))
        out = np.empty(n.value, np.int32)
        fn(self.h, out.ctypes.data, n.value, ctypes.byref(n))
        return out

    def profile_order(self):
        return self._order(self._L.pf_dataset_profile_order)

    def adj_order(self):
        return self._order(self._L.pf_dataset_adj_order)

    def profile_json(self, uid):
        n = ctypes.c_int64()
        rc = self._L.pf_dataset_profile_json(self.h, uid, None, 0, ctypes.byref(n))
        if rc == PF_ENOTFOUND:
            return None
        buf = ctypes.create_string_buffer(n.value + 1)
        self._L.pf_dataset_profile_json(self.h, uid, buf, n.value + 1, ctypes.byref(n))
        return buf.value.decode()

    def club_name(self, cid):
        c = self._L.pf_dataset_club_name(self.h, cid)
        return None if c is None else c.decode()

    def compute_normalizers(self, sample_size, comps_per_user, save_csv=None):
        """compute_column_normalizers (+ save_column_normalizers when save_csv): (mean, sd)
        float arrays in pf_corpus_desc slot order (7 fields, then the text columns)."""
        K = 7 + len(self.columns())
        mean, sd = np.zeros(K, np.float32), np.zeros(K, np.float32)
        rc = self._L.pf_compute_normalizers(self.h, sample_size, comps_per_user,
                                            None if save_csv is None else os.fsencode(save_csv),
                                            mean.ctypes.data, sd.ctypes.data)
        if rc != PF_OK:
            raise FasError(f"pf_compute_normalizers failed ({rc}): {self._L.pf_last_error(None).decode()}")
        return mean, sd

    # -- hold-out drivers (A19); `eng` must be open on this dataset's desc
    def holdout_friends(self, eng, sample_size):
        cap = max(sample_size, 1)
        out = np.empty(cap, np.float64)
        n = ctypes.c_int32()
        rc = self._L.pf_holdout_friends(eng.h, self.h, sample_size, out.ctypes.data, cap, ctypes.byref(n))
        eng._check(rc, "pf_holdout_friends")
        return out[:n.value]

    def recommendation_tests(self, eng, sample_size, topk):
        out = np.zeros(5, np.float64)
        rc = self._L.pf_recommendation_tests(eng.h, self.h, sample_size, topk, out.ctypes.data)
        eng._check(rc, "pf_recommendation_tests")
        return out

    # -- batched, sharded drivers (F1, cfg 5): per-plan-entry results of this shard, NaN / -1 elsewhere
    def eval_holdout_friends(self, eng, sample_size, shard=0, nshards=1, batch=256):
        cap = max(int(sample_size), 1)
        out = np.full(cap, np.nan)
        n = ctypes.c_int32()
        rc = self._L.pf_eval_holdout_friends(eng.h, self.h, sample_size, shard, nshards, batch, out.ctypes.data, cap,
                                             ctypes.byref(n))
        eng._check(rc, "pf_eval_holdout_friends")
        return out[:n.value]

    def eval_recommendation_tests(self, eng, sample_size, topk, shard=0, nshards=1, batch=128):
        cap = max(int(sample_size), 1)
        hits = np.full((cap, 3), -1, np.int8)
        club = np.full((cap, 2), np.nan)
        n = ctypes.c_int32()
        rc = self._L.pf_eval_recommendation_tests(eng.h, self.h, sample_size, topk, shard, nshards, batch,
                                                  hits.ctypes.data, club.ctypes.data, cap, ctypes.byref(n))
        eng._check(rc, "pf_eval_recommendation_tests")
        return hits[:n.value], club[:n.value]


    class EvalPending:
        # ds: the Dataset the carried call's driver reads when it finishes (at pf_wait or the
        # engine's next job call), kept alive with the output arrays while the call is in flight
        def __init__(self, hits, club, n, ticket, ds):
            self.hits, self.club, self.n, self.ticket, self.ds = hits, club, n, ticket, ds

    def eval_recommendation_tests_async(self, eng, sample_size, topk, shard=0, nshards=1, batch=128):
        """pf_eval_recommendation_tests_async: returns at once with the last chunk on the device;
        eval_wait(eng, p) gives eval_recommendation_tests's (hits, club).  The engine keeps the output
        arrays and this Dataset alive until the call completes."""
        cap = max(int(sample_size), 1)
        hits = np.full((cap, 3), -1, np.int8)
        club = np.full((cap, 2), np.nan)
        n = ctypes.c_int32()
        t = ctypes.c_uint64()
        rc = self._L.pf_eval_recommendation_tests_async(eng.h, self.h, sample_size, topk, shard, nshards, batch,
                                                        hits.ctypes.data, club.ctypes.data, cap, ctypes.byref(n),
                                                        ctypes.byref(t))
        eng._check(rc, "pf_eval_recommendation_tests_async")
        p = Dataset.EvalPending(hits, club, n.value, t.value, self)
        eng._inflight[p.ticket] = p
        return p

    def eval_wait(self, eng, p):
        eng._check(self._L.pf_wait(eng.h, p.ticket), "pf_wait")
        eng._prune_inflight()
        return p.hits[:p.n], p.club[:p.n]

    # -- per-user result digests (pokec_io.h pf_result_digest): parity probes of the drivers
    def holdout_friends_digest(self, eng, sample_size):
        cap = max(int(sample_size), 1)
        out = np.zeros(cap, np.uint64)
        n = ctypes.c_int32()
        rc = self._L.pf_holdout_friends_digest(eng.h, self.h, sample_size, out.ctypes.data, cap, ctypes.byref(n))
        eng._check(rc, "pf_holdout_friends_digest")
        return out[:n.value]

    def recommendation_tests_digest(self, eng, sample_size, topk):
        cap = max(int(sample_size), 1)
        out = np.zeros((cap, 4), np.uint64)
        n = ctypes.c_int32()
        rc = self._L.pf_recommendation_tests_digest(eng.h, self.h, sample_size, topk, out.ctypes.data, cap,
                                                    ctypes.byref(n))
        eng._check(rc, "pf_recommendation_tests_digest")
        return out[:n.value]

    def eval_holdout_friends_digest(self, eng, sample_size, shard=0, nshards=1, batch=256):
        cap = max(int(sample_size), 1)
        out = np.zeros(cap, np.uint64)
        n = ctypes.c_int32()
        rc = self._L.pf_eval_holdout_friends_digest(eng.h, self.h, sample_size, shard, nshards, batch,
                                                    out.ctypes.data, cap, ctypes.byref(n))
        eng._check(rc, "pf_eval_holdout_friends_digest")
        return out[:n.value]

    def eval_recommendation_tests_digest(self, eng, sample_size, topk, shard=0, nshards=1, batch=128):
        cap = max(int(sample_size), 1)
        out = np.zeros((cap, 4), np.uint64)
        n = ctypes.c_int32()
        rc = self._L.pf_eval_recommendation_tests_digest(eng.h, self.h, sample_size, topk, shard, nshards, batch,
                                                         out.ctypes.data, cap, ctypes.byref(n))
        eng._check(rc, "pf_eval_recommendation_tests_digest")
        return out[:n.value]


def merge_shards(parts):
    """Entries of plan arrays filled by shards s = 0..n-1 (entry i belongs to shard i % n)."""
    parts = [np.asarray(p) for p in parts]
    out = parts[0].copy()
    for s, p in enumerate(parts):
        out[s::len(parts)] = p[s::len(parts)]
    return out


def rec_tests_summary(hits, club):
    """run_recommendation_tests_sample's five averages from per-user entries, summed in plan
    order exactly like recommendation_tests.cpp:130-169."""
    out = np.zeros(5, np.float64)
    n = len(hits)
    if n:
        for j in range(3):
            out[j] = float(int(np.sum(hits[:, j], dtype=np.int64))) / float(n)
    club = np.asarray(club, np.float64).reshape(-1, 2)
    has = ~np.isnan(club[:, 0])  # the users with clubs
    users = int(np.count_nonzero(has))
    if users:
        # np.add.accumulate adds left to right (the reference's sequential double sum in plan
        # order; np.sum's pairwise summation would round differently)
        out[3] = float(np.add.accumulate(club[has, 0])[-1]) / users
        out[4] = float(np.add.accumulate(club[has, 1])[-1]) / users
    return out
