"""The product's C++ loaders (include/pokec_io.h, pf_dataset.cpp) against the
reference: parsed corpora vs the test-side reader pinned to the reference's own parse
(test_oracle_golden.py), hash-map iteration orders vs order.txt from the reference,
normaliser bits vs norms.txt, and write_profile_json vs the reference api_cli
transcript.  Host only: no GPU needed."""
import ctypes
import gzip
import os
import tempfile

import numpy as np
import pytest

import pokec_testlib as tl


def desc_arrays(ptr):
    d = tl.PfCorpusDesc.from_address(ptr)
    n, T = d.n_users, d.n_cols

    def arr(p, ct, k):
        return np.ctypeslib.as_array((ct * k).from_address(p)).copy() if k else np.zeros(0)

    out = {"n": n, "T": T}
    for name in ["user_id", "public_flag", "completion", "gender", "age"]:
        out[name] = arr(getattr(d, name), ctypes.c_int32, n)
    out["region"] = arr(d.region, ctypes.c_int32, 3 * n)
    out["club_off"] = arr(d.club_off, ctypes.c_int64, n + 1)
    out["club_ids"] = arr(d.club_ids, ctypes.c_uint32, int(out["club_off"][-1]))
    out["friend_off"] = arr(d.friend_off, ctypes.c_int64, n + 1)
    out["friend_ids"] = arr(d.friend_ids, ctypes.c_uint32, int(out["friend_off"][-1]))
    out["tok_off"] = arr(d.tok_off, ctypes.c_int64, n * T + 1)
    nt = int(out["tok_off"][-1])
    out["tok_tid"] = arr(d.tok_tid, ctypes.c_int32, nt)
    out["tok_tf"] = arr(d.tok_tf, ctypes.c_int32, nt)
    out["n_adj"] = d.n_adj
    out["adj_uid"] = arr(d.adj_uid, ctypes.c_int32, d.n_adj)
    out["adj_off"] = arr(d.adj_off, ctypes.c_int64, d.n_adj + 1)
    out["adj_nbr"] = arr(d.adj_nbr, ctypes.c_int32, int(out["adj_off"][-1]))
    K = tl.NUM_FIXED + T
    out["norm_present"] = arr(d.norm_present, ctypes.c_uint8, K)
    out["norm_mean"] = arr(d.norm_mean, ctypes.c_float, K)
    out["norm_sd"] = arr(d.norm_sd, ctypes.c_float, K)
    out["idf_mode"] = d.idf_mode
    return out


@pytest.fixture(scope="module", params=["A", "B", "api"])
def loaded(request):
    name = request.param
    pf = tl.product()
    with tempfile.TemporaryDirectory() as d:
        tl.regen_reference_dir(name, d)
        ds = pf.Dataset(d)
        py = tl.read_reference_dir(d)
        yield name, ds, py


def test_loader_matches_reference_parse(loaded):
    name, ds, py = loaded
    a = desc_arrays(ds.desc_ptr())
    assert a["n"] == py.n_users and a["T"] == py.n_cols
    assert np.array_equal(a["user_id"], py.uid)
    for k, v in [("public_flag", py.pub), ("completion", py.comp), ("gender", py.gen), ("age", py.age),
                 ("region", py.region), ("club_off", py.club_off), ("club_ids", py.clubs),
                 ("friend_off", py.friend_off), ("friend_ids", py.friends), ("tok_off", py.tok_off),
                 ("tok_tid", py.tok_tid), ("tok_tf", py.tok_tf)]:
        assert np.array_equal(a[k], v), k
    assert a["idf_mode"] == tl.PF_IDF_FROM_PROFILES
    # adjacency: same rows (row order is the map's, compared as a dict)
    mine = {int(u): list(a["adj_nbr"][a["adj_off"][i]:a["adj_off"][i + 1]]) for i, u in enumerate(a["adj_uid"])}
    ref = {int(u): list(py.adj_nbr[py.adj_off[i]:py.adj_off[i + 1]]) for i, u in enumerate(py.adj_uid)}
    assert mine == ref
    info = ds.info()
    assert info.n_profiles == py.n_users and info.median_age == py.median
    assert ds.columns() == py.col_names


def test_loader_normalisers_match_reference_bits(loaded):
    name, ds, py = loaded
    a = desc_arrays(ds.desc_ptr())
    if name == "api":
        pytest.skip("no norms fixture for the api corpus")
    rows = [ln.split() for ln in tl.fixture_lines(name, "norms.txt")]
    keys = tl.FIXED_KEYS + ds.columns()
    got = {keys[k]: (int(a["norm_mean"][k].view(np.uint32)), int(a["norm_sd"][k].view(np.uint32)))
           for k in range(len(keys)) if a["norm_present"][k]}
    ref = {r[0]: (int(r[1], 16), int(r[2], 16)) for r in rows}
    assert got == ref


def test_loader_iteration_orders_match_reference(loaded):
    name, ds, py = loaded
    if name == "api":
        pytest.skip("no order fixture for the api corpus")
    lines = tl.fixture_lines(name, "order.txt")
    prof = [int(x) for x in lines[0].split()[1:]]
    adj = [int(x) for x in lines[1].split()[1:]]
    assert list(ds.profile_order()) == prof
    assert list(ds.adj_order()) == adj


def test_profile_json_matches_reference_api_cli():
    pf = tl.product()
    m = tl.manifest()["api_cli"]
    with gzip.open(os.path.join(tl.GOLDEN, "api", "transcript_stdout.txt.gz"), "rt") as f:
        out = [ln.rstrip("\n") for ln in f]
    with tempfile.TemporaryDirectory() as d:
        tl.regen_reference_dir("api", d)
        ds = pf.Dataset(d, int(m["load_users"]))
        profile_lines = [ln for ln in out if ln.startswith('{"profile":')]
        assert len(profile_lines) == len(m["uids"])
        for uid, ln in zip(m["uids"], profile_lines):
            pj = ds.profile_json(uid)
            assert ln.startswith('{"profile":' + pj + ',"recommendations":'), uid
        assert ds.profile_json(999999999) is None
        info = ds.info()
        assert info.lines_read == 10000 and info.median_loaded == 1


def test_loader_line_cap_and_edge_rows():
    """max_lines counts data lines like user_loader.cpp:34 (empty and uid-0 lines included);
    duplicate uids replace the earlier row; a missing directory fails loudly."""
    pf = tl.product()
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "config"))
        os.makedirs(os.path.join(d, "data"))
        with open(os.path.join(d, "config", "text_columns.txt"), "w") as f:
            f.write("about\n\nhobby\n")
        rows = ["uid,pub,comp,gen,region,age,clubs,friends,about,hobby",
                '5,1,40,0,"1;;3",30,7;8;;7,9;10,"2:1;2:5;3:2",',
                "",
                "0,1,1,1,,1,,,,",
                "6,,,,,0,,,1:1;x;4:0,9:2;",
                '5,0,50,1,";2",0,,,"7:7",1:1',
                "7,1,1,1,1;2;3;4,20,1,2,,"]
        with open(os.path.join(d, "data", "users_encoded.csv"), "w") as f:
            f.write("\n".join(rows) + "\n")
        with open(os.path.join(d, "data", "adjacency.csv"), "w") as f:
            f.write("5, 6 ,7\n6\n\n5,9\n 7 , ,5\n")
        ds = pf.Dataset(d)
        py = tl.read_reference_dir(d)
        a = desc_arrays(ds.desc_ptr())
        assert np.array_equal(a["user_id"], py.uid) and list(a["user_id"]) == [5, 6, 7]
        for k, v in [("age", py.age), ("region", py.region), ("club_ids", py.clubs), ("tok_tid", py.tok_tid),
                     ("tok_tf", py.tok_tf), ("tok_off", py.tok_off), ("public_flag", py.pub)]:
            assert np.array_equal(a[k], v), k
        assert ds.info().median_age == 20 and ds.info().median_loaded == 0
        mine = {int(u): list(a["adj_nbr"][a["adj_off"][i]:a["adj_off"][i + 1]]) for i, u in enumerate(a["adj_uid"])}
        assert mine == {5: [6, 7, 9], 7: [5]}
        capped = pf.Dataset(d, 3)  # lines: row 5, empty, uid 0
        assert list(desc_arrays(capped.desc_ptr())["user_id"]) == [5] and capped.info().lines_read == 3
    with pytest.raises(pf.FasError):
        pf.Dataset("/nonexistent/dir")


@pytest.mark.parametrize("name", ["A", "B"])
def test_compute_normalizers_matches_reference(name):
    """compute_column_normalizers + save_column_normalizers (A18, the kurs path when
    data/column_normalizers.csv is missing): float bits and the saved CSV text equal the
    reference's (oracle/ref_norms.cpp goldens)."""
    pf = tl.product()
    sample, comps = tl.manifest()["norm_runs"][name]
    ref_bits = {r.split()[0]: (int(r.split()[1], 16), int(r.split()[2], 16))
                for r in tl.fixture_lines(name, "norms_computed_bits.txt")}
    ref_csv = tl.fixture_lines(name, "norms_computed_csv.txt")
    with tempfile.TemporaryDirectory() as d:
        tl.regen_reference_dir(name, d)
        ds = pf.Dataset(d)
        out = os.path.join(d, "saved.csv")
        mean, sd = ds.compute_normalizers(sample, comps, out)
        with open(out) as f:
            got_csv = [ln.rstrip("\n") for ln in f]
    keys = tl.FIXED_KEYS + ds.columns()
    got = {keys[k]: (int(mean[k].view(np.uint32)), int(sd[k].view(np.uint32))) for k in range(len(keys))}
    assert got == ref_bits
    assert got_csv == ref_csv


def test_parallel_ingest_equals_one_thread():
    """F2: the threaded loaders (line split, parse on threads, ordered insert) give the
    same corpus arrays and the same hash-container iteration orders as one thread, on a
    corpus large enough for many parse chunks (edge-case rows included)."""
    pf = tl.product()
    c = tl.synth.Corpus(n_users=30000, seed=11, edge_cases=1)
    with tempfile.TemporaryDirectory() as d:
        c.write_reference_files(d)
        c.close()
        out = {}
        old = os.environ.get("PF_DEBUG")
        try:
            for th in ("1", "7"):
                os.environ["PF_DEBUG"] = f"load_threads={th}"
                ds = pf.Dataset(d, -1)
                out[th] = (desc_arrays(ds.desc_ptr()), list(ds.profile_order()), list(ds.adj_order()))
                ds.close()
        finally:
            if old is None:
                os.environ.pop("PF_DEBUG", None)
            else:
                os.environ["PF_DEBUG"] = old
    a1, p1, j1 = out["1"]
    a7, p7, j7 = out["7"]
    assert a1["n"] == a7["n"] > 20000
    for k in a1:
        assert np.array_equal(np.asarray(a1[k]), np.asarray(a7[k])), k
    assert p1 == p7 and j1 == j7


def test_ingest_last_line_without_newline_and_cr():
    """std::getline semantics: a last line without '\\n' is a line; a '\\r' stays in the line
    and stops atoi like any other non-digit."""
    pf = tl.product()
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "config"))
        os.makedirs(os.path.join(d, "data"))
        with open(os.path.join(d, "config", "text_columns.txt"), "w") as f:
            f.write("about\n")
        with open(os.path.join(d, "data", "users_encoded.csv"), "w", newline="") as f:
            f.write("uid,pub,comp,gen,region,age,clubs,friends,about\r\n"
                    "3,1,40,0,1;2;3,30,7,9,2:1\r\n"
                    "4,0,50,1,,25,,3,5:2")
        with open(os.path.join(d, "data", "adjacency.csv"), "w", newline="") as f:
            f.write("3,4\r\n4,3")
        ds = pf.Dataset(d)
        a = desc_arrays(ds.desc_ptr())
        assert list(a["user_id"]) == [3, 4] and ds.info().lines_read == 2
        assert list(a["tok_tid"]) == [2, 5] and list(a["tok_tf"]) == [1, 2]
        mine = {int(u): list(a["adj_nbr"][a["adj_off"][i]:a["adj_off"][i + 1]]) for i, u in enumerate(a["adj_uid"])}
        assert mine == {3: [4], 4: [3]}


def _snapshot(ds):
    uids = list(ds.profile_order())
    js = []
    for u in uids[:50] + uids[-50:]:
        js.append(ds.profile_json(u))
    info = ds.info()
    return (desc_arrays(ds.desc_ptr()), uids, list(ds.adj_order()), js,
            (info.lines_read, info.n_profiles, info.n_adj, info.median_age, info.ages_replaced))


def _same(x, y):
    a, b = x[0], y[0]
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
    assert x[1:] == y[1:]


def test_binary_cache_equals_csv_parse():
    """F2 cache: a load served by the binary cache equals the CSV parse (corpus arrays,
    profiles / adj_list iteration orders, profile JSON, info); a changed CSV or a damaged
    cache file falls back to the parse and rewrites the cache."""
    pf = tl.product()
    c = tl.synth.Corpus(n_users=6000, seed=12, edge_cases=1)
    with tempfile.TemporaryDirectory() as d:
        c.write_reference_files(d)
        c.close()
        cache = os.path.join(d, "parse.bin")
        for cap in (-1, 2500):
            if os.path.exists(cache):
                os.remove(cache)
            plain = pf.Dataset(d, cap)
            ref = _snapshot(plain)
            plain.close()
            first = pf.Dataset(d, cap, cache=cache)
            assert not first.from_cache and os.path.exists(cache)
            _same(_snapshot(first), ref)
            first.close()
            hit = pf.Dataset(d, cap, cache=cache)
            assert hit.from_cache
            _same(_snapshot(hit), ref)
            hit.close()
        # the key holds the line cap: another cap re-parses
        other = pf.Dataset(d, 100, cache=cache)
        assert not other.from_cache and other.info().lines_read == 100
        other.close()
        # damaged cache: truncated -> parse again, then served again
        with open(cache, "r+b") as f:
            f.truncate(os.path.getsize(cache) // 2)
        again = pf.Dataset(d, 100, cache=cache)
        assert not again.from_cache
        again.close()
        assert pf.Dataset(d, 100, cache=cache).from_cache
        # a changed adjacency file (size / mtime) is a stale key
        with open(os.path.join(d, "data", "adjacency.csv"), "a") as f:
            f.write("1,2\n")
        stale = pf.Dataset(d, 100, cache=cache)
        assert not stale.from_cache
        fresh = pf.Dataset(d, 100)
        _same(_snapshot(stale), _snapshot(fresh))
