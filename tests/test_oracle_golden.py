"""Pin the oracle (oracle/refcpu.cpp, a CPU restatement) against golden vectors
produced by the REAL reference (oracle/gen_golden.py).  CPU only."""
import numpy as np
import pytest

import pokec_testlib as tl


@pytest.fixture(scope="module", params=["A", "B"])
def gold(request):
    name = request.param
    corpus = tl.golden_corpus(name)
    return name, corpus, tl.Oracle(corpus)


def test_python_reader_matches_reference_parse(gold):
    name, corpus, _ = gold
    lines = tl.fixture_lines(name, "profiles.txt")
    assert int(lines[1].split()[1]) == corpus.median
    rows = [ln for ln in lines[2:]]
    idx = corpus.index()
    assert len(rows) == corpus.n_users
    T = corpus.n_cols
    for ln in rows:
        head, clubs, friends, toks = ln.split("|")
        h = [int(x) for x in head.split()]
        i = idx[h[0]]
        assert [corpus.pub[i], corpus.comp[i], corpus.gen[i], corpus.age[i]] == h[1:5]
        assert list(corpus.region[3 * i:3 * i + 3]) == h[5:8]
        assert list(corpus.clubs[corpus.club_off[i]:corpus.club_off[i + 1]]) == [int(x) for x in clubs.split()]
        assert list(corpus.friends[corpus.friend_off[i]:corpus.friend_off[i + 1]]) == [int(x) for x in friends.split()]
        mine = []
        for t in range(T):
            r = i * T + t
            lo, hi = corpus.tok_off[r], corpus.tok_off[r + 1]
            mine += sorted((t, int(a), int(b)) for a, b in zip(corpus.tok_tid[lo:hi], corpus.tok_tf[lo:hi]))
        ref = [tuple(int(v) for v in x.split(":")) for x in toks.split()]
        assert mine == ref


def test_oracle_idf(gold):
    name, corpus, orc = gold
    N, rows = tl.golden_idf(name)
    assert N == corpus.n_users
    got = np.array([np.float32(orc.idf(t, k)).view(np.uint32) for t, k, _ in rows], np.uint32)
    exp = np.array([h for _, _, h in rows], np.uint32)
    assert np.array_equal(got, exp)


def test_oracle_fas_pairs_bit_exact(gold):
    name, corpus, orc = gold
    a, b, s = tl.golden_pairs(name)
    got = orc.fas_pairs(a, b).view(np.uint32)
    assert np.array_equal(got, s), f"{np.count_nonzero(got != s)} of {len(s)} FAS floats differ"


def test_oracle_recommenders(gold):
    name, corpus, orc = gold
    g = tl.golden_lists(name, "recs.txt")
    for (tag, uid, k, lim), items in g.items():
        if tag in ("graph", "interest"):
            (ids, sc), = orc.interest([uid], min(k, 100000), tl.PF_MODE_FOF, lim)
        elif tag == "collab":
            (ids, sc), = orc.collab([uid], min(k, 100000), lim)
        else:
            (ids, sc), = orc.clubs([uid], min(k, 100000), lim)
        assert list(ids) == [x for x, _ in items], (tag, uid, k, lim)
        assert list(sc.view(np.uint32)) == [h for _, h in items], (tag, uid, k, lim)


def test_oracle_all_candidates(gold):
    name, corpus, orc = gold
    g = tl.golden_lists(name, "all.txt")
    for (tag, uid, k, lim), items in g.items():
        (ids, sc), = orc.interest([uid], k, tl.PF_MODE_ALL, 0)
        assert list(ids) == [x for x, _ in items]
        assert list(sc.view(np.uint32)) == [h for _, h in items]


def test_oracle_profile_iteration_order(gold):
    name, corpus, orc = gold
    ref = [int(x) for x in tl.fixture_lines(name, "order.txt")[0].split()[1:]]
    assert list(orc.profile_order()) == ref


def test_oracle_holdout_drivers():
    corpus = tl.golden_corpus("A")
    m = tl.manifest()["corpora"]["A"]
    orc = tl.Oracle(corpus)
    ref = [float(x) for x in tl.fixture_lines("A", "holdout_friends.txt")]
    got = orc.holdout_friends(m["holdout"])
    assert [f"{x:.6f}" for x in got] == [f"{x:.6f}" for x in ref]
    ref = [float(x) for x in tl.fixture_lines("A", "rectests.txt")[0].split()]
    got = orc.recommendation_tests(m["rectest"], 10)
    assert list(got) == ref


def test_oracle_driver_digests():
    """Every list the two drivers produce (test.cpp:49-89 collaborative under the cumulative
    edits; recommendation_tests.cpp:93-156 graph / collaborative / interest / clubs under each
    user's own edited row), hashed per user, equals the reference's (ref_fixture.cpp replays the
    drivers over the real Recommender)."""
    corpus = tl.golden_corpus("A")
    m = tl.manifest()["corpora"]["A"]
    orc = tl.Oracle(corpus)
    uids, ref = tl.golden_digests("A", "holdout_digest.txt")
    assert len(uids) == m["digest_holdout"]
    assert np.array_equal(orc.holdout_friends_digest(m["digest_holdout"]), ref)
    uids, ref = tl.golden_digests("A", "rectests_digest.txt")
    assert len(uids) == m["digest_rectest"]
    assert np.array_equal(orc.recommendation_tests_digest(m["digest_rectest"], 10), ref)


@pytest.mark.parametrize("name", ["A", "B"])
def test_oracle_explicit_idf(name):
    """A7 and set_tfidf_index: with an explicit idf map that omits columns (raw-count cosine,
    recommender.cpp:141-163), omits tokens (idf 1.0) and holds an empty map, the oracle's FAS
    pairs, all-candidates top-50 and recommenders equal the reference's."""
    c = tl.explicit_idf_corpus(name)
    orc = tl.Oracle(c)
    a, b, s = tl.golden_pairs_file(name, "idf_explicit_pairs.txt")
    got = orc.fas_pairs(a, b).view(np.uint32)
    assert np.array_equal(got, s), f"{np.count_nonzero(got != s)} of {len(s)} FAS floats differ"
    for (tag, uid, k, lim), items in tl.golden_lists(name, "idf_explicit_all.txt").items():
        (ids, sc), = orc.interest([uid], k, tl.PF_MODE_ALL, 0)
        assert list(ids) == [x for x, _ in items] and list(sc.view(np.uint32)) == [h for _, h in items], uid
    for (tag, uid, k, lim), items in tl.golden_lists(name, "idf_explicit_recs.txt").items():
        fn = {"collab": orc.collab, "clubs": orc.clubs}.get(tag)
        (ids, sc), = fn([uid], k, lim) if fn else orc.interest([uid], k, tl.PF_MODE_FOF, lim)
        assert list(ids) == [x for x, _ in items] and list(sc.view(np.uint32)) == [h for _, h in items], (tag, uid)
