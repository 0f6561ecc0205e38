// ref_fixture — golden-vector generator that runs the REAL reference.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile against
// /root/reference/include + oracle/_ref/libref.a (the reference compiled from
// its own sources), run only in the build container by oracle/gen_golden.py.
// Its outputs are committed as small fixtures under tests/golden/; neither this
// program nor the reference ever reach the GPU box or the product library.
//
// Start-up mirrors api_cli (src/api_cli.cpp:86-167) so the fixtures describe
// exactly what the reference's own CLI would compute on the same data/ dir.
//
// usage: ref_fixture <workdir-with-data-and-config> <outdir> <npairs> <seed>
//                    <holdout_samples> <rectest_samples> [<digest_holdout> <digest_rectest>]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>
#include <algorithm>
#include <random>
#include <unordered_map>
#include <unordered_set>
#include <unistd.h>

#include "graph_builder.h"
#include "recommender.h"
#include "user_profile.h"
#include "user_loader.h"
#include "utils.h"
#include "test.h"
#include "recommendation_tests.h"

#include "pokec_io.h"  // pf_result_digest (the engine's parity-probe hash; plain C, no engine code)

static uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

static void dump_list(FILE* f, const char* tag, int uid, int a, int b,
                      const std::vector<std::pair<int, float>>& v) {
    fprintf(f, "%s %d %d %d %zu", tag, uid, a, b, v.size());
    for (auto& p : v) fprintf(f, " %d:%08x", p.first, fbits(p.second));
    fprintf(f, "\n");
}

int main(int argc, char** argv) {
    if (argc < 7) { fprintf(stderr, "usage: ref_fixture work out npairs seed holdout rectest\n"); return 2; }
    std::string work = argv[1], out = argv[2];
    int npairs = atoi(argv[3]);
    unsigned seed = (unsigned)atoi(argv[4]);
    int holdout_n = atoi(argv[5]), rectest_n = atoi(argv[6]);
    const int digest_holdout = argc > 7 ? atoi(argv[7]) : 0, digest_rectest = argc > 8 ? atoi(argv[8]) : 0;
    if (chdir(work.c_str()) != 0) { perror("chdir"); return 1; }

    // ---- api_cli start-up (api_cli.cpp:93-167), minus vocab/lemmatiser ----
    std::vector<std::string> cols = load_text_columns_from_file("config/text_columns.txt");
    GraphBuilder gb;
    if (!gb.load_serialized("data/adjacency.csv")) { fprintf(stderr, "no adjacency\n"); return 1; }
    std::unordered_map<int, std::vector<int>> adj = build_adj_list(gb.adjacency);
    std::unordered_map<int, UserProfile> profiles;
    // the loader prints progress lines to stdout; keep them out of our files
    if (!load_users_encoded("data/users_encoded.csv", cols, profiles, 0)) { fprintf(stderr, "no users\n"); return 1; }
    int median = 0;
    if (!load_median_age("data/median_age.txt", median)) median = compute_median_age_from_profiles(profiles);
    fill_missing_ages(profiles, median);
    std::unordered_map<std::string, std::pair<float, float>> norms;
    load_column_normalizers("data/column_normalizers.csv", norms);
    Recommender rec(&profiles, &adj);
    rec.set_field_normalizers(norms);
    rec.set_column_normalizers(norms);
    rec.compute_idf_from_profiles(cols);
    rec.set_text_columns(cols);

    std::vector<int> uids;
    for (auto& kv : profiles) uids.push_back(kv.first);
    std::vector<int> order = uids;                      // unordered_map iteration order
    std::sort(uids.begin(), uids.end());

    auto open = [&](const char* name) {
        std::string p = out + "/" + name;
        FILE* f = fopen(p.c_str(), "w");
        if (!f) { perror(p.c_str()); exit(1); }
        return f;
    };

    // ---- parsed corpus (A2/A3/A17 loader parity) ----
    FILE* f = open("profiles.txt");
    fprintf(f, "# uid public completion gender age r0 r1 r2 | clubs | friends | t:tid:tf (sorted)\n");
    fprintf(f, "median %d\n", median);
    for (int u : uids) {
        const UserProfile& p = profiles.at(u);
        fprintf(f, "%d %d %d %d %d %d %d %d |", p.user_id, p.public_flag, p.completion_percentage,
                p.gender, p.age, p.region_parts[0], p.region_parts[1], p.region_parts[2]);
        for (auto c : p.clubs) fprintf(f, " %u", c);
        fprintf(f, " |");
        for (auto c : p.friends) fprintf(f, " %u", c);
        fprintf(f, " |");
        for (size_t t = 0; t < p.token_cols.size(); ++t) {
            std::vector<std::pair<int, int>> v(p.token_cols[t].begin(), p.token_cols[t].end());
            std::sort(v.begin(), v.end());
            for (auto& kv : v) fprintf(f, " %zu:%d:%d", t, kv.first, kv.second);
        }
        fprintf(f, "\n");
    }
    fclose(f);
    f = open("order.txt");  // profiles / adj iteration order (hash order drives the hold-out drivers)
    fprintf(f, "profiles");
    for (int u : order) fprintf(f, " %d", u);
    fprintf(f, "\nadj");
    for (auto& kv : adj) fprintf(f, " %d", kv.first);
    fprintf(f, "\n");
    fclose(f);
    f = open("adj.txt");
    {
        std::vector<int> keys;
        for (auto& kv : adj) keys.push_back(kv.first);
        std::sort(keys.begin(), keys.end());
        for (int k : keys) {
            fprintf(f, "%d %zu", k, adj.at(k).size());
            for (int v : adj.at(k)) fprintf(f, " %d", v);
            fprintf(f, "\n");
        }
    }
    fclose(f);
    f = open("norms.txt");
    {
        std::vector<std::string> keys;
        for (auto& kv : norms) keys.push_back(kv.first);
        std::sort(keys.begin(), keys.end());
        for (auto& k : keys) fprintf(f, "%s %08x %08x\n", k.c_str(), fbits(norms[k].first), fbits(norms[k].second));
    }
    fclose(f);

    // ---- A4 IDF (float32 logf) ----
    f = open("idf.txt");
    fprintf(f, "N %zu\n", profiles.size());
    for (size_t t = 0; t < cols.size(); ++t) {
        auto it = rec.idf_per_col.find(cols[t]);
        if (it == rec.idf_per_col.end()) continue;
        std::vector<std::pair<int, float>> v(it->second.begin(), it->second.end());
        std::sort(v.begin(), v.end());
        for (auto& kv : v) fprintf(f, "%zu %d %08x\n", t, kv.first, fbits(kv.second));
    }
    fclose(f);

    // ---- A10 FAS pairs ----
    f = open("pairs.txt");
    std::mt19937 rng(seed);
    std::uniform_int_distribution<size_t> pick(0, uids.size() - 1);
    for (int i = 0; i < npairs; ++i) {
        int a = uids[pick(rng)], b = uids[pick(rng)];
        if (i % 97 == 0) b = a;  // self pairs
        float s = rec.profile_similarity(profiles.at(a), profiles.at(b));
        fprintf(f, "%d %d %08x\n", a, b, fbits(s));
    }
    // friend pairs (shared-friend overlaps are rare for random pairs)
    for (size_t i = 0; i < uids.size() && i < 4000; i += 3) {
        int a = uids[i];
        auto it = adj.find(a);
        if (it == adj.end()) continue;
        for (size_t k = 0; k < it->second.size() && k < 4; ++k) {
            int b = it->second[k];
            auto pb = profiles.find(b);
            if (pb == profiles.end()) continue;
            fprintf(f, "%d %d %08x\n", a, b, fbits(rec.profile_similarity(profiles.at(a), pb->second)));
        }
    }
    fclose(f);

    // ---- query set ----
    std::vector<int> queries;
    for (size_t i = 0; i < uids.size(); i += std::max<size_t>(1, uids.size() / 60)) queries.push_back(uids[i]);
    int hub = -1; size_t hubdeg = 0;
    for (auto& kv : adj) if (profiles.count(kv.first) && kv.second.size() > hubdeg) { hubdeg = kv.second.size(); hub = kv.first; }
    if (hub >= 0) queries.push_back(hub);
    queries.push_back(uids.front());
    queries.push_back(-5);                 // unknown user
    queries.push_back(uids.back() + 1000); // unknown user
    for (int u : uids) if (!adj.count(u)) { queries.push_back(u); break; }  // no adjacency row

    // ---- A12/A14/A15 recommenders as api_cli calls them (topk 20, limit 5000) + limits ----
    f = open("recs.txt");
    const int big = 1 << 30;
    for (int u : queries) {
        dump_list(f, "graph", u, 20, 5000, rec.recommend_graph_registration(u, 20, 5000));
        dump_list(f, "collab", u, 20, 5000, rec.recommend_collaborative(u, 20, 5000));
        dump_list(f, "interest", u, 20, 5000, rec.recommend_by_interest(u, 20, 5000));
        dump_list(f, "clubs", u, 20, 5000, rec.recommend_clubs_collab(u, 20, 5000));
        dump_list(f, "graph", u, 10, 10000, rec.recommend_graph_registration(u, 10));
        // full candidate sets at small limits pin the 2-hop order (A11 / A14 gathers)
        const int lims[] = {0, 1, 2, 3, 7, 25, 100, 1000};
        for (int L : lims) {
            dump_list(f, "graph", u, big, L, rec.recommend_graph_registration(u, big, L));
            dump_list(f, "collab", u, big, L, rec.recommend_collaborative(u, big, L));
        }
        dump_list(f, "clubs", u, big, 25, rec.recommend_clubs_collab(u, big, 25));
    }
    fclose(f);

    // ---- A13 all-candidates interest (build-defined mode) ----
    f = open("all.txt");
    for (int u : queries) {
        auto itq = profiles.find(u);
        std::vector<std::pair<int, float>> v;
        if (itq != profiles.end()) {
            std::unordered_set<int> excl;
            auto ia = adj.find(u);
            if (ia != adj.end()) excl.insert(ia->second.begin(), ia->second.end());
            excl.insert(u);
            for (auto& kv : profiles) {
                if (excl.count(kv.first)) continue;
                v.emplace_back(kv.first, rec.profile_similarity(itq->second, kv.second));
            }
            std::sort(v.begin(), v.end(), [](const std::pair<int, float>& A, const std::pair<int, float>& B) {
                if (A.second == B.second) return A.first < B.first;
                return A.second > B.second;
            });
            if (v.size() > 50) v.resize(50);
        }
        dump_list(f, "all", u, 50, 0, v);
    }
    fclose(f);

    // ---- A7 / set_tfidf_index: an explicit idf map that omits columns (raw-count cosine,
    //      recommender_similarity.cpp:99-104 -> recommender.cpp:141-163), omits tokens (idf 1.0,
    //      recommender.cpp:78), holds one empty column map, and scales the rest ----
    {
        std::unordered_map<std::string, std::unordered_map<int, float>> em;
        for (size_t t = 0; t < cols.size(); ++t) {
            if (t % 7 == 1 || t == 4) continue;  // absent columns
            auto it = rec.idf_per_col.find(cols[t]);
            std::unordered_map<int, float> m;
            if (t != 10 && it != rec.idf_per_col.end())
                for (auto& kv : it->second) {
                    if (kv.first % 5 == 3) continue;  // absent tokens
                    m[kv.first] = kv.second * (t % 2 ? 1.5f : 0.75f);
                }
            em[cols[t]] = m;
        }
        Recommender rx(&profiles, &adj);
        rx.set_field_normalizers(norms);
        rx.set_column_normalizers(norms);
        rx.set_tfidf_index(em);
        rx.set_text_columns(cols);
        f = open("idf_explicit_map.txt");
        fprintf(f, "cols");
        for (size_t t = 0; t < cols.size(); ++t) if (em.count(cols[t])) fprintf(f, " %zu", t);
        fprintf(f, "\n");
        for (size_t t = 0; t < cols.size(); ++t) {
            auto it = em.find(cols[t]);
            if (it == em.end()) continue;
            std::vector<std::pair<int, float>> v(it->second.begin(), it->second.end());
            std::sort(v.begin(), v.end());
            for (auto& kv : v) fprintf(f, "%zu %d %08x\n", t, kv.first, fbits(kv.second));
        }
        fclose(f);
        f = open("idf_explicit_pairs.txt");
        std::mt19937 rx_rng(seed + 1);
        for (int i = 0; i < npairs / 3; ++i) {
            int a = uids[pick(rx_rng)], b = uids[pick(rx_rng)];
            fprintf(f, "%d %d %08x\n", a, b, fbits(rx.profile_similarity(profiles.at(a), profiles.at(b))));
        }
        fclose(f);
        f = open("idf_explicit_recs.txt");
        for (int u : queries) {
            dump_list(f, "collab", u, 20, 5000, rx.recommend_collaborative(u, 20, 5000));
            dump_list(f, "interest", u, 20, 5000, rx.recommend_by_interest(u, 20, 5000));
            dump_list(f, "clubs", u, 20, 5000, rx.recommend_clubs_collab(u, 20, 5000));
        }
        fclose(f);
        f = open("idf_explicit_all.txt");
        for (int u : queries) {
            auto itq = profiles.find(u);
            std::vector<std::pair<int, float>> v;
            if (itq != profiles.end()) {
                std::unordered_set<int> excl;
                auto ia = adj.find(u);
                if (ia != adj.end()) excl.insert(ia->second.begin(), ia->second.end());
                excl.insert(u);
                for (auto& kv : profiles) {
                    if (excl.count(kv.first)) continue;
                    v.emplace_back(kv.first, rx.profile_similarity(itq->second, kv.second));
                }
                std::sort(v.begin(), v.end(), [](const std::pair<int, float>& A, const std::pair<int, float>& B) {
                    if (A.second == B.second) return A.first < B.first;
                    return A.second > B.second;
                });
                if (v.size() > 50) v.resize(50);
            }
            dump_list(f, "all", u, 50, 0, v);
        }
        fclose(f);
    }

    // ---- A19 hold-out drivers ----
    if (holdout_n > 0) {
        std::string p = out + "/holdout_friends.txt";
        run_friends_holdout_test(profiles, adj, cols, rec, holdout_n, p);
    }
    if (rectest_n > 0) {
        std::unordered_map<int, std::string> names;
        RecommendTestMetrics m = run_recommendation_tests_sample(profiles, adj, names, rec, cols, rectest_n, 10);
        f = open("rectests.txt");
        fprintf(f, "%.17g %.17g %.17g %.17g %.17g\n", m.graph_hit_rate, m.collab_hit_rate, m.interest_hit_rate,
                m.avg_club_prec_at_k, m.avg_club_recall_at_k);
        fclose(f);
    }

    // ---- A19 per-user result digests: the two drivers' loops replayed over the real
    //      Recommender with the drivers' own construction and mutation sequence, each returned
    //      list hashed (pf_result_digest).  The drivers print only averages; these pin every
    //      list they produce under the edited adjacency (clubs included, whose precision the
    //      averages always report as 0).
    auto digest = [](const std::vector<std::pair<int, float>>& v) {
        std::vector<int32_t> ids;
        std::vector<float> sc;
        for (auto& p : v) { ids.push_back(p.first); sc.push_back(p.second); }
        return (unsigned long long)pf_result_digest(ids.data(), sc.data(), (int32_t)ids.size());
    };
    if (digest_holdout > 0) {  // test.cpp:20-89: one adj_mod, edits accumulate
        std::vector<int> cand;
        for (auto& kv : profiles) {
            auto it = adj.find(kv.first);
            if (it != adj.end() && (int)it->second.size() >= 20) cand.push_back(kv.first);
        }
        std::mt19937 rng(1234567);
        std::shuffle(cand.begin(), cand.end(), rng);
        std::unordered_map<int, std::vector<int>> adj_mod = adj;
        Recommender r2(&profiles, &adj_mod);
        r2.set_field_normalizers(rec.field_normalizers);
        r2.set_column_normalizers(rec.column_normalizers);
        r2.set_text_columns(cols);
        r2.set_tfidf_index(rec.idf_per_col);
        f = open("holdout_digest.txt");
        int taken = 0;
        for (int uid : cand) {
            if (taken >= digest_holdout) break;
            const std::vector<int>& fr = adj.at(uid);
            const int F = (int)fr.size();
            if (F < 2 || F / 5 <= 0) continue;
            const int hold = F / 5;
            std::vector<int> idx(F);
            for (int i = 0; i < F; ++i) idx[i] = i;
            std::shuffle(idx.begin(), idx.end(), rng);
            std::unordered_set<int> held;
            for (int i = 0; i < hold; ++i) held.insert(fr[idx[i]]);
            std::vector<int> kept;
            for (int x : fr) if (!held.count(x)) kept.push_back(x);
            adj_mod[uid] = std::move(kept);
            fprintf(f, "%d %016llx\n", uid, digest(r2.recommend_collaborative(uid, hold, 1000)));
            ++taken;
        }
        fclose(f);
    }
    if (digest_rectest > 0) {  // recommendation_tests.cpp:79-156: a fresh adj_mod and Recommender per user
        std::vector<int> all;
        for (auto& kv : profiles) all.push_back(kv.first);
        std::mt19937 rng(1234567);
        std::shuffle(all.begin(), all.end(), rng);
        f = open("rectests_digest.txt");
        int taken = 0;
        for (int uid : all) {
            if (taken >= digest_rectest) break;
            auto it = adj.find(uid);
            if (it == adj.end() || it->second.size() < 4) continue;
            const std::vector<int>& fr = it->second;
            const int hold = std::max(1, (int)fr.size() / 4);
            std::vector<int> idx(fr.size());
            for (size_t i = 0; i < fr.size(); ++i) idx[i] = (int)i;
            std::shuffle(idx.begin(), idx.end(), rng);
            std::unordered_set<int> held;
            for (int i = 0; i < hold; ++i) held.insert(fr[idx[i]]);
            std::unordered_map<int, std::vector<int>> adj_mod = adj;
            std::vector<int> kept;
            for (int x : fr) if (!held.count(x)) kept.push_back(x);
            adj_mod[uid] = kept;
            Recommender r3(&profiles, &adj_mod);
            r3.set_field_normalizers(rec.field_normalizers);
            r3.set_column_normalizers(rec.column_normalizers);
            r3.set_text_columns(cols);
            r3.set_tfidf_index(rec.idf_per_col);
            fprintf(f, "%d %016llx %016llx %016llx %016llx\n", uid, digest(r3.recommend_graph_registration(uid, 10, 5000)),
                    digest(r3.recommend_collaborative(uid, 10, 5000)), digest(r3.recommend_by_interest(uid, 10, 5000)),
                    digest(r3.recommend_clubs_collab(uid, 10, 5000)));
            ++taken;
        }
        fclose(f);
    }
    return 0;
}
