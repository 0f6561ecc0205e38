// facade_check.cpp — test driver for include/pokec/recommender.h (the C++ drop-in for
// the reference's Recommender), in drop-in mode: the program declares its own global
// ::UserProfile (the reference's include/user_profile.h:10-20 fields) and uses the
// reference's names, `Recommender rec(&profiles, &adj)`, unchanged.  Builds the
// reference-shaped maps (profiles, adj_list, one normaliser map) from a data directory
// through pokec_io.h, wires the Recommender exactly like api_cli.cpp:155-163 (or, with a
// second argument, like an explicit set_tfidf_index caller), and answers stdin queries:
//   "<graph|collab|interest|clubs|all> uid topk limit" -> "tag uid topk limit n id:hex ..."
//   "pair a b"                                          -> "pair a b hex"
//   "pair3 a b"   profile_similarity(A, B, text_columns) -> "pair3 a b hex"
//   "sync uid n1 n2 ..."  replaces adj_list[uid] and calls sync_adjacency -> "sync uid rc"
//   "edit uid n1 n2 ..."  replaces adj_list[uid] only (the facade reads adj_list live) -> "edit uid"
//   "holdout N"           test.cpp:13-89 replayed literally over this program's Recommender
//                         (one adj_mod, a Recommender built over it, rows edited between calls)
//                         -> "holdout n r..." (%.6f, test.cpp:96) and "holdout_digest d..."
//   "rectests N K"        recommendation_tests.cpp:68-169 replayed literally (a fresh adj_mod
//                         and Recommender per user) -> "rectests g c i p r" (%.17g) and
//                         "rectests_digest d..." (4 per user: graph, collab, interest, clubs)
//   argv[2] (optional): an explicit idf map ("cols t..." then "t tid float-hex" lines, the
//   golden idf_explicit_map.txt format) given to set_tfidf_index instead of the computed IDF.
// Test infrastructure only (tests/test_gpu_parity.py::test_cpp_facade_*).
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <random>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

// the caller's profile type, as the reference declares it (include/user_profile.h:10-20)
struct UserProfile {
    int user_id = -1;
    int public_flag = -1;
    int completion_percentage = -1;
    int gender = -1;
    int age = 0;
    std::vector<uint32_t> clubs;
    std::vector<uint32_t> friends;
    std::vector<std::unordered_map<int, int>> token_cols;
    std::array<int, 3> region_parts = {-1, -1, -1};
};

#define POKEC_DROP_IN
#include "pokec/recommender.h"
#include "pokec_io.h"

static unsigned bits(float f) {
    unsigned u;
    std::memcpy(&u, &f, 4);
    return u;
}

static unsigned long long digest(const Recommender::Ranked& r) {
    std::vector<int32_t> ids;
    std::vector<float> sc;
    for (auto& p : r) { ids.push_back(p.first); sc.push_back(p.second); }
    return (unsigned long long)pf_result_digest(ids.data(), sc.data(), (int32_t)ids.size());
}

// run_friends_holdout_test (test.cpp:13-105), the caller's side as the reference writes it:
// base_rec's settings copied into a Recommender over adj_mod, adj_mod[uid] edited, then
// recommend_collaborative; no sync call anywhere.
static void replay_holdout(const std::unordered_map<int, UserProfile>& profiles,
                           const std::unordered_map<int, std::vector<int>>& adj_list,
                           const std::vector<std::string>& text_columns, const Recommender& base_rec, int sample_size) {
    std::vector<int> candidates;
    for (auto& kv : profiles) {
        auto it = adj_list.find(kv.first);
        if (it != adj_list.end() && (int)it->second.size() >= 20) candidates.push_back(kv.first);
    }
    std::mt19937 rng(1234567);
    std::shuffle(candidates.begin(), candidates.end(), rng);
    std::unordered_map<int, std::vector<int>> adj_mod = adj_list;
    Recommender rec(&profiles, &adj_mod);
    rec.set_field_normalizers(base_rec.field_normalizers);
    rec.set_column_normalizers(base_rec.column_normalizers);
    rec.set_text_columns(text_columns);
    rec.set_tfidf_index(base_rec.idf_per_col);
    std::vector<double> results;
    std::vector<unsigned long long> dig;
    int taken = 0;
    for (int uid : candidates) {
        if (taken >= sample_size) break;
        const std::vector<int>& friends = adj_list.find(uid)->second;
        const int F = (int)friends.size();
        if (F < 2) continue;
        const int hold_k = F / 5;
        if (hold_k <= 0) continue;
        std::vector<int> idx(F);
        for (int i = 0; i < F; ++i) idx[i] = i;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::unordered_set<int> held;
        for (int i = 0; i < hold_k; ++i) held.insert(friends[idx[i]]);
        std::vector<int> newf;
        for (int f : friends)
            if (held.find(f) == held.end()) newf.push_back(f);
        adj_mod[uid] = std::move(newf);
        auto preds = rec.recommend_collaborative(uid, hold_k, 1000);
        int hits = 0;
        for (size_t i = 0; i < preds.size() && (int)i < hold_k; ++i)
            if (held.find(preds[i].first) != held.end()) ++hits;
        results.push_back((double)hits / (double)hold_k);
        dig.push_back(digest(preds));
        ++taken;
    }
    std::printf("holdout %zu", results.size());
    for (double v : results) std::printf(" %.6f", v);
    std::printf("\nholdout_digest");
    for (auto d : dig) std::printf(" %016llx", d);
    std::printf("\n");
}

// run_recommendation_tests_sample (recommendation_tests.cpp:68-169): per user a fresh adj_mod
// copy and a fresh Recommender over it, then the four recommenders at limit 5000
static void replay_rectests(const std::unordered_map<int, UserProfile>& profiles,
                            const std::unordered_map<int, std::vector<int>>& adj_list, Recommender& base_rec,
                            const std::vector<std::string>& text_columns, int sample_size, int topk) {
    std::vector<int> all;
    for (auto& kv : profiles) all.push_back(kv.first);
    std::mt19937 rng(1234567);
    std::shuffle(all.begin(), all.end(), rng);
    int taken = 0, hits_graph = 0, hits_collab = 0, hits_interest = 0, club_users = 0;
    double club_prec = 0.0, club_rec = 0.0;
    std::vector<unsigned long long> dig;
    for (int uid : all) {
        if (taken >= sample_size) break;
        auto itadj = adj_list.find(uid);
        if (itadj == adj_list.end()) continue;
        const auto& friends = itadj->second;
        if (friends.size() < 4) continue;
        int hold_k = std::max(1, (int)friends.size() / 4);
        std::vector<int> idx(friends.size());
        for (size_t i = 0; i < friends.size(); ++i) idx[i] = (int)i;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::unordered_set<int> held;
        for (int i = 0; i < hold_k; ++i) held.insert(friends[idx[i]]);
        std::unordered_map<int, std::vector<int>> adj_mod = adj_list;
        std::vector<int> newf;
        for (int f : friends)
            if (held.find(f) == held.end()) newf.push_back(f);
        adj_mod[uid] = newf;
        Recommender rec(&profiles, &adj_mod);
        rec.set_field_normalizers(base_rec.field_normalizers);
        rec.set_column_normalizers(base_rec.column_normalizers);
        rec.set_text_columns(text_columns);
        rec.set_tfidf_index(base_rec.idf_per_col);
        auto any = [&](const Recommender::Ranked& r) {
            for (auto& p : r)
                if (held.find(p.first) != held.end()) return true;
            return false;
        };
        auto out_g = rec.recommend_graph_registration(uid, topk, 5000);
        auto out_c = rec.recommend_collaborative(uid, topk, 5000);
        auto out_i = rec.recommend_by_interest(uid, topk, 5000);
        auto club_pred = rec.recommend_clubs_collab(uid, topk, 5000);
        hits_graph += any(out_g);
        hits_collab += any(out_c);
        hits_interest += any(out_i);
        std::unordered_set<int> actual;
        for (auto c : profiles.at(uid).clubs) actual.insert((int)c);
        if (!actual.empty()) {
            int hit = 0;
            for (size_t i = 0; i < club_pred.size() && i < (size_t)topk; ++i)
                if (actual.find(club_pred[i].first) != actual.end()) ++hit;
            club_prec += (double)hit / (double)topk;
            club_rec += (double)hit / (double)actual.size();
            ++club_users;
        }
        for (auto* r : {&out_g, &out_c, &out_i, &club_pred}) dig.push_back(digest(*r));
        ++taken;
    }
    double m[5] = {0, 0, 0, 0, 0};
    if (taken > 0) {
        m[0] = (double)hits_graph / (double)taken;
        m[1] = (double)hits_collab / (double)taken;
        m[2] = (double)hits_interest / (double)taken;
    }
    if (club_users > 0) {
        m[3] = club_prec / (double)club_users;
        m[4] = club_rec / (double)club_users;
    }
    std::printf("rectests %.17g %.17g %.17g %.17g %.17g\nrectests_digest", m[0], m[1], m[2], m[3], m[4]);
    for (auto d : dig) std::printf(" %016llx", d);
    std::printf("\n");
}

int main(int argc, char** argv) {
    if (argc < 2) { std::cerr << "usage: facade_check <root>\n"; return 2; }
    pf_dataset* ds = nullptr;
    if (pf_dataset_load(argv[1], PF_LOAD_REFERENCE_CAP, &ds) != PF_OK) { std::cerr << pf_last_error(nullptr) << "\n"; return 1; }
    const pf_corpus_desc* d = pf_dataset_desc(ds);
    const int T = d->n_cols;
    std::vector<std::string> cols;
    for (int t = 0; t < T; ++t) cols.push_back(pf_dataset_column(ds, t));
    std::unordered_map<int, UserProfile> profiles;
    for (int i = 0; i < d->n_users; ++i) {
        UserProfile p;
        p.user_id = d->user_id[i]; p.public_flag = d->public_flag[i]; p.completion_percentage = d->completion[i];
        p.gender = d->gender[i]; p.age = d->age[i];
        for (int k = 0; k < 3; ++k) p.region_parts[k] = d->region[3 * i + k];
        p.clubs.assign(d->club_ids + d->club_off[i], d->club_ids + d->club_off[i + 1]);
        p.friends.assign(d->friend_ids + d->friend_off[i], d->friend_ids + d->friend_off[i + 1]);
        p.token_cols.resize(T);
        for (int t = 0; t < T; ++t)
            for (int64_t k = d->tok_off[(int64_t)i * T + t]; k < d->tok_off[(int64_t)i * T + t + 1]; ++k)
                p.token_cols[t][d->tok_tid[k]] = d->tok_tf[k];
        profiles[p.user_id] = std::move(p);
    }
    std::unordered_map<int, std::vector<int>> adj;
    for (int i = 0; i < d->n_adj; ++i) adj[d->adj_uid[i]].assign(d->adj_nbr + d->adj_off[i], d->adj_nbr + d->adj_off[i + 1]);
    std::unordered_map<std::string, std::pair<float, float>> norms;
    const char* keys[PF_NUM_FIXED] = {"public", "gender", "completion", "age", "region", "clubs", "friends"};
    for (int k = 0; k < PF_NUM_FIXED + T; ++k)
        if (d->norm_present[k]) norms[k < PF_NUM_FIXED ? keys[k] : cols[k - PF_NUM_FIXED]] = {d->norm_mean[k], d->norm_sd[k]};
    Recommender rec(&profiles, &adj);
    rec.set_field_normalizers(norms);
    rec.set_column_normalizers(norms);
    if (argc > 2) {  // set_tfidf_index with the explicit map (recommender.h:31)
        std::unordered_map<std::string, std::unordered_map<int, float>> em;
        std::ifstream in(argv[2]);
        std::string ln;
        std::getline(in, ln);
        std::istringstream hs(ln);
        std::string word;
        hs >> word;
        int t;
        while (hs >> t) em[cols[t]];
        while (std::getline(in, ln)) {
            std::istringstream ls(ln);
            int tid;
            std::string hex;
            ls >> t >> tid >> hex;
            const uint32_t u = (uint32_t)std::stoul(hex, nullptr, 16);
            float v;
            std::memcpy(&v, &u, 4);
            em[cols[t]][tid] = v;
        }
        rec.set_tfidf_index(em);
    } else {
        rec.compute_idf_from_profiles(cols);
    }
    rec.set_text_columns(cols);
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream iss(line);
        std::string tag;
        iss >> tag;
        if (tag == "pair") {
            int a, b;
            iss >> a >> b;
            std::printf("pair %d %d %08x\n", a, b, bits(rec.profile_similarity(profiles.at(a), profiles.at(b))));
            continue;
        }
        if (tag == "pair3") {
            int a, b;
            iss >> a >> b;
            std::printf("pair3 %d %d %08x\n", a, b, bits(rec.profile_similarity(profiles.at(a), profiles.at(b), cols)));
            continue;
        }
        if (tag == "holdout") {
            int n = 0;
            iss >> n;
            replay_holdout(profiles, adj, cols, rec, n);
            continue;
        }
        if (tag == "rectests") {
            int n = 0, k = 10;
            iss >> n >> k;
            replay_rectests(profiles, adj, rec, cols, n, k);
            continue;
        }
        if (tag == "edit") {
            int u, x;
            iss >> u;
            std::vector<int> row;
            while (iss >> x) row.push_back(x);
            adj[u] = row;
            std::printf("edit %d\n", u);
            continue;
        }
        if (tag == "sync") {
            int u, x;
            iss >> u;
            std::vector<int> row;
            while (iss >> x) row.push_back(x);
            adj[u] = row;
            std::printf("sync %d %d\n", u, rec.sync_adjacency(u));
            continue;
        }
        int uid, k, lim;
        iss >> uid >> k >> lim;
        Recommender::Ranked r;
        if (tag == "graph") r = rec.recommend_graph_registration(uid, k, lim);
        else if (tag == "collab") r = rec.recommend_collaborative(uid, k, lim);
        else if (tag == "interest") r = rec.recommend_by_interest(uid, k, lim);
        else if (tag == "clubs") r = rec.recommend_clubs_collab(uid, k, lim);
        else r = rec.recommend_interest_all(uid, k);
        std::printf("%s %d %d %d %zu", tag.c_str(), uid, k, lim, r.size());
        for (auto& pr : r) std::printf(" %d:%08x", pr.first, bits(pr.second));
        std::printf("\n");
    }
    if (!rec.last_error().empty()) std::cerr << rec.last_error() << "\n";
    pf_dataset_free(ds);
    return 0;
}
