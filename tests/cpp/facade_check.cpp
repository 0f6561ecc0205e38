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
//   argv[2] (optional): an explicit idf map ("cols t..." then "t tid float-hex" lines, the
//   golden idf_explicit_map.txt format) given to set_tfidf_index instead of the computed IDF.
// Test infrastructure only (tests/test_gpu_parity.py::test_cpp_facade_*).
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <unordered_map>
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
