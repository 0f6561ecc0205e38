// ref_timing — SURVEY §8(c) C4-viii: times the REAL reference's all-candidates interest
// scoring, single thread, so the CPU baseline bench.py reports (oracle/refcpu.cpp, kind
// "port") can be calibrated against it on the same corpus and queries.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile against /root/reference/include +
// oracle/_ref/libref.a (the reference compiled from its own sources); run only in the build
// container by oracle/calibrate_cpu.py.  It never reaches the product library.
//
// Start-up is api_cli's (src/api_cli.cpp:93-167, minus vocab/lemmatiser).  Per query uid
// (argv[2..]) it scores every loaded profile c != q with c not in adj[q] through
// Recommender::profile_similarity (recommender_similarity.cpp:10-124), the exclusion and the
// (score desc, uid asc) sort + truncate of recommend_by_interest
// (recommender_graph.cpp:46-54,97-101): the build-defined all-candidates mode, SURVEY A13.
// Timed: scoring + top-k only (steady_clock), as D4 prescribes.
//
// usage: ref_timing <workdir-with-data-and-config> <uid>...
// stdout: one line per query "uid n_scored seconds id:score(hex) x10", then "total n s"
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>
#include <unistd.h>

#include "graph_builder.h"
#include "recommender.h"
#include "user_loader.h"
#include "user_profile.h"
#include "utils.h"

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: ref_timing work uid...\n"); return 2; }
    if (chdir(argv[1]) != 0) { perror("chdir"); return 1; }
    std::vector<std::string> cols = load_text_columns_from_file("config/text_columns.txt");
    GraphBuilder gb;
    if (!gb.load_serialized("data/adjacency.csv")) { fprintf(stderr, "no adjacency\n"); return 1; }
    std::unordered_map<int, std::vector<int>> adj = build_adj_list(gb.adjacency);
    std::unordered_map<int, UserProfile> profiles;
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

    double total_s = 0.0;
    long long total_n = 0;
    for (int a = 2; a < argc; ++a) {
        const int u = atoi(argv[a]);
        auto qi = profiles.find(u);
        if (qi == profiles.end()) { printf("%d 0 0\n", u); continue; }
        const auto t0 = std::chrono::steady_clock::now();
        std::unordered_set<int> skip;
        skip.insert(u);
        auto ai = adj.find(u);
        if (ai != adj.end()) skip.insert(ai->second.begin(), ai->second.end());
        std::vector<std::pair<int, float>> scored;
        scored.reserve(profiles.size());
        for (auto& kv : profiles) {
            if (skip.count(kv.first)) continue;
            scored.emplace_back(kv.first, rec.profile_similarity(qi->second, kv.second));
        }
        const size_t n = scored.size();
        std::sort(scored.begin(), scored.end(), [](const std::pair<int, float>& x, const std::pair<int, float>& y) {
            if (x.second != y.second) return x.second > y.second;
            return x.first < y.first;
        });
        if (scored.size() > 10) scored.resize(10);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        total_s += s;
        total_n += (long long)n;
        printf("%d %zu %.6f", u, n, s);
        for (auto& p : scored) {
            uint32_t b;
            std::memcpy(&b, &p.second, 4);
            printf(" %d:%08x", p.first, b);
        }
        printf("\n");
    }
    printf("total %lld %.6f\n", total_n, total_s);
    return 0;
}
