// ref_norms — golden generator for compute_column_normalizers (src/utils.cpp:155-240)
// and save_column_normalizers (src/utils.cpp:144-153), running the REAL reference.
//
// TEST INFRASTRUCTURE ONLY (built by oracle/Makefile against oracle/_ref/libref.a, run
// by oracle/gen_golden.py in the build container; never shipped).  Start-up mirrors
// api_cli (src/api_cli.cpp:93-153) so the profiles map has the reference's iteration
// order, which the sampler depends on.
//
// usage: ref_norms <workdir-with-data-and-config> <out.csv> <out_bits.txt> <sample> <comps>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <unordered_map>
#include <vector>

#include "graph_builder.h"
#include "user_loader.h"
#include "user_profile.h"
#include "utils.h"

static unsigned fbits(float f) { unsigned u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
    if (argc < 6) { fprintf(stderr, "usage: ref_norms work out.csv out_bits.txt sample comps\n"); return 2; }
    std::string work = argv[1];
    std::string csv = argv[2], bits = argv[3];
    const int sample = atoi(argv[4]), comps = atoi(argv[5]);
    char cwd[4096];
    if (!getcwd(cwd, sizeof cwd)) return 1;
    if (csv[0] != '/') csv = std::string(cwd) + "/" + csv;
    if (bits[0] != '/') bits = std::string(cwd) + "/" + bits;
    if (chdir(work.c_str()) != 0) { perror("chdir"); return 1; }
    std::vector<std::string> cols = load_text_columns_from_file("config/text_columns.txt");
    std::unordered_map<int, UserProfile> profiles;
    if (!load_users_encoded("data/users_encoded.csv", cols, profiles, 0)) return 1;
    int median = 0;
    if (!load_median_age("data/median_age.txt", median)) median = compute_median_age_from_profiles(profiles);
    fill_missing_ages(profiles, median);
    auto m = compute_column_normalizers(profiles, cols, sample, comps);
    if (!save_column_normalizers(csv, m)) return 1;
    FILE* f = fopen(bits.c_str(), "w");
    std::vector<std::string> keys;
    for (auto& kv : m) keys.push_back(kv.first);
    std::sort(keys.begin(), keys.end());
    for (auto& k : keys) fprintf(f, "%s %08x %08x\n", k.c_str(), fbits(m[k].first), fbits(m[k].second));
    fclose(f);
    return 0;
}
