// api_cli.cpp — the reference's stdin/JSON front end (src/api_cli.cpp:86-258) over the
// MI355X engine.  Same files (cwd-relative data/ + config/), same stdout protocol:
// loader progress lines, READY, then one JSON line per input line.  The four
// recommenders run through the C ABI (pokec_fas.h); start-up uses pokec_io.h.
//
//   pokec_api_cli [load_users] [--root DIR] [--device N] [--no-cap] [--cache PATH]
//
// load_users is parsed and ignored exactly like the reference (the loader's cap is
// fixed at 100000 lines, user_loader.cpp:34); --no-cap lifts it for full corpora.
// Differences: no vocabulary/adjacency ETL when tokens.csv / adjacency.csv are missing
// (out of scope): a missing adjacency.csv is an error, a missing
// tokens.csv only drops club names.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "pokec_io.h"

namespace {

// api_cli.cpp:28-47
std::string json_escape(const std::string& s) {
    std::string out;
    for (char c : s) {
        switch (c) {
            case '\\': out += "\\\\"; break;
            case '"': out += "\\\""; break;
            case '\b': out += "\\b"; break;
            case '\f': out += "\\f"; break;
            case '\n': out += "\\n"; break;
            case '\r': out += "\\r"; break;
            case '\t': out += "\\t"; break;
            default:
                if ((unsigned char)c < 0x20) {
                    char buf[8];
                    snprintf(buf, sizeof(buf), "\\u%04x", (int)c);
                    out += buf;
                } else {
                    out += c;
                }
        }
    }
    return out;
}

struct List {
    std::vector<int32_t> id;
    std::vector<float> score;
    int32_t n = 0;
    explicit List(int k) : id(k), score(k) {}
};

void write_list(std::ostringstream& os, const char* name, const List& l, const pf_dataset* clubs) {
    os << "\"" << name << "\":[";
    for (int i = 0; i < l.n; ++i) {
        if (i) os << ",";
        os << "{\"id\":" << l.id[i] << ",\"score\":" << std::fixed << std::setprecision(6) << l.score[i];
        if (clubs) {
            const char* nm = pf_dataset_club_name(clubs, l.id[i]);
            if (nm) os << ",\"name\":\"" << json_escape(nm) << "\"";
        }
        os << "}";
    }
    os << "]";
}

}  // namespace

int main(int argc, char** argv) {
    std::ios::sync_with_stdio(true);
    std::cin.tie(nullptr);
    std::string root = ".";
    int device = 0;
    int64_t cap = PF_LOAD_REFERENCE_CAP;
    std::string cache;  // --cache PATH: binary cache of the CSV parse (F2), off by default
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--root" && i + 1 < argc) root = argv[++i];
        else if (a == "--device" && i + 1 < argc) device = atoi(argv[++i]);
        else if (a == "--no-cap") cap = 0;
        else if (a == "--cache" && i + 1 < argc) cache = argv[++i];
        else {
            try { (void)std::stoi(a); } catch (...) {}  // load_users: no effect, as in the reference
        }
    }
    pf_dataset* ds = nullptr;
    if (pf_dataset_load_cached(root.c_str(), cap, cache.empty() ? nullptr : cache.c_str(), nullptr, &ds) != PF_OK) {
        std::cerr << "[api_cli] " << pf_last_error(nullptr) << "\n";
        return 1;
    }
    pf_dataset_info info{};
    pf_dataset_info_get(ds, &info);
    // load_users_encoded progress lines (user_loader.cpp:35-38,94)
    for (int64_t c = 0; c < info.lines_read; c += 10000) std::cout << "Loaded " << c << " users " << std::endl;
    std::cout << "Loaded " << info.n_profiles << " users total" << std::endl;
    std::cerr << "[api_cli] " << (info.vocab_loaded ? "vocab loaded from data" : "vocab not found (no club names)")
              << "\n[api_cli] adjacency loaded from data/adjacency.csv\n[api_cli] loaded profiles: "
              << info.n_profiles << "\n";
    const std::string median_path = root + "/data/median_age.txt";
    if (info.median_loaded) {
        std::cerr << "[api_cli] loaded median_age=" << info.median_age << " from " << median_path << "\n";
    } else if (info.median_age > 0) {
        std::ofstream out(median_path);  // save_median_age (user_loader.cpp:123-129)
        if (out.is_open()) out << info.median_age << "\n";
        std::cerr << "[api_cli] computed median_age=" << info.median_age << " and saved to " << median_path << "\n";
    } else {
        std::cerr << "[api_cli] computed median_age=0\n";
    }
    std::cerr << "[api_cli] replaced " << info.ages_replaced << " zero-ages with median_age=" << info.median_age
              << "\n";
    if (info.n_normalizers)
        std::cerr << "[api_cli] loaded column normalizers (" << info.n_normalizers << " entries)\n";
    else
        std::cerr << "[api_cli] column_normalizers.csv not found or invalid\n";

    pf_ctx* ctx = nullptr;
    if (pf_open(pf_dataset_desc(ds), device, &ctx) != PF_OK) {
        std::cerr << "[api_cli] engine: " << pf_last_error(nullptr) << "\n";
        pf_dataset_free(ds);
        return 1;
    }

    std::cout << "READY" << std::endl;
    std::cout.flush();
    constexpr int kTop = 20, kLimit = 5000;  // api_cli.cpp:213-234
    std::string line;
    std::vector<char> pj(1 << 16);
    while (std::getline(std::cin, line)) {
        if (line.empty()) {
            std::cout << "{}" << std::endl;
            continue;
        }
        std::string cmd;
        int uid = -1;
        {
            std::istringstream iss(line);
            iss >> cmd;
            if (cmd == "USER") iss >> uid;
        }
        if (cmd == "PING") {
            std::cout << "{\"ok\":true}" << std::endl;
            continue;
        }
        if (cmd == "EXIT") {
            std::cout << "{\"ok\":true, \"exiting\":true}" << std::endl;
            break;
        }
        if (cmd == "USER" && uid >= 0) {
            int64_t len = 0;
            int rc = pf_dataset_profile_json(ds, uid, pj.data(), (int64_t)pj.size(), &len);
            if (rc == PF_ENOTFOUND) {
                std::cout << "{\"error\":\"not found\",\"user_id\":" << uid << "}" << std::endl;
                continue;
            }
            if (len + 1 > (int64_t)pj.size()) {
                pj.resize(len + 1);
                pf_dataset_profile_json(ds, uid, pj.data(), (int64_t)pj.size(), &len);
            }
            const int32_t q = uid;
            List g(kTop), c(kTop), cl(kTop);
            rc = pf_recommend_interest(ctx, &q, 1, kTop, PF_MODE_FOF, kLimit, g.id.data(), g.score.data(), &g.n);
            if (rc == PF_OK) rc = pf_recommend_collab(ctx, &q, 1, kTop, kLimit, c.id.data(), c.score.data(), &c.n);
            if (rc == PF_OK) rc = pf_recommend_clubs(ctx, &q, 1, kTop, kLimit, cl.id.data(), cl.score.data(), &cl.n);
            if (rc != PF_OK) {
                std::cerr << "[api_cli] engine: " << pf_last_error(ctx) << "\n";
                std::cout << "{\"error\":\"engine failure\",\"user_id\":" << uid << "}" << std::endl;
                continue;
            }
            std::ostringstream os;
            os << "{\"profile\":" << pj.data() << ",\"recommendations\":{";
            write_list(os, "graph", g, nullptr);
            os << ",";
            write_list(os, "collaborative", c, nullptr);
            os << ",";
            write_list(os, "interest", g, nullptr);  // recommend_by_interest == graph (recommender_graph.cpp:224-227)
            os << ",";
            write_list(os, "clubs", cl, ds);
            os << "}}";
            std::cout << os.str() << std::endl;
            continue;
        }
        std::cout << "{\"error\":\"unknown command\"}" << std::endl;
    }
    pf_close(ctx);
    pf_dataset_free(ds);
    return 0;
}
