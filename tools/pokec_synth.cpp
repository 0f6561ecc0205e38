// pokec_synth — seeded, Pokec-shaped synthetic corpus.
//
// Test/bench infrastructure, not part of the product library.  It produces
//   * an in-memory pf_corpus_desc (bench.py feeds it straight to pf_open and
//     to the CPU baseline; no CSV round trip at 1.6M users), and
//   * the reference's on-disk formats (users_encoded.csv encoder.cpp:171-180,
//     adjacency.csv graph_builder.cpp:61-75, column_normalizers.csv
//     utils.cpp:144-153, median_age.txt user_loader.cpp:123-129,
//     tokens.csv / clubs_map.csv vocab_builder.cpp:233-287,
//     config/text_columns.txt utils.cpp:13-24) so the compiled reference and
//     the product's own loaders read the very same corpus.
//
// Every user is generated from its own counter-based RNG stream, so the corpus
// is identical for any thread count.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <string>
#include <vector>
#include <algorithm>
#include <numeric>
#include <thread>
#include "pokec_fas.h"

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {  // splitmix64
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    int range(int lo, int hi) { return lo + (int)(uni() * (hi - lo + 1)); }  // inclusive
    double normal() {
        double u1 = uni(), u2 = uni();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

uint64_t mix(uint64_t a, uint64_t b) {
    Rng r(a * 0xD1B54A32D192ED03ull ^ (b + 0x8CB92BA72F3D8DD7ull));
    r.next();
    return r.next();
}

// Inverse-CDF Zipf sampler over ranks 0..n-1 with exponent s.
struct Zipf {
    std::vector<double> cdf;
    Zipf(int n, double s) : cdf(n) {
        double acc = 0;
        for (int i = 0; i < n; ++i) { acc += 1.0 / std::pow(i + 1.0, s); cdf[i] = acc; }
        for (auto& c : cdf) c /= acc;
    }
    int operator()(Rng& r) const {
        double u = r.uni();
        return (int)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()) % (int)cdf.size();
    }
};

}  // namespace

extern "C" {

typedef struct ps_params {
    int32_t  n_users;       // profiles, uids 1..n_users
    int32_t  n_cols;        // text columns (48 in config/text_columns.txt)
    uint64_t seed;
    double   mean_degree;   // mean adjacency out-degree (Pokec: 18.75)
    int32_t  vocab;         // token ids per column
    int32_t  n_club_ids;    // club id universe
    int32_t  edge_cases;    // inject reference edge cases (small fixture corpora)
    int32_t  threads;       // 0 = hardware concurrency
} ps_params;

}  // extern "C"

struct ps_corpus {
    ps_params p{};
    int32_t n = 0, T = 0;
    std::vector<int32_t> uid, pub, comp, gen, age, region;
    std::vector<int64_t> club_off, friend_off, tok_off, adj_off;
    std::vector<uint32_t> clubs, friends;
    std::vector<int32_t> tok_tid, tok_tf;
    std::vector<int32_t> adj_uid, adj_nbr;
    std::vector<uint8_t> norm_present;
    std::vector<float> norm_mean, norm_sd;
    std::vector<std::string> col_names;
    int32_t median_age = 0;
    pf_corpus_desc desc{};
};

namespace {

struct UserGen {
    std::vector<uint32_t> clubs, adj;
    std::vector<int32_t> tid, tf;
    std::vector<int32_t> cnt;  // tokens per column
};

void gen_user(const ps_params& p, const Zipf& ztok, const Zipf& zclub, const Zipf& zpop,
              const std::vector<int32_t>& popperm, int i, UserGen& g,
              int32_t* pub, int32_t* comp, int32_t* gen, int32_t* age, int32_t* reg) {
    const int n = p.n_users, T = p.n_cols;
    const int uid = i + 1;
    Rng r(mix(p.seed, (uint64_t)uid));
    g.clubs.clear(); g.adj.clear(); g.tid.clear(); g.tf.clear(); g.cnt.assign(T, 0);

    double u = r.uni();
    *pub = u < 0.03 ? -1 : (r.uni() < 0.55 ? 1 : 0);
    u = r.uni();
    *gen = u < 0.04 ? -1 : (r.uni() < 0.5 ? 1 : 0);
    u = r.uni();
    *comp = u < 0.02 ? -1 : (u < 0.05 ? 0 : r.range(1, 100));
    u = r.uni();
    *age = u < 0.02 ? 0 : r.range(14, 80);
    // hierarchical region: kraj (8) ; okres (~80) ; obec (~3000)
    int k0 = r.range(0, 7), k1 = k0 * 10 + r.range(0, 9), k2 = k1 * 37 + r.range(0, 36);
    reg[0] = r.uni() < 0.2 ? -1 : k0;
    reg[1] = r.uni() < 0.2 ? -1 : k1;
    reg[2] = r.uni() < 0.2 ? -1 : k2;

    static const int club_counts[5] = {0, 0, 1, 3, 8};
    int nc = club_counts[r.range(0, 4)];
    for (int c = 0; c < nc; ++c) g.clubs.push_back((uint32_t)zclub(r) + 1);

    // heavy-tailed out-degree (lognormal, sigma 1.1) with ~4% isolated users
    int deg = 0;
    if (r.uni() > 0.04) {
        const double sigma = 1.1;
        double mu = std::log(p.mean_degree / 0.96) - 0.5 * sigma * sigma;
        deg = (int)std::floor(std::exp(mu + sigma * r.normal()));
        if (deg > 5000) deg = 5000;
        if (deg > n - 1) deg = n - 1;
    }
    for (int e = 0; e < deg; ++e) {
        int v;
        if (r.uni() < 0.55) {  // local: produces triangles / shared friends
            int w = r.range(-400, 400);
            v = ((i + w) % n + n) % n + 1;
        } else {               // global: preferential (Zipf over a fixed permutation)
            v = popperm[zpop(r)] + 1;
        }
        if (v == uid && !p.edge_cases) v = (v % n) + 1;
        g.adj.push_back((uint32_t)v);
        if (r.uni() < 0.001) g.adj.push_back((uint32_t)v);  // duplicate edge
    }

    for (int t = 0; t < T; ++t) {
        double pt = 0.15 + 0.40 * std::fmod((t + 1) * 0.6180339887, 1.0);
        if (r.uni() >= pt) continue;
        int m = r.range(1, 12);
        size_t base = g.tid.size();
        for (int k = 0; k < m; ++k) {
            int tid = 0;
            for (int a = 0; a < 8; ++a) {  // distinct tids within one column
                tid = ztok(r) + 1;
                bool dup = false;
                for (size_t q = base; q < g.tid.size(); ++q) if (g.tid[q] == tid) { dup = true; break; }
                if (!dup) break;
                tid = -1;
            }
            if (tid < 0) continue;
            double v = r.uni();
            int tf = v < 0.01 ? 0 : (v < 0.61 ? 1 : (v < 0.91 ? 2 : 3));
            g.tid.push_back(tid);
            g.tf.push_back(tf);
        }
        g.cnt[t] = (int32_t)(g.tid.size() - base);
    }
}

template <class F>
void parallel_for(int n, int threads, F f) {
    if (threads <= 1 || n < 1024) { f(0, n, 0); return; }
    std::vector<std::thread> th;
    int chunk = (n + threads - 1) / threads;
    for (int w = 0; w < threads; ++w) {
        int lo = w * chunk, hi = std::min(n, lo + chunk);
        if (lo >= hi) break;
        th.emplace_back(f, lo, hi, w);
    }
    for (auto& t : th) t.join();
}

// raw-count cosine, the normaliser sampler's text similarity (utils.cpp:155-240 uses A7)
double raw_cos(const int32_t* ta, const int32_t* fa, int na, const int32_t* tb, const int32_t* fb, int nb) {
    if (na == 0 || nb == 0) return 0.0;
    double sa = 0, sb = 0, d = 0;
    for (int i = 0; i < na; ++i) sa += (double)fa[i] * fa[i];
    for (int j = 0; j < nb; ++j) sb += (double)fb[j] * fb[j];
    if (sa <= 0 || sb <= 0) return 0.0;
    for (int i = 0; i < na; ++i)
        for (int j = 0; j < nb; ++j)
            if (ta[i] == tb[j]) d += (double)fa[i] * fb[j];
    return (double)(float)(d / (std::sqrt(sa) * std::sqrt(sb)));
}

double set_sim(const uint32_t* a, int na, const uint32_t* b, int nb) {
    if (na == 0 || nb == 0) return 0.0;
    int inter = 0;
    for (int j = 0; j < nb; ++j)
        for (int i = 0; i < na; ++i)
            if (a[i] == b[j]) { ++inter; break; }
    return (double)(float)(inter / (std::sqrt((double)na) * std::sqrt((double)nb)));
}

float round6(double x) {  // ostream default precision (6 significant digits), utils.cpp:144-153
    char buf[64];
    snprintf(buf, sizeof buf, "%g", (double)(float)x);
    return (float)atof(buf);
}

void compute_normalizers(ps_corpus* c) {
    const int n = c->n, T = c->T, K = PF_NUM_FIXED + T;
    std::vector<double> sum(K, 0), sq(K, 0);
    Rng r(mix(c->p.seed, 0xA11CE));
    const int S = std::min<int64_t>(200000, (int64_t)n * 5);
    std::vector<std::vector<double>> vals(K);
    for (int s = 0; s < S; ++s) {
        int a = (int)(r.next() % n), b = (int)(r.next() % n);
        if (a == b) continue;
        double v[PF_NUM_FIXED];
        v[0] = (c->pub[a] >= 0 && c->pub[b] >= 0 && c->pub[a] == c->pub[b]) ? 1.0 : 0.0;
        v[1] = (c->gen[a] >= 0 && c->gen[b] >= 0 && c->gen[a] == c->gen[b]) ? 1.0 : 0.0;
        v[2] = (c->comp[a] > 0 && c->comp[b] > 0) ? (double)std::min(c->comp[a], c->comp[b]) / std::max(c->comp[a], c->comp[b]) : 0.0;
        v[3] = (c->age[a] > 0 && c->age[b] > 0) ? (double)std::min(c->age[a], c->age[b]) / std::max(c->age[a], c->age[b]) : 0.0;
        int ac = 0, bc = 0, m = 0;
        for (int k = 0; k < 3; ++k) {
            int x = c->region[3 * a + k], y = c->region[3 * b + k];
            ac += x >= 0; bc += y >= 0; m += (x >= 0 && y >= 0 && x == y);
        }
        v[4] = (ac && bc) ? (double)(float)(m / (std::sqrt((double)ac) * std::sqrt((double)bc))) : 0.0;
        v[5] = set_sim(&c->clubs[c->club_off[a]], (int)(c->club_off[a + 1] - c->club_off[a]),
                       &c->clubs[c->club_off[b]], (int)(c->club_off[b + 1] - c->club_off[b]));
        v[6] = set_sim(&c->friends[c->friend_off[a]], (int)(c->friend_off[a + 1] - c->friend_off[a]),
                       &c->friends[c->friend_off[b]], (int)(c->friend_off[b + 1] - c->friend_off[b]));
        for (int k = 0; k < PF_NUM_FIXED; ++k) vals[k].push_back(v[k]);
        for (int t = 0; t < T; ++t) {
            int64_t ra = (int64_t)a * T + t, rb = (int64_t)b * T + t;
            int64_t oa = c->tok_off[ra], ob = c->tok_off[rb];
            vals[PF_NUM_FIXED + t].push_back(raw_cos(&c->tok_tid[oa], &c->tok_tf[oa], (int)(c->tok_off[ra + 1] - oa),
                                                     &c->tok_tid[ob], &c->tok_tf[ob], (int)(c->tok_off[rb + 1] - ob)));
        }
    }
    c->norm_present.assign(K, 1);
    c->norm_mean.assign(K, 0.f);
    c->norm_sd.assign(K, 1.f);
    for (int k = 0; k < K; ++k) {
        const auto& v = vals[k];
        double mu = 0;
        for (double x : v) mu += x;
        mu = v.empty() ? 0 : mu / v.size();
        double s = 0;
        for (double x : v) s += (x - mu) * (x - mu);
        s = v.size() > 1 ? std::sqrt(s / (v.size() - 1)) : 1.0;
        if (s == 0.0) s = 1.0;
        c->norm_mean[k] = round6(mu);
        c->norm_sd[k] = round6(s);
    }
    // some keys absent (z = 6(s-0.5)) and some sd = 0 (also default z)
    if (T >= 40) {
        const int absent[5] = {PF_F_AGE, PF_NUM_FIXED + 3, PF_NUM_FIXED + 11, PF_NUM_FIXED + 29, PF_NUM_FIXED + 40};
        for (int k : absent) c->norm_present[k] = 0;
        c->norm_sd[PF_NUM_FIXED + 7] = 0.f;
        c->norm_sd[PF_F_REGION] = 0.f;
    }
}

}  // namespace

extern "C" {

int ps_generate(const ps_params* pin, ps_corpus** out) {
    if (!pin || !out || pin->n_users < 2 || pin->n_cols < 1 || pin->n_cols > PF_MAX_COLS) return -1;
    ps_corpus* c = new ps_corpus();
    c->p = *pin;
    ps_params& p = c->p;
    if (p.vocab <= 0) p.vocab = 2000;
    if (p.n_club_ids <= 0) p.n_club_ids = 20000;
    if (p.mean_degree <= 0) p.mean_degree = 18.75;
    int threads = p.threads > 0 ? p.threads : (int)std::max(1u, std::thread::hardware_concurrency());
    if (threads > 32) threads = 32;
    const int n = p.n_users, T = p.n_cols;
    c->n = n; c->T = T;
    Zipf ztok(p.vocab, 1.1), zclub(p.n_club_ids, 1.0), zpop(n, 0.8);
    std::vector<int32_t> popperm(n);
    std::iota(popperm.begin(), popperm.end(), 0);
    {
        Rng r(mix(p.seed, 0x5EED));
        for (int i = n - 1; i > 0; --i) std::swap(popperm[i], popperm[(int)(r.next() % (uint64_t)(i + 1))]);
    }
    c->uid.resize(n); c->pub.resize(n); c->comp.resize(n); c->gen.resize(n); c->age.resize(n);
    c->region.resize(3 * (size_t)n);
    std::vector<int64_t> nclub(n), nadj(n), ntok(n);
    std::vector<int32_t> tokcnt((size_t)n * T);
    // pass 1: sizes
    parallel_for(n, threads, [&](int lo, int hi, int) {
        UserGen g;
        for (int i = lo; i < hi; ++i) {
            gen_user(p, ztok, zclub, zpop, popperm, i, g, &c->pub[i], &c->comp[i], &c->gen[i], &c->age[i], &c->region[3 * (size_t)i]);
            c->uid[i] = i + 1;
            nclub[i] = (int64_t)g.clubs.size();
            nadj[i] = (int64_t)g.adj.size();
            ntok[i] = (int64_t)g.tid.size();
            std::copy(g.cnt.begin(), g.cnt.end(), &tokcnt[(size_t)i * T]);
        }
    });
    c->club_off.assign(n + 1, 0); c->adj_off.assign(n + 1, 0); c->tok_off.assign((size_t)n * T + 1, 0);
    for (int i = 0; i < n; ++i) { c->club_off[i + 1] = c->club_off[i] + nclub[i]; c->adj_off[i + 1] = c->adj_off[i] + nadj[i]; }
    for (size_t r = 0; r < (size_t)n * T; ++r) c->tok_off[r + 1] = c->tok_off[r] + tokcnt[r];
    c->clubs.resize(c->club_off[n]); c->adj_nbr.resize(c->adj_off[n]);
    c->tok_tid.resize(c->tok_off[(size_t)n * T]); c->tok_tf.resize(c->tok_off[(size_t)n * T]);
    // pass 2: fill (same streams => same values)
    parallel_for(n, threads, [&](int lo, int hi, int) {
        UserGen g;
        int32_t a, b, cc, d, rg[3];
        for (int i = lo; i < hi; ++i) {
            gen_user(p, ztok, zclub, zpop, popperm, i, g, &a, &b, &cc, &d, rg);
            std::copy(g.clubs.begin(), g.clubs.end(), c->clubs.begin() + c->club_off[i]);
            for (size_t k = 0; k < g.adj.size(); ++k) c->adj_nbr[c->adj_off[i] + k] = (int32_t)g.adj[k];
            std::copy(g.tid.begin(), g.tid.end(), c->tok_tid.begin() + c->tok_off[(size_t)i * T]);
            std::copy(g.tf.begin(), g.tf.end(), c->tok_tf.begin() + c->tok_off[(size_t)i * T]);
        }
    });
    // profile friends column = adjacency out-list (encoder.cpp:130-137)
    c->friend_off = c->adj_off;
    c->friends.assign(c->adj_nbr.begin(), c->adj_nbr.end());
    c->adj_uid = c->uid;

    if (p.edge_cases) {
        Rng r(mix(p.seed, 0xED6E));
        // (1) a fully empty profile, (2) hub with a large out-list, (3) friends column that
        //     differs from adjacency, (4) duplicate clubs/friends, (5) adjacency rows for
        //     uids without profiles and users without adjacency rows.
        int e0 = 0;
        c->pub[e0] = c->gen[e0] = c->comp[e0] = -1; c->age[e0] = 0;
        c->region[0] = c->region[1] = c->region[2] = -1;
        // rebuild CSR arrays with per-user edits
        std::vector<std::vector<uint32_t>> cl(n), fr(n);
        std::vector<std::vector<int32_t>> ad(n);
        for (int i = 0; i < n; ++i) {
            cl[i].assign(c->clubs.begin() + c->club_off[i], c->clubs.begin() + c->club_off[i + 1]);
            fr[i].assign(c->friends.begin() + c->friend_off[i], c->friends.begin() + c->friend_off[i + 1]);
            ad[i].assign(c->adj_nbr.begin() + c->adj_off[i], c->adj_nbr.begin() + c->adj_off[i + 1]);
        }
        cl[e0].clear(); fr[e0].clear();
        // hub
        int hub = 7 % n;
        for (int k = 0; k < std::min(n - 1, 300); ++k) ad[hub].push_back((int32_t)(r.next() % n) + 1);
        fr[hub].assign(ad[hub].begin(), ad[hub].end());
        for (int i = 11; i < n; i += 97) {       // duplicates in clubs / friends
            if (!cl[i].empty()) cl[i].push_back(cl[i][0]);
            if (!fr[i].empty()) { fr[i].push_back(fr[i][0]); }
        }
        for (int i = 13; i < n; i += 89) {       // friends column != adjacency
            if (fr[i].size() > 2) fr[i].resize(fr[i].size() / 2);
            fr[i].push_back((uint32_t)(n + 50 + i));  // a friend that has no profile
        }
        for (int i = 17; i < n; i += 101) ad[i].push_back(i + 1);  // self loop
        for (int i = 19; i < n; i += 103) ad[i].push_back(n + 7);  // neighbour without profile
        // tf = 0 only column
        for (int i = 23; i < n; i += 211) {
            int64_t o = c->tok_off[(size_t)i * T];
            for (int64_t q = o; q < c->tok_off[(size_t)i * T + 1]; ++q) c->tok_tf[q] = 0;
        }
        c->club_off[0] = 0; c->friend_off.assign(n + 1, 0);
        c->clubs.clear(); c->friends.clear();
        for (int i = 0; i < n; ++i) {
            c->clubs.insert(c->clubs.end(), cl[i].begin(), cl[i].end());
            c->friends.insert(c->friends.end(), fr[i].begin(), fr[i].end());
            c->club_off[i + 1] = (int64_t)c->clubs.size();
            c->friend_off[i + 1] = (int64_t)c->friends.size();
        }
        // adjacency: drop rows of every 50th user, add rows for missing uids
        c->adj_uid.clear(); c->adj_off.assign(1, 0); c->adj_nbr.clear();
        for (int i = 0; i < n; ++i) {
            if (i % 50 == 29) continue;
            c->adj_uid.push_back(i + 1);
            c->adj_nbr.insert(c->adj_nbr.end(), ad[i].begin(), ad[i].end());
            c->adj_off.push_back((int64_t)c->adj_nbr.size());
        }
        for (int k = 0; k < 3; ++k) {
            c->adj_uid.push_back(n + 7 + k);
            for (int q = 0; q < 5; ++q) c->adj_nbr.push_back((int32_t)(r.next() % n) + 1);
            c->adj_off.push_back((int64_t)c->adj_nbr.size());
        }
    }

    // median age over age > 0 (user_loader.cpp:98-110), then fill (user_loader.cpp:131-140)
    {
        std::vector<int32_t> ages;
        for (int i = 0; i < n; ++i) if (c->age[i] > 0) ages.push_back(c->age[i]);
        std::sort(ages.begin(), ages.end());
        size_t m = ages.size();
        c->median_age = m == 0 ? 0 : (m % 2 ? ages[m / 2] : (ages[m / 2 - 1] + ages[m / 2]) / 2);
    }
    compute_normalizers(c);
    c->col_names.resize(T);
    for (int t = 0; t < T; ++t) {
        char b[32];
        snprintf(b, sizeof b, "col%02d", t);
        c->col_names[t] = b;
    }
    // in-memory desc uses filled ages (api_cli.cpp:152)
    pf_corpus_desc& d = c->desc;
    d.n_users = n; d.n_cols = T;
    d.user_id = c->uid.data(); d.public_flag = c->pub.data(); d.completion = c->comp.data();
    d.gender = c->gen.data(); d.age = c->age.data(); d.region = c->region.data();
    d.club_off = c->club_off.data(); d.club_ids = c->clubs.data();
    d.friend_off = c->friend_off.data(); d.friend_ids = c->friends.data();
    d.tok_off = c->tok_off.data(); d.tok_tid = c->tok_tid.data(); d.tok_tf = c->tok_tf.data();
    d.n_adj = (int32_t)c->adj_uid.size(); d.adj_uid = c->adj_uid.data(); d.adj_off = c->adj_off.data();
    d.adj_nbr = c->adj_nbr.data();
    d.idf_mode = PF_IDF_FROM_PROFILES;
    d.norm_present = c->norm_present.data(); d.norm_mean = c->norm_mean.data(); d.norm_sd = c->norm_sd.data();
    *out = c;
    return 0;
}

// ages with the median filled in (what pf_corpus_desc expects)
const pf_corpus_desc* ps_desc(ps_corpus* c) { return &c->desc; }

int32_t ps_median_age(const ps_corpus* c) { return c->median_age; }

// Fill ages in place (the desc points at c->age).  Raw ages are kept for the CSV writer
// by writing files BEFORE calling this.
void ps_fill_ages(ps_corpus* c) {
    for (auto& a : c->age) if (a == 0) a = c->median_age;
    c->desc.age = c->age.data();
}

int64_t ps_total_tokens(const ps_corpus* c) { return (int64_t)c->tok_tid.size(); }

// Writes the reference's data/ + config/ layout under `root`.
int ps_write_reference_files(const ps_corpus* c, const char* root, int write_normalizers, int write_median) {
    std::string R(root);
    std::string cmd = "mkdir -p '" + R + "/data' '" + R + "/config'";
    if (std::system(cmd.c_str()) != 0) return -1;
    const int n = c->n, T = c->T;
    const bool ec = c->p.edge_cases != 0;
    FILE* f = fopen((R + "/config/text_columns.txt").c_str(), "w");
    if (!f) return -1;
    for (int t = 0; t < T; ++t) fprintf(f, "%s\n", c->col_names[t].c_str());
    fclose(f);

    f = fopen((R + "/data/users_encoded.csv").c_str(), "w");
    if (!f) return -1;
    fprintf(f, "user_id,public,completion_percentage,gender,region,age,clubs,friends");
    for (int t = 0; t < T; ++t) fprintf(f, ",%s_tokens", c->col_names[t].c_str());
    fprintf(f, "\n");
    auto put_int_or_empty = [&](int v, bool missing) { if (!missing) fprintf(f, "%d", v); };
    for (int i = 0; i < n; ++i) {
        if (ec && i == 5) fprintf(f, "\n");                       // blank line (skipped, still counted)
        if (ec && i == 9) fprintf(f, "0,1,50,1,1;2;3,30,,,\n");   // uid 0 row (skipped)
        if (ec && i == 31) {                                        // duplicate uid row, later overwritten
            fprintf(f, "%d,1,1,1,;;,99,5,,", c->uid[i + 1]);
            for (int t = 0; t < T; ++t) fprintf(f, "%s", t + 1 < T ? "," : "");
            fprintf(f, "\n");
        }
        fprintf(f, "%d,", c->uid[i]);
        put_int_or_empty(c->pub[i], c->pub[i] < 0); fprintf(f, ",");
        put_int_or_empty(c->comp[i], c->comp[i] < 0); fprintf(f, ",");
        put_int_or_empty(c->gen[i], c->gen[i] < 0); fprintf(f, ",");
        const int32_t* rg = &c->region[3 * (size_t)i];
        bool quote = ec && (i % 7 == 3);
        if (quote) fprintf(f, "\"");
        for (int k = 0; k < 3; ++k) {
            if (rg[k] >= 0) fprintf(f, "%d", rg[k]);
            if (k < 2) fprintf(f, ";");
        }
        if (ec && i % 13 == 4) fprintf(f, ";77");                 // 4th part ignored
        if (quote) fprintf(f, "\"");
        fprintf(f, ",");
        if (!(ec && i % 19 == 2 && c->age[i] == 0)) fprintf(f, "%d", c->age[i]);
        fprintf(f, ",");
        for (int64_t k = c->club_off[i]; k < c->club_off[i + 1]; ++k)
            fprintf(f, "%s%u", k > c->club_off[i] ? ";" : "", c->clubs[k]);
        fprintf(f, ",");
        for (int64_t k = c->friend_off[i]; k < c->friend_off[i + 1]; ++k)
            fprintf(f, "%s%u", k > c->friend_off[i] ? ";" : "", c->friends[k]);
        for (int t = 0; t < T; ++t) {
            fprintf(f, ",");
            size_t r = (size_t)i * T + t;
            for (int64_t k = c->tok_off[r]; k < c->tok_off[r + 1]; ++k)
                fprintf(f, "%s%d:%d", k > c->tok_off[r] ? ";" : "", c->tok_tid[k], c->tok_tf[k]);
            if (ec && c->tok_off[r + 1] > c->tok_off[r] && (i + t) % 53 == 0) {
                // duplicate tid: last value wins (user_loader.cpp:88); entry without ':' skipped (utils.cpp:62)
                fprintf(f, ";%d:%d;junk", c->tok_tid[c->tok_off[r]], 2);
            }
        }
        fprintf(f, "\n");
    }
    fclose(f);

    f = fopen((R + "/data/adjacency.csv").c_str(), "w");
    if (!f) return -1;
    {
        std::vector<int> order(c->adj_uid.size());
        std::iota(order.begin(), order.end(), 0);
        std::sort(order.begin(), order.end(), [&](int a, int b) { return c->adj_uid[a] < c->adj_uid[b]; });
        for (size_t q = 0; q < order.size(); ++q) {
            int a = order[q];
            fprintf(f, "%d", c->adj_uid[a]);
            int64_t lo = c->adj_off[a], hi = c->adj_off[a + 1];
            int64_t split = (ec && q % 41 == 5) ? lo + (hi - lo) / 2 : hi;
            for (int64_t k = lo; k < split; ++k) fprintf(f, ec && k % 17 == 3 ? ", %d" : ",%d", c->adj_nbr[k]);
            fprintf(f, "\n");
            if (split < hi) {  // repeated uid line appends (graph_builder.cpp:39-59)
                fprintf(f, "%d", c->adj_uid[a]);
                for (int64_t k = split; k < hi; ++k) fprintf(f, ",%d", c->adj_nbr[k]);
                fprintf(f, "\n");
            }
        }
    }
    fclose(f);

    if (write_median) {
        f = fopen((R + "/data/median_age.txt").c_str(), "w");
        if (!f) return -1;
        fprintf(f, "%d\n", c->median_age);
        fclose(f);
    }
    if (write_normalizers) {
        f = fopen((R + "/data/column_normalizers.csv").c_str(), "w");
        if (!f) return -1;
        fprintf(f, "column,mean,stddev\n");
        static const char* fixed[PF_NUM_FIXED] = {"public", "gender", "completion", "age", "region", "clubs", "friends"};
        for (int k = 0; k < PF_NUM_FIXED + T; ++k) {
            if (!c->norm_present[k]) continue;
            const char* name = k < PF_NUM_FIXED ? fixed[k] : c->col_names[k - PF_NUM_FIXED].c_str();
            fprintf(f, "%s,%g,%g\n", name, (double)c->norm_mean[k], (double)c->norm_sd[k]);
        }
        fclose(f);
    }
    // vocab files: tokens.csv must exist or api_cli runs the ETL (api_cli.cpp:101-108)
    f = fopen((R + "/data/tokens.csv").c_str(), "w");
    if (!f) return -1;
    fprintf(f, "column,token,tid,df\n");
    for (int t = 0; t < T; ++t)
        for (int v = 1; v <= std::min(c->p.vocab, 50); ++v)
            fprintf(f, "%s,w%d_%d,%d,%d\n", c->col_names[t].c_str(), t, v, v, 1);
    fclose(f);
    f = fopen((R + "/data/clubs_map.csv").c_str(), "w");
    if (!f) return -1;
    fprintf(f, "club_id,slug,title\n");
    for (int k = 1; k <= std::min(c->p.n_club_ids, 400); ++k) {
        if (k % 3 == 0) continue;  // some clubs without names
        if (k % 10 == 1) fprintf(f, "%d,klub-q%d\\x\t,\"Title, %d\"\n", k, k, k);  // json_escape path
        else fprintf(f, "%d,klub-%d,Title %d\n", k, k, k);
    }
    fclose(f);
    return 0;
}

void ps_free(ps_corpus* c) { delete c; }

}  // extern "C"
