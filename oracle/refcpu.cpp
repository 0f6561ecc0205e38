// refcpu — clean-room CPU restatement of the reference hot path (see refcpu.h).
//
// TEST INFRASTRUCTURE ONLY: used by tests/ as the parity checker and by
// bench.py as the CPU baseline ("kind": "port").  Every function cites the
// reference code it restates; the containers mirror the reference's so the
// arithmetic order (and therefore every float) and the timing profile match.
#include "refcpu.h"

#include "pokec_io.h"  // pf_result_digest (a plain hash; no engine code)

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

using TokMap = std::unordered_map<int, int>;

struct Prof {                       // include/user_profile.h:10-20
    int uid = -1, pub = -1, comp = -1, gen = -1, age = 0;
    std::vector<uint32_t> clubs, friends;
    std::vector<TokMap> cols;
    std::array<int, 3> reg{{-1, -1, -1}};
};

using Ranked = std::vector<std::pair<int, float>>;

void rank_and_cut(Ranked& v, int topk) {       // recommender_graph.cpp:97-101
    std::sort(v.begin(), v.end(), [](const std::pair<int, float>& x, const std::pair<int, float>& y) {
        return x.second == y.second ? x.first < y.first : x.second > y.second;
    });
    if ((int)v.size() > topk) v.resize(topk < 0 ? 0 : topk);
}

}  // namespace

struct ro_ctx {
    int T = 0;
    std::unordered_map<int, Prof> prof;
    std::unordered_map<int, std::vector<int>> adj;
    std::vector<std::unordered_map<int, float>> idf;  // per column
    std::vector<char> has_idf;
    std::vector<char> npres;
    std::vector<float> nmean, nsd;
    mutable int64_t fas_calls = 0;  // profile_similarity evaluations (bench pair counts)

    // --- A10 helpers -------------------------------------------------------
    static double logistic(double x) {            // recommender_similarity.cpp:18-26
        if (x >= 0) { double e = std::exp(-x); return 1.0 / (1.0 + e); }
        double e = std::exp(x);
        return e / (1.0 + e);
    }
    double z_of(int slot, double s) const {       // recommender_similarity.cpp:28-36,105-111
        if (npres[slot] && nsd[slot] > 0.0) return (s - (double)nmean[slot]) / (double)nsd[slot];
        return 6.0 * (s - 0.5);
    }
    // recommender.cpp:119-128: |{b in B : b in set(A)}| / (sqrt|A| sqrt|B|), B with duplicates
    static float overlap(const std::vector<uint32_t>& A, const std::vector<uint32_t>& B) {
        if (A.empty() || B.empty()) return 0.0f;
        std::unordered_map<uint32_t, int> seen;
        for (uint32_t a : A) seen[a] = 1;
        int hits = 0;
        for (uint32_t b : B) hits += seen.find(b) != seen.end();
        double den = std::sqrt((double)A.size()) * std::sqrt((double)B.size());
        return den <= 0.0 ? 0.0f : (float)((double)hits / den);
    }
    // recommender.cpp:130-139
    static float region_sim(const std::array<int, 3>& A, const std::array<int, 3>& B) {
        int na = 0, nb = 0, m = 0;
        for (int i = 0; i < 3; ++i) {
            na += A[i] >= 0;
            nb += B[i] >= 0;
            m += (A[i] >= 0 && B[i] >= 0 && A[i] == B[i]);
        }
        if (!na || !nb) return 0.0f;
        return (float)((double)m / (std::sqrt((double)na) * std::sqrt((double)nb)));
    }
    // recommender.cpp:68-117 (weights tf*idf; absent token -> idf 1.0)
    static float tfidf_cos(const TokMap& A, const TokMap& B, const std::unordered_map<int, float>& w) {
        if (A.empty() || B.empty()) return 0.0f;
        auto idf_of = [&](int tok) -> double {
            return w.count(tok) ? w.at(tok) : 1.0f;
        };
        double dot = 0, na = 0, nb = 0;
        const bool a_small = A.size() < B.size();
        const TokMap& S = a_small ? A : B;     // the map walked for the dot product
        const TokMap& L = a_small ? B : A;
        double& ns = a_small ? na : nb;
        double& nl = a_small ? nb : na;
        for (const auto& e : S) {
            double ws = (double)e.second * idf_of(e.first);
            ns += ws * ws;
            auto hit = L.find(e.first);
            if (hit != L.end()) {
                double wl = (double)hit->second * idf_of(e.first);
                dot += a_small ? ws * wl : wl * ws;
            }
        }
        for (const auto& e : L) {
            double wl = (double)e.second * idf_of(e.first);
            nl += wl * wl;
        }
        double den = std::sqrt(na) * std::sqrt(nb);
        return den <= 0.0 ? 0.0f : (float)(dot / den);
    }
    // recommender.cpp:141-163 (raw counts; used when the column has no idf map)
    static float count_cos(const TokMap& A, const TokMap& B) {
        if (A.empty() || B.empty()) return 0.0f;
        double sa = 0, sb = 0, dot = 0;
        for (const auto& e : A) sa += (double)e.second * e.second;
        for (const auto& e : B) sb += (double)e.second * e.second;
        if (sa <= 0.0 || sb <= 0.0) return 0.0f;
        const bool a_small = A.size() < B.size();
        const TokMap& S = a_small ? A : B;
        const TokMap& L = a_small ? B : A;
        for (const auto& e : S) {
            auto hit = L.find(e.first);
            if (hit != L.end()) dot += (double)e.second * hit->second;
        }
        double den = std::sqrt(sa) * std::sqrt(sb);
        return den <= 0.0 ? 0.0f : (float)(dot / den);
    }

    // recommender_similarity.cpp:10-124
    float fas(const Prof& A, const Prof& B) const {
        ++fas_calls;
        const int possible = PF_NUM_FIXED + T;
        int used = 0;
        double acc = 0.0;
        auto add = [&](int slot, double s) { acc += logistic(z_of(slot, s)); ++used; };
        if (A.pub >= 0 && B.pub >= 0) add(PF_F_PUBLIC, A.pub == B.pub ? 1.0 : 0.0);
        if (A.gen >= 0 && B.gen >= 0) add(PF_F_GENDER, A.gen == B.gen ? 1.0 : 0.0);
        if (A.comp > 0 && B.comp > 0) {
            int lo = std::min(A.comp, B.comp), hi = std::max(A.comp, B.comp);
            add(PF_F_COMPLETION, hi > 0 ? (double)lo / (double)hi : 0.0);
        }
        if (A.age > 0 && B.age > 0) {
            int lo = std::min(A.age, B.age), hi = std::max(A.age, B.age);
            add(PF_F_AGE, hi > 0 ? (double)lo / (double)hi : 0.0);
        }
        const bool ra = A.reg[0] >= 0 || A.reg[1] >= 0 || A.reg[2] >= 0;
        const bool rb = B.reg[0] >= 0 || B.reg[1] >= 0 || B.reg[2] >= 0;
        if (ra && rb) add(PF_F_REGION, region_sim(A.reg, B.reg));
        if (!A.clubs.empty() && !B.clubs.empty()) add(PF_F_CLUBS, overlap(A.clubs, B.clubs));
        if (!A.friends.empty() && !B.friends.empty()) add(PF_F_FRIENDS, overlap(A.friends, B.friends));
        for (int t = 0; t < T; ++t) {
            bool ha = t < (int)A.cols.size() && !A.cols[t].empty();
            bool hb = t < (int)B.cols.size() && !B.cols[t].empty();
            if (!ha || !hb) continue;
            double s = has_idf[t] ? tfidf_cos(A.cols[t], B.cols[t], idf[t]) : count_cos(A.cols[t], B.cols[t]);
            add(PF_NUM_FIXED + t, s);
        }
        if (used == 0) return 0.0f;
        double S = acc / (double)used;
        double F = (double)used / (double)possible;
        if (S <= 0.0 && F <= 0.0) return 0.0f;
        return (float)((2.0 * S * F) / (S + F));
    }

    const Prof* find(int uid) const {
        auto it = prof.find(uid);
        return it == prof.end() ? nullptr : &it->second;
    }
    const std::vector<int>* nbrs(int uid) const {
        auto it = adj.find(uid);
        return it == adj.end() ? nullptr : &it->second;
    }

    // recommender_graph.cpp:10-31 — friends and FoFs in first-seen order, stop at limit
    std::vector<int> gather_graph(int u, int limit) const {
        std::vector<int> out;
        const std::vector<int>* fr = nbrs(u);
        if (!fr) return out;
        std::unordered_set<int> seen;
        for (int f : *fr) {
            if (f == u) continue;
            if (seen.insert(f).second) out.push_back(f);
            if ((int)out.size() >= limit) return out;
            const std::vector<int>* ff = nbrs(f);
            if (!ff) continue;
            for (int x : *ff) {
                if (x == u) continue;
                if (seen.insert(x).second) {
                    out.push_back(x);
                    if ((int)out.size() >= limit) return out;
                }
            }
        }
        return out;
    }
    // recommender_graph.cpp:114-125 — FoFs only, inner loop broken at limit
    std::vector<int> gather_collab(int u, int limit) const {
        std::vector<int> out;
        const std::vector<int>* fr = nbrs(u);
        if (!fr) return out;
        std::unordered_set<int> seen;
        for (int f : *fr) {
            const std::vector<int>* ff = nbrs(f);
            if (!ff) continue;
            for (int x : *ff) {
                if (x == u) continue;
                if (seen.insert(x).second) out.push_back(x);
                if ((int)out.size() >= limit) break;
            }
            if ((int)out.size() >= limit) break;
        }
        return out;
    }

    // recommender_graph.cpp:33-57,97-103
    Ranked rec_graph(int u, int topk, int limit) const {
        Ranked out;
        const Prof* q = find(u);
        if (!q) return out;
        std::vector<int> cand = gather_graph(u, limit);
        std::unordered_set<int> skip;
        if (const std::vector<int>* fr = nbrs(u)) skip.insert(fr->begin(), fr->end());
        skip.insert(u);
        for (int c : cand) {
            if (skip.count(c)) continue;
            const Prof* pc = find(c);
            if (!pc) continue;
            out.emplace_back(c, fas(*q, *pc));
        }
        rank_and_cut(out, topk);
        return out;
    }
    // every loaded profile except u and adj[u]
    Ranked rec_all(int u, int topk) const {
        Ranked out;
        const Prof* q = find(u);
        if (!q) return out;
        std::unordered_set<int> skip;
        if (const std::vector<int>* fr = nbrs(u)) skip.insert(fr->begin(), fr->end());
        skip.insert(u);
        for (const auto& kv : prof) {
            if (skip.count(kv.first)) continue;
            out.emplace_back(kv.first, fas(*q, kv.second));
        }
        rank_and_cut(out, topk);
        return out;
    }
    // recommender_graph.cpp:105-222 (profiles branch)
    Ranked rec_collab(int u, int topk, int limit) const {
        Ranked out;
        std::vector<int> friends;
        if (const std::vector<int>* fr = nbrs(u)) friends = *fr;
        std::vector<int> cand = gather_collab(u, limit);
        const Prof* q = find(u);
        if (!q) return out;
        std::unordered_map<int, float> w;
        for (int f : friends) {
            const Prof* pf = find(f);
            if (pf) w[f] = fas(*q, *pf);
        }
        for (int c : cand) {
            if (c == u) continue;
            const Prof* pc = find(c);
            if (!pc) continue;
            double score = 0.0;
            for (int f : friends) {
                auto it = w.find(f);
                if (it == w.end()) continue;
                const Prof* pf = find(f);
                if (!pf) continue;
                score += (double)it->second * (double)fas(*pf, *pc);
            }
            out.emplace_back(c, (float)score);
        }
        rank_and_cut(out, topk);
        return out;
    }
    // recommender_clubs.cpp:10-73
    Ranked rec_clubs(int u, int topk, int /*limit*/) const {
        Ranked out;
        const Prof* q = find(u);
        if (!q) return out;
        std::vector<int> friends;
        if (const std::vector<int>* fr = nbrs(u)) friends = *fr;
        std::unordered_map<int, float> w;
        for (int f : friends) {
            const Prof* pf = find(f);
            if (pf) w[f] = fas(*q, *pf);
        }
        std::unordered_set<int> own;
        for (uint32_t c : q->clubs) own.insert((int)c);
        std::unordered_map<int, double> score;
        auto weight = [&](int f) -> double { return w.count(f) ? w.at(f) : 0.0; };
        for (int f : friends) {
            const Prof* pf = find(f);
            if (!pf) continue;
            double wf = weight(f);
            if (wf <= 0.0) continue;
            for (uint32_t c : pf->clubs) if (!own.count((int)c)) score[(int)c] += wf;
        }
        for (int f : friends) {
            const std::vector<int>* ff = nbrs(f);
            if (!ff) continue;
            const Prof* pf = find(f);
            if (!pf) continue;
            double wf = weight(f);
            if (wf <= 0.0) continue;
            for (int x : *ff) {
                if (x == u) continue;
                const Prof* px = find(x);
                if (!px) continue;
                double s = fas(*pf, *px);
                if (s <= 0.0) continue;
                double add = wf * s;
                for (uint32_t c : px->clubs) if (!own.count((int)c)) score[(int)c] += add;
            }
        }
        for (auto& kv : score) out.emplace_back(kv.first, (float)kv.second);
        rank_and_cut(out, topk);
        return out;
    }
};

namespace {

int emit(const Ranked& r, int i, int topk, int32_t* ou, float* os, int32_t* oc) {
    int n = std::min<int>((int)r.size(), topk);
    for (int k = 0; k < n; ++k) {
        ou[(int64_t)i * topk + k] = r[k].first;
        os[(int64_t)i * topk + k] = r[k].second;
    }
    oc[i] = n;
    return n;
}

// pf_result_digest (pokec_io.h) of a ranked list
uint64_t ranked_digest(const Ranked& r) {
    std::vector<int32_t> ids;
    std::vector<float> sc;
    for (const auto& p : r) {
        ids.push_back(p.first);
        sc.push_back(p.second);
    }
    return pf_result_digest(ids.data(), sc.data(), (int32_t)ids.size());
}

}  // namespace

extern "C" {

int ro_open(const pf_corpus_desc* d, int32_t max_users, ro_ctx** out) {
    if (!d || !out || d->n_users < 0 || d->n_cols < 0 || d->n_cols > PF_MAX_COLS) return PF_EINVAL;
    ro_ctx* h = new ro_ctx();
    const int T = d->n_cols;
    h->T = T;
    int n = d->n_users;
    if (max_users > 0 && max_users < n) n = max_users;
    for (int i = 0; i < n; ++i) {
        Prof p;
        p.uid = d->user_id[i];
        p.pub = d->public_flag[i];
        p.comp = d->completion[i];
        p.gen = d->gender[i];
        p.age = d->age[i];
        for (int k = 0; k < 3; ++k) p.reg[k] = d->region[3 * (int64_t)i + k];
        p.clubs.assign(d->club_ids + d->club_off[i], d->club_ids + d->club_off[i + 1]);
        p.friends.assign(d->friend_ids + d->friend_off[i], d->friend_ids + d->friend_off[i + 1]);
        p.cols.resize(T);
        for (int t = 0; t < T; ++t) {
            int64_t r = (int64_t)i * T + t;
            for (int64_t k = d->tok_off[r]; k < d->tok_off[r + 1]; ++k) p.cols[t][d->tok_tid[k]] = d->tok_tf[k];
        }
        h->prof[p.uid] = std::move(p);  // user_loader.cpp:91
    }
    for (int a = 0; a < d->n_adj; ++a) {
        std::vector<int>& row = h->adj[d->adj_uid[a]];
        row.insert(row.end(), d->adj_nbr + d->adj_off[a], d->adj_nbr + d->adj_off[a + 1]);
    }
    h->idf.assign(T, {});
    h->has_idf.assign(T, 1);
    if (d->idf_mode == PF_IDF_EXPLICIT) {
        for (int t = 0; t < T; ++t) {
            h->has_idf[t] = d->col_has_idf ? d->col_has_idf[t] : 1;
            if (!h->has_idf[t] || !d->idf_off) continue;
            for (int64_t k = d->idf_off[t]; k < d->idf_off[t + 1]; ++k) h->idf[t][d->idf_tid[k]] = d->idf_val[k];
        }
    } else {  // recommender.cpp:43-66
        const float N = (float)h->prof.size();
        for (int t = 0; t < T; ++t) {
            std::unordered_map<int, int> df;
            for (const auto& kv : h->prof)
                for (const auto& e : kv.second.cols[t]) df[e.first] += 1;
            for (const auto& e : df) h->idf[t][e.first] = logf(1.0f + N / (1.0f + (float)e.second));
        }
    }
    const int K = PF_NUM_FIXED + T;
    h->npres.assign(K, 0);
    h->nmean.assign(K, 0.f);
    h->nsd.assign(K, 0.f);
    if (d->norm_present)
        for (int k = 0; k < K; ++k) {
            h->npres[k] = d->norm_present[k];
            h->nmean[k] = d->norm_mean[k];
            h->nsd[k] = d->norm_sd[k];
        }
    *out = h;
    return PF_OK;
}

void ro_close(ro_ctx* h) { delete h; }
int64_t ro_fas_calls(ro_ctx* h, int reset) {
    const int64_t n = h->fas_calls;
    if (reset) h->fas_calls = 0;
    return n;
}
int32_t ro_num_users(const ro_ctx* h) { return (int32_t)h->prof.size(); }

float ro_idf(const ro_ctx* h, int32_t col, int32_t tid) {
    if (col < 0 || col >= h->T || !h->has_idf[col]) return NAN;
    auto it = h->idf[col].find(tid);
    return it == h->idf[col].end() ? 1.0f : it->second;
}

int ro_fas_pairs(ro_ctx* h, const int32_t* a, const int32_t* b, int64_t n, float* out) {
    for (int64_t i = 0; i < n; ++i) {
        const Prof* pa = h->find(a[i]);
        const Prof* pb = h->find(b[i]);
        out[i] = (pa && pb) ? h->fas(*pa, *pb) : NAN;
    }
    return PF_OK;
}

int ro_recommend_interest(ro_ctx* h, const int32_t* q, int32_t nq, int32_t topk, int32_t mode, int32_t limit,
                          int32_t* ou, float* os, int32_t* oc) {
    for (int i = 0; i < nq; ++i)
        emit(mode == PF_MODE_ALL ? h->rec_all(q[i], topk) : h->rec_graph(q[i], topk, limit), i, topk, ou, os, oc);
    return PF_OK;
}
int ro_recommend_collab(ro_ctx* h, const int32_t* q, int32_t nq, int32_t topk, int32_t limit,
                        int32_t* ou, float* os, int32_t* oc) {
    for (int i = 0; i < nq; ++i) emit(h->rec_collab(q[i], topk, limit), i, topk, ou, os, oc);
    return PF_OK;
}
int ro_recommend_clubs(ro_ctx* h, const int32_t* q, int32_t nq, int32_t topk, int32_t limit,
                       int32_t* ou, float* os, int32_t* oc) {
    for (int i = 0; i < nq; ++i) emit(h->rec_clubs(q[i], topk, limit), i, topk, ou, os, oc);
    return PF_OK;
}

int ro_fof_candidates(ro_ctx* h, int32_t uid, int32_t limit, int32_t flavour, int32_t* out, int32_t cap, int32_t* n) {
    std::vector<int> v = flavour == PF_FOF_COLLAB ? h->gather_collab(uid, limit) : h->gather_graph(uid, limit);
    for (int i = 0; i < (int)v.size() && i < cap; ++i) out[i] = v[i];
    *n = (int32_t)v.size();
    return PF_OK;
}

int ro_set_adj(ro_ctx* h, int32_t uid, const int32_t* nbrs, int32_t n) {
    if (n < 0) { h->adj.erase(uid); return PF_OK; }
    h->adj[uid].assign(nbrs, nbrs + n);
    return PF_OK;
}

int ro_profile_order(const ro_ctx* h, int32_t* out, int32_t cap) {
    int i = 0;
    for (const auto& kv : h->prof) { if (i < cap) out[i] = kv.first; ++i; }
    return i;
}

}  // extern "C"

namespace {

// test.cpp:13-105 — 20% of each eligible user's friends held out, cumulative adj edits.
// digest (may be null): per tested user the pf_result_digest of its collaborative list.
int holdout_friends(ro_ctx* h, int32_t sample, double* ratios, uint64_t* digest, int32_t cap, int32_t* n) {
    std::vector<int> elig;
    for (const auto& kv : h->prof) {
        const std::vector<int>* fr = h->nbrs(kv.first);
        if (fr && fr->size() >= 20) elig.push_back(kv.first);
    }
    *n = 0;
    if (elig.empty()) return PF_OK;
    std::mt19937 rng(1234567);
    std::shuffle(elig.begin(), elig.end(), rng);
    std::unordered_map<int, std::vector<int>> original = h->adj;  // the driver reads the untouched list
    int taken = 0;
    for (int u : elig) {
        if (taken >= sample) break;
        const std::vector<int>& fr = original.at(u);
        int F = (int)fr.size();
        if (F < 2) continue;
        int hold = F / 5;
        if (hold <= 0) continue;
        std::vector<int> idx(F);
        for (int i = 0; i < F; ++i) idx[i] = i;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::unordered_set<int> held;
        for (int i = 0; i < hold; ++i) held.insert(fr[idx[i]]);
        std::vector<int> kept;
        for (int f : fr) if (!held.count(f)) kept.push_back(f);
        h->adj[u] = std::move(kept);
        Ranked pred = h->rec_collab(u, hold, 1000);
        int hits = 0;
        for (size_t i = 0; i < pred.size() && (int)i < hold; ++i) hits += held.count(pred[i].first) ? 1 : 0;
        if (ratios && taken < cap) ratios[taken] = (double)hits / (double)hold;
        if (digest && taken < cap) digest[taken] = ranked_digest(pred);
        ++taken;
    }
    h->adj = std::move(original);
    *n = taken;
    return PF_OK;
}

// recommendation_tests.cpp:68-169 — per-user fresh adjacency copy, four recommenders.
// digest (may be null): per tested user i, digest[4i .. 4i+3] = graph, collab, interest, clubs.
int recommendation_tests(ro_ctx* h, int32_t sample, int32_t topk, double* metrics, uint64_t* digest, int32_t cap,
                         int32_t* n) {
    for (int k = 0; k < 5; ++k) metrics[k] = 0.0;
    if (n) *n = 0;
    if (h->prof.empty() || h->adj.empty()) return PF_OK;
    std::vector<int> all;
    for (const auto& kv : h->prof) all.push_back(kv.first);
    std::mt19937 rng(1234567);
    std::shuffle(all.begin(), all.end(), rng);
    std::unordered_map<int, std::vector<int>> original = h->adj;
    int taken = 0, hg = 0, hc = 0, hi = 0, club_users = 0;
    double prec = 0, rec = 0;
    for (int u : all) {
        if (taken >= sample) break;
        auto it = original.find(u);
        if (it == original.end()) continue;
        const std::vector<int>& fr = it->second;
        if (fr.size() < 4) continue;
        int hold = std::max(1, (int)fr.size() / 4);
        std::vector<int> idx(fr.size());
        for (size_t i = 0; i < fr.size(); ++i) idx[i] = (int)i;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::unordered_set<int> held;
        for (int i = 0; i < hold; ++i) held.insert(fr[idx[i]]);
        h->adj = original;
        std::vector<int> kept;
        for (int f : fr) if (!held.count(f)) kept.push_back(f);
        h->adj[u] = kept;
        auto any_hit = [&](const Ranked& r) {
            for (auto& p : r) if (held.count(p.first)) return true;
            return false;
        };
        const Ranked rg = h->rec_graph(u, topk, 5000), rc = h->rec_collab(u, topk, 5000), ri = h->rec_graph(u, topk, 5000);
        hg += any_hit(rg);
        hc += any_hit(rc);
        hi += any_hit(ri);
        Ranked cp = h->rec_clubs(u, topk, 5000);
        if (digest && taken < cap) {
            uint64_t* d = digest + 4 * (size_t)taken;
            d[0] = ranked_digest(rg);
            d[1] = ranked_digest(rc);
            d[2] = ranked_digest(ri);
            d[3] = ranked_digest(cp);
        }
        std::unordered_set<int> own;
        for (uint32_t c : h->prof.at(u).clubs) own.insert((int)c);
        if (!own.empty()) {
            int got = 0;
            for (size_t i = 0; i < cp.size() && i < (size_t)topk; ++i) got += own.count(cp[i].first) ? 1 : 0;
            prec += (double)got / (double)topk;
            rec += (double)got / (double)own.size();
            ++club_users;
        }
        ++taken;
    }
    h->adj = std::move(original);
    if (taken > 0) {
        metrics[0] = (double)hg / taken;
        metrics[1] = (double)hc / taken;
        metrics[2] = (double)hi / taken;
    }
    if (club_users > 0) {
        metrics[3] = prec / club_users;
        metrics[4] = rec / club_users;
    }
    if (n) *n = taken;
    return PF_OK;
}

}  // namespace

extern "C" {

int ro_holdout_friends(ro_ctx* h, int32_t sample, double* ratios, int32_t cap, int32_t* n) {
    return holdout_friends(h, sample, ratios, nullptr, cap, n);
}
int ro_holdout_friends_digest(ro_ctx* h, int32_t sample, uint64_t* digest, int32_t cap, int32_t* n) {
    return holdout_friends(h, sample, nullptr, digest, cap, n);
}
int ro_recommendation_tests(ro_ctx* h, int32_t sample, int32_t topk, double* metrics) {
    return recommendation_tests(h, sample, topk, metrics, nullptr, 0, nullptr);
}
int ro_recommendation_tests_digest(ro_ctx* h, int32_t sample, int32_t topk, uint64_t* digest, int32_t cap,
                                   int32_t* n) {
    double m[5];
    return recommendation_tests(h, sample, topk, m, digest, cap, n);
}

}  // extern "C"
