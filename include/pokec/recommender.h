// pokec/recommender.h — C++ drop-in for the reference's `Recommender` class
// (include/recommender.h:17-71) over the MI355X engine's C ABI (pokec_fas.h).
//
// Same construction (non-owning pointers to the profiles map and adj_list), same
// setters, same recommender signatures and results (bit-identical scores, same
// order); the scoring runs on the GPU.  Header-only; link libpokec_fas.so.
//
// The class is a template over the profile type, pokec::BasicRecommender<Profile>; any
// struct with the reference's UserProfile fields (include/user_profile.h:10-20) works.
//   - pokec::Recommender = BasicRecommender<pokec::UserProfile> (this header's twin struct);
//   - drop-in mode: a translation unit that includes the reference's user_profile.h and
//     defines POKEC_DROP_IN before this header gets ::Recommender =
//     BasicRecommender<::UserProfile>, so the reference's own call sites (api_cli.cpp:155-234,
//     test.cpp:36-75, recommendation_tests.cpp:50-140) compile unchanged against the engine.
//
// Differences a caller must know:
//   - The engine snapshots the maps when it first scores (pf_open copies them to
//     HBM).  The reference reads *adj_list live, so a caller that mutates the
//     adjacency afterwards (the hold-out drivers' adj_mod) calls
//     sync_adjacency(uid) for each row it changed.  Profiles and normalisers are
//     also fixed at that point; a setter called later re-opens the engine.
//   - profile_similarity(A, B[, text_columns]) scores two profiles OF THE MAP (by
//     user_id), which is how every reference caller uses it.  It returns NaN otherwise.
//     With a text_columns list other than set_text_columns', a second engine context is
//     opened (once per distinct list) with that list as its columns.
//   - The legacy user_feats constructor and recommend_from_supernodes
//     (recommender_clubs.cpp:75-...) are not provided: no live caller uses them
//     (SURVEY.md §8 A12).
//   - No exceptions cross it either: an engine failure yields an empty result,
//     and last_error() says why.
#ifndef POKEC_RECOMMENDER_H
#define POKEC_RECOMMENDER_H

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "pokec_fas.h"

namespace pokec {

// include/user_profile.h:10-20
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

template <class Profile>
class BasicRecommender {
public:
    using Ranked = std::vector<std::pair<int, float>>;
    using NormMap = std::unordered_map<std::string, std::pair<float, float>>;
    using IdfMap = std::unordered_map<std::string, std::unordered_map<int, float>>;

    BasicRecommender(const std::unordered_map<int, Profile>* profiles_in,
                     const std::unordered_map<int, std::vector<int>>* al, int device = 0)
        : profiles(profiles_in), adj_list(al), device_(device) {
        total_users = profiles ? profiles->size() : 0;
    }
    ~BasicRecommender() { close_(); }
    BasicRecommender(const BasicRecommender&) = delete;
    BasicRecommender& operator=(const BasicRecommender&) = delete;

    // recommender.cpp:27-41
    void set_field_normalizers(const NormMap& m) { field_normalizers = m; close_(); }
    void set_column_normalizers(const NormMap& m) { column_normalizers = m; close_(); }
    void set_text_columns(const std::vector<std::string>& cols) { text_columns_internal_ = cols; close_(); }
    void set_tfidf_index(const IdfMap& idf_map) {
        idf_per_col = idf_map;
        idf_cols_.clear();
        idf_explicit_ = true;
        close_();
    }
    // recommender.cpp:43-66: computed by the engine at open (float32 logf, N = |profiles|)
    void compute_idf_from_profiles(const std::vector<std::string>& text_columns) {
        idf_cols_ = text_columns;
        idf_explicit_ = false;
        idf_per_col.clear();
        total_users = profiles ? profiles->size() : 0;
        close_();
    }

    // recommender_graph.cpp:33-103,224-227
    Ranked recommend_graph_registration(int user, int topk, int candidate_limit = 10000) const {
        return run_(0, user, topk, candidate_limit);
    }
    Ranked recommend_by_interest(int user, int topk, int candidate_limit = 10000) const {
        return run_(0, user, topk, candidate_limit);
    }
    // recommender_graph.cpp:105-222
    Ranked recommend_collaborative(int user, int topk, int candidate_limit = 10000) const {
        return run_(1, user, topk, candidate_limit);
    }
    // recommender_clubs.cpp:10-73 (ids are club ids)
    Ranked recommend_clubs_collab(int user, int topk, int candidate_limit = 10000) const {
        return run_(2, user, topk, candidate_limit);
    }
    // recommender_graph.cpp:229-237
    Ranked recommend_friends_graph(int user, int topk, int candidate_limit = 10000) const {
        return recommend_graph_registration(user, topk, candidate_limit);
    }
    Ranked recommend_friends_collab(int user, int topk, int candidate_limit = 10000) const {
        return recommend_collaborative(user, topk, candidate_limit);
    }
    Ranked recommend_friends_by_interest(int user, int topk, int candidate_limit = 10000) const {
        return recommend_by_interest(user, topk, candidate_limit);
    }
    // Build-defined all-candidates interest scan: every profile but the
    // user and its adj_list row, one GPU pass.
    Ranked recommend_interest_all(int user, int topk) const { return run_(3, user, topk, 0); }

    // recommender_similarity.cpp:10-124,126-128, for two profiles of the map
    float profile_similarity(const Profile& A, const Profile& B) const {
        if (!open_()) return NAN;
        const int32_t a = A.user_id, b = B.user_id;
        float out = NAN;
        if (pf_fas_pairs(ctx_, &a, &b, 1, &out) != PF_OK) return NAN;
        return out;
    }
    // recommender_similarity.cpp:10-124 over a caller-given column list (include/recommender.h:41):
    // its names pick the normalisers and idf maps, its length the columns compared and F's
    // denominator.  The set_text_columns list is the context's own; another list opens (once)
    // a second context with that list.
    float profile_similarity(const Profile& A, const Profile& B, const std::vector<std::string>& text_columns) const {
        if (text_columns == text_columns_internal_) return profile_similarity(A, B);
        auto it = alt_.find(text_columns);
        if (it == alt_.end()) {
            pf_ctx* c = nullptr;
            if (!open_with_(text_columns, &c)) return NAN;
            it = alt_.emplace(text_columns, c).first;
        }
        const int32_t a = A.user_id, b = B.user_id;
        float out = NAN;
        if (pf_fas_pairs(it->second, &a, &b, 1, &out) != PF_OK) return NAN;
        return out;
    }

    // Re-read adj_list row `uid` into the engine (a caller mutated *adj_list).
    int sync_adjacency(int uid) const {
        if (!adj_list || !open_()) return PF_ENODEV;
        auto it = adj_list->find(uid);
        if (it == adj_list->end()) return pf_set_adj(ctx_, uid, nullptr, -1);
        return pf_set_adj(ctx_, uid, it->second.data(), (int32_t)it->second.size());
    }

    const std::string& last_error() const { return err_; }
    pf_ctx* engine() const { return open_() ? ctx_ : nullptr; }

    // the reference's public data members (include/recommender.h:49-60)
    const std::unordered_map<int, Profile>* profiles = nullptr;
    const std::unordered_map<int, std::vector<int>>* adj_list = nullptr;
    NormMap field_normalizers;
    NormMap column_normalizers;
    IdfMap idf_per_col;
    size_t total_users = 0;

private:
    Ranked run_(int kind, int user, int topk, int limit) const {
        Ranked out;
        if (!profiles || !adj_list || topk <= 0 || !open_()) return out;
        // a result never holds more than every profile (or every club entry): size the
        // buffers by that, not by topk (the reference's callers pass up to 2^30)
        topk = (int)std::min<int64_t>(topk, kind == 2 ? n_club_entries_ + 1 : (int64_t)n_users_ + 1);
        std::vector<int32_t> ids((size_t)topk);
        std::vector<float> sc((size_t)topk);
        int32_t n = 0;
        const int32_t q = user;
        int rc;
        switch (kind) {
            case 0: rc = pf_recommend_interest(ctx_, &q, 1, topk, PF_MODE_FOF, limit, ids.data(), sc.data(), &n); break;
            case 1: rc = pf_recommend_collab(ctx_, &q, 1, topk, limit, ids.data(), sc.data(), &n); break;
            case 2: rc = pf_recommend_clubs(ctx_, &q, 1, topk, limit, ids.data(), sc.data(), &n); break;
            default: rc = pf_recommend_interest(ctx_, &q, 1, topk, PF_MODE_ALL, 0, ids.data(), sc.data(), &n); break;
        }
        if (rc != PF_OK) {
            err_ = pf_last_error(ctx_);
            return out;
        }
        out.reserve((size_t)n);
        for (int i = 0; i < n; ++i) out.emplace_back(ids[i], sc[i]);
        return out;
    }

    void close_() const {
        if (ctx_) pf_close(ctx_);
        ctx_ = nullptr;
        for (auto& kv : alt_) pf_close(kv.second);
        alt_.clear();
    }

    bool open_() const {
        if (ctx_) return true;
        if (!open_with_(text_columns_internal_, &ctx_)) return false;
        return true;
    }

    // Flatten the maps into a pf_corpus_desc over column list `cols` and open an engine context.
    bool open_with_(const std::vector<std::string>& cols, pf_ctx** out) const {
        if (!profiles || !adj_list) { err_ = "null profiles or adj_list"; return false; }
        const int T = (int)cols.size();
        D& d = d_;
        d = D();
        const size_t n = profiles->size();
        d.club_off.push_back(0); d.friend_off.push_back(0); d.tok_off.push_back(0);
        for (auto& kv : *profiles) {
            const Profile& p = kv.second;
            d.uid.push_back(kv.first); d.pub.push_back(p.public_flag); d.comp.push_back(p.completion_percentage);
            d.gen.push_back(p.gender); d.age.push_back(p.age);
            for (int k = 0; k < 3; ++k) d.reg.push_back(p.region_parts[k]);
            d.clubs.insert(d.clubs.end(), p.clubs.begin(), p.clubs.end());
            d.club_off.push_back((int64_t)d.clubs.size());
            d.friends.insert(d.friends.end(), p.friends.begin(), p.friends.end());
            d.friend_off.push_back((int64_t)d.friends.size());
            for (int t = 0; t < T; ++t) {
                if ((size_t)t < p.token_cols.size())
                    for (auto& pr : p.token_cols[t]) { d.tid.push_back(pr.first); d.tf.push_back(pr.second); }
                d.tok_off.push_back((int64_t)d.tid.size());
            }
        }
        d.adj_off.push_back(0);
        for (auto& kv : *adj_list) {
            d.adj_uid.push_back(kv.first);
            d.adj_nbr.insert(d.adj_nbr.end(), kv.second.begin(), kv.second.end());
            d.adj_off.push_back((int64_t)d.adj_nbr.size());
        }
        static const char* const keys[PF_NUM_FIXED] = {"public", "gender", "completion", "age",
                                                       "region", "clubs", "friends"};
        d.npres.assign(PF_NUM_FIXED + T, 0);
        d.nmean.assign(PF_NUM_FIXED + T, 0.f);
        d.nsd.assign(PF_NUM_FIXED + T, 0.f);
        for (int k = 0; k < PF_NUM_FIXED + T; ++k) {
            const NormMap& m = k < PF_NUM_FIXED ? field_normalizers : column_normalizers;
            auto it = m.find(k < PF_NUM_FIXED ? std::string(keys[k]) : cols[k - PF_NUM_FIXED]);
            if (it == m.end()) continue;
            d.npres[k] = 1; d.nmean[k] = it->second.first; d.nsd[k] = it->second.second;
        }
        pf_corpus_desc c{};
        c.n_users = (int32_t)n; c.n_cols = T;
        c.user_id = d.uid.data(); c.public_flag = d.pub.data(); c.completion = d.comp.data();
        c.gender = d.gen.data(); c.age = d.age.data(); c.region = d.reg.data();
        c.club_off = d.club_off.data(); c.club_ids = d.clubs.data();
        c.friend_off = d.friend_off.data(); c.friend_ids = d.friends.data();
        c.tok_off = d.tok_off.data(); c.tok_tid = d.tid.data(); c.tok_tf = d.tf.data();
        c.n_adj = (int32_t)d.adj_uid.size();
        c.adj_uid = d.adj_uid.data(); c.adj_off = d.adj_off.data(); c.adj_nbr = d.adj_nbr.data();
        c.norm_present = d.npres.data(); c.norm_mean = d.nmean.data(); c.norm_sd = d.nsd.data();
        if (!idf_explicit_ && idf_cols_ == cols) {  // recommender.cpp:43-66 over the same columns
            c.idf_mode = PF_IDF_FROM_PROFILES;
        } else {
            // explicit maps: set_tfidf_index, or IDF computed over another column list
            // (idf_per_col keyed by name, recommender_similarity.cpp:97-104)
            IdfMap computed;
            const IdfMap* src = &idf_per_col;
            if (!idf_explicit_) {
                compute_idf_(computed);
                src = &computed;
            }
            c.idf_mode = PF_IDF_EXPLICIT;
            d.has_idf.assign(T, 0);
            d.idf_off.push_back(0);
            for (int t = 0; t < T; ++t) {
                auto it = src->find(cols[t]);
                if (it != src->end()) {
                    d.has_idf[t] = 1;
                    for (auto& pr : it->second) { d.idf_tid.push_back(pr.first); d.idf_val.push_back(pr.second); }
                }
                d.idf_off.push_back((int64_t)d.idf_tid.size());
            }
            c.col_has_idf = d.has_idf.data(); c.idf_off = d.idf_off.data();
            c.idf_tid = d.idf_tid.data(); c.idf_val = d.idf_val.data();
        }
        if (pf_open(&c, device_, out) != PF_OK) {
            err_ = pf_last_error(nullptr);
            *out = nullptr;
            return false;
        }
        n_users_ = (int64_t)n;
        n_club_entries_ = (int64_t)d.clubs.size();
        d_ = D();  // the engine copied everything
        return true;
    }

    // recommender.cpp:43-66 over idf_cols_ (only when it differs from the scoring columns)
    void compute_idf_(IdfMap& out) const {
        const float N = (float)profiles->size();
        for (size_t t = 0; t < idf_cols_.size(); ++t) {
            std::unordered_map<int, int> df;
            for (auto& kv : *profiles)
                if (t < kv.second.token_cols.size())
                    for (auto& pr : kv.second.token_cols[t]) df[pr.first] += 1;
            std::unordered_map<int, float> m;
            for (auto& pr : df) m[pr.first] = logf(1.0f + N / (1.0f + (float)pr.second));
            out[idf_cols_[t]] = std::move(m);
        }
    }

    struct D {
        std::vector<int32_t> uid, pub, comp, gen, age, reg, tid, tf, adj_uid, adj_nbr, idf_tid;
        std::vector<int64_t> club_off, friend_off, tok_off, adj_off, idf_off;
        std::vector<uint32_t> clubs, friends;
        std::vector<uint8_t> npres, has_idf;
        std::vector<float> nmean, nsd, idf_val;
    };

    int device_ = 0;
    std::vector<std::string> text_columns_internal_;
    std::vector<std::string> idf_cols_;
    bool idf_explicit_ = false;
    mutable pf_ctx* ctx_ = nullptr;
    mutable std::map<std::vector<std::string>, pf_ctx*> alt_;  // 3-argument profile_similarity lists
    mutable int64_t n_users_ = 0, n_club_entries_ = 0;
    mutable D d_;
    mutable std::string err_;
};

using Recommender = BasicRecommender<UserProfile>;

}  // namespace pokec

#ifdef POKEC_DROP_IN
// the reference's names: ::UserProfile is the caller's (the reference's user_profile.h)
using Recommender = pokec::BasicRecommender<::UserProfile>;
#endif

#endif  // POKEC_RECOMMENDER_H
