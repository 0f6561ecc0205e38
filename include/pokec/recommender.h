// pokec/recommender.h — C++ drop-in for the reference's `Recommender` class
// (include/recommender.h:17-71) over the MI355X engine's C ABI (pokec_fas.h).
//
// Same construction (non-owning pointers to the profiles map and adj_list), same
// setters, same public data members, same recommender signatures and results
// (bit-identical scores, same order); the scoring runs on the GPU.  Header-only; link
// libpokec_fas.so.
//
// The class is a template over the profile type, pokec::BasicRecommender<Profile>; any
// struct with the reference's UserProfile fields (include/user_profile.h:10-20) works.
//   - pokec::Recommender = BasicRecommender<pokec::UserProfile> (this header's twin struct);
//   - drop-in mode: a translation unit that includes the reference's user_profile.h and
//     defines POKEC_DROP_IN before this header gets ::Recommender =
//     BasicRecommender<::UserProfile>, so the reference's own call sites (api_cli.cpp:155-234,
//     test.cpp:35-75, recommendation_tests.cpp:111-140) compile and behave unchanged.
//
// How it keeps the reference's behaviour:
//   - adj_list is read live, as the reference reads *adj_list: before every recommender call
//     the rows that call reads (the user's row and its friends' rows, recommender_graph.cpp:
//     10-31,114-125, recommender_clubs.cpp:47-58) are compared with the engine's copy and the
//     changed ones are pushed with pf_set_adj.  That is O(sum of those rows), the order of the
//     reference's own walk, so a caller that mutates its adj_mod between calls (test.cpp:73) or
//     builds a fresh Recommender over a fresh adj_mod per user (recommendation_tests.cpp:111-116)
//     needs no extra call.
//   - One engine context (a full HBM replica, pf_open) is shared by every Recommender over the
//     same profiles map, device, text columns, normalisers and idf values, whatever adjacency
//     map each one reads: constructing a Recommender costs a lookup, not a pf_open.  Engines stay
//     open for reuse (at most kMaxEngines idle ones) until release_engines().
//   - compute_idf_from_profiles fills the public idf_per_col on the host with the reference's
//     float32 logf (recommender.cpp:43-66), so callers that copy it (test.cpp:40,
//     recommendation_tests.cpp:120: set_tfidf_index(base_rec.idf_per_col)) see the reference's
//     map; an explicit map equal to the computed one shares the computed engine.
//   - The recommenders are const and may be called from several threads at once on one object
//     or on objects sharing an engine: the engine's calls are serialised by its mutex, and the
//     lazy open is guarded.
//
// Differences a caller must know:
//   - The profiles map (and the normalisers and idf values) are snapshotted when an engine is
//     opened for them; the reference reads *profiles live, but none of its callers mutates the
//     profiles after construction.
//   - profile_similarity(A, B[, text_columns]) scores two profiles OF THE MAP (by user_id), which
//     is how every reference caller uses it.  It returns NaN otherwise.  A text_columns list other
//     than set_text_columns' uses the engine for that list.
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
#include <list>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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

using NormMap = std::unordered_map<std::string, std::pair<float, float>>;
using IdfMap = std::unordered_map<std::string, std::unordered_map<int, float>>;
using AdjMap = std::unordered_map<int, std::vector<int>>;

namespace detail {

// One engine context and the adjacency rows it currently holds.
struct Engine {
    pf_ctx* ctx = nullptr;
    std::mutex mu;  // pokec_fas.h: calls on one context are serialised
    AdjMap rows;    // the engine's adj_list (the open-time rows plus every pf_set_adj since)
    int64_t n_users = 0, n_club_entries = 0;
    Engine() = default;
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    ~Engine() {
        if (ctx) pf_close(ctx);
    }
};

// What an engine was opened for; idf = the values it scores with, compared by content.
struct EngineKey {
    const void* profiles = nullptr;
    size_t n_profiles = 0;
    uint64_t fingerprint = 0;  // a content sample of the map (a recycled address is not reused blindly)
    int device = 0;
    std::vector<std::string> cols;
    NormMap field, column;
    std::shared_ptr<const IdfMap> idf;
    bool same(const EngineKey& o) const {
        return profiles == o.profiles && n_profiles == o.n_profiles && fingerprint == o.fingerprint &&
               device == o.device && cols == o.cols &&
               field == o.field && column == o.column && (idf == o.idf || *idf == *o.idf);
    }
};

// FNV-1a over the first (up to) 64 profiles in the map's iteration order: ids, scalar fields and
// list sizes. O(64) per engine lookup; tells a profiles map destroyed and re-created at the same
// address with the same size from the one the engine was opened for.
template <class Map>
uint64_t profiles_fingerprint(const Map& m) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](int64_t v) {
        for (int i = 0; i < 8; ++i) { h ^= (uint64_t)(v >> (8 * i)) & 0xFFu; h *= 1099511628211ull; }
    };
    int n = 0;
    for (auto it = m.begin(); it != m.end() && n < 64; ++it, ++n) {
        const auto& p = it->second;
        mix(it->first); mix(p.public_flag); mix(p.completion_percentage); mix(p.gender); mix(p.age);
        mix((int64_t)p.clubs.size()); mix((int64_t)p.friends.size()); mix((int64_t)p.token_cols.size());
        for (const auto& c : p.token_cols) mix((int64_t)c.size());
    }
    return h;
}

struct Registry {
    std::mutex mu;
    std::list<std::pair<EngineKey, std::shared_ptr<Engine>>> engines;  // most recent first
};
// never destroyed: engines still registered at exit are not closed during static destruction
// (the HIP runtime may be gone by then); the OS reclaims them
inline Registry& registry() {
    static Registry* r = new Registry();
    return *r;
}

}  // namespace detail

// Engines no Recommender holds are kept for reuse, at most this many.
constexpr int kMaxEngines = 4;

// Closes every engine no Recommender holds (their HBM replicas are freed).
inline void release_engines() {
    auto& R = detail::registry();
    std::lock_guard<std::mutex> g(R.mu);
    R.engines.remove_if([](const std::pair<detail::EngineKey, std::shared_ptr<detail::Engine>>& e) {
        return e.second.use_count() == 1;
    });
}

template <class Profile>
class BasicRecommender {
public:
    using Ranked = std::vector<std::pair<int, float>>;
    using NormMap = pokec::NormMap;
    using IdfMap = pokec::IdfMap;

    BasicRecommender(const std::unordered_map<int, Profile>* profiles_in, const AdjMap* al, int device = 0)
        : profiles(profiles_in), adj_list(al), device_(device) {
        total_users = profiles ? profiles->size() : 0;
    }
    BasicRecommender(const BasicRecommender&) = delete;
    BasicRecommender& operator=(const BasicRecommender&) = delete;

    // recommender.cpp:27-41
    void set_field_normalizers(const NormMap& m) { field_normalizers = m; reset_(); }
    void set_column_normalizers(const NormMap& m) { column_normalizers = m; reset_(); }
    void set_text_columns(const std::vector<std::string>& cols) { text_columns_internal_ = cols; reset_(); }
    void set_tfidf_index(const IdfMap& idf_map) {
        idf_per_col = idf_map;
        idf_computed_ = false;
        reset_();
    }
    // recommender.cpp:43-66: df per column over the profiles, idf = logf(1 + N / (1 + df)) in
    // float32, N = |profiles|; the map the reference's callers copy (test.cpp:40)
    void compute_idf_from_profiles(const std::vector<std::string>& text_columns) {
        idf_per_col.clear();
        total_users = profiles ? profiles->size() : 0;
        if (profiles) compute_idf_(text_columns, idf_per_col);
        idf_cols_ = text_columns;
        idf_computed_ = true;
        reset_();
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
        return pair_(engine_(), A.user_id, B.user_id);
    }
    // recommender_similarity.cpp:10-124 over a caller-given column list (include/recommender.h:41):
    // its names pick the normalisers and idf maps, its length the columns compared and F's
    // denominator.
    float profile_similarity(const Profile& A, const Profile& B, const std::vector<std::string>& text_columns) const {
        if (text_columns == text_columns_internal_) return profile_similarity(A, B);
        return pair_(open_for_(text_columns), A.user_id, B.user_id);
    }

    // Push adj_list row `uid` to the engine now.  Never needed for correctness (every call
    // re-reads the rows it uses); kept for callers of the earlier facade.
    int sync_adjacency(int uid) const {
        std::shared_ptr<detail::Engine> e = engine_();
        if (!e || !adj_list) return PF_ENODEV;
        std::lock_guard<std::mutex> g(e->mu);
        return sync_row_(*e, uid);
    }

    const std::string& last_error() const {
        std::lock_guard<std::mutex> g(err_mu_);
        return err_;
    }
    pf_ctx* engine() const {
        std::shared_ptr<detail::Engine> e = engine_();
        return e ? e->ctx : nullptr;
    }

    // the reference's public data members (include/recommender.h:49-60)
    const std::unordered_map<int, Profile>* profiles = nullptr;
    const AdjMap* adj_list = nullptr;
    NormMap field_normalizers;
    NormMap column_normalizers;
    IdfMap idf_per_col;
    size_t total_users = 0;

private:
    Ranked run_(int kind, int user, int topk, int limit) const {
        Ranked out;
        if (!profiles || !adj_list || topk <= 0) return out;
        std::shared_ptr<detail::Engine> e = engine_();
        if (!e) return out;
        std::lock_guard<std::mutex> g(e->mu);
        // the rows this call reads, as the caller's adj_list holds them now
        int rc = sync_row_(*e, user);
        auto it = adj_list->find(user);
        if (it != adj_list->end() && kind != 3)
            for (int f : it->second)
                if (rc == PF_OK) rc = sync_row_(*e, f);
        if (rc != PF_OK) return fail_(e->ctx, out);
        // a result never holds more than every profile (or every club entry): size the
        // buffers by that, not by topk (the reference's callers pass up to 2^30)
        topk = (int)std::min<int64_t>(topk, kind == 2 ? e->n_club_entries + 1 : e->n_users + 1);
        std::vector<int32_t> ids((size_t)topk);
        std::vector<float> sc((size_t)topk);
        int32_t n = 0;
        const int32_t q = user;
        switch (kind) {
            case 0: rc = pf_recommend_interest(e->ctx, &q, 1, topk, PF_MODE_FOF, limit, ids.data(), sc.data(), &n); break;
            case 1: rc = pf_recommend_collab(e->ctx, &q, 1, topk, limit, ids.data(), sc.data(), &n); break;
            case 2: rc = pf_recommend_clubs(e->ctx, &q, 1, topk, limit, ids.data(), sc.data(), &n); break;
            default: rc = pf_recommend_interest(e->ctx, &q, 1, topk, PF_MODE_ALL, 0, ids.data(), sc.data(), &n); break;
        }
        if (rc != PF_OK) return fail_(e->ctx, out);
        out.reserve((size_t)n);
        for (int i = 0; i < n; ++i) out.emplace_back(ids[i], sc[i]);
        return out;
    }

    float pair_(const std::shared_ptr<detail::Engine>& e, int a, int b) const {
        if (!e) return NAN;
        std::lock_guard<std::mutex> g(e->mu);
        const int32_t x = a, y = b;
        float out = NAN;
        if (pf_fas_pairs(e->ctx, &x, &y, 1, &out) != PF_OK) return NAN;
        return out;
    }

    Ranked fail_(pf_ctx* c, Ranked& out) const {
        std::lock_guard<std::mutex> g(err_mu_);
        err_ = pf_last_error(c);
        return out;
    }

    // The engine's row of x := the caller's adj_list row of x (absent rows erased).
    int sync_row_(detail::Engine& e, int x) const {
        auto ci = adj_list->find(x);
        auto ei = e.rows.find(x);
        const bool cp = ci != adj_list->end(), ep = ei != e.rows.end();
        if (!cp && !ep) return PF_OK;
        if (cp && ep && ci->second == ei->second) return PF_OK;
        if (!cp) {
            e.rows.erase(ei);
            return pf_set_adj(e.ctx, x, nullptr, -1);
        }
        e.rows[x] = ci->second;
        static_assert(sizeof(int) == sizeof(int32_t), "adj_list rows pass as int32");
        return pf_set_adj(e.ctx, x, reinterpret_cast<const int32_t*>(ci->second.data()), (int32_t)ci->second.size());
    }

    void reset_() {
        std::lock_guard<std::mutex> g(open_mu_);
        eng_.reset();
    }

    std::shared_ptr<detail::Engine> engine_() const {
        std::lock_guard<std::mutex> g(open_mu_);
        if (!eng_) eng_ = open_for_(text_columns_internal_);
        return eng_;
    }

    // The shared engine for scoring columns `cols` with this object's settings (opened on first use).
    std::shared_ptr<detail::Engine> open_for_(const std::vector<std::string>& cols) const {
        if (!profiles || !adj_list) {
            std::lock_guard<std::mutex> g(err_mu_);
            err_ = "null profiles or adj_list";
            return nullptr;
        }
        detail::EngineKey key;
        key.profiles = profiles;
        key.n_profiles = profiles->size();
        key.fingerprint = detail::profiles_fingerprint(*profiles);
        key.device = device_;
        key.cols = cols;
        key.field = field_normalizers;
        key.column = column_normalizers;
        // the idf values by column name (recommender_similarity.cpp:97-104), whether computed
        // (compute_idf_from_profiles over these columns: the engine recomputes them, F3) or
        // explicit (set_tfidf_index): equal values score equally
        key.idf = std::make_shared<const IdfMap>(idf_per_col);
        const bool computed = idf_computed_ && idf_cols_ == cols;
        auto& R = detail::registry();
        std::lock_guard<std::mutex> g(R.mu);
        for (auto it = R.engines.begin(); it != R.engines.end(); ++it)
            if (it->first.same(key)) {
                R.engines.splice(R.engines.begin(), R.engines, it);  // most recently used first
                return R.engines.front().second;
            }
        auto e = std::make_shared<detail::Engine>();
        if (!open_with_(cols, computed, *e)) return nullptr;
        R.engines.emplace_front(std::move(key), e);
        int idle = 0;  // keep at most kMaxEngines engines nobody holds
        for (auto it = R.engines.begin(); it != R.engines.end();) {
            if (it->second.use_count() == 1 && ++idle > kMaxEngines) it = R.engines.erase(it);
            else ++it;
        }
        return e;
    }

    // Flatten the maps into a pf_corpus_desc over column list `cols` and open an engine context.
    bool open_with_(const std::vector<std::string>& cols, bool computed, detail::Engine& e) const {
        const int T = (int)cols.size();
        D d;
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
        if (computed) {  // recommender.cpp:43-66 over the same columns: the engine computes it (F3)
            c.idf_mode = PF_IDF_FROM_PROFILES;
        } else {
            c.idf_mode = PF_IDF_EXPLICIT;
            d.has_idf.assign(T, 0);
            d.idf_off.push_back(0);
            for (int t = 0; t < T; ++t) {
                auto it = idf_per_col.find(cols[t]);
                if (it != idf_per_col.end()) {
                    d.has_idf[t] = 1;
                    for (auto& pr : it->second) { d.idf_tid.push_back(pr.first); d.idf_val.push_back(pr.second); }
                }
                d.idf_off.push_back((int64_t)d.idf_tid.size());
            }
            c.col_has_idf = d.has_idf.data(); c.idf_off = d.idf_off.data();
            c.idf_tid = d.idf_tid.data(); c.idf_val = d.idf_val.data();
        }
        if (pf_open(&c, device_, &e.ctx) != PF_OK) {
            std::lock_guard<std::mutex> g(err_mu_);
            err_ = pf_last_error(nullptr);
            e.ctx = nullptr;
            return false;
        }
        e.rows = *adj_list;
        e.n_users = (int64_t)n;
        e.n_club_entries = (int64_t)d.clubs.size();
        return true;
    }

    // recommender.cpp:43-66, one column per thread (the counts and logf per column are the
    // reference's; only independent columns run side by side)
    void compute_idf_(const std::vector<std::string>& cols, IdfMap& out) const {
        const float N = (float)profiles->size();
        std::vector<std::unordered_map<int, float>> per(cols.size());
        auto col = [&](size_t t) {
            std::unordered_map<int, int> df;
            for (auto& kv : *profiles)
                if (t < kv.second.token_cols.size())
                    for (auto& pr : kv.second.token_cols[t]) df[pr.first] += 1;
            for (auto& pr : df) per[t][pr.first] = logf(1.0f + N / (1.0f + (float)pr.second));
        };
        const size_t nt = std::min<size_t>(cols.size(), std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
        std::vector<std::thread> ts;
        for (size_t w = 0; w < nt; ++w)
            ts.emplace_back([&, w]() {
                for (size_t t = w; t < cols.size(); t += nt) col(t);
            });
        for (auto& t : ts) t.join();
        for (size_t t = 0; t < cols.size(); ++t) out[cols[t]] = std::move(per[t]);
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
    bool idf_computed_ = false;
    mutable std::mutex open_mu_, err_mu_;
    mutable std::shared_ptr<detail::Engine> eng_;
    mutable std::string err_;
};

using Recommender = BasicRecommender<UserProfile>;

}  // namespace pokec

#ifdef POKEC_DROP_IN
// the reference's names: ::UserProfile is the caller's (the reference's user_profile.h)
using Recommender = pokec::BasicRecommender<::UserProfile>;
#endif

#endif  // POKEC_RECOMMENDER_H
