// pf_store.cpp — host side of the FAS engine: corpus ingestion from a
// pf_corpus_desc, float32 IDF (recommender.cpp:43-66), per-row candidate norms,
// the length-sorted tile-interleaved record stream, and per-query images with
// host-precomputed sigmoid tables (recommender_similarity.cpp:18-36).
#include "pf_store.h"

#include "pf_debug.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <numeric>
#include <mutex>
#include <thread>

namespace pf {

namespace {

template <class F>
void par_for(int64_t n, F f) {
    int th = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (n < 4096 || th <= 1) { f((int64_t)0, n); return; }
    std::vector<std::thread> ts;
    int64_t chunk = (n + th - 1) / th;
    for (int w = 0; w < th; ++w) {
        int64_t lo = w * chunk, hi = std::min(n, lo + chunk);
        if (lo >= hi) break;
        ts.emplace_back(f, lo, hi);
    }
    for (auto& t : ts) t.join();
}


// f(lo, hi) over [0, n) in chunks handed out dynamically (uneven work per item)
template <class F>
void par_dyn(int64_t n, int64_t chunk, F f) {
    const int th = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        for (;;) {
            const int64_t lo = next.fetch_add(chunk);
            if (lo >= n) return;
            f(lo, std::min(n, lo + chunk));
        }
    };
    std::vector<std::thread> ts;
    for (int w = 1; w < th; ++w) ts.emplace_back(work);
    work();
    for (auto& t : ts) t.join();
}

// v[k] = x for every k, on the par_for threads (the first touch of freshly mapped pages)
template <class V, class X>
void par_fill(V& v, const X& x) {
    auto* p = v.data();
    par_for((int64_t)v.size(), [&](int64_t lo, int64_t hi) { std::fill(p + lo, p + hi, x); });
}

// a[0] = 0 and a[k] = the length of item k - 1 (k >= 1) -> a[k] = the offset of item k, on threads
template <class V>
void par_offsets(V& a) {
    const int64_t n = (int64_t)a.size();
    const int th = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (n < (1 << 16) || th <= 1) {
        for (int64_t k = 1; k < n; ++k) a[k] += a[k - 1];
        return;
    }
    const int64_t chunk = (n + th - 1) / th;
    std::vector<int64_t> part(th + 1, 0);
    std::vector<std::thread> ts;
    for (int w = 0; w < th; ++w)
        ts.emplace_back([&, w]() {
            const int64_t lo = w * chunk, hi = std::min(n, lo + chunk);
            int64_t s = 0;
            for (int64_t k = lo; k < hi; ++k) s += a[k];
            part[w + 1] = s;
        });
    for (auto& t : ts) t.join();
    ts.clear();
    for (int w = 0; w < th; ++w) part[w + 1] += part[w];
    for (int w = 0; w < th; ++w)
        ts.emplace_back([&, w]() {
            const int64_t lo = w * chunk, hi = std::min(n, lo + chunk);
            int64_t s = part[w];
            for (int64_t k = lo; k < hi; ++k) { s += a[k]; a[k] = s; }
        });
    for (auto& t : ts) t.join();
}

// true when pred(k) holds for some k in [0, n), on the par_for threads
template <class P>
bool par_any(int64_t n, P pred) {
    std::atomic<bool> hit{false};
    par_for(n, [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi && !hit.load(std::memory_order_relaxed); ++k)
            if (pred(k)) { hit = true; break; }
    });
    return hit;
}

}  // namespace

// recommender_similarity.cpp:18-26 (stable two-branch logistic, double)
double ref_sigmoid(double x) {
    if (x >= 0) {
        double e = std::exp(-x);
        return 1.0 / (1.0 + e);
    }
    double e = std::exp(x);
    return e / (1.0 + e);
}

int32_t HostCorpus::idx_of(int32_t u) const {
    auto it = std::lower_bound(uid.begin(), uid.end(), u);
    if (it == uid.end() || *it != u) return -1;
    return (int32_t)(it - uid.begin());
}

float HostCorpus::idf_of(int t, int32_t rank) const {
    if (!has_idf[t]) return NAN;
    return (rank >= 0 && (size_t)rank < idf[t].size()) ? idf[t][rank] : 1.0f;
}

float HostCorpus::idf_of_tid(int t, int32_t k) const {
    if (!has_idf[t]) return NAN;
    const auto& v = tid_of_rank[t];
    auto it = std::lower_bound(v.begin(), v.end(), k);
    if (it != v.end() && *it == k) return idf_of(t, (int32_t)(it - v.begin()));
    auto e = idf_explicit[t].find(k);  // recommender.cpp:78: absent -> 1.0
    return e == idf_explicit[t].end() ? 1.0f : e->second;
}

int build_host_corpus(const pf_corpus_desc* d, HostCorpus& hc, std::string& err) {
    if (!d) { err = "null descriptor"; return PF_EINVAL; }
    if (d->n_users < 0 || d->n_cols < 0 || d->n_cols > kMaxCols) { err = "bad n_users/n_cols"; return PF_EINVAL; }
    const int32_t n = d->n_users, T = d->n_cols;
    if (n > 0 && (!d->user_id || !d->public_flag || !d->completion || !d->gender || !d->age || !d->region ||
                  !d->club_off || !d->friend_off || !d->tok_off)) {
        err = "missing profile arrays";
        return PF_EINVAL;
    }
    hc.n = n;
    hc.T = T;
    StageClock sc;
    // candidate index = rank of uid (ascending)
    std::vector<int32_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    if (par_any(n > 0 ? n - 1 : 0, [&](int64_t i) { return d->user_id[i + 1] < d->user_id[i]; }))  // loaders hand uid order
        std::sort(order.begin(), order.end(), [&](int a, int b) { return d->user_id[a] < d->user_id[b]; });
    for (int i = 1; i < n; ++i)
        if (d->user_id[order[i]] == d->user_id[order[i - 1]]) { err = "duplicate user id"; return PF_EINVAL; }
    hc.uid.resize(n); hc.pub.resize(n); hc.comp.resize(n); hc.gen.resize(n); hc.age.resize(n);
    hc.reg.resize(3 * (size_t)n);
    hc.club_off.assign(n + 1, 0); hc.friend_off.assign(n + 1, 0);
    hc.tok_off.resize_uninit((size_t)n * T + 1);  // every entry is written below
    hc.tok_off[0] = 0;
    par_for(n, [&](int64_t lo, int64_t hi) {  // fields and lengths, then the offsets
        for (int64_t i = lo; i < hi; ++i) {
            const int s = order[i];
            hc.uid[i] = d->user_id[s]; hc.pub[i] = d->public_flag[s]; hc.comp[i] = d->completion[s];
            hc.gen[i] = d->gender[s]; hc.age[i] = d->age[s];
            for (int k = 0; k < 3; ++k) hc.reg[3 * (size_t)i + k] = d->region[3 * (size_t)s + k];
            hc.club_off[i + 1] = d->club_off[s + 1] - d->club_off[s];
            hc.friend_off[i + 1] = d->friend_off[s + 1] - d->friend_off[s];
            for (int t = 0; t < T; ++t) {
                const int64_t r = (int64_t)s * T + t;
                hc.tok_off[(size_t)i * T + t + 1] = d->tok_off[r + 1] - d->tok_off[r];
            }
        }
    });
    par_offsets(hc.club_off);
    par_offsets(hc.friend_off);
    par_offsets(hc.tok_off);
    sc.lap("uid order + offsets");
    hc.clubs.resize(hc.club_off[n]); hc.friends.resize(hc.friend_off[n]);
    hc.tid.resize_uninit(hc.tok_off[(size_t)n * T]); hc.tf.resize_uninit(hc.tok_off[(size_t)n * T]);
    par_for(n, [&](int64_t lo, int64_t hi) {
        std::vector<std::pair<int32_t, int32_t>> row;
        for (int64_t i = lo; i < hi; ++i) {
            int s = order[i];
            if (hc.club_off[i + 1] > hc.club_off[i])
                std::memcpy(&hc.clubs[hc.club_off[i]], d->club_ids + d->club_off[s], sizeof(uint32_t) * (hc.club_off[i + 1] - hc.club_off[i]));
            if (hc.friend_off[i + 1] > hc.friend_off[i])
                std::memcpy(&hc.friends[hc.friend_off[i]], d->friend_ids + d->friend_off[s], sizeof(uint32_t) * (hc.friend_off[i + 1] - hc.friend_off[i]));
            // the user's rows are contiguous in both: one copy, then each (short) row sorted by tid
            const int64_t r0 = (int64_t)s * T, o0 = hc.tok_off[(size_t)i * T];
            const int64_t len = d->tok_off[r0 + T] - d->tok_off[r0];
            if (len > 0) {
                std::memcpy(&hc.tid[o0], d->tok_tid + d->tok_off[r0], sizeof(int32_t) * len);
                std::memcpy(&hc.tf[o0], d->tok_tf + d->tok_off[r0], sizeof(int32_t) * len);
            }
            for (int t = 0; t < T; ++t) {
                const int64_t a = hc.tok_off[(size_t)i * T + t], b = hc.tok_off[(size_t)i * T + t + 1];
                bool sorted = true;
                for (int64_t k = a + 1; k < b && sorted; ++k) sorted = hc.tid[k - 1] <= hc.tid[k];
                if (sorted) continue;
                row.clear();
                for (int64_t k = a; k < b; ++k) row.emplace_back(hc.tid[k], hc.tf[k]);
                std::sort(row.begin(), row.end());
                for (int64_t k = a; k < b; ++k) { hc.tid[k] = row[k - a].first; hc.tf[k] = row[k - a].second; }
            }
        }
    });
    sc.lap("rows copied + sorted");
    if (par_any((int64_t)n * T, [&](int64_t r) {
            for (int64_t k = hc.tok_off[r] + 1; k < hc.tok_off[r + 1]; ++k)
                if (hc.tid[k] == hc.tid[k - 1]) return true;
            return false;
        })) {
        err = "duplicate token id within a (user, column) row";
        return PF_EINVAL;
    }

    sc.lap("duplicate-token check");
    // ---- IDF ------------------------------------------------------------
    hc.idf.assign(T, {});
    hc.idf_explicit.assign(T, {});
    hc.has_idf.assign(T, 1);
    if (d->idf_mode == PF_IDF_EXPLICIT) {
        for (int t = 0; t < T; ++t) {
            hc.has_idf[t] = d->col_has_idf ? d->col_has_idf[t] : 1;
            if (!hc.has_idf[t] || !d->idf_off) continue;
            for (int64_t k = d->idf_off[t]; k < d->idf_off[t + 1]; ++k) hc.idf_explicit[t][d->idf_tid[k]] = d->idf_val[k];
        }
    }
    // ---- token ids -> column ranks, df / idf (profiles mode) and the candidate norms
    // sqrt(sum (tf*idf)^2) per (user, col) row: on the device (F3, pf_idf.hip)
    const int rc = device_idf_norms(hc, d->idf_mode != PF_IDF_EXPLICIT, err);
    if (rc != PF_OK) return rc;
    sc.lap("device ranks / idf / norms");
    // ---- normalisers -----------------------------------------------------
    const int K = kNumFixed + T;
    hc.npres.assign(K, 0); hc.nmean.assign(K, 0.f); hc.nsd.assign(K, 0.f);
    if (d->norm_present)
        for (int k = 0; k < K; ++k) { hc.npres[k] = d->norm_present[k]; hc.nmean[k] = d->norm_mean[k]; hc.nsd[k] = d->norm_sd[k]; }
    // ---- equality codes for public / gender ------------------------------
    auto codes = [&](const std::vector<int32_t>& v, std::unordered_map<int32_t, uint32_t>& m) -> bool {
        std::vector<int32_t> vals;
        for (int32_t x : v) if (x >= 0) vals.push_back(x);
        std::sort(vals.begin(), vals.end());
        vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
        if (vals.size() >= kCodeMissing) return false;
        for (size_t k = 0; k < vals.size(); ++k) m[vals[k]] = (uint32_t)k;
        return true;
    };
    if (!codes(hc.pub, hc.pub_code) || !codes(hc.gen, hc.gen_code)) {
        err = "more than 254 distinct public/gender values";
        return PF_EUNSUPP;
    }
    // ---- adjacency ---------------------------------------------------------
    hc.adj.clear();
    if (d->n_adj > 0 && (!d->adj_uid || !d->adj_off || !d->adj_nbr)) { err = "missing adjacency arrays"; return PF_EINVAL; }
    hc.adj.reserve((size_t)d->n_adj);
    for (int a = 0; a < d->n_adj; ++a) {
        auto& row = hc.adj[d->adj_uid[a]];
        row.insert(row.end(), d->adj_nbr + d->adj_off[a], d->adj_nbr + d->adj_off[a + 1]);
    }
    sc.lap("codes + adjacency map");
    return PF_OK;
}

int build_store(const HostCorpus& hc, HostStore& hs, std::string& err) {
    const int32_t n = hc.n, T = hc.T;
    // packed (fast) layout: one word per token and one tagged hash table, which needs
    // column ranks < 2^18 - 1 (the all-ones token key is the padding word's), 0 <= tf < 256
    // and club / friend ids below 2^30 (bits 30-31 are the kind tags)
    bool packed = true;
    for (int t = 0; t < T && packed; ++t) packed = (uint32_t)hc.n_ranks(t) < kTidMask;
    packed = packed && !par_any((int64_t)hc.tf.size(), [&](int64_t k) { return hc.tf[k] < 0 || hc.tf[k] > 255; });
    packed = packed && !par_any((int64_t)hc.clubs.size(), [&](int64_t k) { return hc.clubs[k] >= kIdLimit; });
    packed = packed && !par_any((int64_t)hc.friends.size(), [&](int64_t k) { return hc.friends[k] >= kIdLimit; });
    if (!packed) {
        for (int t = 0; t < T; ++t)
            if ((uint32_t)hc.n_ranks(t) > kWideTidMask + 1u) { err = "more than 2^26 distinct token ids in a column"; return PF_EUNSUPP; }
        if (par_any((int64_t)hc.tf.size(), [&](int64_t k) { return hc.tf[k] < -(1 << 23) || hc.tf[k] >= (1 << 23); })) {
            err = "token count outside [-2^23, 2^23)";
            return PF_EUNSUPP;
        }
    }
    hs.packed = packed;
    StageClock sc;
    // record length in words: clubs, friends, tokens
    std::vector<uint32_t> len(n), ncols(n);
    int64_t alg = 0;
    for (int i = 0; i < n; ++i) {
        // the walk counts club and friend intersections in 16-bit halves of one word
        if (hc.club_off[i + 1] - hc.club_off[i] > 0xFFFF || hc.friend_off[i + 1] - hc.friend_off[i] > 0xFFFF) {
            err = "a profile lists more than 65535 clubs or friends";
            return PF_EUNSUPP;
        }
        const int64_t nc = hc.club_off[i + 1] - hc.club_off[i], nf = hc.friend_off[i + 1] - hc.friend_off[i];
        const int64_t nt = hc.tok_off[(size_t)(i + 1) * T] - hc.tok_off[(size_t)i * T];
        uint32_t nz = 0;
        for (int t = 0; t < T; ++t) nz += hc.tok_off[(size_t)i * T + t + 1] > hc.tok_off[(size_t)i * T + t];
        len[i] = (uint32_t)(nc + nf + nt * (packed ? 1 : 2));
        ncols[i] = nz;
        alg += 32 + 4 * nc + 4 * nf + 8 * nt;
    }
    hs.alg_bytes = alg;
    sc.lap("record lengths");
    // slots: longest records first, so the 64 records of a tile have near-equal length
    // (a stable counting sort by length, longest first: ties keep idx order)
    hs.idx_of_slot.resize(n);
    {
        uint32_t mx = 0;
        for (int i = 0; i < n; ++i) mx = std::max(mx, len[i]);
        std::vector<int32_t> start((size_t)mx + 2, 0);
        for (int i = 0; i < n; ++i) ++start[mx - len[i] + 1];
        for (size_t k = 1; k < start.size(); ++k) start[k] += start[k - 1];
        for (int i = 0; i < n; ++i) hs.idx_of_slot[start[mx - len[i]]++] = i;
    }
    hs.slot_of_idx.resize(n);
    for (int p = 0; p < n; ++p) hs.slot_of_idx[hs.idx_of_slot[p]] = p;
    // tiles: take the next 64 >> lgk slots, lgk the smallest split that keeps the tile's
    // longest chunk (its first record's) within kMaxTileSteps
    hs.tile_off.clear(); hs.tile_steps.clear(); hs.norm_off.clear(); hs.tile_slot0.clear(); hs.tile_lgk.clear();
    hs.slot_tile.assign(n, 0);
    // PF_DEBUG tile_steps lowers the limit (tests use it to split ordinary records)
    const uint32_t max_steps = (uint32_t)std::max<long>(1, debug_long("tile_steps", kMaxTileSteps));
    uint64_t off = 0, noff = 0;
    for (int s0 = 0; s0 < n;) {
        const uint32_t mx = len[hs.idx_of_slot[s0]];
        uint32_t lgk = 0;
        while (lgk < 6 && (chunk_words(mx, lgk, packed) + 3) / 4 > max_steps) ++lgk;
        const int cnt = std::min(n - s0, kTileSlots >> lgk);
        uint32_t mr = 0;
        for (int p = s0; p < s0 + cnt; ++p) {
            mr = std::max(mr, ncols[hs.idx_of_slot[p]]);
            hs.slot_tile[p] = (uint32_t)hs.tile_off.size();
        }
        // steps rounded up to whole 4-step groups: the walk loads whole groups, and what
        // lies past a chunk is padding, never the next tile
        const uint32_t steps = ((chunk_words(mx, lgk, packed) + 15) / 16) * 4;
        hs.tile_off.push_back(off);
        hs.tile_steps.push_back(steps);
        hs.tile_slot0.push_back((uint32_t)s0);
        hs.tile_lgk.push_back((uint8_t)lgk);
        hs.norm_off.push_back(noff);
        off += (uint64_t)steps * kTileSlots;
        noff += (uint64_t)mr * kTileSlots;
        s0 += cnt;
    }
    sc.lap("slot order + tiles");
    // + one group of padding steps past the end: the scan's walk prefetches the group
    // after a tile's last one (never used), and a lane with an empty chunk still loads
    hs.norm_off.push_back(noff);  // sentinel: a tile's rank count = (norm_off[t+1] - norm_off[t]) / 64
    hs.stream.resize_uninit(off + 4 * kTileSlots);
    par_fill(hs.stream, make_uint4(kPadWord, kPadWord, kPadWord, kPadWord));
    // row store (the pair kernel K1'): each slot's record contiguous, padded to 16 B, so a lane
    // walking one candidate reads whole cache lines (the tile stream strides a record by 1 KiB),
    // then the slot's column norms (one double per non-empty column, 16-B padded): the epilogue
    // reads them from the lines after the record, with no tile lookup in front
    hs.row_off.assign((size_t)n + 1, 0);
    for (int p = 0; p < n; ++p) {
        const int i = hs.idx_of_slot[p];
        hs.row_off[p + 1] = hs.row_off[p] + (len[i] + 3) / 4 + (ncols[i] + 1) / 2;
    }
    hs.rows.resize_uninit(hs.row_off[n] + 1);
    par_fill(hs.rows, make_uint4(kPadWord, kPadWord, kPadWord, kPadWord));
    hs.norms.resize_uninit(noff);
    par_fill(hs.norms, 0.0);
    hs.hdr0.resize(n); hs.hdr1.resize(n); hs.hdr2.resize(n);
    sc.lap("stream / rows / norms allocated");
    par_for(n, [&](int64_t lo, int64_t hi) {
        std::vector<uint32_t> w;
        for (int64_t p = lo; p < hi; ++p) {
            const int i = hs.idx_of_slot[p];
            const int tile = (int)hs.slot_tile[p];
            const uint32_t lgk = hs.tile_lgk[tile];
            const int cand = (int)(p - hs.tile_slot0[tile]);
            w.clear();
            uint64_t mask = 0;
            for (int64_t k = hc.club_off[i]; k < hc.club_off[i + 1]; ++k) w.push_back(hc.clubs[k] | (packed ? kTagClub : 0u));
            for (int64_t k = hc.friend_off[i]; k < hc.friend_off[i + 1]; ++k) w.push_back(hc.friends[k]);
            uint32_t rank = 0;
            for (int t = 0; t < T; ++t) {
                const size_t r = (size_t)i * T + t;
                if (hc.tok_off[r + 1] == hc.tok_off[r]) continue;
                mask |= 1ull << t;
                const uint64_t mr = (hs.norm_off[tile + 1] - hs.norm_off[tile]) / kTileSlots;
                hs.norms[hs.norm_off[tile] + (uint64_t)cand * mr + rank] = hc.sqrt_nb[r];
                ++rank;
                for (int64_t k = hc.tok_off[r]; k < hc.tok_off[r + 1]; ++k) {
                    if (packed) {
                        w.push_back(((uint32_t)hc.tf[k] << 24) | ((uint32_t)t << kTidBits) | (uint32_t)hc.tid[k]);
                    } else {
                        w.push_back((uint32_t)hc.tid[k] | ((uint32_t)t << kWideTidBits));
                        w.push_back(((uint32_t)hc.tf[k] << 8) | (uint32_t)t);
                    }
                }
            }
            std::memcpy(reinterpret_cast<uint32_t*>(hs.rows.data() + hs.row_off[p]), w.data(), w.size() * 4);
            {  // the record's norms after its 16-B padded words
                double* rn = reinterpret_cast<double*>(hs.rows.data() + hs.row_off[p] + (w.size() + 3) / 4);
                uint32_t rk = 0;
                for (int t = 0; t < T; ++t) {
                    const size_t r = (size_t)i * T + t;
                    if (hc.tok_off[r + 1] != hc.tok_off[r]) rn[rk++] = hc.sqrt_nb[r];
                }
            }
            // chunk c of the record goes to lane cand * k + c
            const uint32_t q = chunk_words((uint32_t)w.size(), lgk, packed);
            uint32_t* base = reinterpret_cast<uint32_t*>(hs.stream.data() + hs.tile_off[tile]);
            for (size_t x = 0; x < w.size(); ++x) {
                const uint32_t c = (uint32_t)(x / q), o = (uint32_t)(x % q);
                const uint32_t lane = ((uint32_t)cand << lgk) + c;
                base[((o / 4) * kTileSlots + lane) * 4 + (o % 4)] = w[x];
            }
            auto code = [](const std::unordered_map<int32_t, uint32_t>& m, int32_t v) -> uint32_t {
                return v < 0 ? kCodeMissing : m.at(v);
            };
            const int64_t nc = hc.club_off[i + 1] - hc.club_off[i], nf = hc.friend_off[i + 1] - hc.friend_off[i];
            const int64_t nt = hc.tok_off[(size_t)(i + 1) * T] - hc.tok_off[(size_t)i * T];
            hs.hdr0[p] = make_uint4((uint32_t)mask, (uint32_t)(mask >> 32), (uint32_t)hc.comp[i], (uint32_t)hc.age[i]);
            hs.hdr1[p] = make_uint4((uint32_t)hc.reg[3 * (size_t)i], (uint32_t)hc.reg[3 * (size_t)i + 1],
                                    (uint32_t)hc.reg[3 * (size_t)i + 2], (uint32_t)hc.uid[i]);
            hs.hdr2[p] = make_uint4(code(hc.pub_code, hc.pub[i]) | (code(hc.gen_code, hc.gen[i]) << 8),
                                    (uint32_t)nc, (uint32_t)nf, (uint32_t)nt);
        }
    });
    sc.lap("records written");
    return PF_OK;
}

namespace {

// 2-choice cuckoo insertion of (key, val) items into a 2^lg table; false if it does not converge
bool cuckoo_fill(uint64_t* tab, int lg, uint32_t hmul, const std::vector<uint64_t>& items, uint64_t empty) {
    const size_t cap = (size_t)1 << lg;
    for (size_t i = 0; i < cap; ++i) tab[i] = empty;
    for (uint64_t it : items) {
        uint64_t cur = it;
        uint32_t from = cuckoo_h1(cuckoo_x((uint32_t)cur, hmul), lg);
        bool placed = false;
        for (int kick = 0; kick < 500; ++kick) {
            const uint32_t x = cuckoo_x((uint32_t)cur, hmul);
            const uint32_t a = cuckoo_h1(x, lg), b = cuckoo_h2(x, lg);
            if (tab[a] == empty) { tab[a] = cur; placed = true; break; }
            if (tab[b] == empty) { tab[b] = cur; placed = true; break; }
            from = (from == a) ? b : a;  // evict from the slot we did not come from
            std::swap(cur, tab[from]);
        }
        if (!placed) return false;
    }
    return true;
}

}  // namespace

int lg_for(size_t n) {
    int lg = 4;
    while (((size_t)1 << lg) * 2 < n * 5) ++lg;  // load factor <= 0.4
    return lg;
}

// The A side's constants (recommender_similarity.cpp:10-124), in three parts the device image
// builder (pf_jobs.hip K6) shares bit for bit: the query-independent fields (normaliser modes,
// s = 0 terms, equality terms), the region row per a_regcnt and the completion / age rows per
// query value, all glibc-exp sigmoid values.
namespace {
double zval(const HostCorpus& hc, int slot, double s) {
    if (hc.npres[slot] && hc.nsd[slot] > 0.0f) return (s - (double)hc.nmean[slot]) / (double)hc.nsd[slot];
    return 6.0 * (s - 0.5);
}
double term(const HostCorpus& hc, int slot, double s) { return ref_sigmoid(zval(hc, slot, s)); }
}  // namespace

void qconst_template(const HostCorpus& hc, bool packed, QConst& c) {
    const int T = hc.T;
    std::memset(&c, 0, sizeof c);
    c.n_cols = T;
    // normaliser parameters: z = (s-mean)/sd when the key exists and sd > 0, else 6(s-0.5)
    for (int k = 0; k < kNumFixed + T; ++k) {
        bool use = hc.npres[k] && hc.nsd[k] > 0.0f;
        c.zmean[k] = (double)hc.nmean[k];
        c.zsd[k] = (double)hc.nsd[k];
        if (use) {
            if (k < kNumFixed) c.zmode_fx |= 1u << k;
            else if (k - kNumFixed < 32) c.zmode_lo |= 1u << (k - kNumFixed);
            else c.zmode_hi |= 1u << (k - kNumFixed - 32);
        }
    }
    for (int e = 0; e < 2; ++e) {
        c.sig_pub[e] = term(hc, PF_F_PUBLIC, e ? 1.0 : 0.0);
        c.sig_gen[e] = term(hc, PF_F_GENDER, e ? 1.0 : 0.0);
    }
    c.sig0_clubs = term(hc, PF_F_CLUBS, 0.0);
    c.sig0_friends = term(hc, PF_F_FRIENDS, 0.0);
    for (int t = 0; t < T; ++t) c.sig0_col[t] = term(hc, kNumFixed + t, 0.0);
    c.n_hits_max = kHitSlots * (packed ? 4u : 8u);  // + the dump slots
}

void qconst_sig_reg(const HostCorpus& hc, int a_regcnt, double out[4][4]) {
    for (int b = 0; b < 4; ++b)
        for (int m = 0; m < 4; ++m) out[b][m] = 0.0;
    if (a_regcnt <= 0) return;
    for (int b = 1; b <= 3; ++b)
        for (int m = 0; m <= 3; ++m) {
            // recommender.cpp:130-139, cast to float then back to double
            double s = (double)(float)((double)m / (std::sqrt((double)a_regcnt) * std::sqrt((double)b)));
            out[b][m] = term(hc, PF_F_REGION, s);
        }
}

void qconst_ratio_row(const HostCorpus& hc, int slot, int a, double* out) {
    out[0] = 0.0;
    for (int v = 1; v <= kValTab; ++v)
        out[v] = a > 0 ? term(hc, slot, (double)std::min(a, v) / (double)std::max(a, v)) : 0.0;
}

static void fill_qconst(const HostCorpus& hc, bool packed, int32_t i, QConst& c) {
    const int T = hc.T;
    qconst_template(hc, packed, c);
    c.pubcode = hc.pub[i] < 0 ? kCodeMissing : hc.pub_code.at(hc.pub[i]);
    c.gencode = hc.gen[i] < 0 ? kCodeMissing : hc.gen_code.at(hc.gen[i]);
    c.comp = hc.comp[i];
    c.age = hc.age[i];
    for (int k = 0; k < 3; ++k) c.reg[k] = hc.reg[3 * (size_t)i + k];
    c.a_regcnt = (c.reg[0] >= 0) + (c.reg[1] >= 0) + (c.reg[2] >= 0);
    c.n_clubs = (int32_t)(hc.club_off[i + 1] - hc.club_off[i]);
    c.n_friends = (int32_t)(hc.friend_off[i + 1] - hc.friend_off[i]);
    c.sqrt_clubs = std::sqrt((double)c.n_clubs);
    c.sqrt_friends = std::sqrt((double)c.n_friends);
    qconst_sig_reg(hc, c.a_regcnt, c.sig_reg);
    qconst_ratio_row(hc, PF_F_COMPLETION, c.comp, c.sig_comp);
    qconst_ratio_row(hc, PF_F_AGE, c.age, c.sig_age);
    c.colmask = 0;
    for (int t = 0; t < T; ++t) {
        const size_t r = (size_t)i * T + t;
        c.sqrt_na[t] = hc.sqrt_nb[r];
        if (hc.tok_off[r + 1] != hc.tok_off[r]) c.colmask |= 1ull << t;
    }
}

bool build_query(const HostCorpus& hc, bool packed, int32_t i, const std::vector<int32_t>* excl, QImageHost& out) {
    const int T = hc.T;
    QConst& c = out.c;
    fill_qconst(hc, packed, i, c);
    // hash items: distinct clubs (T0), distinct friends (T1), (column, token) weights (T2),
    // exclusions (T3); packed corpora merge T0..T2 into one tagged table (pf_types.h)
    std::vector<uint64_t> items[4];
    std::vector<uint32_t> tmp(hc.clubs.begin() + hc.club_off[i], hc.clubs.begin() + hc.club_off[i + 1]);
    std::sort(tmp.begin(), tmp.end());
    tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
    for (uint32_t x : tmp) items[0].push_back(packed ? make_entry(x | kTagClub, 1u) : make_entry(x, 0));
    tmp.assign(hc.friends.begin() + hc.friend_off[i], hc.friends.begin() + hc.friend_off[i + 1]);
    std::sort(tmp.begin(), tmp.end());
    tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
    for (uint32_t x : tmp) items[1].push_back(packed ? make_entry(x, 0x10000u) : make_entry(x, 0));
    out.vals.clear();
    for (int t = 0; t < T; ++t) {
        const size_t r = (size_t)i * T + t;
        if (hc.tok_off[r + 1] == hc.tok_off[r]) continue;
        for (int64_t k = hc.tok_off[r]; k < hc.tok_off[r + 1]; ++k) {
            const double idf = hc.has_idf[t] ? (double)hc.idf_of(t, hc.tid[k]) : 1.0;  // recommender.cpp:78 (A7)
            QVal v;
            v.wq = (double)hc.tf[k] * idf;
            v.idf = idf;
            const uint32_t vi = (uint32_t)out.vals.size();
            if (packed)
                items[2].push_back(make_entry(kTagTok | ((uint32_t)t << kTidBits) | (uint32_t)hc.tid[k],
                                              kTokVal | vi | ((uint32_t)t << kTidBits)));
            else items[2].push_back(make_entry((uint32_t)hc.tid[k] | ((uint32_t)t << kWideTidBits), (uint32_t)t | (vi << 8)));
            out.vals.push_back(v);
        }
    }
    if (excl) {
        tmp.assign(excl->begin(), excl->end());
        std::sort(tmp.begin(), tmp.end());
        tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
        for (uint32_t x : tmp) items[3].push_back(make_entry(x, packed ? 1u : 0u));
    }
    c.n_vals = (int32_t)out.vals.size();
    if (out.vals.size() >= (packed ? (1u << kTidBits) : (1u << 24))) return false;
    const uint64_t empty = packed ? kEmptyEntryPacked : kEmptyEntry;
    if (packed) {  // one table T for every record word
        items[0].insert(items[0].end(), items[1].begin(), items[1].end());
        items[0].insert(items[0].end(), items[2].begin(), items[2].end());
        items[1].clear();
        items[2].clear();
    }
    const int ntab = packed ? 1 : 3;
    int lg = std::max({lg_for(items[0].size()), lg_for(items[1].size()), lg_for(items[2].size())});
    int lge = lg_for(items[3].size());
    for (; lg <= kMaxHashLog2; ++lg, ++lge) {
        lge = std::min(lge, kMaxHashLog2);
        const size_t eoff = (size_t)ntab << lg;
        out.keys.assign(eoff + ((size_t)1 << lge), empty);
        for (uint32_t s = 0; s < 16; ++s) {
            const uint32_t hmul = kHashMul + 2u * s * 0x6A09E667u;  // odd
            bool ok = true;
            for (int k = 0; k < ntab && ok; ++k)
                ok = cuckoo_fill(out.keys.data() + ((size_t)k << lg), lg, hmul, items[k], empty);
            if (ok) ok = cuckoo_fill(out.keys.data() + eoff, lge, hmul, items[3], empty);
            if (ok) {
                c.lg = lg;
                c.lg_excl = lge;
                c.hmul = hmul;
                c.excl_off = (uint32_t)eoff;
                // SoA per table (pf_types.h soa_words), in the same bytes
                const std::vector<uint64_t> aos(out.keys);
                uint32_t* w = reinterpret_cast<uint32_t*>(out.keys.data());
                for (size_t i = 0; i < aos.size(); ++i) {
                    uint32_t kw, vw;
                    soa_words((uint32_t)i, (uint32_t)eoff, lg, lge, kw, vw);
                    w[kw] = (uint32_t)aos[i];
                    w[vw] = (uint32_t)(aos[i] >> 32);
                }
                return true;
            }
        }
    }
    return false;
}

}  // namespace pf

// ---------------------------------------------------------------- postings store (K5)
namespace pf {

namespace {

constexpr int kBuildThreads = 16;  // host threads of the postings build

// Stable LSD radix sort of 64-bit keys on bits [lo_bit, 64) (16-bit digits), each pass on
// kBuildThreads threads: per-thread digit counts of its chunk, the global digit x thread prefix,
// then every thread scatters its chunk in order.
void par_radix_sort_u64(std::vector<uint64_t>& a, int lo_bit) {
    const size_t n = a.size();
    if (n == 0) return;
    std::vector<uint64_t> b(n);
    const int th = kBuildThreads;
    const size_t chunk = (n + th - 1) / th;
    std::vector<std::vector<size_t>> cnt(th, std::vector<size_t>(65536));
    for (int sh = lo_bit; sh < 64; sh += 16) {
        std::vector<std::thread> ts;
        for (int w = 0; w < th; ++w)
            ts.emplace_back([&, w]() {
                auto& c = cnt[w];
                std::fill(c.begin(), c.end(), 0);
                const size_t lo = w * chunk, hi = std::min(n, lo + chunk);
                for (size_t i = lo; i < hi; ++i) ++c[(a[i] >> sh) & 0xFFFF];
            });
        for (auto& t : ts) t.join();
        ts.clear();
        size_t run = 0;  // digit-major, thread-minor: a thread's items of a digit follow the lower threads'
        for (int d = 0; d < 65536; ++d)
            for (int w = 0; w < th; ++w) {
                const size_t x = cnt[w][d];
                cnt[w][d] = run;
                run += x;
            }
        for (int w = 0; w < th; ++w)
            ts.emplace_back([&, w]() {
                auto& c = cnt[w];
                const size_t lo = w * chunk, hi = std::min(n, lo + chunk);
                for (size_t i = lo; i < hi; ++i) b[c[(a[i] >> sh) & 0xFFFF]++] = a[i];
            });
        for (auto& t : ts) t.join();
        a.swap(b);
    }
}

// cell width 2^shift: the smallest >= one wave block holding ~<= kCellEntries of the list's
// entries.  A block reads whole cells, so a short list costs up to a cell of entries per block
// for the few that fall in it: 8 per cell reads 0.175 GB per cfg-2 query instead of 0.194 at
// 32, and K5 takes 202.8 us instead of 206.0 (r2p A/B; 4 per cell: no further gain).
constexpr uint64_t kCellEntries = 8;
uint32_t list_shift(uint64_t len, int32_t n) {
    uint32_t s = kPostMinShift;
    while (s < 30 && (len << (s + 1)) <= kCellEntries * (uint64_t)n) ++s;
    return s;
}

}  // namespace

void build_postings(const HostCorpus& hc, HostPost& hp) {
    const int32_t n = hc.n, T = hc.T;
    hp.ok = false;
    auto bail = [&](const char* w) {
        hp.why = w;
        hp.hdr.clear(); hp.post.clear(); hp.pnorm.clear(); hp.cells.clear(); hp.lists.clear(); hp.tok_list.clear();
        hp.club_list.clear(); hp.friend_list.clear();
    };
    if (n <= 0) return bail("empty corpus");
    StageClock sc;
    if ((uint32_t)n >= kPostIdxLimit) return bail("more than 2^24 candidates");
    if (T > kPostMaxCols) return bail("more than 48 text columns");
    for (int32_t i = 0; i < n; ++i) {
        if (hc.comp[i] < -32768 || hc.comp[i] > 32767 || hc.age[i] < -32768 || hc.age[i] > 32767)
            return bail("completion / age outside 16 bits");
        if (hc.club_off[i + 1] - hc.club_off[i] > 0xFFFF || hc.friend_off[i + 1] - hc.friend_off[i] > 0xFFFF)
            return bail("more than 65535 clubs or friends");
    }
    for (int t = 0; t < T; ++t)
        if (hc.n_ranks(t) >= (1 << 22)) return bail("more than 2^22 distinct token ids in a column");
    if (par_any((int64_t)hc.tf.size(), [&](int64_t k) { return hc.tf[k] < 0 || hc.tf[k] > 255; }))
        return bail("token count outside the packed encoding");
    // ---- token lists: (column, tid rank) ascending; entries idx << 8 | tf, tf > 0 only (a tf = 0
    // token adds +0 to a dot and never decides a hit: recommender.cpp:74-85)
    hp.tok_list.assign(T, {});
    // per thread (a contiguous range of users) the entries of every (column, rank) key: the counts,
    // later each thread's first entry in every list (its cursors)
    std::vector<int64_t> kbase((size_t)T + 1, 0);
    for (int t = 0; t < T; ++t) kbase[t + 1] = kbase[t] + hc.n_ranks(t);
    const int th = kBuildThreads;
    const int64_t uchunk = ((int64_t)n + th - 1) / th;
    std::vector<std::vector<uint32_t>> tcnt(th);
    auto users = [&](int w, auto f) {
        const int64_t lo = w * uchunk, hi = std::min<int64_t>(n, lo + uchunk);
        for (int64_t i = lo; i < hi; ++i)
            for (int t = 0; t < T; ++t)
                for (int64_t k = hc.tok_off[(size_t)i * T + t]; k < hc.tok_off[(size_t)i * T + t + 1]; ++k)
                    if (hc.tf[k] > 0) f(i, t, k, (size_t)(kbase[t] + hc.tid[k]));
    };
    {
        std::vector<std::thread> ts;
        for (int w = 0; w < th; ++w)
            ts.emplace_back([&, w]() {
                tcnt[w].assign((size_t)kbase[T], 0u);
                users(w, [&](int64_t, int, int64_t, size_t key) { ++tcnt[w][key]; });
            });
        for (auto& x : ts) x.join();
    }
    std::vector<std::vector<uint32_t>> cnt(T);
    for (int t = 0; t < T; ++t) {
        cnt[t].assign((size_t)hc.n_ranks(t), 0u);
        for (int w = 0; w < th; ++w)
            for (size_t r = 0; r < cnt[t].size(); ++r) cnt[t][r] += tcnt[w][kbase[t] + r];
    }
    sc.lap("checks + token counts");
    uint64_t off = 0;
    std::vector<uint64_t> col_off(T + 1, 0);
    for (int t = 0; t < T; ++t) {
        col_off[t] = off;
        hp.tok_list[t].assign(cnt[t].size(), -1);
        for (size_t tid = 0; tid < cnt[t].size(); ++tid) {
            if (!cnt[t][tid]) continue;
            hp.tok_list[t][tid] = (int32_t)hp.lists.size();
            hp.lists.push_back(PList{(uint32_t)off, 0u, 0u, cnt[t][tid]});
            off += cnt[t][tid];
            if (off >= (1ull << 32)) return bail("more than 2^32 postings");
        }
    }
    col_off[T] = off;
    hp.tok_entries = (int64_t)off;
    // ---- set lists: entries idx << 8 | multiplicity (recommender.cpp:119-128 counts B's
    // duplicates); one list per distinct club / friend id
    std::vector<uint64_t> ckeys, fkeys;
    // keys (id, idx, multiplicity) are collected per row range on threads; each (id, idx) pair
    // occurs once, so the radix sort below fixes their order whatever the concatenation order
    auto collect = [&](const std::vector<int64_t>& o, const std::vector<uint32_t>& ids, std::vector<uint64_t>& keys) -> bool {
        std::mutex mu;
        std::vector<std::pair<int64_t, std::vector<uint64_t>>> parts;
        std::atomic<bool> ok{true};
        par_for(n, [&](int64_t lo, int64_t hi) {
            std::vector<uint64_t> mine;
            std::vector<uint32_t> tmp;
            for (int64_t i = lo; i < hi && ok; ++i) {
                tmp.assign(ids.begin() + o[i], ids.begin() + o[i + 1]);
                std::sort(tmp.begin(), tmp.end());
                for (size_t a = 0; a < tmp.size();) {
                    size_t b = a;
                    while (b < tmp.size() && tmp[b] == tmp[a]) ++b;
                    if (b - a > 255) { ok = false; break; }
                    mine.push_back(((uint64_t)tmp[a] << 32) | ((uint64_t)i << 8) | (uint64_t)(b - a));
                    a = b;
                }
            }
            std::lock_guard<std::mutex> g(mu);
            parts.emplace_back(lo, std::move(mine));
        });
        if (!ok) return false;
        std::sort(parts.begin(), parts.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        size_t tot = 0;
        for (auto& pr : parts) tot += pr.second.size();
        keys.reserve(tot);
        for (auto& pr : parts) keys.insert(keys.end(), pr.second.begin(), pr.second.end());
        return true;
    };
    if (!collect(hc.club_off, hc.clubs, ckeys) || !collect(hc.friend_off, hc.friends, fkeys))
        return bail("a club / friend id repeats more than 255 times in one profile");
    sc.lap("token lists + set keys");
    // (id, idx, multiplicity) keys arrive in idx order: a stable sort by id puts each id's
    // entries in idx order
    par_radix_sort_u64(ckeys, 32);
    par_radix_sort_u64(fkeys, 32);
    sc.lap("set keys sorted");
    const uint64_t set_off = off;
    if (off + ckeys.size() + fkeys.size() >= (1ull << 32)) return bail("more than 2^32 postings");
    hp.post.resize_uninit(off + ckeys.size() + fkeys.size());
    auto add_sets = [&](const std::vector<uint64_t>& keys, std::unordered_map<uint32_t, int32_t>& m) {
        uint32_t* dst = hp.post.data() + off;
        par_for((int64_t)keys.size(), [&](int64_t lo, int64_t hi) {
            for (int64_t x = lo; x < hi; ++x) dst[x] = (uint32_t)keys[x];
        });
        size_t nid = 0;
        for (size_t a = 1; a <= keys.size(); ++a) nid += a == keys.size() || (keys[a] >> 32) != (keys[a - 1] >> 32);
        m.reserve(nid);
        hp.lists.reserve(hp.lists.size() + nid);
        for (size_t a = 0; a < keys.size();) {
            const uint32_t id = (uint32_t)(keys[a] >> 32);
            size_t b = a + 1;
            while (b < keys.size() && (uint32_t)(keys[b] >> 32) == id) ++b;
            m[id] = (int32_t)hp.lists.size();
            hp.lists.push_back(PList{(uint32_t)off, 0u, 0u, (uint32_t)(b - a)});
            off += b - a;
            a = b;
        }
    };
    add_sets(ckeys, hp.club_list);
    add_sets(fkeys, hp.friend_list);
    (void)set_off;
    sc.lap("set lists");
    // ---- token entries and their norms, per column in idx order (lists come out sorted)
    hp.pnorm.resize_uninit(hp.tok_entries);
    {
        // each thread's cursor in every list: the list's start + the lower threads' entries; the
        // threads own ascending user ranges, so every list comes out in idx order
        par_for((int64_t)kbase[T], [&](int64_t lo, int64_t hi) {
            int t = 0;
            for (int64_t key = lo; key < hi; ++key) {
                while (kbase[t + 1] <= key) ++t;
                const int32_t li = hp.tok_list[t][key - kbase[t]];
                uint32_t x = li >= 0 ? hp.lists[li].off : 0u;
                for (int w = 0; w < th; ++w) {
                    const uint32_t c = tcnt[w][key];
                    tcnt[w][key] = x;
                    x += c;
                }
            }
        });
        std::vector<std::thread> ts;
        for (int w = 0; w < th; ++w)
            ts.emplace_back([&, w]() {
                auto& cur = tcnt[w];
                users(w, [&](int64_t i, int t, int64_t k, size_t key) {
                    const uint32_t x = cur[key]++;
                    hp.post[x] = ((uint32_t)i << 8) | (uint32_t)hc.tf[k];
                    hp.pnorm[x] = hc.sqrt_nb[(size_t)i * T + t];
                });
            });
        for (auto& x : ts) x.join();
    }
    sc.lap("token entries");
    // ---- cells
    uint64_t coff = 0;
    for (auto& L : hp.lists) {
        L.shift = list_shift(L.len, n);
        L.cell_off = (uint32_t)coff;
        coff += (((uint64_t)(n - 1) >> L.shift) + 1) + 1;
        if (coff >= (1ull << 32)) return bail("cell table beyond 2^32 entries");
    }
    hp.cells.resize_uninit(coff);
    par_dyn((int64_t)hp.lists.size(), 64, [&](int64_t lo, int64_t hi) {  // the token lists come first and are long
        for (int64_t li = lo; li < hi; ++li) {
            const PList& L = hp.lists[li];
            const uint32_t nc = (uint32_t)(((uint64_t)(n - 1) >> L.shift) + 1);
            uint32_t x = 0;
            for (uint32_t c = 0; c <= nc; ++c) {
                const uint64_t lim = (uint64_t)c << L.shift;
                while (x < L.len && (uint64_t)(hp.post[L.off + x] >> 8) < lim) ++x;
                hp.cells[L.cell_off + c] = x;
            }
        }
    });
    sc.lap("cells");
    // ---- headers
    hp.hdr.resize(2 * (size_t)n);
    par_for(n, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            uint64_t cm = 0;
            for (int t = 0; t < T; ++t)
                if (hc.tok_off[(size_t)i * T + t + 1] > hc.tok_off[(size_t)i * T + t]) cm |= 1ull << t;
            const uint32_t pb = hc.pub[i] < 0 ? kCodeMissing : hc.pub_code.at(hc.pub[i]);
            const uint32_t gb = hc.gen[i] < 0 ? kCodeMissing : hc.gen_code.at(hc.gen[i]);
            const uint32_t nc = (uint32_t)(hc.club_off[i + 1] - hc.club_off[i]);
            const uint32_t nf = (uint32_t)(hc.friend_off[i + 1] - hc.friend_off[i]);
            hp.hdr[2 * i] = make_uint4((uint32_t)cm, (uint32_t)((cm >> 32) & 0xFFFFu) | (pb << 16) | (gb << 24),
                                       ((uint32_t)hc.comp[i] & 0xFFFFu) | ((uint32_t)hc.age[i] << 16), nc | (nf << 16));
            hp.hdr[2 * i + 1] = make_uint4((uint32_t)hc.reg[3 * i], (uint32_t)hc.reg[3 * i + 1],
                                           (uint32_t)hc.reg[3 * i + 2], (uint32_t)hc.uid[i]);
        }
    });
    sc.lap("headers");
    hp.ok = true;
}

// The image's part after its QConst: QPostHead | QTok | QCol | PList | excl, offsets from the image
// start (part start - sizeof(QConst)); written to out (out_cap bytes, zero-filled past the data).
// Returns the part's size, or 0 when it exceeds out_cap.
size_t build_query_post_part(const HostCorpus& hc, const HostPost& hp, int32_t i, const std::vector<int32_t>& excl,
                             uint8_t* out, size_t out_cap) {
    const int T = hc.T;
    std::vector<QTok> toks;
    std::vector<QCol> cols;
    for (int t = 0; t < T; ++t) {
        const size_t r = (size_t)i * T + t;
        const int32_t j0 = (int32_t)toks.size();
        for (int64_t k = hc.tok_off[r]; k < hc.tok_off[r + 1]; ++k) {
            const double idf = hc.has_idf[t] ? (double)hc.idf_of(t, hc.tid[k]) : 1.0;  // recommender.cpp:78
            const double wq = (double)hc.tf[k] * idf;
            if (wq == 0.0) continue;  // adds +-0 to every dot it meets
            QTok q;
            q.l = hp.lists[hp.tok_list[t][hc.tid[k]]];  // tf > 0: the query itself is on the list
            q.wq = wq;
            q.idf = idf;
            toks.push_back(q);
        }
        // every non-empty query column is listed (none of its tokens may carry weight: then
        // it has no passes), so the kernel adds every common column's term at its column
        if (hc.tok_off[r + 1] != hc.tok_off[r]) cols.push_back(QCol{t, j0, (int32_t)toks.size(), 0});
    }
    std::vector<PList> sets;
    auto add_sets = [&](const std::vector<int64_t>& o, const std::vector<uint32_t>& ids,
                        const std::unordered_map<uint32_t, int32_t>& m) -> int32_t {
        std::vector<uint32_t> v(ids.begin() + o[i], ids.begin() + o[i + 1]);
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        for (uint32_t x : v) sets.push_back(hp.lists[m.at(x)]);
        return (int32_t)v.size();
    };
    const int32_t ncl = add_sets(hc.club_off, hc.clubs, hp.club_list);
    const int32_t nfr = add_sets(hc.friend_off, hc.friends, hp.friend_list);
    std::vector<uint32_t> ex;
    for (int32_t u : excl) {
        const int32_t x = hc.idx_of(u);
        if (x >= 0) ex.push_back((uint32_t)x);
    }
    std::sort(ex.begin(), ex.end());
    ex.erase(std::unique(ex.begin(), ex.end()), ex.end());
    auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    QPostHead h{};
    h.n_tok = (int32_t)toks.size();
    h.n_act = (int32_t)cols.size();
    h.n_club = ncl;
    h.n_friend = nfr;
    h.n_excl = (int32_t)ex.size();
    size_t o = a16(sizeof(QConst) + sizeof(QPostHead));
    h.tok_off = (int32_t)o;
    o = a16(o + toks.size() * sizeof(QTok));
    h.col_off = (int32_t)o;
    o = a16(o + cols.size() * sizeof(QCol));
    h.set_off = (int32_t)o;
    o = a16(o + sets.size() * sizeof(PList));
    h.excl_off = (int32_t)o;
    o = a16(o + ex.size() * 4);
    const size_t part = o - sizeof(QConst);
    if (part > out_cap) return 0;
    auto at = [&](int32_t img_off) { return out + ((size_t)img_off - sizeof(QConst)); };  // offsets: from the image start
    std::memset(out, 0, out_cap);
    std::memcpy(out, &h, sizeof h);
    if (!toks.empty()) std::memcpy(at(h.tok_off), toks.data(), toks.size() * sizeof(QTok));
    if (!cols.empty()) std::memcpy(at(h.col_off), cols.data(), cols.size() * sizeof(QCol));
    if (!sets.empty()) std::memcpy(at(h.set_off), sets.data(), sets.size() * sizeof(PList));
    if (!ex.empty()) std::memcpy(at(h.excl_off), ex.data(), ex.size() * 4);
    return part;
}

size_t post_part_bound(const HostCorpus& hc, int32_t i, size_t n_excl) {
    auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const int T = hc.T;
    const size_t ntok = (size_t)(hc.tok_off[(size_t)(i + 1) * T] - hc.tok_off[(size_t)i * T]);
    size_t nact = 0;
    for (int t = 0; t < T; ++t) nact += hc.tok_off[(size_t)i * T + t + 1] != hc.tok_off[(size_t)i * T + t];
    const size_t nset = (size_t)(hc.club_off[i + 1] - hc.club_off[i]) + (size_t)(hc.friend_off[i + 1] - hc.friend_off[i]);
    return a16(sizeof(QPostHead)) + a16(ntok * sizeof(QTok)) + a16(nact * sizeof(QCol)) + a16(nset * sizeof(PList)) +
           a16(n_excl * 4);
}

void build_query_post(const HostCorpus& hc, const HostPost& hp, int32_t i, const std::vector<int32_t>& excl,
                      std::vector<uint8_t>& img) {
    QConst c;
    fill_qconst(hc, true, i, c);
    const size_t cap = post_part_bound(hc, i, excl.size());
    img.assign(sizeof(QConst) + cap, 0);
    std::memcpy(img.data(), &c, sizeof c);
    const size_t part = build_query_post_part(hc, hp, i, excl, img.data() + sizeof(QConst), cap);
    img.resize(sizeof(QConst) + part);
}

}  // namespace pf
