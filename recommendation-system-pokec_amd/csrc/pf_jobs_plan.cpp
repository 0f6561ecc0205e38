// pf_jobs_plan.cpp — host side of the device job pipeline (pf_jobs.hip): the graph store and
// image-builder tables built at pf_open, and run_jobs, which plans a batch of the reference's
// recommender calls (recommend_by_interest / _collaborative / recommend_clubs_collab under an
// adjacency view, pf_batch.h) and runs it as one chain of device stages on the context's
// stream: K6 images -> K3 gathers -> K1' pairs -> K4' / K7 -> K8 top-k, one copy back.
//
// The host works on 1-hop data only (the job's own adjacency row and its friends' row lengths,
// for sizing); every 2-hop walk, de-duplication, FAS pair, sum and top-k runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <numeric>
#include <thread>

#include "pf_batch.h"
#include "pf_debug.h"
#include "pf_ctx.h"
#include "pf_kernels.h"

namespace pf {

namespace {

constexpr int kDevTopK = kMaxTopK;           // K8 keeps up to 64 keys per job
constexpr int64_t kChunkElems = 192ll << 20; // element workspace per chunk (x 12 B)
constexpr int64_t kChunkHt = 128ll << 20;    // gather hash tables per chunk (int32 words)
constexpr size_t kPipeJobs = 1024;           // calls of this many jobs or more run as pipelined chunks
constexpr uint32_t kStageLimitJobs = 48 * 1024;  // as pf_api.cpp kStageLimit (LDS-staged tables)
constexpr int64_t kGatherChunk = 2048;          // K3's round (2 x pf_jobs.hip kGatherThreads): the last
                                                // round claims up to this many table slots past the limit

int32_t node_of(const pf_ctx* c, int32_t uid) {
    const auto& dn = c->jb.dense_node;  // uids of a dense range: one load (built at open)
    if (uid >= 0 && (size_t)uid < dn.size()) {
        const int32_t x = dn[uid];
        if (x >= 0 || !c->jb.nodes_dirty) return x;
    }
    const int32_t i = c->hc.idx_of(uid);
    if (i >= 0) return i;
    auto it = c->jb.xnode.find(uid);
    return it == c->jb.xnode.end() ? -1 : it->second;
}

int32_t ensure_node(pf_ctx* c, int32_t uid) {
    int32_t x = node_of(c, uid);
    if (x >= 0) return x;
    auto& J = c->jb;
    x = (int32_t)J.g_uid.size();
    J.xnode.emplace(uid, x);
    J.g_uid.push_back(uid);
    J.g_len.push_back(-1);
    if (uid >= 0 && (size_t)uid < J.dense_node.size()) J.dense_node[uid] = x;
    J.nodes_dirty = true;
    return x;
}

template <class T>
hipError_t up(pf_ctx* c, DBuf& b, const std::vector<T>& v) {
    return upload(c, b, v);
}

int a16(int64_t x) { return (int)((x + 15) & ~15ll); }

// candidates per pair block = the pair kernel's block (one pair per thread, pf_kernels.h)
constexpr int64_t kPairSpan = kPairThreads;
size_t a16z(size_t x) { return (x + 15) & ~(size_t)15; }

int pow2_lg(int64_t n) {
    int lg = 4;
    while (((int64_t)1 << lg) < n) ++lg;
    return lg;
}

// Every user's query image (K6's layout: QConst | table | values) built once at open into one
// resident pool, when it fits a third of the free HBM (at 1.63M users ~10^4 B each: a few
// percent of 288 GB): a job batch then references the images its users and friends need instead
// of building them (K6 left the per-call path: ~70 us of a 64-user collaborative step).  The
// images are a function of the profiles and the idf fixed at open (pf_set_adj changes rows of
// adj_list, which no image holds: the pair images carry no exclusions).  PF_DEBUG
// resident_images=0 keeps the per-call builds.
int build_resident_images(pf_ctx* c) {
    auto& J = c->jb;
    const HostCorpus& hc = c->hc;
    const bool packed = c->hs.packed;
    J.pimg = false;
    if (debug_long("resident_images", 1) == 0 || hc.n == 0) return PF_OK;
    const int32_t n = hc.n;
    const int lge = lg_for(0);
    const size_t ntab = packed ? 1u : 3u;
    auto ntok_of = [&](int32_t idx) { return hc.tok_off[(size_t)(idx + 1) * hc.T] - hc.tok_off[(size_t)idx * hc.T]; };
    std::vector<int64_t> off((size_t)n + 1, 0);
    par_jobs((size_t)n, [&](size_t i) {
        const int lg = J.img_lg[i];
        off[i + 1] = lg ? (int64_t)(a16z(sizeof(QConst) + ((ntab << lg) + ((size_t)1 << lge)) * 8) +
                                    a16z((size_t)ntok_of((int32_t)i) * sizeof(QVal)))
                        : 0;
    }, 1 << 14);
    for (int32_t i = 0; i < n; ++i) off[i + 1] += off[i];
    const size_t total = (size_t)off[n];
    size_t freeb = 0, totb = 0;
    if (hipMemGetInfo(&freeb, &totb) != hipSuccess) return PF_OK;
    if (total == 0 || total > freeb / 3 || total >= ((size_t)1 << 36)) return PF_OK;  // 16-B units in 32 bits
    HIPCHK(c, J.d_pimg.ensure(total));
    // batches of images whose offsets fit K6's 32-bit pool offsets; K6 wants each batch's images
    // ordered small LDS builds | large LDS builds | global-memory builds
    DBuf d_ij, d_scr, d_fail;
    HIPCHK(c, d_fail.ensure(16));
    HIPCHK(c, hipMemsetAsync(d_fail.p, 0, 16, c->stream));
    const size_t kBatchBytes = (size_t)1 << 31;
    int32_t i0 = 0;
    while (i0 < n) {
        int32_t i1 = i0;
        while (i1 < n && (size_t)(off[i1 + 1] - off[i0]) <= kBatchBytes && i1 - i0 < (1 << 18)) ++i1;
        std::vector<ImgJob> ij;
        ij.reserve((size_t)(i1 - i0));
        std::vector<uint8_t> cls;
        cls.reserve((size_t)(i1 - i0));
        for (int32_t idx = i0; idx < i1; ++idx) {
            const int lg = J.img_lg[idx];
            if (!lg) continue;
            ImgJob m{};
            m.idx = idx;
            m.lg = lg;
            m.lge = lge;
            m.dlg = pow2_lg(2 * (int64_t)J.img_nset[idx] + 2);
            m.rows = J.img_rows[idx];
            m.const_off = (uint32_t)(off[idx] - off[i0]);
            m.keys_off = (uint32_t)(m.const_off + sizeof(QConst));
            m.vals_off = (uint32_t)(m.const_off + a16z(sizeof(QConst) + ((ntab << lg) + ((size_t)1 << lge)) * 8));
            const uint32_t need = qimage_lds(lg, lge, m.dlg, (uint32_t)(J.img_nset[idx] + ntok_of(idx)), packed);
            cls.push_back(need == 0 ? 2 : (need <= kImgLdsSmall ? 0 : 1));
            ij.push_back(m);
        }
        std::vector<ImgJob> ord;
        ord.reserve(ij.size());
        int nc[3] = {0, 0, 0};
        int64_t scr = 0;
        for (int k = 0; k < 3; ++k)
            for (size_t x = 0; x < ij.size(); ++x)
                if (cls[x] == k) {
                    ImgJob m = ij[x];
                    m.scr_off = scr;
                    if (k == 2)  // set + u64 items + the table's u64 copy (the SoA transform)
                        scr += ((int64_t)1 << m.dlg) + 2 * ((int64_t)J.img_nset[m.idx] + ntok_of(m.idx)) +
                               2 * (((int64_t)(c->hs.packed ? 1 : 3) << m.lg) + ((int64_t)1 << m.lge));
                    ord.push_back(m);
                    ++nc[k];
                }
        if (!ord.empty()) {
            HIPCHK(c, upload(c, d_ij, ord));
            HIPCHK(c, d_scr.ensure((size_t)std::max<int64_t>(scr, 1) * 4));
            HIPCHK(c, launch_qimages(c->ds, J.js, d_ij.as<ImgJob>(), nc[0], nc[1], nc[2], J.d_pimg.as<uint8_t>() + off[i0],
                                     d_scr.as<uint32_t>(), d_fail.as<int32_t>(), c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));  // d_ij / d_scr are reused by the next batch
        }
        i0 = i1;
    }
    int32_t failed = 0;
    HIPCHK(c, hipMemcpy(&failed, d_fail.p, 4, hipMemcpyDeviceToHost));
    if (failed) {  // a table that did not converge: the per-call builds report it for the calls that need it
        if (J.d_pimg.p) (void)hipFree(J.d_pimg.p);
        J.d_pimg.p = nullptr;
        J.d_pimg.cap = 0;
        return PF_OK;
    }
    J.pimg_off.swap(off);
    J.pimg = true;
    return PF_OK;
}

}  // namespace

// ---------------------------------------------------------------- open
int jobs_open(pf_ctx* c) {
    auto& J = c->jb;
    const HostCorpus& hc = c->hc;
    const HostStore& hs = c->hs;
    const int32_t n = hc.n, T = hc.T;
    const bool packed = hs.packed;
    J.ok = false;
    StageClock sc;
    // image-builder tables: QConst template, region rows, completion / age rows (glibc exp)
    QConst tmpl;
    qconst_template(hc, packed, tmpl);
    std::vector<QConst> tv(1, tmpl);
    std::vector<double> sreg(4 * 16, 0.0);
    for (int a = 1; a <= 3; ++a) {
        double r[4][4];
        qconst_sig_reg(hc, a, r);
        for (int b = 0; b < 4; ++b)
            for (int m = 0; m < 4; ++m) sreg[a * 16 + b * 4 + m] = r[b][m];
    }
    auto ratio_rows = [&](const std::vector<int32_t>& v, int slot, std::vector<int32_t>& vals, std::vector<double>& rows) {
        for (int32_t x : v) if (x > 0) vals.push_back(x);
        std::sort(vals.begin(), vals.end());
        vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
        rows.assign(vals.size() * (kValTab + 1), 0.0);
        par_jobs(vals.size(), [&](size_t i) { qconst_ratio_row(hc, slot, vals[i], &rows[i * (kValTab + 1)]); }, 16);
    };
    std::vector<int32_t> comp_vals, age_vals;
    std::vector<double> comp_rows, age_rows;
    ratio_rows(hc.comp, PF_F_COMPLETION, comp_vals, comp_rows);
    ratio_rows(hc.age, PF_F_AGE, age_vals, age_rows);
    // idf per column by tid rank (pf_store.h: the engine's token ids are column ranks), one dense
    // table for every column with an idf map
    std::vector<int64_t> dense_off(T, -1);
    std::vector<int32_t> dense_len(T, 0);
    std::vector<float> dense;
    for (int t = 0; t < T; ++t) {
        if (!hc.has_idf[t]) continue;
        dense_off[t] = (int64_t)dense.size();
        dense_len[t] = (int32_t)hc.idf[t].size();
        dense.insert(dense.end(), hc.idf[t].begin(), hc.idf[t].end());
    }
    if (dense.empty()) dense.push_back(1.0f);
    sc.lap("image-builder tables");
    // graph: nodes 0..n-1 = profiles (idx), then adj_list uids without a profile
    J.xnode.clear();
    J.g_uid.assign(hc.uid.begin(), hc.uid.end());
    std::vector<const std::pair<const int32_t, std::vector<int32_t>>*> rows;
    rows.reserve(hc.adj.size());
    for (auto& kv : hc.adj) rows.push_back(&kv);
    {
        // uid -> profile idx: a dense table when the uids are non-negative and not too sparse
        // (hc.uid is ascending), else bisection
        std::vector<int32_t> dense_idx;
        if (n > 0 && hc.uid.front() >= 0 && (int64_t)hc.uid.back() < 4 * (int64_t)n + 4096) {
            dense_idx.assign((size_t)hc.uid.back() + 1, -1);
            par_jobs((size_t)n, [&](size_t i) { dense_idx[hc.uid[i]] = (int32_t)i; }, 1 << 16);
        }
        auto profile = [&](int32_t u) -> bool {
            if (dense_idx.empty()) return hc.idx_of(u) >= 0;
            return u >= 0 && (size_t)u < dense_idx.size() && dense_idx[u] >= 0;
        };
        std::vector<std::vector<int32_t>> unknown(16);
        const size_t R = rows.size();
        std::vector<std::thread> ts;
        for (int w = 0; w < 16; ++w)
            ts.emplace_back([&, w]() {
                for (size_t r = w; r < R; r += 16) {
                    if (!profile(rows[r]->first)) unknown[w].push_back(rows[r]->first);
                    for (int32_t x : rows[r]->second)
                        if (!profile(x)) unknown[w].push_back(x);
                }
            });
        for (auto& t : ts) t.join();
        for (auto& u : unknown)
            for (int32_t x : u)
                if (!J.xnode.count(x)) {
                    J.xnode.emplace(x, (int32_t)J.g_uid.size());
                    J.g_uid.push_back(x);
                }
    }
    const int32_t M = (int32_t)J.g_uid.size();
    J.g_len.assign(M, -1);
    sc.lap("graph nodes");
    // uid -> node as a dense table when the uids are non-negative and not too sparse
    J.dense_node.clear();
    {
        int64_t mx = -1;
        bool ok = true;
        for (int32_t u : J.g_uid) {
            if (u < 0) { ok = false; break; }
            mx = std::max<int64_t>(mx, u);
        }
        if (ok && mx >= 0 && mx < 4 * (int64_t)M + 4096) {
            J.dense_node.assign((size_t)mx + 1, -1);
            for (int32_t x = 0; x < M; ++x) J.dense_node[J.g_uid[x]] = x;
        }
    }
    std::vector<int64_t> g_off(M, 0);
    std::vector<int32_t> rnode(rows.size());
    std::vector<int64_t> roff(rows.size() + 1, 0);
    for (size_t r = 0; r < rows.size(); ++r) roff[r + 1] = roff[r] + (int64_t)rows[r]->second.size();
    std::vector<int32_t> g_nbr((size_t)roff.back());
    par_jobs(rows.size(), [&](size_t r) {
        const int32_t x = node_of(c, rows[r]->first);
        rnode[r] = x;
        const auto& row = rows[r]->second;
        for (size_t k = 0; k < row.size(); ++k) g_nbr[roff[r] + k] = node_of(c, row[k]);
    }, 4096);
    for (size_t r = 0; r < rows.size(); ++r) {
        g_off[rnode[r]] = roff[r];
        J.g_len[rnode[r]] = (int32_t)rows[r]->second.size();
    }
    sc.lap("graph CSR");
    // clubs as dense indices (K7), per profile idx in profile order
    std::vector<int32_t> club_id;
    {  // the distinct club ids: each thread's chunk sorted and de-duplicated, then the (short) union
        const size_t N = hc.clubs.size(), th = 16, ch = (N + th - 1) / th;
        std::vector<std::vector<int32_t>> part(th);
        std::vector<std::thread> ts;
        for (size_t w = 0; w < th; ++w)
            ts.emplace_back([&, w]() {
                const size_t lo = std::min(N, w * ch), hi = std::min(N, lo + ch);
                part[w].assign(hc.clubs.begin() + lo, hc.clubs.begin() + hi);
                std::sort(part[w].begin(), part[w].end());
                part[w].erase(std::unique(part[w].begin(), part[w].end()), part[w].end());
            });
        for (auto& t : ts) t.join();
        for (auto& p : part) club_id.insert(club_id.end(), p.begin(), p.end());
        std::sort(club_id.begin(), club_id.end());
        club_id.erase(std::unique(club_id.begin(), club_id.end()), club_id.end());
    }
    std::vector<int32_t> club_dense(hc.clubs.size());
    par_jobs(hc.clubs.size(), [&](size_t k) {
        club_dense[k] = (int32_t)(std::lower_bound(club_id.begin(), club_id.end(), (int32_t)hc.clubs[k]) - club_id.begin());
    }, 1 << 16);
    sc.lap("club indices");
    // per profile: query-table size (pf_store.cpp build_query) and its raw set words
    J.img_lg.assign(n, 0);
    J.img_nset.assign(n, 0);
    par_jobs((size_t)n, [&](size_t i) {
        std::vector<uint32_t> v(hc.clubs.begin() + hc.club_off[i], hc.clubs.begin() + hc.club_off[i + 1]);
        std::sort(v.begin(), v.end());
        const size_t dc = (size_t)(std::unique(v.begin(), v.end()) - v.begin());
        v.assign(hc.friends.begin() + hc.friend_off[i], hc.friends.begin() + hc.friend_off[i + 1]);
        std::sort(v.begin(), v.end());
        const size_t df = (size_t)(std::unique(v.begin(), v.end()) - v.begin());
        const size_t nt = (size_t)(hc.tok_off[(i + 1) * (size_t)T] - hc.tok_off[i * (size_t)T]);
        const int lg = packed ? lg_for(dc + df + nt) : std::max({lg_for(dc), lg_for(df), lg_for(nt)});
        const bool ok = lg <= kMaxHashLog2 && nt < (packed ? (1u << kTidBits) : (1u << 22));
        J.img_lg[i] = ok ? (uint8_t)lg : 0;
        J.img_nset[i] = (int32_t)((hc.club_off[i + 1] - hc.club_off[i]) + (hc.friend_off[i + 1] - hc.friend_off[i]));
    }, 4096);
    // per profile: its completion / age rows in the image-builder tables (ImgJob::rows)
    // (0xFFFFFFFF: more than 65534 distinct values, K6 looks the rows up itself)
    const bool rows16 = comp_vals.size() < 0xFFFFu && age_vals.size() < 0xFFFFu;
    J.img_rows.assign(n, rows16 ? 0u : 0xFFFFFFFFu);
    if (rows16) par_jobs((size_t)n, [&](size_t i) {
        auto row = [](const std::vector<int32_t>& vals, int32_t v) -> uint32_t {
            if (v <= 0) return 0u;
            auto it = std::lower_bound(vals.begin(), vals.end(), v);
            return (it != vals.end() && *it == v) ? (uint32_t)(it - vals.begin()) + 1u : 0u;
        };
        J.img_rows[i] = row(comp_vals, hc.comp[i]) | (row(age_vals, hc.age[i]) << 16);
    }, 1 << 14);
    std::vector<int32_t> slot_of(hs.slot_of_idx.begin(), hs.slot_of_idx.end());
    sc.lap("image sizes");
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = up(c, J.d_tmpl, tv);
    if (e == hipSuccess) e = up(c, J.d_sigreg, sreg);
    if (e == hipSuccess) e = up(c, J.d_comp_vals, comp_vals);
    if (e == hipSuccess) e = up(c, J.d_comp_rows, comp_rows);
    if (e == hipSuccess) e = up(c, J.d_age_vals, age_vals);
    if (e == hipSuccess) e = up(c, J.d_age_rows, age_rows);
    if (e == hipSuccess) e = up(c, J.d_idf_doff, dense_off);
    if (e == hipSuccess) e = up(c, J.d_idf_dlen, dense_len);
    if (e == hipSuccess) e = up(c, J.d_idf_dense, dense);
    if (e == hipSuccess) e = up(c, J.d_slot_of, slot_of);
    if (e == hipSuccess) e = up(c, J.d_goff, g_off);
    if (e == hipSuccess) e = up(c, J.d_glen, J.g_len);
    if (e == hipSuccess) e = up(c, J.d_gnbr, g_nbr);
    if (e == hipSuccess) e = up(c, J.d_guid, J.g_uid);
    if (e == hipSuccess) e = up(c, J.d_club_off, hc.club_off);
    if (e == hipSuccess) e = up(c, J.d_club_dense, club_dense);
    if (e == hipSuccess) e = up(c, J.d_club_id, club_id);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // the host vectors die here
    if (e != hipSuccess) return c->hip_fail(e, "job pipeline upload");
    sc.lap("upload");
    DevJobsStore& g = J.js;
    g.tmpl = J.d_tmpl.as<QConst>();
    g.sig_reg = J.d_sigreg.as<double>();
    g.comp_vals = J.d_comp_vals.as<int32_t>();
    g.comp_rows = J.d_comp_rows.as<double>();
    g.age_vals = J.d_age_vals.as<int32_t>();
    g.age_rows = J.d_age_rows.as<double>();
    g.n_comp = (int32_t)comp_vals.size();
    g.n_age = (int32_t)age_vals.size();
    g.idf_dense_off = J.d_idf_doff.as<int64_t>();
    g.idf_dense_len = J.d_idf_dlen.as<int32_t>();
    g.idf_dense = J.d_idf_dense.as<float>();
    g.slot_of = J.d_slot_of.as<int32_t>();
    g.g_off = J.d_goff.as<int64_t>();
    g.g_len = J.d_glen.as<int32_t>();
    g.g_nbr = J.d_gnbr.as<int32_t>();
    g.g_uid = J.d_guid.as<int32_t>();
    g.n = n;
    g.M = M;
    g.club_off = J.d_club_off.as<int64_t>();
    g.club_dense = J.d_club_dense.as<int32_t>();
    g.club_id = J.d_club_id.as<int32_t>();
    g.n_club_ids = (int32_t)club_id.size();
    J.edited.clear();
    J.edit_gen = 1;
    J.view_gen = 0;
    J.view_over = nullptr;
    J.view_over_n = 0;
    J.nodes_dirty = false;
    sc.lap("handles");
    const int rc = build_resident_images(c);
    if (rc != PF_OK) return rc;
    sc.lap(J.pimg ? ("resident images, " + std::to_string(J.d_pimg.cap >> 20) + " MiB").c_str() : "resident images (off)");
    J.ok = true;
    return PF_OK;
}

// A batched driver call starts or ends: its versioned edit set (a map on the driver's stack) is
// new, so the next call uploads the overrides again even when a later map lands at the same
// address with the same size.
void jobs_view_scope(pf_ctx* c) {
    ++c->jb.call_gen;
    c->jb.view_over = nullptr;
    c->jb.view_over_n = 0;
}

// pf_set_adj (test.cpp:73, recommendation_tests.cpp:111-114 mutate adj_list between queries):
// the host row changes now, the device graph sees it through the override table at the next job
// batch.  An edit that restores the open-time row drops the override, so a caller that edits and
// restores rows (the drivers, the C++ facade) keeps the table small.
int jobs_set_adj(pf_ctx* c, int32_t uid, const int32_t* nbrs, int32_t n) {
    const int rc = jobs_drain(c);  // calls in flight read the adjacency they were launched with
    if (rc != PF_OK) return rc;
    auto& adj = c->hc.adj;
    auto& J = c->jb;
    auto it = adj.find(uid);
    if (J.ok && !J.orig.count(uid))
        J.orig.emplace(uid, it == adj.end() ? std::make_pair(false, std::vector<int32_t>())
                                            : std::make_pair(true, it->second));
    if (n < 0) {
        if (it != adj.end()) adj.erase(it);
    } else {
        adj[uid].assign(nbrs, nbrs + n);
    }
    if (!J.ok) return PF_OK;
    ensure_node(c, uid);
    for (int32_t k = 0; k < n; ++k) ensure_node(c, nbrs[k]);
    const auto& o = J.orig.at(uid);
    const bool base = n < 0 ? !o.first : (o.first && (int64_t)o.second.size() == n &&
                                          std::equal(o.second.begin(), o.second.end(), nbrs));
    if (base) {
        J.edited.erase(uid);
        J.orig.erase(uid);
    } else {
        J.edited.insert(uid);
    }
    ++J.edit_gen;
    return PF_OK;
}

namespace {

// Before a graph / view upload rewrites buffers the device may still read: the context's stream
// waits for every pending asynchronous call's last work (W.done, recorded on aux2 after its K7,
// the clubs jobs' K8 and the result copies), which nothing on the context's stream orders.
int wait_pending_on_stream(pf_ctx* c) {
    auto& J = c->jb;
    for (const auto& p : J.pending)
        if (J.ws[p.slot].done) HIPCHK(c, hipStreamWaitEvent(c->stream, J.ws[p.slot].done, 0));
    if (J.carry.on && J.ws[J.carry.slot].done) HIPCHK(c, hipStreamWaitEvent(c->stream, J.ws[J.carry.slot].done, 0));
    return PF_OK;
}

// the node arrays grew (pf_set_adj named new uids): upload them again
int sync_nodes(pf_ctx* c) {
    auto& J = c->jb;
    if (!J.nodes_dirty) return PF_OK;
    if (const int rc = wait_pending_on_stream(c); rc != PF_OK) return rc;
    const int32_t M = (int32_t)J.g_uid.size();
    std::vector<int64_t> off(M, 0);  // the new nodes have no base row
    std::vector<int64_t> old((size_t)J.js.M);
    HIPCHK(c, hipMemcpyAsync(old.data(), J.js.g_off, old.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::copy(old.begin(), old.end(), off.begin());
    DBuf noff;
    HIPCHK(c, upload(c, noff, off));
    HIPCHK(c, upload(c, J.d_glen, J.g_len));
    HIPCHK(c, upload(c, J.d_guid, J.g_uid));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::swap(J.d_goff.p, noff.p);
    std::swap(J.d_goff.cap, noff.cap);
    J.js.g_off = J.d_goff.as<int64_t>();
    J.js.g_len = J.d_glen.as<int32_t>();
    J.js.g_uid = J.d_guid.as<int32_t>();
    J.js.M = M;
    J.nodes_dirty = false;
    return PF_OK;
}

// The overrides this call sees: pf_set_adj's edits (always) and the batched drivers' versioned
// edits `over` (AdjView::over), uploaded again only when either changed.
int sync_view(pf_ctx* c, const std::unordered_map<int32_t, std::pair<int32_t, std::vector<int32_t>>>* over) {
    auto& J = c->jb;
    const size_t on = over ? over->size() : 0;
    // current: the same edits and the same versioned edit set (a call's over map may reuse a freed
    // one's address, so a non-null set is current only within the driver call that uploaded it)
    if (J.view_gen == J.edit_gen &&
        (over == nullptr ? !J.view_has_over
                         : (J.view_over == (const void*)over && J.view_over_n == on && J.view_call == J.call_gen)))
        return PF_OK;
    struct E { int32_t node, ver; int32_t len; const std::vector<int32_t>* row; };
    std::vector<E> es;
    for (int32_t u : J.edited) {
        auto it = c->hc.adj.find(u);
        es.push_back(E{node_of(c, u), INT_MIN, it == c->hc.adj.end() ? -1 : (int32_t)it->second.size(),
                       it == c->hc.adj.end() ? nullptr : &it->second});
    }
    if (over)
        for (auto& kv : *over)
            es.push_back(E{node_of(c, kv.first), kv.second.first, (int32_t)kv.second.second.size(), &kv.second.second});
    for (const E& x : es)
        if (x.node < 0) return c->fail(PF_EINTERNAL, "adjacency override names an unmapped uid");
    if (const int rc = wait_pending_on_stream(c); rc != PF_OK) return rc;
    std::sort(es.begin(), es.end(), [](const E& a, const E& b) { return a.node != b.node ? a.node < b.node : a.ver > b.ver; });
    std::vector<int32_t> node(es.size()), ver(es.size()), len(es.size()), nbr;
    std::vector<int64_t> off(es.size());
    for (size_t i = 0; i < es.size(); ++i) {
        node[i] = es[i].node;
        ver[i] = es[i].ver;
        len[i] = es[i].len;
        off[i] = (int64_t)nbr.size();
        if (es[i].row)
            for (int32_t x : *es[i].row) {
                const int32_t y = node_of(c, x);
                if (y < 0) return c->fail(PF_EINTERNAL, "adjacency override names an unmapped uid");
                nbr.push_back(y);
            }
    }
    if (nbr.empty()) nbr.push_back(0);
    HIPCHK(c, upload(c, J.d_view_node, node));
    HIPCHK(c, upload(c, J.d_view_ver, ver));
    HIPCHK(c, upload(c, J.d_view_off, off));
    HIPCHK(c, upload(c, J.d_view_len, len));
    HIPCHK(c, upload(c, J.d_view_nbr, nbr));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    J.view.node = J.d_view_node.as<int32_t>();
    J.view.ver = J.d_view_ver.as<int32_t>();
    J.view.off = J.d_view_off.as<int64_t>();
    J.view.len = J.d_view_len.as<int32_t>();
    J.view.nbr = J.d_view_nbr.as<int32_t>();
    J.view.n = (int32_t)es.size();
    J.view_gen = J.edit_gen;
    J.view_over = over;
    J.view_over_n = on;
    J.view_has_over = on > 0;
    J.view_call = J.call_gen;
    return PF_OK;
}

// One planned job (host side).
struct JP {
    int kind = -1;               // DevJobKind, -1 = no device work (empty result)
    int32_t u = -1;              // query node
    std::vector<int32_t> F;      // row(u) as nodes
    std::vector<int32_t> fd;     // distinct friends with a profile, first-occurrence order
    std::vector<int32_t> fpos;   // per row position: index into fd or -1
    std::vector<int32_t> flen;   // clubs: |row(fd[r])| (0 when absent)
    std::vector<int32_t> own;    // own row as nodes (when the view replaces u's row)
    int32_t own_node = -1, own_len = -1;
    int64_t cap = 0, seqlen = 0;
    int ht_lg = 0;
    int64_t elems = 0, ht_words = 0;
    bool unmapped = false;       // a row names a uid without a graph node (never expected: open and
                                 // pf_set_adj give every adjacency uid one); the call fails loudly
};

// Plan job i of `jobs` under its view: 1-hop work only.
void plan_job(pf_ctx* c, const Job& Jb, JP& p, bool raw) {
    const HostCorpus& hc = c->hc;
    const int32_t uid = Jb.uid;
    const int32_t u = raw ? node_of(c, uid) : hc.idx_of(uid);
    if (u < 0 || (!raw && Jb.topk <= 0)) return;  // recommender_graph.cpp:39-40,130; recommender_clubs.cpp:16
    p.u = u;
    const std::vector<int32_t>* ru = Jb.view.row(uid);
    if (Jb.view.own_row) {  // recommendation_tests.cpp:111-114: the user's row replaced
        const int32_t o = node_of(c, Jb.view.own);
        if (o >= 0) {
            p.own_node = o;
            p.own_len = (int32_t)Jb.view.own_row->size();
            for (int32_t x : *Jb.view.own_row) p.own.push_back(node_of(c, x));
        }
    }
    if (ru) {
        p.F.reserve(ru->size());
        for (int32_t x : *ru) p.F.push_back(node_of(c, x));
    }
    // K3's hash table keys nodes as node + 1 (0 = empty): a node of -1 would alias an empty slot
    for (int32_t x : p.F) p.unmapped |= x < 0;
    for (int32_t x : p.own) p.unmapped |= x < 0;
    const int64_t L = std::max<int32_t>(Jb.limit, 1);
    // |row(node)| under the view: the base CSR's length unless an edit or the view covers it.
    // Without pf_set_adj edits or versioned edits, the view differs from the base only in the
    // query's own replaced row (recommendation_tests.cpp:111-114): every other node reads g_len
    // instead of a lookup in the 1.6M-row adjacency hash map
    const bool base_ok = c->jb.edited.empty() && !Jb.view.over;
    auto rowlen = [&](int32_t node) -> int64_t {
        if (base_ok && node >= 0 && node < (int32_t)c->jb.g_len.size()) {
            if (Jb.view.own_row && node == p.own_node) return (int64_t)Jb.view.own_row->size();
            return c->jb.g_len[node];
        }
        const std::vector<int32_t>* r = Jb.view.row(c->jb.g_uid[node]);
        return r ? (int64_t)r->size() : -1;
    };
    if (raw || Jb.kind == kJobInterest) {
        const bool graph = raw ? Jb.limit_flavour == PF_FOF_GRAPH : true;
        if (!raw && Jb.all_candidates) {
            p.kind = kDjAll;
            p.cap = hc.n;
            p.ht_lg = pow2_lg(2 * ((int64_t)p.F.size() + 1));
        } else {
            p.kind = raw ? (graph ? kDjRawGraph : kDjRawCollab) : kDjInterest;
            for (int32_t f : p.F) {
                const int64_t rl = rowlen(f);
                if (graph) p.seqlen += f == u ? 0 : 1 + std::max<int64_t>(rl, 0);
                else p.seqlen += std::max<int64_t>(rl, 0);
            }
            p.cap = std::min<int64_t>(L, p.seqlen);
            p.ht_lg = pow2_lg(2 * ((int64_t)p.F.size() + 1 + p.cap + kGatherChunk));
        }
        p.elems = p.cap;
        p.ht_words = 3ll << p.ht_lg;
        return;
    }
    // collab / clubs: sim_u_f over the distinct friends with a profile (recommender_graph.cpp:132-136)
    p.fpos.reserve(p.F.size());
    p.fd.reserve(p.F.size());
    if (p.F.size() <= 64) {  // the common case: a linear scan beats a hash map's allocations
        for (int32_t f : p.F) {
            if (f < 0 || f >= hc.n) { p.fpos.push_back(-1); continue; }
            int32_t pos = -1;
            for (size_t r = 0; r < p.fd.size(); ++r)
                if (p.fd[r] == f) { pos = (int32_t)r; break; }
            if (pos < 0) {
                pos = (int32_t)p.fd.size();
                p.fd.push_back(f);
            }
            p.fpos.push_back(pos);
        }
    } else {
        std::unordered_map<int32_t, int32_t> seen;
        seen.reserve(p.F.size());
        for (int32_t f : p.F) {
            if (f < 0 || f >= hc.n) { p.fpos.push_back(-1); continue; }
            auto it = seen.find(f);
            if (it == seen.end()) {
                it = seen.emplace(f, (int32_t)p.fd.size()).first;
                p.fd.push_back(f);
            }
            p.fpos.push_back(it->second);
        }
    }
    if (Jb.kind == kJobCollab) {
        p.kind = kDjCollab;
        for (int32_t f : p.F) p.seqlen += std::max<int64_t>(rowlen(f), 0);
        p.cap = std::min<int64_t>(L, p.seqlen);
        p.ht_lg = pow2_lg(2 * ((int64_t)p.F.size() + 1 + p.cap + kGatherChunk));
        p.elems = p.cap + (int64_t)p.fd.size() * (1 + p.cap);
        p.ht_words = 3ll << p.ht_lg;
    } else {
        p.kind = kDjClubs;
        int64_t s = 0;
        for (int32_t f : p.fd) {
            const int64_t rl = std::max<int64_t>(rowlen(f), 0);
            p.flen.push_back((int32_t)rl);
            s += rl;
        }
        p.elems = (int64_t)p.fd.size() + s + c->jb.js.n_club_ids;
    }
}

// Launches jobs[b, e) (planned in P) on the device with workspaces W: every stage and the
// result copies are queued on the context's stream and W.done is recorded after them;
// finish_chunk waits for it and fills jobs[i].out (or raw lists in raw_out).
int launch_chunk(pf_ctx* c, std::vector<Job>& jobs, std::vector<JP>& P, size_t b, size_t e, JobsState::Ws& W) {
    auto& J = c->jb;
    W.active = false;
    const HostCorpus& hc = c->hc;
    const bool packed = c->hs.packed;
    HpLap hl;
    // ---- layout
    std::vector<DevJob> dj;
    std::vector<int32_t> pool32;
    std::vector<int64_t> pool64;
    std::vector<int32_t> jmap;  // dj index -> job index
    int64_t E = 0, HT = 0, SEQ = 0;
    std::vector<int32_t> img_idx;
    if (J.img_stamp.size() != (size_t)hc.n || ++J.img_gen == 0) {  // a stamp per profile idx
        J.img_stamp.assign((size_t)hc.n, 0u);
        J.img_pos.assign((size_t)hc.n, 0);
        J.img_gen = 1;
    }
    const uint32_t gen = J.img_gen;
    auto img = [&](int32_t idx) {
        if (J.img_stamp[idx] == gen) return J.img_pos[idx];
        const int32_t k = (int32_t)img_idx.size();
        J.img_stamp[idx] = gen;
        J.img_pos[idx] = k;
        img_idx.push_back(idx);
        return k;
    };
    // The pair blocks as runs (PairGen, expanded on the device by K9 expand_pairs_kernel): a run is
    // ceil(cap / kPairSpan) candidate chunks x nf (image, row) entries of the pool, chunk-major, so
    // the host writes ~one run per job and image class instead of ~140k 16-B blocks per cfg-5 chunk
    // (their layout was ~2.3 ms of host time per chunk, r4m host clocks).  Runs are built per job
    // here (images as img() indices), then split by the images' LDS class below.
    struct RawGen {
        int32_t nch, cap, cand, out, stride, fl, nf;
    };
    std::vector<RawGen> rgen;
    std::vector<int2> gpool;  // (image, row) entries of the runs
    auto add_gen = [&](int64_t cap, int64_t cand, int64_t out, int64_t stride, const int2* ents, int nf) {
        if (cap <= 0 || nf <= 0) return;
        rgen.push_back(RawGen{(int32_t)((cap + kPairSpan - 1) / kPairSpan), (int32_t)cap, (int32_t)cand, (int32_t)out,
                              (int32_t)stride, (int32_t)gpool.size(), nf});
        gpool.insert(gpool.end(), ents, ents + nf);
    };
    auto add_blocks = [&](int32_t im, int64_t begin, int64_t count, int64_t out) {
        const int2 e = make_int2(im, 0);
        add_gen(count, begin, out, 0, &e, 1);
    };
    std::vector<int32_t> jix_collab, jix_clubs, jix_topk, jix_fused, jix_ctopk;
    int max_cap_collab = 0, ktop = 1;
    const int lge = lg_for(0);
    auto ntok_of = [&](int32_t idx) { return hc.tok_off[(size_t)(idx + 1) * hc.T] - hc.tok_off[(size_t)idx * hc.T]; };
    {
        size_t ng = 0, words = 0;  // the runs and pool words this chunk appends (one allocation)
        for (size_t i = b; i < e; ++i) {
            const JP& p = P[i];
            if (p.kind < 0) continue;
            ng += 2 + p.fd.size();
            words += p.own.size() + p.F.size() + 2 * p.fd.size();
        }
        rgen.reserve(ng);
        gpool.reserve(ng + 2 * (e - b));
        pool32.reserve(words + 1);
    }
    for (size_t i = b; i < e; ++i) {
        JP& p = P[i];
        if (p.kind < 0) continue;
        DevJob d{};
        d.kind = p.kind;
        d.u = p.u;
        d.L = std::max<int32_t>(jobs[i].limit, 1);
        d.version = jobs[i].view.version;
        d.own = p.own_node;
        d.own_len = p.own_len;
        d.own_off = (int64_t)pool32.size();
        pool32.insert(pool32.end(), p.own.begin(), p.own.end());
        d.f_off = (int64_t)pool32.size();
        pool32.insert(pool32.end(), p.F.begin(), p.F.end());
        d.nf = (int32_t)p.F.size();
        d.ht_lg = p.ht_lg;
        d.ht_off = HT;
        HT += p.ht_words;
        d.seg_off = SEQ;
        SEQ += (int64_t)p.F.size() + 1;
        d.cap = (int32_t)p.cap;
        d.topk = jobs[i].topk;
        d.nfd = (int32_t)p.fd.size();
        d.fd_off = (int64_t)pool32.size();
        pool32.insert(pool32.end(), p.fd.begin(), p.fd.end());
        d.fpos_off = (int64_t)pool32.size();
        pool32.insert(pool32.end(), p.fpos.begin(), p.fpos.end());
        const int32_t jn = (int32_t)dj.size();
        if (p.kind == kDjClubs) {
            d.sim_off = E;
            E += d.nfd;
            d.sreg_off = (int64_t)pool64.size();
            for (size_t r = 0; r < p.fd.size(); ++r) {
                pool64.push_back(E);
                E += p.flen[r];
            }
            d.out_off = E;
            d.cand_off = E;
            E += J.js.n_club_ids;
            const int32_t iu = img(p.u);
            add_blocks(iu, d.sim_off, d.nfd, d.sim_off);
            for (size_t r = 0; r < p.fd.size(); ++r) add_blocks(img(p.fd[r]), pool64[d.sreg_off + r], p.flen[r], pool64[d.sreg_off + r]);
            jix_clubs.push_back(jn);
        } else {
            d.cand_off = E;
            d.out_off = E;
            E += p.cap;
            if (p.kind == kDjCollab) {
                d.sim_off = E;
                E += d.nfd;
                d.m_off = E;
                E += (int64_t)d.nfd * p.cap;
                const int32_t iu = img(p.u);
                add_blocks(iu, d.sim_off, d.nfd, d.sim_off);
                // candidate-chunk major: the friends' blocks of one candidate chunk are
                // consecutive, so they run together and share the chunk's records in cache;
                // a block scores span() candidates against one staged friend image
                // (block (x, r): friend r's image, candidates cand_off + x * span, out m_off + r * cap + x * span)
                std::vector<int2> fe(d.nfd);
                for (int r = 0; r < d.nfd; ++r) fe[r] = make_int2(img(p.fd[r]), r);
                add_gen(p.cap, d.cand_off, d.m_off, p.cap, fe.data(), d.nfd);
                jix_collab.push_back(jn);
                max_cap_collab = std::max<int>(max_cap_collab, (int)p.cap);
            } else if (p.kind == kDjInterest || p.kind == kDjAll) {
                add_blocks(img(p.u), d.cand_off, p.cap, d.cand_off);
            }
        }
        if (p.kind != kDjRawGraph && p.kind != kDjRawCollab && jobs[i].topk <= kDevTopK) {
            // a collaborative job with candidates gets its top-k inside K4' (collab_kernel); the
            // clubs jobs' K8 runs after K7 on the second aux stream (jix_ctopk, appended below)
            (p.kind == kDjCollab && p.cap > 0 ? jix_fused : (p.kind == kDjClubs ? jix_ctopk : jix_topk)).push_back(jn);
            ktop = std::max(ktop, jobs[i].topk);
        }
        dj.push_back(d);
        jmap.push_back((int32_t)i);
    }
    if (dj.empty()) return PF_OK;
    const int n_topk_main = (int)jix_topk.size();  // K8 on the context's stream; the clubs jobs' after them
    jix_topk.insert(jix_topk.end(), jix_ctopk.begin(), jix_ctopk.end());
    if (W.done == nullptr) {
        HIPCHK(c, hipEventCreateWithFlags(&W.done, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&W.ev_pairs, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&W.ev_main, hipEventDisableTiming));
    }
    const hipStream_t s = c->stream;
    if (E >= INT32_MAX) return c->fail(PF_EUNSUPP, "job batch too large for one pair launch");
    // ---- images (pf_api.cpp plan_images layout).  Resident (J.pimg, built at open): every
    // user's image already sits in J.d_pimg and the batch only references them.  Otherwise K6
    // builds the batch's images, the ones it builds in LDS first.
    const bool resident = J.pimg;
    const uint32_t ntab = packed ? 1u : 3u;
    auto dlg_of = [&](int32_t idx) { return pow2_lg(2 * (int64_t)J.img_nset[idx] + 2); };
    // K6 builds the images in three launches: small LDS builds (<= kImgLdsSmall, many workgroups
    // per CU), large LDS builds (<= kImgLds), hub users in global memory
    int n_lds = 0, n_small = 0;
    if (!resident) {
        std::vector<int32_t> order(img_idx.size()), pos(img_idx.size());
        std::vector<uint8_t> cls(img_idx.size());  // 0 small, 1 large, 2 global
        for (size_t k = 0; k < img_idx.size(); ++k) {
            const int32_t idx = img_idx[k];
            const uint32_t need = J.img_lg[idx] ? qimage_lds(J.img_lg[idx], lge, dlg_of(idx),
                                                             (uint32_t)(J.img_nset[idx] + ntok_of(idx)), packed)
                                                : 0u;
            cls[k] = need == 0 ? 2 : (need <= kImgLdsSmall ? 0 : 1);
            n_lds += cls[k] < 2;
            n_small += cls[k] == 0;
        }
        int a = 0, b2 = n_small, g2 = n_lds;
        for (size_t k = 0; k < img_idx.size(); ++k) pos[k] = cls[k] == 0 ? a++ : (cls[k] == 1 ? b2++ : g2++);
        for (size_t k = 0; k < img_idx.size(); ++k) order[pos[k]] = img_idx[k];
        img_idx.swap(order);
        for (int2& ge : gpool) ge.x = pos[ge.x];
    }
    std::vector<ImgJob> ij(resident ? 0 : img_idx.size());
    std::vector<QImageRef> refs(img_idx.size());
    size_t ipool = 0;
    int64_t scr = 0;
    for (size_t k = 0; k < img_idx.size(); ++k) {
        const int32_t idx = img_idx[k];
        const int lg = J.img_lg[idx];
        if (lg == 0) return c->fail(PF_EUNSUPP, "query hash table too large");
        const int64_t ntok = ntok_of(idx);
        const size_t nkeys = ((size_t)ntab << lg) + ((size_t)1 << lge);
        QImageRef& r = refs[k];
        r.keys_off = (uint32_t)sizeof(QConst);
        r.vals_off = (uint32_t)a16z(sizeof(QConst) + nkeys * 8);
        if (resident) {
            r.const_off = (uint32_t)(J.pimg_off[idx] >> 4);
        } else {
            ImgJob& m = ij[k];
            m.idx = idx;
            m.lg = lg;
            m.lge = lge;
            m.dlg = dlg_of(idx);
            m.rows = J.img_rows[idx];
            m.const_off = (uint32_t)ipool;
            m.keys_off = (uint32_t)(ipool + r.keys_off);
            m.vals_off = (uint32_t)(ipool + r.vals_off);
            r.const_off = (uint32_t)(ipool >> 4);
            ipool = a16z(m.vals_off + (size_t)ntok * sizeof(QVal));
            if (ipool >= (size_t)UINT32_MAX) return c->fail(PF_EUNSUPP, "query images of one batch exceed 4 GB");
            m.scr_off = scr;
            if ((int)k >= n_lds)  // set + u64 items + the table's u64 copy (the SoA transform)
                scr += ((int64_t)1 << m.dlg) + 2 * ((int64_t)J.img_nset[idx] + ntok) + 2 * (int64_t)nkeys;
        }
        const size_t kv = nkeys * 8 + (size_t)ntok * sizeof(QVal);
        r.lds_bytes = kv <= kStageLimitJobs ? (uint32_t)kv : 0u;
    }
    // The pair blocks in three launches by their image: LDS-staged images whose block fits two
    // workgroups per CU, larger LDS-staged ones, global-memory tables.  One launch sized for the
    // batch's largest image ran every block of 6 % of the cfg-3 steps at one workgroup per CU
    // (484 vs 338 us, r3ad), and one global-table image switched every block to global probes.
    uint32_t lds_c[3] = {0u, 0u, 0u};
    int nb_c[3] = {0, 0, 0};
    std::vector<PairGen> gens;  // by class, `first` = the run's first block
    std::vector<int2> gp2;      // their (image, row) entries
    int64_t nblk = 0;           // pair blocks of the chunk
    {
        constexpr uint32_t kTwoPerCu = 80u * 1024u;  // 160 KB of LDS per CU
        std::vector<uint8_t> icls(refs.size());
        for (size_t k = 0; k < refs.size(); ++k) {
            const uint32_t need = (uint32_t)sizeof(QConst) + refs[k].lds_bytes +
                                  kHitSlots * (packed ? 4u : 8u) * kPairThreads + 4u * kPairThreads + 2048u;
            icls[k] = refs[k].lds_bytes == 0 ? 2 : (need <= kTwoPerCu ? 0 : 1);
            lds_c[icls[k]] = std::max(lds_c[icls[k]], need);
        }
        // each run split by class (its entries of one class keep their order); the classes'
        // blocks are consecutive, class 0 first
        gens.reserve(rgen.size() + 8);
        gp2.reserve(gpool.size());
        for (int k = 0; k < 3; ++k) {
            int64_t cnt = 0;
            for (const RawGen& g : rgen) {
                const int32_t fl = (int32_t)gp2.size();
                for (int f = 0; f < g.nf; ++f)
                    if (icls[gpool[g.fl + f].x] == k) gp2.push_back(gpool[g.fl + f]);
                const int32_t nf = (int32_t)gp2.size() - fl;
                if (nf == 0) continue;
                gens.push_back(PairGen{nf, g.nch, g.cap, g.cand, fl, g.stride, g.out, (int32_t)(nblk + cnt)});
                cnt += (int64_t)g.nch * nf;
            }
            if (nblk + cnt >= INT32_MAX) return c->fail(PF_EUNSUPP, "job batch too large for one pair launch");
            nb_c[k] = (int)cnt;
            nblk += cnt;
        }
    }
    hl.lap(kHpImages);
    // ---- staging: [DevJob | pool32 | pool64 | ImgJob | QImageRef | PairBlock | jix x3], then the
    // chunk's result region [fail word (16 B, uploaded as zero) | ncand | top-k keys], so one
    // upload and one download carry everything (no memset, one result copy)
    if (pool32.empty()) pool32.push_back(0);
    if (pool64.empty()) pool64.push_back(0);
    const size_t o_dj = 0;
    const size_t o_p32 = a16z(o_dj + dj.size() * sizeof(DevJob));
    const size_t o_p64 = a16z(o_p32 + pool32.size() * 4);
    const size_t o_ij = a16z(o_p64 + pool64.size() * 8);
    const size_t o_refs = a16z(o_ij + ij.size() * sizeof(ImgJob));
    const size_t o_blk = a16z(o_refs + refs.size() * sizeof(QImageRef));
    const size_t o_gp = a16z(o_blk + std::max<size_t>(gens.size(), 1) * sizeof(PairGen));
    const size_t o_jc = a16z(o_gp + std::max<size_t>(gp2.size(), 1) * sizeof(int2));
    const size_t o_jk = a16z(o_jc + jix_collab.size() * 4);
    const size_t o_jt = a16z(o_jk + jix_clubs.size() * 4);
    const size_t o_tk = a16z(o_jt + jix_topk.size() * 4);  // K4' top-k tickets (zero), one per collaborative job
    const size_t o_res = a16z(o_tk + jix_collab.size() * 4);
    const size_t o_rcnt = o_res + 16, o_rkeys = o_rcnt + a16z(dj.size() * 4);
    const size_t res_b = o_rkeys - o_res + dj.size() * (size_t)ktop * 8;
    const size_t total = o_res + 16;  // uploaded: the plan and the zero fail word
    HIPCHK(c, W.h_plan.ensure(total));
    uint8_t* h = W.h_plan.as<uint8_t>();
    auto put = [&](size_t o, const void* src, size_t bytes) { if (bytes) std::memcpy(h + o, src, bytes); };
    put(o_dj, dj.data(), dj.size() * sizeof(DevJob));
    put(o_p32, pool32.data(), pool32.size() * 4);
    put(o_p64, pool64.data(), pool64.size() * 8);
    put(o_ij, ij.data(), ij.size() * sizeof(ImgJob));
    put(o_refs, refs.data(), refs.size() * sizeof(QImageRef));
    put(o_blk, gens.data(), gens.size() * sizeof(PairGen));
    put(o_gp, gp2.data(), gp2.size() * sizeof(int2));
    put(o_jc, jix_collab.data(), jix_collab.size() * 4);
    put(o_jk, jix_clubs.data(), jix_clubs.size() * 4);
    put(o_jt, jix_topk.data(), jix_topk.size() * 4);
    if (!jix_collab.empty()) std::memset(h + o_tk, 0, jix_collab.size() * 4);
    std::memset(h + o_res, 0, 16);
    const size_t o_ord = a16z(o_res + res_b);  // the pair blocks' dispatch order (device-written)
    const size_t o_bd = a16z(o_ord + std::max<size_t>((size_t)nblk, 1) * 4);  // the pair blocks (device-written, K9)
    HIPCHK(c, W.d_plan.reserve(o_bd + std::max<size_t>((size_t)nblk, 1) * sizeof(PairBlock)));
    if (J.aux == nullptr) {
        HIPCHK(c, hipStreamCreateWithFlags(&J.aux, hipStreamNonBlocking));
        HIPCHK(c, hipStreamCreateWithFlags(&J.aux2, hipStreamNonBlocking));
        HIPCHK(c, hipEventCreateWithFlags(&J.ev_fork, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&J.ev_join, hipEventDisableTiming));
    }
    // the plan goes up on the aux stream, where this chunk's gathers follow it at once: they run
    // beside the previous chunk's pair kernel (their slot's buffers were released when that slot's
    // previous chunk was unpacked); r3ab: cfg 3 +3 % over forking them from the context's stream
    // Ping-pong (default): consecutive chunks alternate between the aux stream and the context's
    // stream for their upload, gathers, images and pair kernel, so a chunk's pair kernel follows
    // its own gathers in stream order (no cross-stream wait in front of it: ~20 us per chunk in the
    // r7l trace) and may start beside the previous chunk's pair kernel.  A chunk's workspace slot is
    // reused only after its W.done (the caller waits it), so the two streams never share a slot's
    // buffers in flight.  (PF_DEBUG chunk_pingpong=0: the gathers on the aux stream, the images
    // and the pair kernel on the context's stream behind an event, as before)
    static const bool pingpong = debug_long("chunk_pingpong", 1) != 0;
    if (pingpong) J.pp ^= 1;
    const hipStream_t up = (!pingpong || J.pp) ? J.aux : s;  // upload, K9, K3, dispatch orders
    const hipStream_t sp = pingpong ? up : s;                // images, pair kernel, K4' / K8 with clubs
    HIPCHK(c, hipMemcpyAsync(W.d_plan.p, h, total, hipMemcpyHostToDevice, up));
    if (!pingpong) HIPCHK(c, hipEventRecord(J.ev_fork, up));
    uint8_t* d = W.d_plan.as<uint8_t>();
    const DevJob* d_dj = reinterpret_cast<const DevJob*>(d + o_dj);
    const int32_t* d_p32 = reinterpret_cast<const int32_t*>(d + o_p32);
    const int64_t* d_p64 = reinterpret_cast<const int64_t*>(d + o_p64);
    const ImgJob* d_ij = reinterpret_cast<const ImgJob*>(d + o_ij);
    const QImageRef* d_refs = reinterpret_cast<const QImageRef*>(d + o_refs);
    const PairGen* d_gen = reinterpret_cast<const PairGen*>(d + o_blk);
    const int2* d_gpool = reinterpret_cast<const int2*>(d + o_gp);
    PairBlock* d_blk = reinterpret_cast<PairBlock*>(d + o_bd);
    const int32_t* d_jc = reinterpret_cast<const int32_t*>(d + o_jc);
    const int32_t* d_jk = reinterpret_cast<const int32_t*>(d + o_jk);
    const int32_t* d_jt = reinterpret_cast<const int32_t*>(d + o_jt);
    unsigned int* d_tk = reinterpret_cast<unsigned int*>(d + o_tk);
    int32_t* d_fail = reinterpret_cast<int32_t*>(d + o_res);
    int32_t* d_ord = reinterpret_cast<int32_t*>(d + o_ord);
    int32_t* d_ncand = reinterpret_cast<int32_t*>(d + o_rcnt);
    uint64_t* d_keys = reinterpret_cast<uint64_t*>(d + o_rkeys);
    hl.lap(kHpPack);
    // ---- workspaces
    const size_t nE = (size_t)std::max<int64_t>(E, 1);
    HIPCHK(c, W.d_slots.reserve(nE * 4));
    HIPCHK(c, W.d_ids.reserve(nE * 4));
    HIPCHK(c, W.d_fl.reserve(nE * 4));
    HIPCHK(c, W.d_ht.reserve((size_t)std::max<int64_t>(HT, 1) * 4));
    HIPCHK(c, W.d_seq.reserve((size_t)std::max<int64_t>(SEQ, 1) * 4));
    if (!resident) {
        HIPCHK(c, W.d_img.reserve(std::max<size_t>(ipool, 16)));
        HIPCHK(c, W.d_scr.reserve((size_t)std::max<int64_t>(scr, 1) * 4));
    }
    const uint8_t* ipl = resident ? J.d_pimg.as<uint8_t>() : W.d_img.as<uint8_t>();  // the batch's image pool
    const int collab_gx = (max_cap_collab + 63) / 64;  // K4' blocks per job (pf_jobs.hip kCollabCands)
    if (!jix_collab.empty())
        HIPCHK(c, W.d_parts.reserve(jix_collab.size() * (size_t)std::max(collab_gx, 1) * (size_t)ktop * 8));
    hl.lap(kHpPlan);  // workspaces
    if (!jix_clubs.empty()) {
        const int64_t want = (int64_t)jix_clubs.size();
        if (want > W.acc_jobs) {
            const size_t words = (size_t)want * (size_t)std::max(J.js.n_club_ids, 1);
            HIPCHK(c, W.d_acc.ensure(words * 8));
            HIPCHK(c, hipMemsetAsync(W.d_acc.p, 0, W.d_acc.cap, sp));
            W.acc_jobs = want;
        }
    }
    // ---- the stages, in stream order; the gathers and dispatch orders run on the aux stream and
    // join before the pair kernel, beside the images
    if (!pingpong) HIPCHK(c, hipStreamWaitEvent(s, J.ev_fork, 0));  // the plan (images, fail word) is up
    HIPCHK(c, launch_expand_pairs(d_gen, (int)gens.size(), d_gpool, (int)nblk, d_blk, up));  // K9: the blocks
    HIPCHK(c, launch_gather(J.js, J.view, d_dj, (int)dj.size(), d_p32, d_p64, W.d_ht.as<int32_t>(),
                            W.d_seq.as<int32_t>(), W.d_slots.as<int32_t>(), W.d_ids.as<int32_t>(),
                            d_ncand, up));
    for (int k = 0, o = 0; k < 3; o += nb_c[k++])  // each launch's dispatch order (relative to its blocks)
        HIPCHK(c, launch_order_pairs(d_blk + o, nb_c[k], W.d_slots.as<int32_t>(), hc.n, d_ord + o, up));
    if (!pingpong) HIPCHK(c, hipEventRecord(J.ev_join, up));
    if (!resident)
        HIPCHK(c, launch_qimages(c->ds, J.js, d_ij, n_small, n_lds - n_small, (int)ij.size() - n_lds,
                                 W.d_img.as<uint8_t>(), W.d_scr.as<uint32_t>(), d_fail, sp));
    if (!pingpong) HIPCHK(c, hipStreamWaitEvent(s, J.ev_join, 0));
    const bool any_pairs = nblk > 0;
    hipEvent_t pe0 = nullptr, pe1 = nullptr;
    if ((J.stats_on || J.stats_count) && any_pairs) {
        if (J.stat_used == J.stat_ev.size()) {
            hipEvent_t a, b2;
            HIPCHK(c, timing_event(&a));
            HIPCHK(c, timing_event(&b2));
            J.stat_ev.emplace_back(a, b2);
        }
        pe0 = J.stat_ev[J.stat_used].first;
        pe1 = J.stat_ev[J.stat_used].second;
        ++J.stat_used;
        HIPCHK(c, hipEventRecord(pe0, sp));
    }
    for (int k = 0, o = 0; k < 3; o += nb_c[k++]) {  // the pair-scoring stage (timed)
        HIPCHK(c, launch_pairs(c->ds, ipl, d_refs, lds_c[k], k == 2, d_blk + o, nb_c[k], d_ord + o,
                               W.d_slots.as<int32_t>(), W.d_fl.as<float>(), sp));
        J.n_dispatch += nb_c[k] > 0;
    }
    if (pe1) {
        HIPCHK(c, hipEventRecord(pe1, sp));
        ++J.st_launches;
    }
    if (J.stats_count && any_pairs) {
        unsigned long long* acc = J.d_stats.as<unsigned long long>();
        HIPCHK(c, launch_pair_stats(c->ds, d_blk, (int)nblk, W.d_slots.as<int32_t>(), acc, sp));
        for (const PairGen& g : gens)  // the staged image per pair block (QConst + tables)
            for (int f = 0; f < g.nf; ++f) {
                const int32_t k = gp2[g.fl + f].x;
                J.st_img_bytes += (int64_t)g.nch * ((int64_t)refs[k].vals_off + ntok_of(img_idx[k]) * (int64_t)sizeof(QVal));
            }
    }
    hl.lap(kHpCollab);  // images, gathers, pairs launched
    // K7 (clubs) and its jobs' K8 go to the second aux stream once the pairs are scored (K7 ran
    // 0.8-1.4 ms per cfg-5 chunk between two pair kernels with the device mostly idle, r4k), and so
    // do K4' (collaborative, fused top-k) and the interest jobs' K8 when the chunk has no clubs jobs:
    // the context's stream then goes straight on to the next chunk's pair kernel (cfg-3 trace r7e:
    // K4' + K8 took ~40 us of every ~400-us step between two pair kernels; cfg3 +9 %, r7g).  With
    // clubs jobs K4' stays on the context's stream beside K7 (behind K7 on one stream, cfg 5 ran
    // 148k-162k vs 166k-171k users/s, r7h).  The chunk's result copies follow on the aux stream and
    // W.done is recorded last there.  Jobs write disjoint regions of the slot's buffers.
    // (PF_DEBUG collab_main=1: K4' and K8 on the context's stream always, the A/B)
    const hipStream_t s2 = J.aux2;
    static const bool collab_main = debug_long("collab_main", 0) != 0;
    const hipStream_t sc = (collab_main || !jix_clubs.empty()) ? sp : s2;
    HIPCHK(c, hipEventRecord(W.ev_pairs, sp));
    HIPCHK(c, hipStreamWaitEvent(s2, W.ev_pairs, 0));
    HIPCHK(c, launch_collab(d_dj, d_jc, (int)jix_collab.size(), max_cap_collab, d_p32, W.d_fl.as<float>(),
                            W.d_slots.as<int32_t>(), W.d_fl.as<float>(), W.d_ids.as<int32_t>(), W.d_parts.as<uint64_t>(),
                            d_tk, d_keys, ktop, sc));
    HIPCHK(c, launch_job_topk(d_dj, d_jt, n_topk_main, W.d_fl.as<float>(), W.d_ids.as<int32_t>(),
                              W.d_slots.as<int32_t>(), d_ncand, d_keys, ktop, sc));
    if (collab_main) HIPCHK(c, hipEventRecord(W.ev_main, sp));
    HIPCHK(c, launch_clubs(J.js, J.view, d_dj, d_jk, (int)jix_clubs.size(), d_p32, d_p64, W.d_fl.as<float>(),
                           W.d_acc.as<double>(), W.d_fl.as<float>(), W.d_ids.as<int32_t>(),
                           d_ncand, (int64_t)J.js.n_club_ids, s2));
    HIPCHK(c, launch_job_topk(d_dj, d_jt + n_topk_main, (int)jix_topk.size() - n_topk_main, W.d_fl.as<float>(),
                              W.d_ids.as<int32_t>(), W.d_slots.as<int32_t>(), d_ncand, d_keys, ktop, s2));
    if (collab_main) HIPCHK(c, hipStreamWaitEvent(s2, W.ev_main, 0));
    // ---- results: keys (top-k jobs), counts, the fail flag; full lists for the others
    std::vector<int32_t> tpos(dj.size(), -1);
    for (size_t t = 0; t < jix_topk.size(); ++t) tpos[jix_topk[t]] = (int32_t)t;
    for (size_t t = 0; t < jix_fused.size(); ++t) tpos[jix_fused[t]] = (int32_t)(jix_topk.size() + t);
    std::vector<size_t> full;  // dj indices copied whole
    size_t ob = res_b;  // [fail | ncand | keys] as on the device, then the full lists
    std::vector<size_t> full_off;
    for (size_t x = 0; x < dj.size(); ++x) {
        if (tpos[x] >= 0) continue;
        full.push_back(x);
        full_off.push_back(ob);
        ob += a16z((size_t)std::max(dj[x].cap, dj[x].kind == kDjClubs ? J.js.n_club_ids : 0) * 12);
    }
    HIPCHK(c, W.h_out.ensure(ob));
    uint8_t* ho = W.h_out.as<uint8_t>();
    const size_t o_fail = 0, o_cnt = o_rcnt - o_res, o_keys = o_rkeys - o_res;
    HIPCHK(c, hipMemcpyAsync(ho, d + o_res, res_b, hipMemcpyDeviceToHost, s2));
    for (size_t q = 0; q < full.size(); ++q) {
        const DevJob& x = dj[full[q]];
        const size_t cnt = (size_t)std::max(x.cap, x.kind == kDjClubs ? J.js.n_club_ids : 0);
        uint8_t* dst = ho + full_off[q];
        HIPCHK(c, hipMemcpyAsync(dst, W.d_fl.as<float>() + x.out_off, cnt * 4, hipMemcpyDeviceToHost, s2));
        HIPCHK(c, hipMemcpyAsync(dst + cnt * 4, W.d_ids.as<int32_t>() + x.out_off, cnt * 4, hipMemcpyDeviceToHost, s2));
        HIPCHK(c, hipMemcpyAsync(dst + cnt * 8, W.d_slots.as<int32_t>() + x.out_off, cnt * 4, hipMemcpyDeviceToHost,
                                 s2));
    }
    HIPCHK(c, hipEventRecord(W.done, s2));
    hl.lap(kHpStage2);  // launches issued
    W.active = true;
    W.o_cnt = o_cnt;
    W.o_keys = o_keys;
    W.o_fail = o_fail;
    W.ktop = ktop;
    W.dj.swap(dj);
    W.jmap.swap(jmap);
    W.tpos.swap(tpos);
    W.full.swap(full);
    W.full_off.swap(full_off);
    return PF_OK;
}

int finish_chunk(pf_ctx* c, std::vector<Job>& jobs, JobsState::Ws& W, std::vector<std::vector<int32_t>>* raw_out) {
    if (!W.active) return PF_OK;
    W.active = false;
    auto& J = c->jb;
    HpLap hl;
    HIPCHK(c, hipEventSynchronize(W.done));
    hl.lap(kHpGpu);
    const uint8_t* ho = W.h_out.as<uint8_t>();
    const std::vector<DevJob>& dj = W.dj;
    const std::vector<int32_t>& jmap = W.jmap;
    const std::vector<int32_t>& tpos = W.tpos;
    const std::vector<size_t>& full = W.full;
    const std::vector<size_t>& full_off = W.full_off;
    const size_t o_cnt = W.o_cnt, o_keys = W.o_keys, o_fail = W.o_fail;
    const int ktop = W.ktop;
    if (*reinterpret_cast<const int32_t*>(ho + o_fail))
        return c->fail(PF_EINTERNAL, "device query table build did not converge");
    const int32_t* cnt = reinterpret_cast<const int32_t*>(ho + o_cnt);
    if (J.stats_on || J.stats_count) {
        J.st_jobs += (int64_t)dj.size();
        for (size_t x = 0; x < dj.size(); ++x)
            if (dj[x].kind == kDjInterest || dj[x].kind == kDjCollab || dj[x].kind == kDjAll) J.st_cands += cnt[x];
    }
    const uint64_t* keys = reinterpret_cast<const uint64_t*>(ho + o_keys);
    for (size_t x = 0; x < dj.size(); ++x) {
        Job& jb = jobs[jmap[x]];
        jb.out.clear();
        if (tpos[x] >= 0) {
            const uint64_t* kx = keys + (size_t)x * ktop;
            for (int q = 0; q < jb.topk && q < ktop; ++q) {
                if (kx[q] == ~0ull) break;
                jb.out.emplace_back(key_uid(kx[q]), key_score(kx[q]));
            }
        }
    }
    for (size_t q = 0; q < full.size(); ++q) {
        const size_t x = full[q];
        const DevJob& dx = dj[x];
        const size_t cntx = (size_t)std::max(dx.cap, dx.kind == kDjClubs ? J.js.n_club_ids : 0);
        const uint8_t* src = ho + full_off[q];
        const float* sc = reinterpret_cast<const float*>(src);
        const int32_t* id = reinterpret_cast<const int32_t*>(src + cntx * 4);
        const int32_t* sl = reinterpret_cast<const int32_t*>(src + cntx * 8);
        if (dx.kind == kDjRawGraph || dx.kind == kDjRawCollab) {
            auto& v = (*raw_out)[jmap[x]];
            v.assign(id, id + cnt[x]);
            continue;
        }
        Job& jb = jobs[jmap[x]];
        Ranked r;
        if (dx.kind == kDjClubs) {
            for (int32_t k = 0; k < cnt[x]; ++k) r.emplace_back(id[k], sc[k]);
        } else {
            for (size_t k = 0; k < cntx; ++k)
                if (sl[k] >= 0) r.emplace_back(id[k], sc[k]);
        }
        rank(r, jb.topk);
        jb.out = std::move(r);
    }
    hl.lap(kHpUnpack);
    return PF_OK;
}

// Unpack the oldest pending asynchronous call into its caller's buffers (pf_wait).
int finish_pending(pf_ctx* c) {
    auto& J = c->jb;
    JobsState::Pending& p = J.pending.front();
    int rc = finish_chunk(c, p.jobs, J.ws[p.slot], nullptr);
    if (rc == PF_OK)
        for (size_t i = 0; i < p.jobs.size(); ++i) {
            const auto& r = p.jobs[i].out;
            const int n = std::min<int>((int)r.size(), p.topk);
            for (int k = 0; k < n; ++k) {
                p.ou[(int64_t)i * p.topk + k] = r[k].first;
                p.os[(int64_t)i * p.topk + k] = r[k].second;
            }
            p.oc[i] = n;
        }
    J.pending.pop_front();
    if (rc != PF_OK) {
        (void)hipStreamSynchronize(c->stream);
        if (J.aux2) (void)hipStreamSynchronize(J.aux2);
        if (J.aux) (void)hipStreamSynchronize(J.aux);
    }
    return rc;
}

}  // namespace

// Every pending asynchronous call unpacked (before any other use of the job pipeline's state).
// The pending asynchronous recommender calls, unpacked (the carried driver call stays in flight).
int drain_calls(pf_ctx* c) {
    int rc = PF_OK;
    while (!c->jb.pending.empty()) {
        const int r = finish_pending(c);
        if (rc == PF_OK) rc = r;
    }
    return rc;
}

// a carried call's status, kept per ticket (a bounded table: tickets nobody waits for age out)
static void note_carry_rc(JobsState& J, uint64_t ticket, int rc) {
    if (rc == PF_OK) return;
    if (J.carry_fail.size() >= 64) J.carry_fail.clear();
    J.carry_fail[ticket] = rc;
}

// The carried driver call: wait for its last chunk, unpack it, hand the jobs to its driver.
int finish_carry(pf_ctx* c) {
    auto& J = c->jb;
    if (!J.carry.on) return PF_OK;
    JobsState::Carry cr = std::move(J.carry);
    J.carry = JobsState::Carry{};
    int rc = finish_chunk(c, cr.jobs, J.ws[cr.slot], nullptr);
    if (rc == PF_OK && cr.done) cr.done(cr.jobs);
    J.carry_done = cr.ticket;
    note_carry_rc(J, cr.ticket, rc);
    return rc;
}

int jobs_drain(pf_ctx* c) {
    int rc = drain_calls(c);
    const int r = finish_carry(c);
    return rc != PF_OK ? rc : r;
}

namespace {

// leave != nullptr: the call's last chunk stays on the device as the context's carried call (the
// jobs move into it; leave->done gets them once finished).  A carried call of an earlier driver
// call is finished right after this call's first chunk is launched.
int run_all(pf_ctx* c, std::vector<Job>& jobs, bool raw, std::vector<std::vector<int32_t>>* raw_out,
            JobsState::Carry* leave = nullptr) {
    auto& J = c->jb;
    if (!J.ok) return c->fail(PF_EUNSUPP, "device job pipeline unavailable: " + J.why);
    (void)hipSetDevice(c->device);
    int rc0 = drain_calls(c);  // asynchronous calls in flight finish first (they hold the workspaces)
    if (rc0 != PF_OK) return rc0;

    for (Job& jb : jobs) jb.out.clear();
    if (jobs.empty()) return PF_OK;
    int rc = sync_nodes(c);
    if (rc != PF_OK) return rc;
    const std::unordered_map<int32_t, std::pair<int32_t, std::vector<int32_t>>>* over = nullptr;
    for (const Job& jb : jobs) {
        if (jb.view.over && over && jb.view.over != over)
            return c->fail(PF_EINTERNAL, "one call mixes two versioned adjacency edit sets");
        if (jb.view.over) over = jb.view.over;
    }
    rc = sync_view(c, over);
    if (rc != PF_OK) return rc;
    HpLap hl;
    const size_t n = jobs.size();
    std::vector<JP> P(n);
    // Chunks of at most chunk_jobs jobs (and the element budgets), double-buffered: chunk i + 1
    // is planned and launched while chunk i runs on the device, then chunk i is unpacked.
    // Only large calls are cut: splitting a 64-user cfg-3 step into four chunks made it slower
    // (1.09 -> 1.50 ms: four times the launches, each too small to fill the GPU; r2n).
    // Chunk sizes by weight (PF_DEBUG chunk_plan=w1:w2:..., A/B): the first chunk's planning and
    // the last chunk's unpacking are the host work no device stage hides
    static const std::vector<int> weights = [] {
        std::vector<int> w;
        const char* v = debug_str("chunk_plan");
        std::string str = v ? v : "1:1:1";
        for (size_t p = 0; p < str.size();) {
            size_t q = str.find(':', p);
            if (q == std::string::npos) q = str.size();
            w.push_back(std::max(1, std::atoi(str.substr(p, q - p).c_str())));
            p = q + 1;
        }
        return w;
    }();
    int wsum = 0;
    for (int w : weights) wsum += w;
    size_t ck = 0;  // chunks cut so far
    auto chunk_end = [&](size_t b) {
        if (n < kPipeJobs) return n;
        const size_t w = (size_t)weights[std::min(ck, weights.size() - 1)];
        const size_t len = std::max<size_t>(kPipeJobs / 4, (n * w + wsum - 1) / wsum);
        return std::min(n, b + len);
    };
    int slot = J.carry.on ? (J.carry.slot ^ 1) : 0;  // the carried call holds the other workspace
    JobsState::Ws* pending = nullptr;
    auto drain = [&](int code) {  // an error with a chunk in flight: let it finish first
        (void)hipStreamSynchronize(c->stream);
        if (J.aux2) (void)hipStreamSynchronize(J.aux2);
        if (J.aux) (void)hipStreamSynchronize(J.aux);
        for (auto& w : J.ws) w.active = false;
        if (J.carry.on) {  // its results are dropped; pf_eval_wait reports the error
            J.carry_done = J.carry.ticket;
            note_carry_rc(J, J.carry.ticket, code);
            J.carry = JobsState::Carry{};
        }
        return code;
    };
    size_t b = 0;
    while (b < n) {
        const size_t lim = chunk_end(b);
        ++ck;
        // 1-hop planning is a few microseconds per job: threads only for large chunks (spawning
        // them costs more than planning a 64-user step).  Per chunk: planning every job of a call
        // up front measured no faster (cfg 5 113.4k vs 110.4k users/s, r4n)
        par_jobs(lim - b, [&](size_t i) { if (P[b + i].u < 0 && P[b + i].kind < 0) plan_job(c, jobs[b + i], P[b + i], raw); },
                 256);
        hl.lap(kHpPrep);
        for (size_t i = b; i < lim; ++i)
            if (P[i].unmapped) return drain(c->fail(PF_EINTERNAL, "adjacency row names an unmapped uid"));
        size_t e = b;
        int64_t el = 0, ht = 0;
        while (e < lim) {
            const JP& p = P[e];
            if (e > b && (el + p.elems > kChunkElems || ht + p.ht_words > kChunkHt)) break;
            el += p.elems;
            ht += p.ht_words;
            ++e;
        }
        hl.skip();
        JobsState::Ws& W = J.ws[slot];
        rc = launch_chunk(c, jobs, P, b, e, W);
        if (rc != PF_OK) return drain(rc);
        if (J.carry.on) {  // the device runs this chunk behind the carried call's last one
            rc = finish_carry(c);
            if (rc != PF_OK) return drain(rc);
        }
        if (pending) {
            rc = finish_chunk(c, jobs, *pending, raw_out);
            if (rc != PF_OK) return drain(rc);
        }
        pending = &W;
        slot ^= 1;
        b = e;
        hl.skip();
    }
    if (pending && leave && !raw && pending->active) {  // the last chunk stays on the device
        leave->on = true;
        leave->slot = (int)(pending - J.ws);
        leave->jobs = std::move(jobs);
        J.carry = std::move(*leave);
        return PF_OK;
    }
    if (pending) {
        rc = finish_chunk(c, jobs, *pending, raw_out);
        if (rc != PF_OK) return drain(rc);
    }
    if (leave && leave->done) leave->done(jobs);  // nothing left on the device: finished now
    if (leave) J.carry_done = leave->ticket;
    return PF_OK;
}

}  // namespace

int run_jobs(pf_ctx* c, std::vector<Job>& jobs) { return run_all(c, jobs, false, nullptr); }

int run_jobs_carry(pf_ctx* c, std::vector<Job>&& jobs, uint64_t ticket, std::function<void(std::vector<Job>&)> done) {
    JobsState::Carry cr;
    cr.ticket = ticket;
    cr.done = std::move(done);
    std::vector<Job> js = std::move(jobs);
    return run_all(c, js, false, nullptr, &cr);
}

uint64_t next_call_ticket(pf_ctx* c) { return c->jb.next_ticket++; }

int carry_wait(pf_ctx* c, uint64_t ticket) {
    auto& J = c->jb;
    if (J.carry.on && J.carry.ticket <= ticket) (void)finish_carry(c);  // its status lands in carry_fail
    // only this ticket's own status: an earlier call's failure is not reported for a later one
    const auto it = J.carry_fail.find(ticket);
    if (it == J.carry_fail.end()) return PF_OK;
    const int r = it->second;
    J.carry_fail.erase(it);
    return r;
}

// An asynchronous call: planned and launched now into a free workspace slot (the oldest pending
// call is unpacked first when both are taken), unpacked into the caller's buffers by pf_wait.
// Its device stages queue behind the previous call's on the context's stream, so the host plans
// call i + 1 while the device runs call i.  A call that needs more than one chunk runs as
// run_jobs does (its outputs are written before this returns).
int run_jobs_async(pf_ctx* c, std::vector<Job>&& jobs, int32_t topk, int32_t* ou, float* os, int32_t* oc,
                   uint64_t* ticket) {
    auto& J = c->jb;
    *ticket = J.next_ticket++;
    if (!J.ok) return c->fail(PF_EUNSUPP, "device job pipeline unavailable: " + J.why);
    (void)hipSetDevice(c->device);
    for (size_t i = 0; i < jobs.size(); ++i) oc[i] = 0;
    if (jobs.empty() || topk == 0) return PF_OK;
    // the carried driver call (pf_eval_recommendation_tests_async) holds a workspace slot too: with
    // every slot taken the oldest pending call is unpacked, or the carried call finished
    while (J.pending.size() + (J.carry.on ? 1 : 0) >= (size_t)kJobSlots) {
        const int r = J.pending.empty() ? finish_carry(c) : finish_pending(c);
        if (r != PF_OK) return r;
    }
    int rc = sync_nodes(c);
    if (rc == PF_OK) rc = sync_view(c, nullptr);
    if (rc != PF_OK) return rc;
    const size_t n = jobs.size();
    std::vector<JP> P(n);
    // an asynchronous call's jobs (cfg 3: 64 collaborative jobs at limit 10000) on the worker pool
    // from 16 jobs up: the caller takes jobs while the workers wake, so small calls lose nothing
    par_jobs(n, [&](size_t i) { plan_job(c, jobs[i], P[i], false); }, 16);
    int64_t el = 0, ht = 0;
    for (const JP& p : P) {
        if (p.unmapped) return c->fail(PF_EINTERNAL, "adjacency row names an unmapped uid");
        el += p.elems;
        ht += p.ht_words;
    }
    if (n >= kPipeJobs || (n > 1 && (el > kChunkElems || ht > kChunkHt))) {  // several chunks: synchronous
        rc = jobs_drain(c);
        if (rc == PF_OK) rc = run_all(c, jobs, false, nullptr);
        if (rc != PF_OK) return rc;
        for (size_t i = 0; i < n; ++i) {
            const int m = std::min<int>((int)jobs[i].out.size(), topk);
            for (int k = 0; k < m; ++k) {
                ou[(int64_t)i * topk + k] = jobs[i].out[k].first;
                os[(int64_t)i * topk + k] = jobs[i].out[k].second;
            }
            oc[i] = m;
        }
        return PF_OK;
    }
    int slot = 0;  // a slot neither a pending call nor the carried call holds
    for (bool used = true; used; ++slot) {
        used = J.carry.on && J.carry.slot == slot;
        for (const auto& q : J.pending) used |= q.slot == slot;
        if (!used) break;
    }
    JobsState::Pending pd;
    pd.ticket = *ticket;
    pd.slot = slot;
    pd.jobs = std::move(jobs);
    pd.topk = topk;
    pd.ou = ou;
    pd.os = os;
    pd.oc = oc;
    rc = launch_chunk(c, pd.jobs, P, 0, n, J.ws[slot]);
    if (rc != PF_OK) {
        (void)hipStreamSynchronize(c->stream);
        if (J.aux2) (void)hipStreamSynchronize(J.aux2);
        if (J.aux) (void)hipStreamSynchronize(J.aux);
        J.ws[slot].active = false;
        return rc;
    }
    if (!J.ws[slot].active) return PF_OK;  // nothing reached the device (every user unknown)
    J.pending.push_back(std::move(pd));
    return PF_OK;
}

int jobs_wait(pf_ctx* c, uint64_t ticket) {
    auto& J = c->jb;
    int rc = PF_OK;
    while (!J.pending.empty() && J.pending.front().ticket <= ticket) {
        const int r = finish_pending(c);
        if (rc == PF_OK) rc = r;
    }
    const int r = carry_wait(c, ticket);
    return rc != PF_OK ? rc : r;
}

int jobs_stats_reset(pf_ctx* c, int enable) {
    auto& J = c->jb;
    (void)hipSetDevice(c->device);
    const int rc = jobs_drain(c);
    if (rc != PF_OK) return rc;
    HIPCHK(c, J.d_stats.ensure(64));
    HIPCHK(c, hipMemsetAsync(J.d_stats.p, 0, 64, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    J.stats_on = (enable & 1) != 0;
    J.stats_count = (enable & 2) != 0;
    J.stat_used = 0;
    J.st_jobs = J.st_cands = J.st_img_bytes = J.st_launches = 0;
    return PF_OK;
}

int jobs_stats_read(pf_ctx* c, pf_jobs_stats* o) {
    auto& J = c->jb;
    (void)hipSetDevice(c->device);
    const int rc = jobs_drain(c);
    if (rc != PF_OK) return rc;
    std::memset(o, 0, sizeof *o);
    unsigned long long v[3] = {0, 0, 0};
    if (J.d_stats.p) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (J.aux) HIPCHK(c, hipStreamSynchronize(J.aux));  // the counting kernels of ping-pong chunks
        HIPCHK(c, hipMemcpy(v, J.d_stats.p, sizeof v, hipMemcpyDeviceToHost));
    }
    double ms = 0.0;
    for (size_t i = 0; i < J.stat_used; ++i) {
        float t = 0.f;
        HIPCHK(c, hipEventSynchronize(J.stat_ev[i].second));
        HIPCHK(c, hipEventElapsedTime(&t, J.stat_ev[i].first, J.stat_ev[i].second));
        ms += t;
    }
    o->jobs = J.st_jobs;
    o->candidates = J.st_cands;
    o->pairs = (int64_t)v[0];
    o->pair_alg_bytes = (int64_t)v[1];
    o->pair_record_bytes = (int64_t)v[2];
    o->pair_image_bytes = J.st_img_bytes;
    o->pair_ms = ms;
    o->pair_launches = J.st_launches;
    o->pair_dispatches = J.n_dispatch;
    return PF_OK;
}

int fof_device(pf_ctx* c, int32_t uid, int32_t limit, int32_t flavour, std::vector<int32_t>& out) {
    std::vector<Job> jobs(1);
    jobs[0].uid = uid;
    jobs[0].limit = limit;
    jobs[0].limit_flavour = flavour;
    jobs[0].topk = INT32_MAX;
    jobs[0].view.base = &c->hc.adj;
    std::vector<std::vector<int32_t>> raw(1);
    const int rc = run_all(c, jobs, true, &raw);
    out = std::move(raw[0]);
    return rc;
}

}  // namespace pf
