// pf_api.cpp — the C ABI (include/pokec_fas.h): context lifetime, device upload,
// query-image packing, and the host orchestration of the reference's recommenders
// (recommender_graph.cpp:10-237, recommender_clubs.cpp:10-73) around the gfx950
// kernels.  The FAS arithmetic itself runs only on the GPU; there is no CPU path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "pf_batch.h"
#include "pf_ctx.h"
#include "pf_debug.h"
#include "pf_kernels.h"
#include "pf_store.h"
#include "pokec_fas.h"

using pf::DBuf;
using pf::PinBuf;
using pf::Ranked;
using pf::par_jobs;
using pf::rank;

namespace {

thread_local std::string g_open_error;

constexpr uint32_t kLdsLimit = 64 * 1024;  // query images above this probe from global memory
constexpr uint32_t kK5LdsCap = 160u * 1024u;  // one K5 workgroup's LDS (gfx950: 160 KB per CU)
constexpr size_t kProfCap = 1u << 16;      // profiling event pairs kept (pf_profile_*)

}  // namespace

namespace pf {
void set_open_error(const std::string& m) { g_open_error = m; }
}  // namespace pf

namespace {

// Query images -> one byte pool + refs.
struct Images {
    std::vector<uint8_t> pool;
    std::vector<pf::QImageRef> refs;
    uint32_t max_lds = 0;  // dynamic LDS a 256-thread block needs for the largest image
    bool gtab = false;     // some image probes its table in global memory
};

constexpr uint32_t kStageLimit = 48 * 1024;   // keys+vals above this are probed in global memory

// PF_DEBUG stage_limit (bytes) lowers the LDS staging limit; tests use it to force the
// global-memory table variant on small corpora.
uint32_t stage_limit() {
    static const uint32_t lim = (uint32_t)pf::debug_long("stage_limit", kStageLimit);
    return lim;
}
constexpr uint32_t kBlockThreads = 256;

void add_image(Images& im, const pf::QImageHost& q) {
    auto align = [&](size_t a) { while (im.pool.size() % a) im.pool.push_back(0); };
    align(16);
    pf::QImageRef r{};
    const size_t start = im.pool.size();
    r.const_off = (uint32_t)(start / 16);
    const uint8_t* cp = reinterpret_cast<const uint8_t*>(&q.c);
    im.pool.insert(im.pool.end(), cp, cp + sizeof(pf::QConst));
    r.keys_off = (uint32_t)(im.pool.size() - start);
    const uint8_t* kp = reinterpret_cast<const uint8_t*>(q.keys.data());
    im.pool.insert(im.pool.end(), kp, kp + q.keys.size() * 8);
    align(16);
    r.vals_off = (uint32_t)(im.pool.size() - start);
    const uint8_t* vp = reinterpret_cast<const uint8_t*>(q.vals.data());
    im.pool.insert(im.pool.end(), vp, vp + q.vals.size() * sizeof(pf::QVal));
    const size_t kv = q.keys.size() * 8 + q.vals.size() * sizeof(pf::QVal);
    r.lds_bytes = kv <= stage_limit() ? (uint32_t)kv : 0u;
    im.gtab = im.gtab || r.lds_bytes == 0;
    // QConst | staged tables | hit lists | hit counts | merge scratch (stage_query's carve)
    const uint32_t need = (uint32_t)sizeof(pf::QConst) + r.lds_bytes + q.c.n_hits_max * kBlockThreads +
                          4u * kBlockThreads + 2048u;
    im.max_lds = std::max(im.max_lds, need);
    im.refs.push_back(r);
}
constexpr uint32_t kPairThreads = (uint32_t)pf::kPairThreads;

// Many images at once: refs and offsets first (returns the pool bytes), then fill_images
// copies them on threads into `dst` (pinned; a few thousand images per chunk).
size_t plan_images(Images& im, const std::vector<pf::QImageHost>& qs) {
    auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    size_t o = 0;
    for (const auto& q : qs) {
        pf::QImageRef r{};
        r.const_off = (uint32_t)(o / 16);
        r.keys_off = (uint32_t)sizeof(pf::QConst);
        r.vals_off = (uint32_t)a16(r.keys_off + q.keys.size() * 8);
        o = a16(o + r.vals_off + q.vals.size() * sizeof(pf::QVal));
        const size_t kv = q.keys.size() * 8 + q.vals.size() * sizeof(pf::QVal);
        r.lds_bytes = kv <= stage_limit() ? (uint32_t)kv : 0u;
        im.gtab = im.gtab || r.lds_bytes == 0;
        const uint32_t need = (uint32_t)sizeof(pf::QConst) + r.lds_bytes + q.c.n_hits_max * kPairThreads +
                              4u * kPairThreads + 2048u;
        im.max_lds = std::max(im.max_lds, need);
        im.refs.push_back(r);
    }
    return o;
}

void fill_images(const Images& im, const std::vector<pf::QImageHost>& qs, uint8_t* dst, size_t total) {
    par_jobs(qs.size(), [&](size_t i) {
        const pf::QImageHost& q = qs[i];
        const pf::QImageRef& r = im.refs[i];
        const size_t b = (size_t)r.const_off * 16;  // byte offsets from the pool start
        const size_t ko = b + r.keys_off, vo = b + r.vals_off;
        const size_t kend = ko + q.keys.size() * 8, vend = vo + q.vals.size() * sizeof(pf::QVal);
        const size_t next = i + 1 < qs.size() ? (size_t)im.refs[i + 1].const_off * 16 : total;
        std::memcpy(dst + b, &q.c, sizeof(pf::QConst));
        if (!q.keys.empty()) std::memcpy(dst + ko, q.keys.data(), q.keys.size() * 8);
        std::memset(dst + kend, 0, vo - kend);
        if (!q.vals.empty()) std::memcpy(dst + vo, q.vals.data(), q.vals.size() * sizeof(pf::QVal));
        std::memset(dst + vend, 0, next - vend);
    }, 64);
}

pf::AdjView plain_view(const pf_ctx* c) {
    pf::AdjView v;
    v.base = &c->hc.adj;
    return v;
}

// FAS(A = qidx[g], B = slots[g][j]) for every group g, on the GPU.
// Groups go to the GPU in chunks (<= 4096 distinct queries, <= 8M pairs per launch); each
// distinct query's image is built once per chunk, on host threads.
// keep (optional): every chunk's scores stay on the device in one buffer, group g at
// (*goff)[g] (the collaborative sums read their matrix rows there)
int run_pairs(pf_ctx* c, const std::vector<int32_t>& qidx, const std::vector<std::vector<int32_t>>& slots,
              std::vector<std::vector<float>>& out, DBuf* keep = nullptr, std::vector<int64_t>* goff = nullptr) {
    out.assign(qidx.size(), {});
    if (keep) {
        size_t tot = 0;
        goff->assign(qidx.size(), 0);
        for (size_t g = 0; g < qidx.size(); ++g) {
            (*goff)[g] = (int64_t)tot;
            tot += slots[g].size();
        }
        HIPCHK(c, keep->ensure(std::max<size_t>(tot, 1) * sizeof(float)));
    }
    for (size_t g = 0; g < qidx.size(); ++g) out[g].assign(slots[g].size(), 0.f);
    size_t g0 = 0;
    while (g0 < qidx.size()) {
        // chunk [g0, g1)
        std::unordered_map<int32_t, int32_t> img_of;
        std::vector<int32_t> uq;
        size_t g1 = g0, pairs = 0;
        for (; g1 < qidx.size(); ++g1) {
            if (slots[g1].empty()) continue;
            const bool fresh = !img_of.count(qidx[g1]);
            if (g1 > g0 && ((fresh && uq.size() >= 4096) || pairs + slots[g1].size() > (8u << 20))) break;
            if (fresh) {
                img_of.emplace(qidx[g1], (int32_t)uq.size());
                uq.push_back(qidx[g1]);
            }
            pairs += slots[g1].size();
        }
        if (pairs == 0) { g0 = g1; continue; }
        std::vector<pf::QImageHost> qi(uq.size());
        std::vector<uint8_t> ok(uq.size(), 1);
        pf::HpLap hl;
        {
            const int th = (int)std::min<size_t>(16, std::max<size_t>(1, uq.size() / 16));
            std::vector<std::thread> ts;
            for (int w = 0; w < th; ++w)
                ts.emplace_back([&, w]() {
                    for (size_t i = (size_t)w; i < uq.size(); i += (size_t)th)
                        ok[i] = pf::build_query(c->hc, c->hs.packed, uq[i], nullptr, qi[i]) ? 1 : 0;
                });
            for (auto& t : ts) t.join();
        }
        for (uint8_t x : ok)
            if (!x) return c->fail(PF_EUNSUPP, "query hash table too large");
        hl.lap(pf::kHpImages);
        Images im;
        std::vector<pf::PairBlock> blocks;
        const size_t pool_bytes = plan_images(im, qi);
        // per group: first block and first pair (serial, O(groups)); then the copies on threads
        std::vector<size_t> gb(g1 - g0 + 1), gf(g1 - g0 + 1);
        for (size_t g = g0; g < g1; ++g) {
            gb[g - g0 + 1] = gb[g - g0] + (slots[g].size() + kPairThreads - 1) / kPairThreads;
            gf[g - g0 + 1] = gf[g - g0] + slots[g].size();
        }
        const size_t npairs = gf.back();
        HIPCHK(c, c->h_pool.ensure(pool_bytes));
        HIPCHK(c, c->h_slots.ensure(npairs * sizeof(int32_t)));
        HIPCHK(c, c->h_scores.ensure(npairs * sizeof(float)));
        fill_images(im, qi, c->h_pool.as<uint8_t>(), pool_bytes);
        blocks.resize(gb.back());
        int32_t* flat = c->h_slots.as<int32_t>();
        par_jobs(g1 - g0, [&](size_t i) {
            const size_t g = g0 + i;
            if (slots[g].empty()) return;
            const int32_t img = img_of.at(qidx[g]);
            std::memcpy(flat + gf[i], slots[g].data(), slots[g].size() * sizeof(int32_t));
            for (size_t b = 0, x = gb[i]; b < slots[g].size(); b += kPairThreads, ++x)
                blocks[x] = pf::PairBlock{img, (int32_t)(gf[i] + b), (int32_t)std::min<size_t>(kPairThreads, slots[g].size() - b),
                                           (int32_t)(gf[i] + b)};
        }, 256);
        hl.lap(pf::kHpPack);
        // pinned buffers: async copies; they are reused only after this chunk's synchronize
        HIPCHK(c, c->d_pool.ensure(std::max<size_t>(pool_bytes, 16)));
        HIPCHK(c, hipMemcpyAsync(c->d_pool.p, c->h_pool.p, pool_bytes, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, upload(c, c->d_refs, im.refs));
        HIPCHK(c, upload(c, c->d_blocks, blocks));
        HIPCHK(c, c->d_slots.ensure(npairs * sizeof(int32_t)));
        HIPCHK(c, hipMemcpyAsync(c->d_slots.p, flat, npairs * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        float* dsc = nullptr;
        if (keep) {
            dsc = keep->as<float>() + (*goff)[g0];  // groups are laid out in order, chunk after chunk
        } else {
            HIPCHK(c, c->d_scores.ensure(npairs * sizeof(float)));
            dsc = c->d_scores.as<float>();
        }
        HIPCHK(c, pf::launch_pairs(c->ds, c->d_pool.as<uint8_t>(), c->d_refs.as<pf::QImageRef>(), im.max_lds, im.gtab,
                                   c->d_blocks.as<pf::PairBlock>(), (int)blocks.size(), nullptr, c->d_slots.as<int32_t>(), dsc,
                                   c->stream));
        c->jb.n_dispatch += !blocks.empty();  // pf_jobs_stats.pair_dispatches counts every K1' dispatch
        const float* res = c->h_scores.as<float>();
        HIPCHK(c, hipMemcpyAsync(c->h_scores.p, dsc, npairs * sizeof(float), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        hl.lap(pf::kHpGpu);
        par_jobs(g1 - g0, [&](size_t i) {
            const size_t g = g0 + i;
            if (!slots[g].empty()) std::memcpy(out[g].data(), res + gf[i], slots[g].size() * sizeof(float));
        }, 256);
        hl.lap(pf::kHpUnpack);
        g0 = g1;
    }
    return PF_OK;
}

void emit(const Ranked& r, int i, int topk, int32_t* ou, float* os, int32_t* oc) {
    int n = std::min<int>((int)r.size(), topk);
    for (int k = 0; k < n; ++k) {
        ou[(int64_t)i * topk + k] = r[k].first;
        os[(int64_t)i * topk + k] = r[k].second;
    }
    oc[i] = n;
}

// K5 mode word: bit 0 dynamic block hand-out (each workgroup's first block, then the next
// unclaimed one), for one-query launches only.  r2fb A/B: 205.3 / 205.6 us vs 206.9 / 206.9 us
// static per cfg-2 launch; batches (one block per workgroup in L2-sharing order) stay static
// (cfg 4 9.83e9 dynamic vs 9.88e9 static).
// K5 launch mode: bit 0 = dynamic block hand-out (one query); bit 1 = transposed grid (batches:
// the resident workgroups are many queries on the same candidate blocks; PF_DEBUG k5_transposed=1.
// Measured slower than the query-major grid: cfg 4 216.9 vs 203.4 ms per 1024-query launch, r4c)
uint32_t post_mode(int nq) {
    static const bool tr = pf::debug_long("k5_transposed", 0) != 0;
    static const bool st = pf::debug_long("k5_static", 0) != 0;  // A/B: static hand-out for one query
    // each XCD's workgroups take a contiguous range of every static round's blocks (neighbouring
    // blocks share the cache lines at their list segments' ends); the query-major batch grid too
    // (a query's workgroups are a multiple of 8 there, so bx mod 8 is still the XCD); k5_xcd=0 A/B
    static const bool xcd = pf::debug_long("k5_xcd", 1) != 0;
    // every block claimed per XCD group (default; k5_dyn=0 A/B: static rounds, the tail claimed).
    // Neutral on an isolated launch (178.8 vs 179.2 us, r6-era), but with the scan lanes the next
    // query's workgroups start while this one's last blocks run, so a static share of blocks
    // waits on workgroups dispatched late: cfg 2 1.13e10 -> 1.20e10 candidates/s (r8b / r8c)
    static const bool dyn = pf::debug_long("k5_dyn", 1) != 0;
    const uint32_t x = xcd ? 4u : 0u;
    return nq == 1 ? ((st ? 0u : 1u) | x | (dyn ? 8u : 0u)) : (tr ? 2u : x);
}

// Candidates per claimed block past a one-query K5 launch's static rounds (PF_DEBUG k5_tail=N,
// A/B; 0 or >= the block size: whole blocks).  r6g, one box: whole blocks 177.0 us, 256 177.2,
// 128 177.5 / 178.6, 64 180.2: the claimed tail is not where a launch loses time

uint32_t tail_block_cands() {
    static const long n = pf::debug_long("k5_tail", 0);
    return (uint32_t)std::max(0L, n);
}

// Blocks per workgroup of a batched postings scan: a workgroup stages its query's tables once
// for them (blocks w, w + n/4, ... of one query, so the query's neighbouring blocks still run
// side by side and share its lists in L2).  cfg 4, r2bs: 1 -> 9.36e9, 2 -> 9.62e9, 4 -> 9.87e9
// candidates/s.  Round 4 (static block rounds with a claimed tail, the rounds table built once
// per block): r4t/r4v, one box: 2 -> 1.07e10, 4 -> 1.11e10, 8 -> 1.14e10, 16 -> 1.162e10,
// 32 -> 1.162e10, 64 -> 1.14e10, 128 -> 1.09e10.  Round 5 final tree (r8q, one box, alternating):
// 8 -> 1.411e10, 16 -> 1.424-1.428e10, 24 -> 1.435e10, 32 -> 1.432-1.438e10.
constexpr int kBatchBlocksPerWgDefault = 32;
// PF_DEBUG k5_batch_blocks=N (A/B)
int batch_blocks_per_wg() {
    static const int n = (int)std::max(1L, pf::debug_long("k5_batch_blocks", kBatchBlocksPerWgDefault));
    return n;
}

// dynamic LDS of one image's postings scan (K5)
uint32_t post_image_lds(const pf::QPostHead* h) {
    return pf::post_lds(pf::post_var_lds(h->n_tok, h->n_tok + h->n_club + h->n_friend));
}
int post_image_per_cu(const pf::QPostHead* h) {
    return pf::post_blocks_per_cu(pf::post_var_lds(h->n_tok, h->n_tok + h->n_club + h->n_friend));
}

int scan_lanes();

// Workgroups of a one-query postings scan: one resident round, or seven eighths of one on the
// scan lanes, where consecutive queries' launches share the CUs and a launch of fewer workgroups
// lets the next one start sooner.  Over 200-step lines three quarters read best (cfg 2 1.209 /
// 1.205 / 1.200e10 at 1,024 -> 1.216 / 1.229 / 1.214e10 at 768 with three lanes, r9j; 896: 1.224 /
// 1.202e10), but in the driver's 20-step line, where the first and last launches of the timed
// region run with no neighbour, 768 lost 1.5 % (r9zf) and 896 is the best of 1,024 / 896 / two
// lanes of 1,024 (1.199 vs 1.190 / 1.196e10, six runs each, r9zg).  PF_DEBUG k5_wgs=N overrides it.
// More lanes (more hardware queues, scan_lanes) take smaller launches still: 15 lanes of 192 (3/16 of
// a round) 1.273 / 1.277e10, of 256 1.238-1.267e10, of 320 1.256 / 1.265e10; 7 lanes of 512 or 384
// 1.235-1.251e10 (r9x-r9z, tools/hwq_probe.sh).
int one_query_wgs(int resident, bool lanes) {
    static const long n = pf::debug_long("k5_wgs", 0);
    if (n > 0) return (int)n;
    if (!lanes) return resident;
    const int nl = scan_lanes();
    const int w = nl >= 12 ? resident * 3 / 16 : (nl >= 6 ? resident / 2 : (nl >= 3 ? resident * 7 / 8 : resident));
    return std::max(8, w & ~7);
}

// Timing events of one scan launch (the profiling pool when pf_profile_reset is on).  A
// launch the caller passes timed = false, or that sampling skips, records nothing and clears
// last_ev0/last_ev1, so pf_last_scan_ms never reports another launch's time.
int scan_events(pf_ctx* c, bool& timed, hipEvent_t& e0, hipEvent_t& e1) {
    e0 = c->ev0;
    e1 = c->ev1;
    if (!timed) {
        c->last_ev0 = c->last_ev1 = nullptr;
        return PF_OK;
    }
    if (c->prof_on) {
        // a timed launch costs ~9 us of stream time (two timestamped events, measured at
        // 231 vs 222 us per single-query step): sampled launches only when asked
        if (c->prof_seen++ % c->prof_every != 0) {
            timed = false;
            c->last_ev0 = c->last_ev1 = nullptr;
            return PF_OK;
        }
        if (c->prof_used == c->prof_ev.size()) {
            if (c->prof_ev.size() >= kProfCap) {  // pool full: the launch runs untimed
                timed = false;
                c->last_ev0 = c->last_ev1 = nullptr;
                return PF_OK;
            }
            hipEvent_t a, b;
            HIPCHK(c, pf::timing_event(&a));
            HIPCHK(c, pf::timing_event(&b));
            c->prof_ev.emplace_back(a, b);
        }
        e0 = c->prof_ev[c->prof_used].first;
        e1 = c->prof_ev[c->prof_used].second;
        ++c->prof_used;
    }
    return PF_OK;
}

// A single query on a caller's stream runs on the next scan lane (pf_ctx.h ScanLane).  lane_begin
// picks the lane and its next result row (the lane's stream waits for the copies of a ring group
// only when it wraps back to it); lane_end has the caller's stream wait for the launch's stop event
// and copy the row out, and records the group's freed event after its last row's copy.
struct LaneUse {
    pf_ctx::ScanLane* ln = nullptr;
    int row = 0;
    uint64_t* keys = nullptr;  // the lane's result row
};

int scan_lanes() {
    // three by default (the context's stream and both aux streams): 1.204 / 1.205 / 1.206e10 vs
    // 1.202 / 1.195 / 1.192e10 with two, alternating on one box (r9d, resident images).  More lanes run
    // on streams of their own and need a process with more hardware queues (GPU_MAX_HW_QUEUES): 15
    // lanes on 16 queues read +3-5 % over 200 steps but degrade as the backlog grows (1,000 steps
    // 1.17e10, 2,000 1.06-1.08e10, against 1.24e10 for three lanes on four queues at either length,
    // r9zd / r9ze; past 16 queues the process oversubscribes the hardware queue slots, r9za), so
    // they stay an A/B (PF_DEBUG scan_lanes=N, up to 16)
    static const int n = (int)std::min((long)pf_ctx::kMaxLanes, pf::debug_long("scan_lanes", 3));
    return n;
}

int lane_begin(pf_ctx* c, hipStream_t caller, LaneUse& u) {
    u = LaneUse{};
    const int nlanes = scan_lanes();
    if (nlanes < 2 || caller == c->stream) return PF_OK;
    const int li = c->lane_cur;
    pf_ctx::ScanLane* ln = &c->lane[li];
    c->lane_cur = (li + 1) % nlanes;
    if (!ln->done) {
        HIPCHK(c, hipEventCreate(&ln->done));  // a launch's stop event (bound to its dispatch)
        for (hipEvent_t& e : ln->freed) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // the lanes run on the context's stream and the job pipeline's aux streams (created at open):
    // streams of their own would share the process's four hardware queues with them
    // (PF_DEBUG lazy_aux=1: no aux streams yet, every lane on the context's stream)
    const hipStream_t ls[3] = {c->stream, c->jb.aux, c->jb.aux2};
    ln->st = li < 3 ? ls[li] : c->lane_st[li];
    if (!ln->st) ln->st = c->stream;
    const int r = ln->row;
    ln->row = (r + 1) % pf_ctx::kLaneRows;
    const int g = r / pf_ctx::kLaneGroupRows;
    if (r % pf_ctx::kLaneGroupRows == 0 && ln->used[g]) HIPCHK(c, hipStreamWaitEvent(ln->st, ln->freed[g], 0));
    HIPCHK(c, ln->keys.ensure((size_t)pf_ctx::kLaneRows * pf::kMaxTopK * sizeof(uint64_t)));  // once
    u.ln = ln;
    u.row = r;
    u.keys = ln->keys.as<uint64_t>() + (size_t)r * pf::kMaxTopK;
    return PF_OK;
}

int lane_end(pf_ctx* c, const LaneUse& u, hipEvent_t stop, hipStream_t caller, uint64_t* dst, int k) {
    HIPCHK(c, hipStreamWaitEvent(caller, stop, 0));
    HIPCHK(c, hipMemcpyAsync(dst, u.keys, (size_t)k * sizeof(uint64_t), hipMemcpyDeviceToDevice, caller));
    if (u.row % pf_ctx::kLaneGroupRows == pf_ctx::kLaneGroupRows - 1) {
        const int g = u.row / pf_ctx::kLaneGroupRows;
        HIPCHK(c, hipEventRecord(u.ln->freed[g], caller));
        u.ln->used[g] = true;
    }
    return PF_OK;
}

// K5: the postings scan of prebuilt images (pf_types.h QPostHead layout) into d_keys rows
// `rows`.  Staging: [image offsets | rows | sync | images], one async copy.
int scan_post(pf_ctx* c, const std::vector<const std::vector<uint8_t>*>& imgs, const std::vector<int32_t>& rows, int k,
              uint64_t* d_keys, hipStream_t s, bool timed) {
    const int nq = (int)imgs.size();
    if (nq == 0) return PF_OK;
    // LDS classes: a launch's workgroups all take the LDS of its largest query, so the batch goes
    // out in one launch per occupancy class (workgroups per CU), the queries of a class contiguous
    // in the staged arrays; one query with thousands of friends no longer runs every query of a
    // batch at one workgroup per CU
    std::vector<uint32_t> vl(nq);
    std::vector<int> pcu(nq), order(nq);
    for (int q = 0; q < nq; ++q) {
        const pf::QPostHead* h = reinterpret_cast<const pf::QPostHead*>(imgs[q]->data() + sizeof(pf::QConst));
        vl[q] = pf::post_var_lds(h->n_tok, h->n_tok + h->n_club + h->n_friend);
        pcu[q] = post_image_per_cu(h);
        order[q] = q;
    }
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pcu[a] > pcu[b]; });
    std::vector<uint32_t> offs;
    std::vector<int32_t> orows(nq);
    size_t pool_b = 0;
    for (int i = 0; i < nq; ++i) {
        offs.push_back((uint32_t)pool_b);
        pool_b += imgs[order[i]]->size();
        orows[i] = rows[order[i]];
    }
    const uint32_t wave_lds = vl[order[0]];  // the one-query case
    const int nwb = c->wb_end - c->wb_begin;
    const int per_cu = pcu[order[0]];
    // One query: one resident round of workgroups loops over the blocks.  A batch: a few blocks
    // per workgroup (batch_blocks_per_wg), so the resident workgroups (dispatched x-fastest)
    // cover a few queries at a time and share their lists and cells in L2; with one resident
    // round looping over every query's range instead, 256 queries run at once and L2 hits
    // collapse (per-query time 0.2 ms at 4 queries per launch, 0.68 ms at 1024).
    const bool on_lane = nq == 1 && scan_lanes() >= 2 && s != c->stream;  // lane_begin's choice, below
    const int blocks = nq == 1 ? std::max(1, std::min(nwb, one_query_wgs(c->num_cus * per_cu, on_lane)))
                               : std::max(1, (nwb + batch_blocks_per_wg() - 1) / batch_blocks_per_wg());
    const size_t offs_b = ((size_t)nq * 4 + 15) & ~(size_t)15;
    const size_t rows_b = ((size_t)nq * 4 + 15) & ~(size_t)15;
    const size_t sync_b = (size_t)nq * sizeof(pf::ScanSync);
    const size_t total = offs_b + rows_b + sync_b + pool_b;
    // a single query on a caller's stream goes to the next scan lane: its upload and launch on the
    // lane's stream, its row copied out on the caller's stream
    LaneUse lu;
    if (nq == 1) {
        const int rc = lane_begin(c, s, lu);
        if (rc != PF_OK) return rc;
    }
    pf_ctx::ScanLane* ln = lu.ln;
    const hipStream_t caller = s;
    uint64_t* out_keys = d_keys;
    const int32_t out_row0 = rows[order[0]];
    if (ln) {
        s = ln->st;
        out_keys = lu.keys;
        orows[0] = 0;  // the lane's own one-row result
    }
    DBuf& pool_buf = ln ? ln->pool : c->d_pool;
    DBuf& part_buf = ln ? ln->part : c->d_part;
    pf::HpLap lw;
    uint8_t* h = c->stage_acquire(total);
    lw.lap(pf::kHpScanStageWait);
    if (!h) return c->fail(PF_ENOMEM, "pinned staging allocation failed");
    std::memcpy(h, offs.data(), (size_t)nq * 4);
    std::memcpy(h + offs_b, orows.data(), (size_t)nq * 4);
    std::memset(h + offs_b + rows_b, 0, sync_b);
    for (int i = 0; i < nq; ++i)
        std::memcpy(h + offs_b + rows_b + sync_b + offs[i], imgs[order[i]]->data(), imgs[order[i]]->size());
    HIPCHK(c, pool_buf.ensure(total));
    HIPCHK(c, hipMemcpyAsync(pool_buf.p, h, total, hipMemcpyHostToDevice, s));
    HIPCHK(c, c->stage_release(s));
    uint8_t* base = pool_buf.as<uint8_t>();
    HIPCHK(c, part_buf.ensure((size_t)nq * (blocks + 8) * k * sizeof(uint64_t)));  // + 8 group lists (post_tail)
    hipEvent_t e0, e1;
    int rc = scan_events(c, timed, e0, e1);
    if (rc != PF_OK) return rc;
    // timed: the events ride in the kernel's dispatch (its own start / end; r2ff: 1.8 us less
    // per launch than two marker packets around it)
    // one launch per class (the first one's start and the last one's end time the call)
    for (int q0 = 0; q0 < nq;) {
        int q1 = q0;
        uint32_t vmax = 0;
        while (q1 < nq && pcu[order[q1]] == pcu[order[q0]]) vmax = std::max(vmax, vl[order[q1++]]);
        HIPCHK(c, pf::launch_post(c->ps, base + offs_b + rows_b + sync_b, reinterpret_cast<const uint32_t*>(base) + q0,
                                  nq == 1 ? wave_lds : vmax, q1 - q0, c->wb_begin, c->wb_end, k, blocks,
                                  part_buf.as<uint64_t>() + (size_t)q0 * (blocks + 8) * k,
                                  reinterpret_cast<pf::ScanSync*>(base + offs_b + rows_b) + q0, out_keys,
                                  reinterpret_cast<const int32_t*>(base + offs_b) + q0, post_mode(nq),
                                  tail_block_cands(), (timed && q0 == 0) ? e0 : nullptr,
                                  (timed && q1 == nq) ? e1 : (ln ? ln->done : nullptr), s));
        q0 = q1;
    }
    if (ln) {  // the caller's stream: wait for the lane's launch (its stop event), copy its row out
        rc = lane_end(c, lu, (timed ? e1 : ln->done), caller, d_keys + (size_t)out_row0 * k, k);
        if (rc != PF_OK) return rc;
    }
    if (timed) {
        c->last_ev0 = e0;
        c->last_ev1 = e1;
    }
    return PF_OK;
}

// K5 for ONE query from the resident images (pf_ctx.h ResidentPost): no host image build and no
// upload.  The image part and its QConst (the user's resident K1' image) are already in HBM, the
// ScanSync is the lane's own (or the context's, on its own stream), zeroed once and left zeroed by
// every launch (post_tail), and the merge writes the lane's result row.  HIP calls per step on a
// caller's stream: the launch (its stop event bound to the dispatch), the caller's wait on it and
// the row copy (+ one event record per ring group of eight rows).
bool resident_ok(const pf_ctx* c, int32_t i) {
    const auto& R = c->rp;
    return R.on && R.var_lds[i] != 0 && !R.stale[i] && pf::post_lds(R.var_lds[i]) <= kK5LdsCap;
}

int scan_post_resident(pf_ctx* c, int32_t i, int32_t row, int k, uint64_t* d_keys, hipStream_t s, bool timed) {
    auto& R = c->rp;
    const uint32_t vl = R.var_lds[i];
    const int per_cu = pf::post_blocks_per_cu(vl);
    const int nwb = c->wb_end - c->wb_begin;
    LaneUse lu;
    int rc = lane_begin(c, s, lu);
    if (rc != PF_OK) return rc;
    pf_ctx::ScanLane* ln = lu.ln;
    const int blocks = std::max(1, std::min(nwb, one_query_wgs(c->num_cus * per_cu, ln != nullptr)));
    const hipStream_t ls = ln ? ln->st : s;
    DBuf& part_buf = ln ? ln->part : c->d_part;
    DBuf& sync_buf = ln ? ln->sync : R.d_sync;
    if (!sync_buf.p) {  // once: every launch leaves it zeroed
        HIPCHK(c, sync_buf.ensure(sizeof(pf::ScanSync)));
        HIPCHK(c, hipMemsetAsync(sync_buf.p, 0, sizeof(pf::ScanSync), ls));
    }
    HIPCHK(c, part_buf.ensure((size_t)(blocks + 8) * k * sizeof(uint64_t)));  // + 8 group lists (post_tail)
    hipEvent_t e0, e1;
    rc = scan_events(c, timed, e0, e1);
    if (rc != PF_OK) return rc;
    hipEvent_t stop = timed ? e1 : (ln ? ln->done : nullptr);
    uint64_t* out = ln ? lu.keys : d_keys + (size_t)row * k;
    const uint8_t* img = R.d_pool.as<uint8_t>() + R.off[i] - sizeof(pf::QConst);
    const uint8_t* qc = c->jb.d_pimg.as<uint8_t>() + c->jb.pimg_off[i];
    HIPCHK(c, pf::launch_post(c->ps, img, R.d_zero.as<uint32_t>(), vl, 1, c->wb_begin, c->wb_end, k, blocks,
                              part_buf.as<uint64_t>(), sync_buf.as<pf::ScanSync>(), out, R.d_zero.as<int32_t>(),
                              post_mode(1), tail_block_cands(), timed ? e0 : nullptr, stop, ls, qc));
    if (ln) {
        rc = lane_end(c, lu, stop, s, d_keys + (size_t)row * k, k);
        if (rc != PF_OK) return rc;
    }
    if (timed) {
        c->last_ev0 = e0;
        c->last_ev1 = e1;
    }
    return PF_OK;
}

// Every user's K5 image part (ResidentPost) built once at open: host threads write the parts of a
// chunk of users into a pinned buffer (build_query_post_part, the per-call builder's own code, so
// the bytes equal a per-call image's), one async copy per chunk, two buffers in turn.  Needs the
// job pipeline's resident K1' images (their QConst) and the postings store; when the parts do not
// fit a third of the free HBM, or PF_DEBUG resident_post=0, every call builds its image as before.
int build_resident_post(pf_ctx* c) {
    auto& R = c->rp;
    R.on = false;
    const auto& hc = c->hc;
    const auto& J = c->jb;
    if (!c->hp.ok || !J.pimg || pf::debug_long("resident_post", 1) == 0 || hc.n == 0) return PF_OK;
    const int32_t n = hc.n;
    std::vector<const std::vector<int32_t>*> adj((size_t)n, nullptr);
    std::vector<int64_t> off((size_t)n + 1, 0);
    par_jobs((size_t)n, [&](size_t i) {
        auto it = hc.adj.find(hc.uid[i]);
        if (it != hc.adj.end()) adj[i] = &it->second;
        // users without a resident K1' image (outside the device tables' limits) get none either
        off[i + 1] = J.img_lg[i] ? (int64_t)pf::post_part_bound(hc, (int32_t)i, (adj[i] ? adj[i]->size() : 0) + 1) : 0;
    }, 1 << 14);
    off[0] = sizeof(pf::QConst);  // the first image's QConst-sized lead stays inside the pool
    for (int32_t i = 0; i < n; ++i) off[i + 1] += off[i];
    const size_t total = (size_t)off[n];
    size_t freeb = 0, totb = 0;
    if (hipMemGetInfo(&freeb, &totb) != hipSuccess || total > freeb / 3) return PF_OK;
    if (R.d_pool.p) (void)hipFree(R.d_pool.p);
    R.d_pool.p = nullptr;
    R.d_pool.cap = 0;
    if (hipMalloc(&R.d_pool.p, total) != hipSuccess) {  // no room after all: every call builds its image
        R.d_pool.p = nullptr;
        (void)hipGetLastError();
        return PF_OK;
    }
    R.d_pool.cap = total;
    R.var_lds.assign((size_t)n, 0);
    R.stale.assign((size_t)n, 0);
    constexpr size_t kChunkBytes = (size_t)256 << 20;
    PinBuf pin[2];
    hipEvent_t ev[2] = {nullptr, nullptr};
    for (auto& e : ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int rc = PF_OK;
    std::atomic<int> bad{0};
    int b = 0;
    for (int32_t i0 = 0; i0 < n && rc == PF_OK; b ^= 1) {
        int32_t i1 = i0 + 1;
        while (i1 < n && (size_t)(off[i1 + 1] - off[i0]) <= kChunkBytes) ++i1;
        const size_t bytes = (size_t)(off[i1] - off[i0]);
        if (hipEventSynchronize(ev[b]) != hipSuccess || pin[b].ensure(std::max<size_t>(bytes, 16)) != hipSuccess) {
            rc = PF_ENOMEM;  // pinned staging refused: the resident images stay off (below)
            break;
        }
        uint8_t* h = pin[b].as<uint8_t>();
        par_jobs((size_t)(i1 - i0), [&](size_t j) {
            const int32_t i = i0 + (int32_t)j;
            const size_t cap = (size_t)(off[i + 1] - off[i]);
            if (cap == 0) return;
            std::vector<int32_t> ex;
            if (adj[i]) ex = *adj[i];
            ex.push_back(hc.uid[i]);
            uint8_t* dst = h + (off[i] - off[i0]);
            if (pf::build_query_post_part(hc, c->hp, i, ex, dst, cap) == 0) {
                bad.fetch_add(1);
                return;
            }
            pf::QPostHead hd;
            std::memcpy(&hd, dst, sizeof hd);
            R.var_lds[(size_t)i] = pf::post_var_lds(hd.n_tok, hd.n_tok + hd.n_club + hd.n_friend);
        }, 256);
        if (hipMemcpyAsync(R.d_pool.as<uint8_t>() + off[i0], h, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
            hipEventRecord(ev[b], c->stream) != hipSuccess)
            rc = c->fail(PF_ENODEV, "resident postings images: upload failed");
        i0 = i1;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess && rc == PF_OK) rc = c->fail(PF_ENODEV, "resident postings images");
    for (auto& e : ev) (void)hipEventDestroy(e);
    if (rc == PF_ENOMEM) {  // not fatal: the per-call images serve every query
        (void)hipFree(R.d_pool.p);
        R.d_pool.p = nullptr;
        R.d_pool.cap = 0;
        return PF_OK;
    }
    if (rc != PF_OK) return rc;
    if (bad.load()) return c->fail(PF_EINTERNAL, "resident postings image larger than its bound");
    HIPCHK(c, R.d_zero.ensure(64));
    HIPCHK(c, hipMemset(R.d_zero.p, 0, 64));
    R.off.swap(off);
    R.on = true;
    return PF_OK;
}

// K1: the record-stream scan for `idx` (valid query indices) into d_keys rows `rows`.
// One pinned staging buffer [refs | rows | sync | image pool] goes up in a single async copy.
int scan_stream(pf_ctx* c, const std::vector<int32_t>& idx, const std::vector<int32_t>& rows, int k, uint64_t* d_keys,
                hipStream_t s, bool timed) {
    if (idx.empty()) return PF_OK;
    Images im;
    pf::QImageHost qi;
    std::vector<int32_t> excl;
    for (int32_t i : idx) {
        const int32_t u = c->hc.uid[i];
        excl.clear();
        auto it = c->hc.adj.find(u);
        if (it != c->hc.adj.end()) excl = it->second;
        excl.push_back(u);
        if (!pf::build_query(c->hc, c->hs.packed, i, &excl, qi)) return c->fail(PF_EUNSUPP, "query hash table too large");
        add_image(im, qi);
    }
    const int nq = (int)idx.size();
    const int tiles = c->tile_end - c->tile_begin;
    // one resident round of blocks over the batch: tiles come from a per-query queue, so
    // the waves that exist balance the work themselves
    const int per_cu = pf::scan_blocks_per_cu(c->hs.packed, im.gtab, im.max_lds);
    const int blocks = std::max(1, std::min((tiles + 3) / 4, std::max(1, c->num_cus * per_cu / nq)));
    const size_t refs_b = (size_t)nq * sizeof(pf::QImageRef);
    const size_t rows_b = ((size_t)nq * sizeof(int32_t) + 15) & ~(size_t)15;
    const size_t sync_b = (size_t)nq * sizeof(pf::ScanSync);  // zeros: the per-launch rendezvous
    const size_t total = refs_b + rows_b + sync_b + im.pool.size();
    uint8_t* h = c->stage_acquire(total);
    if (!h) return c->fail(PF_ENOMEM, "pinned staging allocation failed");
    std::memcpy(h, im.refs.data(), refs_b);
    std::memcpy(h + refs_b, rows.data(), (size_t)nq * sizeof(int32_t));
    std::memset(h + refs_b + rows_b, 0, sync_b);
    std::memcpy(h + refs_b + rows_b + sync_b, im.pool.data(), im.pool.size());
    HIPCHK(c, c->d_pool.ensure(total));
    HIPCHK(c, hipMemcpyAsync(c->d_pool.p, h, total, hipMemcpyHostToDevice, s));
    HIPCHK(c, c->stage_release(s));
    uint8_t* base = c->d_pool.as<uint8_t>();
    const pf::QImageRef* d_refs = reinterpret_cast<const pf::QImageRef*>(base);
    const int32_t* d_rows = reinterpret_cast<const int32_t*>(base + refs_b);
    pf::ScanSync* d_sync = reinterpret_cast<pf::ScanSync*>(base + refs_b + rows_b);
    const uint8_t* d_images = base + refs_b + rows_b + sync_b;
    HIPCHK(c, c->d_part.ensure((size_t)nq * (blocks + 8) * k * sizeof(uint64_t)));  // + 8 group lists (post_tail)
    hipEvent_t e0, e1;
    int rc = scan_events(c, timed, e0, e1);
    if (rc != PF_OK) return rc;
    if (timed) HIPCHK(c, hipEventRecord(e0, s));
    HIPCHK(c, pf::launch_scan(c->ds, d_images, d_refs, im.max_lds, im.gtab, nq, c->tile_begin, c->tile_end, k, blocks,
                              c->d_part.as<uint64_t>(), d_sync, d_keys, d_rows, s));
    if (timed) {
        HIPCHK(c, hipEventRecord(e1, s));
        c->last_ev0 = e0;
        c->last_ev1 = e1;
    }
    return PF_OK;
}

// All-candidates scan for `idx` (valid query indices) into d_keys rows `rows`.  The postings
// scan (K5) serves every query whose lists fit one workgroup's LDS; a query naming more lists
// (a user with ~15k friends or thousands of tokens) goes to the record-stream scan (K1) in a
// launch of its own, so one heavy user never fails the batch.
int scan_all(pf_ctx* c, const std::vector<int32_t>& idx, const std::vector<int32_t>& rows, int k, uint64_t* d_keys,
             hipStream_t s, bool timed) {
    if (idx.empty()) return PF_OK;
    if (!c->use_post()) return scan_stream(c, idx, rows, k, d_keys, s, timed);
    pf::HpLap lp;  // PF_DEBUG host_prof=1: image build / staging + launch clocks
    if (pf::host_prof().on) pf::host_prof().ns[pf::kHpScanCalls] += 1000000000LL;
    // one query from the resident images: on the context's stream or a scan lane (another stream
    // without lanes takes the upload path: the resident ScanSync of the context's stream is not
    // shared with a stream it is not ordered against)
    if (idx.size() == 1 && resident_ok(c, idx[0]) && (s == c->stream || scan_lanes() >= 2)) {
        const int rc = scan_post_resident(c, idx[0], rows[0], k, d_keys, s, timed);
        lp.lap(pf::kHpScanLaunch);
        return rc;
    }
    // the query images (host, ~35 us each) on threads for a batch
    std::vector<std::vector<uint8_t>> imgs(idx.size());
    std::vector<uint8_t> fits(idx.size(), 1);
    par_jobs(idx.size(), [&](size_t q) {
        const int32_t i = idx[q], u = c->hc.uid[i];
        std::vector<int32_t> ex;
        auto it = c->hc.adj.find(u);
        if (it != c->hc.adj.end()) ex = it->second;
        ex.push_back(u);
        pf::build_query_post(c->hc, c->hp, i, ex, imgs[q]);
        const pf::QPostHead* h = reinterpret_cast<const pf::QPostHead*>(imgs[q].data() + sizeof(pf::QConst));
        fits[q] = post_image_lds(h) <= kK5LdsCap;
    });
    std::vector<const std::vector<uint8_t>*> pi;
    std::vector<int32_t> prow, sidx, srow;
    for (size_t q = 0; q < idx.size(); ++q) {
        if (fits[q]) { pi.push_back(&imgs[q]); prow.push_back(rows[q]); }
        else { sidx.push_back(idx[q]); srow.push_back(rows[q]); }
    }
    lp.lap(pf::kHpScanImage);
    int rc = scan_post(c, pi, prow, k, d_keys, s, timed);
    lp.lap(pf::kHpScanLaunch);
    if (rc != PF_OK) return rc;
    return scan_stream(c, sidx, srow, k, d_keys, s, timed && pi.empty());
}

// Bytes the postings scan (K5) reads for one query image over this context's blocks, by the
// kernel's own access pattern (fas_post_kernel): per block, 32 B of header per candidate, two
// cell words per list, and every entry of the list's cell-rounded range (4 B; token entries
// also their 8-B norm); per block the exclusion list (whole when <= 256 entries); per
// workgroup the staged image.
int64_t post_query_bytes(const pf_ctx* c, const std::vector<uint8_t>& img, int wgs) {
    const pf::QPostHead* h = reinterpret_cast<const pf::QPostHead*>(img.data() + sizeof(pf::QConst));
    const pf::QTok* toks = reinterpret_cast<const pf::QTok*>(img.data() + h->tok_off);
    const pf::PList* sets = reinterpret_cast<const pf::PList*>(img.data() + h->set_off);
    const uint32_t B = (uint32_t)c->ps.bsize, n = (uint32_t)c->ps.n;
    const uint32_t* cells = c->hp.cells.data();
    int64_t bytes = 0;
    auto list_bytes = [&](const pf::PList& L, int per) {
        for (int32_t blk = c->wb_begin; blk < c->wb_end; ++blk) {
            const uint32_t c0 = (uint32_t)blk * B, c1 = std::min(c0 + B, n) - 1;
            const uint32_t lo = cells[L.cell_off + (c0 >> L.shift)], hi = cells[L.cell_off + (c1 >> L.shift) + 1];
            bytes += (int64_t)(hi - lo) * per + 8;
        }
    };
    for (int j = 0; j < h->n_tok; ++j) list_bytes(toks[j].l, 12);
    for (int j = 0; j < h->n_club + h->n_friend; ++j) list_bytes(sets[j], 4);
    const int64_t nb = c->wb_end - c->wb_begin;
    const int64_t cands = std::max<int64_t>(0, std::min<int64_t>((int64_t)c->wb_end * B, n) - (int64_t)c->wb_begin * B);
    bytes += cands * 32;
    bytes += nb * 4 * (int64_t)std::min(h->n_excl, (int32_t)pf::kPostThreads);
    bytes += (int64_t)std::min<int64_t>(nb, wgs) * (int64_t)img.size();
    return bytes;
}

int emit_jobs(pf_ctx* c, std::vector<pf::Job>& jobs, int topk, int32_t* ou, float* os, int32_t* oc) {
    for (size_t i = 0; i < jobs.size(); ++i) oc[i] = 0;
    if (topk == 0 || jobs.empty()) return PF_OK;
    const int rc = pf::run_jobs(c, jobs);
    if (rc != PF_OK) return rc;
    for (size_t i = 0; i < jobs.size(); ++i) emit(jobs[i].out, (int)i, topk, ou, os, oc);
    return PF_OK;
}

}  // namespace

namespace pf {

const std::unordered_map<int32_t, std::vector<int32_t>>& base_adj(const pf_ctx* c) { return c->hc.adj; }

HostProf::HostProf() {
    on = debug_long("host_prof", 0) != 0;
    for (auto& x : ns) x = 0;
}
HostProf::~HostProf() {
    if (!on) return;
    static const char* nm[kHpStages] = {"workspaces", "prep", "layout", "staging", "wait", "decode", "launch-b",
                                        "launch-a", "finish", "scan-image", "scan-launch", "scan-calls(n)", "scan-stage-wait"};
    fprintf(stderr, "pokec_fas host stages (s):");
    for (int i = 0; i < kHpStages; ++i) fprintf(stderr, " %s=%.3f", nm[i], (double)ns[i].load() * 1e-9);
    fprintf(stderr, "\n");
}
HostProf& host_prof() {
    static HostProf h;
    return h;
}

}  // namespace pf

extern "C" {

int pf_abi_version(void) { return PF_ABI_VERSION; }

int pf_open(const pf_corpus_desc* desc, int device, pf_ctx** out) {
    if (!out) { g_open_error = "null out"; return PF_EINVAL; }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        g_open_error = "no HIP device (the FAS engine has no CPU fallback)";
        return PF_ENODEV;
    }
    if (device < 0 || device >= ndev) { g_open_error = "bad device ordinal"; return PF_EINVAL; }
    pf_ctx* c = new pf_ctx();
    c->device = device;
    auto bail = [&](int rc) {
        g_open_error = c->err;
        delete c;
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) { c->err = "hipSetDevice failed"; return bail(PF_ENODEV); }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        c->num_cus = prop.multiProcessorCount;
        if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
            c->err = std::string("device is ") + prop.gcnArchName + ", the kernels are built for gfx950";
            return bail(PF_ENODEV);
        }
    }
    const bool prof = pf::host_prof().on;
    auto t0 = std::chrono::steady_clock::now();
    auto stage = [&](const char* what) {  // PF_DEBUG host_prof=1: pf_open stage clocks on stderr
        const auto t1 = std::chrono::steady_clock::now();
        if (prof) fprintf(stderr, "[pf_open] %s %.3f s\n", what, std::chrono::duration<double>(t1 - t0).count());
        t0 = t1;
    };
    int rc = pf::build_host_corpus(desc, c->hc, c->err);
    if (rc != PF_OK) return bail(rc);
    stage("host corpus (sorted rows, idf, norms)");
    rc = pf::build_store(c->hc, c->hs, c->err);
    if (rc != PF_OK) return bail(rc);
    stage("tile store");
    pf::build_postings(c->hc, c->hp);  // hp.ok = false: the stream scan serves every query
    stage("postings store");
    // PF_DEBUG scan=stream|postings sets the context's initial scan kernel (tests force variants
    // per process with it); pf_set_scan_kernel changes it later
    if (const char* sk = pf::debug_str("scan")) {
        if (!strcmp(sk, "stream")) c->scan_kind = PF_SCAN_STREAM;
        else if (!strcmp(sk, "postings") && c->hp.ok) c->scan_kind = PF_SCAN_POSTINGS;
    }
    // the job pipeline's two aux streams are created here with the context's own, so the three
    // take consecutive hardware queues whatever streams the host process creates later (created
    // at the first job call, after a torch stream pool, they ran the cfg-3 sub-record of the
    // default bench line at 0.466 vs 0.415 ms per step, r5l)
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        (pf::debug_long("lazy_aux", 0) == 0 &&
         (hipStreamCreateWithFlags(&c->jb.aux, hipStreamNonBlocking) != hipSuccess ||
          hipStreamCreateWithFlags(&c->jb.aux2, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&c->jb.ev_fork, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&c->jb.ev_join, hipEventDisableTiming) != hipSuccess)) ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        c->err = "stream/event creation failed";
        return bail(PF_ENODEV);
    }
    for (int l = 3; l < scan_lanes(); ++l)  // lanes past the context's and the aux streams
        if (hipStreamCreateWithFlags(&c->lane_st[l], hipStreamNonBlocking) != hipSuccess) {
            c->err = "stream creation failed";
            return bail(PF_ENODEV);
        }
    auto& hs = c->hs;
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = upload(c, c->d_stream, hs.stream);
    if (e == hipSuccess) e = upload(c, c->d_tile_off, hs.tile_off);
    if (e == hipSuccess) e = upload(c, c->d_tile_steps, hs.tile_steps);
    if (e == hipSuccess) e = upload(c, c->d_tile_slot0, hs.tile_slot0);
    if (e == hipSuccess) e = upload(c, c->d_tile_lgk, hs.tile_lgk);
    if (e == hipSuccess) e = upload(c, c->d_slot_tile, hs.slot_tile);
    if (e == hipSuccess) e = upload(c, c->d_norms, hs.norms);
    if (e == hipSuccess) e = upload(c, c->d_norm_off, hs.norm_off);
    if (e == hipSuccess) e = upload(c, c->d_hdr0, hs.hdr0);
    if (e == hipSuccess) e = upload(c, c->d_hdr1, hs.hdr1);
    if (e == hipSuccess) e = upload(c, c->d_hdr2, hs.hdr2);
    if (e == hipSuccess) e = upload(c, c->d_rowstore, hs.rows);
    if (e == hipSuccess) e = upload(c, c->d_rowstore_off, hs.row_off);
    if (c->hp.ok) {
        auto& hp = c->hp;
        if (e == hipSuccess) e = upload(c, c->d_phdr, hp.hdr);
        if (e == hipSuccess) e = upload(c, c->d_post, hp.post);
        if (e == hipSuccess) e = upload(c, c->d_pnorm, hp.pnorm);
        if (e == hipSuccess) e = upload(c, c->d_cells, hp.cells);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    stage("upload");
    if (e != hipSuccess) {
        c->hip_fail(e, "corpus upload");
        return bail(e == hipErrorOutOfMemory ? PF_ENOMEM : PF_ENODEV);
    }
    c->ds.row_pad = c->d_rowstore.as<uint4>() + hs.row_off[c->hc.n];  // build_store's trailing padding line
    c->stream_bytes = (int64_t)hs.stream.size() * 16;
    c->norm_bytes = (int64_t)hs.norms.size() * 8;
    if (c->hp.ok) {
        c->post_bytes = (int64_t)c->hp.hdr.size() * 16 + (int64_t)c->hp.post.size() * 4 +
                        (int64_t)c->hp.pnorm.size() * 8 + (int64_t)c->hp.cells.size() * 4;
        c->ps.n_post = (uint32_t)c->hp.post.size();
        c->ps.n_tok_entries = (uint32_t)c->hp.pnorm.size();
        c->ps.n_cells = (uint32_t)c->hp.cells.size();
    }
    // the host copies of the device stores (~5 GB at 1.63M users) are returned to the system on a
    // detached thread: unmapping them takes ~0.6 s that pf_open need not wait for
    try {
        std::thread([a = std::move(hs.stream), b = std::move(hs.norms), r = std::move(hs.rows),
                     p = std::move(c->hp.post), q = std::move(c->hp.pnorm)]() mutable {}).detach();
    } catch (...) {  // no thread to be had: free them here (no exception crosses the C ABI)
        hs.stream.clear(); hs.norms.clear(); hs.rows.clear(); c->hp.post.clear(); c->hp.pnorm.clear();
    }
    std::vector<uint64_t>().swap(hs.row_off);
    c->ds.stream = c->d_stream.as<uint4>();
    c->ds.tile_off = c->d_tile_off.as<uint64_t>();
    c->ds.tile_steps = c->d_tile_steps.as<uint32_t>();
    c->ds.tile_slot0 = c->d_tile_slot0.as<uint32_t>();
    c->ds.tile_lgk = c->d_tile_lgk.as<uint8_t>();
    c->ds.slot_tile = c->d_slot_tile.as<uint32_t>();
    c->ds.norms = c->d_norms.as<double>();
    c->ds.norm_off = c->d_norm_off.as<uint64_t>();
    c->ds.hdr0 = c->d_hdr0.as<uint4>();
    c->ds.hdr1 = c->d_hdr1.as<uint4>();
    c->ds.hdr2 = c->d_hdr2.as<uint4>();
    c->ds.rows = c->d_rowstore.as<uint4>();
    c->ds.row_off = c->d_rowstore_off.as<uint64_t>();
    c->ds.n_slots = c->hc.n;
    c->ds.n_tiles = (int32_t)hs.tile_steps.size();
    c->ds.packed = hs.packed ? 1 : 0;
    c->ds.n_cols = c->hc.T;
    c->tile_begin = 0;
    c->tile_end = c->ds.n_tiles;
    if (c->hp.ok) {
        auto& hp = c->hp;
        std::vector<uint4>().swap(hp.hdr);
        // hp.post / hp.pnorm went with the host stores above
        // hp.cells stays on the host too: pf_scan_bytes reads the lists' cell ranges
        c->ps.hdr = c->d_phdr.as<uint4>();
        c->ps.post = c->d_post.as<uint32_t>();
        c->ps.pnorm = c->d_pnorm.as<double>();
        c->ps.cells = c->d_cells.as<uint32_t>();
        c->ps.n = c->hc.n;
        // block size: the LDS capacity.  Sizing blocks to fill whole waves of resident
        // workgroups (798 at 1.6M) measured slower (258 vs 244 us): per-block costs dominate
        // the half-empty last wave.  PF_DEBUG k5_block overrides it (tests).
        {
            const int64_t b = pf::debug_long("k5_block", pf::kBlockCands);
            c->ps.bsize = (int32_t)std::max<int64_t>(64, std::min<int64_t>(pf::kBlockCands, b));
        }
        c->ps.n_blocks = (c->hc.n + c->ps.bsize - 1) / c->ps.bsize;
        c->wb_begin = 0;
        c->wb_end = c->ps.n_blocks;
    }
    rc = pf::jobs_open(c);  // device graph + image-builder tables (the recommenders' pipeline)
    if (rc != PF_OK) return bail(rc);
    stage("job pipeline (graph, image tables)");
    rc = build_resident_post(c);  // every user's K5 image part (the one-query scans' resident images)
    if (rc != PF_OK) return bail(rc);
    stage(c->rp.on ? ("resident postings images, " + std::to_string(c->rp.d_pool.cap >> 20) + " MiB").c_str()
                   : "resident postings images (off)");
    *out = c;
    return PF_OK;
}

void pf_close(pf_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    c->jb.pending.clear();  // calls never waited for: their outputs are not written
    c->jb.carry = pf::JobsState::Carry{};
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->jb.aux2) (void)hipStreamSynchronize(c->jb.aux2);
    for (auto& e : c->prof_ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    for (auto& ln : c->lane) {  // (their streams are the context's, the aux streams and lane_st)
        if (ln.st) (void)hipStreamSynchronize(ln.st);
        if (ln.done) (void)hipEventDestroy(ln.done);
        for (hipEvent_t e : ln.freed)
            if (e) (void)hipEventDestroy(e);
    }
    for (hipStream_t st : c->lane_st)
        if (st) (void)hipStreamDestroy(st);
    for (auto& st : c->stage) {
        if (st.done) (void)hipEventDestroy(st.done);
        if (st.p) (void)hipHostFree(st.p);
    }
    if (c->jb.aux) {
        (void)hipStreamSynchronize(c->jb.aux);
        (void)hipStreamDestroy(c->jb.aux);
    }
    if (c->jb.aux2) {
        (void)hipStreamSynchronize(c->jb.aux2);
        (void)hipStreamDestroy(c->jb.aux2);
    }
    if (c->jb.ev_fork) (void)hipEventDestroy(c->jb.ev_fork);
    if (c->jb.ev_join) (void)hipEventDestroy(c->jb.ev_join);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* pf_last_error(const pf_ctx* c) { return c ? c->err.c_str() : g_open_error.c_str(); }
int32_t pf_num_users(const pf_ctx* c) { return c ? c->hc.n : 0; }
float pf_idf(const pf_ctx* c, int32_t col, int32_t tid) {
    if (!c || col < 0 || col >= c->hc.T) return NAN;
    return c->hc.idf_of_tid(col, tid);
}

int pf_fas_pairs(pf_ctx* c, const int32_t* a, const int32_t* b, int64_t n, float* out) {
    if (!c || n < 0 || (n && (!a || !b || !out))) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    std::unordered_map<int32_t, int32_t> group;  // query idx -> group
    std::vector<int32_t> qidx;
    std::vector<std::vector<int32_t>> slots;
    std::vector<std::pair<int32_t, int32_t>> where(n, {-1, -1});
    for (int64_t i = 0; i < n; ++i) {
        out[i] = NAN;
        int32_t ia = c->hc.idx_of(a[i]), ib = c->hc.idx_of(b[i]);
        if (ia < 0 || ib < 0) continue;
        auto it = group.find(ia);
        if (it == group.end()) {
            it = group.emplace(ia, (int32_t)qidx.size()).first;
            qidx.push_back(ia);
            slots.emplace_back();
        }
        where[i] = {it->second, (int32_t)slots[it->second].size()};
        slots[it->second].push_back(c->hs.slot_of_idx[ib]);
    }
    std::vector<std::vector<float>> res;
    int rc = run_pairs(c, qidx, slots, res);
    if (rc != PF_OK) return rc;
    for (int64_t i = 0; i < n; ++i)
        if (where[i].first >= 0) out[i] = res[where[i].first][where[i].second];
    return PF_OK;
}

int pf_recommend_interest(pf_ctx* c, const int32_t* q, int32_t nq, int32_t topk, int32_t mode, int32_t limit,
                          int32_t* ou, float* os, int32_t* oc) {
    if (!c || nq < 0 || topk < 0 || (nq && (!q || !oc))) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    for (int i = 0; i < nq; ++i) oc[i] = 0;
    if (topk == 0 || nq == 0) return PF_OK;
    if (mode == PF_MODE_ALL && topk <= pf::kMaxTopK) {
        std::vector<int32_t> idx, rows;
        for (int i = 0; i < nq; ++i) {
            int32_t x = c->hc.idx_of(q[i]);
            if (x >= 0) { idx.push_back(x); rows.push_back(i); }
        }
        HIPCHK(c, c->d_out.ensure((size_t)nq * topk * sizeof(uint64_t)));
        if ((int)idx.size() < nq)  // rows of unknown users stay empty
            HIPCHK(c, hipMemsetAsync(c->d_out.p, 0xFF, (size_t)nq * topk * sizeof(uint64_t), c->stream));
        const int chunk = 256;
        for (size_t b = 0; b < idx.size(); b += chunk) {
            std::vector<int32_t> ii(idx.begin() + b, idx.begin() + std::min(idx.size(), b + chunk));
            std::vector<int32_t> rr(rows.begin() + b, rows.begin() + std::min(rows.size(), b + chunk));
            int rc = scan_all(c, ii, rr, topk, c->d_out.as<uint64_t>(), c->stream, b == 0);
            if (rc != PF_OK) return rc;
        }
        std::vector<uint64_t> keys((size_t)nq * topk);
        HIPCHK(c, hipMemcpyAsync(keys.data(), c->d_out.p, keys.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (!idx.empty() && c->last_ev0) HIPCHK(c, hipEventElapsedTime(&c->last_scan_ms, c->last_ev0, c->last_ev1));
        for (int i = 0; i < nq; ++i) pf_decode_keys(&keys[(size_t)i * topk], topk, ou + (size_t)i * topk, os + (size_t)i * topk, &oc[i]);
        return PF_OK;
    }
    // FoF-limited (reference) mode, or ALL with topk beyond the in-kernel bound
    std::vector<pf::Job> jobs(nq);
    for (int i = 0; i < nq; ++i) {
        jobs[i].kind = pf::kJobInterest;
        jobs[i].uid = q[i];
        jobs[i].topk = topk;
        jobs[i].limit = limit;
        jobs[i].all_candidates = mode == PF_MODE_ALL;
        jobs[i].view = plain_view(c);
    }
    return emit_jobs(c, jobs, topk, ou, os, oc);
}

// recommender_graph.cpp:105-222
int pf_recommend_collab(pf_ctx* c, const int32_t* q, int32_t nq, int32_t topk, int32_t limit, int32_t* ou,
                        float* os, int32_t* oc) {
    if (!c || nq < 0 || topk < 0 || (nq && (!q || !oc))) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    std::vector<pf::Job> jobs(nq);
    for (int i = 0; i < nq; ++i) {
        jobs[i].kind = pf::kJobCollab;
        jobs[i].uid = q[i];
        jobs[i].topk = topk;
        jobs[i].limit = limit;
        jobs[i].view = plain_view(c);
    }
    return emit_jobs(c, jobs, topk, ou, os, oc);
}

// recommender_clubs.cpp:10-73
int pf_recommend_clubs(pf_ctx* c, const int32_t* q, int32_t nq, int32_t topk, int32_t limit, int32_t* ou,
                       float* os, int32_t* oc) {
    if (!c || nq < 0 || topk < 0 || (nq && (!q || !oc))) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    std::vector<pf::Job> jobs(nq);
    for (int i = 0; i < nq; ++i) {
        jobs[i].kind = pf::kJobClubs;
        jobs[i].uid = q[i];
        jobs[i].topk = topk;
        jobs[i].limit = limit;
        jobs[i].view = plain_view(c);
    }
    return emit_jobs(c, jobs, topk, ou, os, oc);
}

// Asynchronous forms: plan + launch now, outputs written by pf_wait (pokec_fas.h)
static int job_async(pf_ctx* c, int kind, const int32_t* q, int32_t nq, int32_t topk, int32_t limit, int32_t* ou,
                     float* os, int32_t* oc, uint64_t* ticket) {
    if (!c || !ticket || nq < 0 || topk < 0 || (nq && (!q || !oc || (topk && (!ou || !os))))) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    std::vector<pf::Job> jobs(nq);
    for (int i = 0; i < nq; ++i) {
        jobs[i].kind = kind;
        jobs[i].uid = q[i];
        jobs[i].topk = topk;
        jobs[i].limit = limit;
        jobs[i].view = plain_view(c);
    }
    return pf::run_jobs_async(c, std::move(jobs), topk, ou, os, oc, ticket);
}

int pf_recommend_interest_async(pf_ctx* c, const int32_t* q, int32_t nq, int32_t topk, int32_t limit, int32_t* ou,
                                float* os, int32_t* oc, uint64_t* ticket) {
    return job_async(c, pf::kJobInterest, q, nq, topk, limit, ou, os, oc, ticket);
}
int pf_recommend_collab_async(pf_ctx* c, const int32_t* q, int32_t nq, int32_t topk, int32_t limit, int32_t* ou,
                              float* os, int32_t* oc, uint64_t* ticket) {
    return job_async(c, pf::kJobCollab, q, nq, topk, limit, ou, os, oc, ticket);
}
int pf_recommend_clubs_async(pf_ctx* c, const int32_t* q, int32_t nq, int32_t topk, int32_t limit, int32_t* ou,
                             float* os, int32_t* oc, uint64_t* ticket) {
    return job_async(c, pf::kJobClubs, q, nq, topk, limit, ou, os, oc, ticket);
}
int pf_wait(pf_ctx* c, uint64_t ticket) {
    if (!c) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    return pf::jobs_wait(c, ticket);
}

uint64_t pf_completed_ticket(const pf_ctx* c) {
    if (!c) return 0;
    // tickets are handed out in launch order and completed in launch order
    uint64_t t = c->jb.pending.empty() ? c->jb.next_ticket - 1 : c->jb.pending.front().ticket - 1;
    if (c->jb.carry.on) t = std::min(t, c->jb.carry.ticket - 1);
    return t;
}

int pf_fof_candidates(pf_ctx* c, int32_t uid, int32_t limit, int32_t flavour, int32_t* out, int32_t cap, int32_t* n) {
    if (!c || !n || (cap > 0 && !out)) return PF_EINVAL;
    if (flavour != PF_FOF_GRAPH && flavour != PF_FOF_COLLAB) return PF_EINVAL;
    std::vector<int32_t> v;  // K3 on the device (pf_jobs.hip gather_kernel)
    const int rc = pf::fof_device(c, uid, limit, flavour, v);
    if (rc != PF_OK) return rc;
    for (int32_t i = 0; i < (int32_t)v.size() && i < cap; ++i) out[i] = v[i];
    *n = (int32_t)v.size();
    return PF_OK;
}

int pf_set_adj(pf_ctx* c, int32_t uid, const int32_t* nbrs, int32_t n) {
    if (!c || (n > 0 && !nbrs)) return PF_EINVAL;
    const int rc = pf::jobs_set_adj(c, uid, nbrs, n);
    // the user's exclusions (adj_list row + self) changed: its resident K5 image is stale for good
    if (rc == PF_OK && c->rp.on) {
        const int32_t x = c->hc.idx_of(uid);
        if (x >= 0) c->rp.stale[(size_t)x] = 1;
    }
    return rc;
}

int pf_set_shard(pf_ctx* c, int32_t shard, int32_t nshards) {
    if (!c || nshards < 1 || shard < 0 || shard >= nshards) return PF_EINVAL;
    const auto& steps = c->hs.tile_steps;
    const int T = (int)steps.size();
    std::vector<uint64_t> pre(T + 1, 0);
    for (int t = 0; t < T; ++t) pre[t + 1] = pre[t] + steps[t];
    auto bound = [&](int s) -> int {
        if (s <= 0) return 0;
        if (s >= nshards) return T;
        uint64_t target = pre[T] * (uint64_t)s / (uint64_t)nshards;
        return (int)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
    };
    c->tile_begin = bound(shard);
    c->tile_end = bound(shard + 1);
    // postings scan: contiguous block ranges of equal posting weight.  A block's cost is a
    // fixed part (headers, ranges, top-k: ~60 of ~210 us at cfg 2) plus
    // its share of the lists a query names, i.e. of the postings entries (tokens, clubs,
    // friends) its candidates hold: weight = kBlockFixedWords * candidates + entries.
    const int64_t nwb = c->ps.n_blocks;
    if (nwb > 0) {
        const auto& hc = c->hc;
        const int64_t bs = c->ps.bsize;
        constexpr int64_t kBlockFixedWords = 64;
        std::vector<uint64_t> wpre(nwb + 1, 0);
        for (int64_t b = 0; b < nwb; ++b) {
            const int64_t i0 = b * bs, i1 = std::min<int64_t>(hc.n, i0 + bs);
            const int64_t ent = (hc.tok_off[(size_t)i1 * hc.T] - hc.tok_off[(size_t)i0 * hc.T]) +
                                (hc.club_off[i1] - hc.club_off[i0]) + (hc.friend_off[i1] - hc.friend_off[i0]);
            wpre[b + 1] = wpre[b] + (uint64_t)(kBlockFixedWords * (i1 - i0) + ent);
        }
        auto wbound = [&](int s) -> int32_t {
            if (s <= 0) return 0;
            if (s >= nshards) return (int32_t)nwb;
            const uint64_t target = wpre[nwb] * (uint64_t)s / (uint64_t)nshards;
            return (int32_t)(std::lower_bound(wpre.begin(), wpre.end(), target) - wpre.begin());
        };
        c->wb_begin = wbound(shard);
        c->wb_end = wbound(shard + 1);
    }
    return PF_OK;
}

int pf_set_scan_kernel(pf_ctx* c, int32_t kind) {
    if (!c || kind < PF_SCAN_AUTO || kind > PF_SCAN_POSTINGS) return PF_EINVAL;
    if (kind == PF_SCAN_POSTINGS && !c->hp.ok) return c->fail(PF_EUNSUPP, "postings store unavailable: " + c->hp.why);
    c->scan_kind = kind;
    return PF_OK;
}

int pf_scan_keys_async(pf_ctx* c, const int32_t* q, int32_t nq, int32_t topk, uint64_t* d_keys, void* stream) {
    if (!c || nq < 0 || topk <= 0 || topk > pf::kMaxTopK || (nq && (!q || !d_keys))) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream;  // as given: NULL is the null stream
    std::vector<int32_t> idx, rows;
    for (int i = 0; i < nq; ++i) {
        int32_t x = c->hc.idx_of(q[i]);
        if (x >= 0) { idx.push_back(x); rows.push_back(i); }
    }
    if ((int)idx.size() < nq)  // rows of unknown users stay empty
        HIPCHK(c, hipMemsetAsync(d_keys, 0xFF, (size_t)nq * topk * sizeof(uint64_t), s));
    return scan_all(c, idx, rows, topk, d_keys, s, true);
}

int pf_merge_keys_async(pf_ctx* c, const uint64_t* d_parts, int32_t nparts, int32_t nq, int32_t topk, uint64_t* d_out,
                        void* stream) {
    if (!c || nparts < 1 || nq < 0 || topk <= 0 || topk > pf::kMaxTopK) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(c, pf::launch_merge(d_parts, nparts, (int64_t)nq * topk, topk, nq, topk, d_out, s));
    return PF_OK;
}

int pf_jobs_stats_reset(pf_ctx* c, int32_t enable) { return c ? pf::jobs_stats_reset(c, enable) : PF_EINVAL; }
int pf_jobs_stats_read(pf_ctx* c, pf_jobs_stats* o) { return (c && o) ? pf::jobs_stats_read(c, o) : PF_EINVAL; }

int pf_scan_bytes(pf_ctx* c, const int32_t* q, int32_t nq, int64_t* out) {
    if (!c || nq < 0 || (nq && (!q || !out))) return PF_EINVAL;
    (void)hipSetDevice(c->device);
    // K1: one pass over the shard's tiles and headers, whatever the query
    int64_t k1 = 0;
    for (int32_t t = c->tile_begin; t < c->tile_end; ++t) k1 += (int64_t)c->hs.tile_steps[t] * pf::kTileSlots * 16;
    k1 += (int64_t)(c->tile_end - c->tile_begin) * pf::kTileSlots * 48;
    if (!c->use_post()) {
        for (int i = 0; i < nq; ++i) out[i] = c->hc.idx_of(q[i]) < 0 ? 0 : k1;
        return PF_OK;
    }
    // K5 serves the queries whose lists fit one workgroup's LDS; the others go to K1 in a launch
    // of their own (scan_all's routing): the K5 launch holds only the fitting queries
    std::vector<std::vector<uint8_t>> imgs((size_t)nq);
    std::vector<int8_t> kind((size_t)nq, 0);  // 0 unknown uid, 1 K5, 2 K1
    par_jobs((size_t)nq, [&](size_t i) {
        const int32_t x = c->hc.idx_of(q[i]);
        if (x < 0) return;
        std::vector<int32_t> ex;
        auto it = c->hc.adj.find(q[i]);
        if (it != c->hc.adj.end()) ex = it->second;
        ex.push_back(q[i]);
        pf::build_query_post(c->hc, c->hp, x, ex, imgs[i]);
        const pf::QPostHead* h = reinterpret_cast<const pf::QPostHead*>(imgs[i].data() + sizeof(pf::QConst));
        kind[i] = post_image_lds(h) <= kK5LdsCap ? 1 : 2;
    }, 1);
    int nfit = 0, max_tok = 0, max_lists = 0;
    for (int i = 0; i < nq; ++i) {
        if (kind[i] != 1) continue;
        ++nfit;
        const pf::QPostHead* h = reinterpret_cast<const pf::QPostHead*>(imgs[i].data() + sizeof(pf::QConst));
        max_tok = std::max(max_tok, h->n_tok);
        max_lists = std::max(max_lists, h->n_tok + h->n_club + h->n_friend);
    }
    // workgroups that stage a query's image, as scan_post launches the fitting queries
    const int nwb = c->wb_end - c->wb_begin;
    const int wgs = nfit == 1 ? one_query_wgs(c->num_cus * pf::post_blocks_per_cu(pf::post_var_lds(max_tok, max_lists)), true)
                              : (nwb + batch_blocks_per_wg() - 1) / batch_blocks_per_wg();
    par_jobs((size_t)nq, [&](size_t i) {
        out[i] = kind[i] == 0 ? 0 : (kind[i] == 2 ? k1 : post_query_bytes(c, imgs[i], wgs));
    }, 1);
    return PF_OK;
}

void pf_decode_keys(const uint64_t* keys, int32_t n, int32_t* ou, float* os, int32_t* count) {
    int32_t m = 0;
    for (int32_t i = 0; i < n; ++i) {
        if (keys[i] == ~0ull) break;
        if (ou) ou[m] = pf::key_uid(keys[i]);
        if (os) os[m] = pf::key_score(keys[i]);
        ++m;
    }
    if (count) *count = m;
}

int pf_layout(const pf_ctx* c, pf_layout_stats* o) {
    if (!c || !o) return PF_EINVAL;
    o->n_slots = c->hc.n;
    o->stream_bytes = c->stream_bytes;
    o->header_bytes = (int64_t)c->hc.n * 48;
    o->alg_bytes = c->hs.alg_bytes;
    o->packed_tokens = c->hs.packed ? 1 : 0;
    o->n_tiles = (int32_t)c->hs.tile_steps.size();
    o->post_bytes = c->post_bytes;
    o->scan_kernel = c->use_post() ? PF_SCAN_POSTINGS : PF_SCAN_STREAM;
    o->pad = 0;
    o->shard_cands = 0;
    o->shard_entries = 0;
    if (c->use_post()) {
        const int64_t bs = c->ps.bsize, n = c->hc.n;
        const int64_t i0 = std::min<int64_t>(n, (int64_t)c->wb_begin * bs), i1 = std::min<int64_t>(n, (int64_t)c->wb_end * bs);
        const auto& hc = c->hc;
        o->shard_cands = i1 - i0;
        if (i1 > i0)
            o->shard_entries = (hc.tok_off[(size_t)i1 * hc.T] - hc.tok_off[(size_t)i0 * hc.T]) +
                               (hc.club_off[i1] - hc.club_off[i0]) + (hc.friend_off[i1] - hc.friend_off[i0]);
    } else {
        for (int32_t t = c->tile_begin; t < c->tile_end; ++t) {
            const int64_t s0 = c->hs.tile_slot0[t];
            const int64_t s1 = t + 1 < (int32_t)c->hs.tile_slot0.size() ? (int64_t)c->hs.tile_slot0[t + 1] : (int64_t)c->hc.n;
            o->shard_cands += s1 - s0;
        }
    }
    return PF_OK;
}

float pf_last_scan_ms(const pf_ctx* c) {
    if (!c) return 0.f;
    float ms = c->last_scan_ms;
    if (c->last_ev1 && hipEventSynchronize(c->last_ev1) == hipSuccess)
        (void)hipEventElapsedTime(&ms, c->last_ev0, c->last_ev1);
    return ms;
}

int pf_profile_reset(pf_ctx* c) {
    if (!c) return PF_EINVAL;
    c->prof_on = true;
    c->prof_used = 0;
    c->prof_seen = 0;
    c->last_ev0 = c->last_ev1 = nullptr;  // pool events are re-recorded from here on
    return PF_OK;
}

int pf_profile_sample(pf_ctx* c, int32_t every) {
    if (!c || every < 0) return PF_EINVAL;
    if (every == 0) {  // profiling off: launches use the context's own event pair again
        c->prof_on = false;
        c->prof_used = 0;
        c->last_ev0 = c->last_ev1 = nullptr;
        return PF_OK;
    }
    c->prof_every = every;
    return PF_OK;
}

int pf_profile_read(pf_ctx* c, double* total_ms, int64_t* launches) {
    if (!c || !total_ms || !launches) return PF_EINVAL;
    double tot = 0.0;
    for (size_t i = 0; i < c->prof_used; ++i) {
        HIPCHK(c, hipEventSynchronize(c->prof_ev[i].second));
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->prof_ev[i].first, c->prof_ev[i].second));
        tot += ms;
    }
    *total_ms = tot;
    *launches = (int64_t)c->prof_used;
    return PF_OK;
}

}  // extern "C"
