// pf_ctx.h — the engine context behind the C ABI (pf_api.cpp) and the device job pipeline
// (pf_jobs.cpp): device buffers, host corpus and stores, workspaces.  Engine-internal.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdlib>
#include <cstdint>
#include <deque>
#include <exception>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include <unistd.h>

#include "pf_batch.h"
#include "pf_jobs.h"
#include "pf_store.h"
#include "pokec_fas.h"

namespace pf {

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 4096);
        want = want + want / 4;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    // per-call workspaces: grow to twice the request (at least 1 MiB), so the sizes of
    // successive batches settle after a few calls instead of re-allocating (hipFree syncs)
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        return ensure(std::max<size_t>(2 * bytes, 1u << 20));
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

// Pinned host buffer that only grows (contents are not initialised)
struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 2, 1 << 20);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    ~PinBuf() {
        if (p) (void)hipHostFree(p);
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

using Ranked = std::vector<std::pair<int32_t, float>>;

inline void rank(Ranked& v, int topk) {  // recommender_graph.cpp:97-101
    std::sort(v.begin(), v.end(), [](const std::pair<int32_t, float>& a, const std::pair<int32_t, float>& b) {
        return a.second == b.second ? a.first < b.first : a.second > b.second;
    });
    if ((int)v.size() > topk) v.resize(std::max(topk, 0));
}


// workspace slots: two for a synchronous call's double-buffered chunks, all for asynchronous calls
// in flight (three, so the host plans two calls ahead of the device and a short call's pair
// kernel does not leave the device waiting for the next plan)
constexpr int kJobSlots = 3;

// The device job pipeline's state (pf_jobs.cpp): the graph and image-builder inputs on the
// device, their host mirrors, and the per-call workspaces.
struct JobsState {
    bool ok = false;
    std::string why;
    DevJobsStore js{};
    DBuf d_tmpl, d_sigreg, d_comp_vals, d_comp_rows, d_age_vals, d_age_rows,
        d_idf_doff, d_idf_dlen, d_idf_dense,
        d_slot_of, d_goff, d_glen, d_gnbr, d_guid, d_club_off, d_club_dense, d_club_id;
    std::unordered_map<int32_t, int32_t> xnode;  // uid -> node for adj_list uids without a profile
    std::vector<int32_t> dense_node;             // uid -> node (-1 none) when the uids are dense
    std::vector<int32_t> g_uid, g_len;           // host mirrors (new uids from pf_set_adj append nodes)
    bool nodes_dirty = false;
    std::vector<uint8_t> img_lg;                 // per idx: query-table log2 (0 = outside the device limits)
    std::vector<int32_t> img_nset;               // per idx: clubs + friends words of the record
    std::vector<uint32_t> img_rows;              // per idx: ImgJob::rows (its completion / age table rows)
    std::vector<uint32_t> img_stamp;             // per idx: the layout pass that last gave it an image ...
    std::vector<int32_t> img_pos;                // ... and that image's index (no hash map per call)
    uint32_t img_gen = 0;
    // resident query images (built at open, pf_jobs_plan.cpp build_resident_images): every user's
    // K6 image in one pool, so no call builds images; pimg_off[idx] = its byte offset (16-aligned)
    bool pimg = false;
    DBuf d_pimg;
    std::vector<int64_t> pimg_off;
    // a chunk's K3 gathers (+ the dispatch orders) run on aux beside its K6 images on the context's
    // stream (both latency-bound, independent), joined before the pair kernel
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // K4' (collaborative), K8, K7 (clubs) and a chunk's result copies run on aux2 after its pair
    // kernel (Ws::ev_pairs), beside the next chunk's pair kernel (pf_jobs_plan.cpp launch_chunk)
    hipStream_t aux2 = nullptr;
    int pp = 0;  // the last chunk's ping-pong stream (1: aux, 0: the context's; pf_jobs_plan.cpp launch_chunk)
    std::unordered_set<int32_t> edited;          // uids whose adj_list row differs from the open-time row
    // open-time row of each edited uid (present, row): an edit back to it drops the override
    std::unordered_map<int32_t, std::pair<bool, std::vector<int32_t>>> orig;
    uint64_t edit_gen = 1, view_gen = 0;         // the uploaded edit table is current when equal
    const void* view_over = nullptr;             // the batched drivers' versioned edits last uploaded
    size_t view_over_n = 0;
    bool view_has_over = false;                  // the uploaded table holds versioned edits
    uint64_t call_gen = 0, view_call = 0;        // batched driver calls (jobs_view_scope)
    DevView view{};
    DBuf d_view_node, d_view_ver, d_view_off, d_view_len, d_view_nbr;
    // per-chunk workspaces, double-buffered: chunk i + 1 is planned and launched while chunk i
    // runs (run_all in pf_jobs_plan.cpp).  Both slots queue on the context's stream: a stream per
    // slot, so that consecutive calls overlap on the device, measured slower (r3y: the pair kernel
    // 0.344 -> 0.385 ms beside the next call's images and gathers; cfg 3 1.93e9 -> 1.71e9).
    struct Ws {
        DBuf d_plan, d_ht, d_seq, d_slots, d_ids, d_fl, d_img, d_scr;  // d_plan: the plan, then the results
        DBuf d_acc;                // clubs accumulators (zero between uses)
        DBuf d_parts;              // K4''s per-block top-k lists (the fused collaborative top-k)
        int64_t acc_jobs = 0;      // clubs jobs the accumulators hold
        PinBuf h_plan, h_out;
        hipEvent_t done = nullptr;  // recorded after the chunk's result copies (on aux2)
        hipEvent_t ev_pairs = nullptr, ev_main = nullptr;  // the pair kernel queued on the context's stream / K4' + K8 there (collab_main=1)
        ~Ws() {
            if (done) (void)hipEventDestroy(done);
            if (ev_pairs) (void)hipEventDestroy(ev_pairs);
            if (ev_main) (void)hipEventDestroy(ev_main);
        }
        // what the chunk's unpack needs (host)
        bool active = false;
        std::vector<DevJob> dj;
        std::vector<int32_t> jmap, tpos;
        std::vector<size_t> full, full_off;
        size_t o_cnt = 0, o_keys = 0, o_fail = 0;
        int ktop = 1;
    } ws[kJobSlots];
    // asynchronous calls (pf_recommend_*_async): each holds one workspace slot from its launch
    // until pf_wait unpacks it, so at most kJobSlots are in flight; their jobs live here meanwhile
    struct Pending {
        uint64_t ticket = 0;
        int slot = 0;
        std::vector<Job> jobs;
        int32_t topk = 0;
        int32_t* ou = nullptr;
        float* os = nullptr;
        int32_t* oc = nullptr;
    };
    std::deque<Pending> pending;                 // launch order
    uint64_t next_ticket = 1;
    // A batched driver call whose last chunk is still on the device (pf_eval_recommendation_tests_async):
    // the next job call plans and launches its first chunk, then finishes this one (the chunk's
    // unpack and the driver's per-user results), so the host's planning of step i + 1 runs beside
    // the device's last chunk of step i.  Any other use of the pipeline finishes it first.
    struct Carry {
        bool on = false;
        int slot = 0;                                // the workspace its last chunk holds
        uint64_t ticket = 0;
        std::vector<Job> jobs;
        std::function<void(std::vector<Job>&)> done; // the driver's results from the finished jobs
    } carry;
    uint64_t carry_done = 0;                     // the last carried ticket finished
    // carried tickets that failed (an error drops the call's results), until pf_eval_wait reads them
    std::unordered_map<uint64_t, int> carry_fail;
    // pf_jobs_stats: pair counts / bytes (device counters) and pair-kernel time (HIP events)
    bool stats_on = false;                       // pair-kernel events (pf_jobs_stats_reset bit 0)
    bool stats_count = false;                    // pair counters (bit 1)
    DBuf d_stats;                                // 3 x u64: pairs, D3 bytes, tile-store bytes
    std::vector<std::pair<hipEvent_t, hipEvent_t>> stat_ev;
    size_t stat_used = 0;
    int64_t st_jobs = 0, st_cands = 0, st_img_bytes = 0, st_launches = 0;
    int64_t n_dispatch = 0;                      // K1' dispatches since open (pf_jobs_stats.pair_dispatches)
};

}  // namespace pf

using pf::DBuf;
using pf::PinBuf;

struct pf_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, last_ev0 = nullptr, last_ev1 = nullptr;
    float last_scan_ms = 0.f;
    std::string err;
    pf::HostCorpus hc;
    pf::HostStore hs;       // metadata only after upload (stream freed)
    int64_t stream_bytes = 0, norm_bytes = 0;
    DBuf d_stream, d_tile_off, d_tile_steps, d_tile_slot0, d_tile_lgk, d_slot_tile, d_norms, d_norm_off, d_hdr0, d_hdr1, d_hdr2,
        d_rowstore, d_rowstore_off;
    pf::DevStore ds{};
    // workspaces
    DBuf d_pool, d_refs, d_out, d_slots, d_blocks, d_scores, d_part;
    PinBuf h_pool, h_slots, h_scores;  // pf_fas_pairs batches: images, candidate slots, scores
    int32_t tile_begin = 0, tile_end = 0;
    // postings store (K5); wave blocks [wb_begin, wb_end) are this context's shard
    pf::HostPost hp;
    DBuf d_phdr, d_post, d_pnorm, d_cells;
    pf::PostStore ps{};
    int64_t post_bytes = 0;
    int32_t wb_begin = 0, wb_end = 0;
    int32_t scan_kind = PF_SCAN_AUTO;
    bool use_post() const { return hp.ok && scan_kind != PF_SCAN_STREAM; }
    // pinned staging ring for the per-call query upload (a slot is reused only after
    // the copy that read it has completed)
    struct Stage {
        uint8_t* p = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr;
    };
    Stage stage[4];
    int stage_cur = 0;
    uint8_t* stage_acquire(size_t bytes) {
        Stage& st = stage[stage_cur];
        if (st.done) (void)hipEventSynchronize(st.done);
        if (st.cap < bytes) {
            if (st.p) (void)hipHostFree(st.p);
            st.p = nullptr;
            st.cap = 0;
            size_t want = std::max<size_t>(bytes + bytes / 2, 1 << 16);
            if (hipHostMalloc((void**)&st.p, want, hipHostMallocDefault) != hipSuccess) return nullptr;
            st.cap = want;
        }
        return st.p;
    }
    hipError_t stage_release(hipStream_t s) {
        Stage& st = stage[stage_cur];
        stage_cur = (stage_cur + 1) % 4;
        if (!st.done) {
            hipError_t e = hipEventCreateWithFlags(&st.done, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        return hipEventRecord(st.done, s);
    }
    // Two scan lanes for single-query calls made on a caller's stream (pf_scan_keys_async): each
    // lane has its own stream, staging pool, merge parts and result rows, so query i + 1's upload
    // and launch need not wait for query i's launch to end: its workgroups fill the CUs that query
    // i's last blocks leave idle.  The caller's stream waits for a lane's launch and copies its
    // row out, in call order.  A lane's result rows are used in turn and one is rewritten only
    // after its copy (freed[r]): with one row per lane, the next launch waited on the copy-out,
    // a one-workgroup blit queued behind the running launch's workgroups (48-73 us, r8e trace).
    // The ring holds kLaneRows rows in kLaneGroups groups: the lane waits for a group's copies
    // (freed[g], recorded after the copy of its last row) only when it wraps back to it, so a
    // step costs no event pair of its own.
    static constexpr int kLaneRows = 32, kLaneGroups = 4, kLaneGroupRows = kLaneRows / kLaneGroups;
    struct ScanLane {
        hipStream_t st = nullptr;
        DBuf pool, part, keys;  // keys: kLaneRows rows of kMaxTopK keys
        DBuf sync;              // the resident one-query launches' ScanSync (zeroed once; K5 leaves it zeroed)
        hipEvent_t done = nullptr;  // the stop event of an untimed launch (bound to the kernel's dispatch)
        hipEvent_t freed[kLaneGroups] = {};
        bool used[kLaneGroups] = {};
        int row = 0;
    };
    // three by default (PF_DEBUG scan_lanes=N: 0 / 1 off, 2 without the aux2 stream); lanes past the
    // third run on streams of their own (lane_st, created at open when scan_lanes asks for them):
    // with the process's default four hardware queues they would share them (an A/B for processes
    // that raise GPU_MAX_HW_QUEUES; pf_api.cpp scan_lanes)
    static constexpr int kMaxLanes = 16;
    ScanLane lane[kMaxLanes];
    hipStream_t lane_st[kMaxLanes] = {};
    int lane_cur = 0;
    // Resident postings-scan images (pf_api.cpp build_resident_post): every user's K5 image part
    // after its QConst (QPostHead | tokens | columns | set lists | exclusions = adj_list row + self),
    // built once at open; a one-query scan launches from it with the QConst of the user's resident
    // K1' image (jb.d_pimg), so the call builds and uploads nothing.  A user whose adj_list row
    // pf_set_adj changed (its exclusions) takes the per-call image again (stale).
    struct ResidentPost {
        bool on = false;
        DBuf d_pool;
        std::vector<int64_t> off;        // per idx: byte offset of its part in d_pool
        std::vector<uint32_t> var_lds;   // per idx: post_var_lds of its image (0: no resident image)
        std::vector<uint8_t> stale;      // per idx: exclusions changed since open
        DBuf d_zero;                     // zero words: img_off / out_rows of a one-query launch
        DBuf d_sync;                     // ScanSync of a one-query launch on the context's own stream
    } rp;
    // scan-kernel timing pool (pf_profile_*)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev;
    size_t prof_used = 0;
    bool prof_on = false;
    int64_t prof_seen = 0;   // scan launches since the reset
    int32_t prof_every = 1;  // time launches 0, every, 2 every, ... (pf_profile_sample)

    pf::JobsState jb;  // device job pipeline (pf_jobs.cpp)

    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    int hip_fail(hipError_t e, const char* what) {
        err = std::string(what) + ": " + hipGetErrorString(e);
        return PF_ENODEV;
    }
};


namespace pf {

// A process-wide pool of worker threads (started on first use, never joined: they sleep on a
// condition variable) for the engine's host loops.  Several contexts may submit at once: a call
// posts its range, the workers and the caller take items from it through an atomic cursor, and the
// caller returns when every item is done.  (Spawning 16 std::threads per call cost ~0.5 ms per job
// chunk: three chunks per cfg-5 step.)
class WorkPool {
  public:
    // Leaked on purpose (workers outlive static destruction).  A process forked after first use
    // has no workers (only the forking thread survives a fork): it gets a pool of its own.
    static WorkPool& get() {
        static std::atomic<WorkPool*> pool{nullptr};
        static std::atomic<pid_t> owner{0};
        const pid_t me = getpid();
        WorkPool* w = pool.load(std::memory_order_acquire);
        if (w && owner.load(std::memory_order_relaxed) == me) return *w;
        static std::mutex gm;
        std::lock_guard<std::mutex> g(gm);
        w = pool.load(std::memory_order_acquire);
        if (!w || owner.load(std::memory_order_relaxed) != me) {
            w = new WorkPool();
            owner.store(me, std::memory_order_relaxed);
            pool.store(w, std::memory_order_release);
        }
        return *w;
    }
    int workers() const { return (int)ts_.size(); }
    // fn(i) for i in [0, n), on the caller and up to `helpers` workers
    void run(size_t n, size_t helpers, const std::function<void(size_t)>& fn) {
        Task t;
        t.fn = &fn;
        t.n = n;
        {
            std::lock_guard<std::mutex> g(mu_);
            t.slots = (int)helpers;
            q_.push_back(&t);
        }
        cv_.notify_all();
        work(t);
        {
            std::unique_lock<std::mutex> g(mu_);
            auto it = std::find(q_.begin(), q_.end(), &t);
            if (it != q_.end()) q_.erase(it);  // no further worker joins this task
        }
        std::unique_lock<std::mutex> g(t.m);
        t.cv.wait(g, [&] { return t.active == 0; });
        // every worker has left the task (it lives on this stack): only now rethrow an item's error
        if (t.err) std::rethrow_exception(t.err);
    }

  private:
    struct Task {
        const std::function<void(size_t)>* fn = nullptr;
        size_t n = 0;
        std::atomic<size_t> next{0};
        int slots = 0;   // workers that may still join (under mu_)
        int active = 0;  // workers inside (under m)
        std::exception_ptr err;  // the first item's exception (under m); the other items are skipped
        std::mutex m;
        std::condition_variable cv;
    };
    static void work(Task& t) {
        for (size_t i; (i = t.next.fetch_add(1)) < t.n;) {
            try {
                (*t.fn)(i);
            } catch (...) {
                std::lock_guard<std::mutex> g(t.m);
                if (!t.err) t.err = std::current_exception();
                t.next.store(t.n);
            }
        }
    }
    WorkPool() {
        const int n = (int)std::min<unsigned>(15u, std::max(1u, std::thread::hardware_concurrency()) - 1u);
        for (int w = 0; w < n; ++w) {
            ts_.emplace_back([this]() {
                for (;;) {
                    Task* t = nullptr;
                    {
                        std::unique_lock<std::mutex> g(mu_);
                        cv_.wait(g, [&] { return !q_.empty(); });
                        t = q_.front();
                        if (--t->slots <= 0) q_.pop_front();
                        std::lock_guard<std::mutex> g2(t->m);
                        ++t->active;  // registered before the caller can see the queue without it
                    }
                    work(*t);
                    std::lock_guard<std::mutex> g2(t->m);
                    if (--t->active == 0) t->cv.notify_all();
                }
            });
            ts_.back().detach();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Task*> q_;
    std::vector<std::thread> ts_;
};

// f(0 .. n-1) on up to 16 threads (the caller and pool workers), `grain` items per thread at least
// (the single-user calls of the sequential drivers stay on the caller's thread)
template <class F>
inline void par_jobs(size_t n, F f, size_t grain = 4) {
    const size_t th = std::min<size_t>(16, std::max<size_t>(1, std::min<size_t>(n / grain, std::thread::hardware_concurrency())));
    if (th <= 1) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    const std::function<void(size_t)> fn = [&](size_t i) { f(i); };
    WorkPool::get().run(n, th - 1, fn);
}


#define HIPCHK(ctx, expr)                                   \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return (ctx)->hip_fail(_e, #expr); \
    } while (0)

// A timing event of the profiling pools (pf_profile_*, the job statistics).  Created without
// the system-scope fence (hipEventDisableSystemFence): every read of these events follows a
// stream or device synchronisation, and the fence's L2 write-back and invalidation would
// otherwise run between the timed kernels and perturb them (r2fe: 1.6 us of kernel time).
inline hipError_t timing_event(hipEvent_t* e) { return hipEventCreateWithFlags(e, hipEventDisableSystemFence); }

template <class V>  // std::vector or PodVec
inline hipError_t upload(pf_ctx* c, DBuf& b, const V& v) {
    using T = typename V::value_type;
    hipError_t e = b.ensure(std::max<size_t>(v.size() * sizeof(T), 16));
    if (e != hipSuccess) return e;
    if (v.empty()) return hipSuccess;
    return hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream);
}


// the device job pipeline (pf_jobs.cpp)
int jobs_open(pf_ctx* c);                            // after the tile store is on the device
int jobs_set_adj(pf_ctx* c, int32_t uid, const int32_t* nbrs, int32_t n);  // pf_set_adj
int run_jobs_async(pf_ctx* c, std::vector<Job>&& jobs, int32_t topk, int32_t* ou, float* os, int32_t* oc,
                   uint64_t* ticket);                // pf_recommend_*_async
int jobs_wait(pf_ctx* c, uint64_t ticket);           // pf_wait
int jobs_drain(pf_ctx* c);                           // every pending asynchronous call unpacked
int fof_device(pf_ctx* c, int32_t uid, int32_t limit, int32_t flavour, std::vector<int32_t>& out);
int jobs_stats_reset(pf_ctx* c, int enable);
int jobs_stats_read(pf_ctx* c, pf_jobs_stats* o);

}  // namespace pf
