// pf_batch.h — engine-internal batched recommenders (pf_api.cpp) for the C ABI entry points
// and the batched hold-out drivers (pf_dataset.cpp).  Not part of the public ABI.
#pragma once
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdint>
#include <unordered_map>
#include <utility>
#include <functional>
#include <vector>

struct pf_ctx;

namespace pf {

// The adjacency one query sees (adj_list with edits), without copying it:
//   own_row: this query's own row replaced (recommendation_tests.cpp:111-114, a fresh copy
//            per user);
//   over:    rows edited by earlier users of a cumulative test, each visible to queries whose
//            version is >= the edit's (test.cpp:35,73, one adj_mod for the whole run).
struct AdjView {
    const std::unordered_map<int32_t, std::vector<int32_t>>* base = nullptr;
    const std::unordered_map<int32_t, std::pair<int32_t, std::vector<int32_t>>>* over = nullptr;
    int32_t version = 0;
    int32_t own = INT32_MIN;
    const std::vector<int32_t>* own_row = nullptr;
    const std::vector<int32_t>* row(int32_t v) const {
        if (own_row && v == own) return own_row;
        if (over) {
            auto it = over->find(v);
            if (it != over->end() && it->second.first <= version) return &it->second.second;
        }
        auto it = base->find(v);
        return it == base->end() ? nullptr : &it->second;
    }
};

enum JobKind { kJobInterest = 0, kJobCollab = 1, kJobClubs = 2 };

// One recommender call: recommend_by_interest (FoF-limited, or every candidate when
// all_candidates), recommend_collaborative or recommend_clubs_collab for uid under view.
struct Job {
    int kind = kJobInterest;
    int32_t uid = 0, topk = 0, limit = 0;
    int32_t limit_flavour = 0;  // pf_fof_candidates only: PF_FOF_GRAPH / PF_FOF_COLLAB
    bool all_candidates = false;
    AdjView view;
    std::vector<std::pair<int32_t, float>> out;  // ranked (id, score), <= topk
};

// Host-side stage clocks of the batched drivers (PF_DEBUG host_prof=1: summed over the process and
// printed to stderr at exit; profiling only).
enum HostStage {
    kHpPlan = 0, kHpPrep, kHpImages, kHpPack, kHpGpu, kHpUnpack, kHpStage2, kHpCollab, kHpFinish,
    kHpScanImage, kHpScanLaunch, kHpScanCalls, kHpScanStageWait, kHpStages  // (the scans' stages: pf_api.cpp scan_all)
};
struct HostProf {
    bool on = false;
    std::atomic<long long> ns[kHpStages];
    HostProf();
    ~HostProf();
};
HostProf& host_prof();
// lap(st): the time since the last lap (or construction) goes to stage st; skip(): dropped
struct HpLap {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(int st) {
        const auto n = std::chrono::steady_clock::now();
        HostProf& h = host_prof();
        if (h.on) h.ns[st] += std::chrono::duration_cast<std::chrono::nanoseconds>(n - t).count();
        t = n;
    }
    void skip() { t = std::chrono::steady_clock::now(); }
};

// Runs every job on the device job pipeline (pf_jobs_plan.cpp): one chain of device stages per
// chunk of jobs.  0 = OK, else a PF_* status.
int run_jobs(pf_ctx* c, std::vector<Job>& jobs);
// run_jobs leaving the last chunk on the device as the context's carried call (pf_jobs_plan.cpp):
// done(jobs) runs when it is finished (by carry_wait, the next job call, or any drain)
int run_jobs_carry(pf_ctx* c, std::vector<Job>&& jobs, uint64_t ticket, std::function<void(std::vector<Job>&)> done);
// the carried call with this ticket (or earlier) finished; its status
int carry_wait(pf_ctx* c, uint64_t ticket);
// a ticket of the context's asynchronous calls (pf_wait completes every call up to it)
uint64_t next_call_ticket(pf_ctx* c);
// A batched driver call (its versioned edit set) starts or ends (pf_jobs_plan.cpp).
void jobs_view_scope(pf_ctx* c);
const std::unordered_map<int32_t, std::vector<int32_t>>& base_adj(const pf_ctx* c);

}  // namespace pf
