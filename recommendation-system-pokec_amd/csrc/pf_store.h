// pf_store.h — host-side corpus model and device-layout builder.
#pragma once
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <cstdint>
#include <cstdlib>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "pf_types.h"

namespace pf {

// Host copy of the corpus in candidate-index order (idx = rank of uid,
// ascending, so idx order is the reference's tie-break order).
//
// Token ids: the caller's ids (any int, as the reference's unordered_map<int,int> keys) are
// replaced at open by their rank among the column's distinct ids (F3 on the device,
// pf_idf.hip).  Ranks keep the ids' order, and the path only compares ids for equality and
// looks up their idf, so every score is unchanged; the device layouts then see dense ids.
// A vector of trivially copyable T whose resize leaves the elements uninitialised: the store
// builders write every element (or fill them on threads), so the pages of these multi-GB
// arrays are first touched by the threads that write them, not by a serial value-initialisation.
template <class T>
class PodVec {
  public:
    using value_type = T;
    PodVec() = default;
    PodVec(const PodVec&) = delete;
    PodVec& operator=(const PodVec&) = delete;
    PodVec(PodVec&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
    PodVec& operator=(PodVec&& o) noexcept { swap(o); return *this; }
    ~PodVec() { std::free(p_); }
    // arrays of 32 MB and more sit on 2 MB pages where the kernel offers them (madvise mode of
    // transparent huge pages): 512x fewer first-touch faults, and unmapping them is cheap
    void resize_uninit(size_t n) {
        if (n == n_) return;
        std::free(p_);
        p_ = nullptr;
        n_ = 0;
        if (n == 0) return;
        const size_t bytes = n * sizeof(T);
        if (bytes >= (32u << 20)) {
            const size_t huge = 2u << 20, rounded = (bytes + huge - 1) & ~(huge - 1);
            void* q = nullptr;
            if (posix_memalign(&q, huge, rounded) == 0) {
                madvise(q, rounded, MADV_HUGEPAGE);  // advisory: ignored where THP is off
                p_ = static_cast<T*>(q);
            }
        } else {
            p_ = static_cast<T*>(std::malloc(bytes));
        }
        if (!p_) throw std::bad_alloc();
        n_ = n;
    }
    void clear() { std::free(p_); p_ = nullptr; n_ = 0; }
    void swap(PodVec& o) noexcept { std::swap(p_, o.p_); std::swap(n_, o.n_); }
    T* data() { return p_; }
    const T* data() const { return p_; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    T& operator[](size_t i) { return p_[i]; }
    const T& operator[](size_t i) const { return p_[i]; }
    const T& back() const { return p_[n_ - 1]; }
    T* begin() { return p_; }
    T* end() { return p_ + n_; }
    const T* begin() const { return p_; }
    const T* end() const { return p_ + n_; }

  private:
    T* p_ = nullptr;
    size_t n_ = 0;
};

struct HostCorpus {
    int32_t n = 0, T = 0;
    std::vector<int32_t> uid, pub, comp, gen, age, reg;  // reg: 3 per user
    std::vector<int64_t> club_off, friend_off;
    PodVec<int64_t> tok_off;                             // n*T+1, rows sorted by tid
    std::vector<uint32_t> clubs, friends;
    PodVec<int32_t> tid, tf;                             // tid: the column rank of the token id
    PodVec<double> sqrt_nb;                              // per (user, col) row
    std::vector<uint8_t> has_idf;                        // per column
    std::vector<std::vector<int32_t>> tid_of_rank;       // per column: the caller's id of each rank
    std::vector<std::vector<float>> idf;                 // per column, by rank (empty: no idf map)
    // PF_IDF_EXPLICIT: the caller's map per column; after open only its entries for ids the
    // corpus does not hold remain (pf_idf reports them, no score reads them)
    std::vector<std::unordered_map<int32_t, float>> idf_explicit;
    std::vector<uint8_t> npres;                          // 7 + T
    std::vector<float> nmean, nsd;
    std::unordered_map<int32_t, uint32_t> pub_code, gen_code;
    // live adjacency (adj_list), mutable through pf_set_adj
    std::unordered_map<int32_t, std::vector<int32_t>> adj;

    int32_t idx_of(int32_t u) const;   // -1 when uid has no profile
    float idf_of(int t, int32_t rank) const;     // idf of a rank; NaN if the column has no idf map
    float idf_of_tid(int t, int32_t tid) const;  // by the caller's id: 1.0 for an absent token
    int32_t n_ranks(int t) const { return (int32_t)tid_of_rank[t].size(); }
};

struct HostStore {
    PodVec<uint4> stream;
    std::vector<uint64_t> tile_off;
    std::vector<uint32_t> tile_steps;
    std::vector<uint32_t> tile_slot0;   // first slot of each tile
    std::vector<uint8_t> tile_lgk;      // log2 of the lanes per candidate (long records are split)
    std::vector<uint32_t> slot_tile;    // tile of each slot
    PodVec<double> norms;
    std::vector<uint64_t> norm_off;
    std::vector<uint4> hdr0, hdr1, hdr2;
    PodVec<uint4> rows;                 // row store: slot p's record at rows[row_off[p]], 16-B padded
    std::vector<uint64_t> row_off;      // [n + 1]
    std::vector<int32_t> slot_of_idx;
    std::vector<int32_t> idx_of_slot;
    bool packed = true;
    int64_t alg_bytes = 0;    // SURVEY 8(d) D3 accounting
};

// Query image (A side).  keys: tables T0..T3 (see pf_types.h); vals: token values.
struct QImageHost {
    QConst c;
    std::vector<uint64_t> keys;
    std::vector<QVal> vals;
};

// Postings store (K5, pf_types.h), built when the corpus fits its packed encoding.
struct HostPost {
    bool ok = false;
    std::string why;                                   // reason when !ok
    std::vector<uint4> hdr;                            // [2 * n]
    PodVec<uint32_t> post;                             // token lists, then club lists, then friend lists
    PodVec<double> pnorm;                              // [token entries]
    PodVec<uint32_t> cells;
    std::vector<PList> lists;
    std::vector<std::vector<int32_t>> tok_list;        // [col][tid] -> list (-1: none)
    std::unordered_map<uint32_t, int32_t> club_list, friend_list;
    int64_t tok_entries = 0;
};

int build_host_corpus(const pf_corpus_desc* d, HostCorpus& hc, std::string& err);
// F3 on the device (pf_idf.hip): the distinct (column, tid) pairs of the corpus (radix sort +
// run-length encoding); hc.tid rewritten as column ranks, hc.tid_of_rank; hc.idf by rank (with
// from_profiles: logf over df on the host; else from hc.idf_explicit, 1.0 for absent ids); then
// hc.sqrt_nb for every (user, column) row.  Needs the current HIP device; hc.has_idf (and,
// explicit mode, hc.idf_explicit) set by the caller.
int device_idf_norms(HostCorpus& hc, bool from_profiles, std::string& err);
// fills hp (hp.ok = false with hp.why when the corpus is outside the encoding)
void build_postings(const HostCorpus& hc, HostPost& hp);
// Postings query image of candidate idx (pf_types.h layout); excl = uids to exclude
void build_query_post(const HostCorpus& hc, const HostPost& hp, int32_t idx, const std::vector<int32_t>& excl,
                      std::vector<uint8_t>& img);
// The part of build_query_post's image after its QConst (offsets from the image start), into
// out[0, out_cap); returns its size (0: larger than out_cap).  post_part_bound(i, |excl|) bounds it.
size_t build_query_post_part(const HostCorpus& hc, const HostPost& hp, int32_t idx, const std::vector<int32_t>& excl,
                             uint8_t* out, size_t out_cap);
size_t post_part_bound(const HostCorpus& hc, int32_t idx, size_t n_excl);
int build_store(const HostCorpus& hc, HostStore& hs, std::string& err);
// excl: uids to exclude (all-candidates mode), may be null
// returns false when the cuckoo table cannot be built within kMaxHashLog2
bool build_query(const HostCorpus& hc, bool packed, int32_t idx, const std::vector<int32_t>* excl, QImageHost& out);

// exact reference arithmetic on the host (glibc exp)
double ref_sigmoid(double x);

// QConst in parts (pf_store.cpp fill_qconst; the device image builder K6 assembles the same):
// the query-independent fields, the region row of a query with a_regcnt parts, and the
// completion / age row [kValTab + 1] of query value a (zeros when a <= 0)
void qconst_template(const HostCorpus& hc, bool packed, QConst& c);
void qconst_sig_reg(const HostCorpus& hc, int a_regcnt, double out[4][4]);
void qconst_ratio_row(const HostCorpus& hc, int slot, int a, double* out);
// cuckoo table log2 for n items (load <= 0.4)
int lg_for(size_t n);

}  // namespace pf
