// pf_idf.hip — F3: the corpus statistics in front of the path, on the device.
//
//   df per (column, tid)   Recommender::compute_idf_from_profiles (recommender.cpp:43-66):
//                          df = #profiles whose column map holds the tid (tf 0 included).
//                          Every token's key (column << 32 | tid) is written by a row kernel,
//                          radix-sorted (hipCUB onesweep) and run-length encoded: the runs are
//                          the distinct (column, tid) pairs, their lengths the df.  Any int tid
//                          works, negative ones included (the reference keys unordered_map<int,int>).
//   tid ranks              the rest of the engine sees each tid as its rank among the column's
//                          distinct tids (order kept; only equality and the idf lookup depend
//                          on the id), so every device layout has dense ids.
//   idf                    logf(1 + N / (1 + df)) in float32 on the host, over the distinct pairs
//                          only (~10^5 logf calls): glibc's logf, so the bits are the reference's;
//                          or the caller's map (set_tfidf_index), 1.0 for an absent tid.
//   candidate norms        sqrt(sum (tf * idf)^2) per (user, column) row, in the row's tid order
//                          (recommender.cpp:74-90), one thread per row, in the pass that finds
//                          each token's rank by bisection in its column's segment of the sorted
//                          key table; idf 1.0 for a column without an idf map (A7).  FP64 with
//                          no FMA contraction (-ffp-contract=off): each step rounds as on the host.
// The normaliser statistic (utils.cpp:155-240) stays on the host: its mt19937 pair sampler walks
// the profiles map in hash order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "pf_store.h"

namespace pf {

namespace {

constexpr int kIdfThreads = 256;
constexpr int kKeyBits = 32 + 6;  // tid (any 32-bit value) + column (< kMaxCols = 48 < 64)
static_assert(kMaxCols <= 64, "column fits 6 key bits");

// (column, tid) key; the tid biased by 2^31 so the keys' unsigned order is the tids' signed order
// (ranks then follow each row's ascending-tid order)
__host__ __device__ __forceinline__ uint64_t col_key(int col, int32_t tid) {
    return ((uint64_t)(uint32_t)col << 32) | ((uint32_t)tid ^ 0x80000000u);
}

// keys[k] = (column, tid) of token k; rows r = user * T + column
__global__ __launch_bounds__(kIdfThreads) void idf_keys_kernel(const int64_t* __restrict__ tok_off,
                                                               const int32_t* __restrict__ tid, int64_t rows, int T,
                                                               uint64_t* __restrict__ keys) {
    for (int64_t r = (int64_t)blockIdx.x * kIdfThreads + threadIdx.x; r < rows; r += (int64_t)gridDim.x * kIdfThreads) {
        const int col = (int)(r % T);
        for (int64_t k = tok_off[r]; k < tok_off[r + 1]; ++k) keys[k] = col_key(col, tid[k]);
    }
}

// Per row r (= user * T + column), in the row's token order: the token's index x in the sorted
// distinct (column, tid) table (bisection in the column's segment seg[c] .. seg[c + 1]); its
// column rank x - seg[c] replaces the tid; and sqrt_nb[r] = sqrt(sum ((double)tf * idf)^2)
// with idf = tab_idf[x] (has_idf[c] = 0: 1.0 for the whole column, raw counts, A7).
__global__ __launch_bounds__(kIdfThreads) void idf_norms_kernel(const int64_t* __restrict__ tok_off,
                                                                int32_t* __restrict__ tid,
                                                                const int32_t* __restrict__ tf, int64_t rows, int T,
                                                                const uint64_t* __restrict__ tab_key,
                                                                const float* __restrict__ tab_idf,
                                                                const int64_t* __restrict__ seg,
                                                                const uint8_t* __restrict__ has_idf,
                                                                double* __restrict__ sqrt_nb) {
    for (int64_t r = (int64_t)blockIdx.x * kIdfThreads + threadIdx.x; r < rows; r += (int64_t)gridDim.x * kIdfThreads) {
        const int col = (int)(r % T);
        const bool hi = has_idf[col] != 0;
        const int64_t s0 = seg[col], s1 = seg[col + 1];
        double nb = 0.0;
        for (int64_t k = tok_off[r]; k < tok_off[r + 1]; ++k) {
            const uint64_t key = col_key(col, tid[k]);
            int64_t lo = s0, up = s1;  // first entry >= key (the key is always present)
            while (lo < up) {
                const int64_t mid = (lo + up) >> 1;
                if (tab_key[mid] < key) lo = mid + 1;
                else up = mid;
            }
            tid[k] = (int32_t)(lo - s0);
            const double idf = hi ? (double)tab_idf[lo] : 1.0;
            const double w = (double)tf[k] * idf;
            nb += w * w;
        }
        sqrt_nb[r] = sqrt(nb);
    }
}

template <class T>
struct Dev {
    T* p = nullptr;
    ~Dev() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)); }
};

int grid_for(int64_t rows) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((rows + kIdfThreads - 1) / kIdfThreads, 65536));
}

}  // namespace

#define F3CHK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            err = std::string("F3 (df / ranks / norms on the device): ") + #x + ": " + \
                  hipGetErrorString(e_);                                      \
            (void)hipStreamDestroy(s);                                        \
            return e_ == hipErrorOutOfMemory ? PF_ENOMEM : PF_ENODEV;         \
        }                                                                     \
    } while (0)

int device_idf_norms(HostCorpus& hc, bool from_profiles, std::string& err) {
    const int64_t rows = (int64_t)hc.n * hc.T;
    const int64_t nt = hc.tok_off.empty() ? 0 : hc.tok_off.back();
    const int T = hc.T;
    hc.sqrt_nb.resize_uninit((size_t)rows);  // the device writes every row
    if (rows == 0) return PF_OK;
    if (nt > (int64_t)INT32_MAX) { err = "more than 2^31 tokens"; return PF_EUNSUPP; }
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { err = "F3 stream"; return PF_ENODEV; }
    Dev<int64_t> d_off;
    Dev<int32_t> d_tid, d_tf;
    F3CHK(d_off.alloc((size_t)rows + 1));
    F3CHK(d_tid.alloc((size_t)nt));
    F3CHK(d_tf.alloc((size_t)nt));
    F3CHK(hipMemcpyAsync(d_off.p, hc.tok_off.data(), ((size_t)rows + 1) * 8, hipMemcpyHostToDevice, s));
    if (nt > 0) {
        F3CHK(hipMemcpyAsync(d_tid.p, hc.tid.data(), (size_t)nt * 4, hipMemcpyHostToDevice, s));
        F3CHK(hipMemcpyAsync(d_tf.p, hc.tf.data(), (size_t)nt * 4, hipMemcpyHostToDevice, s));
    }
    // ---- the corpus's distinct (column, tid) keys (sorted) and their df, on the device
    std::vector<uint64_t> tab_key;
    std::vector<int32_t> cnt;
    if (nt > 0) {
        Dev<uint64_t> d_keys, d_sorted, d_uniq;
        Dev<int32_t> d_cnt, d_nruns;
        F3CHK(d_keys.alloc((size_t)nt));
        F3CHK(d_sorted.alloc((size_t)nt));
        F3CHK(d_uniq.alloc((size_t)nt));
        F3CHK(d_cnt.alloc((size_t)nt));
        F3CHK(d_nruns.alloc(1));
        hipLaunchKernelGGL(idf_keys_kernel, dim3(grid_for(rows)), dim3(kIdfThreads), 0, s, d_off.p, d_tid.p, rows, T,
                           d_keys.p);
        F3CHK(hipGetLastError());
        size_t b1 = 0, b2 = 0;
        F3CHK(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, d_keys.p, d_sorted.p, (int)nt, 0, kKeyBits, s));
        F3CHK(hipcub::DeviceRunLengthEncode::Encode(nullptr, b2, d_sorted.p, d_uniq.p, d_cnt.p, d_nruns.p, (int)nt, s));
        Dev<uint8_t> d_tmp;
        F3CHK(d_tmp.alloc(std::max(b1, b2)));
        size_t bt = std::max(b1, b2);
        F3CHK(hipcub::DeviceRadixSort::SortKeys(d_tmp.p, bt, d_keys.p, d_sorted.p, (int)nt, 0, kKeyBits, s));
        bt = std::max(b1, b2);
        F3CHK(hipcub::DeviceRunLengthEncode::Encode(d_tmp.p, bt, d_sorted.p, d_uniq.p, d_cnt.p, d_nruns.p, (int)nt, s));
        int32_t nruns = 0;
        F3CHK(hipMemcpyAsync(&nruns, d_nruns.p, 4, hipMemcpyDeviceToHost, s));
        F3CHK(hipStreamSynchronize(s));
        cnt.resize((size_t)nruns);
        tab_key.resize((size_t)nruns);
        F3CHK(hipMemcpyAsync(tab_key.data(), d_uniq.p, (size_t)nruns * 8, hipMemcpyDeviceToHost, s));
        F3CHK(hipMemcpyAsync(cnt.data(), d_cnt.p, (size_t)nruns * 4, hipMemcpyDeviceToHost, s));
        F3CHK(hipStreamSynchronize(s));
    }
    // column segments of the sorted table; rank = index - segment start
    std::vector<int64_t> seg((size_t)T + 1, 0);
    {
        size_t i = 0;
        for (int t = 0; t < T; ++t) {
            seg[t] = (int64_t)i;
            while (i < tab_key.size() && (int)(tab_key[i] >> 32) == t) ++i;
        }
        seg[T] = (int64_t)tab_key.size();
    }
    // ---- idf per distinct key: recommender.cpp:56-64 logf(1 + N / (1 + df)) in float32 over
    // the profiles (N = profiles loaded), or the caller's map (set_tfidf_index; absent -> 1.0,
    // recommender.cpp:78); by rank on the host
    std::vector<float> tab_idf(tab_key.size(), 1.0f);
    const float N = (float)hc.n;
    hc.tid_of_rank.assign(T, {});
    for (int t = 0; t < T; ++t) {
        const int64_t b = seg[t], e = seg[t + 1];
        auto& ids = hc.tid_of_rank[t];
        ids.resize((size_t)(e - b));
        for (int64_t i = b; i < e; ++i) ids[i - b] = (int32_t)((uint32_t)tab_key[i] ^ 0x80000000u);
        if (!hc.has_idf[t]) continue;
        auto& ex = hc.idf_explicit[t];
        for (int64_t i = b; i < e; ++i) {
            if (from_profiles) {
                tab_idf[i] = logf(1.0f + N / (1.0f + (float)cnt[i]));
            } else {
                auto it = ex.find(ids[i - b]);
                if (it != ex.end()) {
                    tab_idf[i] = it->second;
                    ex.erase(it);  // what remains names ids the corpus does not hold
                }
            }
        }
        hc.idf[t].assign(tab_idf.begin() + b, tab_idf.begin() + e);
    }
    // ---- norms
    Dev<uint64_t> d_tk;
    Dev<float> d_ti;
    Dev<int64_t> d_seg;
    Dev<uint8_t> d_has;
    Dev<double> d_nb;
    F3CHK(d_tk.alloc(tab_key.size()));
    F3CHK(d_ti.alloc(tab_idf.size()));
    F3CHK(d_seg.alloc(seg.size()));
    F3CHK(d_has.alloc((size_t)T));
    F3CHK(d_nb.alloc((size_t)rows));
    if (!tab_key.empty()) {
        F3CHK(hipMemcpyAsync(d_tk.p, tab_key.data(), tab_key.size() * 8, hipMemcpyHostToDevice, s));
        F3CHK(hipMemcpyAsync(d_ti.p, tab_idf.data(), tab_idf.size() * 4, hipMemcpyHostToDevice, s));
    }
    F3CHK(hipMemcpyAsync(d_seg.p, seg.data(), seg.size() * 8, hipMemcpyHostToDevice, s));
    F3CHK(hipMemcpyAsync(d_has.p, hc.has_idf.data(), (size_t)T, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(idf_norms_kernel, dim3(grid_for(rows)), dim3(kIdfThreads), 0, s, d_off.p, d_tid.p, d_tf.p, rows,
                       T, d_tk.p, d_ti.p, d_seg.p, d_has.p, d_nb.p);
    F3CHK(hipGetLastError());
    F3CHK(hipMemcpyAsync(hc.sqrt_nb.data(), d_nb.p, (size_t)rows * 8, hipMemcpyDeviceToHost, s));
    if (nt > 0) F3CHK(hipMemcpyAsync(hc.tid.data(), d_tid.p, (size_t)nt * 4, hipMemcpyDeviceToHost, s));
    F3CHK(hipStreamSynchronize(s));
    (void)hipStreamDestroy(s);
    return PF_OK;
}

}  // namespace pf
