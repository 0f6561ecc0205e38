// pf_jobs.hip — gfx950 kernels of the device job pipeline (pf_types.h DevJob): the reference's
// graph / collaborative / clubs recommenders with the 2-hop work on the device.
//
//   gather_kernel   K3  per job: the ordered, de-duplicated, limit-truncated 2-hop candidate
//                       list over the CSR adjacency (recommender_graph.cpp:10-31 / :114-125),
//                       filtered like the recommender (no profile; row(u) + {u} for interest),
//                       as tile-store slots for the pair kernel; clubs: each friend's row
//   qimage_kernel   K6  per user: the query image the pair kernel stages (pf_store.cpp
//                       build_query's layout): QConst from host-built tables + a 2-choice cuckoo
//                       table of the user's distinct clubs, friends and (column, token) words
//   collab_kernel   K4' score(c) = sum over row(u) positions of (double)FAS(u,f) * FAS(f,c)
//                       (recommender_graph.cpp:167-180), in the reference's order
//   clubs_kernel    K7  club scores in recommender_clubs.cpp:34-66's loop order (per club the
//                       double sum is taken in exactly the reference's sequence)
//   topk_kernel     K8  per job top-k of (score desc, id asc) (recommender_graph.cpp:97-101)
//
// Order-preserving de-duplication (K3): the sequence the reference walks (friend f, then f's
// row, for each friend in order) is processed in 256-element chunks; each element claims its
// node in a per-job open-addressing table and atomicMin's its position there, so after a
// barrier an element is a first occurrence iff the table holds its own position (earlier
// chunks hold smaller positions).  A block prefix sum over the first occurrences places them,
// and the walk stops once `limit` have been found: exactly the reference's truncation.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "pf_device.h"
#include "pf_jobs.h"

namespace pf {

constexpr int kJobThreads = 256;
constexpr int kJobWaves = kJobThreads / 64;
// K3 walks a job's 2-hop sequence in chunks of one workgroup's width: 1024 threads per job
// (a hub's sequence of 40,000 elements is 40 chunks with 4 barriers each instead of 160)
constexpr int kGatherThreads = 1024;
constexpr int kGatherWaves = kGatherThreads / 64;

// ---------------------------------------------------------------- block helpers
// exclusive rank of `flag` among the block's threads and the block total (ballots + LDS)
template <int NW = kJobWaves>
__device__ __forceinline__ int block_rank(bool flag, int* wsum, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = __ballot(flag);
    const int r = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const int x = wsum[w];
        if (w < wave) before += x;
        total += x;
    }
    __syncthreads();
    return before + r;
}

// block_rank for two flags per thread whose items are ordered all-f0-items first (thread order),
// then all f1-items: one LDS exchange (wsum holds 2 * NW words)
template <int NW>
__device__ __forceinline__ void block_rank2(bool f0, bool f1, int* wsum, int& r0, int& r1, int& t0, int& t1) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m0 = __ballot(f0), m1 = __ballot(f1);
    const uint64_t below = (1ull << lane) - 1ull;
    r0 = __popcll(m0 & below);
    r1 = __popcll(m1 & below);
    if (lane == 0) {
        wsum[wave] = __popcll(m0);
        wsum[NW + wave] = __popcll(m1);
    }
    __syncthreads();
    int b0 = 0, b1 = 0;
    t0 = t1 = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const int x0 = wsum[w], x1 = wsum[NW + w];
        if (w < wave) { b0 += x0; b1 += x1; }
        t0 += x0;
        t1 += x1;
    }
    __syncthreads();
    r0 += b0;
    r1 += t0 + b1;
}

// inclusive prefix of v over the block; total in `total`
template <int NW = kJobWaves>
__device__ __forceinline__ int block_scan_incl(int v, int* wsum, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
    x = (int)wave_incl_scan((uint32_t)x);
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const int t = wsum[w];
        if (w < wave) before += t;
        total += t;
    }
    __syncthreads();
    return before + x;
}

// ---------------------------------------------------------------- adjacency under a view
// Row of node x for job J: the job's own row, then the newest visible override, then the
// base CSR.  Returns a pointer to the row's nodes, len = -1 when x has no adj_list row.
__device__ __forceinline__ const int32_t* row_of(const DevJobsStore& g, const DevView& v, const DevJob& J,
                                                 const int32_t* pool, int32_t x, int32_t& len) {
    if (x == J.own) {  // the job's own row lives in the plan pool
        len = J.own_len;
        return pool + J.own_off;
    }
    if (v.n > 0) {
        int lo = 0, hi = v.n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (v.node[mid] < x) lo = mid + 1; else hi = mid;
        }
        for (int i = lo; i < v.n && v.node[i] == x; ++i)
            if (v.ver[i] <= J.version) {
                len = v.len[i];
                return v.nbr + v.off[i];
            }
    }
    if (x < 0 || x >= g.M) {
        len = -1;
        return g.g_nbr;
    }
    len = g.g_len[x];
    return g.g_nbr + g.g_off[x];
}

// ---------------------------------------------------------------- K3: gather
__device__ __forceinline__ uint32_t node_hash(int32_t x) { return (uint32_t)x * 0x9E3779B1u; }

// slot of node x in the job's table (claimed if absent); keys hold node + 1, 0 = empty
__device__ __forceinline__ uint32_t ht_claim(int32_t* keys, uint32_t mask, int32_t x) {
    uint32_t h = (node_hash(x) >> 7) & mask;
    for (;;) {
        const int32_t old = atomicCAS(&keys[h], 0, x + 1);
        if (old == 0 || old == x + 1) return h;
        h = (h + 1) & mask;
    }
}

// Length class of a slot (< 232 for any int32 slot, monotone): slots are assigned longest
// record first, so small slots are the long records, whose lengths spread the most (the synthetic
// D1 corpus: slot 0 holds 2,155 words, slot 1,600 ~430, the median 125).  Classes 0..7 are slots
// 0..7, then eight classes per power of two of the slot (its top four bits).
__device__ __forceinline__ int slot_class(int32_t sl) {
    if (sl < 8) return sl;
    const int lg = 31 - __clz(sl);  // >= 3
    return 8 + ((lg - 3) << 3) + ((sl >> (lg - 3)) & 7);
}

// one workgroup per job
__global__ __launch_bounds__(kGatherThreads) void gather_kernel(DevJobsStore g, DevView vw, const DevJob* __restrict__ jobs,
                                                             const int32_t* __restrict__ pool, int32_t* __restrict__ ht,
                                                             int32_t* __restrict__ seq, int32_t* __restrict__ cand_slot,
                                                             int32_t* __restrict__ cand_id, int32_t* __restrict__ ncand,
                                                             const int64_t* __restrict__ pool64) {
    __shared__ int wsum[2 * kGatherWaves];
    __shared__ int s_count, s_keep, s_done;
    const DevJob J = jobs[blockIdx.x];
    const int tid = threadIdx.x;
    const int32_t u = J.u;
    const int32_t* frow = pool + J.f_off;
    int32_t* slots = cand_slot + J.cand_off;
    int32_t* ids = cand_id + J.cand_off;

    if (J.kind == kDjCollab || J.kind == kDjClubs) {  // the pairs (u, f) of sim_u_f
        const int32_t* fd = pool + J.fd_off;
        for (int r = tid; r < J.nfd; r += kGatherThreads) cand_slot[J.sim_off + r] = g.slot_of[fd[r]];
    }
    if (J.kind == kDjClubs) {
        // recommender_clubs.cpp:47-58: each distinct friend's row, fof != u with a profile
        const int32_t* fd = pool + J.fd_off;
        const int64_t* sreg = pool64 + J.sreg_off;
        for (int r = 0; r < J.nfd; ++r) {
            int32_t len;
            const int32_t* row = row_of(g, vw, J, pool, fd[r], len);
            for (int k = tid; k < len; k += kGatherThreads) {
                const int32_t x = row[k];
                cand_slot[sreg[r] + k] = (x != u && x >= 0 && x < g.n) ? g.slot_of[x] : -1;
            }
        }
        return;
    }

    const uint32_t cap = 1u << J.ht_lg, mask = cap - 1u;
    int32_t* keys = ht + J.ht_off;
    int32_t* pos = keys + cap;
    int32_t* flag = pos + cap;
    for (uint32_t i = tid; i < cap; i += kGatherThreads) {
        keys[i] = 0;
        pos[i] = INT_MAX;
        flag[i] = 0;
    }
    __syncthreads();
    const bool interest = J.kind == kDjInterest || J.kind == kDjAll;
    if (interest) {  // recommender_graph.cpp:46-52: existing = adj[u] + {u}
        for (int j = tid; j <= J.nf; j += kGatherThreads) {
            const int32_t x = j < J.nf ? frow[j] : u;
            __hip_atomic_store(&flag[ht_claim(keys, mask, x)], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();

    if (J.kind == kDjAll) {  // every profile but the excluded ones, in idx order
        for (int32_t i = tid; i < J.cap; i += kGatherThreads) {
            bool ex = false;
            uint32_t h = (node_hash(i) >> 7) & mask;
            for (;;) {
                const int32_t k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (k == 0) break;
                if (k == i + 1) {
                    ex = __hip_atomic_load(&flag[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    break;
                }
                h = (h + 1) & mask;
            }
            slots[i] = ex ? -1 : g.slot_of[i];
            ids[i] = ex ? -1 : g.g_uid[i];
        }
        if (tid == 0) ncand[blockIdx.x] = J.cap;
        return;
    }

    const bool graph = J.kind == kDjInterest || J.kind == kDjRawGraph;
    const bool raw = J.kind == kDjRawGraph || J.kind == kDjRawCollab;
    // segment lengths: graph = [f, row(f)...] unless f == u (skipped whole, :18); collab =
    // row(f) when f has one (:116-118)
    int32_t* seg = seq + J.seg_off;  // [nf + 1] exclusive prefix
    if (tid == 0) s_count = 0;
    {
        int carry = 0;
        for (int b = 0; b < J.nf; b += kGatherThreads) {
            const int j = b + tid;
            int len = 0;
            if (j < J.nf) {
                const int32_t f = frow[j];
                int32_t rl;
                row_of(g, vw, J, pool, f, rl);
                if (graph) len = f == u ? 0 : 1 + (rl > 0 ? rl : 0);
                else len = rl > 0 ? rl : 0;
            }
            int tot;
            const int incl = block_scan_incl<kGatherWaves>(len, wsum, tot);
            if (j < J.nf) seg[j] = carry + incl - len;
            carry += tot;
        }
        if (tid == 0) seg[J.nf] = carry;
    }
    __syncthreads();
    const int total = seg[J.nf];
    if (tid == 0) {
        s_count = 0;
        s_keep = 0;
        s_done = 0;
    }
    __syncthreads();
    // two sequence elements per thread per round (positions base + tid and base + 1024 + tid): a
    // round's table claims go out together and its ranks take one exchange per flag pair
    auto element = [&](int p) -> int32_t {
        if (p >= total) return -1;
        int lo = 0, hi = J.nf;  // last friend j with seg[j] <= p
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (seg[mid] <= p) lo = mid; else hi = mid;
        }
        const int32_t f = frow[lo];
        const int k = p - seg[lo];
        int32_t x;
        if (graph && k == 0) x = f;
        else {
            int32_t rl;
            const int32_t* row = row_of(g, vw, J, pool, f, rl);
            x = row[graph ? k - 1 : k];
        }
        return x == u ? -1 : x;  // :22 / :120
    };
    for (int base = 0; base < total; base += 2 * kGatherThreads) {
        const int p0 = base + tid, p1 = base + kGatherThreads + tid;
        const int32_t x0 = element(p0), x1 = element(p1);
        uint32_t h0 = 0, h1 = 0;
        if (x0 >= 0) h0 = ht_claim(keys, mask, x0);
        if (x1 >= 0) h1 = ht_claim(keys, mask, x1);
        if (x0 >= 0) atomicMin(&pos[h0], p0);
        if (x1 >= 0) atomicMin(&pos[h1], p1);
        __syncthreads();
        // the table lives at L2 (device-scope atomics): read it past the CU's L1
        const bool first0 = x0 >= 0 && __hip_atomic_load(&pos[h0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p0;
        const bool first1 = x1 >= 0 && __hip_atomic_load(&pos[h1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p1;
        int rf0, rf1, nf0, nf1;
        block_rank2<kGatherWaves>(first0, first1, wsum, rf0, rf1, nf0, nf1);
        const int cnt = s_count;
        auto kept = [&](bool first, int rf, int32_t x, uint32_t h) {
            bool keep = first && cnt + rf < J.L;
            if (!raw) {
                if (interest)  // :46-54
                    keep = keep && __hip_atomic_load(&flag[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && x < g.n;
                else keep = keep && x < g.n;                           // :167-170
            }
            return keep;
        };
        const bool keep0 = kept(first0, rf0, x0, h0), keep1 = kept(first1, rf1, x1, h1);
        int rk0, rk1, nk0, nk1;
        block_rank2<kGatherWaves>(keep0, keep1, wsum, rk0, rk1, nk0, nk1);
        const int kb = s_keep;
        if (keep0) {
            slots[kb + rk0] = raw ? 0 : g.slot_of[x0];
            ids[kb + rk0] = g.g_uid[x0];
        }
        if (keep1) {
            slots[kb + rk1] = raw ? 0 : g.slot_of[x1];
            ids[kb + rk1] = g.g_uid[x1];
        }
        __syncthreads();
        if (tid == 0) {
            s_count = cnt + nf0 + nf1;
            s_keep = kb + nk0 + nk1;
        }
        __syncthreads();
        if (s_count >= J.L) break;
    }
    const int nk = s_keep;
    // The scored candidates grouped by length class (slot_class), longest first, so the pair
    // kernel's 64-lane waves walk records of similar length instead of waiting on the longest of
    // 64 random ones: a counting sort into 256 buckets through the (finished) hash table's memory.  The order is free:
    // every later stage keeps slot, id and score together, and the top-k's total order does not
    // depend on it.  (Raw lists keep the reference's order.)
    if (!raw && nk > 64) {
        __shared__ int hist[256];
        int2* tmp = reinterpret_cast<int2*>(keys);  // 3 << ht_lg words >= 2 * nk
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < nk; i += kGatherThreads) atomicAdd(&hist[slot_class(slots[i])], 1);
        __syncthreads();
        if (tid < 64) {  // exclusive scan of 256 counts by one wave
            int v[4], t = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) { v[k] = hist[tid * 4 + k]; t += v[k]; }
            int x = t;
            x = (int)wave_incl_scan((uint32_t)x);
            int run = x - t;
#pragma unroll
            for (int k = 0; k < 4; ++k) { hist[tid * 4 + k] = run; run += v[k]; }
        }
        __syncthreads();
        for (int i = tid; i < nk; i += kGatherThreads) {
            const int32_t sl = slots[i];
            tmp[atomicAdd(&hist[slot_class(sl)], 1)] = make_int2(sl, ids[i]);
        }
        __syncthreads();
        for (int i = tid; i < nk; i += kGatherThreads) {
            const int2 e = tmp[i];
            slots[i] = e.x;
            ids[i] = e.y;
        }
    }
    for (int i = nk + tid; i < J.cap; i += kGatherThreads) {
        slots[i] = -1;
        ids[i] = -1;
    }
    if (tid == 0) ncand[blockIdx.x] = nk;
}

// ---------------------------------------------------------------- pair-block dispatch order
// The pair kernel's blocks longest work first: a block's key is the record length class of its
// first candidate (K3 lists a job's candidates longest first, in slot buckets; slots are
// assigned longest record first, pf_store.cpp build_store), so the blocks holding the few
// hub-length records (up to ~17x the mean) start in the first resident round instead of
// trailing the launch.  One workgroup, a counting sort over 256 slot buckets (+ one for blocks
// without a candidate, last); the order within a bucket is free (each block writes its own
// outputs).
constexpr int kOrderThreads = 1024;

__global__ __launch_bounds__(kOrderThreads) void order_pairs_kernel(const PairBlock* __restrict__ blocks, int nblocks,
                                                                    const int32_t* __restrict__ slots,
                                                                    int32_t* __restrict__ order) {
    __shared__ int hist[258];
    const int tid = threadIdx.x;
    for (int i = tid; i < 258; i += kOrderThreads) hist[i] = 0;
    __syncthreads();
    auto key = [&](int b) {
        const int32_t s0 = slots[blocks[b].begin];
        return s0 < 0 ? 256 : slot_class(s0);
    };
    // a thread's first 8 blocks: keys loaded together and kept (the rest recomputed)
    constexpr int kKeep = 8;
    int kk[kKeep];
#pragma unroll
    for (int u = 0; u < kKeep; ++u) {
        const int b = tid + u * kOrderThreads;
        kk[u] = b < nblocks ? key(b) : -1;
    }
#pragma unroll
    for (int u = 0; u < kKeep; ++u)
        if (kk[u] >= 0) atomicAdd(&hist[kk[u] + 1], 1);
    for (int b = tid + kKeep * kOrderThreads; b < nblocks; b += kOrderThreads) atomicAdd(&hist[key(b) + 1], 1);
    __syncthreads();
    if (tid < 64) {  // exclusive positions of the 257 buckets: hist[k] = first position of bucket k
        int v[5], t = 0;
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const int i = tid * 5 + u;
            v[u] = i < 258 ? hist[i] : 0;
            t += v[u];
        }
        int x = t;
        x = (int)wave_incl_scan((uint32_t)x);
        int run = x - t;
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const int i = tid * 5 + u;
            run += v[u];
            if (i < 258) hist[i] = run;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kKeep; ++u)
        if (kk[u] >= 0) order[atomicAdd(&hist[kk[u]], 1)] = tid + u * kOrderThreads;
    for (int b = tid + kKeep * kOrderThreads; b < nblocks; b += kOrderThreads) order[atomicAdd(&hist[key(b)], 1)] = b;
}

// ---------------------------------------------------------------- K6: query images
__device__ __forceinline__ int find_val(const int32_t* vals, int n, int32_t v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (vals[mid] < v) lo = mid + 1; else hi = mid;
    }
    return (lo < n && vals[lo] == v) ? lo : -1;
}

// float idf of (column t, tid rank) as the reference reads it (recommender.cpp:78; a column
// without an idf map: 1.0, the raw-count cosine A7)
__device__ __forceinline__ double idf_of(const DevJobsStore& g, int t, int32_t tid) {
    const int64_t d = g.idf_dense_off[t];
    if (d < 0) return 1.0;
    return (tid >= 0 && tid < g.idf_dense_len[t]) ? (double)g.idf_dense[d + tid] : 1.0;
}

// One workgroup per image: QConst | table (ntab << lg, then 2^lge exclusions) | vals.
// LDS = true (the common case, table + set + item list <= kImgLds): the de-duplication set, the
// item list and the cuckoo table live in LDS (ds_ atomics) and the table is copied out at the
// end; LDS = false (hub users): the same in global memory (the image's own table and scratch).
constexpr uint32_t kImgLds = 48 * 1024;

template <bool PACKED, bool LDS>
__global__ __launch_bounds__(kJobThreads) void qimage_kernel(DevStore st, DevJobsStore g, const ImgJob* __restrict__ ij,
                                                             uint8_t* __restrict__ pool, uint32_t* __restrict__ scratch,
                                                             int32_t* __restrict__ fail) {
    __shared__ int s_fail, s_nuniq;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const ImgJob I = ij[blockIdx.x];
    const int tid = threadIdx.x;
    const int p = g.slot_of[I.idx];
    const uint4 h0 = st.hdr0[p], h1 = st.hdr1[p], h2 = st.hdr2[p];
    QConst* q = reinterpret_cast<QConst*>(pool + I.const_off);
    // 1. constants: the template, then this user's fields (pf_store.cpp fill_qconst)
    {
        const uint4* src = reinterpret_cast<const uint4*>(g.tmpl);
        uint4* dst = reinterpret_cast<uint4*>(q);
        for (uint32_t i = tid; i < sizeof(QConst) / 16; i += kJobThreads) dst[i] = src[i];
    }
    __syncthreads();
    const int32_t comp = (int32_t)h0.z, age = (int32_t)h0.w;
    const int32_t reg0 = (int32_t)h1.x, reg1 = (int32_t)h1.y, reg2 = (int32_t)h1.z;
    const int a_regcnt = (reg0 >= 0) + (reg1 >= 0) + (reg2 >= 0);
    const uint64_t colmask = (uint64_t)h0.x | ((uint64_t)h0.y << 32);
    // the completion / age rows, looked up on the host (a device bisection is 7 dependent loads)
    const bool rows16 = I.rows != 0xFFFFFFFFu;
    const int ci = comp > 0 ? (rows16 ? (int)(I.rows & 0xFFFFu) - 1 : find_val(g.comp_vals, g.n_comp, comp)) : -1;
    const int ai = age > 0 ? (rows16 ? (int)(I.rows >> 16) - 1 : find_val(g.age_vals, g.n_age, age)) : -1;
    for (int v = tid; v <= kValTab; v += kJobThreads) {
        q->sig_comp[v] = ci >= 0 ? g.comp_rows[(size_t)ci * (kValTab + 1) + v] : 0.0;
        q->sig_age[v] = ai >= 0 ? g.age_rows[(size_t)ai * (kValTab + 1) + v] : 0.0;
    }
    if (tid < 16) q->sig_reg[tid >> 2][tid & 3] = a_regcnt > 0 ? g.sig_reg[a_regcnt * 16 + tid] : 0.0;
    // the user's record and column norms from the row store (contiguous; the tile store strides a
    // record's 16-B steps 1 KiB apart)
    const uint64_t ro = st.row_off[p];
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(st.rows + ro);
    const double* rn = reinterpret_cast<const double*>(st.rows + ro + ((record_words(h2, PACKED) + 3) >> 2));
    for (int t = tid; t < kMaxCols; t += kJobThreads)
        q->sqrt_na[t] = (t < q->n_cols && ((colmask >> t) & 1ull)) ? rn[__popcll(colmask & ((1ull << t) - 1ull))] : 0.0;
    const uint32_t nc = h2.y, nf = h2.z, ntok = h2.w;
    if (tid == 0) {
        q->colmask = colmask;
        q->comp = comp;
        q->age = age;
        q->reg[0] = reg0;
        q->reg[1] = reg1;
        q->reg[2] = reg2;
        q->a_regcnt = a_regcnt;
        q->pubcode = h2.x & 0xFFu;
        q->gencode = (h2.x >> 8) & 0xFFu;
        q->n_clubs = (int32_t)nc;
        q->n_friends = (int32_t)nf;
        q->sqrt_clubs = sqrt((double)nc);
        q->sqrt_friends = sqrt((double)nf);
        q->n_vals = (int32_t)ntok;
        q->lg = I.lg;
        q->lg_excl = I.lge;
        q->excl_off = (uint32_t)((PACKED ? 1u : 3u) << I.lg);
        s_fail = 0;
        s_nuniq = 0;
    }
    // 2. the record's words once (tokens: their value entries, vi = token rank, recommender.cpp:74-85)
    const uint32_t len = record_words(h2, PACKED);
    const uint32_t nset = nc + nf;
    const int lg = I.lg;
    const uint32_t ntab = PACKED ? 1u : 3u;
    const uint32_t tab_total = (ntab << lg) + (1u << I.lge);
    const uint32_t dmask = (1u << I.dlg) - 1u;
    // carve: table (8-B entries) | item list (8 B each) | set (4 B each)
    uint64_t* tab;
    uint64_t* items;
    uint32_t* dset;
    if constexpr (LDS) {
        tab = reinterpret_cast<uint64_t*>(smem);
        items = tab + tab_total;
        dset = reinterpret_cast<uint32_t*>(items + nset + ntok);
    } else {
        tab = reinterpret_cast<uint64_t*>(pool + I.keys_off);
        dset = scratch + I.scr_off;
        items = reinterpret_cast<uint64_t*>(scratch + I.scr_off + (1u << I.dlg));
    }
    QVal* vals = reinterpret_cast<QVal*>(pool + I.vals_off);
    for (uint32_t i = tid; i <= dmask; i += kJobThreads) dset[i] = 0u;
    __syncthreads();
    for (uint32_t k = tid; k < ntok; k += kJobThreads) {
        int t;
        int32_t tid_, tf;
        uint64_t e;
        if (PACKED) {
            const uint32_t w = rw[nset + k];
            t = (int)((w >> kTidBits) & 63u);
            tid_ = (int32_t)(w & kTidMask);
            tf = (int32_t)(w >> 24);
            e = make_entry(kTagTok | ((uint32_t)t << kTidBits) | (w & kTidMask), kTokVal | k | ((uint32_t)t << kTidBits));
        } else {
            const uint32_t w0 = rw[nset + 2 * k];  // tid | col << 26
            tid_ = (int32_t)(w0 & kWideTidMask);
            const uint32_t w = rw[nset + 2 * k + 1];
            t = (int)(w & 0xFFu);
            tf = (int32_t)w >> 8;
            e = make_entry(w0, (uint32_t)t | (k << 8)) | (2ull << 62);
        }
        const double idf = idf_of(g, t, tid_);
        QVal v;
        v.wq = (double)tf * idf;
        v.idf = idf;
        vals[k] = v;
        items[nset + k] = e;  // tokens are distinct (column, tid) pairs
    }
    // 3. distinct clubs / friends: a thread owns a word it claims first in the set; items
    //    [0, nuniq) are the sets, [nset, nset + ntok) the tokens
    for (uint32_t j = tid; j < nset; j += kJobThreads) {
        const uint32_t w = rw[j];
        const bool club = j < nc;
        const uint32_t id = PACKED ? (club ? (w & ~kTagClub) : w) : w;
        const uint32_t key = (id + 1u) | (club ? 0u : 0x80000000u);
        uint32_t h = (node_hash((int32_t)key) >> 5) & dmask;
        bool won = false;
        for (;;) {
            const uint32_t old = atomicCAS(&dset[h], 0u, key);
            if (old == 0u) { won = true; break; }
            if (old == key) break;
            h = (h + 1u) & dmask;
        }
        if (won) {
            uint64_t e;
            if (PACKED) e = club ? make_entry(id | kTagClub, 1u) : make_entry(id, 0x10000u);
            else e = make_entry(id, 0u) | ((uint64_t)(club ? 0u : 1u) << 62);  // table choice in bit 62 (val 0)
            items[atomicAdd(&s_nuniq, 1)] = e;
        }
    }
    __syncthreads();
    const uint32_t nuniq = (uint32_t)s_nuniq;
    // 4. 2-choice cuckoo (pf_store.cpp cuckoo_fill): parallel insertion with atomic exchange;
    //    a chain longer than 500 kicks fails the attempt, the next multiplier is tried
    const uint64_t empty = PACKED ? kEmptyEntryPacked : kEmptyEntry;
    for (uint32_t s = 0; s < 16; ++s) {
        const uint32_t hmul = kHashMul + 2u * s * 0x6A09E667u;
        for (uint32_t i = tid; i < tab_total; i += kJobThreads) tab[i] = empty;
        __syncthreads();
        for (uint32_t i = tid; i < nuniq + ntok; i += kJobThreads) {
            uint64_t cur = items[i < nuniq ? i : nset + (i - nuniq)];
            const uint32_t tsel = PACKED ? 0u : (uint32_t)(cur >> 62);
            cur &= PACKED ? ~0ull : ~(3ull << 62);
            uint64_t* T = tab + ((size_t)tsel << lg);
            uint32_t x = cuckoo_x((uint32_t)cur, hmul);
            uint32_t at = cuckoo_h1(x, lg);
            bool placed = false;
            for (int kick = 0; kick < 500; ++kick) {
                const uint64_t old = (uint64_t)atomicExch(reinterpret_cast<unsigned long long*>(&T[at]),
                                                          (unsigned long long)cur);
                if (old == empty) { placed = true; break; }
                cur = old;  // evicted: to its other slot
                x = cuckoo_x((uint32_t)cur, hmul);
                const uint32_t a = cuckoo_h1(x, lg), b = cuckoo_h2(x, lg);
                at = at == a ? b : a;
            }
            if (!placed) atomicOr(&s_fail, 1);
        }
        __syncthreads();
        const int failed = s_fail;
        __syncthreads();
        if (!failed) {
            if (tid == 0) q->hmul = hmul;
            // out SoA per table (pf_types.h soa_words); a global build goes through the scratch
            // after its item list (the table's own bytes are the destination)
            uint32_t* out = reinterpret_cast<uint32_t*>(pool + I.keys_off);
            const uint64_t* src = tab;
            if constexpr (!LDS) {
                uint64_t* tmp = items + nset + ntok;
                for (uint32_t i = tid; i < tab_total; i += kJobThreads) tmp[i] = tab[i];
                __syncthreads();
                src = tmp;
            }
            const uint32_t excl = ntab << lg;
            for (uint32_t i = tid; i < tab_total; i += kJobThreads) {
                uint32_t kw, vw;
                soa_words(i, excl, lg, I.lge, kw, vw);
                const uint64_t e = src[i];
                out[kw] = (uint32_t)e;
                out[vw] = (uint32_t)(e >> 32);
            }
            return;
        }
        if (tid == 0) s_fail = 0;
        __syncthreads();
    }
    if (tid == 0) atomicOr(fail, 1);
}

// LDS bytes of an image's build (table + item list + set), pf_jobs_plan.cpp splits the launch by it
uint32_t qimage_lds(int lg, int lge, int dlg, uint32_t nitems, bool packed) {
    const uint64_t b = 8ull * (((uint64_t)(packed ? 1 : 3) << lg) + (1ull << lge)) + 8ull * nitems + 4ull * (1ull << dlg);
    return b <= kImgLds ? (uint32_t)b : 0u;
}

// ---------------------------------------------------------------- K4': collaborative sums
// recommender_graph.cpp:167-180: for each candidate, sum over friend-list positions (in order,
// duplicates included) of (double)sim_u_f * (double)FAS(f, c); friends without a profile skip
// A workgroup takes 64 candidates of one job; its four waves compute the products of a tile of
// 64 friend positions (16 each, loads in flight together) into LDS, then wave 0 adds them per
// candidate in position order.  A hub's long friend row costs one memory round trip per 64
// positions over four waves instead of one per few positions on a single lane.
// A job with topk <= kMaxTopK also gets its top-k here (K8's keys, K8 skips the job): each block
// publishes the k best keys of its 64 candidates (write-through stores, post_tail's hand-off),
// takes a ticket, and the job's last block merges every block's list into out[jn * k ..].
constexpr int kCollabCands = 64, kCollabTile = 64;

__device__ __forceinline__ void st_agent64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kJobThreads) void collab_kernel(const DevJob* __restrict__ jobs, const int32_t* __restrict__ jix,
                                                             const int32_t* __restrict__ pool, const float* __restrict__ pout,
                                                             const int32_t* __restrict__ cand_slot, float* __restrict__ score,
                                                             const int32_t* __restrict__ ids, uint64_t* __restrict__ parts,
                                                             unsigned int* __restrict__ tickets, uint64_t* __restrict__ out,
                                                             int k) {
    static_assert(kJobThreads == 4 * kCollabCands && kCollabTile % 4 == 0, "four waves of 64 candidates");
    __shared__ double P[kCollabTile][kCollabCands];
    const DevJob J = jobs[jix[blockIdx.y]];
    const int c0 = (int)blockIdx.x * kCollabCands;
    if (c0 >= J.cap) return;
    const int cl = (int)(threadIdx.x & 63u), g = (int)(threadIdx.x >> 6);
    const int c = c0 + cl;
    const bool live = c < J.cap && cand_slot[J.cand_off + c] >= 0;
    const int32_t* fpos = pool + J.fpos_off;
    const float* sim = pout + J.sim_off;
    const float* M = pout + J.m_off;
    constexpr int U = kCollabTile / 4;
    double s = 0.0;
    for (int j0 = 0; j0 < J.nf; j0 += kCollabTile) {
        const int nj = min(kCollabTile, J.nf - j0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int jj = g * U + u;
            if (jj < nj) {
                const int r = fpos[j0 + jj];
                P[jj][cl] = (r >= 0 && c < J.cap) ? (double)sim[r] * (double)M[(size_t)r * J.cap + c] : 0.0;
            }
        }
        __syncthreads();
        if (g == 0 && live)
            for (int jj = 0; jj < nj; ++jj)
                if (fpos[j0 + jj] >= 0) s += P[jj][cl];  // friends without a profile are skipped
        __syncthreads();
    }
    if (g == 0 && live) score[J.out_off + c] = (float)s;
    if (J.topk > kMaxTopK || g != 0) return;  // K8 ranks this job (or another wave's work is done)
    // the fused top-k (wave 0): score_key as K8 builds it from the stored float and the id
    const int jn = jix[blockIdx.y];
    uint64_t list = ~0ull;
    topk_push(list, live ? score_key((float)s, ids[J.out_off + c]) : ~0ull, k, cl);
    const int nb = (J.cap + kCollabCands - 1) / kCollabCands;
    uint64_t* jp = parts + (size_t)blockIdx.y * gridDim.x * k;
    // Hand-off (pf_device.h take_ticket): ONE wave stores its list sc1 and waits for the stores,
    // its lane 0 takes an agent-scope ticket, and the block whose ticket came last reads every list
    // with sc1 loads in that same wave after the ticket returned.  Under the default
    // PF_TICKET_MODE 0 the ticket is relaxed with no fence: the hand-off rests on the hardware's
    // issue order (the stores drained before the ticket issues, the reads data-dependent on its
    // return) and the sc1 write-through, not on the HIP memory model; a compiler or ISA scheduling
    // change could break it.  PF_TICKET_MODE 1 (release ticket + acquire fence) is the
    // model-correct form, built and run by tests/gpu_variant_check.py.
    if (cl < k) st_agent64(jp + (size_t)blockIdx.x * k + cl, list);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    unsigned t = 0;
    if (cl == 0) t = take_ticket(&tickets[blockIdx.y]);
    t = (unsigned)__shfl((int)t, 0);
    if (t != (unsigned)nb - 1u) return;
    ticket_acquire();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    uint64_t acc = ~0ull;
    const int n = nb * k;
    for (int b = 0; b < n; b += 64) topk_push(acc, b + cl < n ? ld_agent64(jp + b + cl) : ~0ull, k, cl);
    if (cl < k) out[(size_t)jn * k + cl] = acc;
}

// ---------------------------------------------------------------- K7: clubs
// recommender_clubs.cpp:34-66: club_scores[c] += ... in the reference's sequence.  One wave per
// job.  The contribution stream (phase 1: friends in order, each friend's clubs in order;
// phase 2: friends in order, their rows in order, each fof's clubs in order) is generated 64
// stream items at a time, one per lane, into an LDS buffer in sequence order (a prefix sum of
// the lanes' club counts places them); the buffer is then bucketed, stably, by owner lane
// (dense club index % 64), and every lane adds its own bucket in order.  A club's
// contributions all go to one lane and keep their sequence order, so each club's double sum
// is the reference's.  acc[d] == 0.0 marks an untouched club (every contribution is > 0).
constexpr int kClubBuf = 512;  // contributions per round (LDS: 2 x 12 B each)

__device__ __forceinline__ int wave_excl_prefix(int x, int lane, int& total) {
    int v = x;
    v = (int)wave_incl_scan((uint32_t)v);
    total = (int)wave_last((uint32_t)v);
    return v - x;
}

__global__ __launch_bounds__(64) void clubs_kernel(DevJobsStore g, DevView vw, const DevJob* __restrict__ jobs,
                                                   const int32_t* __restrict__ jix, const int32_t* __restrict__ pool,
                                                   const int64_t* __restrict__ pool64, const float* __restrict__ pout,
                                                   double* __restrict__ acc_all, float* __restrict__ score, int32_t* __restrict__ ids,
                                                   int32_t* __restrict__ ncand, int64_t acc_stride) {
    const int slot = blockIdx.x;
    const DevJob J = jobs[jix[slot]];
    const int lane = threadIdx.x;
    double* acc = acc_all + (size_t)slot * acc_stride;     // dense club scores (zero between jobs)
    __shared__ int s_n;
    if (lane == 0) s_n = 0;
    __syncthreads();
    const int32_t u = J.u;
    const int32_t* frow = pool + J.f_off;
    const int32_t* fpos = pool + J.fpos_off;
    const float* sim = pout + J.sim_off;
    const int64_t* sreg = pool64 + J.sreg_off;
    const int64_t uc0 = g.club_off[u], uc1 = g.club_off[u + 1];
    auto own_club = [&](int32_t d) {  // user_clubs (the query's clubs)
        for (int64_t k = uc0; k < uc1; ++k)
            if (g.club_dense[k] == d) return true;
        return false;
    };
    int32_t* list = ids + J.out_off;  // dense indices of the touched clubs
    __shared__ int32_t bd[kClubBuf];  // a round's contributions in sequence order (-1: own club)
    __shared__ double bv[kClubBuf];
    __shared__ int32_t sd[kClubBuf];  // the same bucketed by owner lane, stable
    __shared__ double sv[kClubBuf];
    const uint64_t lt = (1ull << lane) - 1ull;
    // one stream item per lane: weight v for the clubs club_dense[cb .. ce) (nothing if !valid)
    auto chunk = [&](bool valid, double v, int64_t cb, int64_t ce) {
        const int nc = valid ? (int)(ce - cb) : 0;
        int total;
        const int pre = wave_excl_prefix(nc, lane, total);
        for (int r0 = 0; r0 < total; r0 += kClubBuf) {
            const int T = min(total - r0, kClubBuf);
            for (int i = max(pre, r0); i < min(pre + nc, r0 + T); ++i) {
                const int32_t d = g.club_dense[cb + (i - pre)];
                bd[i - r0] = own_club(d) ? -1 : d;
                bv[i - r0] = v;
            }
            __syncthreads();
            // bucket sizes: lane b counts the contributions of bucket b
            int cnt = 0;
            for (int i0 = 0; i0 < T; i0 += 64) {
                const int i = i0 + lane;
                const int d = i < T ? bd[i] : -1;
                uint64_t mine = __ballot(d >= 0);
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const uint64_t B = __ballot((d >> j) & 1);
                    mine &= ((lane >> j) & 1) ? B : ~B;
                }
                cnt += __popcll(mine);
            }
            int placed;
            const int base = wave_excl_prefix(cnt, lane, placed);
            // stable placement: a contribution goes after the earlier ones of its bucket
            int fill = base;
            for (int i0 = 0; i0 < T; i0 += 64) {
                const int i = i0 + lane;
                const int d = i < T ? bd[i] : -1;
                const uint64_t V = __ballot(d >= 0);
                uint64_t peers = V, mine = V;
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const uint64_t B = __ballot((d >> j) & 1);
                    peers &= ((d >> j) & 1) ? B : ~B;
                    mine &= ((lane >> j) & 1) ? B : ~B;
                }
                const int at = __shfl(fill, d & 63) + __popcll(peers & lt);
                if (d >= 0) {
                    sd[at] = d;
                    sv[at] = bv[i];
                }
                fill += __popcll(mine);
            }
            __syncthreads();
            // every lane adds its bucket in order; a run of one club stays in a register
            for (int m = base; m < base + cnt;) {
                const int32_t d = sd[m];
                double a = acc[d];
                if (a == 0.0) list[atomicAdd(&s_n, 1)] = d;
                a += sv[m++];
                while (m < base + cnt && sd[m] == d) a += sv[m++];
                acc[d] = a;
            }
            __syncthreads();
        }
    };
    // phase 1 (:34-44): friends in order, w > 0, their clubs not in user_clubs
    for (int j0 = 0; j0 < J.nf; j0 += 64) {
        const int j = j0 + lane;
        bool ok = false;
        double w = 0.0;
        int64_t cb = 0, ce = 0;
        if (j < J.nf) {
            const int r = fpos[j];
            if (r >= 0) {
                w = (double)sim[r];
                if (!(w <= 0.0)) {  // the serial walk's test, NaN included
                    const int32_t f = frow[j];
                    cb = g.club_off[f];
                    ce = g.club_off[f + 1];
                    ok = true;
                }
            }
        }
        chunk(ok, w, cb, ce);
    }
    // phase 2 (:46-66): friends in order with a row, a profile and w > 0; fof in row order.
    // 64 friends at a time: their rows flattened into one stream (a prefix of the row
    // lengths), 64 items per chunk, so short rows share chunks.
    __shared__ int32_t f_off[64];
    __shared__ const int32_t* f_row[64];
    __shared__ const float* f_S[64];
    __shared__ double f_w[64];
    for (int j0 = 0; j0 < J.nf; j0 += 64) {
        const int j = j0 + lane;
        int32_t len = 0;
        const int32_t* row = nullptr;
        const float* S = nullptr;
        double w = 0.0;
        if (j < J.nf) {
            const int r = fpos[j];
            if (r >= 0) {
                int32_t l;
                const int32_t* rw = row_of(g, vw, J, pool, frow[j], l);
                if (l >= 0) {
                    w = (double)sim[r];
                    if (!(w <= 0.0)) {
                        len = l;
                        row = rw;
                        S = pout + sreg[r];
                    }
                }
            }
        }
        int total;
        const int off = wave_excl_prefix(len, lane, total);
        f_off[lane] = off;
        f_row[lane] = row;
        f_S[lane] = S;
        f_w[lane] = w;
        __syncthreads();
        for (int t0 = 0; t0 < total; t0 += 64) {
            const int t = t0 + lane;
            bool ok = false;
            double contrib = 0.0;
            int64_t cb = 0, ce = 0;
            if (t < total) {
                // the friend whose row holds item t: the last one starting at or before t
                // (friends without items start where the next one does, so they are passed over)
                int fi = 0;
#pragma unroll
                for (int h = 32; h > 0; h >>= 1)
                    if (f_off[fi + h] <= t) fi += h;
                const int k = t - f_off[fi];
                const int32_t x = f_row[fi][k];
                if (x != u && x >= 0 && x < g.n) {
                    const double sx = (double)f_S[fi][k];
                    if (!(sx <= 0.0)) {
                        contrib = f_w[fi] * sx;
                        cb = g.club_off[x];
                        ce = g.club_off[x + 1];
                        ok = true;
                    }
                }
            }
            chunk(ok, contrib, cb, ce);
        }
        __syncthreads();
    }
    __syncthreads();
    const int n = s_n;
    for (int i = lane; i < n; i += 64) {
        const int32_t d = list[i];
        score[J.out_off + i] = (float)acc[d];
        acc[d] = 0.0;
        list[i] = g.club_id[d];
    }
    if (lane == 0) ncand[jix[slot]] = n;
}

// ---------------------------------------------------------------- K8: top-k
// per job: the k smallest keys of (score desc, id asc) over its scored list (ids < 0 skipped)
// (user candidates: the slot >= 0 marks a scored pair; clubs: the first ncand entries)
__global__ __launch_bounds__(kJobThreads) void topk_kernel(const DevJob* __restrict__ jobs, const int32_t* __restrict__ jix,
                                                           const float* __restrict__ score, const int32_t* __restrict__ ids,
                                                           const int32_t* __restrict__ slots,
                                                           const int32_t* __restrict__ ncand, uint64_t* __restrict__ out,
                                                           int k) {
    __shared__ uint64_t sc[kJobWaves * kMaxTopK];
    const int jn = jix[blockIdx.x];
    const DevJob J = jobs[jn];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = ncand[jn];
    const int lim = J.kind == kDjClubs ? n : J.cap;
    uint64_t list = ~0ull;
    for (int b = wave * 64; b < lim; b += kJobThreads) {
        const int i = b + lane;
        uint64_t key = ~0ull;
        if (i < lim) {
            if (J.kind == kDjClubs || slots[J.out_off + i] >= 0) key = score_key(score[J.out_off + i], ids[J.out_off + i]);
        }
        topk_push(list, key, k, lane);
    }
    if (lane < k) sc[wave * k + lane] = list;
    __syncthreads();
    if (wave == 0) {
        uint64_t acc = ~0ull;
        const int m = kJobWaves * k;
        for (int b = 0; b < m; b += 64) topk_push(acc, b + lane < m ? sc[b + lane] : ~0ull, k, lane);
        if (lane < k) out[(size_t)jn * k + lane] = acc;
    }
}

// ---------------------------------------------------------------- pair statistics
// (pf_jobs_stats) per scored pair: 1, SURVEY 8(d) D3's b_c of the candidate, and the bytes the
// pair-scoring stage reads / writes for it by access pattern:
// 48-B headers + 8-B row offset + its record words (K1' walks the pair's record).
template <bool PACKED>
__global__ __launch_bounds__(256) void pair_stats_kernel(DevStore st, const PairBlock* __restrict__ blocks,
                                                         const int32_t* __restrict__ slots,
                                                         unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long red[3][4];
    const PairBlock b = blocks[blockIdx.x];
    const int i = threadIdx.x;
    unsigned long long v[3] = {0ull, 0ull, 0ull};
    for (int x = i; x < b.count; x += 256) {
        const int p = slots[b.begin + x];
        if (p >= 0) {
            const uint4 h2 = st.hdr2[p];
            const unsigned long long rec = 4ull * record_words(h2, PACKED);
            v[0] += 1ull;
            v[1] += 32ull + 4ull * (h2.y + h2.z) + 8ull * h2.w;
            v[2] += 56ull + rec;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        unsigned long long x = v[k];
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, o);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), o);
            x += ((unsigned long long)hi << 32) | lo;
        }
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x < 3) {  // one atomic per counter and block
        const unsigned long long t = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
        if (t) atomicAdd(&acc[threadIdx.x], t);
    }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_pair_stats(const DevStore& st, const PairBlock* blocks, int nblocks, const int32_t* slots,
                             unsigned long long* acc, hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
    if (st.packed)
        hipLaunchKernelGGL(pair_stats_kernel<true>, dim3(nblocks), dim3(256), 0, s, st, blocks, slots, acc);
    else
        hipLaunchKernelGGL(pair_stats_kernel<false>, dim3(nblocks), dim3(256), 0, s, st, blocks, slots, acc);
    return hipGetLastError();
}

// K9: the pair blocks of a chunk from its runs (PairGen), one thread per block; the run by a
// bisection of the runs' first blocks (ascending)
__global__ __launch_bounds__(256) void expand_pairs_kernel(const PairGen* __restrict__ gens, int ngens,
                                                           const int2* __restrict__ pool, int nblocks,
                                                           PairBlock* __restrict__ blocks) {
    const int b = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (b >= nblocks) return;
    int lo = 0, hi = ngens - 1;  // the last run with first <= b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (gens[mid].first <= b) lo = mid; else hi = mid - 1;
    }
    const PairGen g = gens[lo];
    const int loc = b - g.first, x = loc / g.nf, f = loc - x * g.nf;
    const int2 e = pool[g.fl + f];
    const int off = x * kPairThreads;  // kPairSpan (pf_jobs_plan.cpp): one pair per thread of a K1' block
    blocks[b] = PairBlock{e.x, g.cand + off, min(kPairThreads, g.cap - off), g.out + e.y * g.stride + off};
}

hipError_t launch_expand_pairs(const PairGen* gens, int ngens, const int2* pool, int nblocks, PairBlock* blocks,
                               hipStream_t s) {
    if (nblocks <= 0 || ngens <= 0) return hipSuccess;
    hipLaunchKernelGGL(expand_pairs_kernel, dim3((nblocks + 255) / 256), dim3(256), 0, s, gens, ngens, pool, nblocks,
                       blocks);
    return hipGetLastError();
}

hipError_t launch_order_pairs(const PairBlock* blocks, int nblocks, const int32_t* slots, int32_t n_slots,
                              int32_t* order, hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
    (void)n_slots;
    hipLaunchKernelGGL(order_pairs_kernel, dim3(1), dim3(kOrderThreads), 0, s, blocks, nblocks, slots, order);
    return hipGetLastError();
}

hipError_t launch_gather(const DevJobsStore& g, const DevView& v, const DevJob* jobs, int njobs, const int32_t* pool,
                         const int64_t* pool64, int32_t* ht, int32_t* seq, int32_t* cand_slot, int32_t* cand_id,
                         int32_t* ncand, hipStream_t s) {
    if (njobs <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_kernel, dim3(njobs), dim3(kGatherThreads), 0, s, g, v, jobs, pool, ht, seq, cand_slot,
                       cand_id, ncand, pool64);
    return hipGetLastError();
}

hipError_t launch_qimages(const DevStore& st, const DevJobsStore& g, const ImgJob* ij, int n_small, int n_big, int n_glob,
                          uint8_t* pool, uint32_t* scratch, int32_t* fail, hipStream_t s) {
    // images [0, n_small) build in kImgLdsSmall bytes of LDS (most users: ~6 KB, so eight
    // workgroups per CU instead of the three that kImgLds allows), [n_small, + n_big) in kImgLds,
    // then n_glob in global memory
    auto lds_launch = [&](int first, int n, uint32_t bytes) {
        if (n <= 0) return;
        if (st.packed)
            hipLaunchKernelGGL((qimage_kernel<true, true>), dim3(n), dim3(kJobThreads), bytes, s, st, g, ij + first, pool,
                               scratch, fail);
        else
            hipLaunchKernelGGL((qimage_kernel<false, true>), dim3(n), dim3(kJobThreads), bytes, s, st, g, ij + first,
                               pool, scratch, fail);
    };
    lds_launch(0, n_small, kImgLdsSmall);
    lds_launch(n_small, n_big, kImgLds);
    const int n_lds = n_small + n_big;
    if (n_glob > 0) {
        if (st.packed)
            hipLaunchKernelGGL((qimage_kernel<true, false>), dim3(n_glob), dim3(kJobThreads), 0, s, st, g, ij + n_lds,
                               pool, scratch, fail);
        else
            hipLaunchKernelGGL((qimage_kernel<false, false>), dim3(n_glob), dim3(kJobThreads), 0, s, st, g, ij + n_lds,
                               pool, scratch, fail);
    }
    return hipGetLastError();
}

hipError_t launch_collab(const DevJob* jobs, const int32_t* jix, int njobs, int max_cap, const int32_t* pool,
                         const float* pout, const int32_t* cand_slot, float* score, const int32_t* ids, uint64_t* parts,
                         unsigned int* tickets, uint64_t* out, int k, hipStream_t s) {
    if (njobs <= 0 || max_cap <= 0) return hipSuccess;
    const int gx = (max_cap + kCollabCands - 1) / kCollabCands;
    for (int b = 0; b < njobs; b += 65535) {
        const int nb = njobs - b < 65535 ? njobs - b : 65535;
        hipLaunchKernelGGL(collab_kernel, dim3(gx, nb), dim3(kJobThreads), 0, s, jobs, jix + b, pool, pout, cand_slot,
                           score, ids, parts + (size_t)b * gx * k, tickets + b, out, k);
    }
    return hipGetLastError();
}

hipError_t launch_clubs(const DevJobsStore& g, const DevView& v, const DevJob* jobs, const int32_t* jix, int njobs,
                        const int32_t* pool, const int64_t* pool64, const float* pout, double* acc, float* score,
                        int32_t* ids, int32_t* ncand, int64_t acc_stride, hipStream_t s) {
    if (njobs <= 0) return hipSuccess;
    hipLaunchKernelGGL(clubs_kernel, dim3(njobs), dim3(64), 0, s, g, v, jobs, jix, pool, pool64, pout, acc, score, ids,
                       ncand, acc_stride);
    return hipGetLastError();
}

hipError_t launch_job_topk(const DevJob* jobs, const int32_t* jix, int njobs, const float* score, const int32_t* ids,
                           const int32_t* slots, const int32_t* ncand, uint64_t* out, int k, hipStream_t s) {
    if (njobs <= 0) return hipSuccess;
    hipLaunchKernelGGL(topk_kernel, dim3(njobs), dim3(kJobThreads), 0, s, jobs, jix, score, ids, slots, ncand, out, k);
    return hipGetLastError();
}

}  // namespace pf
