// pf_kernels.hip — gfx950 kernels of the FAS engine.
//
//   fas_scan_kernel   K1   all-candidates FAS (A13) over a tile range, one query per
//                          blockIdx.y, fused per-wave / per-block top-k (K2a)
//   topk_merge_kernel K2b  per-query merge of per-block (or per-GPU) key lists
//   fas_pairs_kernel  K1'  FAS for explicit (query, candidate) pairs (A10/A12/A14/A15)
//   collab_sum_kernel K4   score(c) = sum_f (double)w_f * FAS(f,c) in friend-list order (A14)
//
// One lane owns one candidate (64 candidates = one tile per wave).  Records are stored
// tile-interleaved, so each 16-B step of a wave is one coalesced 1 KiB load.  The walk
// over a record is branch-free: a word's kind follows from its position (clubs, friends,
// then self-describing packed tokens), and every word costs one 2-choice cuckoo probe
// of the query's LDS hash (clubs, friends, (column, token) weights, exclusions).  Only
// a token hit (rare) leaves the uniform path: its product is appended to a per-lane
// LDS list of column dot products.  All sigmoid work and the reference's summation
// order (recommender_similarity.cpp:38-113: public, gender, completion, age, region,
// clubs, friends, columns ascending) live in a per-candidate epilogue.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pf_kernels.h"

namespace pf {

static_assert(sizeof(QConst) % 16 == 0, "QConst must keep the LDS carve 16-B aligned");
static_assert(sizeof(QVal) == 16, "QVal is one 16-B load");

// ---------------------------------------------------------------- arithmetic
// recommender_similarity.cpp:18-26 — both branches evaluate exp(-|x|)
__device__ __forceinline__ double dev_sigmoid(double x) {
    const bool pos = x >= 0.0;
    const double e = exp(pos ? -x : x);
    return (pos ? 1.0 : e) / (1.0 + e);
}

__device__ __forceinline__ bool zmode_of(const QConst& q, int slot) {
    if (slot < kNumFixed) return (q.zmode_fx >> slot) & 1u;
    const int t = slot - kNumFixed;
    return t < 32 ? ((q.zmode_lo >> t) & 1u) : ((q.zmode_hi >> (t - 32)) & 1u);
}

// recommender_similarity.cpp:28-36,105-111
__device__ __forceinline__ double term_of(const QConst& q, int slot, double s) {
    const double z = zmode_of(q, slot) ? (s - q.zmean[slot]) / q.zsd[slot] : 6.0 * (s - 0.5);
    return dev_sigmoid(z);
}

// recommender.cpp:119-128: inter counted over B (with duplicates) / (sqrt|A| sqrt|B|), as float
__device__ __forceinline__ double set_term(const QConst& q, int slot, int inter, int nb, double sqrt_na) {
    const double den = sqrt_na * sqrt((double)nb);
    const double s = den <= 0.0 ? 0.0 : (double)(float)((double)inter / den);
    return term_of(q, slot, s);
}

// recommender.cpp:114-116: (float)(dot / (sqrt(na) * sqrt(nb)))
__device__ __forceinline__ double text_term(const QConst& q, int t, double dot, double sqrt_nb) {
    const double den = q.sqrt_na[t] * sqrt_nb;
    const double s = den <= 0.0 ? 0.0 : (double)(float)(dot / den);
    return term_of(q, kNumFixed + t, s);
}

// completion / age ratio outside the host table (recommender_similarity.cpp:40-53)
__device__ __forceinline__ double ratio_term(const QConst& q, int slot, int a, int b) {
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    return term_of(q, slot, (double)lo / (double)hi);
}

// ---------------------------------------------------------------- query hash (cuckoo)
struct QView {
    const QConst* q;
    const uint2* tab;  // T0 clubs | T1 friends | T2 tokens (2^lg each) | T3 excl (2^lg_excl)
    const QVal* vals;
    void* hits;        // LDS [kHitCap][blockDim.x] per-lane token-hit list
    int lg, lge;
    uint32_t seed;
};

// 2-choice probe of table `off` (entries) with capacity 2^lg; returns the entry's val or kEmptyVal
__device__ __forceinline__ uint32_t probe(const QView& v, uint32_t off, int lg, uint32_t key) {
    const uint32_t x = cuckoo_x(key, v.seed);
    const uint2 e1 = v.tab[off + cuckoo_h1(x, lg)];
    const uint2 e2 = v.tab[off + cuckoo_h2(x, lg)];
    // a key sits in at most one of its two slots: AND-combining keeps both reads
    // unconditional (a ?: chain lets the compiler sink the second read into a branch)
    const uint32_t r1 = e1.x == key ? e1.y : kEmptyVal;
    const uint32_t r2 = e2.x == key ? e2.y : kEmptyVal;
    return r1 & r2;
}

__device__ __forceinline__ bool excluded(const QView& v, uint32_t uid) {
    return probe(v, 3u << v.lg, v.lge, uid) != kEmptyVal;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = (uint32_t)__shfl_xor((int)v, o);
        v = u > v ? u : v;
    }
    return v;
}

// Per-lane record walk state
struct Walk {
    uint32_t cnt;        // clubs intersections (low 16 bits) + friends intersections << 16
    uint32_t nh;         // token hits seen (entries beyond kHitCap are not stored)
    uint32_t pend;       // wide tokens: tid word waiting for its (tf, col) word
};

// A token hit is stored as its T2 val plus the candidate's tf:
//   packed: one word  vi | col << 18 | tf << 24        (the walk's only LDS write)
//   wide:   two words {col | vi << 8, tf << 8 | col}
template <bool PACKED>
struct HitT;
template <>
struct HitT<true> {
    using type = uint32_t;
    __device__ static uint32_t col(type e) { return (e >> kTidBits) & 63u; }
    __device__ static uint32_t vi(type e) { return e & kTidMask; }
    __device__ static int32_t tf(type e) { return (int32_t)(e >> 24); }
};
template <>
struct HitT<false> {
    using type = uint2;
    __device__ static uint32_t col(type e) { return e.x & 0xFFu; }
    __device__ static uint32_t vi(type e) { return e.x >> 8; }
    __device__ static int32_t tf(type e) { return (int32_t)e.y >> 8; }
};

template <bool PACKED>
__device__ __forceinline__ void walk_word(Walk& W, uint32_t w, uint32_t j, uint32_t nc, uint32_t nset, uint32_t len,
                                          const QView& v, uint32_t hstride) {
    using H = HitT<PACKED>;
    const bool ok = j < len;
    const bool tok = j >= nset;
    const bool fr = j >= nc;
    const uint32_t cap = 1u << v.lg;
    typename H::type* hits = reinterpret_cast<typename H::type*>(v.hits);
    if (PACKED) {
        // sets: T0/T1 keyed by the id; tokens: T2 keyed by the word's low 24 bits (col:tid)
        const uint32_t key = tok ? (w & 0xFFFFFFu) : w;
        const uint32_t val = probe(v, tok ? 2u * cap : (fr ? cap : 0u), v.lg, key);
        const bool hit = ok && val != kEmptyVal;
        W.cnt += (hit && !tok) ? (fr ? 0x10000u : 1u) : 0u;
        if (tok && hit) {  // rare
            if (W.nh < kHitCap) reinterpret_cast<uint32_t*>(hits)[W.nh * hstride + threadIdx.x] = val | (w & 0xFF000000u);
            W.nh += 1;
        }
    } else {
        // wide tokens: (tid, tf << 8 | col) word pairs, probed at the second word
        const bool second = tok && ((j - nset) & 1u);
        const uint32_t key = second ? W.pend : w;
        if (tok && !second) W.pend = w;
        const uint32_t val = probe(v, tok ? 2u * cap : (fr ? cap : 0u), v.lg, key);
        const bool hit = ok && (!tok || second) && val != kEmptyVal && (!tok || (val & 0xFFu) == (w & 0xFFu));
        W.cnt += (hit && !tok) ? (fr ? 0x10000u : 1u) : 0u;
        if (tok && hit) {
            if (W.nh < kHitCap) reinterpret_cast<uint2*>(hits)[W.nh * hstride + threadIdx.x] = make_uint2(val, w);
            W.nh += 1;
        }
    }
}

// product of one shared token, recommender.cpp:74-85 (wA * wB, wB = tf * idf)
__device__ __forceinline__ double hit_product(const QView& v, uint32_t vi, int32_t tf) {
    const QVal qv = v.vals[vi];
    return qv.wq * ((double)tf * qv.idf);
}

__device__ __forceinline__ double col_norm(const DevStore& st, int p, uint64_t cmask, int t) {
    const uint32_t r = (uint32_t)__popcll(cmask & ((1ull << t) - 1ull));
    return st.norms[st.norm_off[p >> 6] + (uint64_t)r * kTileSlots + (p & 63)];
}

// Text terms of a lane whose hit list overflowed: re-walk its token words from global
// memory, accumulating each column's dot in stream order (rare path).
template <bool PACKED>
__device__ __forceinline__ double text_terms_slow(const DevStore& st, const QView& v, int p, uint32_t nset,
                                                  uint32_t len, uint64_t cmask, double sum) {
    const QConst& q = *v.q;
    const uint32_t* base = reinterpret_cast<const uint32_t*>(st.stream + st.tile_off[p >> 6] + (p & 63));
    auto word = [&](uint32_t j) { return base[(size_t)(j >> 2) * (kTileSlots * 4) + (j & 3)]; };
    const uint32_t cap = 1u << v.lg;
    int cur = -1;
    double dot = 0.0;
    auto close = [&]() {
        if (cur >= 0 && ((q.colmask >> cur) & 1ull))
            sum += dot == 0.0 ? q.sig0_col[cur] : text_term(q, cur, dot, col_norm(st, p, cmask, cur));
    };
    for (uint32_t j = nset; j < len; j += PACKED ? 1 : 2) {
        uint32_t key, col, val;
        int32_t tf;
        if (PACKED) {
            const uint32_t w = word(j);
            key = w & 0xFFFFFFu;
            col = (w >> kTidBits) & 63u;
            tf = (int32_t)(w >> 24);
            val = probe(v, 2u * cap, v.lg, key);
        } else {
            const uint32_t w = word(j + 1);
            key = word(j);
            col = w & 0xFFu;
            tf = (int32_t)w >> 8;
            val = probe(v, 2u * cap, v.lg, key);
            if (val != kEmptyVal && (val & 0xFFu) != col) val = kEmptyVal;
        }
        if ((int)col != cur) {
            close();
            cur = (int)col;
            dot = 0.0;
        }
        if (val != kEmptyVal) dot += hit_product(v, PACKED ? (val & kTidMask) : (val >> 8), tf);
    }
    close();
    return sum;
}

// FAS(A = staged query, B = candidate slot p).  Every lane of the wave calls it.
template <bool PACKED>
__device__ __forceinline__ float fas_slot(const DevStore& st, const QView& v, int p, bool active) {
    using H = HitT<PACKED>;
    const QConst& q = *v.q;
    const uint32_t hstride = blockDim.x;
    uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0, h2 = h0;
    if (active) {
        h0 = st.hdr0[p];
        h1 = st.hdr1[p];
        h2 = st.hdr2[p];
    }
    const uint32_t nc = h2.y, nf = h2.z, nt = h2.w;
    const uint32_t nset = nc + nf;
    const uint32_t len = PACKED ? nset + nt : nset + 2 * nt;
    const uint32_t steps = active ? (len + 3) >> 2 : 0;
    const uint4* base = st.stream + (active ? st.tile_off[p >> 6] + (p & 63) : 0);

    Walk W;
    W.cnt = 0; W.nh = 0; W.pend = 0;
    const uint32_t smax = wave_max_u32(steps);
    // Loads past a lane's record re-read its last step (always a valid address); those
    // words are masked by j < len.
    const uint32_t last = steps ? steps - 1 : 0;
    auto ld = [&](uint32_t s) { return base[(size_t)(s < last ? s : last) * kTileSlots]; };
    // Double buffer of 4 steps: the next group's 4 loads are issued before the current
    // group is walked, so every wait is covered by a whole group of work.  (Loads kept in
    // flight across the loop back-edge make the waitcnt pass drain them at the loop head.)
    auto step = [&](const uint4& cur, uint32_t s) {
        const uint32_t j = s * 4;
        walk_word<PACKED>(W, cur.x, j + 0, nc, nset, len, v, hstride);
        walk_word<PACKED>(W, cur.y, j + 1, nc, nset, len, v, hstride);
        walk_word<PACKED>(W, cur.z, j + 2, nc, nset, len, v, hstride);
        walk_word<PACKED>(W, cur.w, j + 3, nc, nset, len, v, hstride);
    };
    uint4 c0 = ld(0), c1 = ld(1), c2 = ld(2), c3 = ld(3);
    for (uint32_t s = 0; s < smax; s += 4) {
        const uint4 n0 = ld(s + 4), n1 = ld(s + 5), n2 = ld(s + 6), n3 = ld(s + 7);
        step(c0, s);
        step(c1, s + 1);
        step(c2, s + 2);
        step(c3, s + 3);
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    if (!active) return 0.0f;

    // ---- epilogue: the reference's terms in the reference's order -------------
    double sum = 0.0;
    int used = 0;
    const uint32_t pb = h2.x & 0xFFu, gb = (h2.x >> 8) & 0xFFu;
    if (q.pubcode != kCodeMissing && pb != kCodeMissing) { sum += q.sig_pub[pb == q.pubcode]; ++used; }
    if (q.gencode != kCodeMissing && gb != kCodeMissing) { sum += q.sig_gen[gb == q.gencode]; ++used; }
    const int cb = (int)h0.z, ab = (int)h0.w;
    if (q.comp > 0 && cb > 0) { sum += cb <= kValTab ? q.sig_comp[cb] : ratio_term(q, PF_F_COMPLETION, q.comp, cb); ++used; }
    if (q.age > 0 && ab > 0) { sum += ab <= kValTab ? q.sig_age[ab] : ratio_term(q, PF_F_AGE, q.age, ab); ++used; }
    const int r0 = (int)h1.x, r1 = (int)h1.y, r2 = (int)h1.z;
    const int bcnt = (r0 >= 0) + (r1 >= 0) + (r2 >= 0);
    if (q.a_regcnt > 0 && bcnt > 0) {
        const int m = (r0 >= 0 && r0 == q.reg[0]) + (r1 >= 0 && r1 == q.reg[1]) + (r2 >= 0 && r2 == q.reg[2]);
        sum += q.sig_reg[bcnt][m];
        ++used;
    }
    const int ic = (int)(W.cnt & 0xFFFFu), ifr = (int)(W.cnt >> 16);
    if (q.n_clubs > 0 && nc > 0) {
        sum += ic == 0 ? q.sig0_clubs : set_term(q, PF_F_CLUBS, ic, (int)nc, q.sqrt_clubs);
        ++used;
    }
    if (q.n_friends > 0 && nf > 0) {
        sum += ifr == 0 ? q.sig0_friends : set_term(q, PF_F_FRIENDS, ifr, (int)nf, q.sqrt_friends);
        ++used;
    }
    const uint64_t cmask = (uint64_t)h0.x | ((uint64_t)h0.y << 32);
    uint64_t common = q.colmask & cmask;
    used += __popcll(common);
    if (W.nh <= kHitCap) {
        const typename H::type* hits = reinterpret_cast<const typename H::type*>(v.hits);
        uint32_t h = 0;
        while (common) {
            const int t = __ffsll((unsigned long long)common) - 1;
            common &= common - 1;
            double dot = 0.0;
            while (h < W.nh) {  // this column's hits, in stream (ascending tid) order
                const typename H::type e = hits[h * hstride + threadIdx.x];
                if ((int)H::col(e) != t) break;
                dot += hit_product(v, H::vi(e), H::tf(e));
                ++h;
            }
            sum += dot == 0.0 ? q.sig0_col[t] : text_term(q, t, dot, col_norm(st, p, cmask, t));
        }
    } else {
        sum = text_terms_slow<PACKED>(st, v, p, nset, len, cmask, sum);
    }
    if (used == 0) return 0.0f;
    // recommender_similarity.cpp:114-123
    const double S = sum / (double)used;
    const double F = (double)used / (double)(kNumFixed + q.n_cols);
    if (S <= 0.0 && F <= 0.0) return 0.0f;
    return (float)((2.0 * S * F) / (S + F));
}

// ---------------------------------------------------------------- wave top-k
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

// ascending bitonic sort of one key per lane across the wave
__device__ __forceinline__ uint64_t wave_sort64(uint64_t x, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t y = shfl_xor64(x, j);
            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
            x = keep_min ? (x < y ? x : y) : (x < y ? y : x);
        }
    }
    return x;
}

// The wave keeps the 64 smallest keys seen so far, sorted ascending across lanes
// (lane i = i-th best); a top-k caller reads lanes < k.  Few qualifying keys are
// inserted one by one; many are merged with a bitonic sort + merge (O(log^2 64)).
__device__ __forceinline__ void topk_push(uint64_t& list, uint64_t x, int k, int lane) {
    uint64_t thr = rdlane64(list, k - 1);
    uint64_t m = __ballot(x < thr);
    if (!m) return;
    if (__popcll(m) > 3) {
        uint64_t xs = wave_sort64(x < thr ? x : ~0ull, lane);
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)xs, 63 - lane);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(xs >> 32), 63 - lane);
        const uint64_t rev = ((uint64_t)hi << 32) | lo;
        uint64_t y = list < rev ? list : rev;  // bitonic: the 64 smallest of both lists
#pragma unroll
        for (int j = 32; j > 0; j >>= 1) {
            const uint64_t z = shfl_xor64(y, j);
            y = (lane & j) ? (y < z ? z : y) : (y < z ? y : z);
        }
        list = y;
        return;
    }
    while (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint64_t y = rdlane64(x, src);
        if (y < thr) {
            const int pos = __popcll(__ballot(list < y));
            const uint64_t up = __shfl_up(list, 1);
            if (lane > pos) list = up;
            if (lane == pos) list = y;
            thr = rdlane64(list, k - 1);
        }
    }
}

// ---------------------------------------------------------------- LDS staging
__device__ __forceinline__ void stage(void* dst, const void* src, uint32_t bytes) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* s = reinterpret_cast<const uint4*>(src);
    for (uint32_t i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

// LDS carve: [QConst][tables][vals][hit lists kHitCap x blockDim][merge scratch 2 KiB].
// GTAB = false: the cuckoo table and the token values are staged in LDS, so every probe
// is a ds_read (pointer provenance is the LDS symbol only, never merged with a global
// pointer: a merged pointer would compile to flat loads, whose waits also drain the
// HBM prefetch).  GTAB = true (query too large for LDS): probes read global memory.
template <bool GTAB>
__device__ __forceinline__ QView stage_query(char* smem, const uint8_t* pool, const QImageRef& r, char** scratch) {
    stage(smem, pool + r.const_off, sizeof(QConst));
    __syncthreads();
    const QConst* q = reinterpret_cast<const QConst*>(smem);
    QView v;
    v.q = q;
    v.lg = q->lg;
    v.lge = q->lg_excl;
    v.seed = q->seed;
    const uint32_t kb = 8u * ((3u << q->lg) + (1u << q->lg_excl)), vb = (uint32_t)q->n_vals * 16u;
    char* p = smem + sizeof(QConst);
    if constexpr (!GTAB) {
        stage(p, pool + r.keys_off, kb);
        stage(p + kb, pool + r.vals_off, vb);
        v.tab = reinterpret_cast<const uint2*>(p);
        v.vals = reinterpret_cast<const QVal*>(p + kb);
        p += kb + vb;
    } else {
        v.tab = reinterpret_cast<const uint2*>(pool + r.keys_off);
        v.vals = reinterpret_cast<const QVal*>(pool + r.vals_off);
    }
    v.hits = p;
    p += (size_t)q->n_hits_max * blockDim.x;  // n_hits_max = bytes per lane of the hit list
    *scratch = p;
    __syncthreads();
    return v;
}

// ---------------------------------------------------------------- K1: scan
// write-through store / L1-bypassing load of a word handed between workgroups of a launch
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool PACKED, bool GTAB>
__global__ __launch_bounds__(kScanThreads) void fas_scan_kernel(DevStore st, const uint8_t* __restrict__ pool,
                                                                const QImageRef* __restrict__ refs, int32_t tile_begin,
                                                                int32_t tile_end, int32_t k,
                                                                uint64_t* __restrict__ parts,
                                                                ScanSync* __restrict__ sync,
                                                                uint64_t* __restrict__ out,
                                                                const int32_t* __restrict__ out_rows) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const QImageRef r = refs[blockIdx.y];
    char* scratch;
    const QView v = stage_query<GTAB>(smem, pool, r, &scratch);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t list = ~0ull;
    for (int tile = tile_begin + (int)blockIdx.x * 4 + wave; tile < tile_end; tile += (int)gridDim.x * 4) {
        const int p = tile * kTileSlots + lane;
        const bool active = p < st.n_slots;
        const float f = fas_slot<PACKED>(st, v, p, active);
        uint64_t key = ~0ull;
        if (active) {
            const int32_t uid = (int32_t)st.hdr1[p].w;
            if (!excluded(v, (uint32_t)uid)) key = score_key(f, uid);
        }
        topk_push(list, key, k, lane);
    }
    // block merge: the 4 wave lists are packed densely (k keys each) and wave 0 takes
    // them 64 at a time, so 4*k <= 64 keys cost a single push
    uint64_t* sc = reinterpret_cast<uint64_t*>(scratch);
    __syncthreads();
    if (lane < k) sc[wave * k + lane] = list;
    __syncthreads();
    // Fused cross-block merge (no second launch).  Each block publishes its sorted k-list
    // with write-through (sc1) stores, drains them and takes a ticket; the last block of
    // the query merges, reading the lists with sc1 loads (cdna_hip_programming.md
    // Guideline 16, R1: no L2 write-back or acquire fence needed).
    ScanSync* sy = sync + blockIdx.y;
    uint64_t* qparts = parts + (size_t)blockIdx.y * gridDim.x * k;
    // tail scratch in the (now idle) hit lists: flag, threshold, block count, block ids
    int* s_flag = reinterpret_cast<int*>(v.hits);
    int* s_cnt = s_flag + 1;
    uint64_t* s_T = reinterpret_cast<uint64_t*>(s_flag + 2);
    int* s_blk = s_flag + 4;
    if (wave == 0) {
        uint64_t acc = ~0ull;
        const int n = (kScanThreads / 64) * k;
        for (int b = 0; b < n; b += 64) topk_push(acc, b + lane < n ? sc[b + lane] : ~0ull, k, lane);
        if (lane < k) st_agent(qparts + (size_t)blockIdx.x * k + lane, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(&sy->done, 1u);
        if (lane == 0) {
            *s_flag = t == gridDim.x - 1;
            *s_cnt = 0;
        }
    }
    __syncthreads();
    if (!*s_flag) return;
    const int nb = (int)gridDim.x;
    const int row = out_rows ? out_rows[blockIdx.y] : (int)blockIdx.y;
    // Pass 1: the k smallest of every block's first j keys (j * nb >= 2k).  Its k-th key T
    // bounds the final k-th key from above, and a block can hold further keys <= T only
    // if its j-th key is <= T, which at most k blocks satisfy (keys are distinct).
    const int j = min(k, max(1, (2 * k + nb - 1) / nb));
    const int n1 = nb * j;
    list = ~0ull;
    for (int base = wave * 512; base < n1; base += kScanThreads * 8) {
        uint64_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = base + u * 64 + lane;
            x[u] = ~0ull;
            if (i < n1) {
                const int blk = i / j;
                x[u] = ld_agent(qparts + (size_t)blk * k + (i - blk * j));
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) topk_push(list, x[u], k, lane);
    }
    if (lane < k) sc[wave * k + lane] = list;
    __syncthreads();
    uint64_t acc = ~0ull;
    if (wave == 0) {
        const int n = (kScanThreads / 64) * k;
        for (int b = 0; b < n; b += 64) topk_push(acc, b + lane < n ? sc[b + lane] : ~0ull, k, lane);
        if (lane == 0) *s_T = rdlane64(acc, k - 1);
    }
    __syncthreads();
    const uint64_t T = *s_T;
    if (T == ~0ull) {
        // fewer than k keys among the first j of every block: merge every list in full
        list = ~0ull;
        const int total = nb * k;
        for (int base = wave * 512; base < total; base += kScanThreads * 8) {
            uint64_t x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = base + u * 64 + lane;
                x[u] = i < total ? ld_agent(qparts + i) : ~0ull;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) topk_push(list, x[u], k, lane);
        }
        __syncthreads();
        if (lane < k) sc[wave * k + lane] = list;
        __syncthreads();
        if (wave == 0) {
            acc = ~0ull;
            const int n = (kScanThreads / 64) * k;
            for (int b = 0; b < n; b += 64) topk_push(acc, b + lane < n ? sc[b + lane] : ~0ull, k, lane);
            if (lane < k) out[(size_t)row * k + lane] = acc;
        }
        return;
    }
    // Pass 2: the remaining keys of the blocks whose j-th key is <= T
    if (j < k) {
        for (int b = (int)threadIdx.x; b < nb; b += kScanThreads) {
            const uint64_t y = ld_agent(qparts + (size_t)b * k + (j - 1));
            if (y <= T) {
                const int p = atomicAdd(s_cnt, 1);
                if (p < kMaxTopK) s_blk[p] = b;
            }
        }
    }
    __syncthreads();
    if (wave == 0) {
        const int nblk = min(*s_cnt, kMaxTopK), rest = k - j, n2 = nblk * rest;
        for (int base = 0; base < n2; base += 512) {
            uint64_t x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = base + u * 64 + lane;
                x[u] = ~0ull;
                if (i < n2) {
                    const int bi = i / rest;
                    x[u] = ld_agent(qparts + (size_t)s_blk[bi] * k + j + (i - bi * rest));
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) topk_push(acc, x[u] <= T ? x[u] : ~0ull, k, lane);
        }
        if (lane < k) out[(size_t)row * k + lane] = acc;
    }
}

// ---------------------------------------------------------------- K2: merge
// Key lists in[part * part_stride + q * query_stride + j] (j < k) -> out[q * k + j]
// (the cross-shard merge after the all-gather; one block per query, every wave pushes
// its share of the keys, then wave 0 merges the wave lists).
constexpr int kMergeThreads = 1024;
__global__ __launch_bounds__(kMergeThreads) void topk_merge_kernel(const uint64_t* __restrict__ in, int32_t nparts,
                                                                   int64_t part_stride, int64_t query_stride, int32_t k,
                                                                   uint64_t* __restrict__ out) {
    __shared__ uint64_t sc[16 * 64];
    const int q = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t total = (int64_t)nparts * k;
    uint64_t list = ~0ull;
    for (int64_t base = 0; base < total; base += (int64_t)blockDim.x * 8) {
        uint64_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = base + (int64_t)u * blockDim.x + threadIdx.x;
            x[u] = ~0ull;
            if (i < total) {
                const int32_t part = (int32_t)(i / k), j = (int32_t)(i - (int64_t)part * k);
                x[u] = in[(int64_t)part * part_stride + q * query_stride + j];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) topk_push(list, x[u], k, lane);
    }
    if (lane < k) sc[wave * k + lane] = list;
    __syncthreads();
    if (wave == 0) {
        uint64_t acc = ~0ull;
        const int n = (int)(blockDim.x >> 6) * k;
        for (int b = 0; b < n; b += 64) topk_push(acc, b + lane < n ? sc[b + lane] : ~0ull, k, lane);
        if (lane < k) out[(size_t)q * k + lane] = acc;
    }
}

// ---------------------------------------------------------------- K1': pairs
template <bool PACKED, bool GTAB>
__global__ __launch_bounds__(256) void fas_pairs_kernel(DevStore st, const uint8_t* __restrict__ pool,
                                                        const QImageRef* __restrict__ refs,
                                                        const PairBlock* __restrict__ blocks,
                                                        const int32_t* __restrict__ slots, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const PairBlock b = blocks[blockIdx.x];
    char* scratch;
    const QView v = stage_query<GTAB>(smem, pool, refs[b.qimg], &scratch);
    const int i = (int)threadIdx.x;
    const bool active = i < b.count;
    const int p = active ? slots[b.begin + i] : 0;
    const float f = fas_slot<PACKED>(st, v, p, active);
    if (active) out[b.begin + i] = f;
}

// ---------------------------------------------------------------- K4: collaborative sum
// score(c) = sum over friend-list positions j (in order) of (double)w[j] * (double)M[row[j]][c]
// (recommender_graph.cpp:167-180); row[j] < 0 -> friend skipped.
__global__ __launch_bounds__(256) void collab_sum_kernel(const float* __restrict__ M, const float* __restrict__ w,
                                                         const int32_t* __restrict__ row, int32_t F, int32_t nc,
                                                         float* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    double s = 0.0;
    for (int j = 0; j < F; ++j) {
        const int r = row[j];
        if (r < 0) continue;
        s += (double)w[j] * (double)M[(size_t)r * nc + c];
    }
    out[c] = (float)s;
}

// ---------------------------------------------------------------- launchers
hipError_t launch_scan(const DevStore& st, const uint8_t* pool, const QImageRef* refs_dev, uint32_t lds, bool gtab,
                       int nq, int tile_begin, int tile_end, int k, int blocks, uint64_t* parts, ScanSync* sync,
                       uint64_t* out, const int32_t* out_rows, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    dim3 grid(blocks, nq), block(kScanThreads);
#define PF_SCAN(P, G) hipLaunchKernelGGL((fas_scan_kernel<P, G>), grid, block, lds, s, st, pool, refs_dev, tile_begin, \
                                         tile_end, k, parts, sync, out, out_rows)
    if (st.packed) { if (gtab) PF_SCAN(true, true); else PF_SCAN(true, false); }
    else { if (gtab) PF_SCAN(false, true); else PF_SCAN(false, false); }
#undef PF_SCAN
    return hipGetLastError();
}

hipError_t launch_merge(const uint64_t* in, int nparts, int64_t part_stride, int64_t query_stride, int nq, int k,
                        uint64_t* out, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(topk_merge_kernel, dim3(nq), dim3(kMergeThreads), 0, s, in, nparts, part_stride, query_stride,
                       k, out);
    return hipGetLastError();
}

hipError_t launch_pairs(const DevStore& st, const uint8_t* pool, const QImageRef* refs_dev, uint32_t max_lds,
                        bool gtab, const PairBlock* blocks, int nblocks, const int32_t* slots, float* out,
                        hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
#define PF_PAIRS(P, G) hipLaunchKernelGGL((fas_pairs_kernel<P, G>), dim3(nblocks), dim3(256), max_lds, s, st, pool, \
                                          refs_dev, blocks, slots, out)
    if (st.packed) { if (gtab) PF_PAIRS(true, true); else PF_PAIRS(true, false); }
    else { if (gtab) PF_PAIRS(false, true); else PF_PAIRS(false, false); }
#undef PF_PAIRS
    return hipGetLastError();
}

hipError_t launch_collab_sum(const float* M, const float* w, const int32_t* row, int F, int nc, float* out, hipStream_t s) {
    if (nc <= 0) return hipSuccess;
    hipLaunchKernelGGL(collab_sum_kernel, dim3((nc + 255) / 256), dim3(256), 0, s, M, w, row, F, nc, out);
    return hipGetLastError();
}

}  // namespace pf
