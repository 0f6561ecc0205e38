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
    const uint64_t* keys;
    const QVal* vals;
    double* hits;      // LDS [H][blockDim.x] per-lane column dot products
    int lg;
    uint32_t seed;
};

__device__ __forceinline__ int lookup(const QView& v, uint32_t tag, uint32_t id) {
    const uint32_t mx = cuckoo_mix(tag, id, v.seed);
    const uint64_t want = make_key(tag, id);
    const uint64_t k1 = v.keys[cuckoo_h1(mx, v.lg)];
    const uint64_t k2 = v.keys[cuckoo_h2(mx, v.lg)];
    int r = -1;
    if ((k1 & kKeyMask) == want) r = (int)(k1 >> 40);
    if ((k2 & kKeyMask) == want) r = (int)(k2 >> 40);
    return r;
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
    int ic, ifr;         // clubs / friends intersections
    uint32_t nh;         // hit columns recorded
    uint32_t last_col;   // column of the last hit
    uint64_t hitmask;
    uint32_t pend;       // wide tokens: tid word waiting for its (tf, col) word
};

template <bool PACKED>
__device__ __forceinline__ void walk_word(Walk& W, uint32_t w, uint32_t j, uint32_t nc, uint32_t nset, uint32_t len,
                                          const QView& v, uint32_t hstride) {
    const bool ok = j < len;
    const bool tok = j >= nset;
    const bool fr = j >= nc;
    uint32_t tag, id, tfw;
    bool probe;
    if (PACKED) {
        tag = tok ? (w >> 26) : (fr ? kTagFriends : kTagClubs);
        id = tok ? (w & kTidMask) : w;
        tfw = (w >> kTidBits) & 0xFFu;
        probe = ok;
    } else {
        const bool second = tok && ((j - nset) & 1u);
        tag = second ? (w & 0xFFu) : (fr ? kTagFriends : kTagClubs);
        id = second ? W.pend : w;
        tfw = (uint32_t)((int32_t)w >> 8);
        if (tok && !second) W.pend = w;
        probe = ok && (!tok || second);
    }
    int vi = lookup(v, tag, id);
    vi = probe ? vi : -1;
    const bool hit = vi >= 0;
    W.ic += (!fr && hit) ? 1 : 0;
    W.ifr += (fr && !tok && hit) ? 1 : 0;
    if (tok && hit) {  // rare: accumulate this token's product into its column's dot
        const QVal qv = v.vals[vi];
        const double prod = qv.wq * ((double)(int32_t)tfw * qv.idf);
        if (tag != W.last_col) {
            v.hits[W.nh * hstride + threadIdx.x] = prod;
            W.nh += 1;
            W.last_col = tag;
            W.hitmask |= 1ull << tag;
        } else {
            v.hits[(W.nh - 1) * hstride + threadIdx.x] += prod;
        }
    }
}

// FAS(A = staged query, B = candidate slot p).  Every lane of the wave calls it.
template <bool PACKED>
__device__ __forceinline__ float fas_slot(const DevStore& st, const QView& v, int p, bool active) {
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
    W.ic = 0; W.ifr = 0; W.nh = 0; W.last_col = 0xFFFFFFFFu; W.hitmask = 0; W.pend = 0;
    const uint32_t smax = wave_max_u32(steps);
    // 4-deep software prefetch of the 16-B steps.  Loads past a lane's record re-read its
    // last step (always a valid address); those words are masked by j < len.
    const uint32_t last = steps ? steps - 1 : 0;
    auto ld = [&](uint32_t s) { return base[(size_t)(s < last ? s : last) * kTileSlots]; };
    // Unrolled by 4 so every buffer is consumed and refilled in place: a register
    // rotation (b0 = b1 ...) would make the compiler wait for the newest load.
    uint4 b0 = ld(0), b1 = ld(1), b2 = ld(2), b3 = ld(3);
    auto step = [&](const uint4& cur, uint32_t s) {
        const uint32_t j = s * 4;
        walk_word<PACKED>(W, cur.x, j + 0, nc, nset, len, v, hstride);
        walk_word<PACKED>(W, cur.y, j + 1, nc, nset, len, v, hstride);
        walk_word<PACKED>(W, cur.z, j + 2, nc, nset, len, v, hstride);
        walk_word<PACKED>(W, cur.w, j + 3, nc, nset, len, v, hstride);
    };
    // straight-line body (no early exit): the waitcnt pass then keeps 3 loads in flight
    // across the back-edge; steps past smax only see words with j >= len (masked).
    for (uint32_t s = 0; s < smax; s += 4) {
        step(b0, s);
        b0 = ld(s + 4);
        step(b1, s + 1);
        b1 = ld(s + 5);
        step(b2, s + 2);
        b2 = ld(s + 6);
        step(b3, s + 3);
        b3 = ld(s + 7);
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
    if (q.n_clubs > 0 && nc > 0) {
        sum += W.ic == 0 ? q.sig0_clubs : set_term(q, PF_F_CLUBS, W.ic, (int)nc, q.sqrt_clubs);
        ++used;
    }
    if (q.n_friends > 0 && nf > 0) {
        sum += W.ifr == 0 ? q.sig0_friends : set_term(q, PF_F_FRIENDS, W.ifr, (int)nf, q.sqrt_friends);
        ++used;
    }
    const uint64_t cmask = (uint64_t)h0.x | ((uint64_t)h0.y << 32);
    uint64_t common = q.colmask & cmask;
    used += __popcll(common);
    uint32_t h = 0;
    while (common) {
        const int t = __ffsll((unsigned long long)common) - 1;
        common &= common - 1;
        double term = q.sig0_col[t];
        if ((W.hitmask >> t) & 1ull) {
            const double dot = v.hits[h * hstride + threadIdx.x];
            ++h;
            if (dot != 0.0) {
                const uint32_t r = (uint32_t)__popcll(cmask & ((1ull << t) - 1ull));
                const double nb = st.norms[st.norm_off[p >> 6] + (uint64_t)r * kTileSlots + (p & 63)];
                term = text_term(q, t, dot, nb);
            }
        }
        sum += term;
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

// lane i < k holds the i-th smallest key seen so far (ascending key = best first)
__device__ __forceinline__ void topk_push(uint64_t& list, uint64_t x, int k, int lane) {
    uint64_t thr = rdlane64(list, k - 1);
    uint64_t m = __ballot(x < thr);
    while (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint64_t y = rdlane64(x, src);
        if (y < thr) {
            const int pos = __popcll(__ballot(lane < k && list < y));
            const uint64_t up = __shfl_up(list, 1);
            if (lane > pos && lane < k) list = up;
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

// LDS carve: [QConst][keys][vals][hits H x blockDim doubles][merge scratch 2 KiB].
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
    v.lg = q->cap_log2;
    v.seed = q->seed;
    const uint32_t kb = 8u << q->cap_log2, vb = (uint32_t)q->n_vals * 16u;
    char* p = smem + sizeof(QConst);
    if constexpr (!GTAB) {
        stage(p, pool + r.keys_off, kb);
        stage(p + kb, pool + r.vals_off, vb);
        v.keys = reinterpret_cast<const uint64_t*>(p);
        v.vals = reinterpret_cast<const QVal*>(p + kb);
        p += kb + vb;
    } else {
        v.keys = reinterpret_cast<const uint64_t*>(pool + r.keys_off);
        v.vals = reinterpret_cast<const QVal*>(pool + r.vals_off);
    }
    v.hits = reinterpret_cast<double*>(p);
    p += (size_t)q->n_hits_max * blockDim.x * 8;
    *scratch = p;
    __syncthreads();
    return v;
}

// ---------------------------------------------------------------- K1: scan
template <bool PACKED, bool GTAB>
__global__ __launch_bounds__(kScanThreads) void fas_scan_kernel(DevStore st, const uint8_t* __restrict__ pool,
                                                                const QImageRef* __restrict__ refs, int32_t tile_begin,
                                                                int32_t tile_end, int32_t k,
                                                                uint64_t* __restrict__ out_keys) {
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
            if (lookup(v, kTagExcl, (uint32_t)uid) < 0) key = score_key(f, uid);
        }
        topk_push(list, key, k, lane);
    }
    uint64_t* sc = reinterpret_cast<uint64_t*>(scratch);
    __syncthreads();
    if (wave) sc[(wave - 1) * 64 + lane] = lane < k ? list : ~0ull;
    __syncthreads();
    if (wave == 0) {
        for (int w = 0; w < kScanThreads / 64 - 1; ++w) topk_push(list, sc[w * 64 + lane], k, lane);
        if (lane < k) out_keys[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * k + lane] = list;
    }
}

// ---------------------------------------------------------------- K2: merge
// Key lists in[part * part_stride + q * query_stride + j] (j < k) -> out[row(q) * k + j].
// 1024 threads per query; every lane keeps 8 loads in flight, then the 16 wave
// lists meet in LDS.
__global__ __launch_bounds__(1024) void topk_merge_kernel(const uint64_t* __restrict__ in, int32_t nparts,
                                                          int64_t part_stride, int64_t query_stride, int32_t k,
                                                          uint64_t* __restrict__ out,
                                                          const int32_t* __restrict__ out_rows) {
    __shared__ uint64_t sc[16 * 64];
    const int q = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t list = ~0ull;
    const int64_t total = (int64_t)nparts * k;
    for (int64_t base = 0; base < total; base += (int64_t)blockDim.x * 8) {
        uint64_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = base + (int64_t)u * blockDim.x + threadIdx.x;
            x[u] = ~0ull;
            if (i < total) x[u] = in[(i / k) * part_stride + q * query_stride + (i % k)];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) topk_push(list, x[u], k, lane);
    }
    sc[wave * 64 + lane] = lane < k ? list : ~0ull;
    __syncthreads();
    if (wave == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) topk_push(list, sc[w * 64 + lane], k, lane);
        const int row = out_rows ? out_rows[q] : q;
        if (lane < k) out[(size_t)row * k + lane] = list;
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
                       int nq, int tile_begin, int tile_end, int k, int blocks, uint64_t* out_keys, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    dim3 grid(blocks, nq), block(kScanThreads);
#define PF_SCAN(P, G) hipLaunchKernelGGL((fas_scan_kernel<P, G>), grid, block, lds, s, st, pool, refs_dev, tile_begin, \
                                         tile_end, k, out_keys)
    if (st.packed) { if (gtab) PF_SCAN(true, true); else PF_SCAN(true, false); }
    else { if (gtab) PF_SCAN(false, true); else PF_SCAN(false, false); }
#undef PF_SCAN
    return hipGetLastError();
}

hipError_t launch_merge(const uint64_t* in, int nparts, int64_t part_stride, int64_t query_stride, int nq, int k,
                        uint64_t* out, const int32_t* out_rows, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(topk_merge_kernel, dim3(nq), dim3(1024), 0, s, in, nparts, part_stride, query_stride, k, out,
                       out_rows);
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
