// pf_kernels.hip — gfx950 kernels of the FAS engine.
//
//   fas_scan_kernel   K1+K2a  all-candidates FAS (A13) over a tile range, one query per
//                             blockIdx.y, fused per-wave/per-block top-k
//   topk_merge_kernel K2b     per-query merge of per-block (or per-GPU) key lists
//   fas_pairs_kernel  K1'     FAS for explicit (query, candidate) pairs (A10/A12/A14/A15)
//   collab_sum_kernel K4      score(c) = sum_f (double)w_f * FAS(f,c), friend-list order (A14)
//
// One lane owns one candidate and walks its record through a small state machine
// (clubs -> friends -> text columns, i.e. exactly the reference's summation order,
// recommender_similarity.cpp:38-113).  Records are stored tile-interleaved (64
// candidates x 16 B per step) so every step of a wave is one coalesced 1 KiB load.
// The query (A side) lives in LDS: constants + sigmoid tables + an open-addressing
// hash of its clubs, friends and (column, token) weights.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pf_kernels.h"

namespace pf {

static_assert(sizeof(QConst) % 16 == 0, "QConst must keep the LDS carve 16-B aligned");
static_assert(sizeof(QVal) == 16, "QVal is one 16-B load");

enum : uint32_t {
    PH_NCLUB = 0, PH_CLUB, PH_NFRI, PH_FRI, PH_CHDR, PH_NB0, PH_NB1, PH_TOK, PH_TF, PH_DONE
};

// ---------------------------------------------------------------- arithmetic
// recommender_similarity.cpp:18-26: both branches evaluate exp(-|x|)
__device__ __forceinline__ double dev_sigmoid(double x) {
    const bool pos = x >= 0.0;
    const double e = exp(pos ? -x : x);
    return (pos ? 1.0 : e) / (1.0 + e);
}

__device__ __forceinline__ bool zmode_of(const QConst& q, int slot) {
    if (slot < kNumFixed) return (q.zmode_fx >> slot) & 1u;
    int t = slot - kNumFixed;
    return t < 32 ? ((q.zmode_lo >> t) & 1u) : ((q.zmode_hi >> (t - 32)) & 1u);
}

// recommender_similarity.cpp:28-36,105-111
__device__ __forceinline__ double term_of(const QConst& q, int slot, double s) {
    double z = zmode_of(q, slot) ? (s - q.zmean[slot]) / q.zsd[slot] : 6.0 * (s - 0.5);
    return dev_sigmoid(z);
}

// recommender.cpp:119-128 (inter counted over B with duplicates)
__device__ __noinline__ double set_term(const QConst& q, int slot, int inter, int nb, double sqrt_na) {
    double den = sqrt_na * sqrt((double)nb);
    double s = den <= 0.0 ? 0.0 : (double)(float)((double)inter / den);
    return term_of(q, slot, s);
}

// recommender.cpp:68-117 tail: (float)(dot / (sqrt(na) * sqrt(nb)))
__device__ __noinline__ double text_term(const QConst& q, int t, double dot, double sqrt_nb) {
    double den = q.sqrt_na[t] * sqrt_nb;
    double s = den <= 0.0 ? 0.0 : (double)(float)(dot / den);
    return term_of(q, kNumFixed + t, s);
}

// completion / age ratio outside the host table (recommender_similarity.cpp:40-53)
__device__ __noinline__ double ratio_term(const QConst& q, int slot, int a, int b) {
    int lo = a < b ? a : b, hi = a < b ? b : a;
    return term_of(q, slot, (double)lo / (double)hi);
}

// ---------------------------------------------------------------- query table
struct Table {
    const uint64_t* keys;
    const QVal* vals;
    uint32_t mask;
};

__device__ __forceinline__ int probe(const Table& tb, uint32_t tag, uint32_t id) {
    const uint64_t want = make_key(tag, id);
    uint32_t s = hash_key(tag, id) & tb.mask;
    for (;;) {
        uint64_t k = tb.keys[s];
        if ((k & kKeyMask) == want) return (int)(k >> 40);
        if (k == kEmptyKey) return -1;
        s = (s + 1) & tb.mask;
    }
}

// ---------------------------------------------------------------- lane state machine
struct Lane {
    uint32_t phase, rem, tag, cols_left, nb_lo;
    int32_t inter, nB, vpend, used;
    double dot, sqrt_nb, sum;
};

template <bool PACKED>
__device__ __forceinline__ void walk_word(Lane& L, uint32_t w, const QConst& q, const Table& tb, uint64_t qmask) {
    const uint32_t ph = L.phase;
    const bool is_set = (ph == PH_CLUB) | (ph == PH_FRI);
    const bool is_tok = ph == PH_TOK;
    const uint32_t id = (PACKED && is_tok) ? (w & kPackedTidMask) : w;
    const uint32_t tg = ph == PH_CLUB ? kTagClubs : (ph == PH_FRI ? kTagFriends : L.tag);
    const bool want = is_set || (is_tok && ((qmask >> (L.tag & 63)) & 1ull));
    int vi = -1;
    if (want) vi = probe(tb, tg, id);

    bool fin_set = false, fin_col = false;
    int set_slot = PF_F_CLUBS;
    switch (ph) {
        case PH_NCLUB:
            L.nB = (int32_t)w; L.inter = 0; L.rem = w;
            if (w) L.phase = PH_CLUB; else { fin_set = true; set_slot = PF_F_CLUBS; }
            break;
        case PH_CLUB:
            L.inter += vi >= 0;
            if (--L.rem == 0) { fin_set = true; set_slot = PF_F_CLUBS; }
            break;
        case PH_NFRI:
            L.nB = (int32_t)w; L.inter = 0; L.rem = w;
            if (w) L.phase = PH_FRI; else { fin_set = true; set_slot = PF_F_FRIENDS; }
            break;
        case PH_FRI:
            L.inter += vi >= 0;
            if (--L.rem == 0) { fin_set = true; set_slot = PF_F_FRIENDS; }
            break;
        case PH_CHDR:
            L.tag = w & 0xFFu; L.rem = w >> 8; L.dot = 0.0; L.phase = PH_NB0;
            break;
        case PH_NB0:
            L.nb_lo = w; L.phase = PH_NB1;
            break;
        case PH_NB1:
            L.sqrt_nb = __hiloint2double((int)w, (int)L.nb_lo); L.phase = PH_TOK;
            break;
        case PH_TOK:
            if (PACKED) {
                if (vi >= 0) { QVal v = tb.vals[vi]; L.dot += v.wq * ((double)(w >> 24) * v.idf); }
                if (--L.rem == 0) fin_col = true;
            } else {
                L.vpend = vi; L.phase = PH_TF;
            }
            break;
        case PH_TF:
            if (L.vpend >= 0) { QVal v = tb.vals[L.vpend]; L.dot += v.wq * ((double)(int32_t)w * v.idf); }
            if (--L.rem == 0) fin_col = true; else L.phase = PH_TOK;
            break;
        default:
            break;
    }
    if (fin_set) {
        const bool clubs = set_slot == PF_F_CLUBS;
        const int na = clubs ? q.n_clubs : q.n_friends;
        if (na > 0 && L.nB > 0) {
            L.used += 1;
            L.sum += L.inter == 0 ? (clubs ? q.sig0_clubs : q.sig0_friends)
                                  : set_term(q, set_slot, L.inter, L.nB, clubs ? q.sqrt_clubs : q.sqrt_friends);
        }
        L.phase = clubs ? PH_NFRI : (L.cols_left ? PH_CHDR : PH_DONE);
    }
    if (fin_col) {
        const uint32_t t = L.tag;
        if ((qmask >> t) & 1ull) {
            L.used += 1;
            L.sum += L.dot == 0.0 ? q.sig0_col[t] : text_term(q, (int)t, L.dot, L.sqrt_nb);
        }
        L.cols_left -= 1;
        L.phase = L.cols_left ? PH_CHDR : PH_DONE;
    }
}

// FAS(A = LDS query, B = candidate slot p).  Every lane of the wave must call it
// (probing is divergent-safe; `active` lanes only).
template <bool PACKED>
__device__ __forceinline__ float fas_slot(const DevStore& st, const QConst& q, const Table& tb, int p, bool active) {
    Lane L;
    L.phase = PH_NCLUB; L.rem = 0; L.tag = 0; L.nb_lo = 0; L.inter = 0; L.nB = 0; L.vpend = -1;
    L.used = 0; L.dot = 0.0; L.sqrt_nb = 0.0; L.sum = 0.0;
    const uint64_t qmask = q.colmask;
    uint32_t steps = 0;
    const uint4* base = st.stream;
    if (active) {
        const uint4 h0 = st.hdr0[p];
        const uint4 h1 = st.hdr1[p];
        const uint64_t cmask = (uint64_t)h0.x | ((uint64_t)h0.y << 32);
        L.cols_left = (uint32_t)__popcll(cmask);
        // fixed fields, reference order: public, gender, completion, age, region
        const uint32_t pb = h1.w & 0xFFu, gb = (h1.w >> 8) & 0xFFu;
        if (q.pubcode != kCodeMissing && pb != kCodeMissing) { L.sum += q.sig_pub[pb == q.pubcode]; L.used++; }
        if (q.gencode != kCodeMissing && gb != kCodeMissing) { L.sum += q.sig_gen[gb == q.gencode]; L.used++; }
        const int cb = (int)h0.z, ab = (int)h0.w;
        if (q.comp > 0 && cb > 0) {
            L.sum += cb <= kValTab ? q.sig_comp[cb] : ratio_term(q, PF_F_COMPLETION, q.comp, cb);
            L.used++;
        }
        if (q.age > 0 && ab > 0) {
            L.sum += ab <= kValTab ? q.sig_age[ab] : ratio_term(q, PF_F_AGE, q.age, ab);
            L.used++;
        }
        const int r0 = (int)h1.x, r1 = (int)h1.y, r2 = (int)h1.z;
        const int bcnt = (r0 >= 0) + (r1 >= 0) + (r2 >= 0);
        if (q.a_regcnt > 0 && bcnt > 0) {
            const int m = (r0 >= 0 && r0 == q.reg[0]) + (r1 >= 0 && r1 == q.reg[1]) + (r2 >= 0 && r2 == q.reg[2]);
            L.sum += q.sig_reg[bcnt][m];
            L.used++;
        }
        steps = (st.slot_len[p] + 3) >> 2;
        base = st.stream + st.tile_off[p >> 6] + (p & 63);
    }
    uint4 cur = steps ? base[0] : make_uint4(0, 0, 0, 0);
    for (uint32_t s = 0;; ++s) {
        const bool live = s < steps;
        if (!__any(live)) break;
        if (live) {
            const uint4 nxt = (s + 1 < steps) ? base[(size_t)(s + 1) * kTileSlots] : make_uint4(0, 0, 0, 0);
            walk_word<PACKED>(L, cur.x, q, tb, qmask);
            walk_word<PACKED>(L, cur.y, q, tb, qmask);
            walk_word<PACKED>(L, cur.z, q, tb, qmask);
            walk_word<PACKED>(L, cur.w, q, tb, qmask);
            cur = nxt;
        }
    }
    if (!active || L.used == 0) return 0.0f;
    // recommender_similarity.cpp:114-123
    const double S = L.sum / (double)L.used;
    const double F = (double)L.used / (double)(kNumFixed + q.n_cols);
    if (S <= 0.0 && F <= 0.0) return 0.0f;
    return (float)((2.0 * S * F) / (S + F));
}

// ---------------------------------------------------------------- wave top-k
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// lane i < k holds the i-th smallest key seen so far (ascending = best first)
__device__ __forceinline__ void topk_push(uint64_t& list, uint64_t x, int k, int lane) {
    uint64_t thr = rdlane64(list, k - 1);
    uint64_t m = __ballot(x < thr);
    while (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint64_t y = rdlane64(x, src);
        if (y < thr) {
            const uint64_t lt = __ballot(lane < k && list < y);
            const int pos = __popcll(lt);
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

// Stages query image `r` into LDS; returns the table view (LDS or global).
__device__ __forceinline__ Table stage_query(char* smem, const uint8_t* pool, const QImageRef& r, const QConst*& qc) {
    stage(smem, pool + r.const_off, sizeof(QConst));
    qc = reinterpret_cast<const QConst*>(smem);
    __syncthreads();
    const uint32_t cap = 1u << qc->cap_log2;
    Table tb;
    tb.mask = cap - 1;
    if (r.lds_bytes) {
        char* kp = smem + sizeof(QConst);
        char* vp = kp + (size_t)cap * 8;
        stage(kp, pool + r.keys_off, cap * 8);
        stage(vp, pool + r.vals_off, (uint32_t)qc->n_vals * 16);
        tb.keys = reinterpret_cast<const uint64_t*>(kp);
        tb.vals = reinterpret_cast<const QVal*>(vp);
    } else {
        tb.keys = reinterpret_cast<const uint64_t*>(pool + r.keys_off);
        tb.vals = reinterpret_cast<const QVal*>(pool + r.vals_off);
    }
    __syncthreads();
    return tb;
}

// ---------------------------------------------------------------- K1: scan
// grid: (blocks, nq); block 256 = 4 waves; wave handles one 64-candidate tile at a time.
// out_keys[(q * gridDim.x + blockIdx.x) * k + i]
template <bool PACKED>
__global__ __launch_bounds__(256) void fas_scan_kernel(DevStore st, const uint8_t* __restrict__ pool,
                                                       const QImageRef* __restrict__ refs, int32_t tile_begin,
                                                       int32_t tile_end, int32_t k, uint64_t* __restrict__ out_keys) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const QImageRef r = refs[blockIdx.y];
    const QConst* qc;
    const Table tb = stage_query(smem, pool, r, qc);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t list = ~0ull;
    for (int tile = tile_begin + (int)blockIdx.x * 4 + wave; tile < tile_end; tile += (int)gridDim.x * 4) {
        const int p = tile * kTileSlots + lane;
        const bool active = p < st.n_slots;
        const float f = fas_slot<PACKED>(st, *qc, tb, p, active);
        uint64_t key = ~0ull;
        if (active) {
            const int32_t uid = st.slot_uid[p];
            if (probe(tb, kTagExcl, (uint32_t)uid) < 0) key = score_key(f, uid);
        }
        topk_push(list, key, k, lane);
    }
    // block merge: waves 1..3 hand their lists to wave 0 through LDS
    uint64_t* scratch = reinterpret_cast<uint64_t*>(smem + (r.lds_bytes ? r.lds_bytes - 2048 : sizeof(QConst)));
    __syncthreads();
    if (wave) scratch[(wave - 1) * 64 + lane] = lane < k ? list : ~0ull;
    __syncthreads();
    if (wave == 0) {
        for (int w = 0; w < 3; ++w) topk_push(list, scratch[w * 64 + lane], k, lane);
        if (lane < k) out_keys[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * k + lane] = list;
    }
}

// ---------------------------------------------------------------- K2: merge
// in[(part * nq + q) * stride_part ... ] layout via strides; one wave per query
__global__ __launch_bounds__(64) void topk_merge_kernel(const uint64_t* __restrict__ in, int32_t nparts, int64_t part_stride,
                                                        int64_t query_stride, int32_t k, uint64_t* __restrict__ out,
                                                        const int32_t* __restrict__ out_rows) {
    const int q = blockIdx.x, lane = threadIdx.x;
    uint64_t list = ~0ull;
    const int64_t total = (int64_t)nparts * k;
    for (int64_t base = 0; base < total; base += 64) {
        const int64_t i = base + lane;
        uint64_t x = ~0ull;
        if (i < total) {
            const int64_t part = i / k, j = i % k;
            x = in[part * part_stride + q * query_stride + j];
        }
        topk_push(list, x, k, lane);
    }
    const int row = out_rows ? out_rows[q] : q;
    if (lane < k) out[(size_t)row * k + lane] = list;
}

// ---------------------------------------------------------------- K1': pairs
template <bool PACKED>
__global__ __launch_bounds__(256) void fas_pairs_kernel(DevStore st, const uint8_t* __restrict__ pool,
                                                        const QImageRef* __restrict__ refs,
                                                        const PairBlock* __restrict__ blocks,
                                                        const int32_t* __restrict__ slots, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const PairBlock b = blocks[blockIdx.x];
    const QImageRef r = refs[b.qimg];
    const QConst* qc;
    const Table tb = stage_query(smem, pool, r, qc);
    const int i = (int)threadIdx.x;
    const bool active = i < b.count;
    const int p = active ? slots[b.begin + i] : 0;
    const float f = fas_slot<PACKED>(st, *qc, tb, p, active);
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
static uint32_t scan_lds(const QImageRef* refs_host, int nq) {
    uint32_t mx = sizeof(QConst) + 2048;
    for (int i = 0; i < nq; ++i) mx = refs_host[i].lds_bytes > mx ? refs_host[i].lds_bytes : mx;
    return mx;
}

hipError_t launch_scan(const DevStore& st, const uint8_t* pool, const QImageRef* refs_dev, const QImageRef* refs_host,
                       int nq, int tile_begin, int tile_end, int k, int blocks, uint64_t* out_keys, hipStream_t s) {
    const uint32_t lds = scan_lds(refs_host, nq);
    dim3 grid(blocks, nq), block(256);
    if (st.packed)
        hipLaunchKernelGGL(fas_scan_kernel<true>, grid, block, lds, s, st, pool, refs_dev, tile_begin, tile_end, k, out_keys);
    else
        hipLaunchKernelGGL(fas_scan_kernel<false>, grid, block, lds, s, st, pool, refs_dev, tile_begin, tile_end, k, out_keys);
    return hipGetLastError();
}

hipError_t launch_merge(const uint64_t* in, int nparts, int64_t part_stride, int64_t query_stride, int nq, int k,
                        uint64_t* out, const int32_t* out_rows, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(topk_merge_kernel, dim3(nq), dim3(64), 0, s, in, nparts, part_stride, query_stride, k, out, out_rows);
    return hipGetLastError();
}

hipError_t launch_pairs(const DevStore& st, const uint8_t* pool, const QImageRef* refs_dev, uint32_t max_lds,
                        const PairBlock* blocks, int nblocks, const int32_t* slots, float* out, hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
    if (st.packed)
        hipLaunchKernelGGL(fas_pairs_kernel<true>, dim3(nblocks), dim3(256), max_lds, s, st, pool, refs_dev, blocks, slots, out);
    else
        hipLaunchKernelGGL(fas_pairs_kernel<false>, dim3(nblocks), dim3(256), max_lds, s, st, pool, refs_dev, blocks, slots, out);
    return hipGetLastError();
}

hipError_t launch_collab_sum(const float* M, const float* w, const int32_t* row, int F, int nc, float* out, hipStream_t s) {
    if (nc <= 0) return hipSuccess;
    hipLaunchKernelGGL(collab_sum_kernel, dim3((nc + 255) / 256), dim3(256), 0, s, M, w, row, F, nc, out);
    return hipGetLastError();
}

}  // namespace pf
