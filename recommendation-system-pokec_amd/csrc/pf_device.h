// pf_device.h — device helpers shared by the gfx950 kernel files (pf_kernels.hip,
// pf_jobs.hip): the reference's FAS arithmetic, query-table probes, tile-store record
// access and the wave top-k.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pf_types.h"

namespace pf {

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
// (out of line, like ratio_term: the fixed-term phase calls them for four candidates per thread,
// and eight inlined exp + division chains made the scan's hot code larger than the instruction cache)
__device__ __forceinline__ double set_term_inl(const QConst& q, int slot, int inter, int nb, double sqrt_na) {
    const double den = sqrt_na * sqrt((double)nb);
    const double s = den <= 0.0 ? 0.0 : (double)(float)((double)inter / den);
    return term_of(q, slot, s);
}
static __device__ __attribute__((noinline)) double set_term(const QConst& q, int slot, int inter, int nb,
                                                             double sqrt_na) {
    return set_term_inl(q, slot, inter, nb, sqrt_na);
}

// recommender.cpp:114-116: (float)(dot / (sqrt(na) * sqrt(nb)))
__device__ __forceinline__ double text_term(const QConst& q, int t, double dot, double sqrt_nb) {
    const double den = q.sqrt_na[t] * sqrt_nb;
    const double s = den <= 0.0 ? 0.0 : (double)(float)(dot / den);
    return term_of(q, kNumFixed + t, s);
}

// completion / age ratio outside the host table (recommender_similarity.cpp:40-53)
static __device__ __attribute__((noinline)) double ratio_term(const QConst& q, int slot, int a, int b) {
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    return term_of(q, slot, (double)lo / (double)hi);
}

// ---------------------------------------------------------------- query hash (cuckoo)
struct QView {
    const QConst* q;
    const uint32_t* tab;  // packed: T | T3;  wide: T0 | T1 | T2 (2^lg each) | T3 (2^lg_excl); SoA per table
    const QVal* vals;
    void* hits;        // LDS [kHitCap + 1][blockDim.x] per-lane token-hit list
    uint32_t* nh;      // LDS [blockDim.x] hit counts, read across the lanes of a split record
    int lg, lge;
    uint32_t hmul, excl_off;
};

// Wide tables: 2-choice probe of table `off` (entries), capacity 2^lg; val or kEmptyVal
__device__ __forceinline__ uint32_t probe(const QView& v, uint32_t off, int lg, uint32_t key) {
    const uint32_t x = cuckoo_x(key, v.hmul);
    const uint32_t* K = v.tab + 2u * off;
    const uint32_t* V = K + (1u << lg);
    const uint32_t a = cuckoo_h1(x, lg), b = cuckoo_h2(x, lg);
    // a key sits in at most one of its two slots: AND-combining keeps both reads
    // unconditional (a ?: chain lets the compiler sink the second read into a branch)
    const uint32_t r1 = K[a] == key ? V[a] : kEmptyVal;
    const uint32_t r2 = K[b] == key ? V[b] : kEmptyVal;
    return r1 & r2;
}

// Packed tables: the same probe with miss = 0 (empty slots are {~0, 0}); x = the key's hash
__device__ __forceinline__ uint32_t probe_px(const QView& v, uint32_t off, int lg, uint32_t key, uint32_t x) {
    const uint32_t* K = v.tab + 2u * off;
    const uint32_t* V = K + (1u << lg);
    const uint32_t a = cuckoo_h1(x, lg), b = cuckoo_h2(x, lg);
    return (K[a] == key ? V[a] : 0u) | (K[b] == key ? V[b] : 0u);
}
// the record table T
__device__ __forceinline__ uint32_t probe_p(const QView& v, uint32_t key) {
    return probe_px(v, 0u, v.lg, key, cuckoo_x(key, v.hmul));
}

template <bool PACKED>
__device__ __forceinline__ bool excluded(const QView& v, uint32_t uid) {
    if (PACKED) return probe_px(v, v.excl_off, v.lge, uid, cuckoo_x(uid, v.hmul)) != 0u;
    return probe(v, v.excl_off, v.lge, uid) != kEmptyVal;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = (uint32_t)__shfl_xor((int)v, o);
        v = u > v ? u : v;
    }
    return v;
}

// product of one shared token, recommender.cpp:74-85 (wA * wB, wB = tf * idf)
__device__ __forceinline__ double hit_product(const QView& v, uint32_t vi, int32_t tf) {
    const QVal qv = v.vals[vi];
    return qv.wq * ((double)tf * qv.idf);
}

// Where a candidate lives: tile, index in the tile, lanes per record (1 << lgk)
struct Loc {
    int tile;
    int cand;
    uint32_t lgk;
};

__device__ __forceinline__ Loc loc_of(const DevStore& st, int p) {
    Loc l;
    l.tile = (int)st.slot_tile[p];
    l.cand = p - (int)st.tile_slot0[l.tile];
    l.lgk = st.tile_lgk[l.tile];
    return l;
}

__device__ __forceinline__ double col_norm(const DevStore& st, const Loc& l, uint64_t cmask, int t) {
    const uint32_t r = (uint32_t)__popcll(cmask & ((1ull << t) - 1ull));
    // [tile][candidate][rank]: a candidate's norms share cache lines, so its hit columns
    // re-use the lines its first one brought in
    const uint64_t base = st.norm_off[l.tile], mr = (st.norm_off[l.tile + 1] - base) >> 6;
    return st.norms[base + (uint64_t)l.cand * mr + r];
}

// word j of a candidate's record (chunk j / q in lane cand * k + j / q)
__device__ __forceinline__ uint32_t word_at(const DevStore& st, const Loc& l, uint32_t q, uint32_t j) {
    const uint32_t c = j / q, o = j - c * q;
    const uint32_t lane = ((uint32_t)l.cand << l.lgk) + c;
    const uint32_t* base = reinterpret_cast<const uint32_t*>(st.stream + st.tile_off[l.tile]);
    return base[((size_t)(o >> 2) * kTileSlots + lane) * 4 + (o & 3)];
}

__device__ __forceinline__ uint32_t record_words(const uint4& h2, bool packed) {
    return h2.y + h2.z + (packed ? h2.w : 2 * h2.w);
}

// ---------------------------------------------------------------- wave scans
// Inclusive prefix sum of one u32 per lane over the wave by DPP (row shifts 1, 2, 4, 8 inside each
// 16-lane row, then row_bcast:15 into rows 1 and 3 and row_bcast:31 into rows 2 and 3): six VALU
// steps with no LDS round trip (a __shfl_up ladder is six dependent ds_bpermute's).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
__device__ __forceinline__ uint32_t wave_last(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }

// ---------------------------------------------------------------- cross-workgroup hand-off
// A workgroup publishes its k-list (agent-scope sc1 stores, drained by s_waitcnt vmcnt(0)) and
// then takes a ticket; the holder of the last ticket reads every list (agent-scope sc1 loads).
// PF_TICKET_MODE selects the ticket's ordering:
//   0 (default) relaxed ticket, no fence: the lists reach the coherence point before the ticket
//     is issued (the wait) and the reads are issued after it returns (a data dependence), so the
//     hand-off is ordered by the hardware's issue order; tests/test_gpu_parity.py
//     test_fused_topk_hand_off_stress compares thousands of fused merges with K8's ranking;
//   1 release ticket, and the last ticket's holder alone runs an agent acquire fence before its
//     reads (ticket_acquire): ordered by the memory model; K5 185.0 / 185.7 vs 179.6 us per
//     cfg-2 launch relaxed (r6d, one box: buffer_wbl2 per workgroup, buffer_inv per merge);
//   2 acquire-release ticket: 186.3 us.
#ifndef PF_TICKET_MODE
#define PF_TICKET_MODE 0
#endif
__device__ __forceinline__ unsigned int take_ticket(unsigned int* p) {
#if PF_TICKET_MODE == 2
    return __hip_atomic_fetch_add(p, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
#elif PF_TICKET_MODE == 1
    return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
#else
    return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}
// the last ticket's holder, before it reads the published lists
__device__ __forceinline__ void ticket_acquire() {
#if PF_TICKET_MODE == 1
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
}

// ---------------------------------------------------------------- wave top-k
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// v of lane ^ m (m = 1, 2, 4, 8, 15, 16 or 32, a constant after unrolling) with no LDS round trip:
// DPP quad permutes, row mirrors and row rotations inside a 16-lane row, the gfx950 permlane swaps
// across rows (a __shfl_xor is a ds_bpermute: ~20 dependent ones made a 64-key sort ~1.5 us)
__device__ __forceinline__ uint32_t lane_xor32(uint32_t v, int m) {
    switch (m) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    case 4: {  // row_half_mirror (i -> 7 - i), then quad_perm [3,2,1,0]: i -> 7 - (i ^ 3) = i ^ 4
        const int h = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);
        return (uint32_t)__builtin_amdgcn_mov_dpp(h, 0x1B, 0xf, 0xf, false);
    }
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);   // row_ror:8
    case 15: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false);  // row_mirror
    case 16: {  // odd rows of the first operand swapped with even rows of the second
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16u) ? r[0] : r[1];
    }
    case 32: {  // upper half of the first operand swapped with lower half of the second
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32u) ? r[0] : r[1];
    }
    default: return (uint32_t)__shfl_xor((int)v, m);
    }
}
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v, int m) {
    return ((uint64_t)lane_xor32((uint32_t)(v >> 32), m) << 32) | lane_xor32((uint32_t)v, m);
}
// v of lane 63 - lane (= lane ^ 63)
__device__ __forceinline__ uint64_t lane_rev64(uint64_t v) { return lane_xor64(lane_xor64(lane_xor64(v, 15), 16), 32); }
// the smallest v over the wave, in every lane
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
    for (int m = 1; m <= 32; m <<= 1) {
        const uint64_t y = lane_xor64(v, m);
        v = y < v ? y : v;
    }
    return v;
}

// ascending bitonic sort of one key per lane across the wave
__device__ __forceinline__ uint64_t wave_sort64(uint64_t x, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t y = lane_xor64(x, j);
            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
            x = keep_min ? (x < y ? x : y) : (x < y ? y : x);
        }
    }
    return x;
}

// The wave keeps the 64 smallest keys seen so far, sorted ascending across lanes
// (lane i = i-th best); a top-k caller reads lanes < k.  Few qualifying keys are
// inserted one by one; many are merged with a bitonic sort + merge (O(log^2 64)).
// Out of line: the scan tails inline dozens of pushes, and only the first test is hot.
static __device__ __attribute__((noinline)) uint64_t topk_insert(uint64_t list, uint64_t x, uint64_t thr, uint64_t m,
                                                                  int k, int lane) {
    if (__popcll(m) > 3) {
        const uint64_t rev = lane_rev64(wave_sort64(x < thr ? x : ~0ull, lane));
        uint64_t y = list < rev ? list : rev;  // bitonic: the 64 smallest of both lists
#pragma unroll
        for (int j = 32; j > 0; j >>= 1) {
            const uint64_t z = lane_xor64(y, j);
            y = (lane & j) ? (y < z ? z : y) : (y < z ? y : z);
        }
        return y;
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
    return list;
}

__device__ __forceinline__ void topk_push(uint64_t& list, uint64_t x, int k, int lane) {
    const uint64_t thr = rdlane64(list, k - 1);
    const uint64_t m = __ballot(x < thr);
    if (m) list = topk_insert(list, x, thr, m, k, lane);
}

}  // namespace pf
