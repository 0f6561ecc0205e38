// pf_kernels.hip — gfx950 kernels of the FAS engine.
//
//   fas_scan_kernel   K1   all-candidates FAS (A13) over a tile range, one query per
//                          blockIdx.y, fused per-wave / per-block top-k (K2a)
//   topk_merge_kernel K2b  per-query merge of per-block (or per-GPU) key lists
//   fas_pairs_kernel  K1'  FAS for explicit (query, candidate) pairs (A10/A12/A14/A15)
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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <unordered_map>
#include <vector>
#include <cstdio>
#include <cstdlib>

#include "pf_device.h"
#include "pf_kernels.h"

namespace pf {

static_assert(sizeof(QConst) % 16 == 0, "QConst must keep the LDS carve 16-B aligned");
static_assert(sizeof(QVal) == 16, "QVal is one 16-B load");

#ifdef PF_K5_TIMERS
// profiling build only (make K5T=1): per-phase clock64() sums over every wave (K5: launch_post,
// K1': launch_pairs print them every 10th launch)
__device__ unsigned long long g_k5t[16];
// K1': staging, walk, epilogue, total, dense, assembly, overflow, waves, fas, then the epilogue's
// waves past the item queue (per-lane fallback), items, epilogue waves
__device__ unsigned long long g_k1t[12];
#endif

#ifdef PF_K5_BLOCKLOG
// profiling build only (tools/build_variant.sh blog XFLAGS=-DPF_K5_BLOCKLOG): K5's per-block start /
// end times (s_memrealtime, 100 MHz, one clock for every CU), summarised by launch_post
constexpr unsigned kBlogCap = 16384;
__device__ unsigned long long g_blog_t[2 * kBlogCap];
__device__ unsigned int g_blog_meta[kBlogCap];
__device__ unsigned int g_blog_n;
#endif

// Orders a wave's LDS accesses across its lanes (LDS serves a wave's operations in order;
// this keeps the compiler from moving accesses across the point).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-lane record walk state
struct Walk {
    uint32_t cnt;        // clubs intersections (low 16 bits) + friends intersections << 16
    uint32_t nh;         // token hits seen (entries beyond kHitCap are not stored)
    uint32_t pend;       // wide tokens: tid word waiting for its (tf, col) word
};

// A token hit is stored as its T2 val plus the candidate's tf:
//   packed: one word  vi | col << 18 | tf << 24        (the walk's only LDS write)
//   wide:   two words {col | vi << 8, tf << 8 | col}; the record's token words are
//           {tid | col << 26, tf << 8 | col}, the first being the table key
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

// One 16-B step (4 record words) of a lane, branch-free.  All four probes are issued
// before any result is used, so the step's 8 LDS reads are in flight together; then the
// words update the counters in order.  Every word costs one (possibly dead) hit-list
// store: a non-hit writes the lane's next free slot, which the next real hit
// overwrites; hits past kHitCap go to a dump slot (the list then reads as overflowed
// and the epilogue re-walks the record).
//
// Packed corpora: one tagged table, so a word's probe key is the word itself (sets) or
// kTagTok | its low 24 bits (tokens), and the probe's value is directly the club / friend
// counter increment or the token's value entry.  sj = the step's first word index in the
// chunk (wave-uniform), tb = nset - j0 = where the chunk's tokens start, lim = chunk
// length (MASKED only: lanes of different tiles, whose padding is not guaranteed).
template <bool MASKED>
__device__ __forceinline__ void walk_step_p(Walk& W, const uint4& cw, int sj, int tb, int lim, const QView& v,
                                            uint32_t hstride) {
    const uint32_t w[4] = {cw.x, cw.y, cw.z, cw.w};
    uint32_t val[4];
    bool tok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        tok[i] = sj + i >= tb;
        uint32_t key = tok[i] ? (kTagTok | (w[i] & 0xFFFFFFu)) : w[i];
        if (MASKED) key = sj + i < lim ? key : kPadWord;
        val[i] = probe_p(v, key);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        W.cnt += tok[i] ? 0u : val[i];
        const uint32_t slot = (W.nh < kHitCap ? W.nh : kHitCap) * hstride + threadIdx.x;
        reinterpret_cast<uint32_t*>(v.hits)[slot] = (w[i] & 0xFF000000u) | (val[i] & 0xFFFFFFu);
        W.nh += (tok[i] && val[i] != 0u) ? 1u : 0u;
    }
}

// Wide corpora: three tables, token (tid, tf:col) word pairs probed at the second word.
__device__ __forceinline__ void walk_step_w(Walk& W, const uint4& cw, uint32_t j0, uint32_t nc, uint32_t nset,
                                            uint32_t len, const QView& v, uint32_t hstride) {
    const uint32_t w[4] = {cw.x, cw.y, cw.z, cw.w};
    uint32_t val[4];
    bool tok[4], fr[4], second[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t j = j0 + i;
        tok[i] = j >= nset;
        fr[i] = j >= nc;
        const uint32_t off = ((uint32_t)fr[i] + (uint32_t)tok[i]) << v.lg;  // T0 clubs, T1 friends, T2 tokens
        second[i] = tok[i] && ((j - nset) & 1u);
        const uint32_t key = second[i] ? (i ? w[i - 1] : W.pend) : w[i];
        val[i] = probe(v, off, v.lg, key);
    }
    W.pend = w[3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t j = j0 + i;
        const bool ok = j < len;
        const bool hit = ok && (!tok[i] || second[i]) && val[i] != kEmptyVal &&
                         (!tok[i] || (val[i] & 0xFFu) == (w[i] & 0xFFu));
        W.cnt += (hit && !tok[i]) ? (fr[i] ? 0x10000u : 1u) : 0u;
        const uint32_t slot = (W.nh < kHitCap ? W.nh : kHitCap) * hstride + threadIdx.x;
        reinterpret_cast<uint2*>(v.hits)[slot] = make_uint2(val[i], w[i]);
        W.nh += (hit && tok[i]) ? 1u : 0u;
    }
}

// A candidate's record and column norms as the epilogue reads them: word j of the record, and
// sqrt(sum w_B^2) of column t (cmask = its non-empty columns).
//   TileRec: the tile store (K1, the record-stream scan): words interleaved per tile, norms in
//            the tile's [candidate][rank] block (two dependent loads);
//   RowRec:  the row store (K1', pairs): the record contiguous, its norms right after it.
struct TileRec {
    const DevStore* st;
    Loc l;
    uint32_t qw;
    __device__ uint32_t word(uint32_t j) const { return word_at(*st, l, qw, j); }
    __device__ double norm(uint64_t cmask, int t) const { return col_norm(*st, l, cmask, t); }
};
struct RowRec {
    const uint32_t* w;
    const double* n;
    __device__ uint32_t word(uint32_t j) const { return w[j]; }
    __device__ double norm(uint64_t cmask, int t) const { return n[__popcll(cmask & ((1ull << t) - 1ull))]; }
};

// Text terms of a candidate whose hit list overflowed: re-walk its token words from
// global memory, accumulating each column's dot in stream order (rare path).
template <bool PACKED, class Rec>
__device__ __forceinline__ double text_terms_slow(const QView& v, const Rec& rec, uint32_t nset, uint32_t len,
                                                  uint64_t cmask, double sum) {
    const QConst& q = *v.q;
    const uint32_t cap = 1u << v.lg;
    int cur = -1;
    double dot = 0.0;
    auto close = [&]() {
        if (cur >= 0 && ((q.colmask >> cur) & 1ull))
            sum += dot == 0.0 ? q.sig0_col[cur] : text_term(q, cur, dot, rec.norm(cmask, cur));
    };
    for (uint32_t j = nset; j < len; j += PACKED ? 1 : 2) {
        uint32_t key, col, val;
        int32_t tf;
        if (PACKED) {
            const uint32_t w = rec.word(j);
            key = kTagTok | (w & 0xFFFFFFu);
            col = (w >> kTidBits) & 63u;
            tf = (int32_t)(w >> 24);
            val = probe_p(v, key);
            if (val == 0u) val = kEmptyVal;
        } else {
            const uint32_t w = rec.word(j + 1);
            key = rec.word(j);
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

// The same for a record in the row store (the pair kernel's overflowed hit lists): the token
// words in 16-B steps, four steps in flight (a lane alone walks its record here, so the
// loads' latency is the cost).
__device__ __forceinline__ double text_terms_row(const QView& v, const uint4* base, const double* norms, uint32_t nset,
                                              uint32_t len, uint64_t cmask, double sum) {
    const QConst& q = *v.q;
    int cur = -1;
    double dot = 0.0;
    auto close = [&]() {
        if (cur >= 0 && ((q.colmask >> cur) & 1ull))
            sum += dot == 0.0 ? q.sig0_col[cur]
                              : text_term(q, cur, dot, norms[__popcll(cmask & ((1ull << cur) - 1ull))]);
    };
    const uint32_t steps = (len + 3) >> 2, s0 = nset >> 2;
    if (len <= nset) return sum;
    auto ld = [&](uint32_t s) { return base[s < steps ? s : steps - 1]; };
    uint4 r0 = ld(s0), r1 = ld(s0 + 1), r2 = ld(s0 + 2), r3 = ld(s0 + 3);
    for (uint32_t s = s0; s < steps; ++s) {
        const uint4 cw = r0;
        r0 = r1; r1 = r2; r2 = r3;
        r3 = ld(s + 4);
        const uint32_t w4[4] = {cw.x, cw.y, cw.z, cw.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t j = 4 * s + (uint32_t)i;
            if (j < nset || j >= len) continue;
            const uint32_t w = w4[i];
            const int col = (int)((w >> kTidBits) & 63u);
            if (col != cur) {
                close();
                cur = col;
                dot = 0.0;
            }
            const uint32_t val = probe_p(v, kTagTok | (w & 0xFFFFFFu));
            if (val != 0u) dot += hit_product(v, val & kTidMask, (int32_t)(w >> 24));
        }
    }
    close();
    return sum;
}

// Walk record words [j0, j0 + clen) of the lane's chunk; base = the lane's stream column
// (step s at base[s * kTileSlots]).  Every lane of the wave calls it (clen = 0 when idle).
// Double buffer of 4-step groups: the next group's 4 loads are issued before the current
// group is walked, so every wait is covered by a whole group of work.  (Loads kept in
// flight across the loop back-edge make the waitcnt pass drain them at the loop head.)
// MASKED = false (scan): every lane of the wave is in one tile, whose steps come in whole
// groups with padding words past each chunk, and the stream ends with a group of
// padding, so loads need no clamp and words no mask.  MASKED = true (pairs): lanes of
// different tiles; loads are clamped to the lane's last step and words past the chunk
// are masked.
// STRIDE: uint4 distance between a lane's successive steps (kTileSlots in the tile stream,
// 1 in the row store).
template <bool PACKED, bool MASKED, int STRIDE = kTileSlots>
__device__ __forceinline__ void walk_chunk(Walk& W, const uint4* base, uint32_t j0, uint32_t clen, uint32_t nc,
                                           uint32_t nset, const QView& v, uint32_t hstride) {
    const uint32_t steps = (clen + 3) >> 2;
    const uint32_t smax = wave_max_u32(steps);
    const uint32_t last = steps ? steps - 1 : 0;
    auto ld = [&](uint32_t s) { return base[(size_t)(MASKED ? (s < last ? s : last) : s) * STRIDE]; };
    const int tb = (int)nset - (int)j0, lim = (int)clen;
    const uint32_t len = j0 + clen;
    auto walk = [&](const uint4& c, uint32_t s) {
        if (PACKED) walk_step_p<MASKED>(W, c, (int)s * 4, tb, lim, v, hstride);
        else walk_step_w(W, c, j0 + s * 4, nc, nset, len, v, hstride);
    };
    uint4 c0 = ld(0), c1 = ld(1), c2 = ld(2), c3 = ld(3);
    for (uint32_t s = 0; s < smax; s += 4) {
        const uint4 n0 = ld(s + 4), n1 = ld(s + 5), n2 = ld(s + 6), n3 = ld(s + 7);
        walk(c0, s);
        walk(c1, s + 1);
        walk(c2, s + 2);
        walk(c3, s + 3);
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
}

// FAS(A = staged query, B = slot p) from the walk's results: the reference's terms in the
// reference's order.  The candidate's token hits are the hit lists of threads
// first .. first + nl - 1 (its chunks, in record order); nh_of(g) = hits of thread first + g.
// RAW (packed only): the list holds the hit record words themselves (the pair walk), whose
// values are probed again here.
template <bool PACKED, bool RAW = false, class Rec, class NH>
__device__ __forceinline__ float fas_epilogue(const QView& v, const Rec& rec, const uint4& h0, const uint4& h1,
                                              const uint4& h2, uint32_t cnt, uint32_t first, uint32_t nl, NH nh_of,
                                              uint64_t* tep = nullptr) {
    static_assert(PACKED || !RAW, "raw hit words: packed corpora only");
    using H = HitT<PACKED>;
    const QConst& q = *v.q;
    const uint32_t hstride = blockDim.x;
    const uint32_t nc = h2.y, nf = h2.z;
    const uint64_t cmask = (uint64_t)h0.x | ((uint64_t)h0.y << 32);
    uint64_t common = q.colmask & cmask;
    bool overflow = false;
    for (uint32_t g = 0; g < nl; ++g) overflow |= nh_of(g) > kHitCap;
    // token hits of the chunks in order: (g, h) walks thread first + g's list
    const typename H::type* hits = reinterpret_cast<const typename H::type*>(v.hits);
    uint32_t g = 0, h = 0, nhg = overflow ? 0u : nh_of(0);
    typename H::type e{};
    auto next = [&]() -> bool {
        while (h >= nhg) {
            if (++g >= nl) return false;
            h = 0;
            nhg = nh_of(g);
        }
        e = hits[h * hstride + first + g];
        if constexpr (RAW) {
            const uint32_t w = (uint32_t)e;
            e = (w & 0xFF000000u) | (probe_p(v, kTagTok | (w & 0xFFFFFFu)) & 0xFFFFFFu);
        }
        ++h;
        return true;
    };
    bool have = next();
    // the first hit column's norm (global) is requested now and lands under the fixed terms
    double nrm = have ? rec.norm(cmask, (int)H::col(e)) : 0.0;

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
    const int ic = (int)(cnt & 0xFFFFu), ifr = (int)(cnt >> 16);
    if (q.n_clubs > 0 && nc > 0) {
        sum += ic == 0 ? q.sig0_clubs : set_term(q, PF_F_CLUBS, ic, (int)nc, q.sqrt_clubs);
        ++used;
    }
    if (q.n_friends > 0 && nf > 0) {
        sum += ifr == 0 ? q.sig0_friends : set_term(q, PF_F_FRIENDS, ifr, (int)nf, q.sqrt_friends);
        ++used;
    }
    used += __popcll(common);
    if (tep) tep[0] = clock64();
    if (!overflow) {
        // One pass in the reference's column order, driven by the HIT columns: the wave's
        // i-th iteration computes every lane's i-th hit column (the only place the
        // expensive term runs, so lanes stay aligned), after adding the s = 0 term of each
        // common column the lane skips on the way (cheap table reads).  The next hit
        // column's norm is requested before this column's term is computed.
        while (have) {
            const int t = (int)H::col(e);
            const double nrm_t = nrm;
            double dot = 0.0;
            while (have && (int)H::col(e) == t) {  // this column's hits, in stream (ascending tid) order
                dot += hit_product(v, H::vi(e), H::tf(e));
                have = next();
            }
            if (have) nrm = rec.norm(cmask, (int)H::col(e));
            uint64_t below = common & ((1ull << t) - 1ull);
            common &= ~below & ~(1ull << t);
            while (below) {
                const int c = __ffsll((unsigned long long)below) - 1;
                below &= below - 1;
                sum += q.sig0_col[c];
            }
            sum += dot == 0.0 ? q.sig0_col[t] : text_term(q, t, dot, nrm_t);
        }
        while (common) {
            const int c = __ffsll((unsigned long long)common) - 1;
            common &= common - 1;
            sum += q.sig0_col[c];
        }
    } else if constexpr (RAW) {
        sum = text_terms_row(v, reinterpret_cast<const uint4*>(rec.w), rec.n, nc + nf, record_words(h2, true), cmask, sum);
    } else {
        sum = text_terms_slow<PACKED>(v, rec, nc + nf, record_words(h2, PACKED), cmask, sum);
    }
    if (tep) tep[1] = clock64();
    if (used == 0) return 0.0f;
    // recommender_similarity.cpp:114-123
    const double S = sum / (double)used;
    const double F = (double)used / (double)(kNumFixed + q.n_cols);
    if (S <= 0.0 && F <= 0.0) return 0.0f;
    return (float)((2.0 * S * F) / (S + F));
}

// ---------------------------------------------------------------- K1' record walk (packed)
// A pair-kernel lane walks one candidate's contiguous row-store record against the staged
// query table.  The probe compares keys only (one 4-B read per cuckoo choice, the value is
// probed again for the few hits in the epilogue) and every word stores itself, the raw record
// word, at the lane's next hit slot, which only a token hit advances; so a token word costs
// its key, hash, two addresses, two reads, two compares and the slot pointer.  Groups of 4
// steps past every lane's last club / friend word take the token-only step (no set
// bookkeeping).  A lane past its record loads the padding line (kPadWord never matches, and
// build_store pads the record's last step with it), so no word needs a mask.
struct RowWalk {
    uint32_t cnt;  // clubs intersections (low 16 bits) + friends intersections << 16
    uint32_t ptr;  // the lane's next hit slot, hit list word index (slot * kPairThreads + lane)
};

__device__ __forceinline__ bool has_key(const QView& v, uint32_t key, uint32_t x) {
    // the table's keys (SoA: the packed table T is at entry offset 0, its keys in words [0, 2^lg))
    const uint32_t k1 = v.tab[cuckoo_h1(x, v.lg)];
    // cuckoo_h2 as one bit-field extract (the compiler emits a shift and a mask)
    const uint32_t k2 = v.tab[__builtin_amdgcn_ubfe(x, 32u - 2u * (uint32_t)v.lg, (uint32_t)v.lg)];
    return (k1 == key) | (k2 == key);
}

// words j0 .. j0 + 3; SETS: the step may hold club / friend words (j < nset; clubs j < nc)
template <bool SETS>
__device__ __forceinline__ void row_step(RowWalk& W, const uint4& cw, uint32_t j0, uint32_t nc, uint32_t nset,
                                         const QView& v, uint32_t pcap) {
    const uint32_t w[4] = {cw.x, cw.y, cw.z, cw.w};
    bool hit[4], tok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        tok[i] = !SETS || j0 + i >= nset;
        const uint32_t key = tok[i] ? (kTagTok | (w[i] & 0xFFFFFFu)) : w[i];
        hit[i] = has_key(v, key, cuckoo_x(key, v.hmul));
    }
    uint32_t* hl = reinterpret_cast<uint32_t*>(v.hits);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (SETS) W.cnt += (hit[i] && !tok[i]) ? (j0 + i < nc ? 1u : 0x10000u) : 0u;
        hl[W.ptr] = w[i];
        W.ptr += (hit[i] && tok[i]) ? kPairThreads : 0u;
    }
    W.ptr = W.ptr < pcap ? W.ptr : pcap;  // <= 3 writes past pcap per step: the dump slots
}

__device__ __forceinline__ void walk_row(RowWalk& W, const uint4* base, const uint4* pad, uint32_t len, uint32_t nc,
                                         uint32_t nset, const QView& v, uint32_t pcap) {
    const uint32_t steps = (len + 3) >> 2;
    const uint32_t smax = wave_max_u32(steps);
    const uint32_t sset = wave_max_u32((nset + 3) >> 2);  // steps holding a set word on some lane
    auto ld = [&](uint32_t s) { return *(s < steps ? base + s : pad); };
    uint4 c0 = ld(0), c1 = ld(1), c2 = ld(2), c3 = ld(3);
    uint32_t s = 0;
    for (; s < sset; s += 4) {
        const uint4 n0 = ld(s + 4), n1 = ld(s + 5), n2 = ld(s + 6), n3 = ld(s + 7);
        row_step<true>(W, c0, 4 * s, nc, nset, v, pcap);
        row_step<true>(W, c1, 4 * s + 4, nc, nset, v, pcap);
        row_step<true>(W, c2, 4 * s + 8, nc, nset, v, pcap);
        row_step<true>(W, c3, 4 * s + 12, nc, nset, v, pcap);
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    for (; s < smax; s += 4) {
        const uint4 n0 = ld(s + 4), n1 = ld(s + 5), n2 = ld(s + 6), n3 = ld(s + 7);
        row_step<false>(W, c0, 0, 0, 0, v, pcap);
        row_step<false>(W, c1, 0, 0, 0, v, pcap);
        row_step<false>(W, c2, 0, 0, 0, v, pcap);
        row_step<false>(W, c3, 0, 0, 0, v, pcap);
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
}

// K1' epilogue, wave-dense (packed).  fas_epilogue's per-lane loop runs the expensive terms (two
// FP64 divisions and an exp per text column, a sqrt more per set term) once per hit column of
// the lane with the most, so a wave pays ~8 rounds for a mean of ~4 hit columns per pair.  Here
// every lane turns its hit words (held in registers) into items — one per hit column (its dot,
// in the record's ascending-tid order) and one per nonzero club / friend intersection — written
// as 16-B entries to a queue in the wave's strip of the (now consumed) hit lists; the wave then
// computes every item's term one per lane, and each lane adds its terms in the reference's order
// (public .. friends, then the common columns ascending, s = 0 terms between).  A wave whose
// items exceed its strip (320) takes fas_epilogue; overflowed hit lists take its record re-walk.
enum : uint32_t { kItemText = 0, kItemClubs = 1, kItemFriends = 2 };

// the candidate's column norm a text item needs (row store), 0 for a set item
__device__ __forceinline__ double item_norm(const DevStore& st, const uint4& it) {
    return (it.w >> 16) == kItemText ? reinterpret_cast<const double*>(st.rows + it.z)[(it.w >> 8) & 0xFFu] : 0.0;
}

__device__ __forceinline__ double item_term(const QConst& q, const uint4& it, double nrm) {
    const uint32_t kind = it.w >> 16;
    if (kind == kItemText) {
        const int t = (int)(it.w & 0xFFu);
        const double dot = __hiloint2double((int)it.y, (int)it.x);
        return dot == 0.0 ? q.sig0_col[t] : text_term(q, t, dot, nrm);
    }
    const bool cl = kind == kItemClubs;  // one inlined chain for both (a call here would spill the loop)
    return set_term_inl(q, cl ? PF_F_CLUBS : PF_F_FRIENDS, (int)it.x, (int)it.y, cl ? q.sqrt_clubs : q.sqrt_friends);
}

__device__ __forceinline__ float pair_epilogue(const QView& v, const DevStore& st, const RowRec& rec, uint64_t ro,
                                               uint32_t len, const uint4& h0, const uint4& h1, const uint4& h2,
                                               uint32_t cnt, uint32_t nh, bool active, uint64_t* tep) {
    const QConst& q = *v.q;
    const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
    const bool overflow = nh > kHitCap;
    uint32_t* hl = reinterpret_cast<uint32_t*>(v.hits);
    const uint32_t nhl = (active && !overflow) ? nh : 0u;
    // the hit words of the lane's LDS hit list (its own walk)
    uint32_t hw[kHitCap];
#pragma unroll
    for (int i = 0; i < (int)kHitCap; ++i) hw[i] = (uint32_t)i < nhl ? hl[i * kPairThreads + threadIdx.x] : 0u;
    auto colw = [](uint32_t w) { return (w >> kTidBits) & 63u; };
    uint32_t ncol = 0;
#pragma unroll
    for (int i = 0; i < (int)kHitCap; ++i)
        ncol += ((uint32_t)i < nhl && (i == 0 || colw(hw[i]) != colw(hw[i > 0 ? i - 1 : 0]))) ? 1u : 0u;
    const uint32_t nc = h2.y, nf = h2.z;
    const int ic = (int)(cnt & 0xFFFFu), ifr = (int)(cnt >> 16);
    const bool dense = active && !overflow;
    const bool club_it = dense && q.n_clubs > 0 && nc > 0 && ic > 0;
    const bool fr_it = dense && q.n_friends > 0 && nf > 0 && ifr > 0;
    const uint32_t nit = dense ? ncol + (club_it ? 1u : 0u) + (fr_it ? 1u : 0u) : 0u;
    uint32_t x = nit;
    x = wave_incl_scan(x);
    const uint32_t base = x - nit, total = wave_last(x);
    constexpr uint32_t kQueue = kHitSlots * 64u / 4u;
    // A wave whose items exceed the queue takes two rounds: the lanes whose items end within it
    // (a prefix of the lanes) first, then the others from the queue's start; only a second round
    // past the queue too takes the per-lane epilogue (r3: 11 % of the waves needed two rounds)
    const uint32_t rnd = x > kQueue ? 1u : 0u;
    const uint64_t r1m = __ballot(rnd != 0u);
    const uint32_t total0 = r1m ? (uint32_t)__shfl((int)base, __ffsll((unsigned long long)r1m) - 1) : total;
    const uint32_t total1 = total - total0;
#ifdef PF_K5_TIMERS
    if (lane == 0) {
        atomicAdd(&g_k1t[9], total1 > kQueue ? 1ull : 0ull);
        atomicAdd(&g_k1t[10], (unsigned long long)total);
        atomicAdd(&g_k1t[11], 1ull);
    }
#endif
    if (total1 > kQueue) {  // (wave-uniform) the per-lane epilogue, hit lists intact
        if (!active) return 0.0f;
        return fas_epilogue<true, true>(v, rec, h0, h1, h2, cnt, threadIdx.x, 1u, [nh](uint32_t) { return nh; }, tep);
    }
    auto item = [&](uint32_t k) {  // 16-B entry k of the wave's strip (rows of 64 words)
        return reinterpret_cast<uint4*>(hl + ((4u * k) >> 6) * kPairThreads + (uint32_t)wv * 64u + ((4u * k) & 63u));
    };
    auto term_at = [&](uint32_t kk) {
        const uint4 it = *item(kk);
        return __hiloint2double((int)it.y, (int)it.x);
    };
    const uint64_t cmask = (uint64_t)h0.x | ((uint64_t)h0.y << 32);
    const uint32_t nbase = (uint32_t)(ro + ((len + 3u) >> 2));  // the record's column norms (uint4 index)
    // every active lane: the fixed terms (an overflowed lane computes its set terms itself)
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
    const bool has_clubs = q.n_clubs > 0 && nc > 0, has_friends = q.n_friends > 0 && nf > 0;
    used += (has_clubs ? 1 : 0) + (has_friends ? 1 : 0);
    uint64_t common = q.colmask & cmask;
    used += __popcll(common);
    const uint32_t rbase = rnd ? base - total0 : base;  // the lane's first item in its round
    const uint32_t nrounds = r1m ? 2u : 1u;
#pragma unroll
    for (uint32_t r = 0; r < 2u; ++r) {
        if (r >= nrounds) break;
        const bool mine = rnd == r;
        wave_sync();  // every lane holds its hit words / the previous round is consumed: the strip is free
        if (mine && nit) {
            uint32_t k = rbase;
            if (club_it) *item(k++) = make_uint4((uint32_t)ic, nc, 0u, kItemClubs << 16);
            if (fr_it) *item(k++) = make_uint4((uint32_t)ifr, nf, 0u, kItemFriends << 16);
            double dot = 0.0;
#pragma unroll
            for (int i = 0; i < (int)kHitCap; ++i) {
                if ((uint32_t)i < nhl) {
                    const uint32_t w = hw[i], col = colw(w);
                    const uint32_t val = probe_p(v, kTagTok | (w & 0xFFFFFFu));
                    const bool first = i == 0 || col != colw(hw[i > 0 ? i - 1 : 0]);
                    dot = (first ? 0.0 : dot) + hit_product(v, val & kTidMask, (int32_t)(w >> 24));
                    const bool last = (uint32_t)(i + 1) == nhl || col != colw(hw[i + 1 < (int)kHitCap ? i + 1 : i]);
                    if (last) {
                        const uint32_t rank = (uint32_t)__popcll(cmask & ((1ull << col) - 1ull));
                        *item(k++) = make_uint4((uint32_t)__double2loint(dot), (uint32_t)__double2hiint(dot), nbase,
                                                (kItemText << 16) | (rank << 8) | col);
                    }
                }
            }
        }
        wave_sync();
        const uint32_t tr = r ? total1 : total0;
        for (uint32_t j = (uint32_t)lane; j < tr; j += 64u) {  // the round's terms, one per lane
            uint4 it = *item(j);
            const double term = item_term(q, it, item_norm(st, it));
            it.x = (uint32_t)__double2loint(term);
            it.y = (uint32_t)__double2hiint(term);
            *item(j) = it;
        }
        wave_sync();
        if (tep && r == 0) tep[0] = clock64();
        if (!mine) continue;
        // the lane's round: clubs, friends, then the common columns ascending (a hit column's term,
        // the items being in column order, else s = 0), recommender_similarity.cpp:80-113
        uint32_t kk = rbase;
        if (has_clubs)
            sum += ic == 0 ? q.sig0_clubs : (overflow ? set_term(q, PF_F_CLUBS, ic, (int)nc, q.sqrt_clubs) : term_at(kk++));
        if (has_friends)
            sum += ifr == 0 ? q.sig0_friends
                            : (overflow ? set_term(q, PF_F_FRIENDS, ifr, (int)nf, q.sqrt_friends) : term_at(kk++));
        if (active && !overflow) {
            // a uniform loop over the query's columns (scalar control, the s = 0 term a broadcast
            // read), adding where the candidate has the column too
            const uint32_t ke = rbase + nit;
            uint32_t nextc = kk < ke ? (item(kk)->w & 0xFFu) : 0xFFu;
            uint64_t qm = __builtin_amdgcn_readfirstlane((uint32_t)q.colmask) |
                          ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(q.colmask >> 32)) << 32);
            while (qm) {
                const uint32_t c = (uint32_t)__ffsll((unsigned long long)qm) - 1u;
                qm &= qm - 1ull;
                const double s0 = q.sig0_col[c];
                if ((common >> c) & 1ull) {
                    if (c == nextc) {
                        sum += term_at(kk++);
                        nextc = kk < ke ? (item(kk)->w & 0xFFu) : 0xFFu;
                    } else {
                        sum += s0;
                    }
                }
            }
        }
    }
    if (tep) tep[1] = clock64();
    // Overflowed hit lists (> kHitCap token hits, ~0.4 % of pairs, a quarter of the waves): the
    // wave walks each such record together, 64 words per round (one coalesced load), and
    // accumulates the hits' products in record order on every lane (the reference's per-column
    // dot order); lane t then computes column t's term, and the owner's sum takes the common
    // columns ascending.
    uint64_t ovm = __ballot(active && overflow);
    while (ovm) {
        const int l = __ffsll((unsigned long long)ovm) - 1;
        ovm &= ovm - 1ull;
        const uint64_t rol = (uint64_t)__shfl((long long)ro, l), cml = (uint64_t)__shfl((long long)cmask, l);
        const uint32_t lenl = (uint32_t)__shfl((int)len, l), nsetl = (uint32_t)__shfl((int)(nc + nf), l);
        const uint32_t* wl = reinterpret_cast<const uint32_t*>(st.rows + rol);
        int cur = -1;
        double dot = 0.0, mydot = 0.0;
        bool myhas = false;
        for (uint32_t b = nsetl; b < lenl; b += 64u) {
            const uint32_t j = b + (uint32_t)lane;
            const uint32_t w = j < lenl ? wl[j] : kPadWord;
            const uint32_t val = j < lenl ? probe_p(v, kTagTok | (w & 0xFFFFFFu)) : 0u;
            const double pr = val != 0u ? hit_product(v, val & kTidMask, (int32_t)(w >> 24)) : 0.0;
            uint64_t hm = __ballot(val != 0u);
            while (hm) {  // the hits in record order
                const int x = __ffsll((unsigned long long)hm) - 1;
                hm &= hm - 1ull;
                const int cx = (int)(((uint32_t)__shfl((int)w, x) >> kTidBits) & 63u);
                const double px = __shfl(pr, x);
                if (cx != cur) {
                    if (cur >= 0 && lane == cur) { mydot = dot; myhas = true; }
                    cur = cx;
                    dot = 0.0;
                }
                dot += px;
            }
        }
        if (cur >= 0 && lane == cur) { mydot = dot; myhas = true; }
        double term = 0.0;
        if (myhas) {
            const double nrm = reinterpret_cast<const double*>(st.rows + rol + ((lenl + 3u) >> 2))
                [__popcll(cml & ((1ull << lane) - 1ull))];
            term = mydot == 0.0 ? q.sig0_col[lane] : text_term(q, lane, mydot, nrm);
        }
        const uint64_t hasm = __ballot(myhas);
        uint64_t cm = q.colmask & cml;
        double sl = __shfl(sum, l);
        while (cm) {
            const int c = __ffsll((unsigned long long)cm) - 1;
            cm &= cm - 1ull;
            const double tc = __shfl(term, c);
            sl += ((hasm >> c) & 1ull) ? tc : q.sig0_col[c];
        }
        if (lane == l) sum = sl;
    }
    if (tep) tep[2] = clock64();
    if (!active || used == 0) return 0.0f;
    // recommender_similarity.cpp:114-123
    const double S = sum / (double)used;
    const double F = (double)used / (double)(kNumFixed + q.n_cols);
    if (S <= 0.0 && F <= 0.0) return 0.0f;
    return (float)((2.0 * S * F) / (S + F));
}

// FAS of slot p by one lane alone (pairs kernel): the lane walks the slot's record in the row
// store (contiguous 16-B steps, so the lane's loads consume whole cache lines), its own hit list
// then holds the whole record's hits in order; the column norms follow the record in the row
// store, so no tile lookup sits in front of them.
// A pair candidate's headers and row offset, loaded before the block stages its image (the loads
// are in flight across the staging round trip and its barrier)
struct PairHdr {
    uint4 h0, h1, h2;
    uint64_t ro;
};
__device__ __forceinline__ PairHdr load_pair_hdr(const DevStore& st, int p, bool active) {
    PairHdr H;
    H.h0 = H.h1 = H.h2 = make_uint4(0, 0, 0, 0);
    H.ro = 0;
    if (active) {
        H.h0 = st.hdr0[p];
        H.h1 = st.hdr1[p];
        H.h2 = st.hdr2[p];
        H.ro = st.row_off[p];
    }
    return H;
}

template <bool PACKED>
__device__ __forceinline__ float fas_slot(const DevStore& st, const QView& v, const PairHdr& H, bool active,
                                          uint64_t* twalk = nullptr) {
    const uint4 h0 = H.h0, h1 = H.h1, h2 = H.h2;
    const uint64_t ro = H.ro;
    const uint32_t nc = h2.y, nset = h2.y + h2.z;
    const uint32_t len = active ? record_words(h2, PACKED) : 0u;
    const RowRec rec{reinterpret_cast<const uint32_t*>(st.rows + ro),
                     reinterpret_cast<const double*>(st.rows + ro + ((len + 3) >> 2))};
    if constexpr (PACKED) {
        const uint32_t pcap = kHitCap * kPairThreads + threadIdx.x;
        RowWalk W{0u, threadIdx.x};
        walk_row(W, st.rows + ro, st.row_pad, len, nc, active ? nset : 0u, v, pcap);
        if (twalk) twalk[0] = clock64();
        // a list that reached kHitCap reads as overflowed (the slow path re-walks the record)
        const uint32_t nh = W.ptr >= pcap ? kHitCap + 1 : (W.ptr - threadIdx.x) / kPairThreads;
        return pair_epilogue(v, st, rec, ro, len, h0, h1, h2, W.cnt, nh, active, twalk ? twalk + 1 : nullptr);
    } else {
        Walk W;
        W.cnt = 0; W.nh = 0; W.pend = 0;
        walk_chunk<false, true, 1>(W, st.rows + ro, 0u, len, nc, nset, v, kPairThreads);
        if (!active) return 0.0f;
        const uint32_t nh = W.nh;
        return fas_epilogue<false>(v, rec, h0, h1, h2, W.cnt, threadIdx.x, 1u, [&](uint32_t) { return nh; });
    }
}

// ---------------------------------------------------------------- LDS staging
__device__ __forceinline__ void stage(void* dst, const void* src, uint32_t bytes) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* s = reinterpret_cast<const uint4*>(src);
    for (uint32_t i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

// The same with every thread's loads of a round (4 per thread) issued before its stores, so a
// round costs one memory round trip (the pair kernel stages a 5-20 KB image per block)
__device__ __forceinline__ void stage4(void* dst, const void* src, uint32_t bytes) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* s = reinterpret_cast<const uint4*>(src);
    const uint32_t n = bytes / 16;
    if (n == 0) return;
    const uint32_t bd = blockDim.x;
    for (uint32_t base = threadIdx.x; base < n; base += 4 * bd) {
        // clamped loads (always in range), guarded stores: four in flight per thread
        const uint32_t i1 = base + bd, i2 = base + 2 * bd, i3 = base + 3 * bd;
        const uint4 r0 = s[base], r1 = s[min(i1, n - 1)], r2 = s[min(i2, n - 1)], r3 = s[min(i3, n - 1)];
        d[base] = r0;
        if (i1 < n) d[i1] = r1;
        if (i2 < n) d[i2] = r2;
        if (i3 < n) d[i3] = r3;
    }
}

// LDS carve: [QConst][tables][vals][hit lists kHitCap x blockDim][merge scratch 2 KiB].
// GTAB = false: the cuckoo table and the token values are staged in LDS, so every probe
// is a ds_read (pointer provenance is the LDS symbol only, never merged with a global
// pointer: a merged pointer would compile to flat loads, whose waits also drain the
// HBM prefetch).  GTAB = true (query too large for LDS): probes read global memory.
template <bool GTAB>
__device__ __forceinline__ QView stage_query(char* smem, const uint8_t* pool, const QImageRef& r, char** scratch) {
    if constexpr (!GTAB) {
        // the sizes from the image in global memory; QConst | tables | values are contiguous in
        // every image pool (tables of >= 2^4 8-B entries keep the values 16-B aligned)
        const uint8_t* base = pool + (size_t)r.const_off * 16u;
        const QConst* g = reinterpret_cast<const QConst*>(base);
        const uint32_t kb = 8u * (g->excl_off + (1u << g->lg_excl)), vb = (uint32_t)g->n_vals * 16u;
        if (r.keys_off == sizeof(QConst) && r.vals_off == r.keys_off + kb) {
            stage4(smem, g, (uint32_t)sizeof(QConst) + kb + vb);
        } else {
            stage4(smem, g, sizeof(QConst));
            stage4(smem + sizeof(QConst), base + r.keys_off, kb);
            stage4(smem + sizeof(QConst) + kb, base + r.vals_off, vb);
        }
    } else {
        stage(smem, pool + (size_t)r.const_off * 16u, sizeof(QConst));
    }
    __syncthreads();
    const QConst* q = reinterpret_cast<const QConst*>(smem);
    // the image's sizes are workgroup-uniform: read into SGPRs (as LDS loads they would sit in a
    // VGPR each for the whole kernel, and the walk loops are register-bound)
    auto uni = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
    QView v;
    v.q = q;
    v.lg = (int)uni((uint32_t)q->lg);
    v.lge = (int)uni((uint32_t)q->lg_excl);
    v.hmul = uni(q->hmul);
    v.excl_off = uni(q->excl_off);
    const uint32_t kb = 8u * (v.excl_off + (1u << v.lge)), vb = uni((uint32_t)q->n_vals) * 16u;
    char* p = smem + sizeof(QConst);
    if constexpr (!GTAB) {
        v.tab = reinterpret_cast<const uint32_t*>(p);
        v.vals = reinterpret_cast<const QVal*>(p + kb);
        p += kb + vb;
    } else {
        v.tab = reinterpret_cast<const uint32_t*>(pool + (size_t)r.const_off * 16u + r.keys_off);
        v.vals = reinterpret_cast<const QVal*>(pool + (size_t)r.const_off * 16u + r.vals_off);
    }
    v.hits = p;
    p += (size_t)uni(q->n_hits_max) * blockDim.x;  // n_hits_max = bytes per lane of the hit list
    v.nh = reinterpret_cast<uint32_t*>(p);     // per-thread hit counts (split records)
    p += 4u * blockDim.x;
    *scratch = p;
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

// the low n bits
__device__ __forceinline__ uint64_t low_bits(uint32_t n) { return n >= 64u ? ~0ull : ((1ull << n) - 1ull); }

// The k smallest keys of nl ascending k-lists (list w at at(w), read with L1-bypassing loads), ascending
// in lanes < k, by one wave.  Any k distinct keys of the lists bound the k-th smallest from above:
// t0 = the smaller of the k-th smallest list head (when there are >= k lists: a wave sort of each
// lane's smallest head) and the smallest k-th key of a list.  Only keys <= t0 are gathered, into buf
// (LDS, 64 keys) while they fit, and sorted once; a list is read only down to its first key past t0.
// (The k-th keys alone bound it loosely: ~450 of a cfg-2 XCD group's 1,280 keys pass.)  More than 64
// such keys take the push path.  The 128 lists of a one-query launch's XCD group went through five
// 64-key sort-and-merge pushes per wave before.
template <class At>
__device__ __forceinline__ uint64_t merge_lists(At at, int nl, int k, uint64_t* buf, int lane) {
    uint64_t tk = ~0ull, hd = ~0ull;
    for (int w = lane; w < nl; w += 64) {
        const uint64_t x = ld_agent(at(w) + k - 1), h = ld_agent(at(w));
        tk = x < tk ? x : tk;
        hd = h < hd ? h : hd;
    }
    uint64_t t0 = wave_min64(tk);
    if (nl >= k) {
        const uint64_t th = rdlane64(wave_sort64(hd, lane), k - 1);
        t0 = th < t0 ? th : t0;
    }
    uint32_t ns = 0;
    for (int w0 = 0; w0 < nl; w0 += 64) {
        const int w = w0 + lane;
        const uint64_t* L = at(min(w, nl - 1));
        for (int e0 = 0; e0 < k; e0 += 4) {
            uint64_t x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = (w < nl && e0 + u < k) ? ld_agent(L + e0 + u) : ~0ull;
            bool more = false;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const bool in = x[u] <= t0 && x[u] != ~0ull;
                const uint64_t m = __ballot(in);
                const uint32_t pos = ns + (uint32_t)__popcll(m & low_bits((uint32_t)lane));
                if (in && pos < 64u) buf[pos] = x[u];
                ns += (uint32_t)__popcll(m);
                more = in;  // the batch's last key in range: the list may hold more below t0
            }
            if (!__ballot(more)) break;  // ascending lists: nothing further down is <= t0
        }
    }
    if (ns <= 64u) return wave_sort64(lane < (int)ns ? buf[lane] : ~0ull, lane);
    uint64_t acc = ~0ull;
    for (int w0 = 0; w0 < nl; w0 += 64) {
        const int w = w0 + lane;
        const uint64_t* L = at(min(w, nl - 1));
        for (int e = 0; e < k; ++e) {
            const uint64_t x = w < nl ? ld_agent(L + e) : ~0ull;
            const bool in = x <= t0 && x != ~0ull;
            if (!__ballot(in)) break;
            topk_push(acc, in ? x : ~0ull, k, lane);
        }
    }
    return acc;
}

// The scans' (K5, K1) fused cross-block merge, in two levels.  The workgroups of group g = bx mod 8 (with the
// round-robin dispatch, the workgroups of one XCD) publish their k-lists and take a ticket on the
// group's counter; the group's last workgroup merges the group's lists into slot nbx + g and takes
// a ticket on the query's counter; the last of those merges the <= 8 group lists into out[row].
// Each counter sees ~nbx / 8 tickets: with one counter for all 1,024 workgroups of a one-query
// launch the tail cost ~15 us of a 185 us launch (r4n, a no-merge build).  After the workgroup's
// own list only wave 0 runs: no barrier on the launch's critical path past the last block.
// parts: per query (nbx + 8) lists of k keys.  sc: LDS for max(nw * k, 64) keys.  Hand-offs
// (pf_device.h take_ticket): a list is published with write-through stores drained before the
// ticket and read with L1-bypassing loads after it.
__device__ __forceinline__ void post_tail(uint64_t list, int k, uint64_t* sc, ScanSync* __restrict__ sync,
                                          uint64_t* __restrict__ parts, uint64_t* __restrict__ out,
                                          const int32_t* __restrict__ out_rows, int qy, int bx, int nbx) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
    __syncthreads();
    if (lane < k) sc[wave * k + lane] = list;
    __syncthreads();
    if (wave != 0) return;
    ScanSync* sy = sync + qy;
    uint64_t* qparts = parts + (size_t)qy * (nbx + 8) * k;
    const int ng = min(8, nbx), g = bx % ng, n_g = (nbx - g + ng - 1) / ng;
    uint64_t acc;
    {  // the workgroup's list: its waves' lists (one sort when they fit a wave)
        const int n = nw * k;
        if (n <= 64) {
            acc = wave_sort64(lane < n ? sc[lane] : ~0ull, lane);
        } else {
            acc = ~0ull;
            for (int b = 0; b < n; b += 64) topk_push(acc, b + lane < n ? sc[b + lane] : ~0ull, k, lane);
        }
    }
    if (lane < k) st_agent(qparts + (size_t)bx * k + lane, acc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // program order: stores, wait, ticket
    unsigned t = 0;
    if (lane == 0) t = take_ticket(&sy->grp[g * 16]);
    t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
    if (t != (unsigned)n_g - 1u) return;
    ticket_acquire();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    // the group's lists: workgroups g, g + ng, ...
    acc = merge_lists([&](int w) { return qparts + (size_t)(g + w * ng) * k; }, n_g, k, sc, lane);
    if (lane < k) st_agent(qparts + (size_t)(nbx + g) * k + lane, acc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    t = 0;
    if (lane == 0) t = take_ticket(&sy->done);
    t = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
    if (t != (unsigned)ng - 1u) return;
    ticket_acquire();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint64_t fin = merge_lists([&](int w) { return qparts + (size_t)(nbx + w) * k; }, ng, k, sc, lane);
    const int row = out_rows ? out_rows[qy] : qy;
    if (lane < k) out[(size_t)row * k + lane] = fin;
    // the query's rendezvous left zeroed for the next launch that uses it (a one-query launch from
    // the resident images reuses its lane's ScanSync with no upload): every workgroup of the query
    // took its group ticket after its last block claim, and every group its done ticket, so nothing
    // reads, claims or counts from it any more (plain vector stores; the next launch sees them)
    uint4* z = reinterpret_cast<uint4*>(sy);
    for (int i = lane; i < (int)(sizeof(ScanSync) / 16); i += 64) z[i] = make_uint4(0u, 0u, 0u, 0u);
}

template <bool PACKED, bool GTAB>
__global__ __launch_bounds__(kScanThreads, 4) void fas_scan_kernel(DevStore st, const uint8_t* __restrict__ pool,
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
    // Tile hand-out, longest tiles first.  Static zig-zag for all but the last two bands
    // (band b = tiles [b*W, (b+1)*W) holds W near-equal tiles; wave w takes one per band,
    // alternating direction), then the tail from per-XCD counters, so waves that drew
    // cheap tiles (few hits) take more.  One shared counter for every tile serialises at
    // ~13 ns per fetch and halved the streaming rate; per-XCD counters on the last
    // bands only keep the fetches few and uncontended.
    const int W = (int)gridDim.x * (kScanThreads / 64), wid = (int)blockIdx.x * (kScanThreads / 64) + wave;
    const int ntiles = tile_end - tile_begin;
    const int nstatic = max(0, ntiles / W - 2) * W;
    // blocks are dispatched to the 8 XCDs round-robin; with fewer than 8 blocks every
    // group still has one, so every residue class of the tail is drained
    const int ngrp = min(8, (int)gridDim.x), xcd = (int)blockIdx.x % ngrp;
    unsigned* xctr = &sync[blockIdx.y].xcd_next[xcd * 16];
    for (int b = 0;; ++b) {
        int tile;
        if (b * W < nstatic) {
            tile = tile_begin + b * W + ((b & 1) ? W - 1 - wid : wid);
        } else {
            unsigned t = 0;
            if (lane == 0) t = atomicAdd(xctr, 1u);
            t = __builtin_amdgcn_readfirstlane(t);
            tile = tile_begin + nstatic + (int)t * ngrp + xcd;  // group x drains tail tiles = x (mod ngrp)
        }
        if (tile >= tile_end) break;
        const uint32_t lgk = st.tile_lgk[tile];
        const int slot0 = (int)st.tile_slot0[tile];
        const int cand = lane >> lgk, ci = lane & ((1 << lgk) - 1);
        const bool active = cand < min(kTileSlots >> lgk, st.n_slots - slot0);
        const int p = slot0 + cand;
        // h0 / h1 are loaded after the walk (the epilogue's first reads): holding them across the
        // walk's double buffer spilled registers
        uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0, h2 = h0;
        if (active) h2 = st.hdr2[p];
        const uint32_t nc = h2.y, nset = h2.y + h2.z;
        const uint32_t len = record_words(h2, PACKED);
        const uint32_t q = chunk_words(len, lgk, PACKED);
        const uint32_t j0 = (uint32_t)ci * q;
        const uint32_t clen = (active && len > j0) ? min(q, len - j0) : 0u;
        const Loc l{tile, cand, lgk};
        Walk W;
        W.cnt = 0; W.nh = 0; W.pend = 0;
        if (!PACKED && clen > 0 && j0 > 0) W.pend = word_at(st, l, q, j0 - 1);  // a token pair may straddle chunks
        walk_chunk<PACKED, false>(W, st.stream + st.tile_off[tile] + lane, j0, clen, nc, nset, v, blockDim.x);
        // one epilogue site (a second inlined copy for split records cost K1 64 B of scratch per
        // lane): a split record sums its chunk counters over its lanes, publishes the hit counts,
        // and its first lane finishes it; a whole record (lgk = 0) is the one-chunk case
        if (active) {
            h0 = st.hdr0[p];
            h1 = st.hdr1[p];
        }
        float f = 0.0f;
        uint32_t cnt = W.cnt;
        for (int m = 1; m < (1 << lgk); m <<= 1) cnt += (uint32_t)__shfl_xor((int)cnt, m);
        v.nh[threadIdx.x] = W.nh;
        __builtin_amdgcn_wave_barrier();
        if (active && ci == 0) {
            const uint32_t* nhp = v.nh + threadIdx.x;
            const TileRec rec{&st, l, q};
            f = fas_epilogue<PACKED>(v, rec, h0, h1, h2, cnt, threadIdx.x, 1u << lgk, [&](uint32_t g) { return nhp[g]; });
        }
        uint64_t key = ~0ull;
        if (active && ci == 0) {
            const int32_t uid = (int32_t)h1.w;
            if (!excluded<PACKED>(v, (uint32_t)uid)) key = score_key(f, uid);
        }
        topk_push(list, key, k, lane);
    }
    post_tail(list, k, reinterpret_cast<uint64_t*>(scratch), sync, parts, out,
              out_rows, (int)blockIdx.y, (int)blockIdx.x, (int)gridDim.x);
}

// ---------------------------------------------------------------- K5: postings scan
// All-candidates FAS (A13) through the postings store (pf_types.h): a workgroup scores one
// block of kBlockCands (512) consecutive candidates at a time (thread i owns candidates i and
// i + 256) from the lists the query names, never the candidates' records:
//   1. ranges: every list's sub-range for this block (one cell lookup per list);
//   2. sets: club / friend list entries add their multiplicity to per-candidate LDS
//      counters (integer, order-free) and the exclusion list marks adj[q] + {q};
//   3. fixed terms (public .. friends) per owned candidate from its 32-B header;
//   4. text, in ROUNDS of <= 64 query tokens (whole columns where they fit, the columns in
//      ascending order) whose list entries in the block fit the round's kRoundCap hit slots:
//      a. walk: every entry of the round's lists, flattened over the workgroup (all loads in
//         flight at once), sets bit (token - round start) of its candidate's 64-bit hit mask;
//      b. slots: each wave gives its candidates' hits a contiguous range of hit slots, a
//         candidate's hits in token order (= column, then tid ascending);
//      c. place: every entry writes its tf and token into its slot (the slot index is the
//         popcount of the mask below its bit), and the first hit of a column its
//         (candidate, column) norm;
//      d. terms, wave-dense: one lane per (candidate, column) item sums the products of its
//         hits in ascending tid order (recommender.cpp:74-85) and computes the cosine ->
//         sigmoid term (recommender_similarity.cpp:93-113), so the FP64 divisions and exp
//         run on as many lanes as there are items, not once per column for the whole wave;
//      e. the owners add, in the reference's order, each common column's term, or its s = 0
//         term when the candidate has no hit in it.
//      A column longer than a round (> 64 tokens, or more entries than kRoundCap) is split
//      over rounds; its owners carry the dot in registers and compute its term themselves.
//   5. FAS (recommender_similarity.cpp:114-123), idx-keyed wave top-k, fused cross-block merge.
// A block costs 2 + 4 x rounds barriers and one memory round trip per round (the walk); the
// round-1 design paid two barriers and a round trip per 8-token pass (21.6 passes per block).

// A query token in LDS: its weight and idf (the product wq * (tf * idf), recommender.cpp:74-85)
struct PTok {
    double wq, idf;
};

// LDS carve of the fixed part (after QConst)
constexpr uint32_t kLdsMask = 0;                                          // u64 [kBlockCands] hit masks
constexpr uint32_t kLdsSlot = kLdsMask + 8 * kBlockCands;                 // f64 [kRoundCap] norm -> term
constexpr uint32_t kLdsHit = kLdsSlot + 8 * kRoundCap;                    // u16 [kRoundCap] hits
constexpr uint32_t kLdsHbase = kLdsHit + 2 * kRoundCap;                   // u16 [kBlockCands] first slot
// the set counters and exclusion bits are read by the fixed terms only, before any thread passes
// round 0's walk barrier and writes a slot: they live in the slots
constexpr uint32_t kLdsCnt = kLdsSlot;                                    // u32 [kBlockCands] set counters
constexpr uint32_t kLdsExb = kLdsCnt + 4 * kBlockCands;                   // u32 [kBlockCands / 32] excluded
static_assert(4 * kBlockCands + 4 * (kBlockCands / 32) <= 8 * kRoundCap, "set counters alias the slots");
constexpr uint32_t kLdsItem = kLdsHbase + 2 * kBlockCands;                // u16 [kRoundCap] term items
constexpr uint32_t kLdsMisc = (kLdsItem + 2 * kRoundCap + 15) & ~15u;       // u32 [16]
constexpr uint32_t kLdsCols = kLdsMisc + 64;                              // QCol [kPostMaxCols]
constexpr uint32_t kLdsFtab = kLdsCols + 16 * kPostMaxCols;               // f64 [7 + 48 + 1] F by used
constexpr uint32_t kLdsSeg = kLdsFtab + 8 * (kNumFixed + kPostMaxCols + 1);  // u32 [kRoundToks] token segments
constexpr uint32_t kLdsCidx = kLdsSeg + 4 * kRoundToks;                   // end of the fixed tables
// round list maps, two buffers (the next round's is built during this one): flat entry f < kRoundCap
// -> its list without a search (bits of the nonempty lists' starts, nonempty lists before each
// 64-entry word, and per nonempty list {entry index of flat 0, token - round start})
constexpr uint32_t kMapWords = kRoundCap / 64;
constexpr uint32_t kLdsMapB = (kLdsCidx + 7) & ~7u;                            // u64 [2][kMapWords]
constexpr uint32_t kLdsMapN = kLdsMapB + 2 * 8 * kMapWords;                   // uint2 [2][kRoundToks]
constexpr uint32_t kLdsMapC = kLdsMapN + 2 * 8 * kRoundToks;                  // u8 [2][kMapWords]
// per column number of the current round: the round-relative tokens before its end (a mask); per
// active column index c: the column numbers of active columns < c as a mask (a round's columns
// [ca, ce) = cpre[ce] & ~cpre[ca])
constexpr uint32_t kLdsLmk = (kLdsMapC + 2 * kMapWords + 7) & ~7u;            // u64 [kPostMaxCols]
constexpr uint32_t kLdsCpre = kLdsLmk + 8 * kPostMaxCols;                     // u64 [kPostMaxCols + 1]
constexpr uint32_t kPostFixedLds = (kLdsCpre + 8 * (kPostMaxCols + 1) + 15) & ~15u;
static_assert(kBlockCands == 2 * kPostThreads, "two candidates per thread");
static_assert(kRoundCap < 65536 && kBlockCands <= kRoundCap, "u16 slots; a one-token round fits");
static_assert(kPostWaves * kMaxTopK * 8 + 16 + 4 * kMaxTopK <= 8 * kRoundCap, "post_tail scratch in the slots");

// hit slot: tf | token - round start << 8 | first hit of its column segment | first hit of its candidate
constexpr uint32_t kHitFirst = 1u << 14;
constexpr uint32_t kHitCand = 1u << 15;
// token segment (per token of a round): segment start | end << 8 (round-relative) | column << 16 |
// split (the column spans several rounds) << 24
constexpr uint32_t kSegSplit = 1u << 24;

#ifdef PF_K5_CHECK
// checked build (tools/build_variant.sh k5chk XFLAGS=-DPF_K5_CHECK): every global index of K5 is
// range-checked; a bad one is reported and replaced by 0 instead of faulting
__device__ __forceinline__ uint32_t k5_chk(uint32_t i, uint32_t n, int what) {
    if (i >= n) {
        printf("K5 CHECK %d: index %u >= %u (block %d thread %d)\n", what, i, n, (int)blockIdx.x, (int)threadIdx.x);
        return 0u;
    }
    return i;
}
#define K5CHK(i, n, w) k5_chk((i), (n), (w))
#else
#define K5CHK(i, n, w) (i)
#endif


// entries of list L for candidates [c0, c1] (cells c0 >> shift .. c1 >> shift)
__device__ __forceinline__ uint2 list_range(const PostStore& ps, const PList& L, uint32_t c0, uint32_t c1) {
    return make_uint2(L.off + ps.cells[K5CHK(L.cell_off + (c0 >> L.shift), ps.n_cells, 1)],
                      L.off + ps.cells[K5CHK(L.cell_off + (c1 >> L.shift) + 1, ps.n_cells, 2)]);
}

// the set list of flat entry f < spre[n]: the last j with spre[j] <= f (a nonempty one)
__device__ __forceinline__ int set_list(const uint32_t* spre, int n, uint32_t f) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (spre[mid] <= f) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// gpre[j] = sum of the lengths of ranges 0 .. j-1 (j <= nl), by one wave
__device__ __forceinline__ void wave_prefix(uint32_t* gpre, const uint2* rng, int nl, int lane) {
    uint32_t carry = 0;
    for (int b = 0; b < nl; b += 64) {
        const int j = b + lane;
        const uint32_t len = j < nl ? rng[j].y - rng[j].x : 0u;
        uint32_t x = len;
        x = wave_incl_scan(x);
        if (j < nl) gpre[j] = carry + x - len;
        carry += wave_last(x);
    }
    if (lane == 0) gpre[nl] = carry;
}

// the list of flat round entry g (gpre[ja] <= g < gpre[jb], jb - ja <= 64): the last list
// starting at or before g, branch-free (a probe past the round reads gpre[jb] > g)
__device__ __forceinline__ int round_list(const uint32_t* gpre, int ja, int jb, uint32_t g) {
    int j = ja;
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) j += gpre[min(j + s, jb)] <= g ? s : 0;
    return j;
}

// The list map of round [ja, jb) into buffer (mb, mc, mn), by one wave (lane = its lane): bit
// s_j of mb for each list j whose entries start at flat s_j < kRoundCap and are nonempty, mc[w] =
// such lists starting before word w, mn[k] = the k-th one's {entry index of flat 0, j - ja}.
template <int CAP = kRoundCap>
__device__ __forceinline__ void build_map(uint64_t* mb, uint8_t* mc, uint2* mn, const uint32_t* gpre,
                                          const uint2* rng, int ja, int jb, int lane) {
    constexpr int kMW = CAP / 64;
    const uint32_t g0 = gpre[ja];
    const int j = ja + lane;
    uint32_t s = 0;
    bool ne = false;
    if (j < jb) {
        s = gpre[j] - g0;
        ne = gpre[j + 1] - g0 > s && s < (uint32_t)CAP;
    }
    if (lane < kMW) mb[lane] = 0ull;
    const uint64_t bal = __ballot(ne);
    const uint32_t k = (uint32_t)__popcll(bal & low_bits((uint32_t)lane));
    wave_sync();
    if (ne) {
        atomicOr(reinterpret_cast<unsigned long long*>(&mb[s >> 6]), 1ull << (s & 63u));
        mn[k] = make_uint2(rng[j].x - s, (uint32_t)lane);
    }
    wave_sync();
    const uint32_t c = lane < kMW ? (uint32_t)__popcll(mb[lane]) : 0u, x = wave_incl_scan(c);
    if (lane < kMW) mc[lane] = (uint8_t)(x - c);
}

// A term item: the slot of a (candidate, column)'s first hit in the round and the column's hit
// count there (kItemRunMax: count the run by the hit flags instead)
constexpr uint32_t kItemRunShift = 11, kItemSlotMask = (1u << kItemRunShift) - 1u, kItemRunMax = 31;
static_assert(kRoundCap <= (int)kItemSlotMask + 1, "item slots fit 11 bits");
// hits of a candidate's column segment [lo, hi) of the round (its mask's bits there), capped
__device__ __forceinline__ uint32_t hit_run(uint64_t m, uint32_t lo, uint32_t hi) {
    return min((uint32_t)__popcll((m >> lo) & low_bits(hi - lo)), kItemRunMax);
}
// dot + slot[r + 1] + ... + slot[r + run - 1], added in that order (recommender.cpp:74-85 sums a
// column's products one by one): the reads are independent, four issued ahead of the adds
__device__ __forceinline__ double run_dot(const double* slot, uint32_t r, uint32_t run, double dot) {
    for (uint32_t k = 1; k < run; k += 4) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = k + u < run ? slot[r + k + u] : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k + u < run) dot += v[u];
    }
    return dot;
}

// product of one shared token, recommender.cpp:74-85: wA * wB, wB = tf * idf
__device__ __forceinline__ double tok_product(const PTok* pt, int j, uint32_t tf) {
    const PTok v = pt[j];
    return v.wq * ((double)tf * v.idf);
}

// The next round from (column ci, token jcur): tokens [ja, jb), columns [ca, ce) touched (ce - 1
// is left unfinished when ci_next == ce - 1).  Greedy: whole columns while the round holds <= 64
// tokens and <= kRoundCap entries; a column that does not fit an empty round is split (at least
// one token, whose entries in the block are <= kBlockCands hits).
struct Round {
    int ja, jb, ca, ce;
};
template <int CAP = kRoundCap>
__device__ __forceinline__ Round next_round(const QCol* scol, const uint32_t* gpre, int n_act, int& ci, int& jcur) {
    Round r;
    r.ja = jcur;
    r.jb = jcur;
    r.ca = ci;
    const uint32_t g0 = gpre[r.ja];
    while (ci < n_act) {
        const int j1 = scol[ci].j1;
        if (j1 - r.ja <= kRoundToks && gpre[j1] - g0 <= (uint32_t)CAP) {
            r.jb = j1;
            ++ci;
            continue;
        }
        if (r.jb == r.ja) {
            int jb = r.ja + 1;
            const int lim = min(j1, r.ja + kRoundToks);
            while (jb < lim && gpre[jb + 1] - g0 <= (uint32_t)CAP) ++jb;
            r.jb = jb;
            if (jb == j1) ++ci;
        }
        break;
    }
    jcur = r.jb;
    r.ce = (ci < n_act && scol[ci].j0 < r.jb) ? ci + 1 : ci;
    return r;
}

#ifdef PF_K5_TIMERS
// profiling build only (make K5T=1): per-phase clock64() sums over every wave, printed by
// launch_post every 10th launch
#define K5T(slot) do { const uint64_t t_ = clock64(); tacc[slot] += t_ - tprev; tprev = t_; } while (0)
#else
#define K5T(slot) do { } while (0)
#endif

#ifndef PF_K5_MINB
#define PF_K5_MINB 4  // workgroups per CU the register budget is sized for (LDS allows 4 for most queries)
#endif
__global__ __launch_bounds__(kPostThreads, PF_K5_MINB) void fas_post_kernel(PostStore ps, const uint8_t* __restrict__ pool,
                                                              const uint32_t* __restrict__ img_off, int32_t blk_begin,
                                                              int32_t blk_end, int32_t k, uint64_t* __restrict__ parts,
                                                              ScanSync* __restrict__ sync, uint64_t* __restrict__ out,
                                                              const int32_t* __restrict__ out_rows, uint32_t mode,
                                                              uint32_t tail_bs, const uint8_t* __restrict__ qconst) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // mode bit 1 (batches): the grid is transposed, blockIdx.x = the query and blockIdx.y = the block
    // group, so the workgroups resident at once are many queries on the same candidate blocks and
    // the lists they share (popular tokens, clubs) are read from HBM once and then served by L2
    const bool tr = (mode & 2u) != 0u;
    const int qy = tr ? (int)blockIdx.x : (int)blockIdx.y;
    const int bx = tr ? (int)blockIdx.y : (int)blockIdx.x;
    const int nbx = tr ? (int)gridDim.y : (int)gridDim.x;
    const uint8_t* img = pool + img_off[qy];
    // the query's QConst: the image's own prefix, or (qconst given: one-query launches from the
    // resident images) the job pipeline's resident K1' image of the same user, whose QConst K6
    // builds from the same tables; the image's own part then starts sizeof(QConst) past img
    const uint8_t* qcp = qconst ? qconst : img;
    const QPostHead H = *reinterpret_cast<const QPostHead*>(img + sizeof(QConst));
    const QTok* toks = reinterpret_cast<const QTok*>(img + H.tok_off);
    const QCol* cols = reinterpret_cast<const QCol*>(img + H.col_off);
    const PList* sets = reinterpret_cast<const PList*>(img + H.set_off);
    const uint32_t* excl = reinterpret_cast<const uint32_t*>(img + H.excl_off);
    const int tid = (int)threadIdx.x, lane = tid & 63;
    char* base = smem + sizeof(QConst);
    uint64_t* mask = reinterpret_cast<uint64_t*>(base + kLdsMask);
    double* slot = reinterpret_cast<double*>(base + kLdsSlot);
    uint16_t* hit = reinterpret_cast<uint16_t*>(base + kLdsHit);
    uint16_t* hbase = reinterpret_cast<uint16_t*>(base + kLdsHbase);
    uint16_t* item = reinterpret_cast<uint16_t*>(base + kLdsItem);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(base + kLdsCnt);
    uint32_t* exb = reinterpret_cast<uint32_t*>(base + kLdsExb);
    uint32_t* misc = reinterpret_cast<uint32_t*>(base + kLdsMisc);  // [0] next block, [1] hit slots taken
    QCol* scol = reinterpret_cast<QCol*>(base + kLdsCols);
    double* ftab = reinterpret_cast<double*>(base + kLdsFtab);  // F = used / (7 + T) by used
    uint32_t* seg = reinterpret_cast<uint32_t*>(base + kLdsSeg);
    const int nsets = H.n_club + H.n_friend;
    const int nl = H.n_tok + nsets;
    PTok* pt = reinterpret_cast<PTok*>(base + kPostFixedLds);
    // (the list descriptors are not staged: each block reads them from the image, an L2 hit, so a
    // query with ~200 tokens still fits four workgroups per CU)
    uint2* rng = reinterpret_cast<uint2*>(pt + H.n_tok);
    uint2* rtab = rng + nl;  // the block's rounds (ja | jb << 16, ca | ce << 16), <= n_tok of them
    uint32_t* gpre = reinterpret_cast<uint32_t*>(rtab + H.n_tok + 1);
    uint32_t* spre = gpre + H.n_tok + 1;  // the set lists' prefix [nsets + 1]
    uint8_t* colof = reinterpret_cast<uint8_t*>(spre + nsets + 1);  // token -> active column index
    uint64_t* mapb = reinterpret_cast<uint64_t*>(base + kLdsMapB);
    uint2* mapn = reinterpret_cast<uint2*>(base + kLdsMapN);
    uint8_t* mapc = reinterpret_cast<uint8_t*>(base + kLdsMapC);
    uint64_t* lmk = reinterpret_cast<uint64_t*>(base + kLdsLmk);
    uint64_t* cpre = reinterpret_cast<uint64_t*>(base + kLdsCpre);
    stage(smem, qcp, sizeof(QConst));
    for (int j = tid; j < H.n_act; j += kPostThreads) {
        const QCol c = cols[j];
        scol[j] = c;
        for (int x = c.j0; x < c.j1; ++x) colof[x] = (uint8_t)j;
    }
    if (tid == 0) {  // prefix masks of the active columns (<= 48, ascending)
        uint64_t m = 0;
        for (int j = 0; j < H.n_act; ++j) { cpre[j] = m; m |= 1ull << cols[j].t; }
        cpre[H.n_act] = m;
    }
    for (int j = tid; j <= kNumFixed + kPostMaxCols; j += kPostThreads)
        ftab[j] = (double)j / (double)(kNumFixed + reinterpret_cast<const QConst*>(qcp)->n_cols);
    for (int j = tid; j < H.n_tok; j += kPostThreads) {
        const QTok t = toks[j];
        pt[j] = PTok{t.wq, t.idf};
    }
    __syncthreads();  // the staged tables are read by other threads
    const QConst& q = *reinterpret_cast<const QConst*>(smem);
    uint64_t best = ~0ull;
#ifdef PF_K5_TIMERS
    uint64_t tacc[14] = {0};
    uint64_t tprev = clock64();
    const uint64_t tstart = tprev;
#endif
    // Blocks: the workgroup's own first block, then either every gridDim.x-th block (static)
    // or (mode bit 0) the next unclaimed block of the query from a counter in its ScanSync, so the
    // blocks past the first resident round go to the workgroups that finish first.
    unsigned int* next_blk = &sync[qy].next;
    // dynamic mode (one query): whole static rounds of nbx blocks, then the rest of the range by
    // claim, in blocks of tail_bs candidates: the ~117 blocks past three static rounds of a cfg-2
    // launch would run on ~11 % of the workgroups; cut four times finer they spread over ~470
    const int tail = (mode & 1u) ? blk_begin + max(1, (blk_end - blk_begin) / nbx) * nbx : blk_end;
    const uint32_t B = (uint32_t)ps.bsize;
    const uint32_t cend = min((uint32_t)blk_end * B, (uint32_t)ps.n);  // the range's end
    // (mode bit 3 counts every block in whole B-candidate blocks: finer tail blocks apply to the
    // static-rounds mode only)
    const uint32_t tbs = (tail_bs > 0u && tail_bs < B && !(mode & 8u)) ? tail_bs : B;
    const uint32_t cst = min((uint32_t)tail * B, cend);                 // the claimed part's start
    int blk_last = tail + (int)((cend - cst + tbs - 1) / tbs);
    const bool short_excl = H.n_excl <= kPostThreads;
    const uint32_t ex0 = short_excl && H.n_excl > 0 ? excl[min(tid, H.n_excl - 1)] : ~0u;  // the query's, once
    // mode bit 2 (one query, query-major batches): the workgroups of XCD x (bx mod 8 under the
    // round-robin dispatch when nbx is a multiple of 8) take blocks [x nbx/8, (x + 1) nbx/8) of each
    // static round, so a list segment's boundary cache lines are shared inside one L2 instead of
    // fetched by two XCDs (cfg 2 PMC traffic 236 -> 175 MB per launch, r4w -> r5h)
    const int pb = ((mode & 4u) && (nbx & 7) == 0) ? (bx & 7) * (nbx >> 3) + (bx >> 3) : bx;
    // mode bit 3 (one query): every block claimed, per group g = bx mod 8 (with round-robin dispatch,
    // one XCD) from a contiguous eighth of the range, in order, from the group's own counter.  The
    // workgroups dispatched last (the third and fourth of a CU) lose VALU arbitration to the older
    // ones by age and ran their static blocks ~25 % slower every round (r6j block log): claimed
    // blocks let the faster workgroups take more.  The next block is claimed at the start of a
    // block's last text round, so the claim's round trip hides behind that round.
    const bool xdyn = (mode & 8u) != 0u;
    const int xng = min(8, nbx), xg = bx % xng;
    const int x_lo = blk_begin + (int)((int64_t)(blk_end - blk_begin) * xg / xng);
    const int x_hi = blk_begin + (int)((int64_t)(blk_end - blk_begin) * (xg + 1) / xng);
    const int x_nwg = (nbx - xg + xng - 1) / xng;
    unsigned int* xctr = &sync[qy].xcd_next[xg * 16];
    if (xdyn) blk_last = x_hi;
    for (int blk = xdyn ? x_lo + bx / xng : blk_begin + pb; blk < blk_last;) {
        unsigned int xclaim = 0;
        const uint32_t bsz = blk < tail ? B : tbs;  // this block's candidates
        const uint32_t c0 = blk < tail ? (uint32_t)blk * B : cst + (uint32_t)(blk - tail) * tbs;
        const uint32_t c1 = min(c0 + bsz, cend) - 1;  // last candidate of the block
#ifdef PF_K5_BLOCKLOG
        const unsigned long long blog_t0 = __builtin_amdgcn_s_memrealtime();
#endif
        // 1. headers of the owned candidates and every list's range in this block: all loads
        // issued before the first wait, one memory round trip.  (Loading the next static block's
        // headers and ranges before this block's FAS measured slower: 184.8 -> 188.0 us, r4n,
        // the 16 registers they hold spilled)
        uint4 ha[kCandsPerThread], hb[kCandsPerThread];
#pragma unroll
        for (int kk = 0; kk < kCandsPerThread; ++kk) {  // clamped (always valid) index, zeroed below
            const uint32_t c = min(c0 + kk * kPostThreads + tid, c1);
            ha[kk] = ps.hdr[2 * (size_t)c];
            hb[kk] = ps.hdr[2 * (size_t)c + 1];
        }
        for (int j = tid; j < nl; j += kPostThreads)
            rng[j] = list_range(ps, j < H.n_tok ? toks[j].l : sets[j - H.n_tok], c0, c1);
#pragma unroll
        for (int kk = 0; kk < kCandsPerThread; ++kk) {
            const uint32_t c = c0 + kk * kPostThreads + tid;
            if (!(c <= c1 && (uint32_t)(kk * kPostThreads + tid) < bsz)) {
                ha[kk] = make_uint4(0, 0, 0, 0);
                hb[kk] = make_uint4(0, 0, 0, 0);
            }
            cnt[kk * kPostThreads + tid] = 0u;
            mask[kk * kPostThreads + tid] = 0ull;
        }
        if (tid < kBlockCands / 32) exb[tid] = 0u;
        K5T(0);
        __syncthreads();
        K5T(1);
        if (tid < 64) {  // read after the barrier below
            wave_prefix(gpre, rng, H.n_tok, lane);
            wave_sync();
            // the block's rounds, once (every thread used to walk the columns' prefix chain per round)
            {
                int ci0 = 0, j0 = 0, nr = 0;
                while (ci0 < H.n_act) {
                    const Round Rr = next_round(scol, gpre, H.n_act, ci0, j0);
                    if (lane == 0)
                        rtab[nr] = make_uint2((uint32_t)Rr.ja | (uint32_t)Rr.jb << 16, (uint32_t)Rr.ca | (uint32_t)Rr.ce << 16);
                    if (nr == 0) build_map(mapb, mapc, mapn, gpre, rng, Rr.ja, Rr.jb, lane);
                    ++nr;
                }
                if (lane == 0) misc[3] = (uint32_t)nr;
            }
        }
        // exclusion list (sorted idx of adj[q] + {q}): whole list when short (loaded above, no
        // barrier of its own), else bisect and walk until past the block
        if (short_excl) {
            const uint32_t p = ex0 - c0;
            if (tid < H.n_excl && p < bsz) atomicOr(&exb[p >> 5], 1u << (p & 31));
        } else {
            uint32_t lo = 0, hi = (uint32_t)H.n_excl;
            while (lo < hi) {  // first entry >= c0
                const uint32_t mid = (lo + hi) >> 1;
                if (excl[mid] < c0) lo = mid + 1; else hi = mid;
            }
            hi = (uint32_t)H.n_excl;
            for (uint32_t b = lo; b < hi; b += kPostThreads) {
                const uint32_t x = b + tid;
                const uint32_t e = x < hi ? excl[x] : ~0u;
                const uint32_t p = e - c0;
                if (p < bsz) atomicOr(&exb[p >> 5], 1u << (p & 31));
                if (__syncthreads_or(e >= c0 + bsz)) break;  // sorted: the rest lies beyond the block
            }
        }
        // 2. clubs / friends, by waves 1-3 while wave 0 plans the rounds: each computes the set
        // lists' prefix itself (the same values, so no barrier) and takes flat entries by bisection
        // (the round-4 walk scanned every set list per entry group on every thread: 17 us of a
        // cfg-2 launch, r6l)
        if (tid >= 64 && nsets > 0) {
            wave_prefix(spre, rng + H.n_tok, nsets, lane);
            wave_sync();
            const uint32_t tot = spre[nsets];
            constexpr uint32_t kSetThreads = kPostThreads - 64;
            for (uint32_t f0 = (uint32_t)tid - 64u; f0 < tot; f0 += 2u * kSetThreads) {
                int js[2];
                uint32_t e[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint32_t f = f0 + u * kSetThreads;
                    js[u] = f < tot ? set_list(spre, nsets, f) : -1;
                    e[u] = js[u] >= 0 ? ps.post[K5CHK(rng[H.n_tok + js[u]].x + (f - spre[js[u]]), ps.n_post, 3)] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint32_t p = (e[u] >> 8) - c0;
                    if (js[u] >= 0 && p < bsz) atomicAdd(&cnt[p], (e[u] & 0xFFu) << (js[u] < H.n_club ? 0 : 16));
                }
            }
        }
        K5T(2);
        __syncthreads();
        K5T(1);
        // 3. fixed terms, recommender_similarity.cpp:38-91
        double sum[kCandsPerThread];
        uint32_t used = 0;  // byte kk: terms used by candidate kk (<= 7 + 48)
        uint64_t pend[kCandsPerThread];
        uint32_t skip = 0;  // bit kk: candidate kk absent or excluded
#pragma unroll
        for (int kk = 0; kk < kCandsPerThread; ++kk) {
            const int p = kk * kPostThreads + tid;
            const uint32_t ct = cnt[p];
            if ((uint32_t)p >= bsz || c0 + p > c1 || ((exb[p >> 5] >> (p & 31)) & 1u)) skip |= 1u << kk;
            const uint64_t cm = (uint64_t)ha[kk].x | ((uint64_t)(ha[kk].y & 0xFFFFu) << 32);
            pend[kk] = cm & q.colmask;
            double s = 0.0;
            int u = 0;
            const uint32_t pb = (ha[kk].y >> 16) & 0xFFu, gb = ha[kk].y >> 24;
            if (q.pubcode != kCodeMissing && pb != kCodeMissing) { s += q.sig_pub[pb == q.pubcode]; ++u; }
            if (q.gencode != kCodeMissing && gb != kCodeMissing) { s += q.sig_gen[gb == q.gencode]; ++u; }
            const int cb = (int)(int16_t)(ha[kk].z & 0xFFFFu), ab = (int)(int16_t)(ha[kk].z >> 16);
            if (q.comp > 0 && cb > 0) { s += cb <= kValTab ? q.sig_comp[cb] : ratio_term(q, PF_F_COMPLETION, q.comp, cb); ++u; }
            if (q.age > 0 && ab > 0) { s += ab <= kValTab ? q.sig_age[ab] : ratio_term(q, PF_F_AGE, q.age, ab); ++u; }
            const int r0 = (int)hb[kk].x, r1 = (int)hb[kk].y, r2 = (int)hb[kk].z;
            const int bcnt = (r0 >= 0) + (r1 >= 0) + (r2 >= 0);
            if (q.a_regcnt > 0 && bcnt > 0) {
                const int m = (r0 >= 0 && r0 == q.reg[0]) + (r1 >= 0 && r1 == q.reg[1]) + (r2 >= 0 && r2 == q.reg[2]);
                s += q.sig_reg[bcnt][m];
                ++u;
            }
            const uint32_t nc = ha[kk].w & 0xFFFFu, nf = ha[kk].w >> 16;
            const int ic = (int)(ct & 0xFFFFu), ifr = (int)(ct >> 16);
            if (q.n_clubs > 0 && nc > 0) { s += ic == 0 ? q.sig0_clubs : set_term(q, PF_F_CLUBS, ic, (int)nc, q.sqrt_clubs); ++u; }
            if (q.n_friends > 0 && nf > 0) { s += ifr == 0 ? q.sig0_friends : set_term(q, PF_F_FRIENDS, ifr, (int)nf, q.sqrt_friends); ++u; }
            sum[kk] = s;
            used |= (uint32_t)(u + __popcll(pend[kk])) << (8 * kk);
        }
        K5T(3);
        // 4. text columns in rounds (ascending tokens = ascending columns, then tids)
        double cdot[kCandsPerThread], cnrm[kCandsPerThread];  // a split column's dot / norm so far
        uint32_t chit = 0;                                     // bit kk: the split column has a hit
#pragma unroll
        for (int kk = 0; kk < kCandsPerThread; ++kk) { cdot[kk] = 0.0; cnrm[kk] = 0.0; }
        int nrounds = (int)misc[3];  // written before the barrier above
        if (xdyn && nrounds == 0 && tid == 0) xclaim = atomicAdd(xctr, 1u);
        for (int rnd = 0; rnd < nrounds; ++rnd) {
            if (xdyn && rnd == nrounds - 1 && tid == 0) xclaim = atomicAdd(xctr, 1u);
            const uint2 rr = rtab[rnd];
            Round R;
            R.ja = (int)(rr.x & 0xFFFFu);
            R.jb = (int)(rr.x >> 16);
            R.ca = (int)(rr.y & 0xFFFFu);
            R.ce = (int)(rr.y >> 16);
            const int mbuf = rnd & 1;  // this round's list map buffer
            const int ja = R.ja, jb = R.jb;
            const uint32_t g0 = gpre[ja], F = gpre[jb] - g0;  // the round's flat entries
            if (F > 0) {
                // token segments of the round (read after the walk's barrier)
                if (tid < jb - ja) {
                    const int j = ja + tid;
                    const QCol c = scol[colof[j]];
                    const int lo = max(c.j0, ja) - ja, hi = min(c.j1, jb) - ja;
                    seg[tid] = (uint32_t)lo | (uint32_t)hi << 8 | (uint32_t)c.t << 16 |
                               ((c.j0 < ja || c.j1 > jb) ? kSegSplit : 0u);
                }
                // per round column (number t): the round-relative tokens before its end (the owner sums
                // take a candidate's hits in t as the mask bits below lmk[t] not taken by earlier columns)
                if (tid < R.ce - R.ca) {
                    const QCol c = scol[R.ca + tid];
                    lmk[c.t] = low_bits((uint32_t)(min((int)c.j1, jb) - ja));
                }
                if (tid == 0) misc[1] = 0u;
                // a. walk: the round's entries flattened over the workgroup, all loads in flight
                constexpr int U = kRoundCap / kPostThreads;
                uint32_t kp[U];  // p | token << 10 | tf << 16, or ~0
                double kn[U];  // (norms loaded in the place phase for first hits only: 184.6 -> 199.1 us, r4q)
                {
                    uint32_t xs[U];
                    int js[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t f = (uint32_t)(tid + kPostThreads * u);
                        // the list map: nonempty lists starting at or before f, minus one
                        js[u] = -1;
                        xs[u] = 0u;  // a valid address
                        if (f < F) {
                            const uint32_t w = f >> 6;
                            const uint32_t kk = (uint32_t)mapc[mbuf * kMapWords + w] +
                                                (uint32_t)__popcll(mapb[mbuf * kMapWords + w] & low_bits((f & 63u) + 1u)) - 1u;
                            const uint2 L = mapn[mbuf * kRoundToks + kk];
                            js[u] = ja + (int)L.y;
                            xs[u] = L.x + f;
                        }
                    }
                    uint32_t ent[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {  // unconditional: every load of the round in flight
                        ent[u] = ps.post[K5CHK(xs[u], ps.n_tok_entries, 4)];
                        kn[u] = ps.pnorm[K5CHK(xs[u], ps.n_tok_entries, 5)];
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t p = (ent[u] >> 8) - c0;
                        kp[u] = ~0u;
                        if (js[u] >= 0 && p < bsz) {
                            const uint32_t jr = (uint32_t)(js[u] - ja);
                            kp[u] = p | jr << 10 | (ent[u] & 0xFFu) << 16;
                            atomicOr(reinterpret_cast<unsigned long long*>(&mask[p]), 1ull << jr);
                        }
                    }
                }
                for (uint32_t f = (uint32_t)(tid + kRoundCap); f < F; f += kPostThreads) {  // one-token rounds past the cap
                    const int j = round_list(gpre, ja, jb, g0 + f);
                    const uint32_t p = (ps.post[K5CHK(rng[j].x + (g0 + f - gpre[j]), ps.n_tok_entries, 6)] >> 8) - c0;
                    if (p < bsz) atomicOr(reinterpret_cast<unsigned long long*>(&mask[p]), 1ull << (j - ja));
                }
                K5T(4);
                __syncthreads();
                K5T(5);
                if (tid < 64 && rnd + 1 < nrounds) {  // the next round's list map (published by the slots barrier)
                    const uint2 r1 = rtab[rnd + 1];
                    const int nb = mbuf ^ 1;
                    build_map(mapb + nb * kMapWords, mapc + nb * kMapWords, mapn + nb * kRoundToks, gpre, rng,
                              (int)(r1.x & 0xFFFFu), (int)(r1.x >> 16), lane);
                }
                // b. hit slots: the wave's candidates' hits in one contiguous range
                uint32_t nk[kCandsPerThread], tot = 0;
#pragma unroll
                for (int kk = 0; kk < kCandsPerThread; ++kk) {
                    nk[kk] = (uint32_t)__popcll(mask[kk * kPostThreads + tid]);
                    tot += nk[kk];
                }
                uint32_t incl = tot;
                incl = wave_incl_scan(incl);
                const uint32_t wn = wave_last(incl);
                uint32_t wb = 0;
                if (lane == 0) wb = atomicAdd(&misc[1], wn);
                wb = (uint32_t)__shfl((int)wb, 0);
                {
                    uint32_t h0 = wb + incl - tot;
#pragma unroll
                    for (int kk = 0; kk < kCandsPerThread; ++kk) {
                        hbase[kk * kPostThreads + tid] = (uint16_t)h0;
                        h0 += nk[kk];
                    }
                }
                K5T(6);
                __syncthreads();
                K5T(1);
                // c. place every hit at its slot, the column's first hit with its norm
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (kp[u] == ~0u) continue;
                    const uint32_t p = kp[u] & 1023u, jr = (kp[u] >> 10) & 63u, tf = kp[u] >> 16;
                    const uint64_t below = mask[p] & low_bits(jr);
                    const uint32_t r = K5CHK(hbase[p] + (uint32_t)__popcll(below), (uint32_t)kRoundCap, 8);
                    const uint32_t sg = seg[jr], lo = sg & 0xFFu;
                    const bool first = (below >> lo) == 0ull;
                    hit[r] = (uint16_t)(tf | jr << 8 | (first ? kHitFirst : 0u) | (below == 0ull ? kHitCand : 0u));
                    // the column's first hit holds its norm, the others their product (one per lane here,
                    // so the terms below only add them up); the first hit of a column wholly inside the
                    // round records the column's hit count in the round (>= 1), every other slot 0 (item[r],
                    // read once by the compaction below)
                    slot[r] = first ? kn[u] : tok_product(pt, ja + (int)jr, tf);
                    item[r] = (first && !(sg & kSegSplit)) ? (uint16_t)hit_run(mask[p], lo, (sg >> 8) & 0xFFu) : (uint16_t)0;
                }
                for (uint32_t f = (uint32_t)(tid + kRoundCap); f < F; f += kPostThreads) {
                    const int j = round_list(gpre, ja, jb, g0 + f);
                    const uint32_t x = K5CHK(rng[j].x + (g0 + f - gpre[j]), ps.n_tok_entries, 7);
                    const uint32_t e = ps.post[x];
                    const uint32_t p = (e >> 8) - c0;
                    if (p >= bsz) continue;
                    const uint32_t jr = (uint32_t)(j - ja);
                    const uint64_t below = mask[p] & low_bits(jr);
                    const uint32_t r = K5CHK(hbase[p] + (uint32_t)__popcll(below), (uint32_t)kRoundCap, 9);
                    const uint32_t sg = seg[jr];
                    const bool first = (below >> (sg & 0xFFu)) == 0ull;
                    hit[r] = (uint16_t)((e & 0xFFu) | jr << 8 | (first ? kHitFirst : 0u) | (below == 0ull ? kHitCand : 0u));
                    slot[r] = first ? ps.pnorm[x] : tok_product(pt, ja + (int)jr, e & 0xFFu);
                    item[r] = (first && !(sg & kSegSplit)) ? (uint16_t)hit_run(mask[p], sg & 0xFFu, (sg >> 8) & 0xFFu) : (uint16_t)0;
                }
                K5T(7);
                __syncthreads();
                K5T(8);
                // d. terms, one (candidate, column) item per lane over the wave's slots
                {
                // the wave's items (first hits of whole columns; the owner carries a split column),
                // compacted so the terms run on dense lanes
                // (in place: an item is written at or below the slot it was read from, after the read)
                uint16_t* wit = item + wb;
                uint32_t ni = 0;
                for (uint32_t r0 = wb; r0 < wb + wn; r0 += 64) {
                    const uint32_t r = r0 + (uint32_t)lane;
                    const uint32_t run = r < wb + wn ? (uint32_t)item[r] : 0u;
                    const bool is = run != 0u;
                    const uint64_t bal = __ballot(is);
                    wave_sync();
                    if (is) wit[ni + (uint32_t)__popcll(bal & low_bits((uint32_t)lane))] = (uint16_t)(r | run << kItemRunShift);
                    ni += (uint32_t)__popcll(bal);
                }
                wave_sync();
                for (uint32_t i = (uint32_t)lane; i < ni; i += 64) {
                    const uint32_t it = wit[i];
                    const uint32_t r = it & kItemSlotMask, run = it >> kItemRunShift;
                    const uint32_t h = hit[r];
                    const uint32_t jr = (h >> 8) & 63u, sg = seg[jr];
                    const int t = (int)((sg >> 16) & 0xFFu);
                    const double nrm = slot[r];
                    double dot = tok_product(pt, ja + (int)jr, h & 0xFFu);
                    if (run < kItemRunMax) {
                        dot = run_dot(slot, r, run, dot);  // the column's further hits, tid ascending
                    } else {  // a long run (>= kItemRunMax hits): walk it by the hit flags
                        const uint32_t hi = (sg >> 8) & 0xFFu;
                        for (uint32_t r2 = r + 1; r2 < wb + wn; ++r2) {
                            const uint32_t h2 = hit[r2];
                            const uint32_t j2 = (h2 >> 8) & 63u;
                            if ((h2 & kHitCand) || j2 >= hi) break;
                            dot += slot[r2];
                        }
                    }
                    slot[r] = dot == 0.0 ? q.sig0_col[t] : text_term(q, t, dot, nrm);
                }
                }
                wave_sync();
                K5T(9);
            }
            // e. the owners add the round's common columns in ascending order (the candidate's
            // columns among the round's: ~3 per round instead of every round column)
            const uint64_t rtm = cpre[R.ce] & ~cpre[R.ca];  // the round's columns, by column number
            // the round's split columns (<= 2, the only ones not wholly inside it): its first if that
            // began in an earlier round, its last if that goes on past it (column numbers, or -1)
            int t_in = -1, t_on = -1;
            if (R.ce > R.ca) {
                const QCol cf = scol[R.ca], cl = scol[R.ce - 1];
                if (cf.j0 < ja) t_in = cf.t;
                if (cl.j1 > jb) t_on = cl.t;
            }
#pragma unroll
            for (int kk = 0; kk < kCandsPerThread; ++kk) {
                const int p = kk * kPostThreads + tid;
                // the candidate's hits lie in its common columns only, in ascending token order: the
                // remaining mask and a running slot index walk them column by column
                uint64_t mr = F > 0 ? mask[p] : 0ull;
                uint32_t rr = F > 0 ? hbase[p] : 0u;
                for (uint64_t pr = pend[kk] & rtm; pr; pr &= pr - 1) {
                    const int t = __ffsll((unsigned long long)pr) - 1;
                    const uint64_t lm = lmk[t];  // (stale in an empty round: mr is 0 there)
                    const uint64_t h = mr & lm;
                    mr &= ~lm;
                    const uint32_t r0 = rr;
                    rr += (uint32_t)__popcll(h);
                    if (t != t_in && t != t_on) {
                        sum[kk] += h ? slot[r0] : q.sig0_col[t];
                        continue;
                    }
                    // split column (rare): the dot over its segments in ascending order
                    if (h) {
                        uint64_t v = h;
                        uint32_t r = r0;
                        while (v) {
                            const int jr = __ffsll((unsigned long long)v) - 1;
                            v &= v - 1;
                            cdot[kk] += tok_product(pt, ja + jr, hit[r++] & 0xFFu);
                        }
                        cnrm[kk] = slot[r0];
                        chit |= 1u << kk;
                    }
                    if (t != t_on) {
                        const bool hh = (chit >> kk) & 1u;
                        sum[kk] += (hh && cdot[kk] != 0.0) ? text_term(q, t, cdot[kk], cnrm[kk]) : q.sig0_col[t];
                        cdot[kk] = 0.0;
                        chit &= ~(1u << kk);
                    }
                }
                if (F > 0) mask[p] = 0ull;
            }
            K5T(10);
            if (F == 0 && rnd + 1 < nrounds) {  // an empty round built no list map for the next one
                if (tid < 64) {
                    const uint2 r1 = rtab[rnd + 1];
                    const int nb = mbuf ^ 1;
                    build_map(mapb + nb * kMapWords, mapc + nb * kMapWords, mapn + nb * kRoundToks, gpre, rng,
                              (int)(r1.x & 0xFFFFu), (int)(r1.x >> 16), lane);
                }
                __syncthreads();
            }
            if (F > 0) __syncthreads();  // the next round rewrites the masks, slots and segments
        }
        K5T(11);
        // 5. FAS (recommender_similarity.cpp:114-123) and the wave top-k
        uint64_t keys[kCandsPerThread];
#pragma unroll
        for (int kk = 0; kk < kCandsPerThread; ++kk) {
            uint64_t key = ~0ull;
            if (!((skip >> kk) & 1u)) {
                float f = 0.0f;
                const int uk = (int)((used >> (8 * kk)) & 0xFFu);
                if (uk > 0) {
                    const double S = sum[kk] / (double)uk;
                    const double Fv = ftab[uk];  // (double)uk / (double)(kNumFixed + q.n_cols)
                    f = (S <= 0.0 && Fv <= 0.0) ? 0.0f : (float)((2.0 * S * Fv) / (S + Fv));
                }
                // keyed by idx (idx order = uid order); uids are filled in before the merge
                key = score_key(f, (int32_t)(c0 + kk * kPostThreads + tid));
            }
            keys[kk] = key;
        }
        // the lane's 2 keys ascending, then pushed best-first: after the first push the
        // wave's threshold rejects most of the rest
        static_assert(kCandsPerThread == 2, "2-key sort");
        if (keys[1] < keys[0]) { const uint64_t x = keys[0]; keys[0] = keys[1]; keys[1] = x; }
#pragma unroll
        for (int kk = 0; kk < kCandsPerThread; ++kk) topk_push(best, keys[kk], k, lane);
        K5T(12);
#ifdef PF_K5_BLOCKLOG
        if (tid == 0) {
            const unsigned i = atomicAdd(&g_blog_n, 1u);
            if (i < kBlogCap) {
                g_blog_t[2 * i] = blog_t0;
                g_blog_t[2 * i + 1] = __builtin_amdgcn_s_memrealtime();
                g_blog_meta[i] = (unsigned)bx | (unsigned)blk << 16;
            }
        }
#endif
        if (xdyn) {
            if (tid == 0) misc[0] = (uint32_t)(x_lo + x_nwg) + xclaim;
            __syncthreads();
            blk = (int)misc[0];
        } else if ((mode & 1u) && blk + nbx >= tail) {
            // the tail past the static rounds from the query's counter: one claim per workgroup
            // (every workgroup claiming every block serialised ~3,000 atomics on one address).
            // misc[0] was last read before this block's first barrier; claimed here, not at the
            // block's start: an early claim measured 190 -> 200 us (r4i)
            if (tid == 0) misc[0] = (uint32_t)tail + atomicAdd(next_blk, 1u);
            __syncthreads();
            blk = (int)misc[0];
        } else {
            __syncthreads();  // the next block rewrites the exclusion bits the owners read above
            blk += nbx;
        }
    }
#ifdef PF_K5_TIMERS
    tacc[13] = clock64() - tstart;
    if (lane == 0) {
        for (int i = 0; i < 14; ++i) atomicAdd(&g_k5t[i], (unsigned long long)tacc[i]);
        atomicAdd(&g_k5t[15], 1ull);
    }
#endif
    // idx -> uid in the wave's list (the same order: uid ascending == idx ascending)
    if (lane < k && best != ~0ull) {
        const uint32_t idx = (uint32_t)best ^ 0x80000000u;
        best = (best & 0xFFFFFFFF00000000ull) | (ps.hdr[2 * (size_t)idx + 1].w ^ 0x80000000u);
    }
    // tail scratch in the (idle) slots: merge keys, then flag / threshold / block ids
    uint64_t* sc = reinterpret_cast<uint64_t*>(slot);

    post_tail(best, k, sc, sync, parts, out, out_rows, qy, bx, nbx);
}

// ---------------------------------------------------------------- K2: merge
// Key lists in[part * part_stride + q * query_stride + j] (j < k) -> out[q * k + j]
// (the cross-shard merge after the all-gather; one block per query, every wave pushes
// its share of the keys, then wave 0 merges the wave lists).
constexpr int kMergeThreads = 1024;
__global__ __launch_bounds__(kMergeThreads) void topk_merge_kernel(const uint64_t* __restrict__ in, int32_t nparts,
                                                                   int64_t part_stride, int64_t query_stride, int32_t k,
                                                                   uint64_t* __restrict__ out,
                                                                   const int32_t* __restrict__ out_rows) {
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
        const int row = out_rows ? out_rows[q] : q;
        if (lane < k) out[(size_t)row * k + lane] = acc;
    }
}

// ---------------------------------------------------------------- K1': pairs
#ifdef PF_K1P_WPE  // experiment builds: waves per SIMD the pair kernel's registers are sized for
#define PF_K1P_BOUNDS __launch_bounds__(kPairThreads) __attribute__((amdgpu_waves_per_eu(PF_K1P_WPE, PF_K1P_WPE)))
#else
#define PF_K1P_BOUNDS __launch_bounds__(kPairThreads, 4)
#endif
template <bool PACKED, bool GTAB>
__global__ PF_K1P_BOUNDS void fas_pairs_kernel(DevStore st, const uint8_t* __restrict__ pool,
                                                        const QImageRef* __restrict__ refs,
                                                        const PairBlock* __restrict__ blocks,
                                                        const int32_t* __restrict__ order,
                                                        const int32_t* __restrict__ slots, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef PF_K5_TIMERS
    const uint64_t t0 = clock64();
    uint64_t tw[4] = {0, 0, 0, 0};
    uint64_t* twp = tw;
#else
    uint64_t* twp = nullptr;
#endif
    const PairBlock b = blocks[order ? order[blockIdx.x] : (int)blockIdx.x];
    // a block scores b.count <= kPairThreads pairs against its one staged image; the plan sizes
    // candidate blocks by the candidate bound, so a block past a job's candidates has none
    const int i = (int)threadIdx.x;
    int p = i < b.count ? slots[b.begin + i] : -1;
    const bool active = p >= 0;
    if (!__syncthreads_or(active)) return;
    const PairHdr H = load_pair_hdr(st, p, active);
    char* scratch;
    const QView v = stage_query<GTAB>(smem, pool, refs[b.qimg], &scratch);
#ifdef PF_K5_TIMERS
    const uint64_t t1 = clock64();
#endif
    const float f = fas_slot<PACKED>(st, v, H, active, twp);
    if (active) out[b.out + i] = f;
#ifdef PF_K5_TIMERS
    const uint64_t t3 = clock64();
    // the wave's phase ends: the walk is wave-uniform; the epilogue's phases end at the wave's
    // last lane (max over the lanes that ran it)
    // (the epilogue's clocks are taken by every lane at wave-uniform points: lane 0's are the wave's)
    uint64_t we = tw[0], fe = tw[1], he = tw[2], oe = tw[3];
    we = (uint64_t)__shfl((long long)we, 0);
    fe = (uint64_t)__shfl((long long)fe, 0);
    he = (uint64_t)__shfl((long long)he, 0);
    oe = (uint64_t)__shfl((long long)oe, 0);
    if (fe == 0) fe = we;
    if (he == 0) he = fe;
    if (oe == 0) oe = he;
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&g_k1t[0], (unsigned long long)(t1 - t0));
        atomicAdd(&g_k1t[1], (unsigned long long)(we - t1));
        atomicAdd(&g_k1t[2], (unsigned long long)(t3 - we));
        atomicAdd(&g_k1t[3], (unsigned long long)(t3 - t0));
        atomicAdd(&g_k1t[4], (unsigned long long)(fe - we));
        atomicAdd(&g_k1t[5], (unsigned long long)(he - fe));
        atomicAdd(&g_k1t[6], (unsigned long long)(oe - he));
        atomicAdd(&g_k1t[8], (unsigned long long)(t3 - oe));
        atomicAdd(&g_k1t[7], 1ull);
    }
#endif
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

int scan_blocks_per_cu(bool packed, bool gtab, uint32_t lds) {
    // the answer depends only on (variant, LDS bytes): cache it, the query is not free
    static thread_local uint64_t last_key = ~0ull;
    static thread_local int last_nb = 1;
    const uint64_t key = ((uint64_t)lds << 2) | ((uint64_t)packed << 1) | (uint64_t)gtab;
    if (key == last_key) return last_nb;
    int nb = 0;
    hipError_t e;
    if (packed) e = gtab ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fas_scan_kernel<true, true>, kScanThreads, lds)
                         : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fas_scan_kernel<true, false>, kScanThreads, lds);
    else e = gtab ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fas_scan_kernel<false, true>, kScanThreads, lds)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fas_scan_kernel<false, false>, kScanThreads, lds);
    last_key = key;
    last_nb = (e == hipSuccess && nb > 0) ? nb : 1;
    return last_nb;
}

// K5 dynamic LDS: QConst | fixed per-block arrays | PTok[n_tok] | PList[n_lists] | ranges[n_lists] |
// rounds[n_tok + 1] | token prefix[n_tok + 1] | set prefix[n_sets + 1] | token -> column u8[n_tok]
uint32_t post_var_lds(int n_tok, int n_lists) {
    return (uint32_t)(sizeof(PTok) * n_tok + 8 * n_lists + 8 * (n_tok + 1) + 4 * (n_tok + 1) +
                      4 * (n_lists - n_tok + 1) + n_tok + 15) & ~15u;
}
uint32_t post_lds(uint32_t var_lds) { return (uint32_t)sizeof(QConst) + kPostFixedLds + var_lds; }

#ifdef PF_K5_BLOCKLOG
// per-block times of one launch: the span, and per static round (blk / nbx) the blocks' start and
// end offsets and durations (us, from the launch's first block start)
static void blog_report(int nbx) {
    static unsigned long long t[2 * kBlogCap];
    static unsigned int meta[kBlogCap];
    unsigned int n = 0;
    hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_blog_n), sizeof n);
    n = n < kBlogCap ? n : kBlogCap;
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_blog_t), 2 * n * sizeof(unsigned long long));
    hipMemcpyFromSymbol(meta, HIP_SYMBOL(g_blog_meta), n * sizeof(unsigned));
    unsigned long long t0 = ~0ull, t1 = 0;
    for (unsigned i = 0; i < n; ++i) { t0 = t[2 * i] < t0 ? t[2 * i] : t0; t1 = t[2 * i + 1] > t1 ? t[2 * i + 1] : t1; }
    fprintf(stderr, "k5blog: %u blocks, span %.1f us\n", n, (t1 - t0) / 100.0);
    static int dumps = 0;
    if (const char* path = getenv("PF_BLOG_OUT"); path && dumps++ < 3) {  // raw rows: wg blk start end (us)
        char fn[512];
        snprintf(fn, sizeof fn, "%s.%d.csv", path, dumps);
        if (FILE* f = fopen(fn, "w")) {
            for (unsigned i = 0; i < n; ++i)
                fprintf(f, "%u,%u,%.2f,%.2f\n", meta[i] & 0xFFFFu, meta[i] >> 16, (t[2 * i] - t0) / 100.0,
                        (t[2 * i + 1] - t0) / 100.0);
            fclose(f);
        }
    }
    for (int r = 0; r < 8; ++r) {
        std::vector<double> d, st, en;
        for (unsigned i = 0; i < n; ++i) {
            const int blk = (int)(meta[i] >> 16);
            if (blk / nbx != r) continue;
            d.push_back((t[2 * i + 1] - t[2 * i]) / 100.0);
            st.push_back((t[2 * i] - t0) / 100.0);
            en.push_back((t[2 * i + 1] - t0) / 100.0);
        }
        if (d.empty()) continue;
        std::sort(d.begin(), d.end()); std::sort(st.begin(), st.end()); std::sort(en.begin(), en.end());
        auto pc = [](const std::vector<double>& v, double q) { return v[(size_t)(q * (v.size() - 1))]; };
        fprintf(stderr, "k5blog: round %d: %zu blocks, dur p10/50/90/max %.1f/%.1f/%.1f/%.1f, start min/50/max %.1f/%.1f/%.1f, end min/50/max %.1f/%.1f/%.1f\n",
                r, d.size(), pc(d, .1), pc(d, .5), pc(d, .9), d.back(), st.front(), pc(st, .5), st.back(), en.front(),
                pc(en, .5), en.back());
    }
}
#endif

hipError_t launch_post(const PostStore& ps, const uint8_t* pool, const uint32_t* img_off, uint32_t var_lds, int nq,
                       int blk_begin, int blk_end, int k, int blocks, uint64_t* parts, ScanSync* sync, uint64_t* out,
                       const int32_t* out_rows, uint32_t mode, uint32_t tail_bs, hipEvent_t e0, hipEvent_t e1,
                       hipStream_t s, const uint8_t* qconst) {
    if (nq <= 0) return hipSuccess;
    // timed launches (e0, e1 given): the kernel's own start and end timestamps, taken from its
    // dispatch (hipExtLaunchKernelGGL), instead of two marker packets around it
    const dim3 grid = (mode & 2u) ? dim3(nq, blocks) : dim3(blocks, nq);
    hipExtLaunchKernelGGL(fas_post_kernel, grid, dim3(kPostThreads), post_lds(var_lds), s, e0, e1, 0u, ps, pool, img_off,
                          blk_begin, blk_end, k, parts, sync, out, out_rows, mode, tail_bs, qconst);
#ifdef PF_K5_BLOCKLOG
    {
        static int calls = 0;
        hipStreamSynchronize(s);
        if (++calls % 10 == 0 && nq == 1) blog_report(blocks);
        const unsigned zero = 0;
        hipMemcpyToSymbol(HIP_SYMBOL(g_blog_n), &zero, sizeof zero);
    }
#endif
#ifdef PF_K5_TIMERS
    {
        static int calls = 0;
        unsigned long long t[16];
        hipStreamSynchronize(s);
        hipMemcpyFromSymbol(t, HIP_SYMBOL(g_k5t), sizeof(t));
        static const char* nm[14] = {"ranges+hdr", "barriers", "excl+sets", "fixed", "walk", "walk-bar",
                                     "slots", "place", "place-bar", "terms", "owner-add", "rounds-end", "fas+topk",
                                     "total"};
        if (++calls % 10 == 0) {
            fprintf(stderr, "k5t per wave (clock64):");
            for (int i = 0; i < 14; ++i) fprintf(stderr, " %s=%.0f", nm[i], (double)t[i] / (double)t[15]);
            fprintf(stderr, "\n");
        }
        const unsigned long long z[16] = {0};
        hipMemcpyToSymbol(HIP_SYMBOL(g_k5t), z, sizeof(z));
    }
#endif
    return hipGetLastError();
}

int post_blocks_per_cu(uint32_t var_lds) {
    // per thread, by LDS bytes (a batch asks once per query: the occupancy API once per size)
    static thread_local std::unordered_map<uint32_t, int> memo;
    auto it = memo.find(var_lds);
    if (it != memo.end()) return it->second;
    int nb = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fas_post_kernel, kPostThreads, post_lds(var_lds));
    nb = (e == hipSuccess && nb > 0) ? nb : 1;
    if (memo.size() > 4096) memo.clear();
    memo.emplace(var_lds, nb);
    return nb;
}

hipError_t launch_merge(const uint64_t* in, int nparts, int64_t part_stride, int64_t query_stride, int nq, int k,
                        uint64_t* out, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(topk_merge_kernel, dim3(nq), dim3(kMergeThreads), 0, s, in, nparts, part_stride, query_stride,
                       k, out, (const int32_t*)nullptr);
    return hipGetLastError();
}

hipError_t launch_pairs(const DevStore& st, const uint8_t* pool, const QImageRef* refs_dev, uint32_t max_lds,
                        bool gtab, const PairBlock* blocks, int nblocks, const int32_t* order, const int32_t* slots,
                        float* out, hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
#define PF_PAIRS(P, G) hipLaunchKernelGGL((fas_pairs_kernel<P, G>), dim3(nblocks), dim3(kPairThreads), max_lds, s, st, pool, \
                                          refs_dev, blocks, order, slots, out)
    if (st.packed) { if (gtab) PF_PAIRS(true, true); else PF_PAIRS(true, false); }
    else { if (gtab) PF_PAIRS(false, true); else PF_PAIRS(false, false); }
#undef PF_PAIRS
#ifdef PF_K5_TIMERS
    {
        static int calls = 0;
        unsigned long long t[12];
        hipStreamSynchronize(s);
        hipMemcpyFromSymbol(t, HIP_SYMBOL(g_k1t), sizeof(t));
        if (++calls % 10 == 0 && t[7] && t[11])
            fprintf(stderr, "k1pt epilogue: fallback waves %.3f, items per lane %.2f\n", (double)t[9] / t[11],
                    (double)t[10] / (64.0 * t[11]));
        if (calls % 10 == 0 && t[7])
            fprintf(stderr,
                    "k1pt per wave (clock64): staging=%.0f walk=%.0f epilogue=%.0f (dense=%.0f assembly=%.0f "
                    "overflow=%.0f fas=%.0f) total=%.0f waves=%llu blocks=%d\n",
                    (double)t[0] / t[7], (double)t[1] / t[7], (double)t[2] / t[7], (double)t[4] / t[7],
                    (double)t[5] / t[7], (double)t[6] / t[7], (double)t[8] / t[7], (double)t[3] / t[7], t[7], nblocks);
        const unsigned long long z[12] = {0};
        hipMemcpyToSymbol(HIP_SYMBOL(g_k1t), z, sizeof(z));
    }
#endif
    return hipGetLastError();
}

}  // namespace pf
