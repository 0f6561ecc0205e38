// pf_types.h — device data layout shared by the host builder (pf_store.cpp)
// and the gfx950 kernels (pf_kernels.hip).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pokec_fas.h"

namespace pf {

constexpr int kWave = 64;           // CDNA wavefront
constexpr int kTileSlots = 64;      // candidates per tile = lanes per wave
constexpr int kMaxCols = PF_MAX_COLS;
constexpr int kNumFixed = PF_NUM_FIXED;
constexpr int kNormSlots = kNumFixed + kMaxCols;
constexpr int kValTab = 128;        // completion/age sigmoid tables cover values 1..128
constexpr int kMaxTopK = 64;        // in-kernel top-k bound (one key per lane)

// hash-table key tags (bits 32..39 of a key)
constexpr uint32_t kTagClubs = 64;
constexpr uint32_t kTagFriends = 65;
constexpr uint32_t kTagExcl = 66;   // all-candidates exclusion set adj[q] + {q}, keyed by uid
constexpr uint64_t kEmptyKey = ~0ull;
constexpr uint64_t kKeyMask = 0xFFFFFFFFFFull;  // low 40 bits: tag:id

// Record stream words (per candidate, in this order), see DESIGN.md:
//   n_clubs, clubs[n_clubs], n_friends, friends[n_friends],
//   per non-empty text column t (ascending):
//     (t | count << 8), sqrt(nb) lo, sqrt(nb) hi, count token words
//   token word (packed): tid | tf << 24      (needs 0 <= tid < 2^24, 0 <= tf < 256)
//   token words (wide):  tid, tf
constexpr uint32_t kPackedTidMask = 0xFFFFFFu;

// per-slot fixed header, 2 x uint4 (32 B):
//   h0 = {colmask lo, colmask hi, completion, age}
//   h1 = {region0, region1, region2, codes} codes = pub | gen << 8 | (nclubs>0)<<16 ...
constexpr uint32_t kCodeMissing = 0xFFu;

__host__ __device__ inline uint32_t hash_key(uint32_t tag, uint32_t id) {
    uint32_t h = id * 0x9E3779B1u ^ (tag * 0x85EBCA77u);
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}

__host__ __device__ inline uint64_t make_key(uint32_t tag, uint32_t id) {
    return ((uint64_t)tag << 32) | id;
}

// Per-query constants (A side of profile_similarity).  Built on the host with
// glibc exp/logf so every table entry is bit-identical to the reference.
struct QConst {
    uint64_t colmask;          // non-empty text columns of A
    int32_t comp, age;         // > 0 when present
    int32_t reg[3];
    uint32_t pubcode, gencode; // kCodeMissing when < 0
    int32_t a_regcnt;          // parts >= 0 (0 -> region term never used)
    int32_t n_clubs, n_friends;// |A.clubs|, |A.friends| with duplicates
    int32_t cap_log2;          // hash table capacity
    int32_t n_vals;            // token value entries
    int32_t n_cols;            // T
    int32_t pad0;
    double sqrt_clubs, sqrt_friends;     // sqrt((double)|A|)
    double sig_pub[2], sig_gen[2];       // [eq]
    double sig_reg[4][4];                // [b_cnt][matches]
    double sig_comp[kValTab + 1];        // [candidate value], 1..kValTab
    double sig_age[kValTab + 1];
    double sig0_clubs, sig0_friends;     // term at s = 0
    double sig0_col[kMaxCols];           // term at s = 0 per column
    double sqrt_na[kMaxCols];            // sqrt(sum w_A^2) per column
    // normaliser z = zmode ? (s - zmean)/zsd : 6(s - 0.5)   (slots 0..6 fixed, 7+t text)
    double zmean[kNormSlots];
    double zsd[kNormSlots];
    uint32_t zmode_lo, zmode_hi, zmode_fx, pad1;  // bitmask per text column / fixed slot
};

// token value of a query hash entry: dot += wq * (tf * idf)
struct QVal {
    double wq;
    double idf;
};

// One query image in device memory: QConst + keys[1<<cap_log2] + vals[n_vals].
struct QImageRef {
    uint32_t const_off;   // byte offset of QConst in the image pool
    uint32_t keys_off;    // byte offset of the key table
    uint32_t vals_off;    // byte offset of the value table
    uint32_t lds_bytes;   // bytes needed to stage this query in LDS (0 = too big -> global)
};

// top-k key: ascending key == (score desc, uid asc), recommender_graph.cpp:97-101
__host__ __device__ inline uint64_t score_key(float s, int32_t uid) {
    union { float f; uint32_t u; } v;
    v.f = s;
    uint32_t b = v.u;
    if ((b & 0x7FFFFFFFu) == 0) b = 0;  // -0 == +0 in the reference comparator
    uint32_t ord = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    return ((uint64_t)(~ord) << 32) | (uint32_t)((uint32_t)uid ^ 0x80000000u);
}
__host__ __device__ inline float key_score(uint64_t k) {
    uint32_t ord = ~(uint32_t)(k >> 32);
    uint32_t b = (ord & 0x80000000u) ? (ord & 0x7FFFFFFFu) : ~ord;
    union { float f; uint32_t u; } v;
    v.u = b;
    return v.f;
}
__host__ __device__ inline int32_t key_uid(uint64_t k) {
    return (int32_t)((uint32_t)k ^ 0x80000000u);
}

// Device-side corpus (the "tile store").
struct DevStore {
    const uint4* stream;       // [sum tile_steps * 64] interleaved record stream
    const uint64_t* tile_off;  // [n_tiles] uint4 offset of each tile
    const uint32_t* tile_steps;// [n_tiles] 16-B steps of the longest record in the tile
    const uint4* hdr0;         // [n_slots]
    const uint4* hdr1;         // [n_slots]
    const int32_t* slot_uid;   // [n_slots]
    const uint32_t* slot_len;  // [n_slots] record length in words
    int32_t n_slots;
    int32_t n_tiles;
    int32_t packed;
    int32_t n_cols;
};

}  // namespace pf
