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
constexpr int kScanThreads = 256;   // 4 waves per scan block
#ifndef PF_HIT_CAP
#define PF_HIT_CAP 20
#endif
constexpr uint32_t kHitCap = PF_HIT_CAP;  // token hits kept per candidate in LDS (overflow -> slow re-walk)
#ifndef PF_QUEUE_EXTRA
#define PF_QUEUE_EXTRA 0
#endif
// + dump slots: the pair walk clamps its list once per 4-word step; the strip of a wave's lists is
// also K1''s epilogue item queue (kHitSlots * 64 / 4 items of 16 B)
constexpr uint32_t kHitSlots = kHitCap + 4 + PF_QUEUE_EXTRA;
constexpr int kMaxHashLog2 = 16;    // cuckoo tables <= 65536 slots (h1/h2 from one 32-bit product)
constexpr uint32_t kMaxTileSteps = 48;  // a record longer than 48 steps (192 words) is split over lanes

// Query hash: 2-choice cuckoo tables of 8-byte entries {key, val} (uint2), hashed by one
// multiply with a per-query odd multiplier (x = key * hmul; slots = two bit fields of x).
// Packed corpora (the fast path) use ONE table for every record word plus an exclusion
// table, so a word's probe needs no per-kind table choice:
//   T   clubs    key = id | kTagClub                val = 1        (counts clubs, low 16 bits)
//       friends  key = id                           val = 0x10000  (counts friends, high 16 bits)
//       tokens   key = kTagTok | col << 18 | tid    val = kTokVal | col << 18 | value index
//   T3  excl     key = uid (adj[q] + {q})            val = 1
//   empty = {~0, 0}: a miss reads val 0, and the padding word ~0 only ever matches empties
// Wide corpora keep three tables T0 clubs | T1 friends | T2 tokens (2^lg each), keys
// untagged (T2: key = tid, val = col | value index << 8), then T3; empty = {~0, ~0}.
constexpr uint32_t kEmptyVal = 0xFFFFFFFFu;       // wide tables: miss
constexpr uint64_t kEmptyEntry = ~0ull;           // wide tables: empty slot
constexpr uint64_t kEmptyEntryPacked = 0xFFFFFFFFull;  // packed tables: {key ~0, val 0}
constexpr uint32_t kHashMul = 0x9E3779B1u;
constexpr uint32_t kTagClub = 0x80000000u;
constexpr uint32_t kTagTok = 0x40000000u;
constexpr uint32_t kTokVal = 0x01000000u;
constexpr uint32_t kIdLimit = 0x40000000u;        // packed: club / friend ids below 2^30
// wide: a token's first word is tid | col << 26 (the query tables' key: one entry per (column,
// tid), as a tid can sit in several columns), so wide corpora need 0 <= tid < 2^26
constexpr uint32_t kWideTidBits = 26;
constexpr uint32_t kWideTidMask = (1u << kWideTidBits) - 1;
constexpr uint32_t kPadWord = 0xFFFFFFFFu;        // stream padding

// Record stream (per candidate, tile-interleaved in 16-B steps):
//   clubs[n_clubs] | friends[n_friends] | tokens[n_tok]
// packed: club word = id | kTagClub (the T key), friend word = id,
//   token word = tf << 24 | col << 18 | tid  (tid < 2^18 - 1, 0 <= tf < 256, col < 64);
//   kTagTok | (low 24 bits) is the T key; every word past a record is kPadWord
// wide token = 2 words: tid, (tf << 8) | col          (tf in [-2^23, 2^23))
// Tokens are grouped by column (ascending), ascending tid within a column.
constexpr uint32_t kTidBits = 18;
constexpr uint32_t kTidMask = (1u << kTidBits) - 1;

// Tiles: 64 lanes = 64 >> lgk candidates, each candidate's record split into k = 1 << lgk
// contiguous chunks of q = ceil(len / k) words (rounded up to even in the wide format),
// chunk c of candidate i in lane i * k + c, so no tile is longer than kMaxTileSteps
// (unless a single record is longer than 64 * 192 words).  Candidates are sorted by record
// length, so almost every tile has k = 1.
__host__ __device__ inline uint32_t chunk_words(uint32_t len, uint32_t lgk, bool packed) {
    uint32_t q = (len + (1u << lgk) - 1) >> lgk;
    if (!packed) q = (q + 1) & ~1u;
    return q;
}

// Per-slot header, 3 x uint4 (48 B), SoA:
//   h0 = {colmask lo, colmask hi, completion, age}
//   h1 = {region0, region1, region2, uid}
//   h2 = {codes (pub | gen << 8), n_clubs, n_friends, n_tok}
constexpr uint32_t kCodeMissing = 0xFFu;

// 2-choice cuckoo slots of a 32-bit key: one multiply, two bit fields of the product
__host__ __device__ inline uint32_t cuckoo_x(uint32_t key, uint32_t hmul) { return key * hmul; }
__host__ __device__ inline uint32_t cuckoo_h1(uint32_t x, int lg) { return x >> (32 - lg); }
__host__ __device__ inline uint32_t cuckoo_h2(uint32_t x, int lg) { return (x >> (32 - 2 * lg)) & ((1u << lg) - 1u); }
__host__ __device__ inline uint64_t make_entry(uint32_t key, uint32_t val) { return ((uint64_t)val << 32) | key; }
// Query tables are built as 8-B {key, val} entries and stored SoA per table: the table of 2^lg
// entries at entry offset off keeps its keys in words [2 off, 2 off + 2^lg) and its values in the
// next 2^lg words (the same bytes), so a wave's random key probes (ds_read_b32) spread over all 32
// banks instead of the even ones.  Word positions of entry i of the image's tables (ntab tables of
// 2^lg, then the exclusion table of 2^lge at excl = ntab << lg):
__host__ __device__ inline void soa_words(uint32_t i, uint32_t excl, int lg, int lge, uint32_t& kw, uint32_t& vw) {
    const bool ex = i >= excl;
    const uint32_t off = ex ? excl : (i >> lg) << lg, sz = ex ? (1u << lge) : (1u << lg);
    kw = 2u * off + (i - off);
    vw = kw + sz;
}

// Per-query constants (A side of profile_similarity).  Built on the host with
// glibc exp so every table entry is bit-identical to the reference.
struct QConst {
    uint64_t colmask;          // non-empty text columns of A
    int32_t comp, age;         // > 0 when present
    int32_t reg[3];
    uint32_t pubcode, gencode; // kCodeMissing when < 0
    int32_t a_regcnt;          // parts >= 0 (0 -> region term never used)
    int32_t n_clubs, n_friends;// |A.clubs|, |A.friends| with duplicates
    int32_t lg;                // capacity log2 of T (packed) / of each of T0..T2 (wide)
    int32_t lg_excl;           // capacity log2 of T3
    uint32_t hmul;             // cuckoo hash multiplier (odd; all tables)
    int32_t n_vals;            // token value entries
    int32_t n_cols;            // T
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
    uint32_t zmode_lo, zmode_hi, zmode_fx, n_hits_max;  // n_hits_max: hit-list bytes per lane
    uint32_t excl_off;         // entry offset of T3 (1 << lg packed, 3 << lg wide)
};

// token value of a query hash entry: dot += wq * (tf * idf)
struct QVal {
    double wq;
    double idf;
};

// One query image in device memory: QConst + tables[excl_off + 2^lg_excl] + vals[n_vals].
// The image starts at pool + 16 * const_off (pools up to 64 GB: the job pipeline keeps every
// user's image resident); its tables at byte offsets keys_off / vals_off from that start.
struct QImageRef {
    uint32_t const_off;   // image start in 16-B units of the image pool (QConst first)
    uint32_t keys_off;    // byte offset of the key table from the image start
    uint32_t vals_off;    // byte offset of the value table from the image start
    uint32_t lds_bytes;   // bytes of keys+vals staged in LDS (0 = probe global memory)
};

// Per-query rendezvous of one scan launch: blocks finished, K5's block hand-out counter,
// and the tail tile counters.  Zeroed by the host before every launch (it rides in the
// query upload).
struct ScanSync {
    unsigned int done;
    unsigned int pad0[15];
    unsigned int next;  // K5 dynamic hand-out: blocks claimed past the first gridDim.x, 64 B from done
    unsigned int pad[15];
    unsigned int xcd_next[8 * 16];  // tail tile counter per XCD, 64 B apart
    unsigned int grp[8 * 16];       // K5's group tickets (post_tail), 64 B apart
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
    const uint4* stream;       // interleaved record stream, [tile][step][lane] uint4
    const uint64_t* tile_off;  // [n_tiles] uint4 offset of each tile
    const uint32_t* tile_steps;// [n_tiles] 16-B steps of the longest chunk in the tile
    const uint32_t* tile_slot0;// [n_tiles] first slot of the tile
    const uint8_t* tile_lgk;   // [n_tiles] log2 lanes per candidate
    const uint32_t* slot_tile; // [n_slots] tile of the slot
    const double* norms;       // [tile][candidate in tile][rank] sqrt(sum (tf*idf)^2) per non-empty column
    const uint64_t* norm_off;  // [n_tiles + 1] double offset of each tile's norms (64 x ranks per tile)
    const uint4* hdr0;         // [n_slots]
    const uint4* hdr1;
    const uint4* hdr2;
    const uint4* rows;         // row store: slot p's record contiguous from rows[row_off[p]], padded to 16 B,
                               // then its column norms (double per non-empty column, ascending) (pair kernel)
    const uint64_t* row_off;   // [n_slots + 1]
    const uint4* row_pad;      // one 16-B line of kPadWord (a pair-kernel lane past its record reads it)
    int32_t n_slots;
    int32_t n_tiles;
    int32_t packed;
    int32_t n_cols;
};

// ---------------------------------------------------------------- postings store (K5)
// The all-candidates scan inverted: for every query token / club / friend, the list of
// candidates holding it, so a query reads only the lists it names instead of every record.
// Candidates are in idx order (ascending uid, the reference's tie-break order); a workgroup
// scores one block of kBlockCands consecutive candidates at a time.
#ifndef PF_K5_WAVES
#define PF_K5_WAVES 4
#endif
constexpr int kPostWaves = PF_K5_WAVES;    // waves per K5 workgroup
constexpr int kPostThreads = kPostWaves * kWave;
constexpr int kBlockCands = 2 * kPostThreads;  // candidates of a workgroup block (2 per thread)
constexpr int kCandsPerThread = kBlockCands / kPostThreads;
// K5 rounds: a block's query tokens are taken in rounds of <= kRoundToks tokens (one 64-bit hit
// mask per candidate) whose list entries in the block number <= kRoundCap (the round's hit slots,
// PF_K5_RCAP per thread)
#ifndef PF_K5_RCAP
#define PF_K5_RCAP 6
#endif
constexpr int kRoundToks = 64;
constexpr int kRoundCap = PF_K5_RCAP * kPostThreads;
constexpr uint32_t kPostIdxLimit = 1u << 24;  // entry = idx << 8 | tf (tokens) or | multiplicity (sets)
constexpr int kPostMaxCols = 48;           // header packs the column mask into 48 bits
constexpr int kPostMinShift = 7;           // cells of >= 128 candidates (one K5s slice; a 512-block reads whole cells)

// One candidate list: entries [off, off + len) of the postings array, sorted by idx.
// cells[cell_off + c] = first entry (relative) with idx >= c << shift, c = 0 .. ncells,
// so a block's entries are a sub-range of cell (c0 >> shift) (filtered by idx when
// shift > kPostMinShift).
struct PList {
    uint32_t off, cell_off, shift, len;
};

// Query token of the postings scan: dot += wq * (tf * idf)  (recommender.cpp:74-85)
struct QTok {
    PList l;
    double wq, idf;
};

// Active query column: tokens [j0, j1) of the QTok array, in ascending tid order.
struct QCol {
    int32_t t, j0, j1, pad;
};

// Postings query image: QConst | QPostHead | QTok[n_tok] | QCol[n_act] | PList[n_club + n_friend] | int32 excl[n_excl]
struct QPostHead {
    int32_t n_tok, n_act, n_club, n_friend;
    int32_t n_excl, tok_off, col_off, set_off;   // byte offsets from the image start
    int32_t excl_off, pad0, pad1, pad2;
};

// Device postings store.  hdr[2 * idx + 0] = {colmask lo, colmask hi16 | pub << 16 | gen << 24,
// (u16) completion | (u16) age << 16, n_clubs | n_friends << 16}; hdr[2 * idx + 1] =
// {region0, region1, region2, uid}.
struct PostStore {
    const uint4* hdr;
    const uint32_t* post;     // entries: idx << 8 | tf (token lists), idx << 8 | multiplicity (set lists)
    const double* pnorm;      // [token entries] sqrt(sum (tf*idf)^2) of the entry's (candidate, column)
    const uint32_t* cells;
    int32_t n;                // candidates
    int32_t n_blocks;         // ceil(n / bsize)
    int32_t bsize;            // candidates per block (<= kBlockCands)
    uint32_t n_post;          // entries of post (token entries first: pnorm has n_tok_entries)
    uint32_t n_tok_entries;
    uint32_t n_cells;
};


// ---------------------------------------------------------------- device job pipeline (K3, K6-K8)
// The reference's recommenders (recommender_graph.cpp:10-237, recommender_clubs.cpp:10-73) run
// as device stages over a batch of jobs: K3 gathers each job's ordered 2-hop candidates on the
// CSR adjacency, K6 builds the query images of the job's users, K1' scores every pair, K4'
// sums the collaborative scores, K7 accumulates club scores in the reference's loop order, K8
// keeps each job's top-k.  The host plans sizes (1-hop only) and never walks the 2-hop graph.
enum DevJobKind {
    kDjInterest = 0,   // recommend_graph_registration / by_interest: gather_candidates_local, filtered
    kDjCollab = 1,     // recommend_collaborative
    kDjClubs = 2,      // recommend_clubs_collab
    kDjAll = 3,        // every candidate (interest, top-k beyond the scan kernels' bound)
    kDjRawGraph = 4,   // pf_fof_candidates, PF_FOF_GRAPH (uids of the raw list)
    kDjRawCollab = 5,  // pf_fof_candidates, PF_FOF_COLLAB
};

// Graph nodes: 0 .. n-1 are the profiles (node = candidate idx), n .. M-1 the uids of
// adj_list without a profile.  Rows are adj_list's, in its order, as node ids.
struct DevJobsStore {
    // query-image inputs (K6)
    const QConst* tmpl;         // the query-independent QConst fields
    const double* sig_reg;      // [a_regcnt 4][b 4][m 4]
    const int32_t* comp_vals;   // sorted distinct completion values > 0 ...
    const double* comp_rows;    // ... and their sig_comp rows [kValTab + 1]
    const int32_t* age_vals;
    const double* age_rows;
    int32_t n_comp, n_age;
    const int64_t* idf_dense_off;  // [T] a column's float idf by tid rank, -1 = no idf map (1.0)
    const int32_t* idf_dense_len;  // [T]
    const float* idf_dense;
    const int32_t* slot_of;     // [n] idx -> tile-store slot
    // graph
    const int64_t* g_off;       // [M] row start in g_nbr
    const int32_t* g_len;       // [M] row length, -1 = no adj_list row
    const int32_t* g_nbr;
    const int32_t* g_uid;       // [M]
    int32_t n, M;
    // clubs (K7): per profile idx its clubs as dense club indices, in profile order
    const int64_t* club_off;    // [n + 1]
    const int32_t* club_dense;
    const int32_t* club_id;     // [n_club_ids] dense index -> club id
    int32_t n_club_ids, pad;
};

// Row overrides one call sees, sorted by (node asc, version desc): pf_set_adj edits (version
// INT32_MIN: always visible) and the batched drivers' versioned edits (visible to jobs whose
// version is >= theirs).  len -1 = the row is erased.
struct DevView {
    const int32_t* node;
    const int32_t* ver;
    const int64_t* off;         // into nbr
    const int32_t* len;
    const int32_t* nbr;
    int32_t n, pad;
};

// One job of a batch (host-planned; every offset is into the batch's workspaces).
struct DevJob {
    int32_t kind, u, L, version;       // u = query node; L = max(limit, 1)
    int32_t own, own_len;              // own row override (node or -1), its length (-1 = erased)
    int64_t own_off;                   // own row's nodes in the plan's int32 pool
    int64_t f_off;                     // row(u) as nodes in the plan's int32 pool
    int32_t nf;                        // |row(u)|
    int32_t ht_lg;                     // gather hash-table capacity log2
    int64_t ht_off;                    // keys | pos | flags (3 << ht_lg int32) in the hash workspace
    int64_t seg_off;                   // per friend: prefix (nf + 1) int32 in the seq workspace
    int64_t cand_off;                  // candidate slots / ids (cap entries) in the slot / id arrays
    int32_t cap;                       // candidate region size
    int32_t nfd;                       // distinct friends with a profile (collab / clubs)
    int64_t fd_off;                    // Fd nodes (nfd) in the plan's int32 pool; then their slots
    int64_t fpos_off;                  // per row(u) position: index into Fd or -1 (plan int32 pool)
    int64_t sim_off;                   // pair outputs FAS(u, Fd[r]) (nfd floats)
    int64_t m_off;                     // collab: M[r][c] (nfd x cap floats)
    int64_t sreg_off;                  // clubs: per Fd r, the element offset of its S region (plan int64 pool)
    int64_t out_off;                   // scored list (score float, id int32), cap entries
    int32_t topk, pad;
};

}  // namespace pf
