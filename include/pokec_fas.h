/*
 * pokec_fas.h — C ABI of the MI355X-native Fill-Aware-Similarity (FAS) engine.
 *
 * Drop-in boundary for the hot path of pymlex/recommendation-system-pokec:
 *   - Recommender::profile_similarity        src/recommender_similarity.cpp:10-124  (FAS, A10)
 *   - Recommender::tfidf_cosine_for_column   src/recommender.cpp:68-117             (A6)
 *   - Recommender::vec_set_similarity        src/recommender.cpp:119-128            (A8)
 *   - Recommender::region_similarity_local   src/recommender.cpp:130-139            (A9)
 *   - Recommender::compute_idf_from_profiles src/recommender.cpp:43-66              (A4)
 *   - gather_candidates_local                src/recommender_graph.cpp:10-31        (A11)
 *   - recommend_graph_registration / _by_interest  src/recommender_graph.cpp:33-103,224-227 (A12)
 *   - recommend_collaborative                src/recommender_graph.cpp:105-222      (A14)
 *   - recommend_clubs_collab                 src/recommender_clubs.cpp:10-73        (A15)
 *   - build_adj_list / GraphBuilder          src/utils.cpp:26-34, src/graph_builder.cpp:39-59 (A17)
 *
 * The reference exposes these as methods of the C++ class `Recommender`
 * (include/recommender.h:17-71).  This header is the flat C ABI the C++
 * facade (include/pokec/recommender.h) and any FFI (ctypes, cgo, JNI) bind.
 * Shape follows the reference's only FFI precedent, lemmagen
 * (third_party/lemmagen/include/lemmagen.h:40-76): extern "C", int status
 * codes, caller-owned buffers, no exceptions across the boundary.
 *
 * Conventions
 *   - 0 = PF_OK, < 0 = error; pf_last_error() describes the last failure.
 *   - All pointers in pf_corpus_desc are HOST pointers owned by the caller;
 *     pf_open copies everything it needs to the GPU and keeps no reference.
 *   - An unknown query uid yields count 0 (the reference returns an empty
 *     vector: recommender_graph.cpp:36-40,130; recommender_clubs.cpp:13-16).
 *   - One context per host thread; distinct contexts are independent.
 *   - There is NO CPU fallback: if the HIP runtime or a gfx950 device is
 *     missing, pf_open fails with PF_ENODEV.
 */
#ifndef POKEC_FAS_H
#define POKEC_FAS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PF_ABI_VERSION 2

/* status codes */
#define PF_OK          0
#define PF_EINVAL     -1   /* bad argument / malformed descriptor            */
#define PF_ENODEV     -2   /* no HIP device / HIP runtime failure            */
#define PF_ENOMEM     -3   /* host or device allocation failed               */
#define PF_ENOTFOUND  -4   /* query uid has no profile (outputs count 0)     */
#define PF_EUNSUPP    -5   /* input outside what the device layout encodes   */
#define PF_EINTERNAL  -6

/* Number of fixed (structured) fields of FAS, recommender_similarity.cpp:12 */
#define PF_NUM_FIXED   7
#define PF_MAX_COLS    64
/* fixed-field normaliser slots, recommender_similarity.cpp:28-91 order */
#define PF_F_PUBLIC     0
#define PF_F_GENDER     1
#define PF_F_COMPLETION 2
#define PF_F_AGE        3
#define PF_F_REGION     4
#define PF_F_CLUBS      5
#define PF_F_FRIENDS    6

/* IDF source (Recommender::compute_idf_from_profiles vs set_tfidf_index) */
#define PF_IDF_FROM_PROFILES 0  /* idf = logf(1 + N/(1+df)), recommender.cpp:43-66 */
#define PF_IDF_EXPLICIT      1  /* use idf_* arrays below (set_tfidf_index)          */

/* candidate-set modes for interest scoring */
#define PF_MODE_FOF   0  /* reference: 2-hop candidates truncated at candidate_limit (A12) */
#define PF_MODE_ALL   1  /* every loaded profile except q and adj[q] (A13)                 */

/* 2-hop gather flavours (they differ, see A11 vs A14 in SURVEY.md) */
#define PF_FOF_GRAPH  0  /* gather_candidates_local, recommender_graph.cpp:10-31  */
#define PF_FOF_COLLAB 1  /* collaborative candidate loop, recommender_graph.cpp:114-125 */

/*
 * In-memory corpus: the reference's unordered_map<int,UserProfile>
 * (include/user_profile.h:10-20) plus adj_list, normalisers and IDF,
 * flattened to CSR.  Profiles may be given in any order; user ids must be
 * distinct.  Ages must already be median-filled (api_cli.cpp:139-153).
 */
typedef struct pf_corpus_desc {
    int32_t         n_users;
    int32_t         n_cols;        /* T: number of text columns (<= PF_MAX_COLS)  */

    const int32_t*  user_id;       /* [n_users]                                    */
    const int32_t*  public_flag;   /* [n_users]  -1 = missing                      */
    const int32_t*  completion;    /* [n_users]  used when > 0                     */
    const int32_t*  gender;        /* [n_users]  -1 = missing                      */
    const int32_t*  age;           /* [n_users]  used when > 0                     */
    const int32_t*  region;        /* [3*n_users] -1 = missing part                */

    const int64_t*  club_off;      /* [n_users+1]                                  */
    const uint32_t* club_ids;      /* clubs in profile order, duplicates allowed   */
    const int64_t*  friend_off;    /* [n_users+1]                                  */
    const uint32_t* friend_ids;    /* profile `friends` column (NOT adj_list)      */

    const int64_t*  tok_off;       /* [n_users*n_cols+1], row (u,t) = u*n_cols+t   */
    const int32_t*  tok_tid;       /* token ids; distinct within a row             */
    const int32_t*  tok_tf;        /* token counts                                 */

    /* adj_list (unordered_map<int, vector<int>>): directed, file order, dups kept */
    int32_t         n_adj;
    const int32_t*  adj_uid;       /* [n_adj] distinct                             */
    const int64_t*  adj_off;       /* [n_adj+1]                                    */
    const int32_t*  adj_nbr;

    /* IDF (idf_per_col).  idf_mode = PF_IDF_FROM_PROFILES ignores the arrays.
     * PF_IDF_EXPLICIT: col_has_idf[t] = 0 means the column name is absent from
     * idf_per_col (raw-count cosine, recommender_similarity.cpp:102-104);
     * otherwise row t of (idf_off, idf_tid, idf_val) is its map; a token absent
     * from a present map gets idf 1.0 (recommender.cpp:78). */
    int32_t         idf_mode;
    const uint8_t*  col_has_idf;   /* [n_cols]                                     */
    const int64_t*  idf_off;       /* [n_cols+1]                                   */
    const int32_t*  idf_tid;
    const float*    idf_val;

    /* normalisers, slots 0..6 = field_normalizers["public".."friends"],
     * 7+t = column_normalizers[text_columns[t]]; norm_present = 0 means the key
     * is absent (then z = 6(s-0.5), recommender_similarity.cpp:28-36). */
    const uint8_t*  norm_present;  /* [PF_NUM_FIXED + n_cols]                      */
    const float*    norm_mean;
    const float*    norm_sd;
} pf_corpus_desc;

typedef struct pf_ctx pf_ctx;

int         pf_abi_version(void);
/* Copies the corpus to device `device` (HIP ordinal) and builds the tile store. */
int         pf_open(const pf_corpus_desc* desc, int device, pf_ctx** out);
void        pf_close(pf_ctx* ctx);
/* Message of the last failure on ctx (or of the last failed pf_open when ctx is NULL). */
const char* pf_last_error(const pf_ctx* ctx);
int32_t     pf_num_users(const pf_ctx* ctx);
/* float32 IDF the context uses for (col, tid); 1.0 for an absent token; NaN when
 * the column has no idf map (raw-count cosine). */
float       pf_idf(const pf_ctx* ctx, int32_t col, int32_t tid);

/* FAS(A=a_uid[i], B=b_uid[i]) for n pairs (profile_similarity(A,B)); a pair with
 * an unknown uid scores NaN.  Parity probe for recommender_similarity.cpp:10-124. */
int pf_fas_pairs(pf_ctx* ctx, const int32_t* a_uid, const int32_t* b_uid,
                 int64_t n, float* out);

/*
 * Top-k recommenders.  For every query i the results go to
 * out_uid[i*topk .. ], out_score[i*topk .. ], out_count[i] (<= topk), sorted
 * by (score desc, id asc) exactly as recommender_graph.cpp:97-101.
 *   pf_recommend_interest: mode PF_MODE_FOF = recommend_graph_registration /
 *       recommend_by_interest(u, topk, candidate_limit); PF_MODE_ALL = the
 *       all-candidates scan (candidate_limit ignored).
 *   pf_recommend_collab:  recommend_collaborative(u, topk, candidate_limit).
 *   pf_recommend_clubs:   recommend_clubs_collab(u, topk, candidate_limit)
 *       (ids are club ids).
 * Returns PF_OK even when some queries are unknown (their count is 0).
 */
int pf_recommend_interest(pf_ctx* ctx, const int32_t* query_uid, int32_t nq,
                          int32_t topk, int32_t mode, int32_t candidate_limit,
                          int32_t* out_uid, float* out_score, int32_t* out_count);
int pf_recommend_collab(pf_ctx* ctx, const int32_t* query_uid, int32_t nq,
                        int32_t topk, int32_t candidate_limit,
                        int32_t* out_uid, float* out_score, int32_t* out_count);
int pf_recommend_clubs(pf_ctx* ctx, const int32_t* query_uid, int32_t nq,
                       int32_t topk, int32_t candidate_limit,
                       int32_t* out_uid, float* out_score, int32_t* out_count);

/*
 * Asynchronous forms of the three job recommenders (interest in PF_MODE_FOF): the call plans the
 * batch on the host and queues its device stages on the context's stream, then returns; the
 * outputs (same layout as above) are written when pf_wait(ctx, ticket) returns, so the caller
 * keeps its buffers alive until then.  While call i runs on the device the host can plan call
 * i + 1: one context then keeps the GPU busy where the synchronous calls leave it idle during
 * planning (what several contexts per GPU were used for).  At most three calls are in flight: a
 * fourth waits for the oldest itself.  Any other call on the context (synchronous recommenders,
 * pf_set_adj, pf_jobs_stats_*) first completes the pending ones; pf_close drops them unwritten.
 * pf_wait(ticket) completes every call up to that ticket, in launch order; it returns the first
 * failure among them (PF_OK for a ticket already completed).
 */
int pf_recommend_interest_async(pf_ctx* ctx, const int32_t* query_uid, int32_t nq, int32_t topk,
                                int32_t candidate_limit, int32_t* out_uid, float* out_score,
                                int32_t* out_count, uint64_t* ticket);
int pf_recommend_collab_async(pf_ctx* ctx, const int32_t* query_uid, int32_t nq, int32_t topk,
                              int32_t candidate_limit, int32_t* out_uid, float* out_score,
                              int32_t* out_count, uint64_t* ticket);
int pf_recommend_clubs_async(pf_ctx* ctx, const int32_t* query_uid, int32_t nq, int32_t topk,
                             int32_t candidate_limit, int32_t* out_uid, float* out_score,
                             int32_t* out_count, uint64_t* ticket);
int pf_wait(pf_ctx* ctx, uint64_t ticket);
/* The highest ticket whose call has completed (its outputs written): every ticket <= it is
 * done, by pf_wait or by another call that completed the pending ones first.  0 when no
 * asynchronous call has completed (or ctx is NULL).  Bindings drop their references to a
 * call's output buffers once its ticket is <= this. */
uint64_t pf_completed_ticket(const pf_ctx* ctx);

/* Ordered, de-duplicated, limit-truncated 2-hop candidate list of uid
 * (flavour PF_FOF_GRAPH or PF_FOF_COLLAB).  Writes at most `cap` ids; *n gets
 * the full list length. */
int pf_fof_candidates(pf_ctx* ctx, int32_t uid, int32_t limit, int32_t flavour,
                      int32_t* out, int32_t cap, int32_t* n);

/* Replace adj_list[uid] (hold-out drivers mutate the adjacency between
 * queries: test.cpp:73, recommendation_tests.cpp:111-114).  n = -1 erases the
 * row (uid absent from adj_list). */
int pf_set_adj(pf_ctx* ctx, int32_t uid, const int32_t* nbrs, int32_t n);

/* Restrict the all-candidates scan to shard `shard` of `nshards`: contiguous
 * candidate ranges of equal stream bytes (K1 tiles) and of equal posting weight
 * (K5 blocks: a fixed share per candidate plus its tokens, clubs and friends);
 * the multi-GPU path merges the per-shard top-k. */
int pf_set_shard(pf_ctx* ctx, int32_t shard, int32_t nshards);

/* All-candidates scan kernel.  PF_SCAN_AUTO (default) takes the postings scan
 * (K5: per-token candidate lists, only the lists the query names are read) when the
 * corpus fits its encoding, else the record-stream scan (K1: every candidate's record
 * is walked).  Both give bit-identical results; forcing POSTINGS on a corpus outside
 * its encoding returns PF_EUNSUPP. */
#define PF_SCAN_AUTO     0
#define PF_SCAN_STREAM   1
#define PF_SCAN_POSTINGS 2
int pf_set_scan_kernel(pf_ctx* ctx, int32_t kind);

/*
 * Device-resident all-candidates scan for the multi-GPU bench: scores the
 * queries against this context's shard and writes, per query, `topk` packed
 * 64-bit keys to DEVICE memory d_keys[nq*topk] on `stream` (a hipStream_t).
 * Key = (~orderable(score) << 32) | (uid ^
 * 0x80000000): ascending key = (score desc, uid asc); unused slots are
 * UINT64_MAX.  `stream` is used as given (NULL = the HIP null stream, not the
 * context's stream), so the caller's collectives on that stream are ordered
 * after the scan.  No host synchronisation.
 * The context's device workspaces (query images, partial keys, rendezvous
 * tickets) are shared by every call on it: all calls on one context must be
 * serialised on ONE stream (the context's own calls use its internal stream and
 * synchronise before returning, so mixing them with this call is safe only after
 * the caller has synchronised `stream`).
 * nq = 1 on a stream other than the context's runs on the context's scan lanes:
 * the launch goes to the next lane's stream (the context's stream and its two aux
 * streams in turn; seven eighths of a resident round of workgroups each) without waiting for work the caller queued on `stream`
 * earlier, and `stream` waits for it and copies its row into d_keys, in call
 * order; so consecutive single-query calls overlap on the device.  A single
 * query whose resident postings image is current (built at pf_open; a
 * pf_set_adj of that user makes it stale) builds and uploads nothing: one
 * launch, one wait, one row copy.
 */
int pf_scan_keys_async(pf_ctx* ctx, const int32_t* query_uid, int32_t nq,
                       int32_t topk, uint64_t* d_keys, void* stream);
/* Merge nparts key lists laid out [part][nq][topk] (device) into d_out[nq][topk]
 * on `stream` (as given, NULL = null stream). */
int pf_merge_keys_async(pf_ctx* ctx, const uint64_t* d_parts, int32_t nparts,
                        int32_t nq, int32_t topk, uint64_t* d_out, void* stream);
/* Host-side decode of packed keys; count = number of non-empty keys. */
void pf_decode_keys(const uint64_t* keys, int32_t n, int32_t* out_uid,
                    float* out_score, int32_t* count);

/* Statistics of the device layout (for roofline accounting). */
typedef struct pf_layout_stats {
    int64_t n_slots;          /* candidates in the tile store                  */
    int64_t stream_bytes;     /* bytes of the interleaved record stream        */
    int64_t header_bytes;     /* bytes of the fixed per-candidate headers      */
    int64_t alg_bytes;        /* sum 32+4|clubs|+4|friends|+8nnz */
    int32_t packed_tokens;    /* 1 if tokens are stored as one word            */
    int32_t n_tiles;
    int64_t post_bytes;       /* postings store: entries + norms + cells + headers (0 if absent) */
    int32_t scan_kernel;      /* kernel the next all-candidates scan uses: PF_SCAN_STREAM / PF_SCAN_POSTINGS */
    int32_t pad;
    int64_t shard_cands;      /* candidates in this context's shard (pf_set_shard) for that kernel */
    int64_t shard_entries;    /* their postings entries (tokens, clubs, friends; 0 without postings) */
} pf_layout_stats;
int pf_layout(const pf_ctx* ctx, pf_layout_stats* out);

/* Bytes the all-candidates scan kernel reads from device memory for each query
 * over this context's shard, by the kernel's access pattern (the physical byte
 * model of DESIGN.md section 4): K5 = per candidate block, the 32-B headers, two
 * cell words per query list and every entry of each list's cell range (4 B;
 * token entries also their 8-B norm), the exclusion list, and the staged query
 * image per workgroup; K1 = the shard's record stream and headers.  0 for an
 * unknown uid.  The nq queries are taken as ONE launch, as pf_recommend_interest
 * runs them: nq = 1 is the single-query scan (one resident round of workgroups,
 * each staging the image once); nq > 1 a batch (each workgroup stages its query's
 * image once for its four blocks). */
int pf_scan_bytes(pf_ctx* ctx, const int32_t* query_uid, int32_t nq, int64_t* out_bytes);

/* Statistics of the recommenders' device job pipeline (pf_recommend_collab / _clubs /
 * _interest FoF and the batched drivers) since pf_jobs_stats_reset(ctx, 1): jobs run,
 * candidate-list entries scored, FAS pairs scored by the pair kernel (K1'), their
 * SURVEY 8(d) D3 bytes (b_c of each pair's candidate), the bytes the pair-scoring stage
 * reads for them by access pattern (pair_record_bytes: the 48-B headers + the record words
 * of every pair's candidate), the staged query-image bytes (one image per 512-pair block),
 * and the pair-scoring stage's device time (HIP events around K1' in each launch) and
 * launch count.  enable: bit 0 = time the pair kernel (HIP events around each
 * launch), bit 1 = count pairs and bytes (one extra small kernel per launch); 0 stops
 * both.  Fields of a part that is off read 0.  pair_dispatches: every pair-kernel (K1')
 * dispatch since pf_open (the job pipeline's stages, up to three per stage by image LDS
 * class, and pf_fas_pairs), never reset, so a profiler's per-dispatch rows can be grouped
 * into the calls they belong to. */
typedef struct pf_jobs_stats {
    int64_t jobs, candidates, pairs;
    int64_t pair_alg_bytes, pair_record_bytes, pair_image_bytes;
    double  pair_ms;
    int64_t pair_launches;
    int64_t pair_dispatches;
} pf_jobs_stats;
int pf_jobs_stats_reset(pf_ctx* ctx, int32_t enable);
int pf_jobs_stats_read(pf_ctx* ctx, pf_jobs_stats* out);

/* Device time (ms) of the last all-candidates scan kernel (HIP events on the
 * stream it was launched on). */
float pf_last_scan_ms(const pf_ctx* ctx);
/* Per-launch timing of the scan kernel over a region: reset, run, then read the
 * summed device time of every scan launch since the reset (synchronises). */
int pf_profile_reset(pf_ctx* ctx);
int pf_profile_read(pf_ctx* ctx, double* total_ms, int64_t* launches);
/* Time only scan launches 0, every, 2*every, ... after a reset (default 1 = all); the
 * others run without timing events.  *launches in pf_profile_read counts timed launches.
 * every = 0 turns profiling off (until the next pf_profile_reset).  At most 65536 launches
 * are timed per reset; later ones run untimed. */
int pf_profile_sample(pf_ctx* ctx, int32_t every);

#ifdef __cplusplus
}
#endif
#endif /* POKEC_FAS_H */
