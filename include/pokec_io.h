/*
 * pokec_io.h — C ABI of the host-side data path around the FAS engine: the
 * reference's start-up loaders and its hold-out drivers, in front of
 * pokec_fas.h.
 *
 *   pf_dataset_load      api_cli.cpp:86-167 start-up, from a directory holding
 *                        config/text_columns.txt and data/:
 *                          load_text_columns_from_file   src/utils.cpp:13-24
 *                          GraphBuilder::load_serialized src/graph_builder.cpp:39-59   (A17)
 *                          build_adj_list                src/utils.cpp:26-34           (A17)
 *                          load_users_encoded            src/user_loader.cpp:10-96     (A2)
 *                          split_csv_line / parse_tok_field src/utils.cpp:36-68        (A2)
 *                          load_median_age / compute_median_age_from_profiles /
 *                          fill_missing_ages             src/user_loader.cpp:98-140    (A3)
 *                          load_column_normalizers       src/utils.cpp:123-142         (A18)
 *                          VocabBuilder::load_vocab (club names only)
 *                                                        src/vocab_builder.cpp:133-197
 *   pf_dataset_profile_json  write_profile_json          src/api_cli.cpp:49-84
 *   pf_compute_normalizers   compute_column_normalizers + save_column_normalizers
 *                                                        src/utils.cpp:144-240         (A18)
 *   pf_holdout_friends       run_friends_holdout_test    src/test.cpp:13-105           (A19)
 *   pf_recommendation_tests  run_recommendation_tests_sample
 *                                                        src/recommendation_tests.cpp:68-169 (A19)
 *   pf_eval_holdout_friends / pf_eval_recommendation_tests: the same two drivers batched and
 *                            sharded over GPUs (F1, cfg 5)
 *
 * The loaders keep the reference's hash containers (same key types, same
 * insertion sequence), so every order the reference derives from
 * unordered_map iteration is reproduced: the profile order the drivers
 * shuffle, the adjacency order, and the token order in profile JSON.
 * The loaders run on the host only and need no GPU. The drivers call the engine.
 * Status codes and pf_last_error(NULL) are shared with pokec_fas.h.
 */
#ifndef POKEC_IO_H
#define POKEC_IO_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "pokec_fas.h"

#ifdef __cplusplus
extern "C" {
#endif

/* load_users_encoded reads at most this many data lines (user_loader.cpp:34) */
#define PF_LOAD_REFERENCE_CAP 100000

typedef struct pf_dataset pf_dataset;

typedef struct pf_dataset_info {
    int64_t lines_read;      /* data lines consumed by the user loader (its counter c)  */
    int32_t n_profiles;      /* profiles after de-duplication by uid                    */
    int32_t n_cols;          /* text columns                                            */
    int32_t n_adj;           /* adjacency rows                                          */
    int32_t median_age;      /* loaded or computed median                               */
    int32_t median_loaded;   /* 1: from data/median_age.txt                             */
    int32_t ages_replaced;   /* zero ages filled with the median                        */
    int32_t n_normalizers;   /* entries of column_normalizers.csv (0 = absent/empty)    */
    int32_t vocab_loaded;    /* 1: data/tokens.csv exists (VocabBuilder::load_vocab)    */
    int32_t n_club_names;
} pf_dataset_info;

/* Load `root`/config + `root`/data like api_cli's start-up.  max_lines caps
 * the user loader's data lines (PF_LOAD_REFERENCE_CAP reproduces the
 * reference; 0 = no cap, for the full 1.6M-user configurations).  Fails with
 * PF_EINVAL when config/text_columns.txt, data/users_encoded.csv or
 * data/adjacency.csv cannot be read. */
int pf_dataset_load(const char* root, int64_t max_lines, pf_dataset** out);
/* F2 (no reference symbol; the reference re-parses the CSVs at every start, user_loader.cpp:
 * 10-96, graph_builder.cpp:39-59): pf_dataset_load with a binary cache of the parse at
 * cache_path.  A cache whose key (the sizes and mtimes of users_encoded.csv and
 * adjacency.csv, max_lines, the text columns) matches is read instead of the CSVs; otherwise
 * the CSVs are parsed and the cache is (re)written, best effort (a failed write is not an
 * error).  *from_cache (may be NULL) gets 1 when the cache served.  The result, its
 * iteration orders included, equals pf_dataset_load's.  cache_path NULL = pf_dataset_load. */
int pf_dataset_load_cached(const char* root, int64_t max_lines, const char* cache_path, int32_t* from_cache,
                           pf_dataset** out);
void pf_dataset_free(pf_dataset* ds);
/* Engine input view (valid while ds lives): IDF from profiles, normalisers as loaded. */
const pf_corpus_desc* pf_dataset_desc(const pf_dataset* ds);
int pf_dataset_info_get(const pf_dataset* ds, pf_dataset_info* out);
/* Text column name t (NULL if out of range). */
const char* pf_dataset_column(const pf_dataset* ds, int32_t t);
/* uids in the iteration order of the reference's profiles map / adj_list map;
 * *n gets the full count, at most cap ids are written. */
int pf_dataset_profile_order(const pf_dataset* ds, int32_t* out, int32_t cap, int32_t* n);
int pf_dataset_adj_order(const pf_dataset* ds, int32_t* out, int32_t cap, int32_t* n);
/* write_profile_json for uid into buf (NUL-terminated when it fits); *len gets the
 * length without the NUL.  PF_ENOTFOUND for an unknown uid. */
int pf_dataset_profile_json(const pf_dataset* ds, int32_t uid, char* buf, int64_t cap, int64_t* len);
/* Club slug for a club id from data/clubs_map.csv (NULL if none). */
const char* pf_dataset_club_name(const pf_dataset* ds, int32_t club_id);

/* compute_column_normalizers(profiles, text_columns, sample_size, comps_per_user) as
 * kurs runs it when data/column_normalizers.csv is missing (main.cpp:118-128): the
 * mt19937(12345) pair sampler over the profiles map in the reference's iteration
 * order, field and raw-count column similarities, sample mean / sd per key.  A host
 * statistic of the offline step (the pairs are random, so there is no scan to run),
 * bit-exact with the reference.  Writes PF_NUM_FIXED + n_cols (mean, sd) pairs in the
 * pf_corpus_desc slot order to out_mean/out_sd (either may be NULL) and, when
 * save_csv is not NULL, the CSV save_column_normalizers writes (same key order and
 * number formatting). */
int pf_compute_normalizers(const pf_dataset* ds, int32_t sample_size, int32_t comps_per_user, const char* save_csv,
                           float* out_mean, float* out_sd);

/* run_friends_holdout_test: per tested user, hits/hold_k in file order.
 * ctx must have been opened on pf_dataset_desc(ds); its adjacency is restored on return. */
int pf_holdout_friends(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, double* out_ratios, int32_t cap,
                       int32_t* n_out);
/* run_recommendation_tests_sample: out[5] = {graph_hit_rate, collab_hit_rate,
 * interest_hit_rate, avg_club_prec_at_k, avg_club_recall_at_k}. */
int pf_recommendation_tests(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk, double* out5);

/* Result digest of one recommender call (a parity probe): FNV-1a over the 32-bit words of
 * every returned (id, score bits) pair in result order, then the count.  Two runs returned the
 * same list, ids and score bits, iff (practically) their digests are equal. */
static inline uint64_t pf_result_digest(const int32_t* ids, const float* scores, int32_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (int32_t i = 0; i < n; ++i) {
        uint32_t w[2];
        w[0] = (uint32_t)ids[i];
        memcpy(&w[1], &scores[i], 4);
        for (int k = 0; k < 2; ++k) {
            h ^= w[k];
            h *= 0x100000001b3ull;
        }
    }
    h ^= (uint32_t)n;
    h *= 0x100000001b3ull;
    return h;
}

/* The two drivers with every tested user's results as digests (parity probes of the
 * drivers' adjacency handling; the metrics alone cannot see most of a wrong list, e.g.
 * recommend_clubs_collab never returns the user's own clubs, so the club precision of
 * recommendation_tests.cpp:140-153 is always 0):
 *   pf_holdout_friends_digest:      out_digest[i] = user i's collaborative list;
 *   pf_recommendation_tests_digest: out_digest[4i .. 4i+3] = graph, collaborative, interest,
 *                                   clubs lists of user i.
 * *n_out = users tested.  The batched forms below have _digest twins in plan order. */
int pf_holdout_friends_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, uint64_t* out_digest,
                              int32_t cap, int32_t* n_out);
int pf_recommendation_tests_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk,
                                   uint64_t* out_digest, int32_t cap, int32_t* n_out);

/* Batched, shardable forms of the two drivers (BASELINE cfg 5).  The plan
 * (sampled users and their held-out friends, in the sequential driver's rng order) is computed
 * up front; each user's query reads the adjacency it would have seen (test.cpp: every earlier
 * user's edit, one adj_mod for the run; recommendation_tests.cpp: only its own row) through a
 * view, so users are independent: shard s of n evaluates plan entries i with i % n == s,
 * `batch` users per GPU pass, and writes per-entry results (other entries untouched):
 *   pf_eval_holdout_friends:      out_ratio[i]
 *   pf_eval_recommendation_tests: out_hits[3i .. 3i+2] = graph / collaborative / interest hit
 *                                 (0/1); out_club[2i], out_club[2i+1] = club precision,
 *                                 recall@k, NaN for a user without clubs.
 * *n_plan = plan length.  Averaging the merged entries in plan order reproduces
 * pf_holdout_friends / pf_recommendation_tests bit for bit. */
int pf_eval_holdout_friends(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t shard,
                            int32_t nshards, int32_t batch, double* out_ratio, int32_t cap, int32_t* n_plan);
int pf_eval_recommendation_tests(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk,
                                 int32_t shard, int32_t nshards, int32_t batch, int8_t* out_hits,
                                 double* out_club, int32_t cap, int32_t* n_plan);
/* Asynchronous form of pf_eval_recommendation_tests (BASELINE cfg 5's step): the batches are
 * planned and queued as the synchronous form does, but the call returns with its last chunk still
 * on the device; out_hits / out_club are written when pf_wait(ctx, *ticket) returns, or when the
 * next call on the context that uses the job pipeline completes it first (that call plans and
 * launches its own first chunk before, so one context overlaps step i + 1's host planning with
 * step i's last device chunk).  The caller keeps the output buffers alive until then; the call
 * holds ds (its driver reads ds's profiles when its last chunk is unpacked), so a pf_dataset_free
 * meanwhile defers the delete until the call completes or its context is closed.  *n_plan is
 * written before this returns. */
int pf_eval_recommendation_tests_async(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk,
                                       int32_t shard, int32_t nshards, int32_t batch, int8_t* out_hits,
                                       double* out_club, int32_t cap, int32_t* n_plan, uint64_t* ticket);
/* digests of the plan entries this shard evaluates (layout as the sequential _digest forms) */
int pf_eval_holdout_friends_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t shard,
                                   int32_t nshards, int32_t batch, uint64_t* out_digest, int32_t cap,
                                   int32_t* n_plan);
int pf_eval_recommendation_tests_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk,
                                        int32_t shard, int32_t nshards, int32_t batch, uint64_t* out_digest,
                                        int32_t cap, int32_t* n_plan);

#ifdef __cplusplus
}
#endif
#endif /* POKEC_IO_H */
