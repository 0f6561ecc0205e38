/* refcpu — clean-room CPU restatement of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (the parity checker and bench.py's cpu_baseline
 * leg).  The product library never links or calls it.  Parity of this
 * restatement is pinned against golden vectors produced by the real reference
 * (oracle/gen_golden.py -> tests/golden/), see tests/test_oracle_golden.py.
 *
 * It keeps the reference's data structures on purpose (unordered_map per
 * profile and per text column, hash-set based set overlap) so that its timing
 * is a faithful stand-in for the reference CPU path on the GPU box, where the
 * reference itself is not available.
 */
#ifndef POKEC_REFCPU_H
#define POKEC_REFCPU_H
#include <stdint.h>
#include "pokec_fas.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef struct ro_ctx ro_ctx;
/* max_users > 0 keeps only the first max_users profiles of desc (bounded CPU samples) */
int   ro_open(const pf_corpus_desc* d, int32_t max_users, ro_ctx** out);
void  ro_close(ro_ctx* h);
/* profile_similarity evaluations since the last reset (reset != 0 zeroes the count) */
int64_t ro_fas_calls(ro_ctx* h, int reset);
int32_t ro_num_users(const ro_ctx* h);
float ro_idf(const ro_ctx* h, int32_t col, int32_t tid);
int   ro_fas_pairs(ro_ctx* h, const int32_t* a, const int32_t* b, int64_t n, float* out);
int   ro_recommend_interest(ro_ctx* h, const int32_t* q, int32_t nq, int32_t topk, int32_t mode,
                            int32_t limit, int32_t* out_uid, float* out_score, int32_t* out_count);
int   ro_recommend_collab(ro_ctx* h, const int32_t* q, int32_t nq, int32_t topk, int32_t limit,
                          int32_t* out_uid, float* out_score, int32_t* out_count);
int   ro_recommend_clubs(ro_ctx* h, const int32_t* q, int32_t nq, int32_t topk, int32_t limit,
                         int32_t* out_uid, float* out_score, int32_t* out_count);
int   ro_fof_candidates(ro_ctx* h, int32_t uid, int32_t limit, int32_t flavour, int32_t* out,
                        int32_t cap, int32_t* n);
int   ro_set_adj(ro_ctx* h, int32_t uid, const int32_t* nbrs, int32_t n);
/* profiles iteration order (unordered_map<int,UserProfile>) */
int   ro_profile_order(const ro_ctx* h, int32_t* out, int32_t cap);
/* test.cpp:13-105 (friends hold-out, collaborative); writes per-user ratios */
int   ro_holdout_friends(ro_ctx* h, int32_t sample, double* ratios, int32_t cap, int32_t* n);
/* recommendation_tests.cpp:68-169; metrics[5] = graph, collab, interest hit rates, club P@k, R@k */
int   ro_recommendation_tests(ro_ctx* h, int32_t sample, int32_t topk, double* metrics);
/* the same drivers with per-user result digests (pokec_io.h pf_result_digest): holdout one per
 * user (collaborative list), rectests four per user (graph, collab, interest, clubs) */
int   ro_holdout_friends_digest(ro_ctx* h, int32_t sample, uint64_t* digest, int32_t cap, int32_t* n);
int   ro_recommendation_tests_digest(ro_ctx* h, int32_t sample, int32_t topk, uint64_t* digest, int32_t cap,
                                     int32_t* n);
#ifdef __cplusplus
}
#endif
#endif
