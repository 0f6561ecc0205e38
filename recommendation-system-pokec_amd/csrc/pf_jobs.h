// pf_jobs.h — launchers of the device job pipeline (pf_jobs.hip) and its per-image plan.
#pragma once
#include <hip/hip_runtime.h>

#include "pf_kernels.h"
#include "pf_types.h"

namespace pf {

// One query image K6 builds (layout of pf_api.cpp plan_images): byte offsets into the image
// pool; lg = table log2 (load <= 0.4), lge = exclusion table log2, dlg = log2 of the set
// de-duplication table in scratch (u32 words from scr_off; the item list follows it).
struct ImgJob {
    int32_t idx, lg, lge, dlg;
    uint32_t const_off, keys_off, vals_off;
    uint32_t rows;  // (completion row + 1) | (age row + 1) << 16 in the image-builder tables (0: none;
                    // 0xFFFFFFFF: too many distinct values, K6 bisects the tables)
    int64_t scr_off;
};

hipError_t launch_gather(const DevJobsStore& g, const DevView& v, const DevJob* jobs, int njobs, const int32_t* pool,
                         const int64_t* pool64, int32_t* ht, int32_t* seq, int32_t* cand_slot, int32_t* cand_id,
                         int32_t* ncand, hipStream_t s);
// images [0, n_small) build with kImgLdsSmall bytes of LDS, the next n_big with kImgLds, the next n_glob in
// global memory
constexpr uint32_t kImgLdsSmall = 16 * 1024;
hipError_t launch_qimages(const DevStore& st, const DevJobsStore& g, const ImgJob* ij, int n_small, int n_big, int n_glob,
                          uint8_t* pool, uint32_t* scratch, int32_t* fail, hipStream_t s);
uint32_t qimage_lds(int lg, int lge, int dlg, uint32_t nitems, bool packed);
// K4' (+ the fused top-k of jobs with topk <= kMaxTopK: parts = gridDim.x * k keys per job,
// tickets = one zeroed counter per job, out = the chunk's key rows, k = their width)
hipError_t launch_collab(const DevJob* jobs, const int32_t* jix, int njobs, int max_cap, const int32_t* pool,
                         const float* pout, const int32_t* cand_slot, float* score, const int32_t* ids, uint64_t* parts,
                         unsigned int* tickets, uint64_t* out, int k, hipStream_t s);
hipError_t launch_clubs(const DevJobsStore& g, const DevView& v, const DevJob* jobs, const int32_t* jix, int njobs,
                        const int32_t* pool, const int64_t* pool64, const float* pout, double* acc,
                        float* score, int32_t* ids, int32_t* ncand, int64_t acc_stride, hipStream_t s);
// the pair blocks' dispatch order, longest first record first (pf_jobs.hip order_pairs_kernel)
hipError_t launch_expand_pairs(const PairGen* gens, int ngens, const int2* pool, int nblocks, PairBlock* blocks,
                               hipStream_t s);
hipError_t launch_order_pairs(const PairBlock* blocks, int nblocks, const int32_t* slots, int32_t n_slots,
                              int32_t* order, hipStream_t s);
// pair counts and bytes of the pair blocks (pf_jobs_stats)
hipError_t launch_pair_stats(const DevStore& st, const PairBlock* blocks, int nblocks, const int32_t* slots,
                             unsigned long long* acc, hipStream_t s);
hipError_t launch_job_topk(const DevJob* jobs, const int32_t* jix, int njobs, const float* score, const int32_t* ids,
                           const int32_t* slots, const int32_t* ncand, uint64_t* out, int k, hipStream_t s);

}  // namespace pf
