// pf_kernels.h — host-callable launchers of the gfx950 kernels (pf_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "pf_types.h"

namespace pf {

// One block of the pair kernel, kPairThreads threads, one pair each: FAS(image qimg,
// slots[begin + i]) -> out[out + i] for i < count <= kPairThreads; a slot < 0 is skipped (its
// output is not written).  512: one staged image serves eight waves, and two workgroups per CU
// hold 16 waves where 256-thread ones held 12 (their LDS, mostly the per-lane hit lists).
constexpr int kPairThreads = 512;
struct PairBlock {
    int32_t qimg, begin, count, out;
};

// A run of pair blocks, expanded on the device (pf_jobs.hip expand_pairs_kernel): block
// first + x * nf + f (chunk x < nch, entry f < nf) scores image pool[fl + f].x against candidates
// [cand + x * kPairThreads, + min(kPairThreads, cap - x * kPairThreads)) into out + pool[fl + f].y * stride
// + x * kPairThreads (chunk-major: one candidate chunk's friends consecutive, sharing its records
// in cache)
struct PairGen {
    int32_t nf, nch, cap, cand, fl, stride, out, first;
};


// lds: dynamic LDS bytes per block = max over the batch of
//   sizeof(QConst) + staged keys/vals + n_hits_max * threads + 2048
// gtab: at least one image of the batch probes its table in global memory (lds_bytes == 0);
// the whole launch then uses the global-table variant.
hipError_t launch_scan(const DevStore& st, const uint8_t* pool, const QImageRef* refs_dev, uint32_t lds, bool gtab,
                       int nq, int tile_begin, int tile_end, int k, int blocks, uint64_t* parts, ScanSync* sync,
                       uint64_t* out, const int32_t* out_rows, hipStream_t s);
// resident scan blocks per CU at this dynamic LDS size (HIP occupancy API)
int scan_blocks_per_cu(bool packed, bool gtab, uint32_t lds);
// K5 postings scan over candidate blocks [blk_begin, blk_end) for nq query images (byte
// offsets img_off[] into pool); var_lds = post_var_lds(max n_tok, max lists of an image)
uint32_t post_var_lds(int n_tok, int n_lists);
uint32_t post_lds(uint32_t var_lds);
// tail_bs: a one-query launch's claimed blocks past its static rounds take tail_bs candidates each.
// qconst: nullptr (each image starts with its QConst) or, for a one-query launch from the resident
// images, the user's QConst elsewhere (its K1' resident image); img = the resident part's start
// minus sizeof(QConst).  The launch leaves each query's ScanSync zeroed (post_tail).
hipError_t launch_post(const PostStore& ps, const uint8_t* pool, const uint32_t* img_off, uint32_t var_lds, int nq,
                       int blk_begin, int blk_end, int k, int blocks, uint64_t* parts, ScanSync* sync, uint64_t* out,
                       const int32_t* out_rows, uint32_t mode, uint32_t tail_bs, hipEvent_t e0, hipEvent_t e1,
                       hipStream_t s, const uint8_t* qconst = nullptr);
int post_blocks_per_cu(uint32_t var_lds);
// plain merge of key lists (cross-shard merge after the all-gather)
hipError_t launch_merge(const uint64_t* in, int nparts, int64_t part_stride, int64_t query_stride, int nq, int k,
                        uint64_t* out, hipStream_t s);
// order (nullable): the dispatch order, block blockIdx.x scores blocks[order[blockIdx.x]]
hipError_t launch_pairs(const DevStore& st, const uint8_t* pool, const QImageRef* refs_dev, uint32_t max_lds,
                        bool gtab, const PairBlock* blocks, int nblocks, const int32_t* order, const int32_t* slots,
                        float* out, hipStream_t s);

}  // namespace pf
