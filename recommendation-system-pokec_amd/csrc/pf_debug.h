// pf_debug.h — the engine's only environment switch, PF_DEBUG: comma-separated name=value
// settings that force code paths the tests cover, or turn on profiling output.  Unset, the
// engine runs its fixed configuration (the measured winners); nothing on the
// product path reads any other variable.
//
//   scan=stream|postings  initial all-candidates scan kernel of every context (default: postings
//                         when the corpus fits its encoding; tests: test_kernel_variants)
//   stage_limit=BYTES     query tables above this are probed in global memory (default 49152)
//   tile_steps=N          tile-store chunk limit in 16-B steps, splits records over lanes (48)
//   k5_block=N            postings-scan block size in candidates (kBlockCands, 512; tests)
//   k5_transposed=1       batched postings scans on the query-fastest grid (A/B; measured slower)
//   k5_static=1           one-query postings scans with the static block hand-out (A/B)
//   k5_batch_blocks=N     blocks per workgroup of a batched postings scan (default 32; A/B)
//   k5_wgs=N              workgroups of a one-query postings scan (default: one resident round; on the
//                         scan lanes 7/8 of one with 3-5 lanes, 1/2 with 6-11, 3/16 with 12-15; A/B)
//   lazy_aux=1            create the job pipeline's aux streams at the first job call, not at open (A/B)
//   scan_lanes=N          single-query scans on a caller's stream: 0 or 1 launch on that stream (A/B);
//                         default 3 (the context's stream, aux, aux2), so consecutive queries' launches
//                         overlap; 2 leaves out aux2; 4..16 add lanes on streams of their own (for a
//                         process with more hardware queues, GPU_MAX_HW_QUEUES)
//   k5_dyn=0              K5: one-query launches in static block rounds, the tail claimed (A/B;
//                         default: every block claimed per XCD group)
//   chunk_pingpong=0      the job pipeline's chunks all gather on the aux stream and score on the
//                         context's stream behind an event (A/B; default: alternate the two)
//   collab_main=1         the job pipeline's K4' / K8 on the context's stream after the pair kernel
//                         also in chunks without clubs jobs (A/B)
//   k5_xcd=0|1            K5: contiguous block ranges per XCD in each static round (default 1; A/B)
//   k5_tail=N             K5: candidates per claimed block past a one-query launch's static rounds
//                         (default 0 = whole blocks; A/B)
//   k5_slice=1            K5s, the wave-private slice kernel: only in the variant build
//                         PATCH=tools/k5_exp/k5s_slice.patch tools/build_variant.sh k5s
//                         (A/B: bit-exact, slower)
//   k5s_static=1          K5s (variant build): static slice hand-out instead of claimed slices (A/B)
//   k5s_batch_slices=N    K5s (variant build): slices per wave of a batched launch (default 16; A/B)
//   chunk_plan=W1:W2:..   relative chunk sizes of large job-pipeline calls (default 1:1:1; A/B)
//   load_threads=N        loader threads (default: min(16, hardware threads))
//   resident_post=0       one-query all-candidates scans build and upload their K5 image per call
//                         instead of launching from the postings images built at open (A/B)
//   resident_images=0     the job pipeline builds its query images per call (K6) instead of
//                         referencing the ones built for every user at open
//   host_prof=1           host stage clocks on stderr (pf_open, the loaders, the job pipeline)
//
// e.g. PF_DEBUG=scan=stream,stage_limit=0
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace pf {

// The value of PF_DEBUG's `name` setting, or nullptr when absent (read at each call: the
// engine calls it at open / load time only).
inline const char* debug_str(const char* name) {
    const char* e = std::getenv("PF_DEBUG");
    const std::string all(e ? e : "");
    static thread_local std::string val;
    const size_t n = std::strlen(name);
    size_t p = 0;
    while (p < all.size()) {
        size_t q = all.find(',', p);
        if (q == std::string::npos) q = all.size();
        if (q - p > n && all.compare(p, n, name) == 0 && all[p + n] == '=') {
            val.assign(all, p + n + 1, q - p - n - 1);
            return val.c_str();
        }
        p = q + 1;
    }
    return nullptr;
}

// PF_DEBUG's `name` as an integer, dflt when absent.
inline long debug_long(const char* name, long dflt) {
    const char* v = debug_str(name);
    return v ? std::strtol(v, nullptr, 0) : dflt;
}

// Sub-stage clock of pf_open's builders: lap(what) prints the time since the last lap on stderr
// when PF_DEBUG host_prof is set.
struct StageClock {
    bool on = debug_long("host_prof", 0) != 0;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[pf_open]     %s %.3f s\n", what, std::chrono::duration<double>(n - t).count());
        t = n;
    }
};

}  // namespace pf
