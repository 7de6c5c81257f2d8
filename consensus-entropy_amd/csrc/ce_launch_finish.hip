// ce_launch_finish.hip -- stage 2: merges of best-first candidate lists
// (blocks of a pool, ranks after the all-gather, chunks of a chunked job).
// The only TU that instantiates k_merge_reg / k_finish_heads / k_finish /
// k_merge_wave.
#include "ce_host.hpp"

using namespace ce;

// ocand != nullptr: write candidate records instead of (val, idx).
template <bool FROM_VALS>
static void launch_finish(ListSrc<FROM_VALS> src, int segments, int nl, int q, double* oval, int64_t* oidx,
                          hipStream_t st, Cand* ocand = nullptr) {
    const int64_t L = (int64_t)nl * q;
    if (q <= kStreamMaxQ) {  // (the LDS-buffer merges below measured slower for q <= 64)
        hipLaunchKernelGGL((k_merge_reg<FROM_VALS>), dim3(segments), dim3(1024), 0, st, src, nl, q, oval, oidx,
                           ocand);
        return;
    }
    if (q <= kHeadsMaxQ && L > 256) {
        hipLaunchKernelGGL((k_finish_heads<FROM_VALS, 10>), dim3(segments), dim3(kHeadsBS), 0, st, src, nl, q, oval,
                           oidx, ocand);
        return;
    }
    if (L <= 256 && q <= 128)
        hipLaunchKernelGGL((k_finish<FROM_VALS, 512, 256, 1>), dim3(segments), dim3(256), 0, st, src, nl, q, oval,
                           oidx, ocand);
    else if (L <= 4096 && q <= 512)
        hipLaunchKernelGGL((k_finish<FROM_VALS, 2048, 256, 16>), dim3(segments), dim3(256), 0, st, src, nl, q, oval,
                           oidx, ocand);
    else
        hipLaunchKernelGGL((k_finish<FROM_VALS, 4096, kFinBS, 16>), dim3(segments), dim3(kFinBS), 0, st, src, nl,
                           q, oval, oidx, ocand);
}

void launch_finish_lists(const Cand* c, int segments, int nl, int q, double* oval, int64_t* oidx, hipStream_t st,
                         Cand* ocand) {
    launch_finish(ListSrc<false>{c, nullptr, nullptr}, segments, nl, q, oval, oidx, st, ocand);
}

void launch_finish_vals(const double* vals, const int64_t* idx, int segments, int nl, int q, double* oval,
                        int64_t* oidx, hipStream_t st) {
    launch_finish(ListSrc<true>{nullptr, vals, idx}, segments, nl, q, oval, oidx, st, nullptr);
}

void launch_merge_wave(const Cand* c, int segs, int nl, int q, double* oval, int64_t* oidx, hipStream_t st) {
    hipLaunchKernelGGL((k_merge_wave<false>), dim3((segs + 3) / 4), dim3(256), 0, st,
                       ListSrc<false>{c, nullptr, nullptr}, segs, nl, q, oval, oidx);
}
