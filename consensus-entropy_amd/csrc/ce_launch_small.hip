// ce_launch_small.hip -- pools small enough for one block each: a single
// pool, batched users (one block per user), the two-segment mix, and the
// multi-block k_stream_seg path.  The only TU that instantiates
// k_select_small / k_stream_seg.
#include "ce_host.hpp"

using namespace ce;

// Single-block pools (k_select_small): IPT items per thread (2 for C = 8
// rows), UNR member loads per item in flight (f64 / C = 8 rows are twice as
// wide: 2).  Returns false (nothing launched) when the pool exceeds BS * IPT.
template <class Src>
constexpr int small_ipt() { return Src::kC > 4 ? 2 : 4; }
template <class Src, int BS>
static void launch_small(const Src& src, int grid, const int64_t* offsets, int64_t n, int64_t base_idx, int q,
                         double* oval, int64_t* oidx, const uint32_t* excl, hipStream_t st) {
    constexpr int UNR = (Src::kDT == kF64 || Src::kC > 4 || BS > kSmallBS) ? 2 : 4;
    hipLaunchKernelGGL((k_select_small<Src, Src, small_ipt<Src>(), 0, UNR, 1, BS>), dim3((unsigned)grid), dim3(BS), 0,
                       st, src, src, offsets, n, (int64_t)0, base_idx, q, oval, oidx, excl);
}
// mix in one block: committee items (A) then the hc table rows (B, a 1-member
// f64 committee); IPT 2 per segment at 1024 threads: up to 2048 + 2048 rows
template <class SrcA, class SrcB>
static void launch_small_mix_t(const SrcA& a, const SrcB& b, int64_t n, int64_t nB, int q, double* oval,
                             int64_t* oidx, hipStream_t st) {
    constexpr int UNRA = (SrcA::kDT == kF64 || SrcA::kC > 4) ? 2 : 4;
    hipLaunchKernelGGL((k_select_small<SrcA, SrcB, 2, 2, UNRA, 1, kSmallBSWide>), dim3(1), dim3(kSmallBSWide), 0, st, a,
                       b, (const int64_t*)nullptr, n, nB, (int64_t)0, q, oval, oidx, (const uint32_t*)nullptr);
}

// The same for k_stream_seg: up to 16-wave blocks (<= 128 VGPRs), so fewer loads per lane.
template <class Src, class F>
static inline void with_seg_batching(F&& f) {
    if constexpr (Src::kC > 4) f(std::integral_constant<int, 4>(), std::integral_constant<int, 1>());
    else f(std::integral_constant<int, 4>(), std::integral_constant<int, 2>());
}

bool launch_small_pool(const CommArgs& a, int64_t base_idx, int q, double* oval, int64_t* oidx, const uint32_t* excl,
                       hipStream_t st) {
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        if (a.N <= (int64_t)kSmallBS * small_ipt<S>()) {
            launch_small<S, kSmallBS>(src, 1, nullptr, a.N, base_idx, q, oval, oidx, excl, st);
            launched = true;
        } else if (a.N <= (int64_t)kSmallBSWide * small_ipt<S>()) {
            launch_small<S, kSmallBSWide>(src, 1, nullptr, a.N, base_idx, q, oval, oidx, excl, st);
            launched = true;
        }
    });
    return rc == CE_OK && launched;
}

bool launch_small_users(const CommArgs& a, const int64_t* offsets, int U, int q, double* oval, int64_t* oidx,
                        hipStream_t st) {
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        if (cdiv(a.N, U) <= (int64_t)kSmallBS * small_ipt<S>()) {
            launch_small<S, kSmallBS>(src, U, offsets, 0, 0, q, oval, oidx, nullptr, st);
            launched = true;
        }
    });
    return rc == CE_OK && launched;
}

bool launch_small_mix(const CommArgs& a, const CommArgs& t, int q, double* oval, int64_t* oidx, hipStream_t st) {
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        if constexpr (S::kC == 4 || S::kC == 8) {
            constexpr int CC = S::kC;
            if (vec_ok(t, CC))
                launch_small_mix_t(src, make_src<kF64, CC, true>(t), a.N, t.N, q, oval, oidx, st);
            else
                launch_small_mix_t(src, make_src<kF64, CC, false>(t), a.N, t.N, q, oval, oidx, st);
            launched = true;
        }
    });
    return rc == CE_OK && launched;
}

bool launch_seg(const CommArgs& a, const int64_t* offsets, int64_t n, int64_t base_idx, int q, int nblocks, int bpu,
                int threads, double* oval, int64_t* oidx, Cand* wc, const uint32_t* excl, hipStream_t st) {
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        with_seg_batching<S>([&](auto unr, auto ipl) {
            hipLaunchKernelGGL((k_stream_seg<S, decltype(ipl)::value, decltype(unr)::value, kSegWaves>),
                               dim3((unsigned)nblocks), dim3(threads), 0, st, src, offsets, n, base_idx, q, bpu, oval,
                               oidx, wc, excl);
        });
    });
    return rc == CE_OK;
}
