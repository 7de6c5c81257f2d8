// ce_launch_stream.hip -- the streaming stage-1 launcher (the only TU that
// instantiates k_stream_nmc / k_stream_direct / k_stream_wide2 / k_stream_wide).
#include "ce_host.hpp"

using namespace ce;

// (UNR members x IPL items) loads in flight per lane for the direct paths:
// small committees batch items, large ones batch members.
template <class Src, class F>
static inline void with_batching(int M, F&& f) {
    if constexpr (Src::kDT == kF64 || Src::kC > 4) {
        (void)M;
        f(std::integral_constant<int, 4>(), std::integral_constant<int, 2>());
    } else {
        if (M <= 4) f(std::integral_constant<int, 4>(), std::integral_constant<int, 4>());
        else f(std::integral_constant<int, 8>(), std::integral_constant<int, 2>());
    }
}


static int launch_stream_impl(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
                              const uint32_t* excl, const FoldOut* fold);

// the LDS-DMA loads' cache-policy bits (2: non-temporal -- the pool is read once)
#ifndef CE_NMC_AUX
#define CE_NMC_AUX 2
#endif

// items (M x C x size bytes) from which the wide stream runs one block per CU
// with a deep register ring (below)
constexpr int64_t kWideHeavyBytes = 16384;

bool launch_stream(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
                   const uint32_t* excl) {
    return launch_stream_impl(a, G, q, base_idx, w, st, excl, nullptr) != 0;
}

int launch_stream_fold(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
                       const uint32_t* excl, FoldOut out) {
    return launch_stream_impl(a, G, q, base_idx, w, st, excl, &out);
}

static int launch_stream_impl(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
                              const uint32_t* excl, const FoldOut* fold) {
    note_kernel("%s", "");
    if (q > kStreamMaxQ || a.N == 0) return 0;
    StreamArgs sa = stream_args(a, G, base_idx);
    sa.excl = excl;
    if (fold) {  // kernels that fold read these; k_stream_wide (below) does not
        sa.ctr = w.ctr;
        sa.oval = fold->oval;
        sa.oidx = fold->oidx;
        sa.ocand = fold->ocand;
        sa.extra = fold->extra;
    }
    const int folded = fold ? 2 : 1;
    const int eb = elem_bytes(a.dt);
    const int64_t R = (int64_t)a.M * a.C * eb;
    const bool dense_nmc = a.sC == 1 && a.sM == a.C && a.sN == (int64_t)a.M * a.C && (uintptr_t)a.p % 16 == 0;
    if (dense_nmc && (R == 256 || R == 512)) {
#define CE_S(DT_, C_, S_)                                                                                   \
    if (a.dt == DT_ && a.C == C_ && R == 16 * S_) {                                                       \
        constexpr int RING_ = S_ == 16 ? 2 : 1; /* two 16-KiB tiles per wave: one block per CU */          \
        auto kern = k_stream_nmc<DT_, C_, S_, CE_NMC_AUX, false, RING_>;                                  \
        const int grid = resident_grid(kern, 0, G);                                                       \
        note_kernel("ce::k_stream_nmc<%d, %d, %d, %d, false, %d>", DT_, C_, S_, CE_NMC_AUX, RING_);        \
        stream_grid(sa, grid);                                                                            \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, sa, q, w.c);                               \
        return folded;                                                                                    \
    }
        CE_S(kF32, 4, 16) CE_S(kF32, 4, 32) CE_S(kBF16, 4, 16) CE_S(kBF16, 4, 32) CE_S(kF64, 4, 32)
        CE_S(kF32, 8, 16) CE_S(kF32, 8, 32)
#undef CE_S
    }
    // member-major stack (the reference's np.array(pred_prob) order) with
    // 16-B member rows: LDS-DMA tiles of one 1 KiB run per member
    const bool dense_mnc = a.sC == 1 && a.sN == a.C && a.C * eb == 16 && (a.sM * eb) % 16 == 0 &&
                           (uintptr_t)a.p % 16 == 0 && a.M >= 4;
    if (dense_mnc) {
#define CE_SM(DT_, C_, M_)                                                                              \
    if (a.dt == DT_ && a.C == C_ && a.M == M_) {                                                       \
        constexpr int RING_ = M_ == 16 ? 2 : 1; /* as measured: 16 members (16-KiB tiles) */          \
        auto kern = k_stream_nmc<DT_, C_, M_, 2, true, RING_>;                                         \
        const int grid = resident_grid(kern, 0, G);                                                    \
        note_kernel("ce::k_stream_nmc<%d, %d, %d, 2, true, %d>", DT_, C_, M_, RING_);                   \
        stream_grid(sa, grid);                                                                         \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, sa, q, w.c);                            \
        return folded;                                                                                 \
    }
        CE_SM(kF32, 4, 4) CE_SM(kF32, 4, 8) CE_SM(kF32, 4, 16) CE_SM(kF32, 4, 20) CE_SM(kF32, 4, 32)
        CE_SM(kF64, 2, 8) CE_SM(kF64, 2, 16) CE_SM(kBF16, 8, 16)
#undef CE_SM
    }
    int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        with_batching<S>(a.M, [&](auto unr, auto ipl) {
            auto kern = k_stream_direct<S, decltype(ipl)::value, decltype(unr)::value>;
            note_kernel("ce::k_stream_direct<ce::CommitteeSrc<%d, %d, %s>, %d, %d>", S::kDT, S::kC,
                        S::kVec ? "true" : "false", decltype(ipl)::value, decltype(unr)::value);
            const int grid = resident_grid(kern, 0, G);
            stream_grid(sa, grid);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, src, sa, q, w.c);
        });
    });
    if (rc == CE_OK) return folded;
    const WideArgs wa = wide_args(a);
    const PwPlan pl = pw_plan(a.C);
    const size_t lds = wide_lds_bytes(a.C);
    int rc_excl = CE_OK;
    bool wide_folded = fold != nullptr;
    rc = with_wide_v(a, [&](auto dt, auto npl, auto vec) {
        constexpr int DT = decltype(dt)::value, NPL = decltype(npl)::value;
        if constexpr (decltype(vec)::value) {
            constexpr int KCH = NPL / ChunkT<DT>::CPC > 0 ? NPL / ChunkT<DT>::CPC : 1;
            // member rows per batch: 4 / KCH (>= 1), or 1 when that does not divide M
            constexpr int UNR = KCH >= 4 ? 1 : 4 / KCH;
            const int unr = a.M % UNR == 0 ? UNR : 1;
            auto go = [&](auto kern, int nb, int per_cu, StreamArgs s) {
                note_kernel("ce::k_stream_wide2<%d, %d, %d, %d>", DT, KCH, unr, nb);
                const int grid = std::min(resident_grid(kern, lds, G), per_cu * device_cus());
                stream_grid(s, grid);
                hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, wa, pl, s, q, w.c);
            };
            // A chunked job's chunks after the first (a running list seeds the
            // prefilter's floor, so nearly every item skips its exact entropy)
            // with heavy items (>= 16 KiB; the C5 config: 64 KB) run ONE block (4
            // waves) per CU, each wave with an 8-batch register ring -- 7 batches
            // (28 KB at C5) in flight.  Fewer concurrent item streams with more
            // bytes each read HBM better: on the full C5 job 0.861 of HBM vs 0.833
            // for the occupancy grid's 3 blocks with a 2-batch ring, and the spread
            // 0.005 vs 0.044 (profiles/r05_c5_grid_ab.json: 2 blocks per CU 0.820,
            // 1 block with a 2-batch ring 0.741, deeper rings at 2 per CU
            // 0.813-0.817, a 12-batch ring spills).  Only 4 waves per CU cannot
            // hide exact entropies, though: with every item exact (the build
            // without the prefilter) the same grid reads 0.56 against 0.78, so it
            // runs only where a floor makes nearly every item skip: the floor is
            // sampled from the pool itself (and a chunked job's running list),
            // and the grid vote sends the launch to the occupancy grid when more
            // than 1/16 of the samples would still be exact -- a chunk order of
            // rising entropies read 0.51 on the deep grid against 0.79-0.82 on the
            // occupancy grid (profiles/r06_c5_vote.json).  A wave PAIR per item
            // on the deep grid (two waves per SIMD, each half the classes) was
            // measured and dropped: 0.61 on that pool, 0.77-0.79 where the deep
            // grid reads 0.86-0.89 (the same file).
            // heavy items in a launch that folds its lists (single selections, the
            // multi-GPU records, every chunk of a job): the sampled floor + grid
            // vote (k_wide_seed / k_wide_seed_pick, ce_kernels.hpp), then both grids
            bool voted = false;
            if constexpr (KCH <= 2)  // (wider lanes: 8 batches would spill)
                voted = R >= kWideHeavyBytes && fold != nullptr && fold->wide_ws != nullptr &&
                        a.N >= kWideSeedMinItems && CE_WIDE_PREFILTER;
            if (voted) {
                if constexpr (KCH <= 2) {
                    const WideSeedWs sw = wide_seed_carve(fold->wide_ws);
                    const int ns = (int)wide_nsamples(a.N);
                    auto sk = unr == UNR ? k_wide_seed<DT, KCH, UNR> : k_wide_seed<DT, KCH, 1>;
                    hipLaunchKernelGGL(sk, dim3((unsigned)cdiv(ns, 4)), dim3(256), lds, st, wa, pl, sa.base_idx, sa.excl,
                                       sw.samp, sw.sapx);
                    hipLaunchKernelGGL(k_wide_seed_pick<kWideVoteSamples>, dim3(1), dim3(1024), 0, st, sw.samp, sw.sapx, ns, q,
                                       fold->extra, sw.seed, sw.vote);
                    StreamArgs sh = sa, so = sa;
                    sh.vote = so.vote = sw.vote;
                    sh.seed = so.seed = sw.seed;
                    sh.vote_heavy = 1;
                    so.vote_heavy = 0;
                    if (unr == UNR) {
                        go(k_stream_wide2<DT, KCH, UNR, 8>, 8, 1, sh);
                        go(k_stream_wide2<DT, KCH, UNR, 2>, 2, 1 << 20, so);
                    } else {
                        go(k_stream_wide2<DT, KCH, 1, 8>, 8, 1, sh);
                        go(k_stream_wide2<DT, KCH, 1, 2>, 2, 1 << 20, so);
                    }
                    note_kernel("ce::k_stream_wide2<%d, %d, %d, 8>|ce::k_stream_wide2<%d, %d, %d, 2>", DT, KCH, unr,
                                DT, KCH, unr);
                }
            } else {
                // a 2-batch register ring at the occupancy grid (3 and 4 measured:
                // 72.8 / 71.9 % vs 72.6 % at C5 in round 2)
                if (unr == UNR) go(k_stream_wide2<DT, KCH, UNR, 2>, 2, 1 << 20, sa);
                else go(k_stream_wide2<DT, KCH, 1, 2>, 2, 1 << 20, sa);
            }
        } else {  // strided / unaligned rows: the unpipelined wave-per-item kernel
            if (sa.excl) {  // k_stream_wide takes no bitmap
                rc_excl = CE_EUNSUPPORTED;
                return;
            }
            sa.ctr = nullptr;  // ... and does not fold
            wide_folded = false;
            auto kern = k_stream_wide<DT, NPL, false>;
            note_kernel("ce::k_stream_wide<%d, %d, false>", DT, NPL);
            const int grid = resident_grid(kern, lds, G);
            stream_grid(sa, grid);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, wa, pl, sa, q, w.c);
        }
    });
    if (rc != CE_OK || rc_excl != CE_OK) return 0;
    return wide_folded ? 2 : 1;
}
