// ce_launch_small.hip -- pools of a few thousand items: a single pool,
// batched users, the two-segment mix (tiled, ce_small.hpp), and the
// multi-block k_stream_seg path.  The only TU that instantiates
// k_select_tiles / k_stream_seg.
#include "ce_host.hpp"

using namespace ce;

// Small pools (k_select_tiles, ce_small.hpp).  IPT items per thread (2 for
// C = 8 rows), so a tile holds up to BS * IPT items; UNR member loads per item
// in flight (f64 / C = 8 rows, and 16-wave blocks, take 2).
template <class Src>
constexpr int small_ipt() { return Src::kC > 4 ? 2 : 4; }
// (f64 C = 4 rows take 4 too since the slot throttle: one item slot of M <= 4
// members in flight per lane, so keys_small's progressive path runs for the
// reference's 4-member f64 committee, configs[0])
template <class Src, int BS>
constexpr int small_unr() { return (Src::kC > 4 || BS > 512) ? 2 : 4; }

// ONE block per problem (the whole pool / user / mix selected by one block,
// no hand-off).  Measured on MI355X (profiles/r03_small.json): splitting a
// problem over several blocks with an arrival-ticket merge of their lists was
// slower at the reference's sizes -- the hand-off (write-through lists, one
// agent-scope atomic, sc1 reads by the last block) costs more than spreading
// 1608 items over more CUs saves (C1 9.4 -> 11.1-13.0 us, C3 15.7 -> 19.0 us).
// LONG: a problem may exceed BS * IPT items (the per-wave streaming path is compiled in)
template <class SrcA, class SrcB, int IPTA, int IPTB, int BS, int UNRA, bool LONG>
static void launch_tiles(const SrcA& a, const SrcB& b, const TileArgs& ta, int problems, int q, double* oval,
                         int64_t* oidx, const uint32_t* excl, hipStream_t st) {
    note_kernel("ce::k_select_tiles<ce::CommitteeSrc<%d, %d, %s>, ce::CommitteeSrc<%d, %d, %s>, %d, %d, %d, 1, %d, %s>",
                SrcA::kDT, SrcA::kC, SrcA::kVec ? "true" : "false", SrcB::kDT, SrcB::kC, SrcB::kVec ? "true" : "false",
                IPTA, IPTB, UNRA, BS, LONG ? "true" : "false");
    hipLaunchKernelGGL((k_select_tiles<SrcA, SrcB, IPTA, IPTB, UNRA, 1, BS, LONG>), dim3((unsigned)problems), dim3(BS),
                       0, st, a, b, ta, q, oval, oidx, excl);
}

bool launch_small_pool(const CommArgs& a, int64_t base_idx, int q, double* oval, int64_t* oidx, const uint32_t* excl,
                       WsLists w, hipStream_t st) {
    (void)w;
    if (a.N < 1 || a.N > kSmallPoolItems) return false;
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        constexpr int IPT = small_ipt<S>();
        const TileArgs ta{nullptr, a.N, 0, base_idx};
        if (a.N <= 512 * IPT) {  // one block; the pool fits it: no long path
            if constexpr (S::kDT == kF64 && S::kC == 4) {
                // one-member f64 tables (the hc select, amg_test.py:451-452): one load per
                // item slot, not UNR copies of member 0 (measured 8.0 -> 7.3 us)
                if (a.M == 1) {
                    launch_tiles<S, S, IPT, 0, 512, 1, false>(src, src, ta, 1, q, oval, oidx, excl, st);
                    launched = true;
                    return;
                }
            }
            launch_tiles<S, S, IPT, 0, 512, small_unr<S, 512>(), false>(src, src, ta, 1, q, oval, oidx, excl, st);
        } else if (a.N <= 1024 * IPT) {
            launch_tiles<S, S, IPT, 0, 1024, small_unr<S, 1024>(), false>(src, src, ta, 1, q, oval, oidx, excl, st);
        } else {
            return;
        }
        launched = true;
    });
    return rc == CE_OK && launched;
}

bool launch_small_users(const CommArgs& a, const int64_t* offsets, int U, int q, double* oval, int64_t* oidx,
                        hipStream_t st) {
    if (U < 1) return false;
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        constexpr int IPT = small_ipt<S>();
        // one 512-thread block per user: 2 per CU, all 500 users of configs[2] resident;
        // the average user must fit its block (a longer one streams inside it)
        if (cdiv(a.N, U) > (int64_t)512 * IPT) return;
        const TileArgs ta{offsets, 0, 0, 0};
        launch_tiles<S, S, IPT, 0, 512, small_unr<S, 512>(), true>(src, src, ta, U, q, oval, oidx, nullptr, st);
        launched = true;
    });
    return rc == CE_OK && launched;
}

// mix: committee items (segment A) then the hc table rows (segment B, a
// 1-member f64 committee), 2 items per thread per segment, in one 1024-thread
// block (up to 2048 + 2048 rows)
bool launch_small_mix(const CommArgs& a, const CommArgs& t, int q, double* oval, int64_t* oidx, hipStream_t st) {
    if (a.N < 1 || t.N < 1) return false;
    if (a.N > 2 * 1024 || t.N > 2 * 1024) return false;
    const TileArgs ta{nullptr, a.N, t.N, 0};
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        if constexpr (S::kC == 4) {  // the reference's 4 quadrants (other C: the streaming engine + merge)
            constexpr int CC = S::kC;
            // committee loads: all of an item's members in one batch for f32 C = 4 (UNR 4), as round 2's
            // one-block mix (a 16-wave block with UNR 2 measured 12.2 vs 10.0 us at C2)
            constexpr int UNRA = (S::kDT == kF64 || S::kC > 4) ? 2 : 4;
            auto go = [&](auto hsrc) {
                using H = decltype(hsrc);
                launch_tiles<S, H, 2, 2, 1024, UNRA, false>(src, hsrc, ta, 1, q, oval, oidx, nullptr, st);
            };
            if (vec_ok(t, CC)) go(make_src<kF64, CC, true>(t));
            else go(make_src<kF64, CC, false>(t));
            launched = true;
        }
    });
    return rc == CE_OK && launched;
}

// The same for k_stream_seg: up to 16-wave blocks (<= 128 VGPRs), so fewer loads per lane.
template <class Src, class F>
static inline void with_seg_batching(F&& f) {
    if constexpr (Src::kC > 4) f(std::integral_constant<int, 4>(), std::integral_constant<int, 1>());
    else f(std::integral_constant<int, 4>(), std::integral_constant<int, 2>());
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

#ifdef CE_PHASE_TIMING
extern "C" int ce_debug_phase(uint64_t* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), (size_t)n * 16 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif
