// ce_launch_small.hip -- pools of a few thousand items: a single pool,
// batched users, the two-segment mix (tiled, ce_small.hpp), and the
// multi-block k_stream_seg path.  The only TU that instantiates
// k_select_tiles / k_stream_seg.
#include "ce_host.hpp"

using namespace ce;

// Tiled small pools (k_select_tiles, ce_small.hpp).  IPT items per thread
// (2 for C = 8 rows), so a tile holds up to kTileBS * IPT items; UNR member
// loads per item in flight (f64 / C = 8 rows are twice as wide: 2).
template <class Src>
constexpr int small_ipt() { return Src::kC > 4 ? 2 : 4; }
template <class Src>
constexpr int small_unr() { return (Src::kDT == kF64 || Src::kC > 4) ? 2 : 4; }

// Tile-size targets (items per tile).  A/B knobs: CE_AMD_TILE_POOL (one pool,
// the hc table), CE_AMD_TILE_USER (batched users), CE_AMD_TILE_MIX (each mix
// segment).
static int64_t tile_target(const char* env, int64_t dflt) {
    const char* e = getenv(env);
    const long v = e ? atol(e) : 0;
    return v > 0 ? (int64_t)v : dflt;
}
static int64_t target_pool() {
    static const int64_t v = tile_target("CE_AMD_TILE_POOL", 256);
    return v;
}
static int64_t target_user() {
    static const int64_t v = tile_target("CE_AMD_TILE_USER", 1024);
    return v;
}
static int64_t target_mix() {
    static const int64_t v = tile_target("CE_AMD_TILE_MIX", 256);
    return v;
}

// tiles for `len` items at <= `target` per tile, within the merge's capacity
static int tiles_for(int64_t len, int64_t target, int q, int smax) {
    int64_t s = cdiv(len < 1 ? 1 : len, target);
    const int64_t cap = std::min<int64_t>(smax, kTileMergeCap / q);
    if (s > cap) s = cap;
    return (int)(s < 1 ? 1 : s);
}

template <class SrcA, class SrcB, int IPTA, int IPTB>
static void launch_tiles(const SrcA& a, const SrcB& b, const TileArgs& ta, int problems, int q, double* oval,
                         int64_t* oidx, const uint32_t* excl, hipStream_t st) {
    hipLaunchKernelGGL((k_select_tiles<SrcA, SrcB, IPTA, IPTB, small_unr<SrcA>(), 1, kTileBS>),
                       dim3((unsigned)(problems * (ta.SA + ta.SB))), dim3(kTileBS), 0, st, a, b, ta, q, oval, oidx,
                       excl);
}

bool launch_small_pool(const CommArgs& a, int64_t base_idx, int q, double* oval, int64_t* oidx, const uint32_t* excl,
                       WsLists w, hipStream_t st) {
    if (a.N < 1 || a.N > kSmallPoolItems) return false;
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        const int SA = tiles_for(a.N, target_pool(), q, 16);
        if (cdiv(a.N, SA) > (int64_t)kTileBS * small_ipt<S>()) return;  // tiles would be long: not this path
        const TileArgs ta{nullptr, a.N, 0, base_idx, SA, 0, w.c, w.ctr};
        launch_tiles<S, S, small_ipt<S>(), 0>(src, src, ta, 1, q, oval, oidx, excl, st);
        launched = true;
    });
    return rc == CE_OK && launched;
}

int small_users_tiles(int64_t total_items, int U, int q) {
    if (U < 1) U = 1;
    if (q < 1) q = 1;
    return tiles_for(cdiv(total_items, U), target_user(), q, 16);
}

bool launch_small_users(const CommArgs& a, const int64_t* offsets, int U, int q, double* oval, int64_t* oidx,
                        WsLists w, hipStream_t st) {
    if (U < 1 || U > kWsCounters) return false;
    const int SA = small_users_tiles(a.N, U, q);
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        // the average user must fit its tiles (a longer one streams inside its tile)
        if (cdiv(cdiv(a.N, U), SA) > (int64_t)kTileBS * small_ipt<S>()) return;
        const TileArgs ta{offsets, 0, 0, 0, SA, 0, w.c, w.ctr};
        launch_tiles<S, S, small_ipt<S>(), 0>(src, src, ta, U, q, oval, oidx, nullptr, st);
        launched = true;
    });
    return rc == CE_OK && launched;
}

// mix: committee items (segment A) then the hc table rows (segment B, a
// 1-member f64 committee), 2 items per thread per segment
bool launch_small_mix(const CommArgs& a, const CommArgs& t, int q, double* oval, int64_t* oidx, WsLists w,
                      hipStream_t st) {
    if (a.N < 1 || t.N < 1) return false;
    const int SA = tiles_for(a.N, target_mix(), q, 8), SB = tiles_for(t.N, target_mix(), q, 8);
    if (cdiv(a.N, SA) > 2 * kTileBS || cdiv(t.N, SB) > 2 * kTileBS || (SA + SB) * q > kTileMergeCap) return false;
    const TileArgs ta{nullptr, a.N, t.N, 0, SA, SB, w.c, w.ctr};
    bool launched = false;
    const int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        if constexpr (S::kC == 4 || S::kC == 8) {
            constexpr int CC = S::kC;
            if (vec_ok(t, CC))
                launch_tiles<S, CommitteeSrc<kF64, CC, true>, 2, 2>(src, make_src<kF64, CC, true>(t), ta, 1, q, oval,
                                                                     oidx, nullptr, st);
            else
                launch_tiles<S, CommitteeSrc<kF64, CC, false>, 2, 2>(src, make_src<kF64, CC, false>(t), ta, 1, q,
                                                                      oval, oidx, nullptr, st);
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
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), (size_t)n * 6 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif
