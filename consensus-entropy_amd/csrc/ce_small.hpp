// ce_small.hpp -- pools of a few thousand items (BASELINE configs[0..2]: one
// reference-sized pool, the hc table, the [mc; hc] mix, 500 users in one
// launch), each problem (the pool, a user, the mix) selected by ONE block:
//
// Per block (amg_test.py:441-445 on the problem's items):
//   1. the log table's loads are issued, then the member loads of the
//      thread's item slots (item lo + tid + BS*v: each wave's loads coalesced);
//      each item's mean + entropy runs as soon as its own loads have landed;
//   2. the best key of each group of BS/64 lanes (lane-exchange butterfly) ->
//      64 group bests (distinct items) in LDS; every thread ranks one of them
//      against a 1/W slice of the others; the group best of rank q-1 is an
//      exact floor (q items are >= it);
//   3. items >= the floor are appended to an LDS list (one atomic per wave);
//      survivor t counts the survivors that beat it and writes itself to
//      output slot `rank` (< q).
// A problem longer than BS*IPT items (a long user of a ragged batch), or more
// than 64*W survivors (floods of exact ties at the floor), takes per-wave
// register lists + a tree merge instead (block-uniform branches, same answer).
#pragma once
#include "ce_stream.hpp"

namespace ce {

#ifdef CE_PHASE_TIMING
// diagnostic build only (-DCE_PHASE_TIMING): per-block wall-clock stamps (100 MHz)
// [0] start, [1] wave 0's keys done, [2] floor, [3] append, [4] rank, [5] merge,
// [6 + w] wave w's keys done (w < 8)
__device__ uint64_t g_phase[8192][16];
#define CE_STAMP(b, k) \
    if (threadIdx.x == 0 && (b) < 8192) g_phase[b][k] = wall_clock64();
#define CE_WSTAMP(b) \
    if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) < 8 && (b) < 8192) g_phase[b][6 + (threadIdx.x >> 6)] = wall_clock64();
#else
#define CE_STAMP(b, k)
#define CE_WSTAMP(b)
#endif

// Geometry: block p selects problem p -- segment A (committee items: one
// pool [0, n) or user p's [offsets[p], offsets[p+1])) and, for the mix,
// segment B (the hc rows [0, nB), positions n + row).
struct TileArgs {
    const int64_t* offsets;  // [P+1] problem offsets (batched users), or nullptr: one problem
    int64_t n;               // segment-A items (offsets == nullptr)
    int64_t nB;              // segment-B rows (mix), 0 otherwise
    int64_t base_idx;        // position of item 0 (offsets == nullptr)
};

template <int WAVES>
struct TileSmem {
    static constexpr int CAP = 64 * WAVES;  // one survivor per thread
    uint64_t gk[64];                        // group bests
    int64_t gi[64];
    int part[WAVES][64];                    // partial ranks of the group bests
    int cnt;                                // survivors appended
    uint64_t ck[CAP];
    int64_t ci[CAP];
    WaveListsT<WAVES> lists;                // fallback tree merge
};

// Keys of this thread's IPT items lo + tid + BS*v of [lo, hi) into slots
// [OFF, OFF + IPT) (all loads in flight before the arithmetic; COMMIT: `tab`
// is committed once the data is awaited -- exactly one tile_keys call of a
// block commits).  Slots outside [OFF, OFF + IPT) are left as they are.
template <class Src, int IPT, int UNR, int BS, int K, int OFF, bool COMMIT>
__device__ __forceinline__ void tile_keys(const Src& src, int64_t lo, int64_t hi, int64_t rel, const uint32_t* excl,
                                          LogTablePrefetch& tab, uint64_t (&k)[K], int64_t (&pos)[K],
                                          bool (&ok)[K]) {
    static_assert(OFF + IPT <= K, "");
    const int tid = threadIdx.x, w = tid >> 6;
    const int64_t len = hi - lo;
    int64_t items[IPT];
    uint64_t kk[IPT];
    int nlive = 0;  // this wave's item slots holding at least one real item (a prefix)
#pragma unroll
    for (int v = 0; v < IPT; ++v) {
        const int64_t j = tid + (int64_t)BS * v;
        items[v] = lo + (j < len ? j : (len > 0 ? len - 1 : 0));
        kk[v] = 0;
        nlive += (int64_t)BS * v + 64 * w < len;
        pos[OFF + v] = items[v] + rel;
        ok[OFF + v] = j < len;
        if (excl) ok[OFF + v] = ok[OFF + v] && !excluded(excl, items[v]);
    }
    if (len > 0) {  // block-uniform
        if constexpr (COMMIT) src.template keys_small<UNR, IPT>(items, kk, nlive, [&]() { tab.commit(); });
        else src.template keys_small<UNR, IPT>(items, kk, nlive);
    } else if constexpr (COMMIT) {
        tab.commit();
    }
#pragma unroll
    for (int v = 0; v < IPT; ++v) k[OFF + v] = kk[v];
}

// LONG: a problem may exceed BS * IPT items (the per-wave streaming path is
// compiled in).  Launches whose host checks bound the problem (one pool, the
// mix) drop it -- half the code of the kernel.
template <class SrcA, class SrcB, int IPTA, int IPTB, int UNRA, int UNRB, int BS, bool LONG = true>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4))) void k_select_tiles(
    SrcA srcA, SrcB srcB, TileArgs ta, int q, double* __restrict__ oval, int64_t* __restrict__ oidx,
    const uint32_t* __restrict__ excl) {
    constexpr int W = BS / 64, GS = BS / 64;  // waves; lanes per group (64 groups)
    constexpr int K = IPTA + IPTB;  // slots: segment A's, then segment B's (both segments in one block)
    static_assert(BS % 64 == 0 && BS >= 128 && GS <= 16 && (GS & (GS - 1)) == 0, "block size");
    using SM = TileSmem<W>;
    __shared__ SM sm;
    CE_STAMP(blockIdx.x, 0)
    LogTablePrefetch tab;
    tab.fetch();
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int p = blockIdx.x;
    const int64_t lo = ta.offsets ? ta.offsets[p] : 0, hi0 = ta.offsets ? ta.offsets[p + 1] : ta.n;
    const int64_t hi = hi0 > lo ? hi0 : lo;
    const int64_t rel = (ta.offsets ? 0 : ta.base_idx) - lo;  // A: position = item + rel
    const int64_t relB = ta.n + ta.base_idx;                  // B: position = row + relB
    // the mix: the block takes every committee item AND every hc row (slots [0, IPTA) and [IPTA, K))
    const bool both = IPTB > 0 && ta.nB > 0;
    double* ov = oval + (int64_t)p * q;
    int64_t* oi = oidx + (int64_t)p * q;
    CE_DASSERT(q >= 1 && q <= 64);

    const bool long_tile = both ? (hi - lo > (int64_t)BS * IPTA || ta.nB > (int64_t)BS * IPTB)
                                : hi - lo > (int64_t)BS * IPTA;
    CE_DASSERT(LONG || !long_tile);
    if (LONG && long_tile) {  // block-uniform: per-wave streams + tree merge
        tab.commit();
        constexpr int64_t kIt = 64 * 2;
        RegTopQ tq;
        tq.init(q);
        auto wave_part = [&](int64_t a0, int64_t a1, int64_t& wlo, int64_t& whi) {
            const int64_t its = (a1 - a0 + kIt - 1) / kIt, its_w = (its + W - 1) / W;
            wlo = a0 + (int64_t)w * its_w * kIt;
            whi = wlo + its_w * kIt < a1 ? wlo + its_w * kIt : a1;
            if (wlo > whi) wlo = whi;
        };
        int64_t wlo, whi;
        wave_part(lo, hi, wlo, whi);
        stream_direct_range<SrcA, 2, UNRA>(srcA, wlo, whi, rel, q, tq, excl);
        if (both) {
            wave_part(0, ta.nB, wlo, whi);
            if constexpr (IPTB > 0) stream_direct_range<SrcB, 2, UNRB>(srcB, wlo, whi, relB, q, tq, nullptr);
        }
        block_merge_write<W>(tq, sm.lists, q, nullptr, 0, ov, oi);
        return;
    } else {
        // 1. keys of this thread's items
        uint64_t k[K];
        int64_t pos[K];
        bool ok[K];
#pragma unroll
        for (int v = 0; v < K; ++v) {
            k[v] = 0;
            pos[v] = INT64_MAX;
            ok[v] = false;
        }
        tile_keys<SrcA, IPTA, UNRA, BS, K, 0, true>(srcA, lo, hi, rel, excl, tab, k, pos, ok);
        if constexpr (IPTB > 0)
            if (both) tile_keys<SrcB, IPTB, UNRB, BS, K, IPTA, false>(srcB, 0, ta.nB, relB, nullptr, tab, k, pos, ok);
        CE_STAMP(blockIdx.x, 1)
        CE_WSTAMP(blockIdx.x)
        uint64_t bk = 0;
        int64_t bi = INT64_MAX;
#pragma unroll
        for (int v = 0; v < K; ++v)
            if (ok[v] && better(k[v], pos[v], bk, bi)) {
                bk = k[v];
                bi = pos[v];
            }
        // 2. floor = the group best of rank q-1 (ranks split over the waves)
        group_best<GS>(bk, bi);
        if ((tid & (GS - 1)) == 0) {
            sm.gk[tid / GS] = bk;
            sm.gi[tid / GS] = bi;
        }
        if (tid == 0) sm.cnt = 0;
        __syncthreads();
        {
            const uint64_t mk = sm.gk[lane];
            const int64_t mi = sm.gi[lane];
            int r = 0;
#pragma unroll
            for (int j = 0; j < 64 / W; ++j) {
                const int o = w * (64 / W) + j;
                r += better(sm.gk[o], sm.gi[o], mk, mi);
            }
            sm.part[w][lane] = r;
        }
        __syncthreads();
        uint64_t fk = 0;  // no group best of rank q-1 (fewer valid groups): admit every valid item
        int64_t fi = INT64_MAX;
        {
            int r = 0;
#pragma unroll
            for (int j = 0; j < W; ++j) r += sm.part[j][lane];
            const uint64_t hit = __ballot(r == q - 1);
            if (hit) {
                const int sl = __builtin_ctzll(hit);
                fk = sm.gk[sl];
                fi = sm.gi[sl];
            }
        }
        CE_STAMP(blockIdx.x, 2)
        // 3. survivors (not worse than the floor) -> LDS list: the wave's K
        //    ballots first, then ONE atomic per wave for all of its survivors
        //    (each returning LDS atomic is a ~100-cycle round trip)
        {
            bool pass[K];
            uint64_t m[K];
            int tot = 0;
#pragma unroll
            for (int v = 0; v < K; ++v) {
                pass[v] = ok[v] && !better(fk, fi, k[v], pos[v]);
                m[v] = __ballot(pass[v]);
                tot += __popcll(m[v]);
            }
            if (tot) {  // wave-uniform
                int base = 0;
                if (lane == 0) base = atomicAdd(&sm.cnt, tot);
                base = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
                for (int v = 0; v < K; ++v) {
                    const int slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m[v] >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m[v], 0));
                    if (pass[v] && slot < SM::CAP) {
                        sm.ck[slot] = k[v];
                        sm.ci[slot] = pos[v];
                    }
                    base += __popcll(m[v]);
                }
            }
        }
        __syncthreads();
        CE_STAMP(blockIdx.x, 3)
        const int nc = sm.cnt;
        if (nc <= SM::CAP) {
            if (tid < nc) {  // survivor tid takes the slot of its rank
                const uint64_t mk = sm.ck[tid];
                const int64_t mi = sm.ci[tid];
                int r = 0;
                // (batching 8 LDS reads per step measured slower: rank 0.64 -> 0.80 us)
                for (int j = 0; j < nc; ++j) r += better(sm.ck[j], sm.ci[j], mk, mi);
                if (r < q) {
                    ov[r] = key_to_val(mk);
                    oi[r] = mi;
                }
            } else if (tid < q) {  // fewer survivors than q: padding
                ov[tid] = __longlong_as_double(0x7ff8000000000000ll);
                oi[tid] = -1;
            }
            CE_STAMP(blockIdx.x, 4)
        } else {
            // overflow (> CAP items tie at or above the floor): per-wave lists + tree merge
            RegTopQ tq;
            tq.init(q, fk, fi == INT64_MAX ? fi : fi + 1);  // admit candidates >= the floor
#pragma unroll
            for (int v = 0; v < K; ++v) tq.offer(k[v], pos[v], ok[v]);
            block_merge_write<W>(tq, sm.lists, q, nullptr, 0, ov, oi);
        }
    }
}

}  // namespace ce
