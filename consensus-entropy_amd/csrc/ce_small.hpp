// ce_small.hpp -- pools of a few thousand items (BASELINE configs[0..2]: one
// reference-sized pool, the hc table, the [mc; hc] mix, 500 users in one
// launch), each problem (the pool, a user, the mix) selected by ONE block:
//
// Per block (amg_test.py:441-445 on the problem's items):
//   1. the log table's loads are issued, then the member loads of the
//      thread's item slots (item lo + tid + BS*v: each wave's loads coalesced);
//      each item's mean + entropy runs as soon as its own loads have landed;
//   2. the max key of each group of BS/64 lanes (DPP mirrors) -> 64 group
//      items (distinct) in LDS; every thread ranks one of them against a 1/W
//      slice of the others; the group item of rank q-1 is an exact floor (q
//      items are >= it);
//   3. items >= the floor are appended to an LDS list (one atomic per wave);
//      survivor t counts the survivors that beat it and writes itself to
//      output slot `rank` (< q).
// Items are compared as (key, ~local slot) triples -- the local slot v*BS+tid
// orders a problem's items as their positions do -- with a 96-bit subtract's
// borrow (add_if_beats), and no position or validity array stays live across
// the keys phase (round 3's kept one and spilled it to scratch in the batched
// kernel: the reload sat at the head of the floor phase).
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
// [14], [15]: shader-clock counter at [0] and [4] (the clock rate over the block)
#define CE_STAMP(b, k)                                        \
    if (threadIdx.x == 0 && (b) < 8192) {                     \
        g_phase[b][k] = wall_clock64();                       \
        if ((k) == 0 || (k) == 4) g_phase[b][14 + (k) / 4] = clock64(); \
    }
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
    uint4 gb[64];                           // group items (~local slot, key lo, key hi, -)
    int part[WAVES][64];                    // partial ranks of the group items
    int cnt;                                // survivors appended
    uint4 cs[CAP];                          // survivors (~local slot, key lo, key hi, -)
    WaveListsT<WAVES> lists;                // fallback tree merge
};

// Keys of this thread's IPT items lo + tid + BS*v of [lo, hi) into slots
// [OFF, OFF + IPT): key 0 for a slot past the end or an excluded item (all
// loads in flight before the arithmetic; COMMIT: `tab` is committed once the
// data is awaited -- exactly one tile_keys call of a block commits).  Slots
// outside [OFF, OFF + IPT) are left as they are.
template <class Src, int IPT, int UNR, int BS, int K, int OFF, bool COMMIT>
__device__ __forceinline__ void tile_keys(const Src& src, int64_t lo, int64_t hi, const uint32_t* excl,
                                          LogTablePrefetch& tab, uint64_t (&k)[K]) {
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
    }
    if (len > 0) {  // block-uniform
        if constexpr (COMMIT) src.template keys_small<UNR, IPT>(items, kk, nlive, [&]() { tab.commit(); });
        else src.template keys_small<UNR, IPT>(items, kk, nlive);
    } else if constexpr (COMMIT) {
        tab.commit();
    }
#pragma unroll
    for (int v = 0; v < IPT; ++v) {
        bool ok = tid + (int64_t)BS * v < len;
        if (excl) ok = ok && !excluded(excl, items[v]);
        k[OFF + v] = ok ? kk[v] : 0ull;
    }
}

// r + 1 when triple a beats triple m, (~local slot, key lo, key hi) each: the
// borrow of the 96-bit difference m - a (higher key first, then lower slot) --
// three subtracts and an add-with-carry, no compare masks or scalar ops.
__device__ __forceinline__ int add_if_beats(int r, const uint4& m, const uint4& a) {
    int out;
    uint32_t t;
    asm("v_sub_co_u32 %1, vcc, %2, %5\n\t"
        "v_subb_co_u32 %1, vcc, %3, %6, vcc\n\t"
        "v_subb_co_u32 %1, vcc, %4, %7, vcc\n\t"
        "v_addc_co_u32 %0, vcc, 0, %8, vcc"
        : "=v"(out), "=&v"(t)
        : "v"(m.x), "v"(m.y), "v"(m.z), "v"(a.x), "v"(a.y), "v"(a.z), "v"(r)
        : "vcc");
    return out;
}

// The max key of each group of GS lanes (and the slot of one item holding it)
// in the group's lanes: DPP mirrors within quads, half rows and rows.
template <int GS>
__device__ __forceinline__ void group_max(uint64_t& k, uint32_t& n) {
#define CE_GM(J, CTL)                                                                                  \
    if constexpr (GS > J) {                                                                            \
        const uint32_t p0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)k, CTL, 0xF, 0xF, false);         \
        const uint32_t p1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(k >> 32), CTL, 0xF, 0xF, false); \
        const uint32_t pn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)n, CTL, 0xF, 0xF, false);                   \
        const uint64_t pk = ((uint64_t)p1 << 32) | p0;                                                 \
        if (pk > k) {                                                                                  \
            k = pk;                                                                                    \
            n = pn;                                                                                    \
        }                                                                                              \
    }
    CE_GM(1, 0xB1) CE_GM(2, 0x4E) CE_GM(4, 0x141) CE_GM(8, 0x140)  // quad [1,0,3,2], [2,3,0,1]; half-row, row mirror
#undef CE_GM
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
        uint64_t kz[K];  // key 0: no item
#pragma unroll
        for (int v = 0; v < K; ++v) kz[v] = 0;
        tile_keys<SrcA, IPTA, UNRA, BS, K, 0, true>(srcA, lo, hi, excl, tab, kz);
        if constexpr (IPTB > 0)
            if (both) tile_keys<SrcB, IPTB, UNRB, BS, K, IPTA, false>(srcB, 0, ta.nB, nullptr, tab, kz);
        CE_STAMP(blockIdx.x, 1)
        CE_WSTAMP(blockIdx.x)
        // 2. every slot as a triple (~local slot, key lo, key hi): local slot
        //    L = v * BS + tid orders the block's items as their positions do,
        //    so "a beats b" is the 96-bit compare of the triples (key 0: no item)
        const uint32_t ntid = ~(uint32_t)tid;
        uint32_t nl[K];
#pragma unroll
        for (int v = 0; v < K; ++v) nl[v] = ntid - (uint32_t)(v * BS);  // ~(v * BS + tid)
        // the lane's max key, its lowest slot on ties; then the group's max key
        // (a tie keeps the lane's own item: any item holding the group's max
        // key stands for the group -- 64 distinct items)
        uint64_t bk = kz[0];
        uint32_t bn = nl[0];
#pragma unroll
        for (int v = 1; v < K; ++v)
            if (kz[v] > bk) {
                bk = kz[v];
                bn = nl[v];
            }
        group_max<GS>(bk, bn);
        if ((tid & (GS - 1)) == 0) sm.gb[tid / GS] = make_uint4(bn, (uint32_t)bk, (uint32_t)(bk >> 32), 0u);
        if (tid == 0) sm.cnt = 0;
        __syncthreads();
        // floor = the group item of rank q-1 (ranks split over the waves; the
        // 64 triples are distinct, so exactly one lane holds rank q-1 <= 63)
        const uint4 mg = sm.gb[lane];
        {
            int r = 0;
#pragma unroll
            for (int j = 0; j < 64 / W; ++j) r = add_if_beats(r, mg, sm.gb[w * (64 / W) + j]);
            sm.part[w][lane] = r;
        }
        __syncthreads();
        uint64_t fk;
        uint32_t fn;
        {
            int r = 0;
#pragma unroll
            for (int j = 0; j < W; ++j) r += sm.part[j][lane];
            const int sl = __builtin_ctzll(__ballot(r == q - 1));
            fn = (uint32_t)__builtin_amdgcn_readlane((int)mg.x, sl);
            fk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mg.z, sl) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane((int)mg.y, sl);
        }
        const bool floor = fk != 0;  // else fewer than q groups hold an item: admit every item
        if (!floor) fn = 0;
        if (!floor) fk = 1;  // every valid key is > 1, key 0 (no item) is not
        // position of local slot L (segment A's slots first, then segment B's)
        auto pos_of = [&](uint32_t L) -> int64_t {
            return L < (uint32_t)(IPTA * BS) ? lo + rel + (int64_t)L : (int64_t)(L - (uint32_t)(IPTA * BS)) + relB;
        };
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
                pass[v] = (kz[v] > fk) | ((kz[v] == fk) & (nl[v] >= fn));  // bitwise: no per-slot branches
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
                    if (pass[v] && slot < SM::CAP)
                        sm.cs[slot] = make_uint4(nl[v], (uint32_t)kz[v], (uint32_t)(kz[v] >> 32), 0u);
                    base += __popcll(m[v]);
                }
            }
        }
        __syncthreads();
        CE_STAMP(blockIdx.x, 3)
        const int nc = sm.cnt;
        if (nc <= SM::CAP) {
            if (tid < nc) {  // survivor tid takes the slot of its rank
                const uint4 me = sm.cs[tid];
                int r = 0;
#pragma unroll 8
                for (int j = 0; j < nc; ++j) r = add_if_beats(r, me, sm.cs[j]);
                if (r < q) {
                    ov[r] = key_to_val(((uint64_t)me.z << 32) | me.y);
                    oi[r] = pos_of(~me.x);
                }
            } else if (tid < q) {  // fewer survivors than q: padding
                ov[tid] = __longlong_as_double(0x7ff8000000000000ll);
                oi[tid] = -1;
            }
            CE_STAMP(blockIdx.x, 4)
        } else {
            // overflow (> CAP items tie at or above the floor): per-wave lists + tree merge
            RegTopQ tq;
            if (floor) tq.init(q, fk, pos_of(~fn) + 1);  // admit candidates >= the floor
            else tq.init(q, 0, INT64_MAX);
#pragma unroll
            for (int v = 0; v < K; ++v) tq.offer(kz[v], pos_of(~nl[v]), kz[v] != 0);
            block_merge_write<W>(tq, sm.lists, q, nullptr, 0, ov, oi);
        }
    }
}

}  // namespace ce
