// ce_small.hpp -- pools of a few thousand items (BASELINE configs[0..2]: one
// reference-sized pool, the hc table, the [mc; hc] mix, 500 users in one
// launch), each problem (the pool, a user, the mix) selected by ONE block:
//
// Per block (amg_test.py:441-445 on the problem's items):
//   1. the log table's loads are issued, then the member loads of the
//      thread's item slots (item lo + tid + BS*v: each wave's loads coalesced);
//      each item's exact consensus row (f64 means) is formed as soon as its
//      own loads have landed, and kept in registers; from it an APPROXIMATE
//      entropy -- f32 copies, one hardware reciprocal, one hardware log2 per
//      class -- within e = kApproxErr2PerClass * C of the exact one (log2
//      units; ce_device.hpp), as a 32-bit key;
//   2. the max approximate key of each group of BS/64 lanes (DPP) -> 64 group
//      maxima (distinct items) in LDS; every thread counts, for one of them,
//      the maxima above / not below it over a 1/W slice; the value T of rank
//      q-1 has q distinct items at or above it;
//   3. survivors = items whose approximate entropy is >= T - 2 e,
//      plus every "special" row (negative / non-finite means, a sum outside
//      [2^-100, 2^100]: NaN / -inf entropies and the like, which the
//      approximation does not cover): a superset of the exact top q (q items
//      are exactly >= T - eps, so an item below T - eps cannot be among them,
//      and its approximation is below T - 2 eps).  Their rows go to LDS (one
//      atomic per wave);
//   4. the survivors' EXACT entropies (glibc log, scipy's quotients:
//      bit-identical to the reference), P = C rounded up to 2/4/8 lanes per
//      survivor, one class per lane (the wave issues each instruction once
//      for all lanes: one log chain instead of C in a row), terms gathered by
//      lane shuffles and summed in numpy's order; then every survivor counts
//      the survivors that beat it -- (key, ~local slot) triples, a 96-bit
//      subtract's borrow (add_if_beats) -- and writes itself to output slot
//      `rank` (< q).  Up to 64/P survivors (the usual case) are evaluated and
//      ranked by wave 0 alone, with no second block barrier.
// The exact entropy (the ~150-VALU glibc-log row) runs for the ~q survivors
// only, not for every item: the keys phase of round 3 was VALU-bound at two
// blocks per CU (configs[2]).  The local slot v*BS+tid orders a problem's
// items as their positions do, so no position array stays live.
// A problem longer than BS*IPT items (a long user of a ragged batch), or more
// than 64*W survivors (floods of near-ties at the floor), takes per-wave
// register lists + a tree merge instead (block-uniform branches, same answer).
#pragma once
#include "ce_stream.hpp"

namespace ce {

#ifdef CE_PHASE_TIMING
// diagnostic build only (-DCE_PHASE_TIMING): per-block wall-clock stamps (100 MHz)
// [0] start, [1] wave 0's keys done, [2] floor, [3] append, [4] rank, [5] exact keys (wave 0),
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

template <int WAVES, int C>
struct TileSmem {
    static constexpr int CAP = 64 * WAVES;  // one survivor per thread
    uint32_t gm[64];                        // group maxima of the approximate keys
    int part[WAVES][64];                    // partial counts (above | not below << 16)
    int cnt;                                // survivors appended
    uint4 cs[CAP + 8];                      // survivors' exact (~local slot, key lo, key hi, -), + 8 zero triples
    union {
        struct {
            double m[C][CAP];               // survivors' exact rows
            uint32_t nl[CAP];               // ... and ~local slots
        } sv;
        WaveListsT<WAVES> lists;            // fallback tree merge
    };
};

// Rows of this thread's IPT items lo + tid + BS*v of [lo, hi) into slots
// [OFF, OFF + IPT): the exact row in m, its approximate key in ak (0: no item
// -- past the end, excluded -- or a special row) and sp (special).  COMMIT:
// `tab` is committed once the first data is awaited -- exactly one tile_rows
// call of a block commits.  Slots outside [OFF, OFF + IPT) are left as they are.
template <class Src, int IPT, int UNR, int BS, int K, int C, int OFF, bool COMMIT, int THR = kSmallThrottle>
__device__ __forceinline__ void tile_rows(const Src& src, int64_t lo, int64_t hi, const uint32_t* excl,
                                          LogTablePrefetch& tab, double (&m)[K][C], uint32_t (&ak)[K],
                                          bool (&sp)[K]) {
    static_assert(OFF + IPT <= K && Src::kC == C, "");
    const int tid = threadIdx.x, w = tid >> 6;
    const int64_t len = hi - lo;
    int64_t items[IPT];
    int nlive = 0;  // this wave's item slots holding at least one real item (a prefix)
#pragma unroll
    for (int v = 0; v < IPT; ++v) {
        const int64_t j = tid + (int64_t)BS * v;
        items[v] = lo + (j < len ? j : (len > 0 ? len - 1 : 0));
        nlive += (int64_t)BS * v + 64 * w < len;
        ak[OFF + v] = 0;
        sp[OFF + v] = false;
#pragma unroll
        for (int c = 0; c < C; ++c) m[OFF + v][c] = 0.0;
    }
    auto sink = [&](int u, const double (&row)[C]) {
#pragma unroll
        for (int c = 0; c < C; ++c) m[OFF + u][c] = row[c];
        bool s;
        const uint32_t a = approx_key<C>(row, s);
        ak[OFF + u] = s ? 0u : a;
        sp[OFF + u] = s;
    };
    if (len > 0) {  // block-uniform
        auto commit = [&]() { tab.commit(); };
        if constexpr (COMMIT) src.template rows_small<UNR, IPT, decltype(sink)&, decltype(commit), THR>(items, nlive, sink, commit);
        else src.template rows_small<UNR, IPT, decltype(sink)&, NoHook, THR>(items, nlive, sink);
    } else if constexpr (COMMIT) {
        tab.commit();
    }
#pragma unroll
    for (int v = 0; v < IPT; ++v) {
        bool ok = tid + (int64_t)BS * v < len;
        if (excl) ok = ok && !excluded(excl, items[v]);
        if (!ok) {
            ak[OFF + v] = 0;
            sp[OFF + v] = false;
        }
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

// The max of each group of GS lanes in the group's lanes: DPP mirrors within
// quads, half rows and rows (one v_max per step).
template <int GS>
__device__ __forceinline__ uint32_t group_max(uint32_t k) {
#define CE_GM(J, CTL)                                                                              \
    if constexpr (GS > J) {                                                                        \
        const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k, CTL, 0xF, 0xF, false); \
        k = k > o ? k : o;                                                                         \
    }
    CE_GM(1, 0xB1) CE_GM(2, 0x4E) CE_GM(4, 0x141) CE_GM(8, 0x140)  // quad [1,0,3,2], [2,3,0,1]; half-row, row mirror
#undef CE_GM
    return k;
}

// LONG: a problem may exceed BS * IPT items (the per-wave streaming path is
// compiled in).  Launches whose host checks bound the problem (one pool, the
// mix) drop it -- half the code of the kernel.
template <class SrcA, class SrcB, int IPTA, int IPTB, int UNRA, int UNRB, int BS, bool LONG = true>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(LONG ? 4 : BS / 256))) void k_select_tiles(
    SrcA srcA, SrcB srcB, TileArgs ta, int q, double* __restrict__ oval, int64_t* __restrict__ oidx,
    const uint32_t* __restrict__ excl) {
    constexpr int W = BS / 64, GS = BS / 64;  // waves; lanes per group (64 groups)
    constexpr int K = IPTA + IPTB;  // slots: segment A's, then segment B's (both segments in one block)
    static_assert(BS % 64 == 0 && BS >= 128 && GS <= 16 && (GS & (GS - 1)) == 0, "block size");
    constexpr int C = SrcA::kC;
    static_assert(IPTB == 0 || SrcB::kC == C, "both segments' rows have C classes");
    using SM = TileSmem<W, C>;
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
        // 1. exact rows + approximate keys of this thread's items
        double mrow[K][C];
        uint32_t ak[K];
        bool sp[K];
        tile_rows<SrcA, IPTA, UNRA, BS, K, C, 0, true>(srcA, lo, hi, excl, tab, mrow, ak, sp);
        if constexpr (IPTB > 0)
            if (both) tile_rows<SrcB, IPTB, UNRB, BS, K, C, IPTA, false>(srcB, 0, ta.nB, nullptr, tab, mrow, ak, sp);
        CE_STAMP(blockIdx.x, 1)
        CE_WSTAMP(blockIdx.x)
        const uint32_t ntid = ~(uint32_t)tid;
        // position of local slot L (segment A's slots first, then segment B's)
        auto pos_of = [&](uint32_t L) -> int64_t {
            return L < (uint32_t)(IPTA * BS) ? lo + rel + (int64_t)L : (int64_t)(L - (uint32_t)(IPTA * BS)) + relB;
        };
        // 2. T = the group maximum of rank q-1 (with multiplicity): q distinct
        //    items have approximate keys >= T
        uint32_t bk = ak[0];
#pragma unroll
        for (int v = 1; v < K; ++v) bk = bk > ak[v] ? bk : ak[v];
        bk = group_max<GS>(bk);
        if ((tid & (GS - 1)) == 0) sm.gm[tid / GS] = bk;
        if (tid == 0) sm.cnt = 0;
        __syncthreads();
        const uint32_t mg = sm.gm[lane];
        {
            int r = 0;
#pragma unroll
            for (int j = 0; j < 64 / W; ++j) {
                const uint32_t o = sm.gm[w * (64 / W) + j];
                r += (o > mg ? 1 : 0) + (o >= mg ? 0x10000 : 0);
            }
            sm.part[w][lane] = r;
        }
        __syncthreads();
        uint32_t thr;  // survivors: approximate key >= thr (>= 1: never a slot without an item)
        {
            int r = 0;
#pragma unroll
            for (int j = 0; j < W; ++j) r += sm.part[j][lane];
            const int above = r & 0xffff, notbelow = r >> 16;
            const int sl = __builtin_ctzll(__ballot(above < q && notbelow >= q));
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)mg, sl);
            thr = 1;
            if (T != 0) {  // else fewer than q ordinary items: every item survives
                const float lim = approx_key_value(T) - 2.0f * kApproxErr2PerClass * C;
                const uint32_t b = __float_as_uint(lim);
                const uint32_t tk = (b >> 31) ? ~b : (b | 0x80000000u);
                thr = tk > 1 ? tk : 1;
            }
        }
        CE_STAMP(blockIdx.x, 2)
        // 3. survivors -> LDS rows: the wave's K ballots first, then ONE atomic
        //    per wave for all of its survivors
        {
            bool pass[K];
            uint64_t msk[K];
            int tot = 0;
#pragma unroll
            for (int v = 0; v < K; ++v) {
                pass[v] = sp[v] | (ak[v] >= thr);
                msk[v] = __ballot(pass[v]);
                tot += __popcll(msk[v]);
            }
            if (tot) {  // wave-uniform
                int base = 0;
                if (lane == 0) base = atomicAdd(&sm.cnt, tot);
                base = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
                for (int v = 0; v < K; ++v) {
                    const int slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(msk[v] >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)msk[v], 0));
                    CE_DASSERT(slot >= 0);
                    if (pass[v] && slot < SM::CAP) {
#pragma unroll
                        for (int c = 0; c < C; ++c) sm.sv.m[c][slot] = mrow[v][c];
                        sm.sv.nl[slot] = ntid - (uint32_t)(v * BS);  // ~(v * BS + tid)
                    }
                    base += __popcll(msk[v]);
                }
            }
        }
        __syncthreads();
        CE_STAMP(blockIdx.x, 3)
        const int nc = sm.cnt;
        if (nc <= SM::CAP) {
            // 4. exact entropies of the survivors, P lanes per survivor (one
            //    class each: one glibc log per lane instead of C in a row --
            //    the wave issues each instruction once for all its lanes), the
            //    terms gathered by lane shuffles and summed in numpy's order;
            //    then ranks.  Up to 64/P survivors (the usual case) stay in
            //    wave 0: no second block barrier.
            constexpr int P = C <= 2 ? 2 : (C <= 4 ? 4 : 8);
            constexpr int SPW = 64 / P;
            static_assert(C <= 8, "single-block pools hold rows of <= 8 classes");
            CE_DASSERT(nc >= 0 && nc + 8 <= SM::CAP + 8);
            if (tid < 8) sm.cs[nc + tid] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll 1
            for (int t0 = w * SPW; t0 < nc; t0 += W * SPW) {  // wave-uniform
                const int t = t0 + lane / P, c = lane % P;
                const int ts = t < nc ? t : 0;
                double x[C];
#pragma unroll
                for (int cc = 0; cc < C; ++cc) x[cc] = sm.sv.m[cc][ts];
                const double xc = sm.sv.m[c < C ? c : 0][ts];
                const double s = row_sum<C>(x);
                const double e = entr(row_quotient_one<C>(x, s, xc));
                double ee[C];
#pragma unroll
                for (int j = 0; j < C; ++j) ee[j] = __shfl(e, (lane & ~(P - 1)) + j);
                const uint64_t key = order_key(row_sum<C>(ee));
                CE_DASSERT(ts >= 0 && ts < SM::CAP);
                if (t < nc && c == 0) sm.cs[t] = make_uint4(sm.sv.nl[t], (uint32_t)key, (uint32_t)(key >> 32), 0u);
            }
            CE_STAMP(blockIdx.x, 5)
            auto rank_write = [&](int i) {  // survivor i takes the slot of its rank
                const uint4 me = sm.cs[i];
                int r = 0;
                // 8 triples per LDS round trip (the asm keeps the compiler from
                // unrolling a runtime-bounded loop itself: one round trip per
                // survivor measured 0.84 us); cs[nc, nc + 8) holds zero triples,
                // which beat nothing
#pragma unroll 1
                for (int j0 = 0; j0 < nc; j0 += 8) {
                    CE_DASSERT(j0 + 8 <= SM::CAP + 8);  // the zero-padded triples [nc, nc + 8)
                    uint4 a[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) a[k] = sm.cs[j0 + k];
#pragma unroll
                    for (int k = 0; k < 8; ++k) r = add_if_beats(r, me, a[k]);
                }
                CE_DASSERT(i < nc && r >= 0 && r < nc);
                if (r < q) {
                    ov[r] = key_to_val(((uint64_t)me.z << 32) | me.y);
                    oi[r] = pos_of(~me.x);
                }
            };
            auto pad = [&](int i) {  // fewer survivors than q: padding
                ov[i] = __longlong_as_double(0x7ff8000000000000ll);
                oi[i] = -1;
            };
            if (nc <= SPW) {  // block-uniform: wave 0 wrote every triple and ranks them
                if (w == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    if (lane < nc) rank_write(lane);
                    else if (lane < q) pad(lane);
                }
            } else {
                __syncthreads();
                if (tid < nc) rank_write(tid);
                else if (tid < q) pad(tid);
            }
            CE_STAMP(blockIdx.x, 4)
        } else {
            // overflow (> CAP items at or near the floor): exact keys of every
            // item, per-wave lists + tree merge
            RegTopQ tq;
            tq.init(q);
#pragma unroll
            for (int v = 0; v < K; ++v) {
                const bool ok = sp[v] | (ak[v] != 0);
                const uint64_t key = ok ? order_key(entropy_row<C>(mrow[v])) : 0ull;
                tq.offer(key, pos_of((uint32_t)(v * BS + tid)), ok);
            }
            block_merge_write<W>(tq, sm.lists, q, nullptr, 0, ov, oi);
        }
    }
}

}  // namespace ce
