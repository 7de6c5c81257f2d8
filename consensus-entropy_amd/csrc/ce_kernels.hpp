// ce_kernels.hpp -- MI355X (gfx950) kernel templates shared by the C-ABI translation units
// (ce_abi_core.hip, ce_abi_select.hip, ce_abi_batch.hip).
//
// Kernels (DESIGN.md has the roofline of each):
//   k_partial<Src>   score items (committee consensus entropy, an entropy
//                    vector, or an hc table row) and keep a per-block top-q in
//                    LDS; one pass over HBM, entropies never written back.
//                    Replaces amg_test.py:441-445 / :451-452 / :479-480.
//   k_finish         merge the blocks' (or ranks') candidate lists into the
//                    final top-q; one block per segment (user / pool).
//   k_entropy        per-item entropy to HBM (ce_committee_entropy).
//   k_vote / k_va    hc frequency table + entropy from votes (amg_test.py:88-117).
//   k_segment_mean   frame -> song mean of one member (groupby mean, amg_test.py:437).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdarg.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "../../include/ce.h"
#include "ce_device.hpp"
#include "ce_topq.hpp"
#include "ce_wide.hpp"
#include "ce_stream.hpp"
#include "ce_small.hpp"
#include "ce_members.hpp"
#include "ce_abi.hpp"

namespace ce {

constexpr int kBS = 256;          // stage-1 block: 4 waves
constexpr int kFinBS = 1024;      // stage-2 block: 16 waves
constexpr int kMinItemsPerBlock = 64;
constexpr int64_t kSmallPoolBytes = 256 * 1024;  // below this one block does the whole selection
constexpr int kMaxBlocks = 1024;  // stage-1 blocks per pool (4 per CU on 256 CUs)
constexpr int kSegWaves = 16;     // waves per single-block pool / per user (k_stream_seg)

// ---------------------------------------------------------------------------
// Item sources.  key(i) returns the order key of global item i.
// ---------------------------------------------------------------------------



template <int DT, int C, bool VEC>
struct CommitteeSrc {
    const void* p;
    int64_t sN, sM, sC;
    int M;
    double dM, invM;
    bool pow2;
    static constexpr int kC = C;
    static constexpr int kDT = DT;
    static constexpr bool kVec = VEC;
    static constexpr int kUnr = DT == kF64 ? 4 : 8;
    __device__ __forceinline__ void mean(int64_t i, double (&m)[C]) const {
        committee_mean<DT, C, VEC, kUnr>(p, i * sN, M, sM, sC, dM, invM, pow2, m);
    }
    // IPL items at once: all their member loads in flight together
    // hook() runs after the means, before the first log (e.g. LogTablePrefetch::commit)
    template <int UNR, int IPL, class Hook = NoHook>
    __device__ __forceinline__ void keys(const int64_t (&items)[IPL], uint64_t (&k)[IPL], Hook hook = {}) const {
        int64_t offs[IPL];
#pragma unroll
        for (int u = 0; u < IPL; ++u) offs[u] = items[u] * sN;
        double m[IPL][C];
        committee_mean_multi<DT, C, VEC, UNR, IPL>(p, offs, M, sM, sC, dM, invM, pow2, m);
        hook();
#pragma unroll
        for (int u = 0; u < IPL; ++u) k[u] = order_key(entropy_row<C>(m[u]));
    }
    // The exact consensus rows (amg_test.py:441) of IPL item slots for the
    // latency-bound single-block pools: sink(u, m) receives slot u's row, for
    // u < nlive only (wave-uniform: no lane of the wave owns a real item at u
    // >= nlive).  When the whole committee fits one batch (M <= UNR) the loads
    // are issued item by item and each item's mean runs as soon as ITS loads
    // have landed.  Every slot's loads are issued, also for slots without a
    // real item (their addresses are clamped to the pool's last item: one
    // cache line per wave): loads under a branch leave the compiler unable to
    // count them, and it then waits for ALL of them (vmcnt(0)) before the log
    // table's commit.  hook() runs after the first means (e.g.
    // LogTablePrefetch::commit).
    template <int UNR, int IPL, class Sink, class Hook = NoHook, int THR = kSmallThrottle>
    __device__ __forceinline__ void rows_small(const int64_t (&items)[IPL], int nlive, Sink&& sink,
                                               Hook hook = {}) const {
        if (M > UNR) {
            // committees larger than one batch: f32 rows keep all IPL items' member
            // batches in flight (IPL x UNR x 4 VGPRs); f64 rows of C >= 4 would need
            // twice that, so they go item by item (UNR members in flight)
            if constexpr (!(DT == kF64 && C >= 4)) {
                int64_t offs[IPL];
#pragma unroll
                for (int u = 0; u < IPL; ++u) offs[u] = items[u] * sN;
                double m[IPL][C];
                committee_mean_multi<DT, C, VEC, UNR, IPL>(p, offs, M, sM, sC, dM, invM, pow2, m);
                hook();
#pragma unroll
                for (int u = 0; u < IPL; ++u)
                    if (u < nlive) sink(u, m[u]);
                return;
            }
#pragma unroll
            for (int u = 0; u < IPL; ++u) {
                double m[C];
                committee_mean<DT, C, VEC, UNR>(p, items[u] * sN, M, sM, sC, dM, invM, pow2, m);
                if (u == 0) hook();
                if (u < nlive) sink(u, m);
            }
            return;
        }
        MemberLoad<DT, C, VEC> ld[IPL][UNR];
        auto issue = [&](int u) {
#pragma unroll
            for (int v = 0; v < UNR; ++v) ld[u][v].load(p, items[u] * sN + (int64_t)(v < M ? v : M - 1) * sM, sC);
        };
        // THR item slots in flight per lane (THR < IPL: slot u + THR is issued
        // only once slot u has landed, so every block keeps a bounded share of
        // the memory queues instead of all of its bytes at once)
        constexpr int D = (THR > 0 && THR < IPL) ? THR : IPL;
#pragma unroll
        for (int i = 0; i < D; ++i) issue(i);
        hook();
        auto item = [&](auto full) {
#pragma unroll
            for (int i = 0; i < IPL; ++i) {
                const int u = i;
                if constexpr (D < IPL) {
                    if (i + D < IPL) {
                        // slot u landed (the asm reads its registers: the compiler waits
                        // for exactly those loads), then the next slot is issued; the
                        // memory clobber keeps that issue behind the wait
#pragma unroll
                        for (int v = 0; v < UNR; ++v) ld[u][v].pin();
                        asm volatile("" ::: "memory");
                        issue(i + D);
                    }
                }
                if (u >= nlive) continue;  // wave-uniform
                double acc[C];
#pragma unroll
                for (int c = 0; c < C; ++c) acc[c] = 0.0;
#pragma unroll
                for (int v = 0; v < UNR; ++v) {
                    if constexpr (decltype(full)::value) ld[u][v].add_to(acc);  // M == UNR: no padding
                    else ld[u][v].add_masked(acc, v < M);
                }
                double m[C];
#pragma unroll
                for (int c = 0; c < C; ++c) m[c] = div_members(acc[c], dM, invM, pow2);
                sink(u, m);
            }
        };
        if (M == UNR) item(std::true_type());
        else item(std::false_type());
    }
    __device__ __forceinline__ double entropy(int64_t i) const {
        double m[C];
        mean(i, m);
        return entropy_row<C>(m);
    }
    __device__ __forceinline__ uint64_t key(int64_t i) const { return order_key(entropy(i)); }
};

struct ArraySrc {  // precomputed entropies
    const double* e;
    __device__ __forceinline__ uint64_t key(int64_t i) const { return order_key(e[i]); }
};

template <int C>
struct TableSrc {  // hc frequency table rows [N_h, C] f64 (amg_test.py:451)
    const double* t;
    int64_t ld;
    __device__ __forceinline__ uint64_t key(int64_t i) const {
        double row[C];
#pragma unroll
        for (int c = 0; c < C; ++c) row[c] = t[i * ld + c];
        return order_key(entropy_row<C>(row));
    }
};

// Segment geometry: block b -> segment b / bpu, chunk b % bpu.
struct Seg {
    const int64_t* offsets;  // [U+1] device, or nullptr: one segment [0, N)
    int64_t N;
    int bpu;
    int64_t base_idx;
    const uint32_t* excl;    // exclusion bitmap over items 0..N-1 (one segment), or nullptr
};

__device__ __forceinline__ void seg_range(const Seg& sg, int64_t& s0, int64_t& lo, int64_t& hi) {
    const int b = blockIdx.x;
    const int u = b / sg.bpu, c = b % sg.bpu;
    int64_t s1;
    if (sg.offsets) {
        s0 = sg.offsets[u];
        s1 = sg.offsets[u + 1];
    } else {
        s0 = 0;
        s1 = sg.N;
    }
    const int64_t len = s1 > s0 ? s1 - s0 : 0;
    int64_t per = (len + sg.bpu - 1) / sg.bpu;
    per = (per + kBS - 1) / kBS * kBS;
    lo = s0 + (int64_t)c * per;
    hi = lo + per < s1 ? lo + per : s1;
    if (lo > hi) lo = hi;
}

// Write a finished top-q: either (key, idx) candidates into the workspace, or
// the final (val, idx) outputs.  Slots past `cnt` are padding (idx -1).
template <int CAP, bool FINAL>
__device__ __forceinline__ void write_list(const TopQSmem<CAP>& s, int cnt, int q, Cand* wc, double* oval,
                                           int64_t* oidx) {
    for (int r = threadIdx.x; r < q; r += blockDim.x) {
        const bool ok = r < cnt;
        if constexpr (FINAL) {
            oval[r] = ok ? key_to_val(s.key[r]) : __longlong_as_double(0x7ff8000000000000ll);
            oidx[r] = ok ? s.idx[r] : -1;
        } else {
            wc[r] = Cand{ok ? s.key[r] : 0ull, ok ? s.idx[r] : -1};
        }
    }
}

// ---------------------------------------------------------------------------
// Stage 1: score + per-block top-q.  One item per thread per round.
// ---------------------------------------------------------------------------
template <class Src, int CAP, bool FINAL>
__global__ __launch_bounds__(kBS) void k_partial(Src src, Seg sg, int q, Cand* __restrict__ wc, double* __restrict__ oval,
                                                 int64_t* __restrict__ oidx) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    __shared__ TopQSmem<CAP> sm;
    TopQ<CAP, kBS> tq(sm);
    tq.init();
    CE_DASSERT(q >= 1 && q <= CAP);
    int64_t s0, lo, hi;
    seg_range(sg, s0, lo, hi);
    const int64_t rel = sg.base_idx - s0;
    for (int64_t i0 = lo; i0 < hi; i0 += kBS) {
        const int64_t i = i0 + threadIdx.x;
        const bool valid = i < hi && !(sg.excl && excluded(sg.excl, i));
        uint64_t k = 0;
        if (valid) k = src.key(i);
        tq.offer(k, i + rel, valid);
        tq.end_round(q, kBS);
    }
    const int cnt = tq.finish(q);
    const int64_t slot = (int64_t)blockIdx.x * q;
    write_list<CAP, FINAL>(sm, cnt, q, wc + slot, oval + (FINAL ? slot : 0), oidx + (FINAL ? slot : 0));
}

// Wide-class variant of k_partial (q > 64 / segments): a wave scores 64
// consecutive items (one per lane slot), so a block round is still 256.
template <int DT, int NPL, bool VEC, int CAP, bool FINAL>
__global__ __launch_bounds__(kBS) void k_partial_wide(WideArgs a, PwPlan pl, Seg sg, int q, Cand* __restrict__ wc,
                                                      double* __restrict__ oval, int64_t* __restrict__ oidx);

// Wide classes on the streaming engine (q <= 64): one wave per item, every
// wave independent, per-wave top-q.  NPL = classes owned per lane (C <= 64*NPL).
template <int DT, int NPL, bool VEC>
__device__ __forceinline__ double wide_item(const WideArgs& a, const PwPlan& pl, int64_t it, double* row,
                                            double* scratch) {
    if constexpr (VEC) {
        constexpr int KCH = NPL / ChunkT<DT>::CPC;
        constexpr int UNR = KCH >= 8 ? 1 : 8 / KCH;
        return wave_item_entropy_vec<DT, KCH, UNR>(a.p, it * a.sN, a.M, a.C, a.sM, a.dM, a.invM, a.pow2, pl, row,
                                                   scratch);
    } else {
        return wave_item_entropy<DT, NPL>(a.p, it * a.sN, a.M, a.C, a.sM, a.sC, a.dM, a.invM, a.pow2, pl, row,
                                          scratch, nullptr);
    }
}

template <int DT, int NPL, bool VEC, int CAP, bool FINAL>
__global__ __launch_bounds__(kBS) void k_partial_wide(WideArgs a, PwPlan pl, Seg sg, int q, Cand* __restrict__ wc,
                                                      double* __restrict__ oval, int64_t* __restrict__ oidx) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    __shared__ TopQSmem<CAP> sm;
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    TopQ<CAP, kBS> tq(sm);
    tq.init();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* row = wsm + w * wide_lds_doubles(a.C);
    double* scratch = row + a.C;
    int64_t s0, lo, hi;
    seg_range(sg, s0, lo, hi);
    const int64_t rel = sg.base_idx - s0;
    for (int64_t i0 = lo; i0 < hi; i0 += kBS) {
        uint64_t mykey = 0;
        const int64_t wbase = i0 + 64 * w;
        for (int j = 0; j < 64; ++j) {
            const int64_t it = wbase + j;
            if (it >= hi) break;  // wave-uniform
            const double h = wide_item<DT, NPL, VEC>(a, pl, it, row, scratch);
            if (lane == j) mykey = order_key(h);
        }
        const int64_t i = i0 + threadIdx.x;
        tq.offer(mykey, i + rel, i < hi && !(sg.excl && excluded(sg.excl, i)));
        tq.end_round(q, kBS);
    }
    const int cnt = tq.finish(q);
    const int64_t slot = (int64_t)blockIdx.x * q;
    write_list<CAP, FINAL>(sm, cnt, q, wc + slot, oval + (FINAL ? slot : 0), oidx + (FINAL ? slot : 0));
}

template <int DT, int NPL, bool VEC>
__global__ __launch_bounds__(kBS) void k_stream_wide(WideArgs a, PwPlan pl, StreamArgs sa, int q,
                                                     Cand* __restrict__ wc) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    __shared__ WaveLists sm;
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* row = wsm + w * wide_lds_doubles(a.C);
    double* scratch = row + a.C;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    int64_t lo = gw * sa.per_wave;
    int64_t hi = lo + sa.per_wave;
    if (hi > a.N) hi = a.N;
    if (lo > hi) lo = hi;
    RegTopQ tq;
    tq.init(q);
    for (int64_t t0 = lo; t0 < hi; t0 += 64) {
        uint64_t mykey = 0;
        for (int j = 0; j < 64; ++j) {
            const int64_t it = t0 + j;
            if (it >= hi) break;  // wave-uniform
            const double h = wide_item<DT, NPL, VEC>(a, pl, it, row, scratch);
            if (lane == j) mykey = order_key(h);
        }
        const int64_t i = t0 + lane;
        tq.offer(mykey, i + sa.base_idx, i < hi);
    }
    block_merge_write<4>(tq, sm, q, wc + (int64_t)blockIdx.x * q, sa.nlists);
}

// Wide classes, vectorised rows (q <= 64): one wave per item, lanes over 16-B
// chunks, software-pipelined over the wave's flat sequence of (item, member
// batch) pairs -- batch t+1 is in flight while batch t is added, and the next
// item's first batch while an item's entropy is computed, so the wave always
// has 2 x UNR x KCH 16-B loads per lane outstanding.  Items per wave are not
// rounded to 64 (a wide item is tens of KB): every wave of the resident grid
// gets work.
// Measured and not kept: a 3-deep ring (0.782-0.784 vs
// 0.790-0.801 of HBM), a 4-wave register cap, the entr pass fed from the LDS
// row, and 16 KiB LDS-DMA tiles per wave (1.5-2.5 % slower on the C5 job).
#ifndef CE_WIDE_PREFILTER
#define CE_WIDE_PREFILTER 1
#endif
// The wide stream's floor and grid, chosen on the device before the stream
// (ce_launch_stream.hip; every wide launch with heavy items that folds its
// lists: single selections, the multi-GPU records, every chunk of a job):
//   k_wide_seed       wide_nsamples(N) items, one per stratum of the pool at a
//                     hashed offset, one wave each: the EXACT entropy (the
//                     stream's own arithmetic) and the approximate one;
//   k_wide_seed_pick  the floor = the better of the samples' q-th best (key,
//                     any position: every one of those q items is in the pool
//                     and re-enters the stream's lists, ties included) and a
//                     chunked job's running q-th entry; then the vote = the
//                     samples that would still take the exact entropy against it.
// Both grids are launched; the one the vote does not pick exits at its first
// instruction.  The deep-ring grid (one block per CU, 8-batch ring) reads a
// pool whose items nearly all skip at 0.86-0.89 of HBM but one whose items
// mostly take the exact entropy at 0.51, where the occupancy grid keeps
// 0.79-0.82 (profiles/r06_c5_vote.json): it runs iff at most 1/kWideVoteDen
// of the samples are exact.  The sampled floor leaves ~q / kWideVoteSamples of
// any pool above it whatever the pool's order (a rising-entropy pool included),
// so single selections and first chunks get the deep grid too.  The samples
// read 1/16 of a small launch's items and 256 MB of a 128 GB C5 chunk.
constexpr int kWideVoteSamples = 4096;
constexpr int kWideVoteDen = 16;
// samples of an N-item launch: N / 16, at most kWideVoteSamples (the launcher
// runs the path from 1024 samples on: N >= 16384)
__host__ __device__ __forceinline__ int64_t wide_nsamples(int64_t N) {
    return N / 16 < kWideVoteSamples ? N / 16 : kWideVoteSamples;
}
__device__ __forceinline__ bool wide_vote_heavy(uint32_t v, int64_t N) {
    return (int64_t)v * kWideVoteDen <= wide_nsamples(N);
}
// sample s of ns over [0, N): stratum s at a hashed offset (no periodic pool
// pattern lines up with the samples)
__host__ __device__ __forceinline__ int64_t wide_sample_pos(int64_t s, int64_t ns, int64_t N) {
    const int64_t lo = s * N / ns, hi = (s + 1) * N / ns;
    uint32_t h = (uint32_t)s * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    return hi > lo ? lo + (int64_t)(h % (uint64_t)(hi - lo)) : lo;
}
template <int DT, int KCH, int UNR>
__global__ __launch_bounds__(kBS) void k_wide_seed(WideArgs a, PwPlan pl, int64_t base_idx,
                                                   const uint32_t* __restrict__ excl, Cand* __restrict__ samp,
                                                   float* __restrict__ sapx) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t ns = wide_nsamples(a.N);
    const int64_t s = (int64_t)blockIdx.x * 4 + w;
    if (s >= ns) return;  // wave-uniform (after the block's only barrier)
    CE_DASSERT(a.M % UNR == 0);
    constexpr int CPC = ChunkT<DT>::CPC, EB = 16 / CPC;
    const int K = a.C / CPC;
    double* row = wsm + w * wide_lds_doubles(a.C);
    double* scratch = row + a.C;
    uint32_t off[KCH];
#pragma unroll
    for (int kk = 0; kk < KCH; ++kk) {
        const int ch = lane + 64 * kk;
        off[kk] = 16u * (uint32_t)(ch < K ? ch : K - 1);
    }
    const int64_t i = wide_sample_pos(s, ns, a.N);
    const char* item = static_cast<const char*>(a.p) + i * a.sN * EB;
    double acc[KCH * CPC];
#pragma unroll
    for (int x = 0; x < KCH * CPC; ++x) acc[x] = 0.0;
    WideBatch<DT, KCH, UNR> b;
    for (int m = 0; m < a.M; m += UNR) {  // member order, as the stream adds
        b.issue(item, m, a.sM * EB, off);
        b.add(acc);
    }
    bool special;
    const float ap = wave_approx_entropy<DT, KCH>(acc, K, special);
    const double h = wave_entropy_from_sums<DT, KCH>(acc, K, a.dM, a.invM, a.pow2, pl, row, scratch);
    if (lane == 0) {
        const bool out = excl != nullptr && excluded(excl, i);
        samp[s] = Cand{out ? 0ull : order_key(h), i + base_idx};
        sapx[s] = out ? -__builtin_inff() : (special ? __builtin_inff() : ap);  // -inf: never exact; +inf: always
    }
}
// one block of 16 waves (a template: defined in a header that several
// translation units include, instantiated in one)
template <int NS>
__global__ __launch_bounds__(1024) void k_wide_seed_pick(const Cand* __restrict__ samp, const float* __restrict__ sapx,
                                                         int ns, int q, const Cand* __restrict__ extra,
                                                         Cand* __restrict__ seed, uint32_t* __restrict__ vote) {
    __shared__ WaveListsT<16> sm;
    __shared__ Cand lst[kStreamMaxQ];
    __shared__ Cand pick;
    __shared__ uint32_t cnt;
    CE_DASSERT(ns <= NS && q >= 1 && q <= kStreamMaxQ && blockDim.x == 1024);
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    // the samples' top q (per-wave register lists over 64-sample rounds, then the
    // block's merge tree): lst[q - 1] is the q-th best
    RegTopQ tq;
    tq.init(q);
    for (int j0 = w * 64; j0 < ns; j0 += 1024) {  // wave-uniform
        const int j = j0 + lane;
        const Cand c = j < ns ? samp[j] : Cand{0ull, -1};
        tq.offer(c.key, c.idx, j < ns && c.key != 0);
    }
    block_merge_write<16>(tq, sm, q, lst, 1);
    if (t == 0) cnt = 0u;
    __syncthreads();
    if (t == 0) {
        // the q-th best sample as a floor admitting every item of its key (each of
        // the q samples is in the pool and re-enters the stream's lists, ties
        // included); a chunked job's running list's q-th entry is a floor too
        const Cand s = lst[q - 1];
        Cand f = (s.idx >= 0 && s.key != 0) ? Cand{s.key, INT64_MAX} : Cand{0ull, -1};
        if (extra != nullptr) {
            const Cand e = extra[q - 1];
            if (e.idx >= 0 && e.key != 0 && (f.idx < 0 || better(e.key, e.idx, f.key, f.idx))) f = e;
        }
        pick = f;
    }
    __syncthreads();
    const Cand f = pick;
    // the vote: samples the prefilter would still send to the exact entropy
    uint32_t mine = 0;
    for (int j = t; j < ns; j += 1024) {
        bool exact = true;
        if (f.idx >= 0 && f.key != 0)
            exact = !(sapx[j] == -__builtin_inff()) &&
                    !(f.key == ~0ull || (double)sapx[j] < key_to_val(f.key) * 1.4426950408889634 - 2.0 * kWideApproxErr2);
        mine += exact ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
    if (lane == 0 && mine) atomicAdd(&cnt, mine);
    __syncthreads();
    if (t == 0) {
        seed[0] = f;
        vote[0] = cnt;
    }
}

template <int DT, int KCH, int UNR, int NB = 2>
__global__ __launch_bounds__(kBS) void k_stream_wide2(WideArgs a, PwPlan pl, StreamArgs sa, int q,
                                                      Cand* __restrict__ wc) {
    // the device-side grid choice (k_wide_seed_pick's vote): the other grid runs
    if (sa.vote && wide_vote_heavy(*sa.vote, sa.N) != (sa.vote_heavy != 0)) return;
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    CE_DASSERT((int)gridDim.x <= sa.nlists && q >= 1 && q <= kStreamMaxQ && a.M % UNR == 0);
    __shared__ WaveLists sm;
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    constexpr int CPC = ChunkT<DT>::CPC, EB = 16 / CPC;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* row = wsm + w * wide_lds_doubles(a.C);
    double* scratch = row + a.C;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    // the wave's items: cnt items lo0, lo0 + stride, ...  -- grid-cyclic (wave
    // g takes items g, g + W, ...: the items in flight at any moment are one
    // contiguous sweep; C5 job 0.754-0.770 -> 0.779-0.781 of HBM against a
    // contiguous run per wave on one box, profiles/r03_tile_order.json)
    const int64_t W = (int64_t)gridDim.x * 4;
    const int64_t lo0 = gw, stride = W;
    const int64_t cnt = a.N > gw ? (a.N - gw + W - 1) / W : 0;
    RegTopQ tq;
    tq.init(q);
#if CE_WIDE_PREFILTER
    // the floor (k_wide_seed_pick: sampled items, or a chunked job's running
    // list -- sa.extra, the top q of every chunk so far): an item not better
    // than it cannot enter the top q, so the prefilter skips from the first
    // item on
    if (sa.seed || sa.extra) {
        CE_DASSERT(q >= 1 && q <= kStreamMaxQ);
        const Cand e = sa.seed ? sa.seed[0] : sa.extra[q - 1];
        if (e.idx >= 0 && e.key != 0) tq.init(q, e.key, e.idx);
    }
#endif
    const char* base = static_cast<const char*>(a.p);
    const int64_t sNb = a.sN * EB, sMb = a.sM * EB;
    const int K = a.C / CPC;
    const int NBM = a.M / UNR;  // member batches per item (UNR divides M, host)
    double acc[KCH * CPC];
#pragma unroll
    for (int e = 0; e < KCH * CPC; ++e) acc[e] = 0.0;
    uint64_t mykey = 0;
    int64_t myidx = 0;
    // issue cursor (item ordinal, batch) and consume cursor
    int64_t ii = 0, ci = 0;
    int ib = 0, cb = 0;
    uint32_t off[KCH];  // this lane's chunk offsets in a member row (clamped into the row)
#pragma unroll
    for (int kk = 0; kk < KCH; ++kk) {
        const int ch = lane + 64 * kk;
        off[kk] = 16u * (uint32_t)(ch < K ? ch : K - 1);
    }
    WideBatch<DT, KCH, UNR> buf[NB];  // ring: NB - 1 batches in flight while one is added
    auto issue = [&](WideBatch<DT, KCH, UNR>& X) {
        X.issue(base + (lo0 + ii * stride) * sNb, ib * UNR, sMb, off);
        if (++ib == NBM) {
            ib = 0;
            ++ii;
        }
    };
    auto consume = [&](const WideBatch<DT, KCH, UNR>& X) {
        X.add(acc);
        if (++cb == NBM) {  // item ci complete
            cb = 0;
            // approximate prefilter (wave-uniform): an item whose approximate
            // entropy is more than 2 kWideApproxErr2 below the wave's current
            // threshold (its q-th best exact key, or the running floor) cannot
            // enter the top q -- its exact entropy is below the threshold -- and
            // skips the exact entropy (the row sums through LDS, C glibc logs)
            bool skip = false;
#if CE_WIDE_PREFILTER
            if (tq.tk != 0) {
                bool special;
                const float ap = wave_approx_entropy<DT, KCH>(acc, K, special);
                if (!special)
                    skip = tq.tk == ~0ull ||  // q NaN entropies held: only a NaN ties
                           (double)ap < key_to_val(tq.tk) * 1.4426950408889634 - 2.0 * kWideApproxErr2;
            }
#endif
            double h = 0.0;
            if (!skip) h = wave_entropy_from_sums<DT, KCH>(acc, K, a.dM, a.invM, a.pow2, pl, row, scratch);
#pragma unroll
            for (int e = 0; e < KCH * CPC; ++e) acc[e] = 0.0;
            const int j = (int)(ci & 63);
            if (lane == j) {
                mykey = skip ? 0ull : order_key(h);
                myidx = lo0 + ci * stride;
            }
            if (j == 63 || ci == cnt - 1) {
                bool ok = lane <= j;
                if (sa.excl) ok = ok && !excluded(sa.excl, lane <= j ? myidx : lo0 + ci * stride);
                tq.offer(mykey, myidx + sa.base_idx, ok);
                mykey = 0;
            }
            ++ci;
        }
    };
#pragma unroll
    for (int b = 0; b < NB - 1; ++b)
        if (ii < cnt) issue(buf[b]);
    while (ci < cnt) {
#pragma unroll
        for (int s = 0; s < NB; ++s) {  // compile-time ring slots: no register-array indexing
            if (ii < cnt) issue(buf[(s + NB - 1) % NB]);
            consume(buf[s]);
            if (ci >= cnt) break;
        }
    }
    block_merge_write<4>(tq, sm, q, wc + (int64_t)blockIdx.x * q, sa.nlists, nullptr, nullptr, 4, sa.ctr != nullptr);
    if (sa.ctr) fold_merge<4>(sa.ctr, sa.oval, sa.oidx, sa.ocand, q, wc, sm, sa.extra);
}

template <int DT, int NPL, bool VEC>
__global__ __launch_bounds__(kBS) void k_wide_entropy_v(WideArgs a, PwPlan pl, double* __restrict__ ent) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    const int w = threadIdx.x >> 6;
    double* row = wsm + w * wide_lds_doubles(a.C);
    double* scratch = row + a.C;
    for (int64_t i = (int64_t)blockIdx.x * 4 + w; i < a.N; i += (int64_t)gridDim.x * 4) {
        const double h = wide_item<DT, NPL, VEC>(a, pl, i, row, scratch);
        if ((threadIdx.x & 63) == 0) ent[i] = h;
    }
}

// ---------------------------------------------------------------------------
// Stage 2: merge `nl` lists of q slots (per segment = blockIdx.x) into top-q.
// A list's worst entry bounds the answer from below: with T = the best of the
// full lists' worst entries, at least q candidates are >= T, so only
// candidates >= T can be selected -- the filter is exact and usually leaves
// ~q survivors.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_best(uint64_t& k, int64_t& i) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t k2 = __shfl_xor(k, off);
        const int64_t i2 = __shfl_xor(i, off);
        if (better(k2, i2, k, i)) {
            k = k2;
            i = i2;
        }
    }
}

// ocand != nullptr: the top-q as candidate records instead of (val, idx).
template <bool FROM_VALS, int CAP, int BS, int IPT>
__global__ __launch_bounds__(BS) void k_finish(ListSrc<FROM_VALS> src, int nl, int q,
                                               double* __restrict__ oval, int64_t* __restrict__ oidx,
                                               Cand* __restrict__ ocand) {
    __shared__ TopQSmem<CAP> sm;
    __shared__ uint64_t wk[BS / 64];
    __shared__ int64_t wi[BS / 64];
    const int64_t seg0 = (int64_t)blockIdx.x * nl * q;
    const int64_t L = (int64_t)nl * q;
    // 1. T = best over FULL lists of the list's worst entry; lists are
    //    best-first, so a list is full iff slot q-1 is used and that slot is
    //    its worst entry: one load per list.
    uint64_t tk = 0;
    int64_t ti = INT64_MAX;  // "nothing": admits every candidate
    for (int g = threadIdx.x; g < nl; g += BS) {
        uint64_t k;
        int64_t i;
        src.get(seg0 + (int64_t)g * q + q - 1, k, i);
        if (i >= 0 && better(k, i, tk, ti)) {
            tk = k;
            ti = i;
        }
    }
    wave_best(tk, ti);
    if (lane_id() == 0) {
        wk[threadIdx.x >> 6] = tk;
        wi[threadIdx.x >> 6] = ti;
    }
    __syncthreads();
    tk = wk[0];
    ti = wi[0];
    for (int w = 1; w < BS / 64; ++w)
        if (better(wk[w], wi[w], tk, ti)) {
            tk = wk[w];
            ti = wi[w];
        }
    // admit candidates >= T: strictly better than (T.key, T.idx + 1)
    TopQ<CAP, BS> tq(sm);
    tq.init(tk, ti == INT64_MAX ? INT64_MAX : ti + 1);
    // 2. filter every candidate; IPT independent loads per thread in flight
    //    (addresses clamped, never a branch around a load)
    for (int64_t b0 = 0; b0 < L; b0 += (int64_t)BS * IPT) {
        uint64_t k[IPT];
        int64_t id[IPT];
#pragma unroll
        for (int u = 0; u < IPT; ++u) {
            int64_t j = b0 + (int64_t)u * BS + threadIdx.x;
            const bool in = j < L;
            src.get(seg0 + (in ? j : L - 1), k[u], id[u]);
            if (!in) id[u] = -1;
        }
#pragma unroll
        for (int u = 0; u < IPT; ++u) {
            if (b0 + (int64_t)u * BS >= L) break;  // block-uniform
            tq.offer(k[u], id[u], id[u] >= 0);
            tq.end_round(q, BS);
        }
    }
    const int cnt = tq.finish(q);
    const int64_t slot = (int64_t)blockIdx.x * q;
    if (ocand) write_list<CAP, false>(sm, cnt, q, ocand + slot, nullptr, nullptr);
    else write_list<CAP, true>(sm, cnt, q, nullptr, oval + slot, oidx + slot);
}

// Stage 2 for q <= kHeadsMaxQ (the common case, q = 10).  The lists are
// best-first, so list heads are each list's best entry; T1 = the q-th best
// head is an exact lower bound (q distinct lists hold an entry >= T1) and a
// tight one: the global top-q sit in ~q different lists, so only ~q
// candidates survive the filter.  Cost: one 1024-entry bitonic sort of the
// heads + one pass over the (prefetched) candidates + a tiny final sort.
constexpr int kHeadsBS = 1024;
constexpr int kHeadsMaxQ = 512;

template <bool FROM_VALS, int IPT>
__global__ __launch_bounds__(kHeadsBS) void k_finish_heads(ListSrc<FROM_VALS> src, int nl, int q,
                                                           double* __restrict__ oval, int64_t* __restrict__ oidx,
                                                           Cand* __restrict__ ocand) {
    __shared__ TopQSmem<2048> sm;
    const int64_t seg0 = (int64_t)blockIdx.x * nl * q;
    const int64_t L = (int64_t)nl * q;
    const int tid = threadIdx.x;
    // prefetch this thread's first IPT candidates (clamped, unconditional)
    uint64_t k[IPT];
    int64_t id[IPT];
#pragma unroll
    for (int u = 0; u < IPT; ++u) {
        const int64_t j = (int64_t)u * kHeadsBS + tid;
        src.get(seg0 + (j < L ? j : L - 1), k[u], id[u]);
        if (j >= L) id[u] = -1;
    }
    // best head among this thread's lists (distinct threads -> distinct lists)
    uint64_t hk = 0;
    int64_t hi = INT64_MAX;
    for (int g = tid; g < nl; g += kHeadsBS) {
        uint64_t kk;
        int64_t ii;
        src.get(seg0 + (int64_t)g * q, kk, ii);
        if (ii >= 0 && better(kk, ii, hk, hi)) {
            hk = kk;
            hi = ii;
        }
    }
    TopQ<2048, kHeadsBS> tq(sm);
    uint64_t tk = 0;
    int64_t ti = INT64_MAX;
    if (q <= kHeadsBS / 64) {
        // q <= 16: each wave's best head (shuffle reduction) comes from a list
        // of its own; the q-th best of those 16 is the bound.
        wave_best(hk, hi);
        const int w = tid >> 6;
        if ((tid & 63) == 0) {
            sm.key[w] = hk;
            sm.idx[w] = hi;
        }
        __syncthreads();
        if (tid < kHeadsBS / 64) {
            int rank = 0;
            for (int v = 0; v < kHeadsBS / 64; ++v) rank += better(sm.key[v], sm.idx[v], sm.key[tid], sm.idx[tid]);
            if (rank == q - 1) {
                sm.red[0] = sm.key[tid];
                sm.red[1] = (uint64_t)sm.idx[tid];
            }
        }
        __syncthreads();
        const int64_t t1 = (int64_t)sm.red[1];
        if (t1 != INT64_MAX) {  // >= q non-empty lists
            tk = sm.red[0];
            ti = t1 + 1;  // admit candidates >= T1
        }
    } else {
        sm.key[tid] = hk;
        sm.idx[tid] = hi;
        tq.sort_buffer(kHeadsBS);  // barrier inside, before the first compare
        __syncthreads();
        if (q <= kHeadsBS && sm.idx[q - 1] != INT64_MAX) {
            tk = sm.key[q - 1];
            ti = sm.idx[q - 1] + 1;
        }
    }
    __syncthreads();
    tq.init(tk, ti);
    for (int64_t b0 = 0; b0 < L; b0 += (int64_t)kHeadsBS * IPT) {
        if (b0 > 0) {
#pragma unroll
            for (int u = 0; u < IPT; ++u) {
                const int64_t j = b0 + (int64_t)u * kHeadsBS + tid;
                src.get(seg0 + (j < L ? j : L - 1), k[u], id[u]);
                if (j >= L) id[u] = -1;
            }
        }
#pragma unroll
        for (int u = 0; u < IPT; ++u) {
            if (b0 + (int64_t)u * kHeadsBS >= L) break;  // block-uniform
            tq.offer(k[u], id[u], id[u] >= 0);
            tq.end_round(q, kHeadsBS);
        }
    }
    const int cnt = tq.finish(q);
    const int64_t slot = (int64_t)blockIdx.x * q;
    if (ocand) write_list<2048, false>(sm, cnt, q, ocand + slot, nullptr, nullptr);
    else write_list<2048, true>(sm, cnt, q, nullptr, oval + slot, oidx + slot);
}

// Stage 2 for q <= 64.  The lists are best-first, so a list's head is its
// best entry.  Phase 1: each of the 16 waves sorts the heads of its share of
// the lists (one per lane) in registers; its q-th best head T_w is an exact
// lower bound (q distinct lists have an entry >= T_w), and so is T = the best
// T_w.  Phase 2: the waves stream all candidates (64 consecutive per wave per
// step, PF steps in flight) through register top-q lists floored at T -- only
// candidates >= T (~q of them) are ever inserted -- and the lists are
// tree-merged.  Output: final (val, idx), or candidate records (wc) for an
// exchange between ranks.
template <bool FROM_VALS>
__global__ __launch_bounds__(1024) void k_merge_reg(ListSrc<FROM_VALS> src, int nl, int q,
                                                    double* __restrict__ oval, int64_t* __restrict__ oidx,
                                                    Cand* __restrict__ ocand) {
    __shared__ WaveListsT<16> sm;
    __shared__ uint64_t bk[16];
    __shared__ int64_t bi[16];
    constexpr int PF = 10;  // 16 x 64 x 10: 1024 lists of q = 10 in one round of loads
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t seg0 = (int64_t)blockIdx.x * nl * q;
    const int64_t L = (int64_t)nl * q;
    CE_DASSERT(nl >= 1 && q >= 1 && q <= kStreamMaxQ);
    // the first round of candidate loads goes out before the head phase
    uint64_t k[PF];
    int64_t id[PF];
    auto load_round = [&](int64_t c0) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int64_t j = c0 + (int64_t)u * 16 * 64 + lane;
            src.get(seg0 + (j < L ? j : L - 1), k[u], id[u]);  // clamped: no branch around a load
            if (j >= L) id[u] = -1;
        }
    };
    load_round((int64_t)w * 64);
    // phase 1: the head bound (only worth a sort when there are many lists)
    uint64_t fk = 0;
    int64_t fi = INT64_MAX;
    if (nl > 64) {
        RegTopQ hq;
        hq.init(q);
        for (int g0 = w * 64; g0 < nl; g0 += 16 * 64) {
            const int g = g0 + lane;
            uint64_t hk = 0;
            int64_t hid = -1;
            src.get(seg0 + (int64_t)(g < nl ? g : nl - 1) * q, hk, hid);
            hq.offer(hk, hid, g < nl && hid >= 0);
        }
        const uint64_t qk = readlane64(hq.k, q - 1);
        const int64_t qi = (int64_t)readlane64((uint64_t)hq.i, q - 1);
        if (lane == 0) {
            bk[w] = qk;
            bi[w] = qi;
        }
        __syncthreads();
        for (int v = 0; v < 16; ++v)
            if (bi[v] != INT64_MAX && better(bk[v], bi[v], fk, fi)) {
                fk = bk[v];
                fi = bi[v];
            }
        if (fi != INT64_MAX) fi += 1;  // admit candidates >= T: strictly better than (T.key, T.idx + 1)
    }
    RegTopQ tq;
    tq.init(q, fk, fi);
    for (int64_t c0 = (int64_t)w * 64; c0 < L; c0 += (int64_t)16 * 64 * PF) {
        if (c0 != (int64_t)w * 64) load_round(c0);
#pragma unroll
        for (int u = 0; u < PF; ++u) tq.offer(k[u], id[u], id[u] >= 0);
    }
    const int64_t slot = (int64_t)blockIdx.x * q;
    if (ocand)
        block_merge_write<16>(tq, sm, q, ocand + slot, 0);
    else
        block_merge_write<16>(tq, sm, q, nullptr, 0, oval + slot, oidx + slot);
}

// Per-segment merge of a few lists (batched users: bpu lists of q each): one
// wave per segment streams its nl*q candidates through a register top-q.
template <bool FROM_VALS>
__global__ __launch_bounds__(256) void k_merge_wave(ListSrc<FROM_VALS> src, int segs, int nl, int q,
                                                    double* __restrict__ oval, int64_t* __restrict__ oidx) {
    const int seg = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (seg >= segs) return;  // wave-uniform; no block barrier below
    const int64_t L = (int64_t)nl * q, seg0 = (int64_t)seg * L;
    RegTopQ tq;
    tq.init(q);
    for (int64_t c0 = 0; c0 < L; c0 += 64) {
        const int64_t j = c0 + lane;
        uint64_t k;
        int64_t id;
        src.get(seg0 + (j < L ? j : L - 1), k, id);
        tq.offer(k, id, j < L && id >= 0);
    }
    if (lane < q) {
        const bool ok = tq.i != INT64_MAX;
        oval[(int64_t)seg * q + lane] = ok ? key_to_val(tq.k) : __longlong_as_double(0x7ff8000000000000ll);
        oidx[(int64_t)seg * q + lane] = ok ? tq.i : -1;
    }
}

// ---------------------------------------------------------------------------
// Per-item entropy to HBM.
// ---------------------------------------------------------------------------
template <class Src>
__global__ __launch_bounds__(kBS) void k_entropy(Src src, int64_t N, double* __restrict__ mean_out,
                                                 double* __restrict__ ent) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    constexpr int C = Src::kC;
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBS) {
        double mean[C];
        src.mean(i, mean);
        if (mean_out)
#pragma unroll
            for (int c = 0; c < C; ++c) mean_out[i * C + c] = mean[c];
        ent[i] = entropy_row<C>(mean);
    }
}

// ---------------------------------------------------------------------------
// hc tables: one wave per row (amg_test.py:109-117).
// ---------------------------------------------------------------------------
template <int C>
__device__ __forceinline__ void finish_counts(int (&cnt)[C], int64_t n_row, double* freq_out,
                                              double* ent) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) cnt[c] += __shfl_xor(cnt[c], off);
    if (lane_id() == 0) {
        int n = 0;
#pragma unroll
        for (int c = 0; c < C; ++c) n += cnt[c];
        double f[C];
#pragma unroll
        for (int c = 0; c < C; ++c) f[c] = round3((double)cnt[c] / (double)n);
        if (freq_out)
#pragma unroll
            for (int c = 0; c < C; ++c) freq_out[n_row * C + c] = f[c];
        ent[n_row] = entropy_row<C>(f);
    }
}

template <int C>
__global__ __launch_bounds__(kBS) void k_vote(const int8_t* __restrict__ votes, int64_t N, int A, int64_t ld,
                                              double* __restrict__ freq, double* __restrict__ ent) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    const int lane = lane_id();
    for (int64_t n = (int64_t)blockIdx.x * (kBS / 64) + (threadIdx.x >> 6); n < N;
         n += (int64_t)gridDim.x * (kBS / 64)) {
        int cnt[C];
#pragma unroll
        for (int c = 0; c < C; ++c) cnt[c] = 0;
        const int8_t* row = votes + n * ld;
        for (int a = lane; a < A; a += 64) {
            const int v = row[a];
#pragma unroll
            for (int c = 0; c < C; ++c) cnt[c] += (v == c);
        }
        finish_counts<C>(cnt, n, freq, ent);
    }
}

// ---------------------------------------------------------------------------
// Frame -> song segment mean: pd.DataFrame(y_probs, index=X_train.index)
// .groupby(['s_id']).mean() (amg_test.py:437, :469) as pandas 1.1.5's
// group_mean computes it (the reference pins pandas==1.1.5): values upcast to
// f64, per (song, class) a sequential sum over the song's frames in row order
// skipping NaN, divided by the non-NaN count (0 -> NaN); a float32 column is
// cast back to float32 at the end (the result dtype follows the input).
// One thread per (song, class); frames of song n are rows perm[off[n]..off[n+1])
// (perm == nullptr: rows off[n]..off[n+1] themselves, already grouped).
// ---------------------------------------------------------------------------
template <int DT, int ODT>
__global__ __launch_bounds__(kBS) void k_segment_mean(const void* __restrict__ frames, int64_t ld, int C,
                                                      const int64_t* __restrict__ perm,
                                                      const int64_t* __restrict__ offsets, int64_t N,
                                                      void* __restrict__ out, int64_t ldo) {
    const int64_t total = N * C;
    for (int64_t t = (int64_t)blockIdx.x * kBS + threadIdx.x; t < total; t += (int64_t)gridDim.x * kBS) {
        const int64_t n = t / C;
        const int c = (int)(t - n * C);
        const int64_t f0 = offsets[n], f1 = offsets[n + 1];
        CE_DASSERT(f0 >= 0 && f0 <= f1);
        double sum = 0.0;
        int64_t cnt = 0;
        // batches of 8 frames: the 8 loads are issued together (clamped rows,
        // no branch around a load), then added in row order
        constexpr int B = 8;
        for (int64_t fb = f0; fb < f1; fb += B) {
            double v[B];
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const int64_t f = fb + u < f1 ? fb + u : f1 - 1;
                const int64_t r = perm ? perm[f] : f;
                if constexpr (DT == kF32)
                    v[u] = (double)static_cast<const float*>(frames)[r * ld + c];
                else
                    v[u] = static_cast<const double*>(frames)[r * ld + c];
            }
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (fb + u < f1 && v[u] == v[u]) {  // not NaN
                    sum += v[u];
                    ++cnt;
                }
        }
        double m = cnt ? sum / (double)cnt : __longlong_as_double(0x7ff8000000000000ll);
        if constexpr (DT == kF32) m = (double)(float)m;  // the float32 result column
        if constexpr (ODT == kF32)
            static_cast<float*>(out)[n * ldo + c] = (float)m;
        else
            static_cast<double*>(out)[n * ldo + c] = m;
    }
}

}  // namespace ce
