// ce_kernels.hip -- MI355X (gfx950) kernels and the C-ABI of include/ce.h.
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
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};

template <int DT, int C, bool VEC>
struct CommitteeSrc {
    const void* p;
    int64_t sN, sM, sC;
    int M;
    double dM, invM;
    bool pow2;
    static constexpr int kC = C;
    static constexpr int kDT = DT;
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
    // keys() for latency-bound single-block pools: when the whole committee
    // fits one batch (M <= UNR) the loads are issued item by item and each
    // item's mean + entropy runs as soon as ITS loads have landed, so only the
    // last item's arithmetic trails the last load.  Items u >= nlive (wave-
    // uniform: no lane of the wave owns a real item there) skip the arithmetic
    // (key 0).  hook() as in keys().
    template <int UNR, int IPL, class Hook = NoHook>
    __device__ __forceinline__ void keys_small(const int64_t (&items)[IPL], uint64_t (&k)[IPL], int nlive,
                                               Hook hook = {}) const {
        if (M > UNR) {
            keys<UNR, IPL>(items, k, hook);
            return;
        }
        MemberLoad<DT, C, VEC> ld[IPL][UNR];
#pragma unroll
        for (int u = 0; u < IPL; ++u)
#pragma unroll
            for (int v = 0; v < UNR; ++v) ld[u][v].load(p, items[u] * sN + (int64_t)(v < M ? v : M - 1) * sM, sC);
        hook();
        auto item = [&](auto full) {
#pragma unroll
            for (int u = 0; u < IPL; ++u) {
                k[u] = 0;
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
                k[u] = order_key(entropy_row<C>(m));
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
    int64_t s0, lo, hi;
    seg_range(sg, s0, lo, hi);
    const int64_t rel = sg.base_idx - s0;
    for (int64_t i0 = lo; i0 < hi; i0 += kBS) {
        const int64_t i = i0 + threadIdx.x;
        const bool valid = i < hi;
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
        tq.offer(mykey, i + rel, i < hi);
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
template <int DT, int KCH, int UNR>
__global__ __launch_bounds__(kBS) void k_stream_wide2(WideArgs a, PwPlan pl, StreamArgs sa, int q,
                                                      Cand* __restrict__ wc) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    __shared__ WaveLists sm;
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    constexpr int CPC = ChunkT<DT>::CPC, EB = 16 / CPC;
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
    const char* base = static_cast<const char*>(a.p);
    const int64_t sNb = a.sN * EB, sMb = a.sM * EB;
    const int K = a.C / CPC;
    const int NB = a.M / UNR;  // UNR divides M (host)
    double acc[KCH * CPC];
#pragma unroll
    for (int e = 0; e < KCH * CPC; ++e) acc[e] = 0.0;
    uint64_t mykey = 0;
    // issue cursor (item, batch) and consume cursor
    int64_t ii = lo, ci = lo;
    int ib = 0, cb = 0;
    uint32_t off[KCH];  // this lane's chunk offsets in a member row (clamped into the row)
#pragma unroll
    for (int kk = 0; kk < KCH; ++kk) {
        const int ch = lane + 64 * kk;
        off[kk] = 16u * (uint32_t)(ch < K ? ch : K - 1);
    }
    WideBatch<DT, KCH, UNR> A, B;
    auto issue = [&](WideBatch<DT, KCH, UNR>& X) {
        X.issue(base + ii * sNb, ib * UNR, sMb, off);
        if (++ib == NB) {
            ib = 0;
            ++ii;
        }
    };
    auto consume = [&](const WideBatch<DT, KCH, UNR>& X) {
        X.add(acc);
        if (++cb == NB) {  // item ci complete
            cb = 0;
            const double h = wave_entropy_from_sums<DT, KCH>(acc, K, a.dM, a.invM, a.pow2, pl, row, scratch);
#pragma unroll
            for (int e = 0; e < KCH * CPC; ++e) acc[e] = 0.0;
            const int j = (int)((ci - lo) & 63);
            if (lane == j) mykey = order_key(h);
            if (j == 63 || ci == hi - 1) {
                const int64_t t0 = ci - j;
                bool ok = lane <= j;
                if (sa.excl) ok = ok && !excluded(sa.excl, t0 + (lane <= j ? lane : j));
                tq.offer(mykey, t0 + lane + sa.base_idx, ok);
                mykey = 0;
            }
            ++ci;
        }
    };
    if (ii < hi) issue(A);
    while (ci < hi) {
        if (ii < hi) issue(B);
        consume(A);
        if (ci >= hi) break;
        if (ii < hi) issue(A);
        consume(B);
    }
    block_merge_write<4>(tq, sm, q, wc + (int64_t)blockIdx.x * q, sa.nlists);
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
template <bool FROM_VALS>
struct ListSrc {
    const Cand* c;
    const double* val;
    const int64_t* idx;
    __device__ __forceinline__ void get(int64_t j, uint64_t& k, int64_t& i) const {
        if constexpr (FROM_VALS) {
            i = idx[j];
            k = order_key(val[j]);
        } else {
            const Cand x = c[j];
            k = x.key;
            i = x.idx;
        }
    }
};

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

template <bool FROM_VALS, int CAP, int BS, int IPT>
__global__ __launch_bounds__(BS) void k_finish(ListSrc<FROM_VALS> src, int nl, int q,
                                               double* __restrict__ oval, int64_t* __restrict__ oidx) {
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
    write_list<CAP, true>(sm, cnt, q, nullptr, oval + (int64_t)blockIdx.x * q, oidx + (int64_t)blockIdx.x * q);
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
                                                           double* __restrict__ oval, int64_t* __restrict__ oidx) {
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
    write_list<2048, true>(sm, cnt, q, nullptr, oval + (int64_t)blockIdx.x * q, oidx + (int64_t)blockIdx.x * q);
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

// glibc log over a vector (verification of ce_glibc_log.hpp against libm).
__global__ __launch_bounds__(kBS) void k_log(const double* __restrict__ x, int64_t n, double* __restrict__ y) {
    stage_log_table();
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) y[i] = dlog(x[i]);
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

__global__ __launch_bounds__(kBS) void k_va(const double* __restrict__ va, int64_t N, int A,
                                            double* __restrict__ freq, double* __restrict__ ent) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    const int lane = lane_id();
    for (int64_t n = (int64_t)blockIdx.x * (kBS / 64) + (threadIdx.x >> 6); n < N;
         n += (int64_t)gridDim.x * (kBS / 64)) {
        int cnt[4] = {0, 0, 0, 0};
        const double2* row = reinterpret_cast<const double2*>(va) + n * A;
        for (int a = lane; a < A; a += 64) {
            const double2 x = row[a];  // (valence, arousal)
            const int qd = quadrant(x.y, x.x);
#pragma unroll
            for (int c = 0; c < 4; ++c) cnt[c] += (qd == c);
        }
        finish_counts<4>(cnt, n, freq, ent);
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

// ===========================================================================
// Host side: argument checks, geometry, dispatch, C-ABI.
// ===========================================================================
using namespace ce;

static thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(CE_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    g_err[0] = 0;
    return CE_OK;
}

extern "C" const char* ce_last_error(void) { return g_err; }
extern "C" const char* ce_version(void) { return "ce_amd 0.1 gfx950"; }

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// stage-1 blocks for a pool of n items (host arithmetic only: ws sizing and
// launches agree by construction)
static int pool_blocks(int64_t n) {
    // one 64-item tile per wave at least; up to 1024 blocks (4 per CU), so wide
    // items (tens of KB each) still fill the chip
    int64_t g = cdiv(n, (int64_t)kMinItemsPerBlock);
    if (g < 1) g = 1;
    if (g > kMaxBlocks) g = kMaxBlocks;
    return (int)g;
}

static size_t lists_bytes(int64_t nlists, int q) { return (size_t)nlists * (size_t)q * 16u + 256u; }

struct WsLists {
    Cand* c;
};
static WsLists carve(void* ws, int64_t nlists, int q) {
    uintptr_t p = ((uintptr_t)ws + 255) & ~(uintptr_t)255;
    WsLists w;
    w.c = reinterpret_cast<Cand*>(p);
    return w;
}

static int check_q(int q) {
    if (q < 1 || q > CE_MAX_Q) return fail(CE_EINVAL, "q=%d outside [1, %d]", q, CE_MAX_Q);
    return CE_OK;
}

template <class Src>
static void launch_partial(const Src& src, const Seg& sg, int grid, int q, WsLists w, double* oval,
                           int64_t* oidx, bool final_out, hipStream_t st) {
    if (q <= 256) {
        if (final_out)
            hipLaunchKernelGGL((k_partial<Src, 1024, true>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
        else
            hipLaunchKernelGGL((k_partial<Src, 1024, false>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
    } else {
        if (final_out)
            hipLaunchKernelGGL((k_partial<Src, 4096, true>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
        else
            hipLaunchKernelGGL((k_partial<Src, 4096, false>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
    }
}

// A/B knob: CE_AMD_MERGE_REG=0 -> the LDS-buffer merges (k_finish / k_finish_heads) for q <= 64 too
static bool merge_reg_enabled() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_MERGE_REG");
        return !(e && e[0] == '0');
    }();
    return on;
}

// ocand != nullptr: write candidate records (q <= kStreamMaxQ only) instead of (val, idx).
template <bool FROM_VALS>
static void launch_finish(ListSrc<FROM_VALS> src, int segments, int nl, int q, double* oval, int64_t* oidx,
                          hipStream_t st, Cand* ocand = nullptr) {
    const int64_t L = (int64_t)nl * q;
    if (q <= kStreamMaxQ && (merge_reg_enabled() || ocand)) {
        hipLaunchKernelGGL((k_merge_reg<FROM_VALS>), dim3(segments), dim3(1024), 0, st, src, nl, q, oval, oidx,
                           ocand);
        return;
    }
    if (q <= kHeadsMaxQ && L > 256) {
        hipLaunchKernelGGL((k_finish_heads<FROM_VALS, 10>), dim3(segments), dim3(kHeadsBS), 0, st, src, nl, q, oval,
                           oidx);
        return;
    }
    if (L <= 256 && q <= 128)
        hipLaunchKernelGGL((k_finish<FROM_VALS, 512, 256, 1>), dim3(segments), dim3(256), 0, st, src, nl, q, oval,
                           oidx);
    else if (L <= 4096 && q <= 512)
        hipLaunchKernelGGL((k_finish<FROM_VALS, 2048, 256, 16>), dim3(segments), dim3(256), 0, st, src, nl, q, oval,
                           oidx);
    else
        hipLaunchKernelGGL((k_finish<FROM_VALS, 4096, kFinBS, 16>), dim3(segments), dim3(kFinBS), 0, st, src, nl,
                           q, oval, oidx);
}

// ---- committee dispatch ----------------------------------------------------
struct CommArgs {
    const void* p;
    int dt;
    int64_t N;
    int M, C;
    int64_t sN, sM, sC;
};

static int check_comm(const CommArgs& a) {
    if (!a.p && a.N > 0) return fail(CE_EINVAL, "null committee pointer");
    if (a.N < 0 || a.M < 1 || a.C < 1) return fail(CE_EINVAL, "bad shape N=%lld M=%d C=%d", (long long)a.N, a.M, a.C);
    if (a.dt < 0 || a.dt > 2) return fail(CE_EINVAL, "bad dtype %d", a.dt);
    return CE_OK;
}

static int elem_bytes(int dt) { return dt == kF64 ? 8 : (dt == kF32 ? 4 : 2); }

static bool vec_ok(const CommArgs& a, int C) {
    if (a.sC != 1) return false;
    const int eb = elem_bytes(a.dt);
    const int vb = a.dt == kBF16 ? 8 : 16;  // bytes per vector load
    if (a.dt == kF64 ? (C % 2) : (C % 4)) return false;
    if ((uintptr_t)a.p % vb) return false;
    if ((a.sN * eb) % vb || (a.sM * eb) % vb) return false;
    return true;
}

template <int DT, int C, bool VEC>
static CommitteeSrc<DT, C, VEC> make_src(const CommArgs& a) {
    CommitteeSrc<DT, C, VEC> s;
    s.p = a.p;
    s.sN = a.sN;
    s.sM = a.sM;
    s.sC = a.sC;
    s.M = a.M;
    s.dM = (double)a.M;
    s.invM = 1.0 / (double)a.M;
    s.pow2 = (a.M & (a.M - 1)) == 0;
    return s;
}

// Calls f(src) with the CommitteeSrc instantiation matching (dtype, C, vec).
template <class F>
static int with_committee(const CommArgs& a, F&& f) {
#define CE_CASE(DT_, C_)                                       \
    if (a.dt == DT_ && a.C == C_) {                            \
        if (vec_ok(a, C_)) f(make_src<DT_, C_, true>(a));      \
        else f(make_src<DT_, C_, false>(a));                   \
        return CE_OK;                                          \
    }
    CE_CASE(kF32, 4) CE_CASE(kF64, 4) CE_CASE(kBF16, 4)
    CE_CASE(kF32, 8) CE_CASE(kF64, 8) CE_CASE(kBF16, 8)
    CE_CASE(kF64, 2)
#undef CE_CASE
#define CE_CASE_S(DT_, C_)                                     \
    if (a.dt == DT_ && a.C == C_) {                            \
        f(make_src<DT_, C_, false>(a));                        \
        return CE_OK;                                          \
    }
    CE_CASE_S(kF32, 2) CE_CASE_S(kBF16, 2)
    CE_CASE_S(kF32, 3) CE_CASE_S(kF64, 3) CE_CASE_S(kBF16, 3)
#undef CE_CASE_S
    return CE_EUNSUPPORTED;
}

// ---- wide-class dispatch (C not in the register-path set) -------------------
static WideArgs wide_args(const CommArgs& a) {
    WideArgs w{a.p, a.N, a.M, a.C, a.sN, a.sM, a.sC, (double)a.M, 1.0 / (double)a.M, (a.M & (a.M - 1)) == 0};
    return w;
}
static size_t wide_lds_bytes(int C) { return (size_t)4 * wide_lds_doubles(C) * sizeof(double); }

static bool wide_vec_ok(const CommArgs& a) {
    const int eb = elem_bytes(a.dt);
    return a.sC == 1 && (a.C * eb) % 16 == 0 && (a.sM * eb) % 16 == 0 && (a.sN * eb) % 16 == 0 &&
           (uintptr_t)a.p % 16 == 0;
}

// f(dt, npl, vec) with compile-time values
template <class F>
static int with_wide_v(const CommArgs& a, F&& f) {
    if (a.C > kWideMaxC) return CE_EUNSUPPORTED;
    const bool vec = wide_vec_ok(a);
#define CE_WV(DT_, NPL_)                                                                              \
    if (vec) f(std::integral_constant<int, DT_>(), std::integral_constant<int, NPL_>(), std::true_type()); \
    else f(std::integral_constant<int, DT_>(), std::integral_constant<int, NPL_>(), std::false_type());
#define CE_WD(DT_)                                   \
    if (a.dt == DT_) {                               \
        if (a.C <= 512) { CE_WV(DT_, 8) }            \
        else if (a.C <= 1024) { CE_WV(DT_, 16) }     \
        else { CE_WV(DT_, 32) }                      \
        return CE_OK;                                \
    }
    CE_WD(kF32) CE_WD(kF64) CE_WD(kBF16)
#undef CE_WD
#undef CE_WV
    return CE_EUNSUPPORTED;
}

static void launch_partial_wide(const CommArgs& a, const Seg& sg, int grid, int q, WsLists w, double* oval,
                                int64_t* oidx, bool fin, hipStream_t st) {
    const WideArgs wa = wide_args(a);
    const PwPlan pl = pw_plan(a.C);
    const size_t lds = wide_lds_bytes(a.C);
    with_wide_v(a, [&](auto dt, auto npl, auto vec) {
        constexpr int DT = decltype(dt)::value, NPL = decltype(npl)::value;
        constexpr bool VEC = decltype(vec)::value;
        if (q <= 256) {
            if (fin)
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 1024, true>), dim3(grid), dim3(kBS), lds, st, wa, pl,
                                   sg, q, w.c, oval, oidx);
            else
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 1024, false>), dim3(grid), dim3(kBS), lds, st, wa,
                                   pl, sg, q, w.c, oval, oidx);
        } else {
            if (fin)
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 4096, true>), dim3(grid), dim3(kBS), lds, st, wa, pl,
                                   sg, q, w.c, oval, oidx);
            else
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 4096, false>), dim3(grid), dim3(kBS), lds, st, wa,
                                   pl, sg, q, w.c, oval, oidx);
        }
    });
}

// ---- streaming stage 1 (q <= 64): wave-independent, LDS-DMA for item-major ----
static bool stream_enabled() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_STREAM");  // A/B knob: CE_AMD_STREAM=0 -> block-synchronous k_partial
        return !(e && e[0] == '0');
    }();
    return on;
}

// Cache policy of the item-major LDS-DMA stream: nt (default) or the default
// policy (A/B knob CE_AMD_DMA_NT=0).
static bool dma_nt() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_DMA_NT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B knob: CE_AMD_WIDE2=0 -> the unpipelined wide kernel (k_stream_wide)
static bool wide2_enabled() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_WIDE2");
        return !(e && e[0] == '0');
    }();
    return on;
}

// (UNR members x IPL items) loads in flight per lane for the direct paths:
// small committees batch items, large ones batch members.
template <class Src, class F>
static void with_batching(int M, F&& f) {
    if constexpr (Src::kDT == kF64 || Src::kC > 4) {
        (void)M;
        f(std::integral_constant<int, 4>(), std::integral_constant<int, 2>());
    } else {
        if (M <= 4) f(std::integral_constant<int, 4>(), std::integral_constant<int, 4>());
        else f(std::integral_constant<int, 8>(), std::integral_constant<int, 2>());
    }
}

// The same for k_stream_seg: up to 16-wave blocks (<= 128 VGPRs), so fewer loads per lane.
template <class Src, class F>
static void with_seg_batching(F&& f) {
    if constexpr (Src::kC > 4) f(std::integral_constant<int, 4>(), std::integral_constant<int, 1>());
    else f(std::integral_constant<int, 4>(), std::integral_constant<int, 2>());
}

// Single-block pools (k_select_small): IPT items per thread (2 for C = 8
// rows), UNR member loads per item in flight (f64 / C = 8 rows are twice as
// wide: 2).  Returns false (nothing launched) when the pool exceeds BS * IPT.
constexpr int kSmallBS = 512;       // batched users: 2 blocks per CU, all 500 users resident
constexpr int kSmallBSWide = 1024;  // one pool of up to 4096 items
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
static void launch_small_mix(const SrcA& a, const SrcB& b, int64_t n, int64_t nB, int q, double* oval,
                             int64_t* oidx, hipStream_t st) {
    constexpr int UNRA = (SrcA::kDT == kF64 || SrcA::kC > 4) ? 2 : 4;
    hipLaunchKernelGGL((k_select_small<SrcA, SrcB, 2, 2, UNRA, 1, kSmallBSWide>), dim3(1), dim3(kSmallBSWide), 0, st, a,
                       b, (const int64_t*)nullptr, n, nB, (int64_t)0, q, oval, oidx, (const uint32_t*)nullptr);
}
static bool small_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("CE_AMD_SMALL");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

// Blocks of `kernel` resident on the whole device (occupancy API x CUs), cached.
static int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

template <class K>
static int resident_grid(K kernel, size_t dyn_lds, int cap) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, dyn_lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    (void)hipGetLastError();
    const int g = per_cu * device_cus();
    return g < cap ? g : cap;
}

static StreamArgs stream_args(const CommArgs& a, int G, int64_t base_idx) {
    StreamArgs s;
    s.p = a.p;
    s.N = a.N;
    s.M = a.M;
    s.sN = a.sN;
    s.sM = a.sM;
    s.sC = a.sC;
    s.dM = (double)a.M;
    s.invM = 1.0 / (double)a.M;
    s.pow2 = (a.M & (a.M - 1)) == 0;
    s.base_idx = base_idx;
    s.nlists = G;
    s.per_wave = 0;
    s.excl = nullptr;
    return s;
}

// the grid actually launched (<= G workspace lists) and its per-wave share
static void stream_grid(StreamArgs& s, int grid) {
    const int64_t W = (int64_t)grid * 4;
    s.per_wave = (cdiv(s.N, W) + 63) / 64 * 64;
}

// Launches the streaming kernel when it applies; returns false otherwise.
static bool launch_stream(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
                          const uint32_t* excl = nullptr) {
    if (!stream_enabled() || q > kStreamMaxQ || a.N == 0) return false;
    StreamArgs sa = stream_args(a, G, base_idx);
    sa.excl = excl;
    const int eb = elem_bytes(a.dt);
    const int64_t R = (int64_t)a.M * a.C * eb;
    const bool dense_nmc = a.sC == 1 && a.sM == a.C && a.sN == (int64_t)a.M * a.C && (uintptr_t)a.p % 16 == 0;
    if (dense_nmc && (R == 256 || R == 512)) {
#define CE_S(DT_, C_, S_)                                                                                   \
    if (a.dt == DT_ && a.C == C_ && R == 16 * S_) {                                                       \
        auto kern = dma_nt() ? k_stream_nmc<DT_, C_, S_, 2> : k_stream_nmc<DT_, C_, S_, 0>;              \
        const int grid = resident_grid(kern, 0, G);                                                       \
        stream_grid(sa, grid);                                                                            \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, sa, q, w.c);                               \
        return true;                                                                                      \
    }
        CE_S(kF32, 4, 16) CE_S(kF32, 4, 32) CE_S(kBF16, 4, 16) CE_S(kBF16, 4, 32) CE_S(kF64, 4, 32)
        CE_S(kF32, 8, 16) CE_S(kF32, 8, 32)
#undef CE_S
    }
    int rc = with_committee(a, [&](auto src) {
        using S = decltype(src);
        with_batching<S>(a.M, [&](auto unr, auto ipl) {
            auto kern = k_stream_direct<S, decltype(ipl)::value, decltype(unr)::value>;
            const int grid = resident_grid(kern, 0, G);
            stream_grid(sa, grid);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, src, sa, q, w.c);
        });
    });
    if (rc == CE_OK) return true;
    const WideArgs wa = wide_args(a);
    const PwPlan pl = pw_plan(a.C);
    const size_t lds = wide_lds_bytes(a.C);
    int rc_excl = CE_OK;
    rc = with_wide_v(a, [&](auto dt, auto npl, auto vec) {
        constexpr int DT = decltype(dt)::value, NPL = decltype(npl)::value;
        if constexpr (decltype(vec)::value) {
            if (wide2_enabled()) {
                constexpr int KCH = NPL / ChunkT<DT>::CPC > 0 ? NPL / ChunkT<DT>::CPC : 1;
                // member rows per batch: 4 / KCH (>= 1), or 1 when that does not divide M
                constexpr int UNR = KCH >= 4 ? 1 : 4 / KCH;
                auto kern = (a.M % UNR == 0) ? k_stream_wide2<DT, KCH, UNR> : k_stream_wide2<DT, KCH, 1>;
                const int grid = resident_grid(kern, lds, G);
                stream_grid(sa, grid);
                sa.per_wave = cdiv(a.N, (int64_t)grid * 4);  // whole items, not 64-item tiles
                hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, wa, pl, sa, q, w.c);
                return;
            }
        }
        if (sa.excl) {  // k_stream_wide takes no bitmap
            rc_excl = CE_EUNSUPPORTED;
            return;
        }
        auto kern = k_stream_wide<DT, NPL, decltype(vec)::value>;
        const int grid = resident_grid(kern, lds, G);
        stream_grid(sa, grid);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, wa, pl, sa, q, w.c);
    });
    return rc == CE_OK && rc_excl == CE_OK;
}

// Committee stage 1 for any supported shape: register path or wide path.
static int committee_partial(const CommArgs& a, const Seg& sg, int grid, int q, WsLists w, double* oval,
                             int64_t* oidx, bool fin, hipStream_t st) {
    int rc = with_committee(a, [&](auto src) { launch_partial(src, sg, grid, q, w, oval, oidx, fin, st); });
    if (rc != CE_EUNSUPPORTED) return rc;
    if (a.C > kWideMaxC) return CE_EUNSUPPORTED;
    launch_partial_wide(a, sg, grid, q, w, oval, oidx, fin, st);
    return CE_OK;
}

// ===========================================================================
// C-ABI
// ===========================================================================
static int dispatch_err(int rc, const CommArgs& a) {
    if (rc == CE_EUNSUPPORTED)
        return fail(CE_EUNSUPPORTED, "committee shape C=%d dtype=%d has no kernel in this build", a.C, a.dt);
    return rc;
}

extern "C" int ce_committee_entropy(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                    int64_t sM, int64_t sC, double* mean_or_null, double* ent,
                                    ce_stream_t stream) {
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int rc = check_comm(a);
    if (rc) return rc;
    if (!ent) return fail(CE_EINVAL, "null ent");
    if (N == 0) return CE_OK;
    hipStream_t st = (hipStream_t)stream;
    const int grid = (int)std::min<int64_t>(cdiv(N, kBS), 4096);
    rc = with_committee(a, [&](auto src) {
        hipLaunchKernelGGL((k_entropy<decltype(src)>), dim3(grid), dim3(kBS), 0, st, src, N, mean_or_null, ent);
    });
    if (rc == CE_EUNSUPPORTED) {
        const WideArgs wa = wide_args(a);
        const PwPlan pl = pw_plan(C);
        const size_t lds = wide_lds_bytes(C);
        const int wgrid = (int)std::min<int64_t>(cdiv(N, 4), 8192);
        if (mean_or_null) return fail(CE_EUNSUPPORTED, "mean output for C=%d is not implemented", C);
        rc = with_wide_v(a, [&](auto dt, auto npl, auto vec) {
            hipLaunchKernelGGL((k_wide_entropy_v<decltype(dt)::value, decltype(npl)::value, decltype(vec)::value>),
                               dim3(wgrid), dim3(256), lds, st, wa, pl, ent);
        });
    }
    if (rc) return dispatch_err(rc, a);
    return check_launch("ce_committee_entropy");
}

#ifdef CE_PHASE_TIMING
extern "C" int ce_debug_phase(uint64_t* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), (size_t)n * 6 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int ce_log_f64(const double* x, int64_t n, double* y, ce_stream_t stream) {
    if (n < 0 || (n > 0 && (!x || !y))) return fail(CE_EINVAL, "bad log arguments");
    if (n == 0) return CE_OK;
    const int grid = (int)std::min<int64_t>(cdiv(n, kBS), 8192);
    hipLaunchKernelGGL(k_log, dim3(grid), dim3(kBS), 0, (hipStream_t)stream, x, n, y);
    return check_launch("ce_log_f64");
}

extern "C" int ce_log_f64_host(const double* x, int64_t n, double* y) {
    if (n < 0 || (n > 0 && (!x || !y))) return fail(CE_EINVAL, "bad log arguments");
    const LogEntry* tab = host_log_table();
    for (int64_t i = 0; i < n; ++i) y[i] = glibc_log_fast(x[i], tab);
    return CE_OK;
}

extern "C" int ce_vote_entropy(const int8_t* votes, int64_t N, int32_t A, int32_t C, int64_t ld,
                               double* freq_or_null, double* ent, ce_stream_t stream) {
    if (N < 0 || A < 0 || ld < A) return fail(CE_EINVAL, "bad vote matrix N=%lld A=%d ld=%lld", (long long)N, A, (long long)ld);
    if (!ent || (N > 0 && !votes)) return fail(CE_EINVAL, "null pointer");
    if (N == 0) return CE_OK;
    hipStream_t st = (hipStream_t)stream;
    const int grid = (int)std::min<int64_t>(cdiv(N, kBS / 64), 8192);
    switch (C) {
#define CE_V(CC) case CC: hipLaunchKernelGGL((k_vote<CC>), dim3(grid), dim3(kBS), 0, st, votes, N, A, ld, freq_or_null, ent); break;
        CE_V(1) CE_V(2) CE_V(3) CE_V(4) CE_V(5) CE_V(6) CE_V(7) CE_V(8)
#undef CE_V
        default: return fail(CE_EUNSUPPORTED, "vote classes C=%d outside [1, 8]", C);
    }
    return check_launch("ce_vote_entropy");
}

extern "C" int ce_va_entropy(const double* va, int64_t N, int32_t A, double* freq_or_null, double* ent,
                             ce_stream_t stream) {
    if (N < 0 || A < 0) return fail(CE_EINVAL, "bad annotation array");
    if (!ent || (N > 0 && !va)) return fail(CE_EINVAL, "null pointer");
    if ((uintptr_t)va % 16) return fail(CE_EINVAL, "va must be 16-byte aligned");
    if (N == 0) return CE_OK;
    hipStream_t st = (hipStream_t)stream;
    const int grid = (int)std::min<int64_t>(cdiv(N, kBS / 64), 8192);
    hipLaunchKernelGGL(k_va, dim3(grid), dim3(kBS), 0, st, va, N, A, freq_or_null, ent);
    return check_launch("ce_va_entropy");
}

// ---- frame -> song segment mean (amg_test.py:437, :469) ----------------------
extern "C" int ce_segment_mean(const void* frames, ce_dtype dt, int64_t F, int32_t C, int64_t ld,
                               const int64_t* perm_or_null, const int64_t* offsets, int64_t N, void* out,
                               ce_dtype out_dt, int64_t ld_out, ce_stream_t stream) {
    if (F < 0 || N < 0 || C < 1 || ld < C || ld_out < C) return fail(CE_EINVAL, "bad segment-mean shape");
    if ((N > 0 && (!offsets || !out)) || (F > 0 && !frames)) return fail(CE_EINVAL, "null pointer");
    if ((dt != CE_F32 && dt != CE_F64) || (out_dt != CE_F32 && out_dt != CE_F64))
        return fail(CE_EUNSUPPORTED, "segment mean takes float32/float64 frames and outputs");
    if (N == 0) return CE_OK;
    hipStream_t st = (hipStream_t)stream;
    const int grid = (int)std::min<int64_t>(cdiv(N * C, kBS), 8192);
#define CE_SM(D_, O_)                                                                                        \
    if (dt == D_ && out_dt == O_)                                                                            \
        hipLaunchKernelGGL((k_segment_mean<D_, O_>), dim3(grid), dim3(kBS), 0, st, frames, ld, C, perm_or_null, \
                           offsets, N, out, ld_out);
    CE_SM(CE_F32, CE_F32) CE_SM(CE_F32, CE_F64) CE_SM(CE_F64, CE_F32) CE_SM(CE_F64, CE_F64)
#undef CE_SM
    return check_launch("ce_segment_mean");
}

// ---- exclusion bitmaps (SelectionSession) -----------------------------------
__global__ void k_mark(uint32_t* __restrict__ bits, int64_t N, const int64_t* __restrict__ idx, int n,
                       int64_t base_idx) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const int64_t p = idx[t] - base_idx;
        if (idx[t] >= 0 && p >= 0 && p < N) atomicOr(&bits[p >> 5], 1u << (p & 31));
    }
}

extern "C" int ce_mark_selected(uint32_t* excl, int64_t N, const int64_t* idx, int32_t n, int64_t base_idx,
                                ce_stream_t stream) {
    if (N < 0 || n < 0 || (N > 0 && !excl) || (n > 0 && !idx)) return fail(CE_EINVAL, "bad mark arguments");
    if (n == 0 || N == 0) return CE_OK;
    hipLaunchKernelGGL(k_mark, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, excl, N, idx, n, base_idx);
    return check_launch("ce_mark_selected");
}

// ---- committee member inference ---------------------------
// features per lane of the 8-lanes-per-frame kernels: ceil(D / 8), rounded up to a multiple of 8
template <class F>
static int with_nx(int D, F&& f) {
    const int nx = (D + 7) / 8;
#define CE_NX(N_) if (nx <= N_) { f(std::integral_constant<int, N_>()); return CE_OK; }
    CE_NX(8) CE_NX(16) CE_NX(24) CE_NX(32) CE_NX(36) CE_NX(40) CE_NX(48) CE_NX(56) CE_NX(64)
#undef CE_NX
    return CE_EUNSUPPORTED;
}

// >= ~8 eight-frame passes per wave, so each block's LDS staging is amortised
static int member_grid8(int64_t F) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(F, 256), 2048)); }

extern "C" int ce_gnb_predict_proba(const double* X, int64_t F, int32_t D, int64_t ld, const double* theta,
                                    const double* var, const double* log_prior, int32_t C, double* out,
                                    int64_t ld_out, ce_stream_t stream) {
    if (F < 0 || D < 1 || D > kMaxFeat || ld < D || C < 1 || C > kMaxMemberC || ld_out < C)
        return fail(CE_EINVAL, "bad GaussianNB shapes F=%lld D=%d C=%d", (long long)F, D, C);
    if ((F > 0 && (!X || !out)) || !theta || !var || !log_prior) return fail(CE_EINVAL, "null pointer");
    // numpy sums fewer than 8 features sequentially; the 8-lane pairwise kernel
    // has no leaf for them (the reference's members have 260 features)
    if (D < 8) return fail(CE_EUNSUPPORTED, "GaussianNB needs D >= 8 features (got %d)", D);
    if (F == 0) return CE_OK;
    GnbArgs a{X, F, D, ld, theta, var, log_prior, C, out, ld_out};
    const PwPlan pl = pw_plan(D);
    const size_t lds = (size_t)3 * C * D * sizeof(double);  // up to 96 KB at C = 8, D = 512
    if (D == 260) {  // the reference's feature count: constant pairwise plan
        hipLaunchKernelGGL((k_gnb_proba8<36, 260>), dim3(member_grid8(F)), dim3(256), lds, (hipStream_t)stream, a, pl);
        return check_launch("ce_gnb_predict_proba");
    }
    with_nx(D, [&](auto nx) {
        auto kern = k_gnb_proba8<decltype(nx)::value, 0>;
        if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3(member_grid8(F)), dim3(256), lds, (hipStream_t)stream, a, pl);
    });
    return check_launch("ce_gnb_predict_proba");
}

extern "C" int ce_sgd_predict_proba(const double* X, int64_t F, int32_t D, int64_t ld, const double* coef,
                                    const double* intercept, int32_t K, int32_t C, double* out, int64_t ld_out,
                                    ce_stream_t stream) {
    if (F < 0 || D < 1 || D > kMaxFeat || ld < D || C < 2 || C > kMaxMemberC || ld_out < C ||
        !(K == C || (K == 1 && C == 2)))
        return fail(CE_EINVAL, "bad SGD shapes F=%lld D=%d K=%d C=%d", (long long)F, D, K, C);
    if ((F > 0 && (!X || !out)) || !coef || !intercept) return fail(CE_EINVAL, "null pointer");
    if (F == 0) return CE_OK;
    SgdArgs a{X, F, D, ld, coef, intercept, K, C, out, ld_out};
    const size_t lds = (size_t)K * D * sizeof(double);
    if (D == 260 && ld == 260 && K == 4 && C == 4 && ((uintptr_t)X & 15) == 0) {
        // the reference's contiguous rows: coalesced 16-B span loads; 76 KB LDS -> 2 blocks per CU, one resident wave of blocks
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(F, 32), 512));
        hipLaunchKernelGGL((k_sgd_span260<4>), dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
        return check_launch("ce_sgd_predict_proba");
    }
    with_nx(D, [&](auto nx) {
        hipLaunchKernelGGL((k_sgd_proba8<decltype(nx)::value>), dim3(member_grid8(F)), dim3(256), lds,
                           (hipStream_t)stream, a);
    });
    return check_launch("ce_sgd_predict_proba");
}

// ---- top-q of an entropy vector -------------------------------------------
extern "C" size_t ce_topq_workspace_bytes(int64_t N, int32_t q) {
    return lists_bytes(pool_blocks(N), q < 1 ? 1 : q);
}

static int finish_lists(WsLists w, int segments, int nl, int q, double* val_out, int64_t* idx_out,
                        hipStream_t st) {
    ListSrc<false> ls{w.c, nullptr, nullptr};
    launch_finish(ls, segments, nl, q, val_out, idx_out, st);
    return CE_OK;
}

extern "C" int ce_topq(const double* ent, int64_t N, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes,
                       double* val_out, int64_t* idx_out, ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (N < 0 || !val_out || !idx_out || (N > 0 && !ent)) return fail(CE_EINVAL, "bad topq arguments");
    const int G = pool_blocks(N);
    if (!ws || ws_bytes < lists_bytes(G, q)) return fail(CE_EWORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    WsLists w = carve(ws, G, q);
    Seg sg{nullptr, N, G, base_idx};
    launch_partial(ArraySrc{ent}, sg, G, q, w, val_out, idx_out, G == 1, st);
    if (G > 1) finish_lists(w, 1, G, q, val_out, idx_out, st);
    return check_launch("ce_topq");
}

extern "C" int ce_topq_merge(const double* vals, const int64_t* idx, int32_t nlists, int32_t q, double* val_out,
                             int64_t* idx_out, ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (nlists < 1 || !vals || !idx || !val_out || !idx_out) return fail(CE_EINVAL, "bad merge arguments");
    ListSrc<true> ls{nullptr, vals, idx};
    launch_finish(ls, 1, nlists, q, val_out, idx_out, (hipStream_t)stream);
    return check_launch("ce_topq_merge");
}

// ---- fused mc ----------------------------------------------------------------
extern "C" size_t ce_select_mc_workspace_bytes(int64_t N, int32_t q) { return ce_topq_workspace_bytes(N, q); }

static int mc_partial(const CommArgs& a, int q, int64_t base_idx, void* ws, size_t ws_bytes, double* val_out,
                      int64_t* idx_out, bool allow_final, int* G_out, bool* final_out, hipStream_t st) {
    int rc = check_comm(a);
    if (rc) return rc;
    rc = check_q(q);
    if (rc) return rc;
    const int G = pool_blocks(a.N);
    if (!ws || ws_bytes < lists_bytes(G, q)) return fail(CE_EWORKSPACE, "workspace too small");
    WsLists w = carve(ws, G, q);
    *G_out = G;
    *final_out = false;
    if (launch_stream(a, G, q, base_idx, w, st)) return CE_OK;
    Seg sg{nullptr, a.N, G, base_idx};
    const bool fin = allow_final && G == 1;
    rc = committee_partial(a, sg, G, q, w, val_out, idx_out, fin, st);
    if (rc) return dispatch_err(rc, a);
    *final_out = fin;
    return CE_OK;
}

static int select_mc_impl(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                          int64_t sC, const uint32_t* excl, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes,
                          double* val_out, int64_t* idx_out, ce_stream_t stream);

extern "C" int ce_select_mc(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                            int64_t sC, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes, double* val_out,
                            int64_t* idx_out, ce_stream_t stream) {
    return select_mc_impl(p, dt, N, M, C, sN, sM, sC, nullptr, q, base_idx, ws, ws_bytes, val_out, idx_out, stream);
}

extern "C" size_t ce_excl_words(int64_t N) { return N > 0 ? (size_t)((N + 31) / 32) : 0; }

extern "C" int ce_select_mc_excl(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                 int64_t sM, int64_t sC, const uint32_t* excl, int32_t q, int64_t base_idx, void* ws,
                                 size_t ws_bytes, double* val_out, int64_t* idx_out, ce_stream_t stream) {
    if (!excl && N > 0) return fail(CE_EINVAL, "null exclusion bitmap");
    if (q > kStreamMaxQ) return fail(CE_EUNSUPPORTED, "exclusion bitmaps need q <= %d (got %d)", kStreamMaxQ, q);
    return select_mc_impl(p, dt, N, M, C, sN, sM, sC, excl, q, base_idx, ws, ws_bytes, val_out, idx_out, stream);
}

static int select_mc_impl(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                          int64_t sC, const uint32_t* excl, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes,
                          double* val_out, int64_t* idx_out, ce_stream_t stream) {
    if (!val_out || !idx_out) return fail(CE_EINVAL, "null output");
    hipStream_t st = (hipStream_t)stream;
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int rc0 = check_comm(a);
    if (rc0) return rc0;
    rc0 = check_q(q);
    if (rc0) return rc0;
    // the workspace contract holds on every path, even the one that does not touch it
    if (!ws || ws_bytes < lists_bytes(pool_blocks(N), q)) return fail(CE_EWORKSPACE, "workspace too small");
    if (small_enabled() && q <= kStreamMaxQ && N > 0) {
        // one block scores and selects the whole pool (k_select_small)
        bool launched = false;
        const int rc = with_committee(a, [&](auto src) {
            using S = decltype(src);
            if (N <= (int64_t)kSmallBS * small_ipt<S>()) {
                launch_small<S, kSmallBS>(src, 1, nullptr, N, base_idx, q, val_out, idx_out, excl, st);
                launched = true;
            } else if (N <= (int64_t)kSmallBSWide * small_ipt<S>()) {
                launch_small<S, kSmallBSWide>(src, 1, nullptr, N, base_idx, q, val_out, idx_out, excl, st);
                launched = true;
            }
        });
        if (rc == CE_OK && launched) return check_launch("ce_select_mc");
    }
    if (stream_enabled() && q <= kStreamMaxQ && N > 0 &&
        N * (int64_t)M * C * elem_bytes((int)dt) <= kSmallPoolBytes) {
        // small pool: ~512 items per 4-wave block on a few CUs (one block: it
        // is the final answer), then one wave merges the blocks' lists
        const int nb = (int)std::min<int64_t>(std::min<int64_t>(cdiv(N, 512), 32), pool_blocks(N));
        WsLists w = carve(ws, nb, q);
        const int rc = with_committee(a, [&](auto src) {
            using S = decltype(src);
            with_seg_batching<S>([&](auto unr, auto ipl) {
                hipLaunchKernelGGL((k_stream_seg<S, decltype(ipl)::value, decltype(unr)::value, kSegWaves>), dim3(nb),
                                   dim3(256), 0, st, src, nullptr, N, base_idx, q, nb, val_out, idx_out, w.c, excl);
            });
        });
        if (rc == CE_OK) {
            if (nb > 1)
                hipLaunchKernelGGL((k_merge_wave<false>), dim3(1), dim3(256), 0, st, ListSrc<false>{w.c, nullptr, nullptr},
                                   1, nb, q, val_out, idx_out);
            return check_launch("ce_select_mc");
        }
    }
    int G = 0;
    bool fin = false;
    int rc;
    if (excl) {  // the streaming engine only (the q > 64 paths take no bitmap)
        G = pool_blocks(N);
        if (!stream_enabled() || !wide2_enabled() || !launch_stream(a, G, q, base_idx, carve(ws, G, q), st, excl))
            return fail(CE_EUNSUPPORTED, "exclusion bitmap: no streaming kernel for this shape");
    } else {
        rc = mc_partial(a, q, base_idx, ws, ws_bytes, val_out, idx_out, true, &G, &fin, st);
        if (rc) return rc;
    }
    if (!fin) finish_lists(carve(ws, G, q), 1, G, q, val_out, idx_out, st);
    return check_launch("ce_select_mc");
}

extern "C" int ce_select_mc_partial(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                    int64_t sM, int64_t sC, int32_t q, int64_t base_idx, void* ws,
                                    size_t ws_bytes, ce_stream_t stream) {
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int G = 0;
    bool fin = false;
    int rc = mc_partial(a, q, base_idx, ws, ws_bytes, nullptr, nullptr, false, &G, &fin, (hipStream_t)stream);
    if (rc) return rc;
    return check_launch("ce_select_mc_partial");
}

extern "C" int ce_select_finish(int64_t N, int32_t q, void* ws, size_t ws_bytes, double* val_out, int64_t* idx_out,
                                ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (N < 0 || !val_out || !idx_out) return fail(CE_EINVAL, "bad finish arguments");
    const int G = pool_blocks(N);
    if (!ws || ws_bytes < lists_bytes(G, q)) return fail(CE_EWORKSPACE, "workspace too small");
    finish_lists(carve(ws, G, q), 1, G, q, val_out, idx_out, (hipStream_t)stream);
    return check_launch("ce_select_finish");
}

// ---- exchange records (multi-GPU) -------------------------------------------
static_assert(sizeof(ce_cand) == sizeof(Cand) && alignof(ce_cand) <= alignof(Cand), "ce_cand must mirror Cand");

extern "C" int ce_select_finish_cands(int64_t N, int32_t q, void* ws, size_t ws_bytes, ce_cand* out,
                                      ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (q > kStreamMaxQ) return fail(CE_EUNSUPPORTED, "candidate records need q <= %d (got %d)", kStreamMaxQ, q);
    if (N < 0 || !out) return fail(CE_EINVAL, "bad finish arguments");
    if ((uintptr_t)out % 16) return fail(CE_EINVAL, "ce_cand output must be 16-byte aligned");
    const int G = pool_blocks(N);
    if (!ws || ws_bytes < lists_bytes(G, q)) return fail(CE_EWORKSPACE, "workspace too small");
    ListSrc<false> ls{carve(ws, G, q).c, nullptr, nullptr};
    launch_finish(ls, 1, G, q, nullptr, nullptr, (hipStream_t)stream, reinterpret_cast<Cand*>(out));
    return check_launch("ce_select_finish_cands");
}

extern "C" int ce_merge_cands(const ce_cand* c, int32_t nlists, int32_t q, double* val_out, int64_t* idx_out,
                              ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (nlists < 1 || !c || !val_out || !idx_out) return fail(CE_EINVAL, "bad merge arguments");
    if ((uintptr_t)c % 16) return fail(CE_EINVAL, "ce_cand input must be 16-byte aligned");
    ListSrc<false> ls{reinterpret_cast<const Cand*>(c), nullptr, nullptr};
    launch_finish(ls, 1, nlists, q, val_out, idx_out, (hipStream_t)stream);
    return check_launch("ce_merge_cands");
}

// ---- chunked pools (larger than HBM) ----------------------------------------
__global__ void k_cand_empty(Cand* __restrict__ c, int q) {
    for (int r = threadIdx.x; r < q; r += blockDim.x) c[r] = Cand{0ull, -1};
}

extern "C" size_t ce_select_mc_chunk_workspace_bytes(int64_t N, int32_t q) {
    return lists_bytes((int64_t)pool_blocks(N) + 1, q < 1 ? 1 : q);
}

// Stage 1 on the chunk (its G block lists), then ONE merge of those G lists
// plus the running list (copied to list slot G of the workspace) back into
// `running`: the running list always holds the top-q of every chunk so far
// (the top-q of a union is within the union of the parts' top-qs).
extern "C" int ce_select_mc_chunk(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                  int64_t sM, int64_t sC, int32_t q, int64_t base_idx, ce_cand* running,
                                  int32_t first, void* ws, size_t ws_bytes, ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (q > kStreamMaxQ) return fail(CE_EUNSUPPORTED, "chunked selection needs q <= %d (got %d)", kStreamMaxQ, q);
    if (!running || (uintptr_t)running % 16) return fail(CE_EINVAL, "running list must be 16-byte aligned device memory");
    if (N < 0 || base_idx < 0) return fail(CE_EINVAL, "bad chunk N=%lld base_idx=%lld", (long long)N, (long long)base_idx);
    hipStream_t st = (hipStream_t)stream;
    Cand* run = reinterpret_cast<Cand*>(running);
    if (N == 0) {
        if (first) hipLaunchKernelGGL(k_cand_empty, dim3(1), dim3(64), 0, st, run, q);
        return check_launch("ce_select_mc_chunk");
    }
    const int G = pool_blocks(N);
    if (!ws || ws_bytes < lists_bytes((int64_t)G + 1, q)) return fail(CE_EWORKSPACE, "workspace too small");
    WsLists w = carve(ws, (int64_t)G + 1, q);
    if (!first && hipMemcpyAsync(w.c + (int64_t)G * q, run, (size_t)q * sizeof(Cand), hipMemcpyDeviceToDevice, st) !=
                      hipSuccess)
        return fail(CE_ELAUNCH, "running-list copy failed");
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int Gs = 0;
    bool fin = false;
    rc = mc_partial(a, q, base_idx, ws, ws_bytes, nullptr, nullptr, false, &Gs, &fin, st);
    if (rc) return rc;
    launch_finish(ListSrc<false>{w.c, nullptr, nullptr}, 1, G + (first ? 0 : 1), q, nullptr, nullptr, st, run);
    return check_launch("ce_select_mc_chunk");
}

// ---- fused mix ---------------------------------------------------------------
extern "C" size_t ce_select_mix_workspace_bytes(int64_t N, int64_t N_h, int32_t q) {
    return lists_bytes((int64_t)pool_blocks(N) + pool_blocks(N_h), q < 1 ? 1 : q);
}

extern "C" int ce_select_mix(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                             int64_t sC, const double* hc, int64_t N_h, int64_t ld_hc, int32_t q, void* ws,
                             size_t ws_bytes, double* val_out, int64_t* idx_out, ce_stream_t stream) {
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int rc = check_comm(a);
    if (rc) return rc;
    rc = check_q(q);
    if (rc) return rc;
    if (N_h < 0 || (N_h > 0 && (!hc || ld_hc < C)) || !val_out || !idx_out)
        return fail(CE_EINVAL, "bad hc table / outputs");
    const int G1 = pool_blocks(N), G2 = pool_blocks(N_h);
    if (!ws || ws_bytes < lists_bytes((int64_t)G1 + G2, q)) return fail(CE_EWORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    WsLists w = carve(ws, (int64_t)G1 + G2, q);
    if (small_enabled() && q <= kStreamMaxQ && N > 0 && N_h > 0 && N <= 2 * kSmallBSWide &&
        N_h <= 2 * kSmallBSWide && (C == 4 || C == 8)) {
        // both segments in ONE block (k_select_small, two segments)
        const CommArgs t{hc, kF64, N_h, 1, C, ld_hc, C, 1};
        bool launched = false;
        rc = with_committee(a, [&](auto src) {
            using S = decltype(src);
            if constexpr (S::kC == 4 || S::kC == 8) {
                constexpr int CC = S::kC;
                if (vec_ok(t, CC))
                    launch_small_mix(src, make_src<kF64, CC, true>(t), N, N_h, q, val_out, idx_out, st);
                else
                    launch_small_mix(src, make_src<kF64, CC, false>(t), N, N_h, q, val_out, idx_out, st);
                launched = true;
            }
        });
        if (rc == CE_OK && launched) return check_launch("ce_select_mix");
    }
    // both segments on the streaming engine when it applies (q <= 64): the hc
    // table is a committee of M = 1 member ([N_h, 1, C] f64, row stride ld_hc)
    if (!launch_stream(a, G1, q, 0, w, st)) {
        Seg s1{nullptr, N, G1, 0};
        rc = committee_partial(a, s1, G1, q, w, nullptr, nullptr, false, st);
        if (rc) return dispatch_err(rc, a);
    }
    WsLists w2{w.c + (size_t)G1 * q};
    const CommArgs t{hc, kF64, N_h, 1, C, ld_hc, C, 1};
    if (launch_stream(t, G2, q, N, w2, st)) {
        finish_lists(w, 1, G1 + G2, q, val_out, idx_out, st);
        return check_launch("ce_select_mix");
    }
    Seg s2{nullptr, N_h, G2, N};
    switch (C) {
#define CE_T(CC) case CC: launch_partial(TableSrc<CC>{hc, ld_hc}, s2, G2, q, w2, nullptr, nullptr, false, st); break;
        CE_T(2) CE_T(3) CE_T(4) CE_T(8)
#undef CE_T
        default: return fail(CE_EUNSUPPORTED, "mix with C=%d has no kernel in this build", C);
    }
    finish_lists(w, 1, G1 + G2, q, val_out, idx_out, st);
    return check_launch("ce_select_mix");
}

// ---- batched users -------------------------------------------------------------
// blocks per user: ~1024 items per block (two iterations per wave of a
// 4-wave block), at most ~4096 blocks in all.  Measured at 500 x 1608 items:
// 512 items/block 33.2 us, 1024 31.4 us, 2048 (one block per user, no merge
// launch) 31.0 us; 256 45 us.
static int batched_bpu(int64_t total, int U) {
    if (U < 1) return 1;
    const int64_t avg = cdiv(total, U);
    int64_t bpu = cdiv(avg, (int64_t)1024);
    const int64_t cap = std::max<int64_t>(1, 4096 / U);
    bpu = std::max<int64_t>(1, std::min(bpu, cap));
    return (int)bpu;
}

extern "C" size_t ce_select_batched_workspace_bytes(int64_t total_items, int32_t U, int32_t q) {
    if (U < 1) U = 1;
    return lists_bytes((int64_t)batched_bpu(total_items, U) * U, q < 1 ? 1 : q);
}

extern "C" int ce_select_batched(const void* p, ce_dtype dt, int64_t total_items, int32_t M, int32_t C, int64_t sN,
                                 int64_t sM, int64_t sC, const int64_t* offsets, int32_t U, int32_t q, void* ws,
                                 size_t ws_bytes, double* val_out, int64_t* idx_out, ce_stream_t stream) {
    CommArgs a{p, (int)dt, total_items, M, C, sN, sM, sC};
    int rc = check_comm(a);
    if (rc) return rc;
    rc = check_q(q);
    if (rc) return rc;
    if (U < 1 || !offsets || !val_out || !idx_out) return fail(CE_EINVAL, "bad batched arguments");
    const int bpu = batched_bpu(total_items, U);
    const int64_t nl = (int64_t)bpu * U;
    if (!ws || ws_bytes < lists_bytes(nl, q)) return fail(CE_EWORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    WsLists w = carve(ws, nl, q);
    if (small_enabled() && q <= kStreamMaxQ) {
        // one 512-thread block per user when the average user fits one sweep
        // (k_select_small; a longer user streams inside its block)
        bool launched = false;
        rc = with_committee(a, [&](auto src) {
            using S = decltype(src);
            if (cdiv(total_items, U) <= (int64_t)kSmallBS * small_ipt<S>()) {
                launch_small<S, kSmallBS>(src, U, offsets, 0, 0, q, val_out, idx_out, nullptr, st);
                launched = true;
            }
        });
        if (rc == CE_OK && launched) return check_launch("ce_select_batched");
    }
    if (stream_enabled() && q <= kStreamMaxQ) {
        // bpu 4-wave blocks per user, then one wave per user merges its bpu lists
        rc = with_committee(a, [&](auto src) {
            using S = decltype(src);
            with_seg_batching<S>([&](auto unr, auto ipl) {
                hipLaunchKernelGGL((k_stream_seg<S, decltype(ipl)::value, decltype(unr)::value, kSegWaves>),
                                   dim3((unsigned)nl), dim3(bpu == 1 && U < 64 ? 64 * kSegWaves : 256), 0, st, src, offsets,
                                   (int64_t)0, (int64_t)0, q, bpu, val_out, idx_out, w.c, (const uint32_t*)nullptr);
            });
        });
        if (rc == CE_OK) {
            if (bpu > 1)
                hipLaunchKernelGGL((k_merge_wave<false>), dim3((U + 3) / 4), dim3(256), 0, st,
                                   ListSrc<false>{w.c, nullptr, nullptr}, U, bpu, q, val_out, idx_out);
            return check_launch("ce_select_batched");
        }
    }
    Seg sg{offsets, total_items, bpu, 0};
    const bool fin = bpu == 1;
    rc = committee_partial(a, sg, (int)nl, q, w, val_out, idx_out, fin, st);
    if (rc) return dispatch_err(rc, a);
    if (!fin) finish_lists(w, U, bpu, q, val_out, idx_out, st);
    return check_launch("ce_select_batched");
}
