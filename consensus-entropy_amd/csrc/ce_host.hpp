// ce_host.hpp -- host side shared by the C-ABI translation units: argument
// checks, workspace geometry, kernel dispatch (ce_abi_*.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "../../include/ce.h"
#include "ce_abi.hpp"
#include "ce_kernels.hpp"

using namespace ce;

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// stage-1 blocks for a pool of n items (host arithmetic only: ws sizing and
// launches agree by construction)
static inline int pool_blocks(int64_t n) {
    // one 64-item tile per wave at least; up to 1024 blocks (4 per CU), so wide
    // items (tens of KB each) still fill the chip
    int64_t g = cdiv(n, (int64_t)kMinItemsPerBlock);
    if (g < 1) g = 1;
    if (g > kMaxBlocks) g = kMaxBlocks;
    return (int)g;
}

static inline size_t lists_bytes(int64_t nlists, int q) { return (size_t)nlists * (size_t)q * 16u + 256u; }

struct WsLists {
    Cand* c;
};
static inline WsLists carve(void* ws, int64_t nlists, int q) {
    uintptr_t p = ((uintptr_t)ws + 255) & ~(uintptr_t)255;
    WsLists w;
    w.c = reinterpret_cast<Cand*>(p);
    return w;
}

static inline int check_q(int q) {
    if (q < 1 || q > CE_MAX_Q) return fail(CE_EINVAL, "q=%d outside [1, %d]", q, CE_MAX_Q);
    return CE_OK;
}

template <class Src>
static inline void launch_partial(const Src& src, const Seg& sg, int grid, int q, WsLists w, double* oval,
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
static inline bool merge_reg_enabled() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_MERGE_REG");
        return !(e && e[0] == '0');
    }();
    return on;
}

// ocand != nullptr: write candidate records (q <= kStreamMaxQ only) instead of (val, idx).
template <bool FROM_VALS>
static inline void launch_finish(ListSrc<FROM_VALS> src, int segments, int nl, int q, double* oval, int64_t* oidx,
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

static inline int check_comm(const CommArgs& a) {
    if (!a.p && a.N > 0) return fail(CE_EINVAL, "null committee pointer");
    if (a.N < 0 || a.M < 1 || a.C < 1) return fail(CE_EINVAL, "bad shape N=%lld M=%d C=%d", (long long)a.N, a.M, a.C);
    if (a.dt < 0 || a.dt > 2) return fail(CE_EINVAL, "bad dtype %d", a.dt);
    return CE_OK;
}

static inline int elem_bytes(int dt) { return dt == kF64 ? 8 : (dt == kF32 ? 4 : 2); }

static inline bool vec_ok(const CommArgs& a, int C) {
    if (a.sC != 1) return false;
    const int eb = elem_bytes(a.dt);
    const int vb = a.dt == kBF16 ? 8 : 16;  // bytes per vector load
    if (a.dt == kF64 ? (C % 2) : (C % 4)) return false;
    if ((uintptr_t)a.p % vb) return false;
    if ((a.sN * eb) % vb || (a.sM * eb) % vb) return false;
    return true;
}

template <int DT, int C, bool VEC>
static inline CommitteeSrc<DT, C, VEC> make_src(const CommArgs& a) {
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
static inline int with_committee(const CommArgs& a, F&& f) {
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
static inline WideArgs wide_args(const CommArgs& a) {
    WideArgs w{a.p, a.N, a.M, a.C, a.sN, a.sM, a.sC, (double)a.M, 1.0 / (double)a.M, (a.M & (a.M - 1)) == 0};
    return w;
}
static inline size_t wide_lds_bytes(int C) { return (size_t)4 * wide_lds_doubles(C) * sizeof(double); }

static inline bool wide_vec_ok(const CommArgs& a) {
    const int eb = elem_bytes(a.dt);
    return a.sC == 1 && (a.C * eb) % 16 == 0 && (a.sM * eb) % 16 == 0 && (a.sN * eb) % 16 == 0 &&
           (uintptr_t)a.p % 16 == 0;
}

// f(dt, npl, vec) with compile-time values
template <class F>
static inline int with_wide_v(const CommArgs& a, F&& f) {
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

static inline void launch_partial_wide(const CommArgs& a, const Seg& sg, int grid, int q, WsLists w, double* oval,
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
static inline bool stream_enabled() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_STREAM");  // A/B knob: CE_AMD_STREAM=0 -> block-synchronous k_partial
        return !(e && e[0] == '0');
    }();
    return on;
}

// Cache policy of the item-major LDS-DMA stream: nt (default) or the default
// policy (A/B knob CE_AMD_DMA_NT=0).
static inline bool dma_nt() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_DMA_NT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// A/B knob: CE_AMD_WIDE2=0 -> the unpipelined wide kernel (k_stream_wide)
static inline bool wide2_enabled() {
    static const bool on = [] {
        const char* e = getenv("CE_AMD_WIDE2");
        return !(e && e[0] == '0');
    }();
    return on;
}

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

// The same for k_stream_seg: up to 16-wave blocks (<= 128 VGPRs), so fewer loads per lane.
template <class Src, class F>
static inline void with_seg_batching(F&& f) {
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
static inline void launch_small(const Src& src, int grid, const int64_t* offsets, int64_t n, int64_t base_idx, int q,
                         double* oval, int64_t* oidx, const uint32_t* excl, hipStream_t st) {
    constexpr int UNR = (Src::kDT == kF64 || Src::kC > 4 || BS > kSmallBS) ? 2 : 4;
    hipLaunchKernelGGL((k_select_small<Src, Src, small_ipt<Src>(), 0, UNR, 1, BS>), dim3((unsigned)grid), dim3(BS), 0,
                       st, src, src, offsets, n, (int64_t)0, base_idx, q, oval, oidx, excl);
}
// mix in one block: committee items (A) then the hc table rows (B, a 1-member
// f64 committee); IPT 2 per segment at 1024 threads: up to 2048 + 2048 rows
template <class SrcA, class SrcB>
static inline void launch_small_mix(const SrcA& a, const SrcB& b, int64_t n, int64_t nB, int q, double* oval,
                             int64_t* oidx, hipStream_t st) {
    constexpr int UNRA = (SrcA::kDT == kF64 || SrcA::kC > 4) ? 2 : 4;
    hipLaunchKernelGGL((k_select_small<SrcA, SrcB, 2, 2, UNRA, 1, kSmallBSWide>), dim3(1), dim3(kSmallBSWide), 0, st, a,
                       b, (const int64_t*)nullptr, n, nB, (int64_t)0, q, oval, oidx, (const uint32_t*)nullptr);
}
static inline bool small_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("CE_AMD_SMALL");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

// Blocks of `kernel` resident on the whole device (occupancy API x CUs), cached.
static inline int device_cus() {
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
static inline int resident_grid(K kernel, size_t dyn_lds, int cap) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, dyn_lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    (void)hipGetLastError();
    const int g = per_cu * device_cus();
    return g < cap ? g : cap;
}

static inline StreamArgs stream_args(const CommArgs& a, int G, int64_t base_idx) {
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
static inline void stream_grid(StreamArgs& s, int grid) {
    const int64_t W = (int64_t)grid * 4;
    s.per_wave = (cdiv(s.N, W) + 63) / 64 * 64;
}

// Launches the streaming kernel when it applies; returns false otherwise.
static inline bool launch_stream(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
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
                // a 2-batch register ring (3 and 4 measured: 72.8 / 71.9 % vs 72.6 % at C5)
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
static inline int committee_partial(const CommArgs& a, const Seg& sg, int grid, int q, WsLists w, double* oval,
                             int64_t* oidx, bool fin, hipStream_t st) {
    int rc = with_committee(a, [&](auto src) { launch_partial(src, sg, grid, q, w, oval, oidx, fin, st); });
    if (rc != CE_EUNSUPPORTED) return rc;
    if (a.C > kWideMaxC) return CE_EUNSUPPORTED;
    launch_partial_wide(a, sg, grid, q, w, oval, oidx, fin, st);
    return CE_OK;
}

static inline int dispatch_err(int rc, const CommArgs& a) {
    if (rc == CE_EUNSUPPORTED)
        return fail(CE_EUNSUPPORTED, "committee shape C=%d dtype=%d has no kernel in this build", a.C, a.dt);
    return rc;
}

static inline int finish_lists(WsLists w, int segments, int nl, int q, double* val_out, int64_t* idx_out,
                        hipStream_t st) {
    ListSrc<false> ls{w.c, nullptr, nullptr};
    launch_finish(ls, segments, nl, q, val_out, idx_out, st);
    return CE_OK;
}
