// ce_host.hpp -- host side shared by the C-ABI translation units: argument
// checks, workspace geometry, dispatch helpers, and the declarations of the
// launchers (each defined in one ce_launch_*.hip).
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
#include "ce_sort.hpp"

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

// Workspace layout (every *_workspace_bytes / carve agree): a fixed header of
// kWsCounters u32 arrival counters (the tiled kernels' tickets, one per
// problem; zero at rest: the caller zero-fills the workspace once, every call
// leaves the counters zero) followed by the candidate lists, 16 B per slot.
// The header is the same for every entry point, so one workspace can serve
// any sequence of calls.
constexpr int kWsCounters = 16384;
constexpr size_t kWsHeader = (size_t)kWsCounters * sizeof(uint32_t);  // 64 KiB
static inline size_t lists_bytes(int64_t nlists, int q) {
    return kWsHeader + (size_t)nlists * (size_t)q * 16u + 256u;
}

// The wide stream's floor + grid vote scratch (k_wide_seed / k_wide_seed_pick),
// carved right after a launch's lists: every workspace size that can reach a
// folded wide launch adds kWideSeedBytes (ce_topq_workspace_bytes,
// ce_select_mc_chunk_workspace_bytes).
constexpr size_t kWideSeedBytes = 256 + 256 + (size_t)kWideVoteSamples * (sizeof(Cand) + sizeof(float)) + 256;
constexpr int64_t kWideSeedMinItems = 16 * 1024;  // >= 1024 samples (wide_nsamples: 1/16 of the items)
struct WideSeedWs {
    uint32_t* vote;
    Cand* seed;
    Cand* samp;   // [kWideVoteSamples]
    float* sapx;  // [kWideVoteSamples]
};
static inline WideSeedWs wide_seed_carve(void* base) {
    const uintptr_t p = ((uintptr_t)base + 255) & ~(uintptr_t)255;
    WideSeedWs w;
    w.vote = reinterpret_cast<uint32_t*>(p);
    w.seed = reinterpret_cast<Cand*>(p + 16);
    w.samp = reinterpret_cast<Cand*>(p + 256);
    w.sapx = reinterpret_cast<float*>(p + 256 + (size_t)kWideVoteSamples * sizeof(Cand));
    return w;
}

struct WsLists {
    Cand* c;        // candidate lists
    uint32_t* ctr;  // arrival counters (header)
};
static inline WsLists carve(void* ws, int64_t nlists, int q) {
    (void)nlists;
    (void)q;
    uintptr_t p = ((uintptr_t)ws + 255) & ~(uintptr_t)255;
    WsLists w;
    w.ctr = reinterpret_cast<uint32_t*>(p);
    w.c = reinterpret_cast<Cand*>(p + kWsHeader);
    return w;
}

// Any q >= 0, as the reference's -q (amg_test.py:547-553): argsort[::-1][:q]
// returns min(q, N) positions, none for q = 0.  q <= CE_MAX_Q runs on the list
// kernels; above it on the sort path (ce_sort.hpp, its workspace grows with N).
static inline int check_q(int q) {
    if (q < 0) return fail(CE_EINVAL, "q=%d is negative", q);
    return CE_OK;
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

// ---- streaming stage 1 (q <= 64): wave-independent, LDS-DMA for item-major ----
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
    s.ctr = nullptr;
    s.oval = nullptr;
    s.oidx = nullptr;
    s.ocand = nullptr;
    s.extra = nullptr;
    s.vote = nullptr;
    s.vote_heavy = 0;
    s.seed = nullptr;
    return s;
}

// the grid actually launched (<= G workspace lists) and its per-wave share
static inline void stream_grid(StreamArgs& s, int grid) {
    const int64_t W = (int64_t)grid * 4;
    s.per_wave = (cdiv(s.N, W) + 63) / 64 * 64;
}

static inline int dispatch_err(int rc, const CommArgs& a) {
    if (rc == CE_EUNSUPPORTED)
        return fail(CE_EUNSUPPORTED, "committee shape C=%d dtype=%d has no kernel in this build", a.C, a.dt);
    return rc;
}

// ---------------------------------------------------------------------------
// Launchers.  Each is DEFINED in exactly one translation unit (named below),
// so every kernel instantiation lives in one code object of libce_amd.so;
// the entry points (ce_abi_*.hip) only call these.
// ---------------------------------------------------------------------------
// ce_launch_stream.hip: streaming stage 1 (q <= 64): k_stream_nmc (item-major
// LDS-DMA), k_stream_direct (any strides), k_stream_wide2 / k_stream_wide
// (wide classes).  Returns false (nothing launched) when no kernel applies.
CE_HIDDEN bool launch_stream(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
                             const uint32_t* excl = nullptr);
// The same with stage 2 folded in: the grid's last block merges the block
// lists into the final (oval, oidx), or into q records at ocand (one launch
// for the whole selection).  Returns 0 (no streaming kernel applies), 1
// (launched WITHOUT the fold: the lists are in w, run a finish) or 2 (folded).
struct FoldOut {
    double* oval;
    int64_t* oidx;
    Cand* ocand;
    const Cand* extra;  // one more list to merge (a chunked job's running list), or nullptr
    void* wide_ws;      // kWideSeedBytes of workspace for the wide stream's floor + grid vote, or nullptr
};
CE_HIDDEN int launch_stream_fold(const CommArgs& a, int G, int q, int64_t base_idx, WsLists w, hipStream_t st,
                                 const uint32_t* excl, FoldOut out);
// ce_launch_partial.hip: block-synchronous stage 1 (any q): committee,
// precomputed entropies, an hc table.
CE_HIDDEN int committee_partial(const CommArgs& a, const Seg& sg, int grid, int q, WsLists w, double* oval,
                                int64_t* oidx, bool fin, hipStream_t st);
CE_HIDDEN void partial_entropies(const double* ent, const Seg& sg, int grid, int q, WsLists w, double* oval,
                                 int64_t* oidx, bool fin, hipStream_t st);
CE_HIDDEN int partial_table(const double* hc, int64_t ld, int C, const Seg& sg, int grid, int q, WsLists w,
                            hipStream_t st);
// ce_launch_finish.hip: stage 2 merges of candidate lists.
CE_HIDDEN void launch_finish_lists(const Cand* c, int segments, int nl, int q, double* oval, int64_t* oidx,
                                   hipStream_t st, Cand* ocand = nullptr);
CE_HIDDEN void launch_finish_vals(const double* vals, const int64_t* idx, int segments, int nl, int q,
                                  double* oval, int64_t* oidx, hipStream_t st);
CE_HIDDEN void launch_merge_wave(const Cand* c, int segs, int nl, int q, double* oval, int64_t* oidx,
                                 hipStream_t st);
// ce_launch_small.hip: pools of a few thousand items, one block per problem
// (k_select_tiles, ce_small.hpp).
// one pool of a.N items (<= kSmallPoolItems); false: too large / no kernel
constexpr int64_t kSmallPoolItems = 4096;
CE_HIDDEN bool launch_small_pool(const CommArgs& a, int64_t base_idx, int q, double* oval, int64_t* oidx,
                                 const uint32_t* excl, WsLists w, hipStream_t st);
// U users (offsets[U+1]) in one launch, one block per user
CE_HIDDEN bool launch_small_users(const CommArgs& a, const int64_t* offsets, int U, int q, double* oval,
                                  int64_t* oidx, hipStream_t st);
// the mix of amg_test.py:473-480 ([mc; hc] rows, C = 4) in one launch
CE_HIDDEN bool launch_small_mix(const CommArgs& a, const CommArgs& t, int q, double* oval, int64_t* oidx,
                                hipStream_t st);
// k_stream_seg over `nblocks` blocks of `threads` (bpu blocks per segment)
CE_HIDDEN bool launch_seg(const CommArgs& a, const int64_t* offsets, int64_t n, int64_t base_idx, int q, int nblocks,
                          int bpu, int threads, double* oval, int64_t* oidx, Cand* wc, const uint32_t* excl,
                          hipStream_t st);

// ce_launch_sort.hip: the sort path for q > CE_MAX_Q (ce_sort.hpp).  Workspace:
// the 64 KiB header, then n entropies, two n-record buffers, the digit counts
// and `extra_cands` records.
CE_HIDDEN size_t sort_ws_bytes(int64_t n, int64_t extra_cands = 0);
CE_HIDDEN SortWs sort_carve(void* ws, int64_t n, int64_t extra_cands = 0);
// records {order key (0 if excluded), idx0 + i} of ent[0..n) into out
CE_HIDDEN void sort_keys(const double* ent, int64_t n, int64_t idx0, const uint32_t* excl, Cand* out, hipStream_t st);
CE_HIDDEN void sort_keys_users(const double* ent, int64_t n, const int64_t* offsets, int U, Cand* out, hipStream_t st);
// sorts s.a[0..s.g.n) (generated in ascending position) by key descending, then
// user_passes passes over the user bits; returns the buffer holding the result
CE_HIDDEN const Cand* sort_run(const SortWs& s, int user_passes, hipStream_t st);
CE_HIDDEN int user_sort_passes(int U);
// the first q slots of sorted records as (val, idx) or records (ocand)
CE_HIDDEN void sort_out(const Cand* s, int64_t n, int64_t q, double* oval, int64_t* oidx, Cand* ocand, hipStream_t st);
CE_HIDDEN void sort_out_users(const Cand* s, const int64_t* offsets, int U, int64_t q, double* oval, int64_t* oidx,
                              hipStream_t st);
// merge of nl best-first lists of q slots (records c, or (vals, idx)) by rank
CE_HIDDEN void rank_merge_lists(const Cand* c, const double* vals, const int64_t* idx, int nl, int64_t q, double* oval,
                                int64_t* oidx, Cand* ocand, hipStream_t st);
// ce_abi_core.hip: per-item committee entropy (and optional mean) to HBM, any supported shape
CE_HIDDEN int launch_entropy(const CommArgs& a, double* mean_or_null, double* ent, hipStream_t st);

// The sort path counts records per wave and per digit in 32 bits
// (ce_launch_sort.hip): it takes fewer than 2^32 records per call.
constexpr int64_t kSortMaxRecords = 0xFFFFFFFFll;
static inline int check_sort_n(int64_t n) {
    if (n > kSortMaxRecords)
        return fail(CE_EUNSUPPORTED, "q > %d sorts the pool: it takes < 2^32 items per call (got %lld)", CE_MAX_Q,
                    (long long)n);
    return CE_OK;
}

// entropies ent[0..n) -> the first q slots of the total order (sort path)
static inline void sort_select(const SortWs& s, const double* ent, int64_t n, int64_t idx0, const uint32_t* excl,
                               int64_t q, double* oval, int64_t* oidx, Cand* ocand, hipStream_t st) {
    sort_keys(ent, n, idx0, excl, s.a, st);
    sort_out(sort_run(s, 0, st), n, q, oval, oidx, ocand, st);
}

static inline int finish_lists(WsLists w, int segments, int nl, int q, double* val_out, int64_t* idx_out,
                               hipStream_t st) {
    launch_finish_lists(w.c, segments, nl, q, val_out, idx_out, st);
    return CE_OK;
}
