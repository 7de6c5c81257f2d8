// ce_abi_core.hip -- C-ABI (include/ce.h): errors, per-item entropy, hc tables,
// the device log, segment mean, exclusion bitmaps, member inference, top-q and
// merges.  Kernels: ce_kernels.hpp; dispatch helpers: ce_host.hpp.
#include "ce_glibc_exp.hpp"
#include "ce_host.hpp"

using namespace ce;

namespace ce {
// glibc log over a vector (verification of ce_glibc_log.hpp against libm).
__global__ __launch_bounds__(kBS) void k_log(const double* __restrict__ x, int64_t n, double* __restrict__ y) {
    stage_log_table();
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) y[i] = dlog(x[i]);
}

// glibc exp over a vector (verification of ce_glibc_exp.hpp against libm).
__global__ __launch_bounds__(kBS) void k_exp(const double* __restrict__ x, int64_t n, double* __restrict__ y) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) y[i] = dexp(x[i]);
}

// x[i] / s[i] through the entropy path's shared-reciprocal division
// (row_quotients, ce_device.hpp) -- verification against IEEE division.
__global__ __launch_bounds__(kBS) void k_rowdiv(const double* __restrict__ x, const double* __restrict__ s, int64_t n,
                                                double* __restrict__ y) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS)
    {
        const double xi[1] = {x[i]};  // the row-level range test of the entropy kernels, one class per row
        double d[1];
        row_quotients<1>(xi, s[i], d);
        y[i] = d[0];
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
}  // namespace ce

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

static thread_local char g_kernel[256] = "";

void note_kernel(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_kernel, sizeof g_kernel, fmt, ap);
    va_end(ap);
}

extern "C" const char* ce_last_error(void) { return g_err; }
extern "C" const char* ce_last_kernel(void) { return g_kernel; }
extern "C" const char* ce_version(void) { return "ce_amd 0.1 gfx950"; }


int launch_entropy(const CommArgs& a, double* mean_or_null, double* ent, hipStream_t st) {
    const int64_t N = a.N;
    if (N == 0) return CE_OK;
    const int grid = (int)std::min<int64_t>(cdiv(N, kBS), 4096);
    int rc = with_committee(a, [&](auto src) {
        hipLaunchKernelGGL((k_entropy<decltype(src)>), dim3(grid), dim3(kBS), 0, st, src, N, mean_or_null, ent);
    });
    if (rc == CE_EUNSUPPORTED) {
        const WideArgs wa = wide_args(a);
        const PwPlan pl = pw_plan(a.C);
        const size_t lds = wide_lds_bytes(a.C);
        const int wgrid = (int)std::min<int64_t>(cdiv(N, 4), 8192);
        if (mean_or_null) return fail(CE_EUNSUPPORTED, "mean output for C=%d is not implemented", a.C);
        rc = with_wide_v(a, [&](auto dt, auto npl, auto vec) {
            hipLaunchKernelGGL((k_wide_entropy_v<decltype(dt)::value, decltype(npl)::value, decltype(vec)::value>),
                               dim3(wgrid), dim3(256), lds, st, wa, pl, ent);
        });
    }
    return rc ? dispatch_err(rc, a) : CE_OK;
}

extern "C" int ce_committee_entropy(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                    int64_t sM, int64_t sC, double* mean_or_null, double* ent,
                                    ce_stream_t stream) {
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int rc = check_comm(a);
    if (rc) return rc;
    if (!ent) return fail(CE_EINVAL, "null ent");
    if (N == 0) return CE_OK;
    rc = launch_entropy(a, mean_or_null, ent, (hipStream_t)stream);
    if (rc) return rc;
    return check_launch("ce_committee_entropy");
}


extern "C" int ce_log_f64(const double* x, int64_t n, double* y, ce_stream_t stream) {
    if (n < 0 || (n > 0 && (!x || !y))) return fail(CE_EINVAL, "bad log arguments");
    if (n == 0) return CE_OK;
    const int grid = (int)std::min<int64_t>(cdiv(n, kBS), 8192);
    hipLaunchKernelGGL(k_log, dim3(grid), dim3(kBS), 0, (hipStream_t)stream, x, n, y);
    return check_launch("ce_log_f64");
}

extern "C" int ce_exp_f64(const double* x, int64_t n, double* y, ce_stream_t stream) {
    if (n < 0 || (n > 0 && (!x || !y))) return fail(CE_EINVAL, "bad exp arguments");
    if (n == 0) return CE_OK;
    const int grid = (int)std::min<int64_t>(cdiv(n, kBS), 8192);
    hipLaunchKernelGGL(k_exp, dim3(grid), dim3(kBS), 0, (hipStream_t)stream, x, n, y);
    return check_launch("ce_exp_f64");
}

// the small pools' approximate entropy (ce_device.hpp approx_key) of n exact
// rows [n, C]: log2 units, and the special flag (those rows take the exact path)
template <int C>
__global__ __launch_bounds__(kBS) void k_approx(const double* __restrict__ rows, int64_t n, float* __restrict__ h2,
                                                uint8_t* __restrict__ special) {
    for (int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
        double m[C];
#pragma unroll
        for (int c = 0; c < C; ++c) m[c] = rows[i * C + c];
        bool sp;
        const uint32_t k = approx_key<C>(m, sp);
        h2[i] = approx_key_value(k);
        special[i] = sp ? 1 : 0;
    }
}

extern "C" int ce_approx_entropy(const double* rows, int64_t n, int32_t C, float* h2, uint8_t* special,
                                 ce_stream_t stream) {
    if (n < 0 || (n > 0 && (!rows || !h2 || !special))) return fail(CE_EINVAL, "bad approx-entropy arguments");
    if (n == 0) return CE_OK;
    const int grid = (int)std::min<int64_t>(cdiv(n, kBS), 8192);
    const hipStream_t st = (hipStream_t)stream;
    switch (C) {
        case 2: hipLaunchKernelGGL(k_approx<2>, dim3(grid), dim3(kBS), 0, st, rows, n, h2, special); break;
        case 3: hipLaunchKernelGGL(k_approx<3>, dim3(grid), dim3(kBS), 0, st, rows, n, h2, special); break;
        case 4: hipLaunchKernelGGL(k_approx<4>, dim3(grid), dim3(kBS), 0, st, rows, n, h2, special); break;
        case 8: hipLaunchKernelGGL(k_approx<8>, dim3(grid), dim3(kBS), 0, st, rows, n, h2, special); break;
        default: return fail(CE_EINVAL, "approx entropy: C must be 2, 3, 4 or 8 (the single-block pools' classes)");
    }
    return check_launch("ce_approx_entropy");
}

// the wide stream's approximate prefilter (ce_wide.hpp wave_approx_entropy) of n
// rows [n, C] f64 -- the member sums (or means) of one item each -- laid out in
// registers as k_stream_wide2<DT, KCH, *> holds them: one wave per row
template <int DT, int KCH>
__global__ __launch_bounds__(256) void k_wide_approx(const double* __restrict__ rows, int64_t n, int C,
                                                     float* __restrict__ h2, uint8_t* __restrict__ special) {
    constexpr int CPC = ChunkT<DT>::CPC;
    const int lane = threadIdx.x & 63, K = C / CPC;
    for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (int64_t)gridDim.x * 4) {
        double acc[KCH * CPC];
#pragma unroll
        for (int kk = 0; kk < KCH; ++kk) {
            const int ch = lane + 64 * kk;
#pragma unroll
            for (int e = 0; e < CPC; ++e) acc[kk * CPC + e] = ch < K ? rows[i * C + ch * CPC + e] : 0.0;
        }
        bool sp;
        const float a = wave_approx_entropy<DT, KCH>(acc, K, sp);
        if (lane == 0) {
            h2[i] = a;
            special[i] = sp ? 1 : 0;
        }
    }
}

extern "C" int ce_wide_approx_entropy(const double* rows, int64_t n, int32_t C, ce_dtype dt, float* h2,
                                      uint8_t* special, ce_stream_t stream) {
    if (n < 0 || (n > 0 && (!rows || !h2 || !special))) return fail(CE_EINVAL, "bad approx-entropy arguments");
    if (dt != CE_F32 && dt != CE_F64 && dt != CE_BF16) return fail(CE_EINVAL, "bad dtype %d", (int)dt);
    const int cpc = dt == CE_F32 ? 4 : (dt == CE_F64 ? 2 : 8);
    if (C < 1 || C > kWideMaxC || C % cpc)
        return fail(CE_EINVAL, "wide approx entropy: C=%d must be a multiple of %d in [1, %d] (the vector stream's rows)",
                    C, cpc, kWideMaxC);
    if (n == 0) return CE_OK;
    const hipStream_t st = (hipStream_t)stream;
    const int grid = (int)std::min<int64_t>(cdiv(n, 4), 8192);
    const int npl = C <= 512 ? 8 : (C <= 1024 ? 16 : 32);  // with_wide_v's per-lane classes
#define CE_WA(DT_, CPC_)                                                                                       \
    if ((int)dt == DT_) {                                                                                      \
        if (npl == 8) hipLaunchKernelGGL((k_wide_approx<DT_, (8 / CPC_ > 0 ? 8 / CPC_ : 1)>), dim3(grid), dim3(256), 0, st, rows, n, C, h2, special); \
        else if (npl == 16) hipLaunchKernelGGL((k_wide_approx<DT_, 16 / CPC_>), dim3(grid), dim3(256), 0, st, rows, n, C, h2, special); \
        else hipLaunchKernelGGL((k_wide_approx<DT_, 32 / CPC_>), dim3(grid), dim3(256), 0, st, rows, n, C, h2, special); \
    }
    CE_WA(kF32, 4) CE_WA(kF64, 2) CE_WA(kBF16, 8)
#undef CE_WA
    return check_launch("ce_wide_approx_entropy");
}

extern "C" int ce_exp_f64_host(const double* x, int64_t n, double* y) {
    if (n < 0 || (n > 0 && (!x || !y))) return fail(CE_EINVAL, "bad exp arguments");
    const uint64_t* tab = host_exp_table();
    for (int64_t i = 0; i < n; ++i) y[i] = glibc_exp(x[i], tab);
    return CE_OK;
}

extern "C" int ce_row_div_f64(const double* x, const double* s, int64_t n, double* y, ce_stream_t stream) {
    if (n < 0 || (n > 0 && (!x || !s || !y))) return fail(CE_EINVAL, "bad division arguments");
    if (n == 0) return CE_OK;
    const int grid = (int)std::min<int64_t>(cdiv(n, kBS), 8192);
    hipLaunchKernelGGL(k_rowdiv, dim3(grid), dim3(kBS), 0, (hipStream_t)stream, x, s, n, y);
    return check_launch("ce_row_div_f64");
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
    if (D == 260 && ld == 260 && C == 4) {  // the reference's contiguous rows: feature-streamed
        // 3 waves per SIMD (166 VGPRs, no spills) measured fastest: 2.48 ms at 4M
        // frames vs 2.69 ms for 4 waves with spills
        auto kern = k_gnb_stream260<4, 3>;
        const int grid = resident_grid(kern, 0, (int)std::min<int64_t>(cdiv(F, 32), 1 << 20));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
        return check_launch("ce_gnb_predict_proba");
    }
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
    if (q > CE_MAX_Q) return sort_ws_bytes(N);
    return lists_bytes(pool_blocks(N), q < 1 ? 1 : q);
}


extern "C" int ce_topq(const double* ent, int64_t N, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes,
                       double* val_out, int64_t* idx_out, ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (N < 0 || (q > 0 && (!val_out || !idx_out)) || (N > 0 && !ent)) return fail(CE_EINVAL, "bad topq arguments");
    if (q == 0) return CE_OK;
    if (!ws || ws_bytes < ce_topq_workspace_bytes(N, q)) return fail(CE_EWORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    if (q > CE_MAX_Q) {
        rc = check_sort_n(N);
        if (rc) return rc;
        sort_select(sort_carve(ws, N), ent, N, base_idx, nullptr, q, val_out, idx_out, nullptr, st);
        return check_launch("ce_topq");
    }
    const int G = pool_blocks(N);
    WsLists w = carve(ws, G, q);
    Seg sg{nullptr, N, G, base_idx};
    partial_entropies(ent, sg, G, q, w, val_out, idx_out, G == 1, st);
    if (G > 1) finish_lists(w, 1, G, q, val_out, idx_out, st);
    return check_launch("ce_topq");
}

extern "C" int ce_topq_merge(const double* vals, const int64_t* idx, int32_t nlists, int32_t q, double* val_out,
                             int64_t* idx_out, ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (q == 0) return CE_OK;
    if (nlists < 1 || !vals || !idx || !val_out || !idx_out) return fail(CE_EINVAL, "bad merge arguments");
    if (q > CE_MAX_Q)  // no workspace here: the lists merge by rank (binary searches)
        rank_merge_lists(nullptr, vals, idx, nlists, q, val_out, idx_out, nullptr, (hipStream_t)stream);
    else
        launch_finish_vals(vals, idx, 1, nlists, q, val_out, idx_out, (hipStream_t)stream);
    return check_launch("ce_topq_merge");
}
