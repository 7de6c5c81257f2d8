// ce_members.hpp -- on-device committee member inference:
// the predict_proba of the reference's linear members over the 260 scaled
// audio features (amg_test.py:435, :467 -> deam_classifier.py:211-218), so the
// committee's frame probabilities never leave the GPU before the segment mean
// (ce_segment_mean) and the selection.
//
//   GaussianNB (sklearn 0.24.1 _joint_log_likelihood + predict_log_proba):
//     jll_c = log(prior_c) + ((-0.5 * sum_f log(2 pi var_cf)) - 0.5 * sum_f (x_f - theta_cf)^2 / var_cf)
//     p_c   = exp(jll_c - logsumexp(jll)),  logsumexp = log(sum_c exp(jll_c - max)) + max
//     Every sum over features is numpy's pairwise sum (np.sum along the row),
//     reproduced with the same tree as the entropy row sums, and exp / log are
//     glibc's restated (gexp / glog below: numpy 1.19.5 -- the reference's pin
//     -- calls the C library for float64 exp / log), so predict_proba is the
//     reference's bit for bit (tests: against the numpy restatement with libm's
//     exp / log, oracle/ce_oracle.py ref_gnb_predict_proba).
//   SGDClassifier(loss='log') (_predict_proba_lr): d_k = x . coef_k + b_k,
//     p_k = expit(d_k) = 1 / (1 + exp(-d_k)) (glibc's exp), then p /= sum_k p_k (OvR, K > 1),
//     or [1 - p, p] for a binary model.  The dot products are BLAS dgemm in the
//     reference (an unspecified order); here a fixed wave-reduction order --
//     parity is to a tolerance (tests state it).
//
// Eight lanes per frame, eight frames per wave: lane j of a group owns the
// features f = 8m + j -- exactly numpy's eight pairwise accumulators (leaves
// start at multiples of 8), so a leaf's sum is lane j's sequential chain
// followed by the ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) butterfly of the group.
// theta / var / coef are staged once per block in LDS.
#pragma once
#include "ce_device.hpp"
#include "ce_glibc_exp.hpp"
#include "ce_stream.hpp"
#include "ce_wide.hpp"

namespace ce {

// glibc's f64 exp / log (ce_glibc_exp.hpp, ce_glibc_log.hpp), tables read from
// global memory (L2-resident): the member kernels stage their own LDS data.
__device__ __forceinline__ double gexp(double x) { return glibc_exp(x, g_exp_tab); }
__device__ __forceinline__ double glog(double x) {
    return glibc_log_fast(x, reinterpret_cast<const LogEntry*>(g_log_tab));
}

constexpr int kMaxFeat = 512;   // features per frame (the reference: 260)
constexpr int kMaxMemberC = 8;  // classes (the reference: 4 quadrants)

struct GnbArgs {
    const double* X;
    int64_t F;
    int D;
    int64_t ld;
    const double* theta;      // [C, D]
    const double* var;        // [C, D] (sklearn 0.24: sigma_)
    const double* log_prior;  // [C] = log(class_prior_)
    int C;
    double* out;              // [F, C], row stride ldo
    int64_t ldo;
};

struct SgdArgs {
    const double* X;
    int64_t F;
    int D;
    int64_t ld;
    const double* coef;       // [K, D], K = C (multiclass OvR) or 1 (binary)
    const double* intercept;  // [K]
    int K, C;
    double* out;
    int64_t ldo;
};

// np.sum of the terms t[m] (feature f = 8m + j of this lane's group; 0 past
// D) in numpy's pairwise order; the result in every lane of the 8-lane group.
// The terms are computed once by the caller; the leaf bounds are wave-uniform.
template <int NX>
__device__ __forceinline__ double group_pairwise(const double (&t)[NX], const PwPlan& pl) {
    const int lane = threadIdx.x & 63, j = lane & 7, gb = lane & ~7;
    double lv = 0.0;  // lane gb + l: leaf l's sum
    for (int l = 0; l < pl.nleaves; ++l) {
        const int st = pl.lstart[l], len = pl.llen[l];
        const int nb = len - (len % 8);
        const int m0 = st >> 3, m1 = (st + nb) >> 3;
        double r = 0.0, tl = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            if (m == m0) r = t[m];
            else if (m > m0 && m < m1) r += t[m];
            if (m == m1) tl = t[m];  // tail elements st + nb + k sit in lanes gb + k of column m1
        }
        r = r + __shfl_xor(r, 1);
        r = r + __shfl_xor(r, 2);
        r = r + __shfl_xor(r, 4);
        for (int k = 0; k < len % 8; ++k) r += __shfl(tl, gb + k);
        if (j == l) lv = r;
    }
    for (int rd = 0; rd < pl.nrounds; ++rd) {
        const int p = j < kPwMaxLeaves ? pl.partner[rd][j] : -1;
        const double v = __shfl(lv, gb + (p >= 0 ? p : j));
        if (p >= 0) lv = lv + v;
    }
    return 0.0 + __shfl(lv, gb);
}

// (d * d) / var without a division per term: var is per (class, feature), so
// its reciprocal y = RN(1/var) is computed once per block; q0 = RN(dd * y) is
// within 1 ulp of dd / var, the FMA residual dd - var * q0 is exact, and one
// correction q0 + y * r rounds to the IEEE quotient (Markstein's theorem;
// checked against true division on 4e8 random pairs, near-all-ones divisor
// mantissas included: 0 mismatches).  Non-finite q0 (an infinite feature)
// keeps the plain product's inf / NaN.
__device__ __forceinline__ double div_by_recip(double dd, double v, double y) {
    const double q0 = dd * y;
    const double r = __builtin_fma(-q0, v, dd);
    const double q = __builtin_fma(r, y, q0);
    return __builtin_isfinite(q0) ? q : q0;
}

// group_pairwise for a feature count DF known at compile time (the
// reference's D = 260): the plan is a constant, so the leaf boundaries, the
// column loops and the combine rounds all resolve at compile time -- the same
// additions in the same order, without the per-column selects.
template <int NX, int DF>
__device__ __forceinline__ double group_pairwise_const(const double (&t)[NX]) {
    constexpr PwPlan pl = pw_plan(DF);
    static_assert(pl.nleaves <= 8, "constant plans cover <= 8 leaves (one per lane of the group)");
    const int lane = threadIdx.x & 63, j = lane & 7, gb = lane & ~7;
    double lv = 0.0;
#pragma unroll
    for (int l = 0; l < pl.nleaves; ++l) {
        const int st = pl.lstart[l], len = pl.llen[l];
        const int nb = len - (len % 8), m0 = st >> 3, m1 = (st + nb) >> 3;
        double r = t[m0];
#pragma unroll
        for (int m = m0 + 1; m < m1; ++m) r += t[m];
        r = r + __shfl_xor(r, 1);
        r = r + __shfl_xor(r, 2);
        r = r + __shfl_xor(r, 4);
        if (len % 8) {
            const double tl = t[m1 < NX ? m1 : NX - 1];  // tail elements st + nb + k: lanes gb + k of column m1
#pragma unroll
            for (int k = 0; k < len % 8; ++k) r += __shfl(tl, gb + k);
        }
        if (j == l) lv = r;
    }
#pragma unroll
    for (int rd = 0; rd < pl.nrounds; ++rd) {
        int p = -1;
#pragma unroll
        for (int a = 0; a < 8; ++a)
            if (j == a) p = pl.partner[rd][a];
        const double v = __shfl(lv, gb + (p >= 0 ? p : j));
        if (p >= 0) lv = lv + v;
    }
    return 0.0 + __shfl(lv, gb);
}

template <int NX, int DF>
__device__ __forceinline__ double group_sum(const double (&t)[NX], const PwPlan& pl) {
    if constexpr (DF > 0)
        return group_pairwise_const<NX, DF>(t);
    else
        return group_pairwise<NX>(t, pl);
}

// GaussianNB, 8 lanes per frame.  LDS: theta, var, 1/var [C][D] doubles, and
// the per-class -0.5 * np.sum(np.log(2 pi var_c)) (group c computes class c once).
template <int NX, int DF>  // DF: the feature count when fixed at compile time (0: a.D, runtime plan)
__global__ __launch_bounds__(256) void k_gnb_proba8(GnbArgs a, PwPlan pl) {
    extern __shared__ __attribute__((aligned(16))) double msm[];
    __shared__ double hs1[kMaxMemberC];
    double* th = msm;
    double* vr = msm + (int64_t)a.C * a.D;
    double* rv = msm + (int64_t)2 * a.C * a.D;
    for (int t = threadIdx.x; t < a.C * a.D; t += blockDim.x) {
        th[t] = a.theta[t];
        vr[t] = a.var[t];
        rv[t] = 1.0 / a.var[t];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 7, g = lane >> 3, w = threadIdx.x >> 6;
    if (w * 8 < a.C) {  // wave-uniform: the waves holding groups 0..C-1
        const int gid = w * 8 + g, c = gid < a.C ? gid : 0;
        double t[NX];
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            const int f = 8 * m + j;
            t[m] = f < a.D ? glog(2. * M_PI * vr[c * a.D + f]) : 0.0;
        }
        const double s1 = group_sum<NX, DF>(t, pl);
        if (gid < a.C && j == 0) hs1[gid] = -0.5 * s1;
    }
    __syncthreads();
    const int64_t step = (int64_t)gridDim.x * 32;
    for (int64_t f0 = ((int64_t)blockIdx.x * 4 + w) * 8; f0 < a.F; f0 += step) {
        const int64_t fr = f0 + g;
        const int64_t frc = fr < a.F ? fr : a.F - 1;  // clamped: every group loads
        double x[NX];
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            const int f = 8 * m + j;
            x[m] = f < a.D ? a.X[frc * a.ld + f] : 0.0;
        }
        double jll[kMaxMemberC];
        for (int c = 0; c < a.C; ++c) {
            double t[NX];
#pragma unroll
            for (int m = 0; m < NX; ++m) {
                const int f = 8 * m + j, fc = f < a.D ? f : 0;
                const double d = x[m] - th[c * a.D + fc];
                t[m] = f < a.D ? div_by_recip(d * d, vr[c * a.D + fc], rv[c * a.D + fc]) : 0.0;
            }
            const double s2 = group_sum<NX, DF>(t, pl);
            double n_ij = hs1[c];
            n_ij -= 0.5 * s2;
            jll[c] = a.log_prior[c] + n_ij;
        }
        double mx = jll[0];
        for (int c = 1; c < a.C; ++c) mx = jll[c] > mx ? jll[c] : mx;
        if (!__builtin_isfinite(mx)) mx = 0.0;
        double s = -0.0;
        for (int c = 0; c < a.C; ++c) s += gexp(jll[c] - mx);
        const double lse = glog(0.0 + s) + mx;
        if (fr < a.F && j < a.C) {
            double v = 0.0;
            for (int c = 0; c < a.C; ++c)
                if (c == j) v = gexp(jll[c] - lse);
            a.out[fr * a.ldo + j] = v;
        }
    }
}

// GaussianNB for the reference's shape (D = 260 features, KC = C classes),
// feature-streamed: k_gnb_proba8 holds a frame group's 33 feature values AND
// one class's 33 terms in registers before each pairwise sum, and issues the
// next group's loads only when the group is done.  Here the column loop is
// outermost: x[m] feeds the KC classes' terms at once, and each term goes
// straight into its numpy accumulator -- the pairwise plan of n = 260 is three
// leaves, [0,128) [128,192) [192,260), so lane j's chain of leaf l is a running
// sum over the columns of that leaf (first term assigned, then +=, as numpy's
// r[j]) -- and the register x[m] is refilled with the NEXT group's value as
// soon as it is consumed, so a whole group's loads are in flight during the
// current group's arithmetic.  Per leaf the 8 chains are combined by the xor
// butterfly (((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) in every lane of the group),
// the 4 tail features 256..259 are added in order, and the row sum is
// 0.0 + (L0 + (L1 + L2)) -- the same operations in the same order as
// k_gnb_proba8 and numpy.  LDS: {theta, 1/var} pairs (one ds_read_b128) and
// var, per class and feature.
template <int KC, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_gnb_stream260(GnbArgs a) {
    constexpr int D = 260, NX = 33;
    static_assert(pw_plan(D).nleaves == 3 && pw_plan(D).lstart[1] == 128 && pw_plan(D).lstart[2] == 192 &&
                      pw_plan(D).llen[2] == 68,
                  "the leaf layout this kernel hard-codes");
    __shared__ __attribute__((aligned(16))) f64x2 tr[KC * D];  // {theta, RN(1/var)}
    __shared__ double vr[KC * D];
    __shared__ double hs1[KC];
    for (int t = threadIdx.x; t < KC * D; t += blockDim.x) {
        const double v = a.var[t];
        tr[t] = f64x2{a.theta[t], 1.0 / v};
        vr[t] = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 7, g = lane >> 3, w = threadIdx.x >> 6;
    if (w == 0) {  // -0.5 * np.sum(np.log(2 pi var_c)): group c < KC computes class c
        // leaf by leaf with rolled loops (one log live at a time; an unrolled
        // 33-log body would set the whole kernel's register budget)
        const int c = g < KC ? g : 0;
        const double* v = vr + c * D + j;
        auto lg = [&](int m) { return glog(2. * M_PI * v[8 * m]); };
        double L[3];
        const int m0[3] = {0, 16, 24}, m1[3] = {16, 24, 32};
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            double r = lg(m0[l]);
#pragma unroll 1
            for (int m = m0[l] + 1; m < m1[l]; ++m) r += lg(m);
            r = r + __shfl_xor(r, 1);
            r = r + __shfl_xor(r, 2);
            r = r + __shfl_xor(r, 4);
            L[l] = r;
        }
        const double tl = j < 4 ? lg(32) : 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) L[2] += __shfl(tl, (lane & ~7) + k);
        const double s1 = 0.0 + (L[0] + (L[1] + L[2]));
        if (g < KC && j == 0) hs1[g] = -0.5 * s1;
    }
    __syncthreads();
    const int64_t step = (int64_t)gridDim.x * 32;
    int64_t f0 = ((int64_t)blockIdx.x * 4 + w) * 8;
    auto row_of = [&](int64_t fb) { const int64_t fr = fb + g; return a.X + (fr < a.F ? fr : a.F - 1) * a.ld; };
    double x[NX];
    {
        const double* xr = row_of(f0);
#pragma unroll
        for (int m = 0; m < NX; ++m) x[m] = (m < NX - 1 || j < 4) ? __builtin_nontemporal_load(xr + 8 * m + j) : 0.0;
    }
    for (; f0 < a.F; f0 += step) {
        const double* xn = row_of(f0 + step);  // next group (clamped: always a valid row)
        // the table reads are loop-invariant: left visible, LICM hoists all 33 x KC
        // of them out of the frame loop (hundreds of VGPRs, spills); an opaque
        // per-iteration base keeps them in their column
        int jo = j;
        asm volatile("" : "+v"(jo));
        double r[KC][3], tl[KC];
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            const bool live = m < NX - 1 || j < 4;  // column 32: features 256..259 only
            const double xm = x[m];
            if (live) x[m] = __builtin_nontemporal_load(xn + 8 * m + j);
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int fc = live ? c * D + 8 * m + jo : c * D;
                const f64x2 p = tr[fc];
                const double d = xm - p.x;
                const double t = live ? div_by_recip(d * d, vr[fc], p.y) : 0.0;
                if (m == 0 || m == 16 || m == 24) r[c][m == 0 ? 0 : (m == 16 ? 1 : 2)] = t;
                else if (m < 16) r[c][0] += t;
                else if (m < 24) r[c][1] += t;
                else if (m < 32) r[c][2] += t;
                else tl[c] = t;
                if constexpr (WPE >= 4) asm volatile("" ::: "memory");  // 4 waves: one class's table reads at a time
            }
            // pin each column's terms to their column: unconstrained, the compiler
            // issues all 33 columns' table reads first and sinks every term after
            // them (hundreds of live VGPRs, spills)
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                if (m < 16) asm volatile("" : "+v"(r[c][0]));
                else if (m < 24) asm volatile("" : "+v"(r[c][1]));
                else if (m < 32) asm volatile("" : "+v"(r[c][2]));
                else asm volatile("" : "+v"(tl[c]));
            }
            asm volatile("" ::: "memory");  // and the column's loads (the refill included) to their column
        }
        double jll[KC];
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            double L[3];
#pragma unroll
            for (int l = 0; l < 3; ++l) {
                double v = r[c][l];
                v = v + __shfl_xor(v, 1);
                v = v + __shfl_xor(v, 2);
                v = v + __shfl_xor(v, 4);
                L[l] = v;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) L[2] += __shfl(tl[c], (lane & ~7) + k);
            const double s2 = 0.0 + (L[0] + (L[1] + L[2]));
            double n_ij = hs1[c];
            n_ij -= 0.5 * s2;
            jll[c] = a.log_prior[c] + n_ij;
        }
        double mx = jll[0];
#pragma unroll
        for (int c = 1; c < KC; ++c) mx = jll[c] > mx ? jll[c] : mx;
        if (!__builtin_isfinite(mx)) mx = 0.0;
        // one transcendental at a time (the next group's 33 features are live
        // here; overlapped exps would set the kernel's register peak)
        double s = -0.0;
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            s += gexp(jll[c] - mx);
            asm volatile("" : "+v"(s));
        }
        const double lse = glog(0.0 + s) + mx;
        const int64_t fr = f0 + g;
        if (fr < a.F && j < a.C) {
            double jl = jll[0];
#pragma unroll
            for (int c = 1; c < KC; ++c)
                if (c == j) jl = jll[c];
            a.out[fr * a.ldo + j] = gexp(jl - lse);  // lane j's class only: exp(jll[j] - lse)
        }
    }
}

// Lane j's partial dot product -> the group's d (butterfly) -> expit(d + b).
__device__ __forceinline__ double sgd_expit(double d, double b) {
    d = d + __shfl_xor(d, 1);
    d = d + __shfl_xor(d, 2);
    d = d + __shfl_xor(d, 4);
    d += b;
    return 1.0 / (1.0 + gexp(-d));  // scipy.special.expit
}

template <int KR>
__device__ __forceinline__ void sgd_store(const SgdArgs& a, double (&p)[KR], int K, int64_t fr, int j);

// SGDClassifier(loss='log'), 8 lanes per frame; coef in LDS.
template <int NX>
__global__ __launch_bounds__(256) void k_sgd_proba8(SgdArgs a) {
    extern __shared__ __attribute__((aligned(16))) double msm[];
    for (int t = threadIdx.x; t < a.K * a.D; t += blockDim.x) msm[t] = a.coef[t];
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 7, g = lane >> 3, w = threadIdx.x >> 6;
    const int64_t step = (int64_t)gridDim.x * 32;
    for (int64_t f0 = ((int64_t)blockIdx.x * 4 + w) * 8; f0 < a.F; f0 += step) {
        const int64_t fr = f0 + g;
        const int64_t frc = fr < a.F ? fr : a.F - 1;
        double x[NX];
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            const int f = 8 * m + j;
            x[m] = f < a.D ? a.X[frc * a.ld + f] : 0.0;
        }
        double p[kMaxMemberC];
        for (int c = 0; c < a.K; ++c) {
            double d = 0.0;
#pragma unroll
            for (int m = 0; m < NX; ++m) {
                const int f = 8 * m + j;
                if (f < a.D) d = fma(x[m], msm[c * a.D + f], d);
            }
            p[c] = sgd_expit(d, a.intercept[c]);
        }
        sgd_store(a, p, a.K, fr, j);
    }
}

// The OvR normalisation (or the binary [1 - p, p]) and the store of lane j's class.
template <int KR>
__device__ __forceinline__ void sgd_store(const SgdArgs& a, double (&p)[KR], int K, int64_t fr, int j) {
    if (K == 1) {
        p[1] = p[0];
        p[0] = 1.0 - p[1];
    } else {
        double s = -0.0;
        for (int c = 0; c < K; ++c) s += p[c];
        s = 0.0 + s;
        for (int c = 0; c < K; ++c) p[c] /= s;
    }
    if (fr < a.F && j < a.C) {
        double v = 0.0;
        for (int c = 0; c < a.C; ++c)
            if (c == j) v = p[c];
        a.out[fr * a.ldo + j] = v;
    }
}

// SGD for the reference's contiguous 260-feature rows (ld == D == 260, K == C
// == KC): a wave's 8 frames are one contiguous 16,640-B span, fetched one span
// ahead with 16-B non-temporal loads (1 KiB per instruction, fully coalesced,
// instead of 8 rows x 64 B per 8-B load) and transposed through a wave-private
// LDS slot (rows padded to 264 doubles) into k_sgd_proba8's 8-lanes-per-frame
// layout -- the same FMA chains and butterfly, so the same bits.
template <int KC>
__global__ __launch_bounds__(256) void k_sgd_span260(SgdArgs a) {
    constexpr int D = 260, RP = 264, NX = 33, SPAN = 8 * D / 2, NCH = (SPAN + 63) / 64;  // 1040 chunks, 17 loads
    __shared__ __attribute__((aligned(16))) double cf[KC * D];
    __shared__ __attribute__((aligned(16))) double xs[4][8 * RP];
    for (int t = threadIdx.x; t < KC * D; t += blockDim.x) cf[t] = a.coef[t];
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 7, g = lane >> 3, w = threadIdx.x >> 6;
    const int64_t nchunks = a.F * (D / 2);
    const f64x2* X2 = reinterpret_cast<const f64x2*>(a.X);
    const int64_t step = (int64_t)gridDim.x * 32;
    double* xw = xs[w];
    auto fetch = [&](f64x2(&buf)[NCH], int64_t fb) {
        if (fb >= a.F) return;
        const int64_t c0 = fb * (D / 2);
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            const int c = k * 64 + lane;
            if (c < SPAN && c0 + c < nchunks) buf[k] = __builtin_nontemporal_load(X2 + c0 + c);
        }
    };
    // one span: registers -> LDS slot, refill the registers one span ahead,
    // then the classes' FMA chains (m outer: one x value live at a time)
    auto span = [&](f64x2(&buf)[NCH], int64_t fc) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the previous span's reads precede these writes
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            const int c = k * 64 + lane;
            if (c < SPAN) {
                const int r = (2 * c) / D, col = 2 * c - r * D;  // D even: a chunk never straddles rows
                *reinterpret_cast<f64x2*>(xw + r * RP + col) = buf[k];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        fetch(buf, fc + step);
        double d[KC];
#pragma unroll
        for (int c = 0; c < KC; ++c) d[c] = 0.0;
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            if (m < NX - 1 || j < D - 8 * (NX - 1)) {
                const double x = xw[g * RP + 8 * m + j];
#pragma unroll
                for (int c = 0; c < KC; ++c) d[c] = fma(x, cf[c * D + 8 * m + j], d[c]);
            }
        }
        double p[KC > 1 ? KC : 2];
#pragma unroll
        for (int c = 0; c < KC; ++c) p[c] = sgd_expit(d[c], a.intercept[c]);
        sgd_store(a, p, KC, fc + g, j);
    };
    f64x2 b0[NCH];
    int64_t f0 = ((int64_t)blockIdx.x * 4 + w) * 8;
    fetch(b0, f0);
    for (; f0 < a.F; f0 += step) span(b0, f0);
}

}  // namespace ce

