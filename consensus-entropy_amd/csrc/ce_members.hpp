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
//     reproduced with the same tree as the entropy row sums; only exp / log
//     (ocml vs glibc, <= 1-2 ulp) differ from the reference.
//   SGDClassifier(loss='log') (_predict_proba_lr): d_k = x . coef_k + b_k,
//     p_k = expit(d_k) = 1 / (1 + exp(-d_k)), then p /= sum_k p_k (OvR, K > 1),
//     or [1 - p, p] for a binary model.  The dot products are BLAS dgemm in the
//     reference (an unspecified order); here a fixed wave-reduction order --
//     parity is to a tolerance (tests state it).
//
// One wave per frame: lane l owns features l, l + 64, ... (coalesced row loads).
#pragma once
#include "ce_device.hpp"
#include "ce_stream.hpp"
#include "ce_wide.hpp"

namespace ce {

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

// sum over the wave's LDS row a[0..D) in numpy's pairwise order
__device__ __forceinline__ double row_pairwise(double* row, const PwPlan& pl) {
    __builtin_amdgcn_wave_barrier();
    const double s = wave_row_sum(row, pl, nullptr);
    __builtin_amdgcn_wave_barrier();
    return s;
}

template <int NF>  // features per lane (D <= 64 * NF)
__global__ __launch_bounds__(256) void k_gnb_proba(GnbArgs a, PwPlan pl) {
    __shared__ __attribute__((aligned(16))) double gsm[4 * kMaxFeat];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* row = gsm + w * kMaxFeat;
    // per class: -0.5 * np.sum(np.log(2. * np.pi * var_c)) (every wave computes it once)
    double half_s1[kMaxMemberC];
    for (int c = 0; c < a.C; ++c) {
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            const int f = lane + 64 * k;
            if (f < a.D) row[f] = log(2. * M_PI * a.var[(int64_t)c * a.D + f]);
        }
        half_s1[c] = -0.5 * row_pairwise(row, pl);
    }
    for (int64_t fr = (int64_t)blockIdx.x * 4 + w; fr < a.F; fr += (int64_t)gridDim.x * 4) {
        double x[NF];
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            const int f = lane + 64 * k;
            x[k] = f < a.D ? a.X[fr * a.ld + f] : 0.0;
        }
        double jll[kMaxMemberC];
        for (int c = 0; c < a.C; ++c) {
#pragma unroll
            for (int k = 0; k < NF; ++k) {
                const int f = lane + 64 * k;
                if (f < a.D) {
                    const double d = x[k] - a.theta[(int64_t)c * a.D + f];
                    row[f] = (d * d) / a.var[(int64_t)c * a.D + f];
                }
            }
            const double s2 = row_pairwise(row, pl);
            double n_ij = half_s1[c];
            n_ij -= 0.5 * s2;
            jll[c] = a.log_prior[c] + n_ij;
        }
        // scipy.special.logsumexp(jll, axis=1): max (non-finite -> 0), exp, sequential sum (C < 8), log
        double mx = jll[0];
        for (int c = 1; c < a.C; ++c) mx = jll[c] > mx ? jll[c] : mx;  // np.amax (NaN aside)
        if (!__builtin_isfinite(mx)) mx = 0.0;
        double s = -0.0;
        for (int c = 0; c < a.C; ++c) s += exp(jll[c] - mx);
        const double lse = log(0.0 + s) + mx;
        if (lane < a.C) {
            double v = 0.0;
            for (int c = 0; c < a.C; ++c)
                if (c == lane) v = exp(jll[c] - lse);
            a.out[fr * a.ldo + lane] = v;
        }
    }
}

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

template <int NF>
__global__ __launch_bounds__(256) void k_sgd_proba(SgdArgs a) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t fr = (int64_t)blockIdx.x * 4 + w; fr < a.F; fr += (int64_t)gridDim.x * 4) {
        double x[NF];
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            const int f = lane + 64 * k;
            x[k] = f < a.D ? a.X[fr * a.ld + f] : 0.0;
        }
        double p[kMaxMemberC];
        for (int c = 0; c < a.K; ++c) {
            double d = 0.0;
#pragma unroll
            for (int k = 0; k < NF; ++k) {
                const int f = lane + 64 * k;
                if (f < a.D) d = fma(x[k], a.coef[(int64_t)c * a.D + f], d);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off);
            d += a.intercept[c];
            p[c] = 1.0 / (1.0 + exp(-d));  // scipy.special.expit
        }
        if (a.K == 1) {  // binary: np.vstack([1 - prob, prob]).T
            p[1] = p[0];
            p[0] = 1.0 - p[1];
        } else {
            double s = -0.0;
            for (int c = 0; c < a.K; ++c) s += p[c];
            s = 0.0 + s;
            for (int c = 0; c < a.K; ++c) p[c] /= s;
        }
        if (lane < a.C) {
            double v = 0.0;
            for (int c = 0; c < a.C; ++c)
                if (c == lane) v = p[c];
            a.out[fr * a.ldo + lane] = v;
        }
    }
}

}  // namespace ce
