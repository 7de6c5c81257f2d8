// ce_wide.hpp -- committees with many classes (C up to 2048, e.g. the
// 1000-class wide config): one wave per item, lanes over classes.
//
// The row sums inside scipy.stats.entropy use numpy's pairwise summation
// (leaves of <= 128 elements summed with 8 strided accumulators, combined by a
// fixed binary tree).  The host builds the tree for the call's C once
// (PwPlan: leaves + postfix combine program); each leaf is summed by 8 lanes
// with shuffles reproducing ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), and lane 0
// runs the combine program -- the same additions in the same order as numpy.
#pragma once
#include "ce_device.hpp"
#include "ce_topq.hpp"

namespace ce {

constexpr int kWideMaxC = 2048;
constexpr int kPwMaxLeaves = 32;

struct PwPlan {
    int n;
    int nleaves;
    int nops;
    short lstart[kPwMaxLeaves];
    short llen[kPwMaxLeaves];
    signed char ops[2 * kPwMaxLeaves];  // >= 0: push leaf; -1: pop two, push sum
};

// Host: numpy's recursion (loops_utils.h.src) for n elements.
static inline void pw_build(PwPlan& pl, int start, int n) {
    if (n <= 128) {
        pl.lstart[pl.nleaves] = (short)start;
        pl.llen[pl.nleaves] = (short)n;
        pl.ops[pl.nops++] = (signed char)pl.nleaves;
        pl.nleaves++;
        return;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    pw_build(pl, start, n2);
    pw_build(pl, start + n2, n - n2);
    pl.ops[pl.nops++] = -1;
}

static inline PwPlan pw_plan(int n) {
    PwPlan pl{};
    pl.n = n;
    if (n >= 8) pw_build(pl, 0, n);
    return pl;
}

// Wave-cooperative np.sum(a[0:n]) over an LDS row (returns the same value in
// every lane).  scratch: >= kPwMaxLeaves + 8 doubles of per-wave LDS.
__device__ inline double wave_row_sum(const double* a, const PwPlan& pl, double* scratch) {
    const int lane = threadIdx.x & 63;
    double res = 0.0;
    if (pl.n < 8) {
        if (lane == 0) {
            double r = -0.0;
            for (int i = 0; i < pl.n; ++i) r += a[i];
            res = 0.0 + r;
        }
        return __shfl(res, 0);
    }
    // leaves: 8 lanes per leaf, 8 leaves per pass
    for (int l0 = 0; l0 < pl.nleaves; l0 += 8) {
        const int leaf = l0 + (lane >> 3), j = lane & 7;
        double r = 0.0;
        int st = 0, len = 0;
        if (leaf < pl.nleaves) {
            st = pl.lstart[leaf];
            len = pl.llen[leaf];
            const int nb = len - (len % 8);
            r = a[st + j];
            for (int i = 8; i < nb; i += 8) r += a[st + i + j];
        }
        r = r + __shfl_xor(r, 1);
        r = r + __shfl_xor(r, 2);
        r = r + __shfl_xor(r, 4);
        if (leaf < pl.nleaves && j == 0) {
            for (int i = len - (len % 8); i < len; ++i) r += a[st + i];
            scratch[leaf] = r;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (lane == 0) {
        double* stk = scratch + kPwMaxLeaves;
        int sp = 0;
        for (int o = 0; o < pl.nops; ++o) {
            const int op = pl.ops[o];
            if (op >= 0) {
                stk[sp++] = scratch[op];
            } else {
                const double b = stk[--sp];
                const double x = stk[--sp];
                stk[sp++] = x + b;
            }
        }
        res = 0.0 + stk[0];
    }
    return __shfl(res, 0);
}

template <int DT>
__device__ __forceinline__ double load_one(const void* p, int64_t off) {
    if constexpr (DT == kF32)
        return (double)__builtin_nontemporal_load(static_cast<const float*>(p) + off);
    else if constexpr (DT == kF64)
        return __builtin_nontemporal_load(static_cast<const double*>(p) + off);
    else
        return bf16_to_f64(__builtin_nontemporal_load(static_cast<const uint16_t*>(p) + off));
}

// One item's consensus entropy by one wave.  Lane l owns classes l + 64k.
// row: per-wave LDS row of >= C doubles.  Writes the mean row to mean_out.
template <int DT, int KMAX>
__device__ inline double wave_item_entropy(const void* p, int64_t off, int M, int C, int64_t sM, int64_t sC,
                                           double dM, double invM, bool pow2, const PwPlan& pl, double* row,
                                           double* scratch, double* mean_out) {
    const int lane = threadIdx.x & 63;
    double acc[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) acc[k] = 0.0;
    int m = 0;
    for (; m + 2 <= M; m += 2) {
        double v0[KMAX], v1[KMAX];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int c = lane + 64 * k;
            v0[k] = v1[k] = 0.0;
            if (c < C) {
                v0[k] = load_one<DT>(p, off + (int64_t)m * sM + c * sC);
                v1[k] = load_one<DT>(p, off + (int64_t)(m + 1) * sM + c * sC);
            }
        }
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            acc[k] += v0[k];
            acc[k] += v1[k];
        }
    }
    for (; m < M; ++m) {
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int c = lane + 64 * k;
            if (c < C) acc[k] += load_one<DT>(p, off + (int64_t)m * sM + c * sC);
        }
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int c = lane + 64 * k;
        acc[k] = div_members(acc[k], dM, invM, pow2);
        if (c < C) {
            row[c] = acc[k];
            if (mean_out) mean_out[c] = acc[k];
        }
    }
    __builtin_amdgcn_wave_barrier();
    const double s = wave_row_sum(row, pl, scratch);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int c = lane + 64 * k;
        if (c < C) row[c] = entr(1.0 * acc[k] / s);
    }
    __builtin_amdgcn_wave_barrier();
    const double h = wave_row_sum(row, pl, scratch);
    __builtin_amdgcn_wave_barrier();
    return h;
}

struct WideArgs {
    const void* p;
    int64_t N;
    int M, C;
    int64_t sN, sM, sC;
    double dM, invM;
    bool pow2;
};

// LDS per wave: C row + scratch.
__host__ __device__ constexpr int wide_lds_doubles(int C) { return ((C + kPwMaxLeaves + 8 + 1) / 2) * 2; }

template <int DT, int KMAX>
__global__ __launch_bounds__(256) void k_wide_entropy(WideArgs a, PwPlan pl, double* __restrict__ mean_out,
                                                      double* __restrict__ ent) {
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    const int w = threadIdx.x >> 6;
    double* row = wsm + w * wide_lds_doubles(a.C);
    double* scratch = row + a.C;
    for (int64_t i = (int64_t)blockIdx.x * 4 + w; i < a.N; i += (int64_t)gridDim.x * 4) {
        const double h = wave_item_entropy<DT, KMAX>(a.p, i * a.sN, a.M, a.C, a.sM, a.sC, a.dM, a.invM, a.pow2,
                                                     pl, row, scratch, mean_out ? mean_out + i * a.C : nullptr);
        if ((threadIdx.x & 63) == 0) ent[i] = h;
    }
}

}  // namespace ce
