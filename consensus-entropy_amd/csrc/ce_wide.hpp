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

// Vectorised variant: member rows of C*size bytes, 16-B aligned, C*size % 16
// == 0.  Lane l owns 16-B chunks l, l+64, ... (CPC classes each); UNR member
// rows are in flight per lane before the in-order adds.
template <int DT>
struct ChunkT;
template <>
struct ChunkT<kF32> {
    static constexpr int CPC = 4;
};
template <>
struct ChunkT<kF64> {
    static constexpr int CPC = 2;
};
template <>
struct ChunkT<kBF16> {
    static constexpr int CPC = 8;
};

template <int DT>
__device__ __forceinline__ void chunk_add(const uint32_t (&u)[4], double* acc) {
    if constexpr (DT == kF32) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += (double)__uint_as_float(u[e]);
    } else if constexpr (DT == kF64) {
#pragma unroll
        for (int e = 0; e < 2; ++e)
            acc[e] += __longlong_as_double((long long)(((uint64_t)u[2 * e + 1] << 32) | u[2 * e]));
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf16_to_f64((u[e >> 1] >> (16 * (e & 1))) & 0xffffu);
    }
}

template <int DT>
__device__ __forceinline__ void chunk_add_masked(const uint32_t (&u)[4], double* acc, bool live) {
    if constexpr (DT == kF32) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += live ? (double)__uint_as_float(u[e]) : 0.0;
    } else if constexpr (DT == kF64) {
#pragma unroll
        for (int e = 0; e < 2; ++e)
            acc[e] += live ? __longlong_as_double((long long)(((uint64_t)u[2 * e + 1] << 32) | u[2 * e])) : 0.0;
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += live ? bf16_to_f64((u[e >> 1] >> (16 * (e & 1))) & 0xffffu) : 0.0;
    }
}

// scipy.stats.entropy of the consensus row whose member sums sit in this
// wave's registers (lane l: chunks l, l+64, ... of CPC classes each), via the
// per-wave LDS row: mean = acc / M, row sum, entr, row sum (amg_test.py:441-443).
template <int DT, int KCH>
__device__ __forceinline__ double wave_entropy_from_sums(double* acc, int K, double dM, double invM, bool pow2,
                                                        const PwPlan& pl, double* row, double* scratch) {
    // acc is overwritten with the mean row (its last use), saving KCH*CPC registers
    constexpr int CPC = ChunkT<DT>::CPC;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int kk = 0; kk < KCH; ++kk) {
        const int ch = lane + 64 * kk;
#pragma unroll
        for (int e = 0; e < CPC; ++e) {
            acc[kk * CPC + e] = div_members(acc[kk * CPC + e], dM, invM, pow2);
            if (ch < K) row[ch * CPC + e] = acc[kk * CPC + e];
        }
    }
    __builtin_amdgcn_wave_barrier();
    const double s = wave_row_sum(row, pl, scratch);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int kk = 0; kk < KCH; ++kk) {
        const int ch = lane + 64 * kk;
#pragma unroll
        for (int e = 0; e < CPC; ++e)
            if (ch < K) row[ch * CPC + e] = entr(1.0 * acc[kk * CPC + e] / s);
    }
    __builtin_amdgcn_wave_barrier();
    const double h = wave_row_sum(row, pl, scratch);
    __builtin_amdgcn_wave_barrier();
    return h;
}

template <int DT, int KCH, int UNR>
__device__ inline double wave_item_entropy_vec(const void* p, int64_t off, int M, int C, int64_t sM, double dM,
                                               double invM, bool pow2, const PwPlan& pl, double* row,
                                               double* scratch) {
    constexpr int CPC = ChunkT<DT>::CPC;
    constexpr int EB = 16 / CPC;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int K = C / CPC;  // chunks per member row
    const char* base = static_cast<const char*>(p) + off * EB;
    double acc[KCH * CPC];
#pragma unroll
    for (int e = 0; e < KCH * CPC; ++e) acc[e] = 0.0;
    int m = 0;
    for (; m + UNR <= M; m += UNR) {
        uint32_t v[UNR][KCH][4];
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int kk = 0; kk < KCH; ++kk) {
                const int ch = lane + 64 * kk;
                const int chs = ch < K ? ch : K - 1;
                const u32x4 x = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4*>(base + ((int64_t)(m + u) * sM) * EB) + chs);
                v[u][kk][0] = x.x;
                v[u][kk][1] = x.y;
                v[u][kk][2] = x.z;
                v[u][kk][3] = x.w;
            }
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int kk = 0; kk < KCH; ++kk) chunk_add<DT>(v[u][kk], acc + kk * CPC);
    }
    for (; m < M; ++m) {
#pragma unroll
        for (int kk = 0; kk < KCH; ++kk) {
            const int ch = lane + 64 * kk;
            const int chs = ch < K ? ch : K - 1;
            const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + ((int64_t)m * sM) * EB) + chs);
            const uint32_t t[4] = {x.x, x.y, x.z, x.w};
            chunk_add<DT>(t, acc + kk * CPC);
        }
    }
    return wave_entropy_from_sums<DT, KCH>(acc, K, dM, invM, pow2, pl, row, scratch);
}

// One batch of UNR member rows x KCH 16-B chunks per lane of one item (raw
// words, no conversion until the adds).  Members past M re-load member M-1
// (in bounds) and are added as +0.0 (bit-exact no-op, see committee_mean_multi).
template <int DT, int KCH, int UNR>
struct WideBatch {
    uint32_t v[UNR][KCH][4];

    __device__ __forceinline__ void issue(const char* item, int m0, int M, int64_t sMb, int K) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int m = m0 + u < M ? m0 + u : M - 1;
#pragma unroll
            for (int kk = 0; kk < KCH; ++kk) {
                const int ch = lane + 64 * kk;
                const int chs = ch < K ? ch : K - 1;
                const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(item + (int64_t)m * sMb) + chs);
                v[u][kk][0] = x.x;
                v[u][kk][1] = x.y;
                v[u][kk][2] = x.z;
                v[u][kk][3] = x.w;
            }
        }
    }

    __device__ __forceinline__ void add(double* acc, int m0, int M) const {
        constexpr int CPC = ChunkT<DT>::CPC;
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const bool live = m0 + u < M;
#pragma unroll
            for (int kk = 0; kk < KCH; ++kk) chunk_add_masked<DT>(v[u][kk], acc + kk * CPC, live);
        }
    }
};

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

}  // namespace ce
