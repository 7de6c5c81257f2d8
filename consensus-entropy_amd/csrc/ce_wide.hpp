// ce_wide.hpp -- committees with many classes (C up to 2048, e.g. the
// 1000-class wide config): one wave per item, lanes over classes.
//
// The row sums inside scipy.stats.entropy use numpy's pairwise summation
// (leaves of <= 128 elements summed with 8 strided accumulators, combined by a
// fixed binary tree).  The host builds the tree for the call's C once
// (PwPlan: leaves + the internal nodes as rounds of lane pairs); each leaf is
// summed by 8 lanes with shuffles reproducing ((r0+r1)+(r2+r3))+((r4+r5)+
// (r6+r7)), and the tree is combined by shuffles -- the same additions in the
// same order as numpy.
#pragma once
#include "ce_device.hpp"
#include "ce_topq.hpp"

namespace ce {

constexpr int kWideMaxC = 2048;
constexpr int kPwMaxLeaves = 32;  // leaves hold 64..128 elements when n > 128: <= 32 for n <= 2048
constexpr int kPwMaxRounds = 6;   // tree height (<= 5 for n <= 2048)

// numpy's pairwise-summation tree for one n: the leaves (start, length) in
// order, and the internal nodes as rounds of lane pairs.  Every subtree's sum
// lives in the lane of its leftmost leaf; a node of height h is evaluated in
// round h-1 as lane[a] = lane[a] + lane[b] (a = its left child's leftmost
// leaf, b = its right child's), so the left operand stays on the left.
struct PwPlan {
    int n;
    int nleaves;
    int nrounds;
    short lstart[kPwMaxLeaves];
    short llen[kPwMaxLeaves];
    signed char partner[kPwMaxRounds][kPwMaxLeaves];  // round r: lane a adds lane partner[r][a]; -1 none
};

// Host: numpy's recursion (loops_utils.h.src) for n elements.  Returns the
// subtree height; *first = its leftmost leaf.
constexpr int pw_build(PwPlan& pl, int start, int n, int* first) {
    if (n <= 128) {
        *first = pl.nleaves;
        pl.lstart[pl.nleaves] = (short)start;
        pl.llen[pl.nleaves] = (short)n;
        pl.nleaves++;
        return 0;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    int a = 0, b = 0;
    const int ha = pw_build(pl, start, n2, &a);
    const int hb = pw_build(pl, start + n2, n - n2, &b);
    const int h = 1 + (ha > hb ? ha : hb);
    pl.partner[h - 1][a] = (signed char)b;
    if (h > pl.nrounds) pl.nrounds = h;
    *first = a;
    return h;
}

constexpr PwPlan pw_plan(int n) {
    PwPlan pl{};
    pl.n = n;
    for (int r = 0; r < kPwMaxRounds; ++r)
        for (int l = 0; l < kPwMaxLeaves; ++l) pl.partner[r][l] = -1;
    int first = 0;
    if (n >= 8) pw_build(pl, 0, n, &first);
    return pl;
}

// The per-wave LDS row stores element x at rp(x) = x + 2 * (x >> 5): 16 B of
// padding after every 32 doubles, so the 16 lanes of a ds_write_b64 pass (lane
// l owns the 64-B block of elements 8l .. 8l+7) land in 16 distinct bank pairs
// instead of 4 (measured: ~1,000 LDS bank-conflict cycles per item at C = 1000
// without it).  Readers walk consecutive x, so their pattern is unchanged.
__host__ __device__ __forceinline__ int rp(int x) { return x + 2 * (x >> 5); }

// Wave-cooperative np.sum(a[0:n]) over an LDS row (returns the same value in
// every lane): each leaf is summed by 8 lanes with numpy's 8 strided
// accumulators and ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), leaf l's sum moves
// to lane l, and the tree is combined in pl.nrounds shuffle rounds -- the same
// additions in the same order as numpy, no serial lane-0 section.
__device__ inline double wave_row_sum(const double* a, const PwPlan& pl, double* scratch) {
    (void)scratch;
    const int lane = threadIdx.x & 63;
    if (pl.n < 8) {
        double r = -0.0;
        for (int i = 0; i < pl.n; ++i) r += a[rp(i)];
        return 0.0 + r;  // every lane computes it (LDS broadcast reads)
    }
    double lv = 0.0;  // lane l < nleaves: leaf l's (then its subtree's) sum
    for (int l0 = 0; l0 < pl.nleaves; l0 += 8) {
        const int leaf = l0 + (lane >> 3), j = lane & 7;
        double r = 0.0;
        int st = 0, len = 0;
        if (leaf < pl.nleaves) {
            st = pl.lstart[leaf];
            len = pl.llen[leaf];
            const int nb = len - (len % 8);
            r = a[rp(st + j)];
            for (int i = 8; i < nb; i += 8) r += a[rp(st + i + j)];
        }
        r = r + __shfl_xor(r, 1);
        r = r + __shfl_xor(r, 2);
        r = r + __shfl_xor(r, 4);
        if (leaf < pl.nleaves && j == 0)
            for (int i = len - (len % 8); i < len; ++i) r += a[rp(st + i)];
        const double t = __shfl(r, ((lane - l0) & 7) << 3);
        if (lane >= l0 && lane < l0 + 8) lv = t;
    }
    for (int rd = 0; rd < pl.nrounds; ++rd) {
        const int p = lane < kPwMaxLeaves ? pl.partner[rd][lane] : -1;
        const double v = __shfl(lv, p >= 0 ? p : lane);
        if (p >= 0) lv = lv + v;
    }
    return 0.0 + __shfl(lv, 0);
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
            row[rp(c)] = acc[k];
            if (mean_out) mean_out[c] = acc[k];
        }
    }
    __builtin_amdgcn_wave_barrier();
    const double s = wave_row_sum(row, pl, scratch);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int c = lane + 64 * k;
        if (c < C) row[rp(c)] = entr(1.0 * acc[k] / s);
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
            if (ch < K) row[rp(ch * CPC + e)] = acc[kk * CPC + e];
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
            if (ch < K) row[rp(ch * CPC + e)] = entr(1.0 * acc[kk * CPC + e] / s);
    }
    __builtin_amdgcn_wave_barrier();
    const double h = wave_row_sum(row, pl, scratch);
    __builtin_amdgcn_wave_barrier();
    return h;
}

// The wide stream's approximate prefilter: the approximate entropy (log2
// units, wave-uniform) of the consensus row whose member sums sit in this
// wave's registers, from f32 copies (lane sums of KCH*CPC values + a 6-step
// butterfly, one v_rcp_f32, one v_log_f32 per class).  Error bound for C <=
// 2048: f32 copy 2^-24, row sum <= 22 roundings, v_rcp_f32 2^-22 -> the
// quotients' relative error rho <= 1.7e-6; sum_c p_c |log2 p_c| (rho + 2^-21)
// <= 11 * 2.2e-6, + 2^-20 * sum p_c, + the h sum's <= 22 roundings of <= 11:
// <= 4e-5 -- kWideApproxErr2 is 5x that.  special: a negative / -0.0 /
// non-finite sum or a row sum outside [2^-100, 2^100] (the exact path decides).
constexpr double kWideApproxErr2 = 2e-4;
template <int DT, int KCH>
__device__ __forceinline__ float wave_approx_entropy(const double* acc, int K, bool& special) {
    constexpr int CPC = ChunkT<DT>::CPC;
    const int lane = threadIdx.x & 63;
    float mf[KCH * CPC];
    uint32_t hw = 0;
    float s = 0.0f;
#pragma unroll
    for (int kk = 0; kk < KCH; ++kk) {
        const bool v = lane + 64 * kk < K;
#pragma unroll
        for (int e = 0; e < CPC; ++e) {
            const double x = v ? acc[kk * CPC + e] : 0.0;
            const uint32_t h = (uint32_t)(dbits(x) >> 32);
            hw = hw > h ? hw : h;
            mf[kk * CPC + e] = (float)x;
            s += mf[kk * CPC + e];
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);  // same value in every lane
    special = __ballot(hw >= 0x7ff00000u) != 0 || !(s >= 0x1p-100f && s <= 0x1p100f);
    const float r = __builtin_amdgcn_rcpf(s);
    float hl = 0.0f;
#pragma unroll
    for (int e = 0; e < KCH * CPC; ++e) {
        const float pc = __builtin_fmaxf(mf[e] * r, 0x1p-100f);  // absent classes: ~0
        hl = __builtin_fmaf(-pc, __builtin_amdgcn_logf(pc), hl);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) hl += __shfl_xor(hl, off);
    return hl;
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
// words, no conversion until the adds).  UNR divides M (the host picks UNR = 1
// otherwise), so every batch is full: plain in-order adds, no masking.
template <int DT, int KCH, int UNR>
struct WideBatch {
    uint32_t v[UNR][KCH][4];

    // item/m0 are wave-uniform: the member row base is made a scalar (readfirstlane)
    // so each load is SGPR base + the lane's constant 32-bit chunk offset (off[kk])
    __device__ __forceinline__ void issue(const char* item, int m0, int64_t sMb, const uint32_t (&off)[KCH]) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint64_t rb = (uint64_t)(item + (int64_t)(m0 + u) * sMb);
            const char* row = reinterpret_cast<const char*>(
                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(rb >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)rb));
#pragma unroll
            for (int kk = 0; kk < KCH; ++kk) {
                const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + off[kk]));
                v[u][kk][0] = x.x;
                v[u][kk][1] = x.y;
                v[u][kk][2] = x.z;
                v[u][kk][3] = x.w;
            }
        }
    }

    __device__ __forceinline__ void add(double* acc) const {
        constexpr int CPC = ChunkT<DT>::CPC;
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int kk = 0; kk < KCH; ++kk) chunk_add<DT>(v[u][kk], acc + kk * CPC);
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

// LDS per wave: the C-double row.
__host__ __device__ constexpr int wide_lds_doubles(int C) { return ((C + 2 * (C >> 5) + 1) / 2) * 2; }  // the padded row (16-B multiple)

}  // namespace ce
