// ce_device.hpp -- device-side arithmetic of the selection path (gfx950).
//
// Every routine here restates one piece of the reference's NumPy/SciPy arithmetic
// in f64, in the same operation order, with glibc's log restated
// (ce_glibc_log.hpp), so that the GPU path reproduces the reference bit for bit
// (see DESIGN.md "Numerics"):
//   mean      np.mean(np.array(pred_prob), axis=0)        amg_test.py:441
//   entropy   scipy.stats.entropy(consensus, axis=1)      amg_test.py:443,451,479
//   hc freq   np.round(count / n_votes, 3)                amg_test.py:115
//   quadrant  get_quadrant(arousal, valence)              amg_test.py:69-78
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ce_glibc_log.hpp"

#include "ce_debug.hpp"

namespace ce {

enum DType : int { kF32 = 0, kF64 = 1, kBF16 = 2 };

// ---------------------------------------------------------------------------
// Total order of the selection, as an unsigned 64-bit key: larger key = better.
// NaN -> max (ranked first, as argsort()[::-1] puts NaN first); -0.0 -> +0.0;
// ties on the key are broken by the lower index (the north-star rule).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t order_key(double h) {
    if (__builtin_isnan(h)) return ~0ull;
    const uint64_t b = (uint64_t)__double_as_longlong(h + 0.0);  // -0.0 + 0.0 = +0.0
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ double key_to_val(uint64_t k) {
    if (k == ~0ull) return __longlong_as_double(0x7ff8000000000000ll);
    const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
}

__device__ __forceinline__ bool better(uint64_t ka, int64_t ia, uint64_t kb, int64_t ib) {
    return ka > kb || (ka == kb && ia < ib);
}

// scipy.special.entr: NaN -> NaN, x > 0 -> -x*log(x), x == 0 -> 0, x < 0 -> -inf.
// Branch-free form: for x == 0 and x < 0 the product is replaced, so the
// log of a non-positive argument never reaches the result.  log is glibc's
// (ce_glibc_log.hpp): the calling kernel has run stage_log_table().
__device__ __forceinline__ double entr_general(double x) {
    double r = -x * dlog(x);
    r = (x == 0.0) ? 0.0 : r;
    r = (x < 0.0) ? -__builtin_inf() : r;
    return r;  // NaN input: x==0 and x<0 are false, r = -NaN*log(NaN) = NaN
}
// The common case (x normal in (0, 0.9375): every term of a row with more than
// one non-negligible class) is one multiply on the straight-line log; zeros,
// negatives, NaN, subnormals and x near 1 take entr_general -- same values.
__device__ __forceinline__ double entr(double x) {
    if (__builtin_expect(!glibc_log_common(x), 0)) return entr_general(x);
    return -x * glibc_log_core(x, s_log_tab);
}

// ---------------------------------------------------------------------------
// numpy's pairwise summation (loops_utils.h.src) over a compile-time-sized
// register array, plus the reduction identity: np.sum(row) == 0.0 + pairwise.
// ---------------------------------------------------------------------------
template <int OFF, int N, int TOT>
__device__ __forceinline__ double pairwise(const double (&a)[TOT]) {
    if constexpr (N < 8) {
        double r = -0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) r += a[OFF + i];
        return r;
    } else if constexpr (N <= 128) {
        double r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = a[OFF + j];
        constexpr int NB = N - (N % 8);
#pragma unroll
        for (int i = 8; i < NB; i += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] += a[OFF + i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
        for (int i = NB; i < N; ++i) res += a[OFF + i];
        return res;
    } else {
        constexpr int H = N / 2;
        constexpr int N2 = H - (H % 8);
        return pairwise<OFF, N2, TOT>(a) + pairwise<OFF + N2, N - N2, TOT>(a);
    }
}

template <int C>
__device__ __forceinline__ double row_sum(const double (&a)[C]) {
    return 0.0 + pairwise<0, C, C>(a);
}

// The row's C quotients x[c] / s, bit-identical to C separate IEEE
// divisions, with ONE reciprocal per row.  gfx950's f64 division (LLVM's
// lowering) is d = v_div_scale(s), n = v_div_scale(x); r = v_rcp_f64(d), two
// Newton steps r = fma(r, fma(-d, r, 1), r); q = n * r; rem = fma(-d, q, n);
// v_div_fmas(rem, r, q) = fma(rem, r, q) (+ rescale); v_div_fixup (specials).
// When every x[c] and s is positive with its exponent field in [723, 1323) --
// [2^-300, 2^300) -- both v_div_scale steps return their inputs (no operand is
// zero, tiny or huge, quotient exponents differ by < 768), v_div_fmas is a
// plain fma and v_div_fixup returns its input, so x / s == fma(fma(-s, q, x),
// r, q), q = x * r, with r the division's own refined reciprocal of s:
// 3 instructions per class instead of ~11.  Rows with a zero, a tiny or a
// negative value (and NaN / inf) take the ordinary divisions.  The range test
// is two min/max folds of the high words and one compare.  Measured: C3
// 14.24 -> 13.36 us, the C4 stream unchanged; held bit-exact by
// test_row_division_bit_exact (6e7 pairs across and beyond the range).
template <int C>
__device__ __forceinline__ void row_quotients(const double (&x)[C], double s, double (&d)[C]) {
    const uint32_t hs = (uint32_t)(dbits(s) >> 32);
    uint32_t lo = hs, hi = hs;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t h = (uint32_t)(dbits(x[c]) >> 32);
        lo = lo < h ? lo : h;
        hi = hi > h ? hi : h;
    }
    if (__builtin_expect(lo >= (723u << 20) && hi < (1323u << 20), 1)) {
        double r = __builtin_amdgcn_rcp(s);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const double q = x[c] * r;
            d[c] = __builtin_fma(__builtin_fma(-s, q, x[c]), r, q);
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) d[c] = x[c] / s;
}

// One of row_quotients' quotients, xc = x[c]: the same range test over the
// whole row, the same operations on xc -- bit-identical to d[c].
template <int C>
__device__ __forceinline__ double row_quotient_one(const double (&x)[C], double s, double xc) {
    const uint32_t hs = (uint32_t)(dbits(s) >> 32);
    uint32_t lo = hs, hi = hs;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t h = (uint32_t)(dbits(x[c]) >> 32);
        lo = lo < h ? lo : h;
        hi = hi > h ? hi : h;
    }
    if (__builtin_expect(lo >= (723u << 20) && hi < (1323u << 20), 1)) {
        double r = __builtin_amdgcn_rcp(s);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
        const double q = xc * r;
        return __builtin_fma(__builtin_fma(-s, q, xc), r, q);
    }
    return xc / s;
}

// scipy.stats.entropy of one row held in registers (mean: consensus row).
template <int C>
__device__ __forceinline__ double entropy_row(const double (&mean)[C]) {
    const double s = row_sum<C>(mean);
    double e[C];
    if constexpr (C <= 8) {
        double d[C];
        row_quotients<C>(mean, s, d);
#pragma unroll
        for (int c = 0; c < C; ++c) e[c] = entr(d[c]);
        return row_sum<C>(e);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) e[c] = entr(1.0 * mean[c] / s);
    return row_sum<C>(e);
}

// Approximate entropy error bound, log2 units, per class: f32 copies of the
// exact means (2^-24), their f32 sum (C-1 roundings), v_rcp_f32 and v_log_f32
// (taken as 2^-22 and 2^-21 relative + 2^-20 absolute) give at most ~1.4e-6 *
// C + 2.1e-6; the bound used is ~8x that, and
// tests/test_gpu_parity.py::test_approx_entropy_bound (via ce_approx_entropy) measures the device's
// actual error against it.
constexpr float kApproxErr2PerClass = 2e-5f;

// The approximate entropy of an exact row as a 32-bit order key (0: never a
// valid result), and whether the row is special (the exact path decides).
template <int C>
__device__ __forceinline__ uint32_t approx_key(const double (&m)[C], bool& special) {
    float mf[C];
    uint32_t hw = 0;
    float S = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t h = (uint32_t)(dbits(m[c]) >> 32);
        hw = hw > h ? hw : h;  // sign set (negative, -0.0), inf / NaN: >= 0x7ff00000
        mf[c] = (float)m[c];
        S += mf[c];
    }
    special = hw >= 0x7ff00000u || !(S >= 0x1p-100f && S <= 0x1p100f);
    const float r = __builtin_amdgcn_rcpf(S);
    float h = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const float pc = __builtin_fmaxf(mf[c] * r, 0x1p-100f);
        h = __builtin_fmaf(-pc, __builtin_amdgcn_logf(pc), h);
    }
    const uint32_t b = __float_as_uint(h);
    return (b >> 31) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ float approx_key_value(uint32_t k) {
    return __uint_as_float((k >> 31) ? (k & 0x7fffffffu) : ~k);
}

// mean = acc / M as numpy's true_divide; a power-of-two M divides exactly by a
// multiply with its (exact) reciprocal, which rounds identically.
__device__ __forceinline__ double div_members(double acc, double dM, double invM, bool pow2) {
    return pow2 ? acc * invM : acc / dM;
}

// np.round(count / n, 3) == rint(x * 1000.0) / 1000.0 with x = count / n in f64.
__device__ __forceinline__ double round3(double x) { return rint(x * 1000.0) / 1000.0; }

// amg_test.py:69-78; -1 when either value is NaN (dropna() at :101).
__device__ __forceinline__ int quadrant(double arousal, double valence) {
    if (__builtin_isnan(arousal) || __builtin_isnan(valence)) return -1;
    if (arousal >= 0.0 && valence >= 0.0) return 0;
    if (arousal > 0.0 && valence < 0.0) return 1;
    if (arousal <= 0.0 && valence <= 0.0) return 2;
    return 3;  // arousal < 0 && valence > 0: the only case left for non-NaN input
}

__device__ __forceinline__ double bf16_to_f64(uint32_t h16) {
    return (double)__uint_as_float(h16 << 16);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// Loads of one member's C class probabilities of one item, widened to f64.
// VEC: C contiguous and 16-B (f32/f64) / 8-B (bf16) aligned -> vector loads.
// ---------------------------------------------------------------------------
// the member loads' cache policy: non-temporal (1, default) or plain (0; A/B builds)
#ifndef CE_MEMBER_NT
#define CE_MEMBER_NT 1
#endif
template <class T>
__device__ __forceinline__ T member_ld(const T* p) {
#if CE_MEMBER_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

template <int DT, int C, bool VEC>
struct MemberLoad;

template <int C>
struct MemberLoad<kF32, C, true> {
    static_assert(C % 4 == 0, "");
    f32x4 v[C / 4];
    __device__ __forceinline__ void load(const void* base, int64_t off, int64_t) {
        const f32x4* p = reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + off);
#pragma unroll
        for (int k = 0; k < C / 4; ++k) v[k] = member_ld(p + k);
    }
    __device__ __forceinline__ void pin() const {
#pragma unroll
        for (int k = 0; k < C / 4; ++k) asm volatile("" ::"v"(v[k]));
    }
    __device__ __forceinline__ void add_to(double (&acc)[C]) const {
#pragma unroll
        for (int k = 0; k < C / 4; ++k) {
            acc[4 * k + 0] += (double)v[k].x;
            acc[4 * k + 1] += (double)v[k].y;
            acc[4 * k + 2] += (double)v[k].z;
            acc[4 * k + 3] += (double)v[k].w;
        }
    }
    __device__ __forceinline__ void add_masked(double (&acc)[C], bool live) const {
#pragma unroll
        for (int k = 0; k < C / 4; ++k) {
            acc[4 * k + 0] += live ? (double)v[k].x : 0.0;
            acc[4 * k + 1] += live ? (double)v[k].y : 0.0;
            acc[4 * k + 2] += live ? (double)v[k].z : 0.0;
            acc[4 * k + 3] += live ? (double)v[k].w : 0.0;
        }
    }
};

template <int C>
struct MemberLoad<kF64, C, true> {
    static_assert(C % 2 == 0, "");
    f64x2 v[C / 2];
    __device__ __forceinline__ void load(const void* base, int64_t off, int64_t) {
        const f64x2* p = reinterpret_cast<const f64x2*>(static_cast<const double*>(base) + off);
#pragma unroll
        for (int k = 0; k < C / 2; ++k) v[k] = member_ld(p + k);
    }
    __device__ __forceinline__ void pin() const {
#pragma unroll
        for (int k = 0; k < C / 2; ++k) asm volatile("" ::"v"(v[k]));
    }
    __device__ __forceinline__ void add_to(double (&acc)[C]) const {
#pragma unroll
        for (int k = 0; k < C / 2; ++k) {
            acc[2 * k + 0] += v[k].x;
            acc[2 * k + 1] += v[k].y;
        }
    }
    __device__ __forceinline__ void add_masked(double (&acc)[C], bool live) const {
#pragma unroll
        for (int k = 0; k < C / 2; ++k) {
            acc[2 * k + 0] += live ? v[k].x : 0.0;
            acc[2 * k + 1] += live ? v[k].y : 0.0;
        }
    }
};

template <int C>
struct MemberLoad<kBF16, C, true> {
    static_assert(C % 4 == 0, "");
    u32x2 v[C / 4];
    __device__ __forceinline__ void load(const void* base, int64_t off, int64_t) {
        const u32x2* p = reinterpret_cast<const u32x2*>(static_cast<const uint16_t*>(base) + off);
#pragma unroll
        for (int k = 0; k < C / 4; ++k) v[k] = member_ld(p + k);
    }
    __device__ __forceinline__ void pin() const {
#pragma unroll
        for (int k = 0; k < C / 4; ++k) asm volatile("" ::"v"(v[k]));
    }
    __device__ __forceinline__ void add_to(double (&acc)[C]) const {
#pragma unroll
        for (int k = 0; k < C / 4; ++k) {
            acc[4 * k + 0] += bf16_to_f64(v[k].x & 0xffffu);
            acc[4 * k + 1] += bf16_to_f64(v[k].x >> 16);
            acc[4 * k + 2] += bf16_to_f64(v[k].y & 0xffffu);
            acc[4 * k + 3] += bf16_to_f64(v[k].y >> 16);
        }
    }
    __device__ __forceinline__ void add_masked(double (&acc)[C], bool live) const {
#pragma unroll
        for (int k = 0; k < C / 4; ++k) {
            acc[4 * k + 0] += live ? bf16_to_f64(v[k].x & 0xffffu) : 0.0;
            acc[4 * k + 1] += live ? bf16_to_f64(v[k].x >> 16) : 0.0;
            acc[4 * k + 2] += live ? bf16_to_f64(v[k].y & 0xffffu) : 0.0;
            acc[4 * k + 3] += live ? bf16_to_f64(v[k].y >> 16) : 0.0;
        }
    }
};

// Scalar (any stride / alignment) variant.
template <int DT, int C>
struct MemberLoad<DT, C, false> {
    double v[C];
    __device__ __forceinline__ void load(const void* base, int64_t off, int64_t sC) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int64_t o = off + c * sC;
            if constexpr (DT == kF32)
                v[c] = (double)static_cast<const float*>(base)[o];
            else if constexpr (DT == kF64)
                v[c] = static_cast<const double*>(base)[o];
            else
                v[c] = bf16_to_f64(static_cast<const uint16_t*>(base)[o]);
        }
    }
    __device__ __forceinline__ void pin() const {
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("" ::"v"(v[c]));
    }
    __device__ __forceinline__ void add_to(double (&acc)[C]) const {
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += v[c];
    }
    __device__ __forceinline__ void add_masked(double (&acc)[C], bool live) const {
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += live ? v[c] : 0.0;
    }
};

// Consensus means of IPL items over M members, member-sequential per item
// (amg_test.py:441).  Members are loaded in batches of UNR for all IPL items
// before any add, so UNR*IPL loads are in flight per lane.  A batch past M
// re-loads member M-1 (always in bounds, no branch around a load) and adds
// +0.0 instead: acc starts at +0.0 and a round-to-nearest sum is -0.0 only if
// both operands are, so acc is never -0.0 and x + 0.0 == x exactly -- the
// padding is a bit-exact no-op.
template <int DT, int C, bool VEC, int UNR, int IPL>
__device__ __forceinline__ void committee_mean_multi(const void* p, const int64_t (&item_off)[IPL], int M,
                                                     int64_t sM, int64_t sC, double dM, double invM, bool pow2,
                                                     double (&mean)[IPL][C]) {
    double acc[IPL][C];
#pragma unroll
    for (int u = 0; u < IPL; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[u][c] = 0.0;  // np.add.reduce identity
    for (int m0 = 0; m0 < M; m0 += UNR) {
        MemberLoad<DT, C, VEC> ld[IPL][UNR];
#pragma unroll
        for (int v = 0; v < UNR; ++v) {
            const int m = m0 + v < M ? m0 + v : M - 1;
#pragma unroll
            for (int u = 0; u < IPL; ++u) ld[u][v].load(p, item_off[u] + (int64_t)m * sM, sC);
        }
#pragma unroll
        for (int v = 0; v < UNR; ++v) {
            const bool live = m0 + v < M;
#pragma unroll
            for (int u = 0; u < IPL; ++u) ld[u][v].add_masked(acc[u], live);
        }
    }
#pragma unroll
    for (int u = 0; u < IPL; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) mean[u][c] = div_members(acc[u][c], dM, invM, pow2);
}

template <int DT, int C, bool VEC, int UNR>
__device__ __forceinline__ void committee_mean(const void* p, int64_t item_off, int M, int64_t sM, int64_t sC,
                                               double dM, double invM, bool pow2, double (&mean)[C]) {
    const int64_t offs[1] = {item_off};
    double m1[1][C];
    committee_mean_multi<DT, C, VEC, UNR, 1>(p, offs, M, sM, sC, dM, invM, pow2, m1);
#pragma unroll
    for (int c = 0; c < C; ++c) mean[c] = m1[0][c];
}

}  // namespace ce
