// ce_xgb.hip -- on-device XGBClassifier.predict_proba (the
// 'classifier_xgb' committee member: amg_test.py:435 / :467 ->
// xgboost/sklearn.py:991-1029 -> libxgboost 1.3.3, requirements.txt:50).
//
// What the reference computes (xgboost 1.3.3 CPU predictor, restated):
//   * DMatrix(X): X (f64 DataFrame values) cast to float32 (round to nearest);
//     NaN = missing (sklearn.py:1020, missing=np.nan);
//   * per row, margins preds[g] start at the base margin (base_score for
//     multi:softprob; ProbToMargin(base_score) = -logf(1/b - 1) for
//     binary:logistic) and every tree, IN MODEL ORDER, adds its leaf to the
//     margin of its group tree_info[t]: preds[g] += leaf (float32, sequential);
//   * a tree is walked from the root: missing feature -> the default child,
//     else fvalue < split_cond ? left : right (RegTree::GetNext);
//   * multi:softprob: Softmax over the row (fmaxf maximum; e_c = expf(m_c - max);
//     wsum += e_c in float32 from 0; e_c /= wsum); binary:logistic:
//     p = 1 / (1 + expf(-m)), returned as [1 - p, p] (sklearn.py:1027-1029).
//   * expf is glibc's (>= 2.27, the x86-64 FMA ifunc variant): restated below
//     and verified bit-identical to the host's libm on all 2^32 floats
//     (tests/test_xgb.py on a dense stride, tests/test_gpu_xgb.py exhaustively
//     on the device).
//
// Layout (packed on the host by ce_amd.xgb.XgbForest): every tree is padded to
// a perfect binary tree of the forest's maximum depth d (an early leaf's
// subtree repeats its value, so either branch below it reaches the same leaf);
// internal node i has children 2i+1 / 2i+2.  Trees are stored group-major
// (group g owns trees [goff[g], goff[g+1]), model order kept inside a group,
// which is exactly the order the reference adds them to preds[g]).
//   nodes  [T][2^d - 1] x {feature | default_left << 31, split_cond bits}
//   leaves [T][2^d] f32
//
// Kernel (k_xgb_walk): one block of G x S waves per 64-frame tile.  The tile's
// features are staged ONCE as float32 in LDS, feature-major [D][65] (lane =
// frame).  Each group's trees are split over S waves whose partial chains are
// joined in model order (split_margins); every wave walks 8 trees at a time so
// 8 independent node-gather -> LDS-read -> compare chains are in flight per
// lane.  Bound: latency of those chains (X bytes from HBM, D * sizeof(x) per
// frame, are read once; T * d node steps per frame).
#include <hip/hip_runtime.h>

#include "ce_debug.hpp"
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "../../include/ce.h"
#include "ce_abi.hpp"

namespace ce {

constexpr int kXgbTile = 64;      // frames per block
// LDS tile: feature-major columns of 64 floats, frame r of feature f at f*64 +
// (r ^ (f & 63)) -- the XOR swizzle keeps the staging writes (consecutive
// features of one frame) conflict-free, and a column read by 64 lanes is a
// permutation of one column (conflict-free too).  Byte address of (f, lane):
// fbase(f) ^ 4*lane with fbase(f) = 256 f + 4 (f & 63).
constexpr int kXgbCol = 64;
__device__ __forceinline__ uint32_t xs_fbase(uint32_t f) { return f * 256u + ((f & 63u) << 2); }
__device__ __forceinline__ float xs_at(const float* xs, uint32_t fbase, uint32_t lane4) {
    return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(xs) + (fbase ^ lane4));
}
constexpr int kXgbMaxDepth = 10;  // packed depth limit (2^10 leaves per tree)
constexpr int kXgbLaneDepth = 5;  // lane-table walk: 2^(d+1) - 1 entries fit one wave
constexpr int kXgbMaxFeat = 512;
constexpr int kXgbMaxGroups = 8;
// level 1 of every tree from the wave-uniform node pair {1, 2} (one scalar
// load per tree, picked per lane): 5.45 -> 4.88 ms at 4M frames
constexpr bool kXgbScalarL1 = true;

// glibc expf (sysdeps/ieee754/flt-32/e_expf.c, EXP2F_TABLE_BITS = 5), as the
// x86-64 FMA ifunc variant evaluates it: tab[i] = bits(2^(i/32)) - (i << 52) / 32.
__constant__ uint64_t kExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

__device__ __forceinline__ float glibc_expf(float x) {
    const uint32_t ux = __float_as_uint(x);
    const uint32_t abstop = (ux >> 20) & 0x7ff;
    if (abstop >= 0x42bu) {  // |x| >= 88 or NaN
        if (ux == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8u) return x + x;
        if (x > 0x1.62e42ep6f) return __uint_as_float(0x7f800000u);
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    constexpr double kN = 32.0;
    const double inv_ln2_n = 0x1.71547652b82fep+0 * kN;
    const double c0 = 0x1.c6af84b912394p-5 / kN / kN / kN, c1 = 0x1.ebfce50fac4f3p-3 / kN / kN,
                 c2 = 0x1.62e42ff0c52d6p-1 / kN;
    const double shift = 0x1.8p+52;
    const double xd = (double)x;
    const double z = inv_ln2_n * xd;
    double kd = z + shift;
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd -= shift;
    const double r = __builtin_fma(inv_ln2_n, xd, -kd);  // the FMA build contracts z - kd
    uint64_t t = kExp2fTab[ki % 32];
    t += ki << (52 - 5);
    const double s = __longlong_as_double((long long)t);
    const double zz = __builtin_fma(c0, r, c1);
    const double r2 = r * r;
    double y = __builtin_fma(c2, r, 1.0);
    y = __builtin_fma(zz, r2, y);
    y = y * s;
    return (float)y;
}

struct XgbArgs {
    const void* X;
    int64_t F;
    int D;
    int64_t ld;
    int G, C, S;  // groups, classes, waves per group
    float base;
    void* out;
    int64_t ldo;
};

// Stage frames [f0, f0 + 64) of X as float32 into LDS, feature-major [D][64]
// swizzled (kXgbCol): wave w takes rows w, w + W, ..., its lanes consecutive
// features of a row (coalesced loads; conflict-free writes: bank r ^ lane), 2
// rows x 8 feature chunks per lane in flight; rows past the end repeat the
// last frame.  No index division: the round-5 loop's e / D cost ~40 VALU per
// element -- a third of the kernel's VALU (PMC r06).
// Returns whether this thread staged a NaN (missing value).
template <int XDT, int KF = kXgbMaxFeat / 64>  // KF: 64-feature chunks per row, >= ceil(D / 64)
__device__ __forceinline__ bool stage_tile(const void* X, int64_t F, int D, int64_t ld, int64_t f0, int nf,
                                           float* xs) {
    (void)F;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, W = blockDim.x >> 6;
    bool has_nan = false;
    for (int r0 = w; r0 < kXgbTile; r0 += 2 * W) {  // wave-uniform
        // every load unconditional (clamped row / feature): a load under a branch
        // gets its own s_waitcnt vmcnt(0), serialising the 16 round trips
        typename std::conditional<XDT == CE_F64, double, float>::type v[2][KF];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = min(r0 + h * W, kXgbTile - 1);
            const int64_t row = f0 + min(r, nf - 1);
#pragma unroll
            for (int k = 0; k < KF; ++k) {
                const int f = min(lane + 64 * k, D - 1);
                if constexpr (XDT == CE_F64)
                    v[h][k] = static_cast<const double*>(X)[row * ld + f];
                else
                    v[h][k] = static_cast<const float*>(X)[row * ld + f];
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = r0 + h * W;
#pragma unroll
            for (int k = 0; k < KF; ++k) {
                const int f = lane + 64 * k;
                if (f < D && r < kXgbTile) {
                    const float x = (float)v[h][k];
                    xs[f * kXgbCol + (r ^ lane)] = x;  // (f & 63) == lane
                    has_nan |= __builtin_isnan(x);
                }
            }
        }
    }
    return has_nan;
}

// f64 frames, two features per lane (16-B loads: half the load instructions of
// stage_tile for the same bytes): lane l takes features 2 l, 2 l + 1 of each
// 128-feature chunk; the pair is clamped to start <= D - 2 (D >= 2), so every
// load stays inside the row and is unconditional.  A/B on one box
// (profiles/r06_xgb.json): 3.279 -> 3.245 ms at 4M frames (dense), 3.418 ->
// 3.390 ms (missing values).
#ifndef CE_XGB_PAIRS
#define CE_XGB_PAIRS 1
#endif
template <int KP>  // KP: 128-feature chunks per row, >= ceil(D / 128)
__device__ __forceinline__ bool stage_tile_pairs(const double* X, int D, int64_t ld, int64_t f0, int nf, float* xs) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, W = blockDim.x >> 6;
    bool has_nan = false;
    for (int r0 = w; r0 < kXgbTile; r0 += 2 * W) {  // wave-uniform
        double2 v[2][KP];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = min(r0 + h * W, kXgbTile - 1);
            const int64_t row = f0 + min(r, nf - 1);
#pragma unroll
            for (int k = 0; k < KP; ++k) {
                const int fl = min(2 * lane + 128 * k, D - 2);
                const double* src = X + row * ld + fl;
                v[h][k] = make_double2(src[0], src[1]);
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = r0 + h * W;
#pragma unroll
            for (int k = 0; k < KP; ++k) {
                const int f = 2 * lane + 128 * k, fl = min(f, D - 2);
                if (r < kXgbTile) {
                    if (f < D) {  // f > fl only for f = D - 1 (odd D): the pair's second value
                        const float x = (float)(f == fl ? v[h][k].x : v[h][k].y);
                        xs[f * kXgbCol + (r ^ (f & 63))] = x;
                        has_nan |= __builtin_isnan(x);
                    }
                    if (f + 1 < D && f == fl) {
                        const float x = (float)v[h][k].y;
                        xs[(f + 1) * kXgbCol + (r ^ ((f + 1) & 63))] = x;
                        has_nan |= __builtin_isnan(x);
                    }
                }
            }
        }
    }
    return has_nan;
}

// The objective's transform of the G margins mg[g * 64 + lane] of frame f0 +
// lane, written to out (wave 0, one frame per lane).
template <int ODT>
__device__ __forceinline__ void transform_store(const float* mg, int G, int C, int64_t f0, int nf, void* out,
                                                int64_t ldo) {
    const int lane = threadIdx.x & 63;
    if (threadIdx.x >= 64 || lane >= nf) return;
    const int64_t fr = f0 + lane;
    float p[kXgbMaxGroups];
    if (G == 1) {  // binary:logistic -> [1 - p, p]
        const float m = mg[lane];
        const float p1 = 1.0f / (1.0f + glibc_expf(-m));
        p[0] = 1.0f - p1;
        p[1] = p1;
    } else {  // multi:softprob -> common::Softmax (xgboost src/common/math.h)
        float mx = mg[lane];
        for (int g = 1; g < G; ++g) mx = fmaxf(mg[g * 64 + lane], mx);
        double wsum = 0.0;  // xgboost: double wsum = 0.0f; ... *i /= static_cast<float>(wsum)
        for (int g = 0; g < G; ++g) {
            p[g] = glibc_expf(mg[g * 64 + lane] - mx);
            wsum += p[g];
        }
        const float ws = (float)wsum;
        for (int g = 0; g < G; ++g) p[g] /= ws;
    }
    for (int c = 0; c < C; ++c) {
        if constexpr (ODT == CE_F64)
            static_cast<double*>(out)[fr * ldo + c] = (double)p[c];
        else
            static_cast<float*>(out)[fr * ldo + c] = p[c];
    }
}

// ---- forest layouts: leaf values of 8 consecutive trees of one group --------
// MISS: the tile holds a missing value somewhere (block-uniform).  Without
// one, "missing -> default child" never fires and the test is !(x < split).

// Perfect-tree walk (any tree of depth <= 10): 8 trees walked together, so 8
// independent node-gather -> LDS-read -> compare chains are in flight.
struct WalkForest {
    const uint2* nodes;   // [T][NI] {feature | default_left << 31, split_cond bits}
    const float* leaves;  // [T][NI + 1]
    const int32_t* goff;  // [G + 1]
    int depth, NI;
    int goff_end;         // T = goff[G] trees (debug bounds checks only)

    template <bool MISS>
    static __device__ __forceinline__ bool go_right(uint2 nd, const float* xs, int D, int lane) {
        const int ft = min((int)(nd.x & 0x7fffffffu), D - 1);  // packer checks < D
        const float x = xs_at(xs, xs_fbase((uint32_t)ft), 4u * (uint32_t)lane);
        const float th = __uint_as_float(nd.y);
        if constexpr (MISS)  // missing -> default child; else fvalue < split_cond ? left : right
            return __builtin_isnan(x) ? (nd.x >> 31) == 0u : !(x < th);
        else
            return !(x < th);
    }

    // Level 0 reads the wave-uniform root (a scalar load; its feature read is
    // one LDS column); deeper levels gather per lane.
    template <bool MISS>
    __device__ __forceinline__ void leafidx8(const float* xs, int D, int t0, int t1, int lane, int (&li)[8]) const {
        int idx[8];
        const uint2* tn[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int t = t0 + j < t1 ? t0 + j : t1 - 1;
            tn[j] = nodes + (int64_t)t * NI;
            idx[j] = 0;
        }
        if (depth >= 1) {
            uint2 r[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = tn[j][0];
#pragma unroll
            for (int j = 0; j < 8; ++j) idx[j] = go_right<MISS>(r[j], xs, D, lane) ? 2 : 1;
        }
        int lev0 = 1;
        if (depth >= 2 && kXgbScalarL1) {
            // level 1 from the wave-uniform pair {node 1, node 2} (scalar loads) and a
            // per-lane select: one gather instruction fewer per tree (the walk is
            // bound by the texture path's address rate: TA 79 % busy; 4M frames
            // 5.45 -> 4.88 ms).  Level 2 the same way (4 nodes, two selects) was
            // slower (5.18 ms): the extra VALU outweighs the saved gather.
            // nodes 1 and 2 as two 8-B loads: a tree holds 2^d - 1 nodes (odd), so
            // node 1 of every other tree is only 8-byte aligned (the compiler
            // still merges the pair into one scalar load where it can)
            uint2 n1[8], n2[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                n1[j] = tn[j][1];
                n2[j] = tn[j][2];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint2 nd = idx[j] == 1 ? n1[j] : n2[j];
                idx[j] = 2 * idx[j] + 1 + (go_right<MISS>(nd, xs, D, lane) ? 1 : 0);
            }
            lev0 = 2;
        }
        for (int lev = lev0; lev < depth; ++lev) {
            uint2 nd[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                CE_DASSERT(idx[j] >= 0 && idx[j] < NI);  // an inner node
                nd[j] = tn[j][idx[j]];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) idx[j] = 2 * idx[j] + 1 + (go_right<MISS>(nd[j], xs, D, lane) ? 1 : 0);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            li[j] = idx[j] - NI;
            CE_DASSERT(li[j] >= 0 && li[j] <= NI);  // a leaf of a perfect tree of depth `depth`
        }
    }
    // leaf value of tree t at leaf index li
    __device__ __forceinline__ float value(int t, int li) const {
        CE_DASSERT(t >= 0 && t < goff_end && li >= 0 && li <= NI);
        return leaves[(int64_t)t * (NI + 1) + li];
    }
    // trees [t0, min(t0 + 8, t1)): leaf indices, and (VALS) their leaf values
    template <bool MISS, bool VALS>
    __device__ __forceinline__ void walk8(const float* xs, int D, int t0, int t1, int lane, int (&li)[8],
                                          float (&v)[8]) const {
        leafidx8<MISS>(xs, D, t0, t1, lane, li);
        if constexpr (VALS) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = value(t0 + j < t1 ? t0 + j : t1 - 1, li[j]);
        }
    }
};

// Lane-table walk (perfect trees of depth <= 5: 2^d - 1 nodes + 2^d leaves <=
// 63 entries, the reference's XGBClassifier(max_depth=5)).  A tree's table is
// read with two COALESCED loads -- lane i holds entry i: node i (i < NI) or
// leaf i - NI (NI <= i <= 2 NI) -- and each level fetches every lane's current
// node from the table with ds_bpermute (the LDS crossbar: no memory access,
// no address chain through L2): 2 loads per tree instead of 1 scalar pair + 3
// per-lane gathers + 1 leaf gather on the texture path the walk was bound by
// (TA 74-79 % busy).  The node's feature is kept as its LDS
// column base (xs_fbase, the clamp to D - 1 done once), so a level is two
// bpermutes, one XOR, one ds_read, one compare and the index update.  The
// root (entry 0) is read with v_readlane: wave-uniform.
struct LaneForest {
    const uint2* nodes;   // [T][NI]
    const float* leaves;  // [T][NI + 1]
    const int32_t* goff;
    int depth, NI;
    int goff_end;

    // this lane's table entry of tree t: fx = xs_fbase(feature) (| default_left << 31
    // when MISS), ty = the split condition's bits; at a leaf entry fx = 0, ty = the
    // leaf value's bits; past the table both 0
    template <bool MISS>
    __device__ __forceinline__ void entry(int t, int D, int lane, uint32_t& fx, uint32_t& ty) const {
        fx = 0u;
        ty = 0u;
        if (lane < NI) {
            const uint2 nd = nodes[(int64_t)t * NI + lane];
            const uint32_t ft = min(nd.x & 0x7fffffffu, (uint32_t)(D - 1));  // packer checks < D
            fx = xs_fbase(ft) | (MISS ? (nd.x & 0x80000000u) : 0u);
            ty = nd.y;
        } else if (lane <= 2 * NI) {
            ty = __float_as_uint(leaves[(int64_t)t * (NI + 1) + (lane - NI)]);
        }
    }
    template <bool MISS>
    static __device__ __forceinline__ bool right(uint32_t fx, uint32_t th, const float* xs, uint32_t lane4) {
        const float x = xs_at(xs, MISS ? (fx & 0x7fffffffu) : fx, lane4);
        if constexpr (MISS)  // missing -> default child; else fvalue < split_cond ? left : right
            return __builtin_isnan(x) ? (fx >> 31) == 0u : !(x < __uint_as_float(th));
        else
            return !(x < __uint_as_float(th));
    }
    static __device__ __forceinline__ uint32_t bperm(int idx4, uint32_t v) {
        return (uint32_t)__builtin_amdgcn_ds_bpermute(idx4, (int)v);
    }
    template <bool MISS, bool VALS>
    __device__ __forceinline__ void walk8(const float* xs, int D, int t0, int t1, int lane, int (&li)[8],
                                          float (&v)[8]) const {
        uint32_t fx[8], ty[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) entry<MISS>(t0 + j < t1 ? t0 + j : t1 - 1, D, lane, fx[j], ty[j]);
        const uint32_t lane4 = 4u * (uint32_t)lane;
        int idx4[8];  // 4 x the lane's node index (a ds_bpermute byte address); children 2 idx4 + 4 / + 8
#pragma unroll
        for (int j = 0; j < 8; ++j) idx4[j] = 0;
        if (depth >= 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane((int)fx[j], 0);
                const uint32_t h0 = (uint32_t)__builtin_amdgcn_readlane((int)ty[j], 0);
                idx4[j] = right<MISS>(f0, h0, xs, lane4) ? 8 : 4;
            }
        }
        for (int lev = 1; lev < depth; ++lev) {
            uint32_t f[8], h[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                f[j] = bperm(idx4[j], fx[j]);
                h[j] = bperm(idx4[j], ty[j]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) idx4[j] = 2 * idx4[j] + (right<MISS>(f[j], h[j], xs, lane4) ? 8 : 4);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            li[j] = (idx4[j] >> 2) - NI;
            CE_DASSERT(li[j] >= 0 && li[j] <= NI);
        }
        if constexpr (VALS) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(bperm(idx4[j], ty[j]));
        }
    }
    __device__ __forceinline__ float value(int t, int li) const {
        CE_DASSERT(t >= 0 && t < goff_end && li >= 0 && li <= NI);
        return leaves[(int64_t)t * (NI + 1) + li];
    }
};

// Prebuilt lane tables (ce_xgb_lane_table; depth <= 5): tree t's 64 entries
// [t][64] x {fx, ty} in a 1-based heap -- lane j in [1, 2^d) holds node j - 1
// as {xs_fbase(min(feature, D - 1)) | default_left << 31, split_cond bits},
// lane 2^d + k leaf k as {0, leaf bits}, lane 0 and the rest {0, 0} -- so one
// coalesced dwordx2 load with a scalar base is a tree's whole table (no
// per-lane branches or feature arithmetic), the root comes from a scalar load,
// and a level is child = 2 j + right.  VALU per tree was the limiter of the
// on-the-fly tables (PMC r06: VALU 72 % busy, 80 VALU per tree and wave).  Two
// halves [2][T][64]: the second without the default_left bits, read by tiles
// without a missing value (no mask per node read).
struct LaneTableForest {
    const uint2* table;     // [T][64], fx with default_left in bit 31 (tiles holding a missing value)
    const uint2* table_nd;  // [T][64], fx without it (the other tiles: no mask per node read)
    const int32_t* goff;
    int depth, NI;
    int goff_end;

    template <bool MISS>
    static __device__ __forceinline__ bool right(uint32_t fx, uint32_t th, const float* xs, uint32_t lane4) {
        const float x = xs_at(xs, MISS ? (fx & 0x7fffffffu) : fx, lane4);
        // missing -> the default child, else fvalue < split_cond ? left : right; a
        // NaN fails the compare (right), so flip exactly the NaN lanes whose default
        // is left: three compares and two mask ops
        const bool r = !(x < __uint_as_float(th));
        if constexpr (MISS)
            return r != (__builtin_isnan(x) && (int32_t)fx < 0);
        else
            return r;
    }
    // 4 trees at a time (two rounds per batch of 8): 4 independent chains per
    // lane keep every level's 8 bpermutes in flight within the 64-VGPR budget of
    // 8 waves per SIMD (8 chains forced the compiler to serialize the split
    // conditions' bpermutes behind lgkmcnt(0)); the second round's tables are
    // loaded with the first's.
    template <bool MISS, bool VALS>
    __device__ __forceinline__ void walk8(const float* xs, int D, int t0, int t1, int lane, int (&li)[8],
                                          float (&v)[8]) const {
        (void)D;
        const uint2* tb = MISS ? table : table_nd;
        uint2 e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = tb[(int64_t)(t0 + j < t1 ? t0 + j : t1 - 1) * 64 + lane];
        const uint32_t lane4 = 4u * (uint32_t)lane;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            int h[4];  // the lane's heap index x 4 (a ds_bpermute byte address): root 4, children 2 h + 4 b
#pragma unroll
            for (int j = 0; j < 4; ++j) h[j] = 4;
            // entries 0..3 of each tree (root 1, level-1 pair 2 / 3): 32 wave-uniform
            // bytes, scalar loads issued together before the first use (one wait)
            uint4 q0[4], q1[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = t0 + 4 * g + j < t1 ? t0 + 4 * g + j : t1 - 1;
                const uint4* p = reinterpret_cast<const uint4*>(tb + (int64_t)t * 64);
                q0[j] = p[0];
                q1[j] = p[1];
            }
            if (depth >= 1) {
#pragma unroll
                for (int j = 0; j < 4; ++j) h[j] = right<MISS>(q0[j].z, q0[j].w, xs, lane4) ? 12 : 8;
            }
            if (depth >= 2) {  // level 1 from the pair {2, 3} and a select
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool rt = h[j] == 12;
                    const uint32_t f = rt ? q1[j].z : q1[j].x, th = rt ? q1[j].w : q1[j].y;
                    h[j] = 2 * h[j] + (right<MISS>(f, th, xs, lane4) ? 4 : 0);
                }
            }
            for (int lev = 2; lev < depth; ++lev) {
                uint32_t f[4], th[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    f[j] = LaneForest::bperm(h[j], e[4 * g + j].x);
                    th[j] = LaneForest::bperm(h[j], e[4 * g + j].y);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) h[j] = 2 * h[j] + (right<MISS>(f[j], th[j], xs, lane4) ? 4 : 0);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                li[4 * g + j] = (h[j] >> 2) - (NI + 1);
                CE_DASSERT(li[4 * g + j] >= 0 && li[4 * g + j] <= NI);
                if constexpr (VALS) v[4 * g + j] = __uint_as_float(LaneForest::bperm(h[j], e[4 * g + j].y));
            }
        }
    }
    __device__ __forceinline__ float value(int t, int li) const {
        CE_DASSERT(t >= 0 && t < goff_end && li >= 0 && li <= NI);
        return __uint_as_float(table[(int64_t)t * 64 + NI + 1 + li].y);
    }
};

// ---- one block per 64-frame tile: G x S waves ------------------------------
// Wave (g, s) takes a contiguous run of group g's trees: s = 0 the head, its
// leaves added straight into the margin (a batch's leaf loads are added after
// the next batch is evaluated, hiding their latency); s >= 1 one of the S - 1
// tail chunks of at most kXgbChunk trees, whose leaf indices wait in registers
// (16 bits each) until the wave's phase.
// S ordered phases then hand the margin on through LDS (phase s: wave (g, s)
// adds its leaves in model order), so preds[g] is exactly the reference's
// sequential float chain while S times as many waves hide the latency.
constexpr int kXgbChunk = 24;

template <class L, bool MISS>
__device__ __forceinline__ void split_margins(const XgbArgs& a, const L& fl, const float* xs, float* mg, int g,
                                              int s, int lane) {
    const int k0 = fl.goff[g], k1 = fl.goff[g + 1], n = k1 - k0, S = a.S;
    const int c = min(kXgbChunk, (n + S - 1) / S);
    const int head_end = max(k0, k1 - (S - 1) * c);
    float m = a.base;
    uint32_t packed[kXgbChunk / 2] = {};  // tail waves: leaf indices, 16 bits each
    int lo = 0, cnt = 0;
    if (s == 0) {
        float pend[8];
        int npend = 0;
        for (int k = k0; k < head_end; k += 8) {
            int li[8];
            float v[8];
            fl.template walk8<MISS, true>(xs, a.D, k, head_end, lane, li, v);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < npend) m += pend[j];
#pragma unroll
            for (int j = 0; j < 8; ++j) pend[j] = v[j];
            npend = min(8, head_end - k);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j < npend) m += pend[j];
    } else {
        lo = head_end + (s - 1) * c;
        const int hi = min(k1, lo + c);
        cnt = max(0, hi - lo);
#pragma unroll
        for (int b = 0; b < kXgbChunk / 8; ++b) {
            if (b * 8 < cnt) {
                int li[8];
                float v[8];
                fl.template walk8<MISS, false>(xs, a.D, lo + b * 8, hi, lane, li, v);
#pragma unroll
                for (int j = 0; j < 8; j += 2) packed[b * 4 + j / 2] = (uint32_t)li[j] | ((uint32_t)li[j + 1] << 16);
            }
        }
    }
    // the tail wave's leaf values, all loaded before the ordered phases (one
    // latency, not one per phase: the phases are a chain of S - 1 hand-offs);
    // slots past cnt re-read the clamped last (tree, leaf) -- in bounds, not added
    float tv[kXgbChunk];
#pragma unroll
    for (int i = 0; i < kXgbChunk; ++i)
        tv[i] = (s > 0 && i < cnt) ? fl.value(lo + i, (packed[i / 2] >> (16 * (i & 1))) & 0xffffu) : 0.0f;
    for (int ph = 0; ph < S; ++ph) {
        if (s == ph && s > 0) {
            m = mg[g * 64 + lane];
#pragma unroll
            for (int i = 0; i < kXgbChunk; ++i)
                if (i < cnt) m += tv[i];
        }
        if (s == ph) mg[g * 64 + lane] = m;
        __syncthreads();
    }
}

template <int XDT, int ODT, class L, int KF = kXgbMaxFeat / 64>
__device__ __forceinline__ void xgb_tile(const XgbArgs& a, const L& fl) {
    extern __shared__ float xsm[];
    float* xs = xsm;                  // [D][kXgbCol] swizzled
    float* mg = xsm + a.D * kXgbCol;  // [G][64] margins
    uint32_t* nanw = reinterpret_cast<uint32_t*>(mg + a.G * 64);  // [waves] the tile's missing-value votes
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = w / a.S, s = w - g * a.S;
    const int64_t f0 = (int64_t)blockIdx.x * kXgbTile;
    const int nf = (int)min<int64_t>(kXgbTile, a.F - f0);
    bool has_nan;
    if constexpr (XDT == CE_F64 && CE_XGB_PAIRS && KF < kXgbMaxFeat / 64) {  // (the lane-table kernel's widths)
        if (a.D >= 2)
            has_nan = stage_tile_pairs<(KF + 1) / 2>(static_cast<const double*>(a.X), a.D, a.ld, f0, nf, xs);
        else
            has_nan = stage_tile<XDT, KF>(a.X, a.F, a.D, a.ld, f0, nf, xs);
    } else {
        has_nan = stage_tile<XDT, KF>(a.X, a.F, a.D, a.ld, f0, nf, xs);
    }
    // the block's "any NaN" vote through the dynamic LDS (__syncthreads_or keeps
    // a static LDS word, which puts the tile 256 B off address 0: one more VALU
    // per node read)
    {
        const bool wn = __ballot(has_nan) != 0;
        if (lane == 0) nanw[w] = wn ? 1u : 0u;
    }
    __syncthreads();
    bool any_nan = false;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) any_nan |= nanw[k] != 0u;
    if (any_nan)
        split_margins<L, true>(a, fl, xs, mg, g, s, lane);
    else
        split_margins<L, false>(a, fl, xs, mg, g, s, lane);
    transform_store<ODT>(mg, a.G, a.C, f0, nf, a.out, a.ldo);
}

// LANES: the lane-table walk (depth <= 5), else the perfect-tree gather walk
template <int XDT, int ODT, bool LANES>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_xgb_walk(
    XgbArgs a, const uint2* __restrict__ nodes, const float* __restrict__ leaves, const int32_t* __restrict__ goff,
    int depth) {
#ifdef CE_DEBUG
    const int T = goff[a.G];
#else
    const int T = 0;
#endif
    if constexpr (LANES) {
        CE_DASSERT(depth <= kXgbLaneDepth);
        xgb_tile<XDT, ODT>(a, LaneForest{nodes, leaves, goff, depth, (1 << depth) - 1, T});
    } else {
        xgb_tile<XDT, ODT>(a, WalkForest{nodes, leaves, goff, depth, (1 << depth) - 1, T});
    }
}

// KF: the row's 64-feature chunks the staging loads (>= ceil(D / 64); every load
// is unconditional, so a smaller KF drops dead loads: D = 260 takes 5 of 8)
template <int XDT, int ODT, int KF>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_xgb_lanes(
    XgbArgs a, const uint2* __restrict__ table, const uint2* __restrict__ table_nd, const int32_t* __restrict__ goff,
    int depth) {
#ifdef CE_DEBUG
    const int T = goff[a.G];
#else
    const int T = 0;
#endif
    CE_DASSERT(depth <= kXgbLaneDepth);
    xgb_tile<XDT, ODT, LaneTableForest, KF>(a, LaneTableForest{table, table_nd, goff, depth, (1 << depth) - 1, T});
}

// ce_xgb_lane_table: one wave per tree, lane j writes heap entry j
__global__ __launch_bounds__(256) void k_xgb_lane_table(const uint2* __restrict__ nodes, const float* __restrict__ leaves,
                                                        int T, int depth, int D, uint2* __restrict__ table) {
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int j = threadIdx.x & 63, NI = (1 << depth) - 1;
    if (t >= T) return;
    uint2 e = make_uint2(0u, 0u);
    uint32_t dl = 0u;
    if (j >= 1 && j <= NI) {
        const uint2 nd = nodes[t * NI + (j - 1)];
        const uint32_t ft = min(nd.x & 0x7fffffffu, (uint32_t)(D - 1));
        e = make_uint2(xs_fbase(ft), nd.y);
        dl = nd.x & 0x80000000u;
    } else if (j >= NI + 1 && j <= 2 * NI + 1) {
        e = make_uint2(0u, __float_as_uint(leaves[t * (NI + 1) + (j - NI - 1)]));
    }
    table[t * 64 + j] = make_uint2(e.x | dl, e.y);  // half 0: with default_left
    table[((int64_t)T + t) * 64 + j] = e;           // half 1: without
}

__global__ void k_expf(const float* __restrict__ x, int64_t n, float* __restrict__ y) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        y[i] = glibc_expf(x[i]);
}

}  // namespace ce

using namespace ce;

extern "C" size_t ce_xgb_lds_bytes(int32_t D, int32_t G) {
    return (size_t)D * kXgbCol * sizeof(float) + (size_t)std::max(G, 1) * 64 * sizeof(float) + 16 * sizeof(uint32_t);
}

// waves per group: fill a 16-wave block
static int xgb_splits(int G) { return std::max(1, 16 / G); }

template <class LaunchFn>
static void xgb_dispatch(ce_dtype x_dt, ce_dtype out_dt, LaunchFn&& fn) {
    if (x_dt == CE_F64)
        out_dt == CE_F64 ? fn(std::integral_constant<int, CE_F64>(), std::integral_constant<int, CE_F64>())
                         : fn(std::integral_constant<int, CE_F64>(), std::integral_constant<int, CE_F32>());
    else
        out_dt == CE_F64 ? fn(std::integral_constant<int, CE_F32>(), std::integral_constant<int, CE_F64>())
                         : fn(std::integral_constant<int, CE_F32>(), std::integral_constant<int, CE_F32>());
}

static int xgb_check(const void* X, ce_dtype x_dt, int64_t F, int32_t D, int64_t ld, int32_t G, int32_t C,
                     const void* out, ce_dtype out_dt, int64_t ld_out) {
    if (F < 0 || D < 1 || D > kXgbMaxFeat || ld < D || G < 1 || G > kXgbMaxGroups || ld_out < C ||
        !(G == C || (G == 1 && C == 2)))
        return fail(CE_EINVAL, "bad XGB shapes F=%lld D=%d G=%d C=%d", (long long)F, D, G, C);
    if ((x_dt != CE_F32 && x_dt != CE_F64) || (out_dt != CE_F32 && out_dt != CE_F64))
        return fail(CE_EINVAL, "XGB dtypes must be F32 or F64");
    if (F > 0 && (!X || !out)) return fail(CE_EINVAL, "null pointer");
    return CE_OK;
}

template <class K, class... Args>
static void xgb_launch(K kern, int64_t F, size_t lds, int threads, ce_stream_t stream, Args... args) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)((F + kXgbTile - 1) / kXgbTile)), dim3(threads), lds,
                       (hipStream_t)stream, args...);
}

extern "C" int ce_xgb_predict_proba(const void* X, ce_dtype x_dt, int64_t F, int32_t D, int64_t ld,
                                    const uint32_t* nodes, const float* leaves, const int32_t* group_offsets,
                                    int32_t G, int32_t depth, float base_margin, int32_t C, void* out,
                                    ce_dtype out_dt, int64_t ld_out, ce_stream_t stream) {
    if (int rc = xgb_check(X, x_dt, F, D, ld, G, C, out, out_dt, ld_out)) return rc;
    if (depth < 0 || depth > kXgbMaxDepth) return fail(CE_EINVAL, "XGB depth %d outside [0, %d]", depth, kXgbMaxDepth);
    if (!nodes || !leaves || !group_offsets) return fail(CE_EINVAL, "null pointer");
    if (F == 0) return CE_OK;
    const int S = xgb_splits(G);
    const XgbArgs a{X, F, D, ld, G, C, S, base_margin, out, ld_out};
    xgb_dispatch(x_dt, out_dt, [&](auto xd, auto od) {
        constexpr int XD = decltype(xd)::value, OD = decltype(od)::value;
        const auto kern = depth <= kXgbLaneDepth ? k_xgb_walk<XD, OD, true> : k_xgb_walk<XD, OD, false>;
        xgb_launch(kern, F, ce_xgb_lds_bytes(D, G), 64 * G * S, stream, a, reinterpret_cast<const uint2*>(nodes),
                   leaves, group_offsets, depth);
    });
    return check_launch("ce_xgb_predict_proba");
}

extern "C" int ce_xgb_lane_table(const uint32_t* nodes, const float* leaves, int32_t T, int32_t depth, int32_t D,
                                 uint32_t* table, ce_stream_t stream) {
    if (T < 0 || depth < 0 || depth > kXgbLaneDepth || D < 1 || D > kXgbMaxFeat)
        return fail(CE_EINVAL, "lane tables: T=%d depth=%d (<= %d) D=%d", T, depth, kXgbLaneDepth, D);
    if (T == 0) return CE_OK;
    if (!nodes || !leaves || !table) return fail(CE_EINVAL, "null pointer");
    hipLaunchKernelGGL(k_xgb_lane_table, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint2*>(nodes), leaves, T, depth, D, reinterpret_cast<uint2*>(table));
    return check_launch("ce_xgb_lane_table");
}

extern "C" int ce_xgb_predict_proba_lanes(const void* X, ce_dtype x_dt, int64_t F, int32_t D, int64_t ld,
                                          const uint32_t* table, int32_t T, const int32_t* group_offsets, int32_t G,
                                          int32_t depth, float base_margin, int32_t C, void* out, ce_dtype out_dt,
                                          int64_t ld_out, ce_stream_t stream) {
    if (int rc = xgb_check(X, x_dt, F, D, ld, G, C, out, out_dt, ld_out)) return rc;
    if (depth < 0 || depth > kXgbLaneDepth)
        return fail(CE_EINVAL, "XGB lane tables hold depth <= %d, got %d", kXgbLaneDepth, depth);
    if (!table || !group_offsets || T < 1) return fail(CE_EINVAL, "null pointer or no trees (T=%d)", T);
    if (F == 0) return CE_OK;
    const int S = xgb_splits(G);
    const uint2* tb = reinterpret_cast<const uint2*>(table);
    const XgbArgs a{X, F, D, ld, G, C, S, base_margin, out, ld_out};
    xgb_dispatch(x_dt, out_dt, [&](auto xd, auto od) {
        constexpr int XD = decltype(xd)::value, OD = decltype(od)::value;
        const auto kern = D <= 128 ? k_xgb_lanes<XD, OD, 2>
                        : D <= 256 ? k_xgb_lanes<XD, OD, 4>
                        : D <= 320 ? k_xgb_lanes<XD, OD, 5> : k_xgb_lanes<XD, OD, 8>;
        xgb_launch(kern, F, ce_xgb_lds_bytes(D, G), 64 * G * S, stream, a, tb, tb + (int64_t)T * 64, group_offsets,
                   depth);
    });
    return check_launch("ce_xgb_predict_proba_lanes");
}

extern "C" int ce_xgb_expf(const float* x, int64_t n, float* y, ce_stream_t stream) {
    if (n < 0 || (n > 0 && (!x || !y))) return fail(CE_EINVAL, "bad expf arguments");
    if (n == 0) return CE_OK;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_expf, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, n, y);
    return check_launch("ce_xgb_expf");
}
