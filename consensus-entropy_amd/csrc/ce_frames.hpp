// ce_frames.hpp -- SURVEY.md §8(f)1: the committee built from FRAME-level
// member outputs and selected in ONE pass, without the [M, N, C] stack.
//
// The reference (amg_test.py:426-445) gets, per member, predict_proba over the
// user's X_train frame rows, groups them per song
//     y_probs = pd.DataFrame(y_probs, index=X_train.index).groupby(['s_id']).mean()   (:437)
// stacks the M song-level frames, averages over members and selects:
//     consensus_prob = np.mean(np.array(pred_prob), axis=0)                        (:441)
//     ent = entropy(consensus_prob, axis=1); q_ind = argsort(ent)[::-1][:q]       (:443-445)
// k_frames_select does all of it per song: lane = song, member loop outer
// (member-sequential f64 sum as np.mean), per member the song's frames in row
// order (pandas 1.1.5 group_mean: f64 sequential sum skipping NaN / non-NaN
// count, NaN when none; a float32 member's mean rounded to float32, as the
// groupby result keeps the column dtype), then / M, scipy's entropy, and the
// streaming top-q (per-wave register lists, block merge, the last block merges
// the grid -- one launch).  A song-level member (the CNN, :430-433: already
// one row per song) is read as is.  Frames of song n are rows
// perm[off[n]] .. perm[off[n+1]-1] (perm == nullptr: off[n] .. off[n+1]-1),
// songs in sorted s_id order as groupby returns them.
#pragma once
#include "ce_stream.hpp"

namespace ce {

constexpr int kMaxFrameMembers = 32;

struct FrameMember {
    const void* p;   // [F, C] frames (or [N, C] song rows), row stride ld elements
    int64_t ld;
    int dt;          // kF32 | kF64
    int song_level;  // 1: one row per song (row n), 0: frame rows via off/perm
    int vec;         // rows 16-B aligned (vector loads)
    int pad_;
};

struct FrameArgs {
    FrameMember mem[kMaxFrameMembers];
    int M;
    const int64_t* off;   // [N+1] song offsets into the frame order
    const int64_t* perm;  // [F] frame order -> row, or nullptr
    int64_t N;            // songs
    double dM, invM;
    bool pow2;
    int64_t base_idx;
    int64_t per_wave;  // songs per wave (multiple of 64)
    int nlists;
    uint32_t* ctr;  // fold (last block merges the grid)
    double* oval;
    int64_t* oidx;
    Cand* ocand;
};

// One row of C values of a member, widened to f64.
template <int C>
__device__ __forceinline__ void load_row(const FrameMember& m, int64_t r, double (&v)[C]) {
    if (m.dt == kF64) {
        const double* row = static_cast<const double*>(m.p) + r * m.ld;
        if constexpr (C % 2 == 0) {
            if (m.vec) {
#pragma unroll
                for (int k = 0; k < C / 2; ++k) {
                    const f64x2 x = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(row) + k);
                    v[2 * k] = x.x;
                    v[2 * k + 1] = x.y;
                }
                return;
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = row[c];
    } else {
        const float* row = static_cast<const float*>(m.p) + r * m.ld;
        if constexpr (C % 4 == 0) {
            if (m.vec) {
#pragma unroll
                for (int k = 0; k < C / 4; ++k) {
                    const f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row) + k);
                    v[4 * k] = (double)x.x;
                    v[4 * k + 1] = (double)x.y;
                    v[4 * k + 2] = (double)x.z;
                    v[4 * k + 3] = (double)x.w;
                }
                return;
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = (double)row[c];
    }
}

// groupby(['s_id']).mean() of member m for song n (pandas 1.1.5 group_mean),
// added member-sequentially into acc (np.mean over the stack, :441).  Frames
// are read in batches of B rows, all loads of a batch in flight before the
// in-order adds (rows past the song clamp to its last row and are skipped).
template <int C, int B>
__device__ __forceinline__ void add_member_mean(const FrameMember& m, const FrameArgs& a, int64_t n, bool live,
                                                double (&acc)[C]) {
    double mean[C];
    if (m.song_level) {
        double v[C];
        load_row<C>(m, live ? n : 0, v);
#pragma unroll
        for (int c = 0; c < C; ++c) mean[c] = v[c];
    } else {
        const int64_t f0 = live ? a.off[n] : 0, f1 = live ? a.off[n + 1] : 0;
        CE_DASSERT(f0 >= 0 && f0 <= f1);
        double s[C];
        int cnt[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            s[c] = 0.0;
            cnt[c] = 0;
        }
        for (int64_t fb = f0; fb < f1; fb += B) {  // per lane: its own song's length
            double v[B][C];
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const int64_t f = fb + u < f1 ? fb + u : f1 - 1;
                const int64_t r = a.perm ? a.perm[f] : f;
                load_row<C>(m, r, v[u]);
            }
#pragma unroll
            for (int u = 0; u < B; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c)
                    if (fb + u < f1 && v[u][c] == v[u][c]) {  // not NaN
                        s[c] += v[u][c];
                        ++cnt[c];
                    }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            double x = cnt[c] ? s[c] / (double)cnt[c] : __longlong_as_double(0x7ff8000000000000ll);
            if (m.dt == kF32) x = (double)(float)x;  // the float32 result column
            mean[c] = x;
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] += mean[c];
}

template <int C>
__global__ __launch_bounds__(256) void k_frames_select(FrameArgs a, int q, Cand* __restrict__ wc) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    __shared__ WaveLists sm;
    CE_DASSERT((int)gridDim.x <= a.nlists && q >= 1 && q <= kStreamMaxQ);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    int64_t lo = gw * a.per_wave;
    int64_t hi = lo + a.per_wave;
    if (hi > a.N) hi = a.N;
    if (lo > hi) lo = hi;
    RegTopQ tq;
    tq.init(q);
    for (int64_t t0 = lo; t0 < hi; t0 += 64) {
        const int64_t n = t0 + lane;
        const bool live = n < hi;
        double acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.0;  // np.add.reduce identity
        for (int mm = 0; mm < a.M; ++mm) add_member_mean<C, 8>(a.mem[mm], a, n, live, acc);
        double mean[C];
#pragma unroll
        for (int c = 0; c < C; ++c) mean[c] = div_members(acc[c], a.dM, a.invM, a.pow2);
        const double h = entropy_row<C>(mean);
        tq.offer(order_key(h), n + a.base_idx, live);
    }
    block_merge_write<4>(tq, sm, q, wc + (int64_t)blockIdx.x * q, a.nlists, nullptr, nullptr, 4, a.ctr != nullptr);
    if (a.ctr) fold_merge<4>(a.ctr, a.oval, a.oidx, a.ocand, q, wc, sm);
}

}  // namespace ce
