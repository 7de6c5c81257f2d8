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
    int64_t per_wave;  // songs per wave (a multiple of the kernel's songs per wave step)
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

// Per-song committee entropy to HBM (k_frames_select's arithmetic, lane per
// song): the input of the list (64 < q <= CE_MAX_Q) and sort (q > CE_MAX_Q)
// selections of ce_select_frames.
template <int C>
__global__ __launch_bounds__(256) void k_frames_entropy(FrameArgs a, double* __restrict__ ent) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < a.N; n += (int64_t)gridDim.x * 256) {
        double acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.0;  // np.add.reduce identity
        for (int mm = 0; mm < a.M; ++mm) add_member_mean<C, 8>(a.mem[mm], a, n, true, acc);
        double mean[C];
#pragma unroll
        for (int c = 0; c < C; ++c) mean[c] = div_members(acc[c], a.dM, a.invM, a.pow2);
        ent[n] = entropy_row<C>(mean);
    }
}

// The sum and non-NaN count of column c of this lane's song (rows [f0, f1)
// of a grouped dense member: rows of C elements of EB bytes, 16-B aligned,
// base mb), with the wave's step of songs covering rows [R0, R1): the rows are
// staged TB bytes at a time by LDS-DMA (1 KiB per global_load_lds, fully
// coalesced) into the wave's tile, 16-B units XOR-swizzled within 256 B, and
// every lane adds its song's rows of the tile in row order, NaN skipped
// (pandas group_mean).  Lanes whose song is not in [R0, R1) read no row.
template <int C, int EB, int TB>
__device__ __forceinline__ void tile_song_sum(const char* mb, int64_t R0, int64_t R1, int64_t f0, int64_t f1,
                                              int lane, int c, char* tile, double& s, int& cnt) {
    constexpr int RB = C * EB, TR = TB / RB;  // bytes per row, rows per tile
    static_assert(RB % 16 == 0, "16-B units");
    for (int64_t c0 = R0; c0 < R1; c0 += TR) {
        const int64_t c1 = c0 + TR < R1 ? c0 + TR : R1;
        const int units = (int)(c1 - c0) * RB / 16;
        const char* src = mb + c0 * RB;
        for (int j = 0; j * 64 < units; ++j) {  // wave-uniform
            const int pd = j * 64 + lane;  // LDS unit written by this lane
            int ps = pd ^ ((pd >> 4) & 15);  // its source unit (the swizzle is an involution)
            ps = ps < units ? ps : units - 1;
            CE_DASSERT(j * 1024 + 1024 <= TB);
            __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)ps * 16),
                                             (void __attribute__((address_space(3)))*)(tile + j * 1024), 16, 0, 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // this lane's song's rows in the tile, in order: 8 LDS reads in flight,
        // then the 8 adds (a read per row would wait out an LDS round trip each);
        // rows past lr1 re-read the tile's first row and are skipped.  Row
        // indices relative to the tile (32-bit) and the element size a
        // compile-time constant (a per-row dtype select put a branch and an LDS
        // wait on every row: grouped frames 0.879 -> 0.712 ms, r06_frames_ab.json)
        const int lr0 = (int)((f0 > c0 ? f0 : c0) - c0);
        const int lr1 = (int)((f1 < c1 ? f1 : c1) - c0);  // < lr0: no row of this song here
        for (int rb = lr0; rb < lr1; rb += 8) {
            double v[8];
#pragma unroll
            for (int u8 = 0; u8 < 8; ++u8) {
                const int r = rb + u8 < lr1 ? rb + u8 : 0;
                const int b = r * RB + c * EB;
                const int u = b >> 4;
                const char* e = tile + ((u ^ ((u >> 4) & 15)) << 4) + (b & 15);
                v[u8] = EB == 8 ? *reinterpret_cast<const double*>(e) : (double)*reinterpret_cast<const float*>(e);
            }
#pragma unroll
            for (int u8 = 0; u8 < 8; ++u8)
                if (rb + u8 < lr1 && v[u8] == v[u8]) {  // not NaN
                    s += v[u8];
                    ++cnt;
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tile is read before the next DMA
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The same selection with C lanes per song (lane = (song, class), 64 / C songs
// per wave step): each lane keeps ONE class's sequential group sum, so the
// frame rows of the wave's songs are read as whole rows.  Grouped frames (no
// perm) of a dense member (row = C * size bytes, a multiple of 16) reach the
// wave by LDS-DMA: the wave's songs own the contiguous rows [off[t0],
// off[t0 + G]), staged 16 KiB at a time (1 KiB per global_load_lds, fully
// coalesced) in the wave's LDS tile with the 16-B units XOR-swizzled within
// 256 B (unit p at p ^ ((p >> 4) & 15)), so the songs of a step -- rows a
// song length apart -- read distinct banks; every lane then adds its song's
// rows of the tile in row order (pandas group_mean: NaN skipped, counted
// cells only).  Shuffled frames (perm), strided or 8-B rows are read by direct
// loads in batches of 8 rows, as k_segment_mean.  The class means of a song
// meet by lane shuffles; every lane of the song computes its entropy (the
// group's lane 0 offers it).  Same values as k_frames_select.
// DMA = false: direct loads only, no LDS tiles -- the 64 KiB of tiles would
// cap the gather (shuffled frames) at 2 blocks per CU.  GNT: the direct row
// loads non-temporal -- for large shuffled pools, whose random rows are each
// read once (1M songs x 40 frames: 2.49 -> 2.30 ms); at the reference's 1608
// songs it costs 3 us (39.7 -> 42.2), and grouped rows share their lines (the
// segment mean with nt loads: 374 -> 673 us), so the host picks it only for
// shuffled pools of >= 4 steps per wave (profiles/r05_frames_random_rows.json,
// r05_segment_nt_ab.json).
template <int C, bool DMA, bool GNT = false>
__global__ __launch_bounds__(256) void k_frames_lanes(FrameArgs a, int q, Cand* __restrict__ wc) {
    static_assert(64 % C == 0, "C divides the wave");
    constexpr int G = 64 / C;  // songs per wave step
    constexpr int TB = DMA ? 16384 : 16;  // per-wave LDS tile
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    __shared__ WaveLists sm;
    __shared__ __attribute__((aligned(16))) char tiles[4][TB];
    CE_DASSERT((int)gridDim.x <= a.nlists && q >= 1 && q <= kStreamMaxQ);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sg = lane / C, c = lane - sg * C;
    char* tile = tiles[w];
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    // grid-cyclic steps (wave g: steps g, g + W, ...; ~1 % over a contiguous run per wave)
    const int64_t lo = gw * G, hi = a.N, step = (int64_t)gridDim.x * 4 * G;
    // frame-level members in member order (up to 4 read together by the direct path)
    int nf = 0, f_0 = 0, f_1 = 0, f_2 = 0, f_3 = 0;
    for (int mm = 0; mm < a.M; ++mm)
        if (!a.mem[mm].song_level) {
            f_0 = nf == 0 ? mm : f_0;
            f_1 = nf == 1 ? mm : f_1;
            f_2 = nf == 2 ? mm : f_2;
            f_3 = nf == 3 ? mm : f_3;
            ++nf;
        }
    RegTopQ tq;
    tq.init(q);
    // the step's CSR offsets (this lane's song [f0, f1), the step's rows [R0,
    // R1) of songs [t, t + G)) are loaded ONCE per step and one step ahead:
    // the loads of step t + 1 are issued at the top of step t and land during
    // its tiles, so no member's first tile waits on an offsets round trip
    // (they were re-read per member before: 1M songs grouped 0.911 -> 0.880 ms,
    // profiles/r05_frames_offsets_ab.json)
    int64_t pf0 = 0, pf1 = 0, pR0 = 0, pR1 = 0;
    auto load_offs = [&](int64_t t) {
        const int64_t nn = t + sg;
        const int64_t tg = t + G < hi ? t + G : hi;
        pf0 = nn < hi ? a.off[nn] : 0;
        pf1 = nn < hi ? a.off[nn + 1] : 0;
        pR0 = a.off[t];
        pR1 = a.off[tg];
    };
    if (lo < hi) load_offs(lo);
    for (int64_t t0 = lo; t0 < hi; t0 += step) {
        const int64_t n = t0 + sg;
        const bool live = n < hi;
        double acc = 0.0;  // np.add.reduce identity
        const int64_t sf0 = pf0, sf1 = pf1, sR0 = pR0, sR1 = pR1;
        if (t0 + step < hi) load_offs(t0 + step);
        if (!DMA && nf <= 4) {
            // direct loads (shuffled frames): each batch's 8 frame indices are
            // read ONCE for every frame-level member, then all members' rows of
            // the batch are in flight together (perm read once, 2 serial round
            // trips per batch instead of 2 per batch and member); each member
            // keeps its own sequential group sum, and the means meet in member
            // order below
            const int64_t f0 = sf0, f1 = sf1;
            CE_DASSERT(f0 >= 0 && f0 <= f1);
            constexpr int B = 8;  // (4: 1M songs equal, 1608 songs 38.6 -> 42.4 us)
            double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
            int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
            for (int64_t fb = f0; fb < f1; fb += B) {
                int64_t r[B];
#pragma unroll
                for (int u = 0; u < B; ++u) {
                    const int64_t f = fb + u < f1 ? fb + u : f1 - 1;
                    r[u] = a.perm ? a.perm[f] : f;
                }
                double v[4][B];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k < nf) {  // wave-uniform
                        const FrameMember& fm = a.mem[k == 0 ? f_0 : (k == 1 ? f_1 : (k == 2 ? f_2 : f_3))];
#pragma unroll
                        for (int u = 0; u < B; ++u) {
                            const int64_t o = r[u] * fm.ld + c;
                            if constexpr (GNT)  // shuffled rows of a large pool: each read once
                                v[k][u] = fm.dt == kF64 ? __builtin_nontemporal_load(static_cast<const double*>(fm.p) + o)
                                                        : (double)__builtin_nontemporal_load(static_cast<const float*>(fm.p) + o);
                            else
                                v[k][u] = fm.dt == kF64 ? static_cast<const double*>(fm.p)[o]
                                                        : (double)static_cast<const float*>(fm.p)[o];
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < B; ++u) {
                    const bool in = fb + u < f1;
                    if (nf > 0 && in && v[0][u] == v[0][u]) { s0 += v[0][u]; ++c0; }
                    if (nf > 1 && in && v[1][u] == v[1][u]) { s1 += v[1][u]; ++c1; }
                    if (nf > 2 && in && v[2][u] == v[2][u]) { s2 += v[2][u]; ++c2; }
                    if (nf > 3 && in && v[3][u] == v[3][u]) { s3 += v[3][u]; ++c3; }
                }
            }
            int k = 0;
            for (int mm = 0; mm < a.M; ++mm) {
                const FrameMember& fm = a.mem[mm];
                double mean;
                if (fm.song_level) {
                    const int64_t o = (live ? n : t0) * fm.ld + c;
                    mean = fm.dt == kF64 ? static_cast<const double*>(fm.p)[o]
                                         : (double)static_cast<const float*>(fm.p)[o];
                } else {
                    const double sk = k == 0 ? s0 : (k == 1 ? s1 : (k == 2 ? s2 : s3));
                    const int ck = k == 0 ? c0 : (k == 1 ? c1 : (k == 2 ? c2 : c3));
                    double x = ck ? sk / (double)ck : __longlong_as_double(0x7ff8000000000000ll);
                    if (fm.dt == kF32) x = (double)(float)x;  // the float32 result column
                    mean = x;
                    ++k;
                }
                acc += mean;
            }
        } else
        for (int mm = 0; mm < a.M; ++mm) {
            const FrameMember& fm = a.mem[mm];
            const int EB = fm.dt == kF64 ? 8 : 4;
            double mean;
            if (fm.song_level) {
                const int64_t o = (live ? n : t0) * fm.ld + c;
                mean = fm.dt == kF64 ? static_cast<const double*>(fm.p)[o] : (double)static_cast<const float*>(fm.p)[o];
            } else {
                const int64_t f0 = sf0, f1 = sf1;
                CE_DASSERT(f0 >= 0 && f0 <= f1);
                double s = 0.0;
                int cnt = 0;
                const int RB = C * EB;
                const int64_t R0 = sR0, R1 = sR1;
                // the step's songs tile [R0, R1) (CSR offsets); a wave holding a song outside it
                // (offsets not monotone) reads its rows directly instead
                const bool inside = !live || (f0 >= R0 && f1 <= R1);
                if (DMA && !a.perm && fm.ld == C && RB % 16 == 0 && fm.vec && __all(inside)) {  // wave-uniform: LDS-DMA tiles
                    const char* mb = static_cast<const char*>(fm.p);
                    if (EB == 8) {
                        if constexpr (DMA && (C * 8) % 16 == 0) tile_song_sum<C, 8, TB>(mb, R0, R1, f0, f1, lane, c, tile, s, cnt);
                    } else {
                        if constexpr (DMA && (C * 4) % 16 == 0) tile_song_sum<C, 4, TB>(mb, R0, R1, f0, f1, lane, c, tile, s, cnt);
                    }
                } else {  // direct loads: batches of 8 rows in flight, added in row order
                    constexpr int B = 8;
                    for (int64_t fb = f0; fb < f1; fb += B) {
                        double v[B];
#pragma unroll
                        for (int u = 0; u < B; ++u) {
                            const int64_t f = fb + u < f1 ? fb + u : f1 - 1;
                            const int64_t r = a.perm ? a.perm[f] : f;
                            const int64_t o = r * fm.ld + c;
                            if constexpr (GNT)
                                v[u] = fm.dt == kF64 ? __builtin_nontemporal_load(static_cast<const double*>(fm.p) + o)
                                                     : (double)__builtin_nontemporal_load(static_cast<const float*>(fm.p) + o);
                            else
                                v[u] = fm.dt == kF64 ? static_cast<const double*>(fm.p)[o]
                                                     : (double)static_cast<const float*>(fm.p)[o];
                        }
#pragma unroll
                        for (int u = 0; u < B; ++u)
                            if (fb + u < f1 && v[u] == v[u]) {
                                s += v[u];
                                ++cnt;
                            }
                    }
                }
                double x = cnt ? s / (double)cnt : __longlong_as_double(0x7ff8000000000000ll);
                if (fm.dt == kF32) x = (double)(float)x;  // the float32 result column
                mean = x;
            }
            acc += mean;
        }
        const double mv = div_members(acc, a.dM, a.invM, a.pow2);
        double row[C];
#pragma unroll
        for (int k = 0; k < C; ++k) row[k] = __shfl(mv, sg * C + k);
        const double h = entropy_row<C>(row);
        tq.offer(order_key(h), n + a.base_idx, live && c == 0);
    }
    block_merge_write<4>(tq, sm, q, wc + (int64_t)blockIdx.x * q, a.nlists, nullptr, nullptr, 4, a.ctr != nullptr);
    if (a.ctr) fold_merge<4>(a.ctr, a.oval, a.oidx, a.ocand, q, wc, sm);
}

// frame -> song segment mean of one grouped dense member (ce_segment_mean,
// amg_test.py:437; the same values as k_segment_mean): C lanes per song, the
// step's songs' rows staged by LDS-DMA tiles (tile_song_sum), a wave holding a
// song outside its step's rows (offsets not monotone) reads its rows directly.
// The host takes it once every wave runs >= 4 steps (else k_segment_mean).
template <int C, int DT, int ODT>
__global__ __launch_bounds__(256) void k_segment_mean_tiles(const void* __restrict__ frames,
                                                            const int64_t* __restrict__ offsets, int64_t N,
                                                            void* __restrict__ out, int64_t ldo) {
    constexpr int G = 64 / C, EB = DT == kF64 ? 8 : 4, TB = 16384;
    static_assert(64 % C == 0 && (C * EB) % 16 == 0, "C lanes per song, 16-B rows");
    __shared__ __attribute__((aligned(16))) char tiles[4][TB];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sg = lane / C, c = lane - sg * C;
    const int64_t step = (int64_t)gridDim.x * 4 * G;
    for (int64_t t0 = ((int64_t)blockIdx.x * 4 + w) * G; t0 < N; t0 += step) {
        const int64_t n = t0 + sg;
        const bool live = n < N;
        const int64_t f0 = live ? offsets[n] : 0, f1 = live ? offsets[n + 1] : 0;
        const int64_t R0 = offsets[t0], R1 = offsets[t0 + G < N ? t0 + G : N];
        CE_DASSERT(f0 >= 0 && f0 <= f1);
        double s = 0.0;  // np.add.reduce identity
        int cnt = 0;
        if (__all(!live || (f0 >= R0 && f1 <= R1))) {  // wave-uniform
            tile_song_sum<C, EB, TB>(static_cast<const char*>(frames), R0, R1, f0, f1, lane, c, tiles[w], s, cnt);
        } else {
            for (int64_t f = f0; f < f1; ++f) {
                const double v = DT == kF64 ? static_cast<const double*>(frames)[f * C + c]
                                            : (double)static_cast<const float*>(frames)[f * C + c];
                if (v == v) {
                    s += v;
                    ++cnt;
                }
            }
        }
        if (live) {
            double m = cnt ? s / (double)cnt : __longlong_as_double(0x7ff8000000000000ll);
            if constexpr (DT == kF32) m = (double)(float)m;  // the float32 result column
            if constexpr (ODT == kF32)
                static_cast<float*>(out)[n * ldo + c] = (float)m;
            else
                static_cast<double*>(out)[n * ldo + c] = m;
        }
    }
}

}  // namespace ce
