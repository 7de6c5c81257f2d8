// ce_stream.hpp -- the streaming mc kernel (stage 1 of ce_select_mc, q <= 64).
//
// One pass over the committee tensor at HBM rate.  Every wave is independent
// while streaming (no block barriers in the loop): it owns a contiguous run of
// 64-item tiles, scores one item per lane, and keeps its own top-q candidates
// in registers (RegTopQ, one list slot per lane).  The block's four wave
// lists are merged once at the end.
//
// Item-major [N, M, C] tensors (each item's M*C values contiguous, R bytes)
// are staged through LDS: a wave's 64 x R-byte tile arrives by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per instruction, fully coalesced); each
// lane then reads its own item with ds_read_b128.  The 16-B chunks of row r
// are stored XOR-swizzled (chunk m at slot m ^ (r & 15), done on the SOURCE
// address since the DMA writes LDS linearly) so the 16 lanes of a
// ds_read_b128 group hit 16 different bank groups.  As soon as the tile sits
// in registers the next tile's DMA is issued into the same buffer, so the
// f64 arithmetic of tile t overlaps the HBM fetch of tile t+1.
// Member-major / strided tensors load straight to registers (coalesced across
// lanes for the reference's [M, N, C] stack).
#pragma once
#include "ce_device.hpp"
#include "ce_topq.hpp"

namespace ce {

// ---------------------------------------------------------------------------
// Per-wave top-q held in registers (q <= 64): lane L holds the L-th best
// (order key, position) of the wave so far, best first; empty slots hold the
// sentinel (0, INT64_MAX), worse than every real candidate (no finite, inf or
// NaN entropy maps to key 0).  The threshold is slot q-1, read into scalar
// registers.  A candidate that beats it is rare once the stream is warm: one
// or a few are inserted in place (ballot for the position + one lane shift);
// a large batch (the first tiles) is bitonic-sorted across the wave and
// merged with the list -- shuffles only, no LDS, no barrier.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// (k, i) from lane `src` (per-lane index) -- ds_bpermute on the four halves
__device__ __forceinline__ void shfl_cand(uint64_t& k, int64_t& i, int src) {
    const int a = src << 2;
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)k);
    const uint32_t k1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(k >> 32));
    const uint32_t i0 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(uint64_t)i);
    const uint32_t i1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)((uint64_t)i >> 32));
    k = ((uint64_t)k1 << 32) | k0;
    i = (int64_t)(((uint64_t)i1 << 32) | i0);
}

// Lane exchange "value of lane ^ J" without the LDS crossbar (ds_bpermute
// throughput, not latency, bounded the sort networks): DPP quad_perm for J =
// 1, 2; row_half_mirror (lane ^ 7) then quad reverse (lane ^ 3) for J = 4;
// row_ror:8 for J = 8; the gfx950 permlane16/32 swaps for J = 16, 32.
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (J == 4) {
        const int t = __builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
        return (uint32_t)__builtin_amdgcn_update_dpp(0, t, 0x1B, 0xF, 0xF, false);      // quad_perm [3,2,1,0]
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (J == 16) {
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? p[0] : p[1];
    } else {
        static_assert(J == 32, "lane exchange distance");
        const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? p[0] : p[1];
    }
}

// value of lane - 1 (DPP wave_shr:1)
__device__ __forceinline__ uint64_t lane_above(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

template <int J>
__device__ __forceinline__ void xor_cand(uint64_t& k, int64_t& i) {
    const uint32_t k0 = xor_lane<J>((uint32_t)k), k1 = xor_lane<J>((uint32_t)(k >> 32));
    const uint32_t i0 = xor_lane<J>((uint32_t)(uint64_t)i), i1 = xor_lane<J>((uint32_t)((uint64_t)i >> 32));
    k = ((uint64_t)k1 << 32) | k0;
    i = (int64_t)(((uint64_t)i1 << 32) | i0);
}

// One compare-exchange stage of a bitonic network across the wave: partner
// lane ^ J; `desc` = this lane's block sorts best-first.
template <int J>
__device__ __forceinline__ void cx_stage(uint64_t& k, int64_t& i, bool desc) {
    const int lane = threadIdx.x & 63;
    uint64_t pk = k;
    int64_t pi = i;
    xor_cand<J>(pk, pi);
    const bool lower = (lane & J) == 0;
    const bool pb = better(pk, pi, k, i);
    const bool take = (lower == desc) ? pb : !pb;
    if (take) {
        k = pk;
        i = pi;
    }
}

template <int S, int J>
__device__ __forceinline__ void sort_stages(uint64_t& k, int64_t& i) {
    cx_stage<J>(k, i, ((threadIdx.x & 63) & S) == 0);
    if constexpr (J > 1) sort_stages<S, J / 2>(k, i);
}

template <int S>
__device__ __forceinline__ void sort_levels(uint64_t& k, int64_t& i) {
    sort_stages<S, S / 2>(k, i);
    if constexpr (S < 64) sort_levels<S * 2>(k, i);
}

// The wave's best (k, i) in every lane (6 butterfly stages).
template <int J>
__device__ __forceinline__ void best_stages(uint64_t& k, int64_t& i) {
    uint64_t pk = k;
    int64_t pi = i;
    xor_cand<J>(pk, pi);
    if (better(pk, pi, k, i)) {
        k = pk;
        i = pi;
    }
    if constexpr (J < 32) best_stages<J * 2>(k, i);
}
__device__ __forceinline__ void wave_best64(uint64_t& k, int64_t& i) { best_stages<1>(k, i); }

// Each 16-lane row's best (k, i) in all its lanes (4 butterfly stages).
__device__ __forceinline__ void row_best16(uint64_t& k, int64_t& i) {
    uint64_t pk;
    int64_t pi;
#define CE_RB(J)                          \
    pk = k;                               \
    pi = i;                               \
    xor_cand<J>(pk, pi);                  \
    if (better(pk, pi, k, i)) {           \
        k = pk;                           \
        i = pi;                           \
    }
    CE_RB(1) CE_RB(2) CE_RB(4) CE_RB(8)
#undef CE_RB
}

// Sort the wave's 64 (k, i) best-first (21 stages).
__device__ __forceinline__ void wave_sort64(uint64_t& k, int64_t& i) { sort_levels<2>(k, i); }

// (k, i) := best 64 of the two best-first lists (k, i) and (bk, bi), best-first.
__device__ __forceinline__ void wave_merge64(uint64_t& k, int64_t& i, uint64_t bk, int64_t bi) {
    const int lane = threadIdx.x & 63;
    shfl_cand(bk, bi, 63 - lane);  // reversed: list max(A[L], B[63-L]) is bitonic
    if (better(bk, bi, k, i)) {
        k = bk;
        i = bi;
    }
    sort_stages<64, 32>(k, i);  // half-cleaners 32 .. 1, all best-first
}

// item slots a lane keeps in flight in the single-block pools (rows_small).
// Measured on configs[2] (500 users x 1608, f32): all at once 14.24 us,
// 1 slot 13.52 us, 2 slots 14.68 us
// Round 4, after the approximate prefilter (profiles/r04_small_phase_prefilter.json):
// 1 slot 10.74 us, 2 slots 10.98 us, all 16-23 us (register spills);
// the last short slot issued with slot 0: C1 6.12 -> 6.42 us, C3 even; the
// single-pool launches with 2 / all slots in flight: C1 5.86 -> 6.04 / 6.68 us,
// the mix 6.6 -> 6.92 / 6.94 us.
#ifndef CE_SMALL_THR
#define CE_SMALL_THR 1
#endif
constexpr int kSmallThrottle = CE_SMALL_THR;

// no-op callback of CommitteeSrc::keys / rows_small (ce_kernels.hpp)
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};

// bit i of an exclusion bitmap (SelectionSession: items already queried)
__device__ __forceinline__ bool excluded(const uint32_t* b, int64_t i) { return (b[i >> 5] >> (i & 31)) & 1u; }

struct RegTopQ {
    uint64_t k;   // this lane's slot
    int64_t i;
    uint64_t tk;  // threshold = the better of slot q-1 and the floor (wave-uniform)
    int64_t ti;
    uint64_t fk;  // floor: a known exact lower bound (only candidates beating it can be selected)
    int64_t fi;
    int q;

    __device__ __forceinline__ void init(int q_, uint64_t fk_ = 0, int64_t fi_ = INT64_MAX) {
        k = 0;
        i = INT64_MAX;
        tk = fk = fk_;
        ti = fi = fi_;
        q = q_;
    }

    __device__ __forceinline__ void refresh() {
        const uint64_t sk = readlane64(k, q - 1);
        const int64_t si = (int64_t)readlane64((uint64_t)i, q - 1);
        const bool s_better = better(sk, si, fk, fi);
        tk = s_better ? sk : fk;
        ti = s_better ? si : fi;
    }

    // the list holds no candidate (wave-uniform)
    __device__ __forceinline__ bool empty() const { return readlane64((uint64_t)i, 0) == (uint64_t)INT64_MAX; }

    // insert one wave-uniform candidate that beats the threshold
    __device__ __forceinline__ void insert(uint64_t ck, int64_t ci) {
        const int lane = threadIdx.x & 63;
        const uint64_t below = __ballot(better(ck, ci, k, i));  // slots the candidate beats: a suffix
        const int p = __builtin_ctzll(below);
        const uint64_t uk = lane_above(k);  // lane 0 never takes it
        const int64_t ui = (int64_t)lane_above((uint64_t)i);
        if (lane > p) {
            k = uk;
            i = ui;
        } else if (lane == p) {
            k = ck;
            i = ci;
        }
    }

    __device__ __forceinline__ void offer(uint64_t ck, int64_t ci, bool valid) {
        const bool pass = valid && better(ck, ci, tk, ti);
        uint64_t mask = __ballot(pass);
        if (mask == 0) return;  // wave-uniform: the common case
        if (__popcll(mask) <= 8) {
            do {
                const int s = __builtin_ctzll(mask);
                mask &= mask - 1;
                const uint64_t sk = readlane64(ck, s);
                const int64_t si = (int64_t)readlane64((uint64_t)ci, s);
                if (better(sk, si, tk, ti)) {  // re-check: earlier inserts raised the bar
                    insert(sk, si);
                    refresh();
                }
            } while (mask);
        } else {
            uint64_t bk = pass ? ck : 0ull;
            int64_t bi = pass ? ci : INT64_MAX;
            wave_sort64(bk, bi);
            if (empty()) {
                k = bk;
                i = bi;
            } else {
                wave_merge64(k, i, bk, bi);
            }
            refresh();
        }
    }
};

// ---------------------------------------------------------------------------
// Item-major tile: S 16-B chunks per item (R = 16 S bytes), 64 items per tile.
// ---------------------------------------------------------------------------
template <int S>
struct ItemTile {
    uint32_t u[S * 4];  // this lane's item, raw bytes, member-major [M][C]

    // LDS-DMA the 64-row tile starting at item t0 (rows >= n_valid re-read row
    // n_valid-1, a harmless in-bounds duplicate) into `lds` (64*16*S bytes).
    // AUX = cache-policy bits of the load (0 default, 2 = nt: the pool is
    // streamed once, so it need not displace anything in L2 / MALL).
    template <int AUX>
    __device__ __forceinline__ static void issue(const char* base, int64_t t0, int n_valid, char* lds) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int p = k * 64 + lane;  // 16-B chunk index within the tile
            const int r = p / S, s = p % S;
            const int rs = r < n_valid ? r : n_valid - 1;
            const int m = s ^ (r & 15);
            const char* src = base + (t0 + rs) * (int64_t)(16 * S) + 16 * m;
            __builtin_amdgcn_global_load_lds(
                (const void*)src, (void __attribute__((address_space(3)))*)(lds + k * 1024), 16, 0, AUX);
        }
    }

    // Member-major [M, N, C] (the reference's stack np.array(pred_prob),
    // amg_test.py:441) with 16-B member rows (C * elem = 16): the tile is S = M
    // contiguous 1 KiB runs, member k's 64 items at lds + k*1024 -- one
    // LDS-DMA per member, no swizzle (lane l reads bytes l*16.. of each run:
    // 16 lanes of a ds_read_b128 group hit 16 distinct bank groups).
    template <int AUX>
    __device__ __forceinline__ static void issue_mnc(const char* base, int64_t t0, int n_valid, int64_t sMb,
                                                     char* lds) {
        const int lane = threadIdx.x & 63;
        const int64_t it = t0 + (lane < n_valid ? lane : n_valid - 1);
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const char* src = base + (int64_t)k * sMb + it * 16;
            __builtin_amdgcn_global_load_lds(
                (const void*)src, (void __attribute__((address_space(3)))*)(lds + k * 1024), 16, 0, AUX);
        }
    }

    __device__ __forceinline__ void read_mnc(const char* lds) {
        const int lane = threadIdx.x & 63;
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int m = 0; m < S; ++m) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(lds + m * 1024 + lane * 16);
            u[4 * m + 0] = v.x;
            u[4 * m + 1] = v.y;
            u[4 * m + 2] = v.z;
            u[4 * m + 3] = v.w;
        }
    }

    __device__ __forceinline__ void read(const char* lds) {
        const int lane = threadIdx.x & 63;
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int m = 0; m < S; ++m) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(lds + lane * 16 * S + 16 * (m ^ (lane & 15)));
            u[4 * m + 0] = v.x;
            u[4 * m + 1] = v.y;
            u[4 * m + 2] = v.z;
            u[4 * m + 3] = v.w;
        }
    }

    // element e (= m*C + c) widened to f64
    template <int DT>
    __device__ __forceinline__ double elem(int e) const {
        if constexpr (DT == kF32)
            return (double)__uint_as_float(u[e]);
        else if constexpr (DT == kF64)
            return __longlong_as_double((long long)(((uint64_t)u[2 * e + 1] << 32) | u[2 * e]));
        else
            return bf16_to_f64((u[e >> 1] >> (16 * (e & 1))) & 0xffffu);
    }

    // amg_test.py:441 for this lane's item: member-sequential f64 sum, / M
    template <int DT, int C>
    __device__ __forceinline__ void mean(double dM, double invM, bool pow2, double (&mean)[C]) const {
        constexpr int EB = DT == kF64 ? 8 : (DT == kF32 ? 4 : 2);
        constexpr int M = 16 * S / (C * EB);
        static_assert(M * C * EB == 16 * S, "tile row must hold whole members");
        double acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.0;
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] += elem<DT>(m * C + c);
#pragma unroll
        for (int c = 0; c < C; ++c) mean[c] = div_members(acc[c], dM, invM, pow2);
    }
};

constexpr int kStreamMaxQ = 64;  // one list slot per lane

// block-merge scratch: the wave lists, 64 slots each
template <int WAVES>
struct WaveListsT {
    uint64_t key[WAVES][64];
    int64_t idx[WAVES][64];
};
using WaveLists = WaveListsT<4>;

template <int S, int RING = 1>
struct StreamSmemNMC {
    char tile[4][RING][64 * 16 * S];  // RING staging tiles per wave
    WaveLists lists;
};



struct StreamArgs {
    const void* p;
    int64_t N;
    int M;
    int64_t sN, sM, sC;
    double dM, invM;
    bool pow2;
    int64_t base_idx;
    int64_t per_wave;  // items per wave (multiple of 64)
    const uint32_t* excl;  // exclusion bitmap over items 0..N-1 (1 = out of the pool), or nullptr
    int nlists;        // workspace lists (>= gridDim.x); lists past the grid are written empty
    // stage 2 folded in (ctr != nullptr): the last block merges the grid's
    // lists into (oval, oidx), or into q records at ocand
    uint32_t* ctr;
    double* oval;
    int64_t* oidx;
    Cand* ocand;
    const Cand* extra;  // one more list merged by the fold (chunked jobs: the running list), or nullptr
    // the wide stream's device-side grid choice (heavy items in a folded launch,
    // k_wide_seed_pick): both grids are launched, the one whose role disagrees with
    // the vote exits at once (nullptr: no vote, the kernel runs)
    const uint32_t* vote;
    int vote_heavy;  // 1: run iff the vote picks the deep-ring grid; 0: iff it does not
    // the wide stream's prefilter floor (k_wide_seed_pick), one record, or nullptr
    // (then a chunked job's running list seeds it: extra[q - 1])
    const Cand* seed;
};

// Merge the block's WAVES wave lists (registers, best-first) into the
// block's top-q and write it: to the workspace (wc) or as final (val, idx)
// outputs.  A tree over the waves: at level s, waves w = s mod 2s park their
// list in LDS and waves w = 0 mod 2s merge it in (7 shuffle stages); every
// LDS slot is written once and read once, one barrier per level.
// nw = waves taking part (a power of two <= WAVES; default all of them).
// Cross-block hand-off inside one launch (MI355X_MICROARCH.md, "Valid forms",
// the table's first row): every handed-off byte is stored write-through (sc1:
// relaxed agent-scope atomic stores), every storing wave waits for its stores
// (s_waitcnt vmcnt(0)), the block syncs and ONE lane adds to the problem's
// arrival counter (agent scope); the block whose add returns the last ticket
// reads the bytes with sc1 loads only (relaxed agent-scope atomic loads).  No
// L2 write-back or invalidate: a __threadfence() per block (buffer_wbl2 +
// buffer_inv) made the 1000-block batched launch 118 us instead of ~14.
__device__ __forceinline__ void store_cand_wt(Cand* p, uint64_t k, int64_t i) {
    __hip_atomic_store(&p->key, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&p->idx, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Cand load_cand_wt(const Cand* p) {
    Cand c;
    c.key = __hip_atomic_load(&p->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c.idx = __hip_atomic_load(&p->idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return c;
}
// Every thread of the block calls it after its write-through stores; true in
// every thread of the block whose arrival is the n-th.  The counter wraps
// itself: global_atomic_inc with limit n - 1 returns 0..n-1 and stores 0 after
// the n-th arrival, so the counter is zero again once every block has arrived
// (and stays in [0, n) even when a misuse -- two launches sharing one
// workspace -- interleaves their arrivals: it does not stay broken).
__device__ __forceinline__ bool arrive_last(uint32_t* ctr, uint32_t n, int* lds_ticket) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) *lds_ticket = (int)__builtin_amdgcn_atomic_inc32(ctr, n - 1, __ATOMIC_RELAXED, "agent");
    __syncthreads();
    const int t = *lds_ticket;
    CE_DASSERT(t >= 0 && t < (int)n);
    return t == (int)n - 1;
}

// wt: the list at wc is read inside this launch (a fold / tile merge): store
// it write-through (store_cand_wt).
template <int WAVES>
__device__ inline void block_merge_write(const RegTopQ& tq, WaveListsT<WAVES>& L, int q, Cand* wc, int nlists,
                                         double* oval = nullptr, int64_t* oidx = nullptr, int nw = WAVES,
                                         bool wt = false) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // empty lists for the workspace slots no block of this (occupancy-sized)
    // grid owns: b + gridDim.x, b + 2*gridDim.x, ...
    for (int64_t s = (int64_t)blockIdx.x + gridDim.x; s < nlists; s += gridDim.x)
        for (int r = threadIdx.x; r < q; r += blockDim.x) wc[(s - blockIdx.x) * q + r] = Cand{0ull, -1};
    uint64_t k = tq.k;
    int64_t i = tq.i;
    for (int s = 1; s < WAVES && s < nw; s <<= 1) {  // block-uniform bound
        if ((w & (2 * s - 1)) == s) {
            L.key[w][lane] = k;
            L.idx[w][lane] = i;
        }
        __syncthreads();
        if ((w & (2 * s - 1)) == 0) {
            const uint64_t bk = L.key[w + s][lane];
            const int64_t bi = L.idx[w + s][lane];
            if (readlane64((uint64_t)bi, 0) != (uint64_t)INT64_MAX) {  // partner list not empty
                if (readlane64((uint64_t)i, 0) == (uint64_t)INT64_MAX) {
                    k = bk;  // own list empty: take the partner's as is
                    i = bi;
                } else {
                    wave_merge64(k, i, bk, bi);
                }
            }
        }
    }
    if (w == 0 && lane < q) {
        const bool ok = i != INT64_MAX;
        if (oval) {
            oval[lane] = ok ? key_to_val(k) : __longlong_as_double(0x7ff8000000000000ll);
            oidx[lane] = ok ? i : -1;
        } else if (wt) {
            store_cand_wt(wc + lane, ok ? k : 0ull, ok ? i : -1);
        } else {
            wc[lane] = Cand{ok ? k : 0ull, ok ? i : -1};
        }
    }
}

// A source of best-first candidate lists: Cand records (the workspace, the
// ranks' all-gathered records) or (val, idx) arrays (ce_topq_merge).
template <bool FROM_VALS>
struct ListSrc {
    const Cand* c;
    const double* val;
    const int64_t* idx;
    __device__ __forceinline__ void get(int64_t j, uint64_t& k, int64_t& i) const {
        if constexpr (FROM_VALS) {
            i = idx[j];
            k = order_key(val[j]);
        } else {
            const Cand x = c[j];
            k = x.key;
            i = x.idx;
        }
    }
};

// Merge nl best-first lists of q candidates (empty slots, idx < 0, at each
// list's tail) with the W waves of ONE block into the top-q, written as final
// (oval, oidx) or as records (ocand).  Exact floor from the list heads: the
// q-th best head T_w among a wave's lists is reached by q distinct lists, so
// every global top-q candidate is >= T = the best T_w; only lists whose head
// is >= T (~q of them) are read past their head, and only their entries >= T
// enter the register lists.  One round of head loads (nl / (64 W) per lane)
// plus ~q list loads per block instead of all nl * q candidates.
// bk / bi: W-entry LDS scratch; L: the block-merge scratch.
// The grid's lists followed by one extra list elsewhere (a chunked job's
// running top-q): list g < na at a[g*q..], list na at extra[0..q).
struct FoldSrc {
    const Cand* a;
    int64_t na_q;  // na * q
    const Cand* extra;
    __device__ __forceinline__ void get(int64_t j, uint64_t& k, int64_t& i) const {
        // the grid's lists were handed off in this launch: sc1 loads only
        const Cand x = j < na_q ? load_cand_wt(a + j) : extra[j - na_q];
        k = x.key;
        i = x.idx;
    }
};

template <int W, class Src>
__device__ inline void merge_lists_block(Src src, int64_t seg0, int nl, int q, WaveListsT<W>& L,
                                         uint64_t* bk, int64_t* bi, double* oval, int64_t* oidx, Cand* ocand) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    RegTopQ hq;
    hq.init(q);
    for (int g0 = w * 64; g0 < nl; g0 += W * 64) {
        const int g = g0 + lane;
        uint64_t hk = 0;
        int64_t hid = -1;
        src.get(seg0 + (int64_t)(g < nl ? g : nl - 1) * q, hk, hid);  // clamped: no branch around a load
        hq.offer(hk, hid, g < nl && hid >= 0);
    }
    if (lane == 0) {
        bk[w] = readlane64(hq.k, q - 1);
        bi[w] = (int64_t)readlane64((uint64_t)hq.i, q - 1);
    }
    __syncthreads();
    uint64_t fk = 0;
    int64_t fi = INT64_MAX;
    for (int v = 0; v < W; ++v)
        if (bi[v] != INT64_MAX && better(bk[v], bi[v], fk, fi)) {
            fk = bk[v];
            fi = bi[v];
        }
    if (fi != INT64_MAX) fi += 1;  // admit candidates >= T: strictly better than (T.key, T.idx + 1)
    RegTopQ tq;
    tq.init(q, fk, fi);
    for (int g0 = w * 64; g0 < nl; g0 += W * 64) {
        const int g = g0 + lane;
        uint64_t hk = 0;
        int64_t hid = -1;
        src.get(seg0 + (int64_t)(g < nl ? g : nl - 1) * q, hk, hid);  // L1/L2-hot: read in phase 1
        uint64_t m = __ballot(g < nl && hid >= 0 && better(hk, hid, fk, fi));
        while (m) {  // wave-uniform: each list whose head reaches the floor
            const int s = __builtin_ctzll(m);
            m &= m - 1;
            const int64_t base = seg0 + (int64_t)(g0 + s) * q;
            uint64_t ck = 0;
            int64_t ci = -1;
            src.get(base + (lane < q ? lane : q - 1), ck, ci);
            tq.offer(ck, ci, lane < q && ci >= 0);
        }
    }
    block_merge_write<W>(tq, L, q, ocand, 0, ocand ? nullptr : oval, oidx);
}

// Arrival ticket of a stage-1 grid (a.ctr != nullptr: stage 2 folded into
// stage 1): after its list is written (write-through), every block arrives;
// the last to arrive resets the counter and merges the grid's lists into the
// final output / records.
// The best (k, i) of each group of GS lanes in all its lanes (butterfly).
template <int GS>
__device__ __forceinline__ void group_best(uint64_t& k, int64_t& i) {
    uint64_t pk;
    int64_t pi;
#define CE_GB(J)                    \
    if constexpr (GS > J) {         \
        pk = k;                     \
        pi = i;                     \
        xor_cand<J>(pk, pi);        \
        if (better(pk, pi, k, i)) { \
            k = pk;                 \
            i = pi;                 \
        }                           \
    }
    CE_GB(1) CE_GB(2) CE_GB(4) CE_GB(8)
#undef CE_GB
}

// The fold's merge, one block of W waves over nl <= 64 * W * kLeanJ lists
// handed off in this launch (sc1 loads), in two rounds of loads:
//   1. every thread loads the heads of its lists (t, t + 64W, ...); the best
//      head per group of W lanes gives 64 group bests -- heads of 64 distinct
//      lists -- and the one of rank q-1 is an exact floor T (q lists hold an
//      entry >= T, so every global top-q candidate is >= T); none when fewer
//      than q groups hold a list;
//   2. every thread walks the lists it loaded whose head is >= T: a list's
//      entries >= T are a prefix of it (best-first), read 8 at a time, and
//      appended to a survivor list; every survivor takes the output slot of
//      its rank among the survivors.
// The walk reads only the prefixes (for q = 10 on random data: ~q survivors
// in ~q lists, one round of loads), so q up to 64 stays on this path (round 3
// loaded every entry of every qualifying list, nq * q, and fell back for any
// q > 16).  More than 64 * W survivors (floods of ties at T): the
// register-list merge (merge_lists_block) -- round 2 measured it at ~20 us as
// the last block of the 100M-item grid (sequential per-list loads, sort
// networks on cold lists).
constexpr int kLeanJ = 8;
template <int W>
struct LeanMergeSmem {
    uint64_t gk[64];
    int64_t gi[64];
    int part[W][64];
    int nsurv, ticket;
    uint64_t bk[W];
    int64_t bi[W];
};

template <int W, class Src>
__device__ inline void merge_lists_lean(Src src, int nl, int q, WaveListsT<W>& L, LeanMergeSmem<W>& sm,
                                        double* oval, int64_t* oidx, Cand* ocand) {
    constexpr int BS = 64 * W, GS = W;  // lanes per group: 64 groups
    constexpr int CAP = 64 * W;         // survivors held (the block-merge scratch)
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    uint64_t* sk = &L.key[0][0];  // survivors: the block-merge scratch, 64 W slots
    int64_t* si = &L.idx[0][0];
    // 1. heads, all loads in flight
    uint64_t hk[kLeanJ];
    int64_t hi[kLeanJ];
#pragma unroll
    for (int j = 0; j < kLeanJ; ++j) {
        hk[j] = 0;
        hi[j] = INT64_MAX;
        const int g = tid + BS * j;
        if (g < nl) src.get((int64_t)g * q, hk[j], hi[j]);
    }
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
#pragma unroll
    for (int j = 0; j < kLeanJ; ++j) {
        if (hi[j] < 0) hi[j] = INT64_MAX;  // empty list: no head
        if (hi[j] != INT64_MAX && better(hk[j], hi[j], bk, bi)) {
            bk = hk[j];
            bi = hi[j];
        }
    }
    group_best<GS>(bk, bi);
    if ((tid & (GS - 1)) == 0) {
        sm.gk[tid / GS] = bk;
        sm.gi[tid / GS] = bi;
    }
    if (tid == 0) sm.nsurv = 0;
    __syncthreads();
    {
        const uint64_t mk = sm.gk[lane];
        const int64_t mi = sm.gi[lane];
        int r = 0;
#pragma unroll
        for (int j = 0; j < 64 / W; ++j) {
            const int o = w * (64 / W) + j;
            r += better(sm.gk[o], sm.gi[o], mk, mi);
        }
        sm.part[w][lane] = r;
    }
    __syncthreads();
    uint64_t fk = 0;  // no floor: admit everything
    int64_t fi = INT64_MAX;
    {
        int r = 0;
#pragma unroll
        for (int j = 0; j < W; ++j) r += sm.part[j][lane];
        const uint64_t hit = __ballot(r == q - 1 && sm.gi[lane] != INT64_MAX);
        if (hit) {
            const int sl = __builtin_ctzll(hit);
            fk = sm.gk[sl];
            fi = sm.gi[sl];
        }
    }
    // 2. the prefix >= T of every list whose head is >= T, 8 entries per round.
    // Rolled, re-reading the head (L2-hot) instead of indexing hk / hi: a runtime
    // index would put them in scratch, an unrolled walk raises the register
    // peak of every streaming kernel this merge is inlined into.
#pragma unroll 1
    for (int j = 0; j < kLeanJ; ++j) {
        const int g = tid + BS * j;
        if (g >= nl) break;
        const int64_t base = (int64_t)g * q;
        uint64_t h0;
        int64_t i0;
        src.get(base, h0, i0);
        if (i0 < 0 || better(fk, fi, h0, i0)) continue;
#pragma unroll 1
        for (int e0 = 0; e0 < q; e0 += 8) {
            uint64_t ck[8];
            int64_t ci[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) src.get(base + (e0 + u < q ? e0 + u : q - 1), ck[u], ci[u]);  // clamped
            int take = 0;  // the leading entries of this round that are >= T
#pragma unroll
            for (int u = 0; u < 8; ++u)
                take += (take == u && e0 + u < q && ci[u] >= 0 && !better(fk, fi, ck[u], ci[u])) ? 1 : 0;
            const int s0 = take ? atomicAdd(&sm.nsurv, take) : 0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (u < take && s0 + u < CAP) {
                    sk[s0 + u] = ck[u];
                    si[s0 + u] = ci[u];
                }
            if (take < 8) break;
        }
    }
    __syncthreads();
    const int ns = sm.nsurv;
    if (ns > CAP) {  // block-uniform: floods of ties at T -> the register-list merge
        merge_lists_block<W>(src, 0, nl, q, L, sm.bk, sm.bi, oval, oidx, ocand);
        return;
    }
    if (tid < ns) {
        const uint64_t mk = sk[tid];
        const int64_t mi = si[tid];
        int r = 0;
        for (int j = 0; j < ns; ++j) r += better(sk[j], si[j], mk, mi);
        if (r < q) {
            if (ocand) {
                ocand[r] = Cand{mk, mi};
            } else {
                oval[r] = key_to_val(mk);
                oidx[r] = mi;
            }
        }
    }
    for (int r = ns + tid; r < q; r += BS) {  // fewer candidates than q: padding
        if (ocand) {
            ocand[r] = Cand{0ull, -1};
        } else {
            oval[r] = __longlong_as_double(0x7ff8000000000000ll);
            oidx[r] = -1;
        }
    }
}

template <int W>
__device__ inline void fold_merge(uint32_t* ctr, double* oval, int64_t* oidx, Cand* ocand, int q, const Cand* wc0,
                                  WaveListsT<W>& L, const Cand* extra = nullptr) {
    __shared__ LeanMergeSmem<W> ms;
    if (!arrive_last(ctr, gridDim.x, &ms.ticket)) return;  // block-uniform
    // extra (a chunked job's running list) may be ocand itself: every input is
    // read before the outputs are written (barriers in between)
    const int nl = (int)gridDim.x + (extra ? 1 : 0);
    const FoldSrc src{wc0, (int64_t)gridDim.x * q, extra};
    if (nl <= 64 * W * kLeanJ)
        merge_lists_lean<W>(src, nl, q, L, ms, oval, oidx, ocand);
    else
        merge_lists_block<W>(src, 0, nl, q, L, ms.bk, ms.bi, oval, oidx, ocand);
}

// Item-major, dense rows of 16*S bytes, LDS-DMA staged (AUX: DMA cache policy);
// MNC: the member-major stack with 16-B member rows instead (S = M members,
// member stride a.sM elements).
// RING tiles per wave: 2 (the default for 16-KiB tiles) puts the next two
// tiles in flight while one is read -- 139 KB of LDS, so ONE block (4 waves)
// per CU instead of 2 blocks with one tile each: the same bytes in flight from
// half as many streams.  Measured on one box, alternating (profiles/
// r05_nmc_ring_ab.json): [N,M,C] 0.856-0.860 -> 0.883-0.884 of HBM, [M,N,C]
// 0.835 -> 0.846.
template <int DT, int C, int S, int AUX, bool MNC = false, int RING = 1>
__global__ __launch_bounds__(256) void k_stream_nmc(StreamArgs a, int q, Cand* __restrict__ wc) {
    static_assert(RING == 1 || RING == 2, "one or two tiles per wave");
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    CE_DASSERT((int)gridDim.x <= a.nlists && q >= 1 && q <= kStreamMaxQ);
    __shared__ __attribute__((aligned(16))) StreamSmemNMC<S, RING> sm;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t lo, hi, step;
    // tile distribution (measured on two boxes, alternating runs,
    // profiles/r03_tile_order.json): item-major -- grid-cyclic, equal on a box
    // where a contiguous run per wave reaches 0.871 and +2.5 % (0.836 -> 0.859)
    // on one where it reaches only 0.836; member-major -- block-interleaved
    // (+0.3-0.5 % over runs), grid-cyclic 4 % slower there
    if constexpr (!MNC) {  // grid-cyclic: wave g takes tiles g, g + W, g + 2W, ... (W = the grid's waves), so
        // the tiles in flight at any moment form one contiguous sweep of the pool
        const int64_t W = (int64_t)gridDim.x * 4;
        lo = ((int64_t)blockIdx.x * 4 + w) * 64;
        hi = a.N;
        step = W * 64;
    } else {  // the block's 4 waves take alternate tiles of the block's run (adjacent bursts per member row;
        // 8 or 64 grid-cyclic sweeps, each over 1/8 or 1/64 of the pool, measured no better: r04_mnc_order.json)
        const int64_t blo = (int64_t)blockIdx.x * 4 * a.per_wave;
        hi = blo + 4 * a.per_wave < a.N ? blo + 4 * a.per_wave : a.N;
        lo = blo + 64 * w;
        step = 256;
    }
    if (lo > hi) lo = hi;
    RegTopQ tq;
    tq.init(q);
    const char* base = static_cast<const char*>(a.p);
    constexpr int EB = DT == kF64 ? 8 : (DT == kF32 ? 4 : 2);
    const int64_t sMb = a.sM * EB;
    auto issue = [&](int64_t t, int nv, int slot) {
        char* lds = sm.tile[w][slot];
        if constexpr (MNC) ItemTile<S>::template issue_mnc<AUX>(base, t, nv, sMb, lds);
        else ItemTile<S>::template issue<AUX>(base, t, nv, lds);
    };
    ItemTile<S> t;
#pragma unroll
    for (int r = 0; r < RING; ++r)
        if (lo + r * step < hi) issue(lo + r * step, (int)min<int64_t>(64, hi - lo - r * step), r);
    int slot = 0;
    for (int64_t t0 = lo; t0 < hi; t0 += step) {
        // S DMA instructions per tile (always: short tiles re-read their last row),
        // so the tiles issued after this one are (RING - 1) * S instructions
        if constexpr (RING == 2) {
            if (t0 + step < hi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const char* lds = sm.tile[w][slot];
        if constexpr (MNC) t.read_mnc(lds);
        else t.read(lds);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const int64_t t1 = t0 + RING * step;
        if (t1 < hi) issue(t1, (int)min<int64_t>(64, hi - t1), slot);
        slot = RING == 1 ? 0 : slot ^ 1;
        double mean[C];
        t.template mean<DT, C>(a.dM, a.invM, a.pow2, mean);
        const double h = entropy_row<C>(mean);
        const int64_t i = t0 + lane;
        bool ok = i < hi;
        if (a.excl) ok = ok && !excluded(a.excl, i < hi ? i : hi - 1);
        tq.offer(order_key(h), i + a.base_idx, ok);
    }
    block_merge_write<4>(tq, sm.lists, q, wc + (int64_t)blockIdx.x * q, a.nlists, nullptr, nullptr, 4, a.ctr != nullptr);
    if (a.ctr) fold_merge<4>(a.ctr, a.oval, a.oidx, a.ocand, q, wc, sm.lists, a.extra);
}

// Any strides (vector loads when aligned): member-major [M, N, C] streams
// coalesced across lanes.  IPL items per lane per iteration keep IPL x M
// member loads in flight per lane.
template <class Src, int IPL, int UNR>
__device__ __forceinline__ void stream_direct_range(const Src& src, int64_t lo, int64_t hi, int64_t rel, int q,
                                                    RegTopQ& tq, const uint32_t* excl = nullptr) {
    const int lane = threadIdx.x & 63;
    for (int64_t t0 = lo; t0 < hi; t0 += 64 * IPL) {
        uint64_t k[IPL];
        int64_t items[IPL];
#pragma unroll
        for (int u = 0; u < IPL; ++u) {
            const int64_t i = t0 + 64 * u + lane;
            items[u] = i < hi ? i : hi - 1;  // clamped: every lane loads, no branch per item
        }
        src.template keys<UNR, IPL>(items, k);
#pragma unroll
        for (int u = 0; u < IPL; ++u) {
            const int64_t i = t0 + 64 * u + lane;
            bool ok = i < hi;
            if (excl) ok = ok && !excluded(excl, items[u]);  // items[u]: i clamped into the pool
            tq.offer(k[u], i + rel, ok);
        }
    }
}

template <class Src, int IPL, int UNR>
__global__ __launch_bounds__(256) void k_stream_direct(Src src, StreamArgs a, int q, Cand* __restrict__ wc) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    CE_DASSERT((int)gridDim.x <= a.nlists && q >= 1 && q <= kStreamMaxQ);
    __shared__ WaveLists sm;
    const int w = threadIdx.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    int64_t lo = gw * a.per_wave;
    int64_t hi = lo + a.per_wave;
    if (hi > a.N) hi = a.N;
    if (lo > hi) lo = hi;
    RegTopQ tq;
    tq.init(q);
    stream_direct_range<Src, IPL, UNR>(src, lo, hi, a.base_idx, q, tq, a.excl);
    block_merge_write<4>(tq, sm, q, wc + (int64_t)blockIdx.x * q, a.nlists, nullptr, nullptr, 4, a.ctr != nullptr);
    if (a.ctr) fold_merge<4>(a.ctr, a.oval, a.oidx, a.ocand, q, wc, sm, a.extra);
}

// Batched pools (amg_test.py:345's per-user loop in one launch): user u owns
// segment [offsets[u], offsets[u+1]), split over bpu consecutive blocks (block
// b: user b / bpu, part b % bpu) in whole iterations of 64*IPL items; the
// block's waves split its part the same way.  bpu == 1: the block's merged
// top-q is the user's final answer (oval/oidx, user-local positions); bpu > 1:
// the block writes its list to wc[b*q ..] for a per-user merge.
// offsets == nullptr: one segment [0, n) with positions base_idx + i (the
// single-launch path for small pools).  excl: exclusion bitmap over the
// tensor's items, or nullptr.  Launched with WAVES or fewer waves (a power of two).
template <class Src, int IPL, int UNR, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_stream_seg(Src src, const int64_t* __restrict__ offsets, int64_t n,
                                                            int64_t base_idx, int q, int bpu,
                                                            double* __restrict__ oval, int64_t* __restrict__ oidx,
                                                            Cand* __restrict__ wc, const uint32_t* __restrict__ excl) {
    stage_log_table();  // glibc log table -> LDS (ce_glibc_log.hpp)
    __shared__ WaveListsT<WAVES> sm;
    __shared__ uint64_t fk_s[4 * WAVES];
    __shared__ int64_t fi_s[4 * WAVES];
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = threadIdx.x & 63;
    const int u = blockIdx.x / bpu, part = blockIdx.x % bpu;
    const int64_t s0 = offsets ? offsets[u] : 0, s1 = offsets ? offsets[u + 1] : n;
    const int64_t len = s1 > s0 ? s1 - s0 : 0;
    constexpr int64_t kIt = 64 * IPL;
    const int64_t its = (len + kIt - 1) / kIt;                  // iterations of the segment
    const int64_t its_b = (its + bpu - 1) / bpu;                // per block
    const int64_t its_w = (its_b + nw - 1) / nw;                // per wave
    int64_t lo = s0 + ((int64_t)part * its_b + (int64_t)w * its_w) * kIt;
    int64_t hi_b = s0 + ((int64_t)part + 1) * its_b * kIt;      // this block's end
    if (hi_b > s1) hi_b = s1;
    int64_t hi = lo + its_w * kIt < hi_b ? lo + its_w * kIt : hi_b;
    if (lo > hi) lo = hi;
    const int64_t rel = (offsets ? 0 : base_idx) - s0;
    // First iteration's keys, then a block-wide floor before any offer: the
    // best of each 16-lane row is a distinct item, so the q-th best of the
    // block's 4*nw row bests is an exact lower bound (q items of the block's
    // part are >= it).  Most candidates then fail the first ballot and the
    // sort networks a cold wave list would run on every early batch are skipped.
    uint64_t k0[IPL];
    int64_t it0[IPL];
    bool ok0[IPL];
#pragma unroll
    for (int v = 0; v < IPL; ++v) {
        const int64_t i = lo + 64 * v + lane;
        it0[v] = i < hi ? i : hi - 1;
        ok0[v] = false;
        k0[v] = 0;
    }
    if (lo < hi) {  // wave-uniform
        src.template keys<UNR, IPL>(it0, k0);
#pragma unroll
        for (int v = 0; v < IPL; ++v) {
            ok0[v] = lo + 64 * v + lane < hi;
            if (excl) ok0[v] = ok0[v] && !excluded(excl, it0[v]);
        }
    }
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
#pragma unroll
    for (int v = 0; v < IPL; ++v)
        if (ok0[v] && better(k0[v], lo + 64 * v + lane + rel, bk, bi)) {
            bk = k0[v];
            bi = lo + 64 * v + lane + rel;
        }
    row_best16(bk, bi);
    if ((lane & 15) == 0) {
        fk_s[w * 4 + (lane >> 4)] = bk;
        fi_s[w * 4 + (lane >> 4)] = bi;
    }
    __syncthreads();
    uint64_t fk = 0;
    int64_t fi = INT64_MAX;
    const int nb = 4 * nw;
    if (q <= nb) {
        bool hit = false;
        uint64_t vk = 0;
        int64_t vi = INT64_MAX;
        if (lane < nb) {
            vk = fk_s[lane];
            vi = fi_s[lane];
            int rank = 0;
            for (int v = 0; v < nb; ++v) rank += better(fk_s[v], fi_s[v], vk, vi);
            hit = vi != INT64_MAX && rank == q - 1;
        }
        const uint64_t m = __ballot(hit);
        if (m) {
            const int sl = __builtin_ctzll(m);
            fk = readlane64(vk, sl);
            fi = (int64_t)readlane64((uint64_t)vi, sl) + 1;  // admit candidates >= the bound
        }
    }
    RegTopQ tq;
    tq.init(q, fk, fi);
#pragma unroll
    for (int v = 0; v < IPL; ++v) tq.offer(k0[v], lo + 64 * v + lane + rel, ok0[v]);
    if (lo + kIt < hi) stream_direct_range<Src, IPL, UNR>(src, lo + kIt, hi, rel, q, tq, excl);
    if (bpu == 1) {
        const int64_t slot = (int64_t)u * q;
        block_merge_write<WAVES>(tq, sm, q, nullptr, 0, oval + slot, oidx + slot, nw);
    } else {
        block_merge_write<WAVES>(tq, sm, q, wc + (int64_t)blockIdx.x * q, 0, nullptr, nullptr, nw);
    }
}

}  // namespace ce

