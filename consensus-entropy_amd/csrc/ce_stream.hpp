// ce_stream.hpp -- the streaming mc kernel (stage 1 of ce_select_mc, q <= 64).
//
// One pass over the committee tensor at HBM rate.  Every wave is independent
// while streaming (no block barriers in the loop): it owns a contiguous run of
// 64-item tiles, scores one item per lane, and keeps its own top-q candidates
// in a private LDS buffer (WaveTopQ).  The block's four wave lists are merged
// once at the end.
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
// Per-wave top-q: a CAPW-entry LDS buffer, threshold in (wave-uniform) regs.
// ---------------------------------------------------------------------------
template <int CAPW>
struct WaveTopQ {
    uint64_t* key;
    int64_t* idx;
    int count;
    uint64_t tkey;
    int64_t tidx;

    __device__ __forceinline__ void init(uint64_t* k, int64_t* i) {
        key = k;
        idx = i;
        count = 0;
        tkey = 0;
        tidx = INT64_MAX;
    }

    // bitonic sort of [0, n) best-first (wave-synchronous: a single wave's LDS
    // operations execute in program order, so no barrier is needed)
    __device__ void sort(int n) {
        const int lane = threadIdx.x & 63;
        int P = 1;
        while (P < n) P <<= 1;
        for (int t = n + lane; t < P; t += 64) {
            key[t] = 0;
            idx[t] = INT64_MAX;
        }
        __builtin_amdgcn_wave_barrier();
        for (int k = 2; k <= P; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = lane; t < (P >> 1); t += 64) {
                    const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                    const int l = i + j;
                    const bool desc = (i & k) == 0;
                    const uint64_t ki = key[i], kl = key[l];
                    const int64_t ii = idx[i], il = idx[l];
                    if (better(kl, il, ki, ii) == desc) {
                        key[i] = kl;
                        key[l] = ki;
                        idx[i] = il;
                        idx[l] = ii;
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
    }

    __device__ void flush(int q) {
        const int n = count;
        sort(n);
        count = n < q ? n : q;
        if (n >= q) {
            tkey = key[q - 1];
            tidx = idx[q - 1];
        }
    }

    __device__ __forceinline__ void offer(uint64_t k, int64_t i, bool valid, int q) {
        const bool pass = valid && better(k, i, tkey, tidx);
        const uint64_t mask = __ballot(pass);
        if (mask == 0) return;
        if (pass) {
            const int pos = count + mbcnt(mask);
            key[pos] = k;
            idx[pos] = i;
        }
        __builtin_amdgcn_wave_barrier();
        count += __popcll(mask);
        if (count > CAPW - 64) flush(q);
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

constexpr int kStreamCapW = 128;  // per-wave candidate buffer: q <= 64
constexpr int kStreamMaxQ = kStreamCapW - 64;

template <int S>
struct StreamSmemNMC {
    char tile[4][64 * 16 * S];  // one staging tile per wave
    uint64_t key[4][kStreamCapW];
    int64_t idx[4][kStreamCapW];
};

struct StreamSmemDirect {
    uint64_t key[4][kStreamCapW];
    int64_t idx[4][kStreamCapW];
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
    int nlists;        // workspace lists (>= gridDim.x); lists past the grid are written empty
};

// Merge the block's 4 wave lists (each best-first, <= q entries, counts in
// cnt[]) into the block's top-q and write it to the workspace.  Wave 0 does it
// in LDS scratch that held the wave buffers.
__device__ inline void block_merge_write(uint64_t (*key)[kStreamCapW], int64_t (*idx)[kStreamCapW], int* cnt,
                                         int q, Cand* wc, int nlists, double* oval = nullptr,
                                         int64_t* oidx = nullptr) {
    // empty lists for the workspace slots no block of this (occupancy-sized)
    // grid owns: b + gridDim.x, b + 2*gridDim.x, ...
    for (int64_t s = (int64_t)blockIdx.x + gridDim.x; s < nlists; s += gridDim.x)
        for (int r = threadIdx.x; r < q; r += blockDim.x) wc[(s - blockIdx.x) * q + r] = Cand{0ull, -1};
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        // gather wave 1..3 lists behind wave 0's (wave 0's buffer has room:
        // 4 * q <= 256 entries are staged in the two first rows of key/idx)
        uint64_t* mk = &key[0][0];
        int64_t* mi = &idx[0][0];
        int n = cnt[0];
        // key[0..3] rows are contiguous: [4][128] -> 512 entries of scratch
        for (int w = 1; w < 4; ++w) {
            for (int r = lane; r < cnt[w]; r += 64) {
                mk[n + r] = key[w][r];
                mi[n + r] = idx[w][r];
            }
            n += cnt[w];
            __builtin_amdgcn_wave_barrier();
        }
        WaveTopQ<4 * kStreamCapW> wq;
        wq.init(mk, mi);
        wq.count = n;
        wq.sort(n);
        __builtin_amdgcn_wave_barrier();
        for (int r = lane; r < q; r += 64) {
            const bool ok = r < n;
            if (oval) {
                oval[r] = ok ? key_to_val(mk[r]) : __longlong_as_double(0x7ff8000000000000ll);
                oidx[r] = ok ? mi[r] : -1;
            } else {
                wc[r] = Cand{ok ? mk[r] : 0ull, ok ? mi[r] : -1};
            }
        }
    }
}

// Item-major, dense rows of 16*S bytes, LDS-DMA staged (AUX: DMA cache policy).
template <int DT, int C, int S, int AUX>
__global__ __launch_bounds__(256) void k_stream_nmc(StreamArgs a, int q, Cand* __restrict__ wc) {
    __shared__ __attribute__((aligned(16))) StreamSmemNMC<S> sm;
    __shared__ int cnt[4];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    int64_t lo = gw * a.per_wave;
    int64_t hi = lo + a.per_wave;
    if (hi > a.N) hi = a.N;
    if (lo > hi) lo = hi;
    WaveTopQ<kStreamCapW> tq;
    tq.init(sm.key[w], sm.idx[w]);
    const char* base = static_cast<const char*>(a.p);
    char* lds = sm.tile[w];
    ItemTile<S> t;
    if (lo < hi) ItemTile<S>::template issue<AUX>(base, lo, (int)min<int64_t>(64, hi - lo), lds);
    for (int64_t t0 = lo; t0 < hi; t0 += 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t.read(lds);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const int64_t t1 = t0 + 64;
        if (t1 < hi) ItemTile<S>::template issue<AUX>(base, t1, (int)min<int64_t>(64, hi - t1), lds);
        double mean[C];
        t.template mean<DT, C>(a.dM, a.invM, a.pow2, mean);
        const double h = entropy_row<C>(mean);
        const int64_t i = t0 + lane;
        tq.offer(order_key(h), i + a.base_idx, i < hi, q);
    }
    tq.flush(q);
    if (lane == 0) cnt[w] = tq.count;
    const int64_t slot = (int64_t)blockIdx.x * q;
    block_merge_write(sm.key, sm.idx, cnt, q, wc + slot, a.nlists);
}

// Any strides (vector loads when aligned): member-major [M, N, C] streams
// coalesced across lanes.  IPL items per lane per iteration keep IPL x M
// member loads in flight per lane.
template <class Src, int IPL, int UNR>
__device__ __forceinline__ void stream_direct_range(const Src& src, int64_t lo, int64_t hi, int64_t rel, int q,
                                                    WaveTopQ<kStreamCapW>& tq) {
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
            tq.offer(k[u], i + rel, i < hi, q);
        }
    }
}

template <class Src, int IPL, int UNR>
__global__ __launch_bounds__(256) void k_stream_direct(Src src, StreamArgs a, int q, Cand* __restrict__ wc) {
    __shared__ __attribute__((aligned(16))) StreamSmemDirect sm;
    __shared__ int cnt[4];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    int64_t lo = gw * a.per_wave;
    int64_t hi = lo + a.per_wave;
    if (hi > a.N) hi = a.N;
    if (lo > hi) lo = hi;
    WaveTopQ<kStreamCapW> tq;
    tq.init(sm.key[w], sm.idx[w]);
    stream_direct_range<Src, IPL, UNR>(src, lo, hi, a.base_idx, q, tq);
    tq.flush(q);
    if (lane == 0) cnt[w] = tq.count;
    const int64_t slot = (int64_t)blockIdx.x * q;
    block_merge_write(sm.key, sm.idx, cnt, q, wc + slot, a.nlists);
}

// Batched pools (amg_test.py:345's per-user loop in one launch): block u owns
// segment [offsets[u], offsets[u+1]), its 4 waves split it, and the block's
// merged top-q is the user's final answer (user-local positions).
// offsets == nullptr: one segment [0, n) with positions base_idx + i (the
// single-launch path for small pools).
template <class Src, int IPL, int UNR>
__global__ __launch_bounds__(256) void k_stream_seg(Src src, const int64_t* __restrict__ offsets, int64_t n,
                                                     int64_t base_idx, int q, double* __restrict__ oval,
                                                     int64_t* __restrict__ oidx) {
    __shared__ __attribute__((aligned(16))) StreamSmemDirect sm;
    __shared__ int cnt[4];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t s0 = offsets ? offsets[blockIdx.x] : 0, s1 = offsets ? offsets[blockIdx.x + 1] : n;
    const int64_t len = s1 > s0 ? s1 - s0 : 0;
    const int64_t per = ((len + 3) / 4 + 63) / 64 * 64;
    int64_t lo = s0 + w * per;
    int64_t hi = lo + per < s1 ? lo + per : s1;
    if (lo > hi) lo = hi;
    WaveTopQ<kStreamCapW> tq;
    tq.init(sm.key[w], sm.idx[w]);
    stream_direct_range<Src, IPL, UNR>(src, lo, hi, (offsets ? 0 : base_idx) - s0, q, tq);
    tq.flush(q);
    if (lane == 0) cnt[w] = tq.count;
    const int64_t slot = (int64_t)blockIdx.x * q;
    block_merge_write(sm.key, sm.idx, cnt, q, nullptr, 0, oval + slot, oidx + slot);
}

}  // namespace ce
