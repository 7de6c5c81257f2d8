// ce_topq.hpp -- block-level top-q engine staged in LDS (gfx950, wave64).
//
// Replaces np.argsort(ent)[::-1][:q] (amg_test.py:445, :452, :480) -- a full
// O(N log N) sort for a top-10 -- with a filter + bounded buffer:
//   * every thread offers one candidate (order key, index) per round; a
//     candidate survives only if it beats the block's current threshold (the
//     q-th best seen so far), so after the first few rounds almost nothing
//     is written;
//   * survivors are appended to an LDS buffer with one wave-aggregated atomic
//     (ballot + mbcnt);
//   * when the buffer could overflow in the next round it is bitonic-sorted
//     (best first), cut to q entries and the threshold is raised.
// The total order is (key desc, index asc) -- keys+indices are unique, so the
// sort is a strict order and the result is deterministic.
#pragma once
#include "ce_device.hpp"

namespace ce {

// One workspace candidate: order key + position, one 16-B load/store.
struct __attribute__((aligned(16))) Cand {
    uint64_t key;
    int64_t idx;
};

template <int CAP>
struct TopQSmem {
    uint64_t key[CAP];
    int64_t idx[CAP];
    uint64_t tkey;
    int64_t tidx;
    int count;
    int pad_[3];
    uint64_t red[16];  // per-wave scratch for reductions
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int mbcnt(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <int CAP, int BS>
struct TopQ {
    TopQSmem<CAP>& s;
    uint64_t tkey;  // register copy of the threshold (block-uniform)
    int64_t tidx;

    __device__ __forceinline__ explicit TopQ(TopQSmem<CAP>& sm) : s(sm) {}

    // Start with threshold (k0, i0): candidates must be strictly better.
    __device__ __forceinline__ void init(uint64_t k0 = 0, int64_t i0 = INT64_MAX) {
        if (threadIdx.x == 0) {
            s.count = 0;
            s.tkey = k0;
            s.tidx = i0;
        }
        tkey = k0;
        tidx = i0;
        __syncthreads();
    }

    // Append if better than the threshold.  No barrier.
    __device__ __forceinline__ void offer(uint64_t k, int64_t i, bool valid) {
        const bool pass = valid && better(k, i, tkey, tidx);
        const uint64_t mask = __ballot(pass);
        if (mask == 0) return;  // wave-uniform
        int base = 0;
        if (lane_id() == 0) base = atomicAdd(&s.count, __popcll(mask));
        base = __shfl(base, 0);
        if (pass) {
            const int pos = base + mbcnt(mask);
            s.key[pos] = k;
            s.idx[pos] = i;
        }
    }

    // Sort the first n buffer entries best-first (bitonic over the next power of 2).
    __device__ void sort_buffer(int n) {
        int P = 1;
        while (P < n) P <<= 1;
        for (int t = n + threadIdx.x; t < P; t += BS) {
            s.key[t] = 0;
            s.idx[t] = INT64_MAX;
        }
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = threadIdx.x; t < (P >> 1); t += BS) {
                    const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                    const int l = i + j;
                    const bool desc = (i & k) == 0;
                    const uint64_t ki = s.key[i], kl = s.key[l];
                    const int64_t ii = s.idx[i], il = s.idx[l];
                    if (better(kl, il, ki, ii) == desc) {
                        s.key[i] = kl;
                        s.key[l] = ki;
                        s.idx[i] = il;
                        s.idx[l] = ii;
                    }
                }
                __syncthreads();
            }
        }
    }

    // Sort, keep the best q, raise the threshold.  Block-uniform call.
    __device__ void flush(int n, int q) {
        sort_buffer(n);
        if (threadIdx.x == 0) {
            s.count = n < q ? n : q;
            if (n >= q) {
                s.tkey = s.key[q - 1];
                s.tidx = s.idx[q - 1];
            }
        }
        __syncthreads();
        tkey = s.tkey;
        tidx = s.tidx;
    }

    // End of a round of at most `round` appends per block: flush if the next
    // round could overflow the buffer.
    __device__ __forceinline__ void end_round(int q, int round) {
        __syncthreads();
        const int n = s.count;
        __syncthreads();
        if (n > CAP - round) flush(n, q);
    }

    // Final: sorted best-first, count = min(#candidates, q).  Returns count.
    __device__ int finish(int q) {
        __syncthreads();
        const int n = s.count;
        __syncthreads();
        flush(n, q);
        return n < q ? n : q;
    }
};

}  // namespace ce
