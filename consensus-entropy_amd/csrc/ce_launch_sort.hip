// ce_launch_sort.hip -- the sort path for q beyond the list kernels (ce_sort.hpp):
// the only TU that instantiates its kernels.
#include "ce_host.hpp"

using namespace ce;

namespace ce {
__device__ __forceinline__ uint32_t sort_digit(const Cand& c, SortPass ps) {
    if (ps.field == 0) return 255u - (uint32_t)((c.key >> ps.shift) & 255u);
    return (uint32_t)(((uint64_t)c.idx >> ps.shift) & 255u);
}

// The lanes of this wave holding the same digit (valid lanes only).
__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint64_t m = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? m : ~m;
    }
    return valid ? peers : 0ull;
}

__global__ __launch_bounds__(256) void k_sort_hist(const Cand* __restrict__ in, SortGeom g, SortPass ps,
                                                    uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt[4][256];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + w;
    CE_DASSERT(g.chunk % 64 == 0 && (int64_t)g.nw * g.chunk >= g.n);
    for (int d = lane; d < 256; d += 64) cnt[w][d] = 0;
    __builtin_amdgcn_wave_barrier();
    if (wv >= g.nw) return;  // wave-uniform; no block barrier below
    const int64_t lo = (int64_t)wv * g.chunk, hi = lo + g.chunk < g.n ? lo + g.chunk : g.n;
    for (int64_t i0 = lo; i0 < hi; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool ok = i < hi;
        const uint32_t d = ok ? sort_digit(in[i], ps) : 0u;
        const uint64_t peers = digit_peers(d, ok);
        const uint64_t below = peers & ((1ull << lane) - 1ull);
        if (ok && below == 0) cnt[w][d] += (uint32_t)__popcll(peers);  // the digit's leader lane
        __builtin_amdgcn_wave_barrier();
    }
    for (int d = lane; d < 256; d += 64) hist[(int64_t)d * g.nw + wv] = cnt[w][d];
}

// Block d: exclusive prefix of hist[d][0..nw) in place, the digit's total to dtot[d].
__global__ __launch_bounds__(256) void k_sort_scan(uint32_t* __restrict__ hist, int nw, uint64_t* __restrict__ dtot) {
    __shared__ uint64_t part[256];
    uint32_t* h = hist + (int64_t)blockIdx.x * nw;
    const int per = (nw + 255) / 256;
    const int b0 = threadIdx.x * per;
    uint64_t s = 0;
    for (int j = 0; j < per; ++j)
        if (b0 + j < nw) s += h[b0 + j];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {  // 256 partial sums: one thread
        uint64_t run = 0;
        for (int t = 0; t < 256; ++t) {
            const uint64_t v = part[t];
            part[t] = run;
            run += v;
        }
        dtot[blockIdx.x] = run;
    }
    __syncthreads();
    uint64_t run = part[threadIdx.x];
    for (int j = 0; j < per; ++j)
        if (b0 + j < nw) {
            const uint32_t v = h[b0 + j];
            h[b0 + j] = (uint32_t)run;  // < n <= 2^32 records
            run += v;
        }
}

__global__ __launch_bounds__(256) void k_sort_scatter(const Cand* __restrict__ in, Cand* __restrict__ out, SortGeom g,
                                                       SortPass ps, const uint32_t* __restrict__ hist,
                                                       const uint64_t* __restrict__ dtot) {
    __shared__ uint64_t next[4][256];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + w;
    if (wv >= g.nw) return;  // wave-uniform; no block barrier in this kernel
    // digit bases: lane l owns digits 4l .. 4l+3; exclusive scan of the lanes' sums
    uint64_t t[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        t[j] = dtot[4 * lane + j];
        s += t[j];
    }
    uint64_t inc = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t v = __shfl_up(inc, off);
        if (lane >= off) inc += v;
    }
    uint64_t base = inc - s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int d = 4 * lane + j;
        next[w][d] = base + hist[(int64_t)d * g.nw + wv];
        base += t[j];
    }
    __builtin_amdgcn_wave_barrier();
    const int64_t lo = (int64_t)wv * g.chunk, hi = lo + g.chunk < g.n ? lo + g.chunk : g.n;
    for (int64_t i0 = lo; i0 < hi; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool ok = i < hi;
        Cand c{0ull, -1};
        if (ok) c = in[i];
        const uint32_t d = ok ? sort_digit(c, ps) : 0u;
        const uint64_t peers = digit_peers(d, ok);
        const uint64_t below = peers & ((1ull << lane) - 1ull);
        uint64_t dst = 0;
        if (ok) dst = next[w][d] + (uint64_t)__popcll(below);
        CE_DASSERT(!ok || dst < (uint64_t)g.n);
        __builtin_amdgcn_wave_barrier();
        if (ok) {
            out[dst] = c;
            if (below == 0) next[w][d] += (uint64_t)__popcll(peers);  // the digit's leader lane
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Records of entropies ent[0..n): {order key, idx0 + i}; key 0 for items whose
// exclusion bit is set (excl over items 0..n-1, or nullptr).
__global__ __launch_bounds__(256) void k_sort_keys(const double* __restrict__ ent, int64_t n, int64_t idx0,
                                                    const uint32_t* __restrict__ excl, Cand* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        uint64_t k = order_key(ent[i]);
        if (excl && excluded(excl, i)) k = 0ull;
        out[i] = Cand{k, idx0 + i};
    }
}

// Batched users: item g of user u (offsets[u] <= g < offsets[u+1]) ->
// {order key, (u << kUserShift) | (g - offsets[u])}; items outside every user
// get user U (sorted after all users).
__global__ __launch_bounds__(256) void k_sort_keys_users(const double* __restrict__ ent, int64_t n,
                                                          const int64_t* __restrict__ offsets, int U,
                                                          Cand* __restrict__ out) {
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n; g += (int64_t)gridDim.x * 256) {
        int l = 0, h = U;  // the last u with offsets[u] <= g
        while (l < h) {
            const int mid = (l + h + 1) >> 1;
            if (offsets[mid] <= g) l = mid;
            else h = mid - 1;
        }
        const int64_t u = (g < offsets[0] || g >= offsets[U]) ? U : l;
        const int64_t local = u < U ? g - offsets[u] : 0;
        out[g] = Cand{order_key(ent[g]), (int64_t)(((uint64_t)u << kUserShift) | (uint64_t)local)};
    }
}

// The first q slots of a sorted record array: (val, idx) or records; slots past
// n or holding key 0 (excluded) are padding (val NaN, idx -1 / record {0, -1}).
__global__ __launch_bounds__(256) void k_sort_out(const Cand* __restrict__ s, int64_t n, int64_t q,
                                                   double* __restrict__ oval, int64_t* __restrict__ oidx,
                                                   Cand* __restrict__ ocand) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < q; r += (int64_t)gridDim.x * 256) {
        Cand c{0ull, -1};
        if (r < n) c = s[r];
        const bool ok = r < n && c.key != 0ull;
        if (ocand) {
            ocand[r] = ok ? c : Cand{0ull, -1};
        } else {
            oval[r] = ok ? key_to_val(c.key) : __longlong_as_double(0x7ff8000000000000ll);
            oidx[r] = ok ? c.idx : -1;
        }
    }
}

// Batched users: user u's slots [u*q, (u+1)*q) from its contiguous run of the
// sorted records (it starts at offsets[u] - offsets[0]); user-local positions.
__global__ __launch_bounds__(256) void k_sort_out_users(const Cand* __restrict__ s, const int64_t* __restrict__ offsets,
                                                         int U, int64_t q, double* __restrict__ oval,
                                                         int64_t* __restrict__ oidx) {
    const int64_t total = (int64_t)U * q;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int64_t u = t / q, r = t - u * q;
        const int64_t len = offsets[u + 1] - offsets[u];
        const bool ok = r < len;
        CE_DASSERT(!ok || (offsets[u] >= offsets[0] && len >= 0));
        const Cand c = ok ? s[offsets[u] - offsets[0] + r] : Cand{0ull, -1};
        oval[t] = ok ? key_to_val(c.key) : __longlong_as_double(0x7ff8000000000000ll);
        oidx[t] = ok ? (int64_t)((uint64_t)c.idx & ((1ull << kUserShift) - 1ull)) : -1;
    }
}

// Merge of nl best-first lists of q slots (q beyond the list merges) by rank:
// a candidate's output slot is its slot in its own list plus, in every other
// list, the number of entries before it (a binary search: the entries better
// than it form a prefix of a best-first list; an identical entry counts as
// before it when its list comes first, so duplicates take distinct slots).
// Outputs must be padding-filled first (k_fill_pad): the ranks of the valid
// candidates are exactly 0 .. nvalid-1.
template <bool FROM_VALS>
__global__ __launch_bounds__(256) void k_rank_merge(ListSrc<FROM_VALS> src, int nl, int64_t q, double* __restrict__ oval,
                                                     int64_t* __restrict__ oidx, Cand* __restrict__ ocand) {
    const int64_t L = (int64_t)nl * q;
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < L; j += (int64_t)gridDim.x * 256) {
        uint64_t ck;
        int64_t ci;
        src.get(j, ck, ci);
        if (ci < 0) continue;
        const int a = (int)(j / q);
        int64_t rank = j - (int64_t)a * q;
        for (int b = 0; b < nl; ++b) {
            if (b == a) continue;
            int64_t l = 0, h = q;
            while (l < h) {
                const int64_t mid = (l + h) >> 1;
                uint64_t ek;
                int64_t ei;
                src.get((int64_t)b * q + mid, ek, ei);
                const bool before = ei >= 0 && (better(ek, ei, ck, ci) || (b < a && ek == ck && ei == ci));
                if (before) l = mid + 1;
                else h = mid;
            }
            rank += l;
        }
        if (rank < q) {
            if (ocand) {
                ocand[rank] = Cand{ck, ci};
            } else {
                oval[rank] = key_to_val(ck);
                oidx[rank] = ci;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_fill_pad(int64_t q, double* __restrict__ oval, int64_t* __restrict__ oidx,
                                                   Cand* __restrict__ ocand) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < q; r += (int64_t)gridDim.x * 256) {
        if (ocand) {
            ocand[r] = Cand{0ull, -1};
        } else {
            oval[r] = __longlong_as_double(0x7ff8000000000000ll);
            oidx[r] = -1;
        }
    }
}

}  // namespace ce

static inline size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

static SortGeom sort_geom(int64_t n) {
    SortGeom g;
    g.n = n;
    int64_t chunk = cdiv(n < 1 ? 1 : n, (int64_t)kSortMaxWaves);
    if (chunk < kSortMinChunk) chunk = kSortMinChunk;
    g.chunk = (chunk + 63) / 64 * 64;
    g.nw = (int)cdiv(n < 1 ? 1 : n, g.chunk);
    return g;
}

size_t sort_ws_bytes(int64_t n, int64_t extra_cands) {
    if (n < 0) n = 0;
    const SortGeom g = sort_geom(n);
    return kWsHeader + 256 + al256((size_t)n * 8) + 2 * al256((size_t)n * 16) + al256((size_t)256 * g.nw * 4) +
           al256(256 * 8) + al256((size_t)(extra_cands > 0 ? extra_cands : 0) * 16);
}

SortWs sort_carve(void* ws, int64_t n, int64_t extra_cands) {
    (void)extra_cands;
    SortWs s;
    s.g = sort_geom(n);
    uintptr_t p = (((uintptr_t)ws + 255) & ~(uintptr_t)255) + kWsHeader;
    s.ent = reinterpret_cast<double*>(p);
    p += al256((size_t)n * 8);
    s.a = reinterpret_cast<Cand*>(p);
    p += al256((size_t)n * 16);
    s.b = reinterpret_cast<Cand*>(p);
    p += al256((size_t)n * 16);
    s.hist = reinterpret_cast<uint32_t*>(p);
    p += al256((size_t)256 * s.g.nw * 4);
    s.dtot = reinterpret_cast<uint64_t*>(p);
    p += al256(256 * 8);
    s.extra = reinterpret_cast<Cand*>(p);
    return s;
}

static inline int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), 8192)); }

void sort_keys(const double* ent, int64_t n, int64_t idx0, const uint32_t* excl, Cand* out, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_sort_keys, dim3(grid_for(n)), dim3(256), 0, st, ent, n, idx0, excl, out);
}

void sort_keys_users(const double* ent, int64_t n, const int64_t* offsets, int U, Cand* out, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_sort_keys_users, dim3(grid_for(n)), dim3(256), 0, st, ent, n, offsets, U, out);
}

const Cand* sort_run(const SortWs& s, int user_passes, hipStream_t st) {
    const SortGeom g = s.g;
    if (g.n <= 1) return s.a;
    const Cand* in = s.a;
    Cand* out = s.b;
    const int blocks = (g.nw + 3) / 4;
    auto pass = [&](SortPass ps) {
        hipLaunchKernelGGL(k_sort_hist, dim3(blocks), dim3(256), 0, st, in, g, ps, s.hist);
        hipLaunchKernelGGL(k_sort_scan, dim3(256), dim3(256), 0, st, s.hist, g.nw, s.dtot);
        hipLaunchKernelGGL(k_sort_scatter, dim3(blocks), dim3(256), 0, st, in, out, g, ps, s.hist, s.dtot);
        Cand* t = const_cast<Cand*>(in);
        in = out;
        out = t;
    };
    for (int sh = 0; sh < 64; sh += 8) pass(SortPass{0, sh});  // key, least significant byte first
    for (int j = 0; j < user_passes; ++j) pass(SortPass{1, kUserShift + 8 * j});
    return in;
}

void sort_out(const Cand* s, int64_t n, int64_t q, double* oval, int64_t* oidx, Cand* ocand, hipStream_t st) {
    if (q > 0) hipLaunchKernelGGL(k_sort_out, dim3(grid_for(q)), dim3(256), 0, st, s, n, q, oval, oidx, ocand);
}

void sort_out_users(const Cand* s, const int64_t* offsets, int U, int64_t q, double* oval, int64_t* oidx,
                    hipStream_t st) {
    const int64_t t = (int64_t)U * q;
    if (t > 0) hipLaunchKernelGGL(k_sort_out_users, dim3(grid_for(t)), dim3(256), 0, st, s, offsets, U, q, oval, oidx);
}

void rank_merge_lists(const Cand* c, const double* vals, const int64_t* idx, int nl, int64_t q, double* oval,
                      int64_t* oidx, Cand* ocand, hipStream_t st) {
    if (q <= 0) return;
    hipLaunchKernelGGL(k_fill_pad, dim3(grid_for(q)), dim3(256), 0, st, q, oval, oidx, ocand);
    const int64_t L = (int64_t)nl * q;
    if (c)
        hipLaunchKernelGGL((k_rank_merge<false>), dim3(grid_for(L)), dim3(256), 0, st, ListSrc<false>{c, nullptr, nullptr},
                           nl, q, oval, oidx, ocand);
    else
        hipLaunchKernelGGL((k_rank_merge<true>), dim3(grid_for(L)), dim3(256), 0, st, ListSrc<true>{nullptr, vals, idx},
                           nl, q, oval, oidx, ocand);
}

int user_sort_passes(int U) {
    int p = 0;
    for (uint64_t v = (uint64_t)U; v; v >>= 8) ++p;  // user ids 0..U (U: items outside every user)
    return p;
}
