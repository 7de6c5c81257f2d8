// random_row_probe.hip -- the random-row ceiling of this MI355X for SURVEY.md
// §8(f)1's shuffled frames (frame rows gathered through a permutation): how
// many rows per second can ANY kernel read when each row of S bytes sits at a
// random position of a buffer far larger than the 256 MiB Infinity Cache?
// S/8 lanes read one row (8 B per lane, as k_frames_lanes' shuffled path
// does), 8 rows in flight per lane; row index = an odd-multiplier hash of the
// ordinal mod 2^k (a bijection: every row read once per sweep).
// Build: make -C consensus-entropy_amd probes   (-> tools/_diag/random_row_probe, untracked)
// Run:   tools/_diag/random_row_probe [S]   (one line per row size: rows/s, useful GB/s)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

template <int S, bool NT>
__global__ __launch_bounds__(256) void k_rows(const double* __restrict__ buf, int64_t log2_rows, int64_t n_reads,
                                              double* __restrict__ sink) {
    constexpr int L = S / 8;  // lanes per row
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t grp = tid / L, sub = tid % L;
    const int64_t groups = (int64_t)gridDim.x * 256 / L;
    const uint64_t mask = (1ull << log2_rows) - 1;
    double acc = 0.0;
    for (int64_t i = grp; i < n_reads; i += 8 * groups) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t r = ((uint64_t)(i + u * groups) * 0x9E3779B97F4A7C15ull) & mask;  // odd multiplier: bijective mod 2^k
            v[u] = NT ? __builtin_nontemporal_load(buf + r * L + sub) : buf[r * L + sub];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    if (acc == 1.2345) sink[0] = acc;
}

template <int S, bool NT = false>
static void run(const double* buf, int64_t bytes, double* sink) {
    int64_t log2_rows = 0;
    while (((int64_t)S << (log2_rows + 1)) <= bytes) ++log2_rows;
    const int64_t n_reads = 1ll << 28 < (1ll << log2_rows) ? 1ll << 28 : (1ll << log2_rows);  // 268M rows (or all)
    const int grid = 256 * 8;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_rows<S, NT>), dim3(grid), dim3(256), 0, 0, buf, log2_rows, n_reads, sink);  // warm-up
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL((k_rows<S, NT>), dim3(grid), dim3(256), 0, 0, buf, log2_rows, n_reads, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    printf("{\"row_bytes\": %d, \"nontemporal\": %s, \"rows\": %lld, \"ms\": %.3f, \"G_rows_per_s\": %.2f, \"useful_GB_per_s\": %.1f}\n", S,
           NT ? "true" : "false", (long long)n_reads, best, n_reads / (best * 1e-3) / 1e9, n_reads * (double)S / (best * 1e-3) / 1e9);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main(int argc, char** argv) {
    const int only = argc > 1 ? atoi(argv[1]) : 0;  // one row size (e.g. for a --pmc pass), 0: all
    const int64_t bytes = 16ll << 30;  // 16 GiB: 64x the Infinity Cache
    double* buf = nullptr;
    double* sink = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    hipMemset(buf, 0, bytes);
    hipDeviceSynchronize();
    if (!only || only == 8) run<8>(buf, bytes, sink);
    if (!only || only == 16) run<16>(buf, bytes, sink);
    if (!only || only == 32) run<32>(buf, bytes, sink);
    if (!only || only == 64) run<64>(buf, bytes, sink);
    if (!only || only == 128) run<128>(buf, bytes, sink);
    if (!only || only == 256) run<256>(buf, bytes, sink);
    // non-temporal loads (each random row is read once)
    if (!only || only == 8) run<8, true>(buf, bytes, sink);
    if (!only || only == 32) run<32, true>(buf, bytes, sink);
    if (!only || only == 128) run<128, true>(buf, bytes, sink);
    hipFree(buf);
    hipFree(sink);
    return 0;
}
