// hbm_probe.hip -- the practical HBM read ceiling on this MI355X for the
// stage-1 access patterns (no entropy math): (a) LDS-DMA 64 x 256-B tiles per
// wave (k_stream_nmc's pattern), (b) plain 16-B nt loads, 8 in flight per lane.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o build/hbm_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_dma(const char* base, int64_t n_tiles_per_wave, int64_t tiles, unsigned* sink) {
    __shared__ __attribute__((aligned(16))) char lds[4][16384];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + w;
    int64_t t0 = gw * n_tiles_per_wave, t1 = t0 + n_tiles_per_wave;
    if (t1 > tiles) t1 = tiles;
    unsigned acc = 0;
    for (int64_t t = t0; t < t1; ++t) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const char* src = base + t * 16384 + k * 1024 + lane * 16;
            __builtin_amdgcn_global_load_lds((const void*)src, (void __attribute__((address_space(3)))*)(lds[w] + k * 1024), 16, 0, 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= *(const unsigned*)(lds[w] + lane * 256);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_direct(const u32x4* p, int64_t n_vec, unsigned* sink) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    unsigned acc = 0;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 7 * stride < n_vec; i += 8 * stride) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].w;
    }
    for (; i < n_vec; i += stride) acc ^= __builtin_nontemporal_load(p + i).x;
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const size_t bytes = 25600000000ull;
    char* d = nullptr;
    unsigned* sink = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(d, 1, bytes);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int64_t tiles = bytes / 16384;
    for (int bpc = 1; bpc <= 2; ++bpc) {
        const int grid = cus * bpc;
        const int64_t per = (tiles + grid * 4 - 1) / (grid * 4);
        for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_dma, dim3(grid), dim3(256), 0, 0, d, per, tiles, sink);
        (void)hipEventRecord(a);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k_dma, dim3(grid), dim3(256), 0, 0, d, per, tiles, sink);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("lds-dma  %d blocks/CU: %.1f GB/s\n", bpc, bytes * 10 / (ms * 1e-3) / 1e9);
    }
    const int64_t n_vec = bytes / 16;
    for (int bpc = 2; bpc <= 8; bpc *= 2) {
        const int grid = cus * bpc;
        for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, (const u32x4*)d, n_vec, sink);
        (void)hipEventRecord(a);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, (const u32x4*)d, n_vec, sink);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("direct   %d blocks/CU: %.1f GB/s\n", bpc, bytes * 10 / (ms * 1e-3) / 1e9);
    }
    return 0;
}
