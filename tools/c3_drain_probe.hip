// c3_drain_probe.hip -- the load floor of BASELINE configs[2] (500 users x 4
// members x 1608 items x 4 classes f32, [M, N, C] member-major = 51.46 MB per
// launch): kernels that only READ a user's items the way k_select_tiles does
// (thread = item slot, 16-B member rows, items tid + BS*v) and reduce them to
// one value per block -- no entropy, no selection -- so their duration is the
// dispatch + HBM drain the selection kernel cannot go below.  Launch shapes:
//   <BS=512, UPB=1>   one 512-thread block per user (k_select_tiles today)
//   <BS=512, UPB=2>   two users per 1024-thread block (half the workgroups)
//   THR               item slots in flight per lane (1: slot v+1 issued after
//                     slot v landed, as rows_small; 4: all at once)
// Cold: 8 distinct pools rotated between launches (412 MB > the 256 MiB
// Infinity Cache).  Run under rocprofv3 --kernel-trace --stats:
//   tools/_diag/c3_drain_probe [reps]     (make -C consensus-entropy_amd probes)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int BS, int UPB, int THR>
__global__ __launch_bounds__(BS* UPB) void k_drain(const f32x4* __restrict__ P, int64_t N, int nu, int users,
                                                   float* __restrict__ out) {
    const int half = threadIdx.x / BS, tid = threadIdx.x % BS;
    const int u = blockIdx.x * UPB + half;
    const int64_t lo = (int64_t)(u < users ? u : users - 1) * nu;
    constexpr int IPT = 4, M = 4;
    float acc = 0.0f;
    f32x4 x[IPT][M];
    auto issue = [&](int v) {
        const int j = tid + BS * v;
        const int64_t i = lo + (j < nu ? j : nu - 1);
#pragma unroll
        for (int m = 0; m < M; ++m) x[v][m] = __builtin_nontemporal_load(P + (int64_t)m * N + i);
    };
#pragma unroll
    for (int v = 0; v < THR; ++v) issue(v);
#pragma unroll
    for (int v = 0; v < IPT; ++v) {
        if (THR < IPT && v + THR < IPT) {
#pragma unroll
            for (int m = 0; m < M; ++m) asm volatile("" ::"v"(x[v][m].x), "v"(x[v][m].y), "v"(x[v][m].z), "v"(x[v][m].w));
            asm volatile("" ::: "memory");
            issue(v + THR);
        }
#pragma unroll
        for (int m = 0; m < M; ++m) acc += x[v][m].x + x[v][m].y + x[v][m].z + x[v][m].w;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    __shared__ float s[16];
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.0f;
        for (int w = 0; w < BS * UPB / 64; ++w) t += s[w];
        out[blockIdx.x] = t;
    }
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int users = 500, nu = 1608, M = 4, POOLS = 8;
    const int64_t N = (int64_t)users * nu;
    const size_t bytes = (size_t)M * N * 16;
    f32x4* pools[POOLS];
    for (int k = 0; k < POOLS; ++k) {
        CK(hipMalloc(&pools[k], bytes));
        CK(hipMemset(pools[k], 0x3c + k, bytes));
    }
    float* out;
    CK(hipMalloc(&out, 1024 * sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int r = 0; r < 20; ++r) launch(pools[r % POOLS]);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch(pools[r % POOLS]);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\": \"%s\", \"reps\": %d, \"us_per_launch_incl_gaps\": %.3f, \"bytes\": %zu}\n", name, reps,
               ms * 1e3 / reps, bytes);
    };
    run("k_drain<512,1,1>", [&](f32x4* p) { hipLaunchKernelGGL((k_drain<512, 1, 1>), dim3(users), dim3(512), 0, 0, p, N, nu, users, out); });
    run("k_drain<512,2,1>", [&](f32x4* p) { hipLaunchKernelGGL((k_drain<512, 2, 1>), dim3(users / 2), dim3(1024), 0, 0, p, N, nu, users, out); });
    run("k_drain<512,1,4>", [&](f32x4* p) { hipLaunchKernelGGL((k_drain<512, 1, 4>), dim3(users), dim3(512), 0, 0, p, N, nu, users, out); });
    run("k_drain<512,2,4>", [&](f32x4* p) { hipLaunchKernelGGL((k_drain<512, 2, 4>), dim3(users / 2), dim3(1024), 0, 0, p, N, nu, users, out); });
    run("k_drain<512,1,2>", [&](f32x4* p) { hipLaunchKernelGGL((k_drain<512, 1, 2>), dim3(users), dim3(512), 0, 0, p, N, nu, users, out); });
    CK(hipDeviceSynchronize());
    for (int k = 0; k < POOLS; ++k) CK(hipFree(pools[k]));
    CK(hipFree(out));
    return 0;
}
