// ce_debug.hpp -- the debug build's device bounds checks (CE_DASSERT).
#pragma once
#include <hip/hip_runtime.h>

// Debug build (make -C consensus-entropy_amd debug: -DCE_DEBUG): device-side
// bounds checks on workspace / list / LDS indexing and the XGB walk, which
// print the failing condition and trap.  Compiled out otherwise.
#ifdef CE_DEBUG
#define CE_DASSERT(c)                                                                                   \
    do {                                                                                                \
        if (!(c)) {                                                                                     \
            printf("CE_DEBUG: `%s` failed at %s:%d (block %d, thread %d)\n", #c, __FILE__, __LINE__, \
                   (int)blockIdx.x, (int)threadIdx.x);                                                  \
            __builtin_trap();                                                                           \
        }                                                                                               \
    } while (0)
#else
#define CE_DASSERT(c) ((void)0)
#endif
