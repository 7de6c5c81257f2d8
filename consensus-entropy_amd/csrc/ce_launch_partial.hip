// ce_launch_partial.hip -- block-synchronous stage 1 (k_partial /
// k_partial_wide: any q, per-block LDS top-q) for committees, precomputed
// entropy vectors and hc tables.  The only TU that instantiates them.
#include "ce_host.hpp"

using namespace ce;

template <class Src>
static void launch_partial(const Src& src, const Seg& sg, int grid, int q, WsLists w, double* oval,
                           int64_t* oidx, bool final_out, hipStream_t st) {
    if (q <= 256) {
        if (final_out)
            hipLaunchKernelGGL((k_partial<Src, 1024, true>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
        else
            hipLaunchKernelGGL((k_partial<Src, 1024, false>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
    } else {
        if (final_out)
            hipLaunchKernelGGL((k_partial<Src, 4096, true>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
        else
            hipLaunchKernelGGL((k_partial<Src, 4096, false>), dim3(grid), dim3(kBS), 0, st, src, sg, q, w.c, oval, oidx);
    }
}

static void launch_partial_wide(const CommArgs& a, const Seg& sg, int grid, int q, WsLists w, double* oval,
                                int64_t* oidx, bool fin, hipStream_t st) {
    const WideArgs wa = wide_args(a);
    const PwPlan pl = pw_plan(a.C);
    const size_t lds = wide_lds_bytes(a.C);
    with_wide_v(a, [&](auto dt, auto npl, auto vec) {
        constexpr int DT = decltype(dt)::value, NPL = decltype(npl)::value;
        constexpr bool VEC = decltype(vec)::value;
        if (q <= 256) {
            if (fin)
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 1024, true>), dim3(grid), dim3(kBS), lds, st, wa, pl,
                                   sg, q, w.c, oval, oidx);
            else
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 1024, false>), dim3(grid), dim3(kBS), lds, st, wa,
                                   pl, sg, q, w.c, oval, oidx);
        } else {
            if (fin)
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 4096, true>), dim3(grid), dim3(kBS), lds, st, wa, pl,
                                   sg, q, w.c, oval, oidx);
            else
                hipLaunchKernelGGL((k_partial_wide<DT, NPL, VEC, 4096, false>), dim3(grid), dim3(kBS), lds, st, wa,
                                   pl, sg, q, w.c, oval, oidx);
        }
    });
}

// Committee stage 1 for any supported shape: register path or wide path.
int committee_partial(const CommArgs& a, const Seg& sg, int grid, int q, WsLists w, double* oval,
                             int64_t* oidx, bool fin, hipStream_t st) {
    int rc = with_committee(a, [&](auto src) { launch_partial(src, sg, grid, q, w, oval, oidx, fin, st); });
    if (rc != CE_EUNSUPPORTED) return rc;
    if (a.C > kWideMaxC) return CE_EUNSUPPORTED;
    launch_partial_wide(a, sg, grid, q, w, oval, oidx, fin, st);
    return CE_OK;
}

void partial_entropies(const double* ent, const Seg& sg, int grid, int q, WsLists w, double* oval, int64_t* oidx,
                       bool fin, hipStream_t st) {
    launch_partial(ArraySrc{ent}, sg, grid, q, w, oval, oidx, fin, st);
}

int partial_table(const double* hc, int64_t ld, int C, const Seg& sg, int grid, int q, WsLists w, hipStream_t st) {
    switch (C) {
#define CE_T(CC) case CC: launch_partial(TableSrc<CC>{hc, ld}, sg, grid, q, w, nullptr, nullptr, false, st); return CE_OK;
        CE_T(2) CE_T(3) CE_T(4) CE_T(8)
#undef CE_T
        default: return CE_EUNSUPPORTED;
    }
}
