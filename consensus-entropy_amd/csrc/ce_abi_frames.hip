// ce_abi_frames.hip -- C-ABI (include/ce.h): frames -> committee entropy ->
// top-q in one pass (k_frames_select, ce_frames.hpp).
#include "ce_frames.hpp"
#include "ce_abi.hpp"
#include "ce_host.hpp"

using namespace ce;

// q <= 64: the streaming kernels' lists; 64 < q <= CE_MAX_Q: the lists of the
// entropy vector's selection + the N entropies behind them; q > CE_MAX_Q: the sort path.
extern "C" size_t ce_select_frames_workspace_bytes(int64_t N, int32_t q) {
    if (q > CE_MAX_Q) return sort_ws_bytes(N);
    const size_t lists = lists_bytes(pool_blocks(N), q < 1 ? 1 : q);
    return q > kStreamMaxQ ? lists + 256 + (size_t)(N > 0 ? N : 0) * 8 : lists;
}

extern "C" int ce_select_frames(const ce_member* members, int32_t M, int32_t C, const int64_t* offsets,
                                const int64_t* perm_or_null, int64_t N, int32_t q, int64_t base_idx, void* ws,
                                size_t ws_bytes, double* val_out, int64_t* idx_out, ce_stream_t stream) {
    int rc = check_q(q);
    if (rc) return rc;
    if (!members || M < 1 || M > kMaxFrameMembers) return fail(CE_EINVAL, "need 1..%d members (got %d)", kMaxFrameMembers, M);
    if (N < 0 || (N > 0 && !offsets) || (q > 0 && (!val_out || !idx_out)))
        return fail(CE_EINVAL, "bad frame selection arguments");
    if (C != 2 && C != 3 && C != 4 && C != 8) return fail(CE_EUNSUPPORTED, "frame selection: C=%d not in {2, 3, 4, 8}", C);
    const int G = pool_blocks(N);
    if (!ws || ws_bytes < ce_select_frames_workspace_bytes(N, q)) return fail(CE_EWORKSPACE, "workspace too small");
    FrameArgs fa{};
    for (int m = 0; m < M; ++m) {
        const ce_member& x = members[m];
        if (x.dtype != CE_F32 && x.dtype != CE_F64) return fail(CE_EUNSUPPORTED, "member %d: float32/float64 only", m);
        if (!x.p && N > 0) return fail(CE_EINVAL, "member %d: null pointer", m);
        if (x.ld < C) return fail(CE_EINVAL, "member %d: row stride %lld < C", m, (long long)x.ld);
        const int eb = x.dtype == CE_F64 ? 8 : 4;
        fa.mem[m] = FrameMember{x.p, x.ld, x.dtype == CE_F64 ? kF64 : kF32, x.song_level ? 1 : 0,
                                ((uintptr_t)x.p % 16 == 0 && (x.ld * eb) % 16 == 0) ? 1 : 0, 0};
    }
    fa.M = M;
    fa.off = offsets;
    fa.perm = perm_or_null;
    fa.N = N;
    fa.dM = (double)M;
    fa.invM = 1.0 / (double)M;
    fa.pow2 = (M & (M - 1)) == 0;
    fa.base_idx = base_idx;
    fa.nlists = G;
    hipStream_t st = (hipStream_t)stream;
    note_kernel("%s", "");
    if (q == 0) return CE_OK;
    if (q > kStreamMaxQ) {  // per-song entropies to HBM, then the lists (q <= CE_MAX_Q) or the sort path
        double* ent;
        SortWs s{};
        if (q > CE_MAX_Q) {
            const int rc = check_sort_n(N);
            if (rc) return rc;
            s = sort_carve(ws, N);
            ent = s.ent;
        } else {
            const WsLists wl = carve(ws, G, q);
            ent = reinterpret_cast<double*>(((uintptr_t)(wl.c + (int64_t)G * q) + 255) & ~(uintptr_t)255);
        }
        if (N > 0) {
            const int eg = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(N, 256), 8192));
            switch (C) {
#define CE_FE(CC) case CC: hipLaunchKernelGGL((k_frames_entropy<CC>), dim3(eg), dim3(256), 0, st, fa, ent); break;
                CE_FE(2) CE_FE(3) CE_FE(4) CE_FE(8)
#undef CE_FE
            }
        }
        if (q > CE_MAX_Q) {
            sort_select(s, ent, N, base_idx, nullptr, q, val_out, idx_out, nullptr, st);
        } else {
            WsLists w = carve(ws, G, q);
            Seg sg{nullptr, N, G, base_idx};
            partial_entropies(ent, sg, G, q, w, val_out, idx_out, G == 1, st);
            if (G > 1) finish_lists(w, 1, G, q, val_out, idx_out, st);
        }
        return check_launch("ce_select_frames");
    }
    WsLists w = carve(ws, G, q);
    fa.ctr = w.ctr;
    fa.oval = val_out;
    fa.oidx = idx_out;
    fa.ocand = nullptr;
    auto go = [&](auto kern, int step) {  // step: songs per wave step (64 / lanes per song)
        // no more blocks than waves with a step of songs: an idle block still
        // writes an empty list that the grid's last block merges
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(resident_grid(kern, 0, G), cdiv(N, (int64_t)4 * step)));
        fa.per_wave = (cdiv(N, (int64_t)grid * 4) + step - 1) / step * step;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, fa, q, w.c);
    };
    // C lanes per song (k_frames_lanes: whole-row reads, LDS-DMA tiles for
    // grouped dense members) where C divides the wave; lane per song otherwise
    // (k_frames_select, measured 2.7x slower at 1M songs x 40 frames)
    static const int dma_env = [] {  // test knob: CE_AMD_FRAMES_DMA=0 / 1 forces direct loads / LDS-DMA tiles
        // (test_frames_dma_tiles_vs_oracle runs the tiles at the oracle's sizes with it)
        const char* e = getenv("CE_AMD_FRAMES_DMA");
        return e ? (e[0] == '0' ? 0 : 1) : -1;
    }();
    // LDS-DMA tiles for grouped frames once every wave runs >= 4 steps: at the
    // reference's 1608 songs x 40 frames the tile round trips are exposed
    // (DMA 44.6 us, direct 31.7 us); at 1M songs the tiles win (0.92 vs 1.49 ms)
    // (large shuffled pools: the gather's row loads non-temporal, k_frames_lanes GNT)
    auto lanes_go = [&](auto dma_kern, auto direct_kern, auto gather_kern, int step) {
        const int grid = resident_grid(dma_kern, 0, G);
        const int64_t steps_per_wave = cdiv(cdiv(N, (int64_t)grid * 4), (int64_t)step);
        const bool dma = !perm_or_null && (dma_env >= 0 ? dma_env == 1 : steps_per_wave >= 4);
        const bool gnt = !dma && perm_or_null && steps_per_wave >= 4;
        note_kernel("ce::k_frames_lanes<%d, %s, %s>", 64 / step, dma ? "true" : "false", gnt ? "true" : "false");
        if (dma) go(dma_kern, step);
        else if (gnt) go(gather_kern, step);
        else go(direct_kern, step);
    };
    switch (C) {
        case 2: lanes_go(k_frames_lanes<2, true>, k_frames_lanes<2, false>, k_frames_lanes<2, false, true>, 32); break;
        case 3: note_kernel("%s", "ce::k_frames_select<3>"); go(k_frames_select<3>, 64); break;
        case 4: lanes_go(k_frames_lanes<4, true>, k_frames_lanes<4, false>, k_frames_lanes<4, false, true>, 16); break;
        default: lanes_go(k_frames_lanes<8, true>, k_frames_lanes<8, false>, k_frames_lanes<8, false, true>, 8); break;
    }
    return check_launch("ce_select_frames");
}
