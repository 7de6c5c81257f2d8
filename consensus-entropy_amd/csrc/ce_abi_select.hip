// ce_abi_select.hip -- C-ABI (include/ce.h): the fused mc selection (streaming
// stage 1 + merge, single-block small pools), exclusion-bitmap selection, the
// multi-GPU exchange records and chunked pools larger than HBM.
//
// q (any q >= 0, as the reference's -q, amg_test.py:547-553): q <= 64 runs on
// the streaming / single-block kernels (one launch), 64 < q <= CE_MAX_Q on the
// block-synchronous lists (k_partial) + a list merge, q > CE_MAX_Q on the sort
// path (ce_sort.hpp); q = 0 selects nothing.
#include "ce_host.hpp"

using namespace ce;

// ---- fused mc ----------------------------------------------------------------
extern "C" size_t ce_select_mc_workspace_bytes(int64_t N, int32_t q) { return ce_topq_workspace_bytes(N, q); }

// stage 1 into the workspace lists (q <= CE_MAX_Q): the streaming kernels for
// q <= 64, else k_partial (writing the final outputs itself when allow_final
// and the pool is one block)
static int mc_partial(const CommArgs& a, int q, int64_t base_idx, const uint32_t* excl, void* ws, size_t ws_bytes,
                      double* val_out, int64_t* idx_out, bool allow_final, int* G_out, bool* final_out,
                      hipStream_t st) {
    int rc = check_comm(a);
    if (rc) return rc;
    rc = check_q(q);
    if (rc) return rc;
    const int G = pool_blocks(a.N);
    if (!ws || ws_bytes < lists_bytes(G, q)) return fail(CE_EWORKSPACE, "workspace too small");
    WsLists w = carve(ws, G, q);
    *G_out = G;
    *final_out = false;
    if (launch_stream(a, G, q, base_idx, w, st, excl)) return CE_OK;
    Seg sg{nullptr, a.N, G, base_idx, excl};
    const bool fin = allow_final && G == 1;
    rc = committee_partial(a, sg, G, q, w, val_out, idx_out, fin, st);
    if (rc) return dispatch_err(rc, a);
    *final_out = fin;
    return CE_OK;
}

// q > CE_MAX_Q: entropies into the workspace, then the sort path
static int mc_sort(const CommArgs& a, const uint32_t* excl, int64_t q, int64_t base_idx, void* ws, double* oval,
                   int64_t* oidx, Cand* ocand, hipStream_t st) {
    int rc = check_sort_n(a.N);
    if (rc) return rc;
    const SortWs s = sort_carve(ws, a.N);
    rc = launch_entropy(a, nullptr, s.ent, st);
    if (rc) return rc;
    sort_select(s, s.ent, a.N, base_idx, excl, q, oval, oidx, ocand, st);
    return CE_OK;
}

static int select_mc_impl(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                          int64_t sC, const uint32_t* excl, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes,
                          double* val_out, int64_t* idx_out, ce_stream_t stream);

extern "C" int ce_select_mc(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                            int64_t sC, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes, double* val_out,
                            int64_t* idx_out, ce_stream_t stream) {
    return select_mc_impl(p, dt, N, M, C, sN, sM, sC, nullptr, q, base_idx, ws, ws_bytes, val_out, idx_out, stream);
}

extern "C" size_t ce_excl_words(int64_t N) { return N > 0 ? (size_t)((N + 31) / 32) : 0; }

extern "C" int ce_select_mc_excl(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                 int64_t sM, int64_t sC, const uint32_t* excl, int32_t q, int64_t base_idx, void* ws,
                                 size_t ws_bytes, double* val_out, int64_t* idx_out, ce_stream_t stream) {
    if (!excl && N > 0) return fail(CE_EINVAL, "null exclusion bitmap");
    return select_mc_impl(p, dt, N, M, C, sN, sM, sC, excl, q, base_idx, ws, ws_bytes, val_out, idx_out, stream);
}

static int select_mc_impl(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                          int64_t sC, const uint32_t* excl, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes,
                          double* val_out, int64_t* idx_out, ce_stream_t stream) {
    hipStream_t st = (hipStream_t)stream;
    note_kernel("%s", "");
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int rc0 = check_comm(a);
    if (rc0) return rc0;
    rc0 = check_q(q);
    if (rc0) return rc0;
    if (q > 0 && (!val_out || !idx_out)) return fail(CE_EINVAL, "null output");
    // the workspace contract holds on every path, even the one that does not touch it
    if (!ws || ws_bytes < ce_select_mc_workspace_bytes(N, q)) return fail(CE_EWORKSPACE, "workspace too small");
    if (q == 0) return CE_OK;
    if (q > CE_MAX_Q) {
        const int rc = mc_sort(a, excl, q, base_idx, ws, val_out, idx_out, nullptr, st);
        return rc ? rc : check_launch("ce_select_mc");
    }
    if (q <= kStreamMaxQ && N > 0) {
        // the pool in one block (k_select_tiles)
        if (launch_small_pool(a, base_idx, q, val_out, idx_out, excl, carve(ws, 0, q), st))
            return check_launch("ce_select_mc");
        if (N * (int64_t)M * C * elem_bytes((int)dt) <= kSmallPoolBytes) {
            // small pool: ~512 items per 4-wave block on a few CUs (one block: it
            // is the final answer), then one wave merges the blocks' lists
            const int nb = (int)std::min<int64_t>(std::min<int64_t>(cdiv(N, 512), 32), pool_blocks(N));
            WsLists w = carve(ws, nb, q);
            if (launch_seg(a, nullptr, N, base_idx, q, nb, nb, 256, val_out, idx_out, w.c, excl, st)) {
                if (nb > 1) launch_merge_wave(w.c, 1, nb, q, val_out, idx_out, st);
                return check_launch("ce_select_mc");
            }
        }
        // large pools: the streaming stage 1 with stage 2 folded into its last block
        const int G = pool_blocks(N);
        const WsLists w = carve(ws, G, q);
        const int sr = launch_stream_fold(a, G, q, base_idx, w, st, excl,
                                          FoldOut{val_out, idx_out, nullptr, nullptr, w.c + (int64_t)G * q});
        if (sr == 2) return check_launch("ce_select_mc");
        if (sr == 1) {
            finish_lists(carve(ws, G, q), 1, G, q, val_out, idx_out, st);
            return check_launch("ce_select_mc");
        }
    }
    int Gp = 0;
    bool fin = false;
    const int rc = mc_partial(a, q, base_idx, excl, ws, ws_bytes, val_out, idx_out, true, &Gp, &fin, st);
    if (rc) return rc;
    if (!fin) finish_lists(carve(ws, Gp, q), 1, Gp, q, val_out, idx_out, st);
    return check_launch("ce_select_mc");
}

// ce_select_mc writing the pool's q candidate records (the multi-GPU send
// buffer): for q <= 64 in ONE launch (stage 2 folded into stage 1's last block).
extern "C" int ce_select_mc_cands(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                                  int64_t sC, int32_t q, int64_t base_idx, void* ws, size_t ws_bytes, ce_cand* out,
                                  ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int rc = check_comm(a);
    if (rc) return rc;
    rc = check_q(q);
    if (rc) return rc;
    if (q > 0 && (!out || (uintptr_t)out % 16))
        return fail(CE_EINVAL, "ce_cand output must be 16-byte aligned device memory");
    if (!ws || ws_bytes < ce_select_mc_workspace_bytes(N, q)) return fail(CE_EWORKSPACE, "workspace too small");
    if (q == 0) return CE_OK;
    hipStream_t st = (hipStream_t)stream;
    Cand* oc = reinterpret_cast<Cand*>(out);
    if (q > CE_MAX_Q) {
        rc = mc_sort(a, nullptr, q, base_idx, ws, nullptr, nullptr, oc, st);
        return rc ? rc : check_launch("ce_select_mc_cands");
    }
    const int G = pool_blocks(N);
    WsLists w = carve(ws, G, q);
    const int sr =
        N > 0 ? launch_stream_fold(a, G, q, base_idx, w, st, nullptr, FoldOut{nullptr, nullptr, oc, nullptr, w.c + (int64_t)G * q})
              : 0;
    if (sr == 2) return check_launch("ce_select_mc_cands");
    if (sr == 0) {  // no streaming kernel (q > 64, or an empty pool): the block-synchronous stage 1
        Seg sg{nullptr, N, G, base_idx};
        rc = committee_partial(a, sg, G, q, w, nullptr, nullptr, false, st);
        if (rc) return dispatch_err(rc, a);
    }
    launch_finish_lists(w.c, 1, G, q, nullptr, nullptr, st, oc);
    return check_launch("ce_select_mc_cands");
}

// The two stages as separate launches (q <= CE_MAX_Q).
extern "C" int ce_select_mc_partial(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                    int64_t sM, int64_t sC, int32_t q, int64_t base_idx, void* ws,
                                    size_t ws_bytes, ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    if (q > CE_MAX_Q)
        return fail(CE_EUNSUPPORTED, "two-stage selection needs q <= %d (ce_select_mc takes any q)", CE_MAX_Q);
    if (q <= 0) return check_q(q);
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int G = 0;
    bool fin = false;
    int rc = mc_partial(a, q, base_idx, nullptr, ws, ws_bytes, nullptr, nullptr, false, &G, &fin, (hipStream_t)stream);
    if (rc) return rc;
    return check_launch("ce_select_mc_partial");
}

extern "C" int ce_select_finish(int64_t N, int32_t q, void* ws, size_t ws_bytes, double* val_out, int64_t* idx_out,
                                ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    int rc = check_q(q);
    if (rc) return rc;
    if (q > CE_MAX_Q)
        return fail(CE_EUNSUPPORTED, "two-stage selection needs q <= %d (ce_select_mc takes any q)", CE_MAX_Q);
    if (q == 0) return CE_OK;
    if (N < 0 || !val_out || !idx_out) return fail(CE_EINVAL, "bad finish arguments");
    const int G = pool_blocks(N);
    if (!ws || ws_bytes < lists_bytes(G, q)) return fail(CE_EWORKSPACE, "workspace too small");
    finish_lists(carve(ws, G, q), 1, G, q, val_out, idx_out, (hipStream_t)stream);
    return check_launch("ce_select_finish");
}

// ---- exchange records (multi-GPU) -------------------------------------------
static_assert(sizeof(ce_cand) == sizeof(Cand) && alignof(ce_cand) <= alignof(Cand), "ce_cand must mirror Cand");

extern "C" int ce_select_finish_cands(int64_t N, int32_t q, void* ws, size_t ws_bytes, ce_cand* out,
                                      ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    int rc = check_q(q);
    if (rc) return rc;
    if (q > CE_MAX_Q)
        return fail(CE_EUNSUPPORTED, "two-stage selection needs q <= %d (ce_select_mc_cands takes any q)", CE_MAX_Q);
    if (q == 0) return CE_OK;
    if (N < 0 || !out) return fail(CE_EINVAL, "bad finish arguments");
    if ((uintptr_t)out % 16) return fail(CE_EINVAL, "ce_cand output must be 16-byte aligned");
    const int G = pool_blocks(N);
    if (!ws || ws_bytes < lists_bytes(G, q)) return fail(CE_EWORKSPACE, "workspace too small");
    launch_finish_lists(carve(ws, G, q).c, 1, G, q, nullptr, nullptr, (hipStream_t)stream,
                        reinterpret_cast<Cand*>(out));
    return check_launch("ce_select_finish_cands");
}

extern "C" int ce_merge_cands(const ce_cand* c, int32_t nlists, int32_t q, double* val_out, int64_t* idx_out,
                              ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    int rc = check_q(q);
    if (rc) return rc;
    if (q == 0) return CE_OK;
    if (nlists < 1 || !c || !val_out || !idx_out) return fail(CE_EINVAL, "bad merge arguments");
    if ((uintptr_t)c % 16) return fail(CE_EINVAL, "ce_cand input must be 16-byte aligned");
    const Cand* cc = reinterpret_cast<const Cand*>(c);
    if (q > CE_MAX_Q)  // no workspace here: the lists merge by rank (binary searches)
        rank_merge_lists(cc, nullptr, nullptr, nlists, q, val_out, idx_out, nullptr, (hipStream_t)stream);
    else
        launch_finish_lists(cc, 1, nlists, q, val_out, idx_out, (hipStream_t)stream);
    return check_launch("ce_merge_cands");
}

// ---- chunked pools (larger than HBM) ----------------------------------------
__global__ void k_cand_empty(Cand* __restrict__ c, int q) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < q; r += gridDim.x * blockDim.x) c[r] = Cand{0ull, -1};
}

extern "C" size_t ce_select_mc_chunk_workspace_bytes(int64_t N, int32_t q) {
    if (q > CE_MAX_Q) return sort_ws_bytes(N, 2 * (int64_t)q);
    return lists_bytes((int64_t)pool_blocks(N) + 1, q < 1 ? 1 : q) + kWideSeedBytes;
}

// Stage 1 on the chunk (its G block lists), then ONE merge of those G lists
// plus the running list (copied to list slot G of the workspace) back into
// `running`: the running list always holds the top-q of every chunk so far
// (the top-q of a union is within the union of the parts' top-qs).  q > CE_MAX_Q:
// the chunk's top-q by the sort path, merged with the running list by rank.
extern "C" int ce_select_mc_chunk(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                                  int64_t sM, int64_t sC, int32_t q, int64_t base_idx, ce_cand* running,
                                  int32_t first, void* ws, size_t ws_bytes, ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    int rc = check_q(q);
    if (rc) return rc;
    if (q == 0) return CE_OK;
    if (!running || (uintptr_t)running % 16)
        return fail(CE_EINVAL, "running list must be 16-byte aligned device memory");
    if (N < 0 || base_idx < 0)
        return fail(CE_EINVAL, "bad chunk N=%lld base_idx=%lld", (long long)N, (long long)base_idx);
    hipStream_t st = (hipStream_t)stream;
    Cand* run = reinterpret_cast<Cand*>(running);
    if (N == 0) {
        if (first)
            hipLaunchKernelGGL(k_cand_empty, dim3((unsigned)std::min<int64_t>(cdiv(q, 256), 4096)), dim3(256), 0, st,
                               run, q);
        return check_launch("ce_select_mc_chunk");
    }
    if (!ws || ws_bytes < ce_select_mc_chunk_workspace_bytes(N, q)) return fail(CE_EWORKSPACE, "workspace too small");
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    {
        const int rc0 = check_comm(a);
        if (rc0) return rc0;
    }
    if (q > CE_MAX_Q) {
        const SortWs s = sort_carve(ws, N, 2 * (int64_t)q);
        Cand* mine = s.extra;  // the chunk's top-q, then (unless first) a copy of the running list
        rc = mc_sort(a, nullptr, q, base_idx, ws, nullptr, nullptr, first ? run : mine, st);
        if (rc) return rc;
        if (!first) {
            if (hipMemcpyAsync(mine + q, run, (size_t)q * sizeof(Cand), hipMemcpyDeviceToDevice, st) != hipSuccess)
                return fail(CE_ELAUNCH, "running-list copy failed");
            rank_merge_lists(mine, nullptr, nullptr, 2, q, nullptr, nullptr, run, st);
        }
        return check_launch("ce_select_mc_chunk");
    }
    const int G = pool_blocks(N);
    WsLists w = carve(ws, (int64_t)G + 1, q);
    // q <= 64, one launch per chunk: the streaming stage 1 whose last block merges
    // the grid's lists AND the running list back into `running`
    // the wide stream's floor + grid vote scratch: right after the G + 1 lists
    const int sr = launch_stream_fold(a, G, q, base_idx, w, st, nullptr,
                                      FoldOut{nullptr, nullptr, run, first ? nullptr : run, w.c + ((int64_t)G + 1) * q});
    if (sr == 2) return check_launch("ce_select_mc_chunk");
    if (!first && hipMemcpyAsync(w.c + (int64_t)G * q, run, (size_t)q * sizeof(Cand), hipMemcpyDeviceToDevice, st) !=
                      hipSuccess)
        return fail(CE_ELAUNCH, "running-list copy failed");
    if (sr == 0) {  // no streaming kernel (q > 64, or no shape match): the block-synchronous stage 1
        int Gs = 0;
        bool fin = false;
        rc = mc_partial(a, q, base_idx, nullptr, ws, ws_bytes, nullptr, nullptr, false, &Gs, &fin, st);
        if (rc) return rc;
    }
    launch_finish_lists(w.c, 1, G + (first ? 0 : 1), q, nullptr, nullptr, st, run);
    return check_launch("ce_select_mc_chunk");
}
