// ce_abi_batch.hip -- C-ABI (include/ce.h): the mix ([mc; hc] row stack) and
// batched users in one launch.
#include "ce_host.hpp"

using namespace ce;


// ---- fused mix ---------------------------------------------------------------
extern "C" size_t ce_select_mix_workspace_bytes(int64_t N, int64_t N_h, int32_t q) {
    if (q > CE_MAX_Q) return sort_ws_bytes((N > 0 ? N : 0) + (N_h > 0 ? N_h : 0));
    // (+ kWideSeedBytes: the mix's workspace covers ce_topq_workspace_bytes of its committee part)
    return lists_bytes((int64_t)pool_blocks(N) + pool_blocks(N_h), q < 1 ? 1 : q) + kWideSeedBytes;
}

extern "C" int ce_select_mix(const void* p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                             int64_t sC, const double* hc, int64_t N_h, int64_t ld_hc, int32_t q, void* ws,
                             size_t ws_bytes, double* val_out, int64_t* idx_out, ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    CommArgs a{p, (int)dt, N, M, C, sN, sM, sC};
    int rc = check_comm(a);
    if (rc) return rc;
    rc = check_q(q);
    if (rc) return rc;
    if (N_h < 0 || (N_h > 0 && (!hc || ld_hc < C)) || (q > 0 && (!val_out || !idx_out)))
        return fail(CE_EINVAL, "bad hc table / outputs");
    if (!ws || ws_bytes < ce_select_mix_workspace_bytes(N, N_h, q)) return fail(CE_EWORKSPACE, "workspace too small");
    if (q == 0) return CE_OK;
    hipStream_t st = (hipStream_t)stream;
    const CommArgs t{hc, kF64, N_h, 1, C, ld_hc, C, 1};  // the hc table: a one-member f64 committee [N_h, 1, C]
    if (q > CE_MAX_Q) {  // entropies of [mc; hc] (positions 0..N-1, N..N+N_h-1), then the sort path
        rc = check_sort_n(N + N_h);
        if (rc) return rc;
        const SortWs s = sort_carve(ws, N + N_h);
        rc = launch_entropy(a, nullptr, s.ent, st);
        if (!rc) rc = launch_entropy(t, nullptr, s.ent + N, st);
        if (rc) return rc;
        sort_select(s, s.ent, N + N_h, 0, nullptr, q, val_out, idx_out, nullptr, st);
        return check_launch("ce_select_mix");
    }
    const int G1 = pool_blocks(N), G2 = pool_blocks(N_h);
    WsLists w = carve(ws, (int64_t)G1 + G2, q);
    if (q <= kStreamMaxQ && N > 0 && N_h > 0 && N <= kSmallPoolItems && N_h <= kSmallPoolItems &&
        C == 4) {
        // both segments in ONE block (k_select_tiles)
        if (launch_small_mix(a, t, q, val_out, idx_out, st)) return check_launch("ce_select_mix");
    }
    // both segments on the streaming engine when it applies (q <= 64): the hc
    // table is a committee of M = 1 member ([N_h, 1, C] f64, row stride ld_hc)
    if (!launch_stream(a, G1, q, 0, w, st)) {
        Seg s1{nullptr, N, G1, 0};
        rc = committee_partial(a, s1, G1, q, w, nullptr, nullptr, false, st);
        if (rc) return dispatch_err(rc, a);
    }
    WsLists w2{w.c + (size_t)G1 * q, w.ctr};
    if (launch_stream(t, G2, q, N, w2, st)) {
        finish_lists(w, 1, G1 + G2, q, val_out, idx_out, st);
        return check_launch("ce_select_mix");
    }
    Seg s2{nullptr, N_h, G2, N};
    if (partial_table(hc, ld_hc, C, s2, G2, q, w2, st) != CE_OK)
        return fail(CE_EUNSUPPORTED, "mix with C=%d has no kernel in this build", C);
    finish_lists(w, 1, G1 + G2, q, val_out, idx_out, st);
    return check_launch("ce_select_mix");
}

// ---- batched users -------------------------------------------------------------
// blocks per user: ~1024 items per block (two iterations per wave of a
// 4-wave block), at most ~4096 blocks in all.  Measured at 500 x 1608 items:
// 512 items/block 33.2 us, 1024 31.4 us, 2048 (one block per user, no merge
// launch) 31.0 us; 256 45 us.
static int batched_bpu(int64_t total, int U) {
    if (U < 1) return 1;
    const int64_t avg = cdiv(total, U);
    int64_t bpu = cdiv(avg, (int64_t)1024);
    const int64_t cap = std::max<int64_t>(1, 4096 / U);
    bpu = std::max<int64_t>(1, std::min(bpu, cap));
    return (int)bpu;
}

// lists of the k_stream_seg path: bpu per user (k_select_tiles writes none)
static int64_t batched_lists(int64_t total_items, int U, int q) {
    (void)q;
    return (int64_t)batched_bpu(total_items, U) * U;
}

extern "C" size_t ce_select_batched_workspace_bytes(int64_t total_items, int32_t U, int32_t q) {
    if (U < 1) U = 1;
    if (q > CE_MAX_Q) return sort_ws_bytes(total_items);
    if (q < 1) q = 1;
    return lists_bytes(batched_lists(total_items, U, q), q);
}

extern "C" int ce_select_batched(const void* p, ce_dtype dt, int64_t total_items, int32_t M, int32_t C, int64_t sN,
                                 int64_t sM, int64_t sC, const int64_t* offsets, int32_t U, int32_t q, void* ws,
                                 size_t ws_bytes, double* val_out, int64_t* idx_out, ce_stream_t stream) {
    note_kernel("%s", "");  // ce_last_kernel(): "" unless this call notes a kernel
    CommArgs a{p, (int)dt, total_items, M, C, sN, sM, sC};
    int rc = check_comm(a);
    if (rc) return rc;
    rc = check_q(q);
    if (rc) return rc;
    if (U < 1 || !offsets || (q > 0 && (!val_out || !idx_out))) return fail(CE_EINVAL, "bad batched arguments");
    if (!ws || ws_bytes < ce_select_batched_workspace_bytes(total_items, U, q))
        return fail(CE_EWORKSPACE, "workspace too small");
    if (q == 0) return CE_OK;
    hipStream_t st = (hipStream_t)stream;
    if (q > CE_MAX_Q) {  // every user's items contiguous in the total order: sort by (user, key, position)
        if (U >= kSortMaxUsers) return fail(CE_EUNSUPPORTED, "q > %d needs U < %d users", CE_MAX_Q, kSortMaxUsers);
        // a record's position packs (user << kUserShift) | user-local position
        if (total_items >= (int64_t(1) << kUserShift))
            return fail(CE_EUNSUPPORTED, "q > %d needs fewer than 2^%d items in all", CE_MAX_Q, kUserShift);
        rc = check_sort_n(total_items);
        if (rc) return rc;
        const SortWs s = sort_carve(ws, total_items);
        rc = launch_entropy(a, nullptr, s.ent, st);
        if (rc) return rc;
        sort_keys_users(s.ent, total_items, offsets, U, s.a, st);
        sort_out_users(sort_run(s, user_sort_passes(U), st), offsets, U, q, val_out, idx_out, st);
        return check_launch("ce_select_batched");
    }
    const int bpu = batched_bpu(total_items, U);
    const int64_t nl = (int64_t)bpu * U;
    WsLists w = carve(ws, nl, q);
    if (q <= kStreamMaxQ) {
        // one block per user (k_select_tiles; a user longer than its block streams inside it)
        if (launch_small_users(a, offsets, U, q, val_out, idx_out, st)) return check_launch("ce_select_batched");
    }
    if (q <= kStreamMaxQ) {
        // bpu 4-wave blocks per user, then one wave per user merges its bpu lists
        if (launch_seg(a, offsets, 0, 0, q, (int)nl, bpu, bpu == 1 && U < 64 ? 64 * kSegWaves : 256, val_out, idx_out,
                       w.c, nullptr, st)) {
            if (bpu > 1) launch_merge_wave(w.c, U, bpu, q, val_out, idx_out, st);
            return check_launch("ce_select_batched");
        }
    }
    Seg sg{offsets, total_items, bpu, 0};
    const bool fin = bpu == 1;
    rc = committee_partial(a, sg, (int)nl, q, w, val_out, idx_out, fin, st);
    if (rc) return dispatch_err(rc, a);
    if (!fin) finish_lists(w, U, bpu, q, val_out, idx_out, st);
    return check_launch("ce_select_batched");
}
