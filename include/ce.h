/*
 * ce.h -- C-ABI of the MI355X consensus-entropy query-selection engine (libce_amd.so).
 *
 * The reference (juansgomez87/consensus-entropy) has no plugin/FFI interface: the
 * selection path is ~60 lines of NumPy/SciPy inline in AMG_Tester.run
 * (amg_test.py:425-489).  This header defines the drop-in seam at exactly that
 * place; each entry point names the reference lines it replaces.  The Python
 * mirror of the reference interface (consensus-entropy_amd/ce_amd) binds it with
 * ctypes; INTEGRATION.md shows the binding a maintainer of the reference adds.
 *
 * Conventions (all entry points):
 *   - every pointer is caller-owned DEVICE memory unless stated otherwise;
 *   - every call is stream-ordered on `stream` (a hipStream_t; NULL = legacy
 *     default stream) and asynchronous: nothing is read back to the host;
 *   - nothing allocates: scratch comes from the caller's `ws`, sized by the
 *     matching *_workspace_bytes() function (pure host arithmetic).  A
 *     workspace must be ZERO-FILLED before its first use (e.g. hipMemsetAsync
 *     once after allocating it): its 64 KiB header holds the arrival counters
 *     of the tiled kernels (a block that finishes last merges its problem's
 *     tiles), and every call leaves them zero again, so one workspace serves
 *     any sequence of calls on one stream;
 *   - return 0 (CE_OK) or a negative CE_E* code; ce_last_error() gives a
 *     thread-local message.  Nothing throws across the ABI;
 *   - strides are in ELEMENTS.  Element (n, m, c) of a committee tensor lives at
 *     p[n*sN + m*sM + c*sC]: the reference's member-major stack np.array(pred_prob)
 *     ([M,N,C], amg_test.py:441) is sN=C, sM=N*C, sC=1; the item-major [N,M,C]
 *     tensor is sN=M*C, sM=C, sC=1;
 *   - arithmetic contract (BASELINE.json north_star): inputs are loaded as
 *     f32/f64/bf16 and every sum, mean, normalisation and entropy is computed in
 *     f64 in the reference's order (member-sequential mean, numpy pairwise row
 *     sums, scipy.special.entr);
 *   - selection order: NaN entropies first, then entropy descending, then lowest
 *     index (the reference's argsort()[::-1] with its unspecified tie order
 *     tightened to lowest-index-first; -0.0 == +0.0).  Selected outputs are q
 *     slots, best first; slots beyond the number of candidates hold idx = -1 and
 *     val = NaN;
 *   - q is any integer >= 0, as the reference's -q (amg_test.py:547-553;
 *     argsort()[::-1][:q] returns min(q, N) positions, none for q = 0): q = 0
 *     writes nothing; q <= CE_MAX_Q runs on the list kernels (workspace of a few
 *     KB-MB); a larger q runs on a device radix sort of the pool's order keys
 *     (ce_sort.hpp; its workspace grows with N: ~40 B per item) -- the
 *     *_workspace_bytes functions size either.
 */
#ifndef CE_AMD_CE_H
#define CE_AMD_CE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *ce_stream_t; /* hipStream_t */

typedef enum { CE_F32 = 0, CE_F64 = 1, CE_BF16 = 2 } ce_dtype;

enum {
    CE_OK = 0,
    CE_EINVAL = -1,       /* bad argument (shape, q, stride, null pointer) */
    CE_EWORKSPACE = -2,   /* ws too small */
    CE_ELAUNCH = -3,      /* HIP runtime error on launch */
    CE_EUNSUPPORTED = -4  /* shape outside what this build implements */
};

#define CE_MAX_Q 2048 /* the list kernels' largest q; larger q: the sort path */

const char *ce_last_error(void);
const char *ce_version(void);
/* The main kernel the last selection call on this thread launched, as
 * rocprofv3 names it without "void " and the argument list (e.g.
 * "ce::k_stream_nmc<0, 4, 16, 2, false, 2>"); "" when that call launched none
 * of the noted kernels.  Lets a benchmark tie a profiled figure to the kernel
 * it actually ran. */
const char *ce_last_kernel(void);

/*
 * Per-item committee consensus entropy -- replaces amg_test.py:441 + :443:
 *   consensus_prob = np.mean(np.array(pred_prob), axis=0)
 *   ent = scipy.stats.entropy(consensus_prob, axis=1)
 * p: [N items x M members x C classes] via strides; ent: [N] f64 out.
 * mean_or_null: optional [N, C] f64 out (the consensus_prob matrix).
 */
int ce_committee_entropy(const void *p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                         int64_t sM, int64_t sC, double *mean_or_null, double *ent,
                         ce_stream_t stream);

/*
 * Human-consensus table -- replaces amg_test.py:109-117 (+ :451's entropy):
 *   per row, count votes per class (votes[n*ld + a] in [0, C) is a vote, any
 *   other value e.g. -1 is missing), freq = np.round(count / n_votes, 3),
 *   ent = scipy.stats.entropy(freq).  A row with no vote gives NaN.
 * votes: [N, A] int8 with row stride ld (bytes).  freq_or_null: [N, C] f64 out.
 * C in [1, 8].
 */
int ce_vote_entropy(const int8_t *votes, int64_t N, int32_t A, int32_t C, int64_t ld,
                    double *freq_or_null, double *ent, ce_stream_t stream);

/*
 * Same as ce_vote_entropy from the raw AMG1608 annotation array
 * (amg_test.py:88-106): va[(n*A + a)*2 + 0] = valence, [.. + 1] = arousal, f64,
 * NaN = missing (dropped as dropna() at :101); quadrant rule of :69-78; C = 4.
 */
int ce_va_entropy(const double *va, int64_t N, int32_t A, double *freq_or_null, double *ent,
                  ce_stream_t stream);

/*
 * Frame -> song segment mean of one committee member -- replaces
 *   pd.DataFrame(y_probs, index=X_train.index).groupby(['s_id']).mean()
 * (amg_test.py:437, :469) with pandas 1.1.5 group_mean semantics (the
 * reference pins pandas==1.1.5): per (song, class) an f64 sequential sum over
 * the song's frames in row order, NaN skipped, divided by the non-NaN count
 * (no frame -> NaN); float32 input gives the float32-rounded mean.
 * frames: [F, C] (dt F32|F64, row stride ld elements).  Song n owns the rows
 * perm[offsets[n]] .. perm[offsets[n+1]-1] (perm_or_null == NULL: rows
 * offsets[n] .. offsets[n+1]-1), in their original order; songs are in sorted
 * s_id order as groupby returns them.  out: [N, C] (out_dt F32|F64, row stride
 * ld_out) -- e.g. member m's slice of an [M, N, C] committee stack.
 */
int ce_segment_mean(const void *frames, ce_dtype dt, int64_t F, int32_t C, int64_t ld,
                    const int64_t *perm_or_null, const int64_t *offsets, int64_t N, void *out,
                    ce_dtype out_dt, int64_t ld_out, ce_stream_t stream);

/*
 * Frames -> committee entropy -> top-q in ONE pass --
 * replaces amg_test.py:426-445 from the members' FRAME-level outputs on: per
 * member, pd.DataFrame(y_probs, index=X_train.index).groupby(['s_id']).mean()
 * (:437; pandas 1.1.5 group_mean, as ce_segment_mean), then
 * np.mean(np.array(pred_prob), 0), scipy.stats.entropy and argsort[::-1][:q]
 * (:441-445) -- without materialising the [M, N, C] stack.
 * members: HOST array of M (<= 32) descriptors, in mod_list order; a member is
 * frame-level (rows of X_train: song n owns rows perm[offsets[n]] ..
 * perm[offsets[n+1]-1], perm_or_null == NULL: offsets[n] .. offsets[n+1]-1)
 * or song-level (song_level != 0: row n, e.g. the CNN member, :430-433).
 * Every member is f32/f64 [*, C] with row stride ld; a float32 member's song
 * means are rounded to float32 (the groupby result keeps the dtype) and the
 * stack is accumulated in f64 (north star: fp32 load, fp64 accumulate).
 * C in {2, 3, 4, 8}; any q (q <= 64 in one pass; larger q through the per-song
 * entropies); output as ce_select_mc (positions base_idx + n of the sorted songs).
 */
typedef struct {
    const void *p;
    int32_t dtype;      /* CE_F32 | CE_F64 */
    int32_t song_level; /* 0: frame rows, 1: one row per song */
    int64_t ld;         /* row stride, elements */
} ce_member;

size_t ce_select_frames_workspace_bytes(int64_t N, int32_t q);
int ce_select_frames(const ce_member *members, int32_t M, int32_t C, const int64_t *offsets,
                     const int64_t *perm_or_null, int64_t N, int32_t q, int64_t base_idx, void *ws,
                     size_t ws_bytes, double *val_out, int64_t *idx_out, ce_stream_t stream);

/*
 * Committee member inference on the device -- the
 * predict_proba of the reference's linear members (amg_test.py:435, :467;
 * deam_classifier.py:211-218) over frames X [F, D] f64 (row stride ld),
 * written to out [F, C] f64 (row stride ld_out), e.g. the input of
 * ce_segment_mean.  D <= 512 features (the reference: 260; GaussianNB needs
 * D >= 8, CE_EUNSUPPORTED below), C <= 8 classes.
 *   ce_gnb_predict_proba  GaussianNB (sklearn 0.24.1): theta / var [C, D]
 *                         (theta_, sigma_), log_prior [C] = log(class_prior_);
 *                         numpy's pairwise sums over features, scipy's logsumexp
 *   ce_sgd_predict_proba  SGDClassifier(loss='log'): coef [K, D], intercept [K];
 *                         expit(X coef^T + b), OvR-normalised for K = C > 2,
 *                         [1-p, p] for a binary model (K = 1, C = 2)
 */
int ce_gnb_predict_proba(const double *X, int64_t F, int32_t D, int64_t ld, const double *theta,
                         const double *var, const double *log_prior, int32_t C, double *out,
                         int64_t ld_out, ce_stream_t stream);
int ce_sgd_predict_proba(const double *X, int64_t F, int32_t D, int64_t ld, const double *coef,
                         const double *intercept, int32_t K, int32_t C, double *out, int64_t ld_out,
                         ce_stream_t stream);

/*
 * XGBClassifier.predict_proba on the device (the
 * 'classifier_xgb' member; amg_test.py:435/:467 -> xgboost/sklearn.py:991-1029
 * -> libxgboost 1.3.3 CPU predictor, restated in csrc/ce_xgb.hip).
 * X [F, D] (x_dt F32|F64, row stride ld; cast to float32 like DMatrix, NaN =
 * missing), D <= 512.  The forest is packed by ce_amd.xgb.XgbForest: every tree
 * padded to a perfect tree of depth `depth` (<= 10), stored group-major --
 * group g owns trees [group_offsets[g], group_offsets[g+1]) in model order:
 *   nodes  [T][2^depth - 1][2] u32 {feature | default_left << 31, split_cond bits}
 *   leaves [T][2^depth] f32
 * Every feature index must be < D.  G = C groups -> multi:softprob (softmax),
 * G = 1 and C = 2 -> binary:logistic ([1 - p, p]); C <= 8.  base_margin is the
 * margin every group starts from (base_score for softprob, -logf(1/b - 1) for
 * logistic).  out [F, C] (out_dt F32 = what xgboost returns, F64 = its exact
 * upcast, e.g. a committee stack), row stride ld_out.  Bit-identical to the
 * restated predictor, including glibc's expf in the softmax.
 *   ce_xgb_lds_bytes  dynamic LDS one block uses (host arithmetic)
 *   ce_xgb_expf       the restated glibc expf over x [n] -> y [n] (verification)
 * Forests of depth <= 5 (the reference's XGBClassifier(max_depth=5)) run
 * faster from prebuilt lane tables: ce_xgb_lane_table turns (nodes, leaves)
 * of T trees into table [2][T][64][2] u32 (T * 1024 bytes, device memory) for
 * X with D columns, once per forest; ce_xgb_predict_proba_lanes then takes the
 * table and T in place of nodes / leaves and must be given the same D.  Same
 * results as ce_xgb_predict_proba, bit for bit.
 */
int ce_xgb_predict_proba(const void *X, ce_dtype x_dt, int64_t F, int32_t D, int64_t ld,
                         const uint32_t *nodes, const float *leaves, const int32_t *group_offsets,
                         int32_t G, int32_t depth, float base_margin, int32_t C, void *out,
                         ce_dtype out_dt, int64_t ld_out, ce_stream_t stream);
int ce_xgb_lane_table(const uint32_t *nodes, const float *leaves, int32_t T, int32_t depth, int32_t D,
                      uint32_t *table, ce_stream_t stream);
int ce_xgb_predict_proba_lanes(const void *X, ce_dtype x_dt, int64_t F, int32_t D, int64_t ld,
                               const uint32_t *table, int32_t T, const int32_t *group_offsets, int32_t G,
                               int32_t depth, float base_margin, int32_t C, void *out, ce_dtype out_dt,
                               int64_t ld_out, ce_stream_t stream);
size_t ce_xgb_lds_bytes(int32_t D, int32_t G);
int ce_xgb_expf(const float *x, int64_t n, float *y, ce_stream_t stream);

/*
 * glibc's f64 log as the engine evaluates it inside every entropy
 * (scipy.special.entr's log, amg_test.py:443; csrc/ce_glibc_log.hpp), exposed
 * for verification against the C library:
 *   ce_log_f64       y[i] = log(x[i]) on the device (x, y device memory)
 *   ce_log_f64_host  the same restatement on the host CPU (x, y HOST memory;
 *                    synchronous, no GPU needed)
 */
int ce_log_f64(const double *x, int64_t n, double *y, ce_stream_t stream);
/* y[i] = x[i] / s[i] as every entropy divides its row by the row sum (one
 * reciprocal per row, ce_device.hpp RowDivisor) -- verification against IEEE
 * division (device memory, stream-ordered). */
int ce_row_div_f64(const double *x, const double *s, int64_t n, double *y, ce_stream_t stream);
int ce_log_f64_host(const double *x, int64_t n, double *y);
/* glibc's f64 exp restated (csrc/ce_glibc_exp.hpp; the exp of the GaussianNB
 * member's logsumexp): device (stream-ordered) and host
 * (synchronous, no GPU) builds, for verification against the C library. */
int ce_exp_f64(const double *x, int64_t n, double *y, ce_stream_t stream);
int ce_exp_f64_host(const double *x, int64_t n, double *y);
/* The single-block pools' approximate entropy (f32, hardware rcp / log2; the
 * prefilter of csrc/ce_small.hpp) of n exact consensus rows [n, C] (C in
 * {2, 3, 4, 8}), in log2 units, and whether each row is special (taken by the
 * exact path): verification of the error bound the prefilter's floor relies on. */
int ce_approx_entropy(const double *rows, int64_t n, int32_t C, float *h2, uint8_t *special, ce_stream_t stream);
/* The wide stream's approximate prefilter (csrc/ce_wide.hpp wave_approx_entropy:
 * f32 copies, one v_rcp_f32, a hardware log2 per class) of n rows [n, C] f64 --
 * member sums or means, laid out as k_stream_wide2 holds a dt committee's rows
 * in registers (C a multiple of 4 / 2 / 8 for f32 / f64 / bf16, C <= 2048) --
 * in log2 units, and whether each row is special (taken by the exact path):
 * verification of the kWideApproxErr2 margin the chunked C5 job skips by. */
int ce_wide_approx_entropy(const double *rows, int64_t n, int32_t C, ce_dtype dt, float *h2,
                           uint8_t *special, ce_stream_t stream);

/*
 * Top-q of an entropy vector -- replaces np.argsort(ent)[::-1][:q]
 * (amg_test.py:445, :452, :480).  Positions are reported as base_idx + i.
 * val_out: [q] f64, idx_out: [q] int64.
 */
size_t ce_topq_workspace_bytes(int64_t N, int32_t q);
int ce_topq(const double *ent, int64_t N, int32_t q, int64_t base_idx, void *ws, size_t ws_bytes,
            double *val_out, int64_t *idx_out, ce_stream_t stream);

/*
 * Merge of nlists candidate lists of q slots each (vals/idx: [nlists*q], every
 * list best-first as the ce_* outputs are; idx < 0 = empty slot) into the
 * global top-q.  Used after the RCCL all-gather of per-GPU top-q lists.  No
 * workspace: q > CE_MAX_Q merges by rank (a binary search per candidate and list).
 */
int ce_topq_merge(const double *vals, const int64_t *idx, int32_t nlists, int32_t q,
                  double *val_out, int64_t *idx_out, ce_stream_t stream);

/*
 * Fused mc selection -- replaces amg_test.py:441-445 in one pass over the
 * committee tensor (entropies never reach HBM): scores each item and keeps a
 * per-block top-q, then merges the blocks' candidates -- for q <= 64 inside
 * the same launch (the last block to finish merges), so the whole selection
 * is one kernel.
 * ce_select_mc_partial + ce_select_finish are the same two stages exposed
 * separately (q <= CE_MAX_Q; the bench times them apart).
 */
size_t ce_select_mc_workspace_bytes(int64_t N, int32_t q);
int ce_select_mc(const void *p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                 int64_t sM, int64_t sC, int32_t q, int64_t base_idx, void *ws, size_t ws_bytes,
                 double *val_out, int64_t *idx_out, ce_stream_t stream);
int ce_select_mc_partial(const void *p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                         int64_t sM, int64_t sC, int32_t q, int64_t base_idx, void *ws,
                         size_t ws_bytes, ce_stream_t stream);
/* Stage 2 of ce_select_mc / ce_select_mix / ce_topq on a filled workspace. */
int ce_select_finish(int64_t N, int32_t q, void *ws, size_t ws_bytes, double *val_out,
                     int64_t *idx_out, ce_stream_t stream);

/*
 * Exchange records for the multi-GPU merge (BASELINE.json north_star: "each GPU
 * computes its local top-q, an RCCL allgather over xGMI collects the
 * candidates, and a merge produces the final q").  A ce_cand is 16 bytes of
 * plain data: `key` is an order key monotone in the selection order (NaN first,
 * entropy descending; compare as unsigned), `idx` the global position, -1 for
 * an empty slot.  A list is q records, best first.
 *   ce_select_finish_cands  stage 2 of ce_select_mc_partial, writing the rank's
 *                           q records to `out` (the all-gather send buffer)
 *   ce_merge_cands          merge nlists such lists (the all-gather receive
 *                           buffer, rank-major) into the final top-q
 * Any q (ce_select_finish_cands: q <= CE_MAX_Q, a stage 2 of
 * ce_select_mc_partial) and 16-byte aligned record buffers.
 */
typedef struct {
    uint64_t key;
    int64_t idx;
} ce_cand;

int ce_select_finish_cands(int64_t N, int32_t q, void *ws, size_t ws_bytes, ce_cand *out,
                           ce_stream_t stream);
/* ce_select_mc writing the pool's q records to `out` in ONE launch (stage 2
 * folded into stage 1's last block; ws sized by ce_select_mc_workspace_bytes). */
int ce_select_mc_cands(const void *p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                       int64_t sM, int64_t sC, int32_t q, int64_t base_idx, void *ws, size_t ws_bytes,
                       ce_cand *out, ce_stream_t stream);
int ce_merge_cands(const ce_cand *c, int32_t nlists, int32_t q, double *val_out, int64_t *idx_out,
                   ce_stream_t stream);

/*
 * Chunked mc selection for a pool larger than HBM (BASELINE configs[4]: 50M
 * items x 32 members x 1000 classes bf16 = 3.2 TB) -- amg_test.py:441-445 over
 * a pool that arrives in chunks.  Each call scores one resident chunk (pool
 * items base_idx .. base_idx + N - 1, positions reported as pool positions)
 * and merges its top-q with the caller's running list `running` (q ce_cand
 * records, best first, 16-byte aligned device memory) in place; first != 0
 * starts a job (running's content is ignored and overwritten).  After the
 * last chunk ce_merge_cands(running, 1, q, ...) returns the selection -- the
 * same as ce_select_mc over the whole pool, ties included.  Any q.
 */
size_t ce_select_mc_chunk_workspace_bytes(int64_t N, int32_t q);
int ce_select_mc_chunk(const void *p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                       int64_t sM, int64_t sC, int32_t q, int64_t base_idx, ce_cand *running,
                       int32_t first, void *ws, size_t ws_bytes, ce_stream_t stream);

/*
 * Device-resident multi-epoch selection (amg_test.py:396-397
 * epochs, :455/:484 hc-pool shrink, :521-531 X_train shrink): instead of
 * rebuilding the pool every epoch, the caller keeps the full pool on the device
 * with an exclusion bitmap (bit i of word i/32 set = item i already queried).
 *   ce_excl_words      uint32 words of a bitmap for N items (host arithmetic)
 *   ce_select_mc_excl  ce_select_mc over the items whose bit is clear (any q;
 *                      ws sized by ce_select_mc_workspace_bytes)
 *   ce_mark_selected   set the bits of the n positions idx[0..n) (minus
 *                      base_idx; negative / out-of-range entries ignored) --
 *                      fed the previous call's idx_out, nothing leaves the GPU
 */
size_t ce_excl_words(int64_t N);
int ce_select_mc_excl(const void *p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                      int64_t sM, int64_t sC, const uint32_t *excl, int32_t q, int64_t base_idx,
                      void *ws, size_t ws_bytes, double *val_out, int64_t *idx_out,
                      ce_stream_t stream);
int ce_mark_selected(uint32_t *excl, int64_t N, const int64_t *idx, int32_t n, int64_t base_idx,
                     ce_stream_t stream);

/*
 * Fused mix selection -- replaces amg_test.py:473-480: the ROW stack
 * [mc consensus (N rows); hc table (N_h rows)], entropy, top-q over the union.
 * Positions in [0, N) are committee items, [N, N + N_h) hc rows.
 * hc: [N_h, C] f64 with row stride ld_hc (elements).
 */
size_t ce_select_mix_workspace_bytes(int64_t N, int64_t N_h, int32_t q);
int ce_select_mix(const void *p, ce_dtype dt, int64_t N, int32_t M, int32_t C, int64_t sN,
                  int64_t sM, int64_t sC, const double *hc, int64_t N_h, int64_t ld_hc, int32_t q,
                  void *ws, size_t ws_bytes, double *val_out, int64_t *idx_out,
                  ce_stream_t stream);

/*
 * Batched personalization -- replaces the per-user loop (amg_test.py:345) around
 * :441-445: U independent pools in one launch.  User u owns items
 * [offsets[u], offsets[u+1]) of the committee tensor (offsets: [U+1] int64,
 * DEVICE memory; total_items = offsets[U] is passed for workspace sizing).
 * Output slots [u*q, (u+1)*q); positions are user-local (0-based in the pool).
 */
size_t ce_select_batched_workspace_bytes(int64_t total_items, int32_t U, int32_t q);
int ce_select_batched(const void *p, ce_dtype dt, int64_t total_items, int32_t M, int32_t C,
                      int64_t sN, int64_t sM, int64_t sC, const int64_t *offsets, int32_t U,
                      int32_t q, void *ws, size_t ws_bytes, double *val_out, int64_t *idx_out,
                      ce_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CE_AMD_CE_H */
