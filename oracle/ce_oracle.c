/*
 * ce_oracle.c -- CPU restatement of the reference's query-selection arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path (consensus-entropy_amd/) never links or calls it.
 *
 * What it restates (reference = /root/reference, juansgomez87/consensus-entropy):
 *   amg_test.py:441  consensus_prob = np.mean(np.array(pred_prob), axis=0)
 *   amg_test.py:443  ent = scipy.stats.entropy(consensus_prob, axis=1)
 *   amg_test.py:445  q_ind = np.argsort(ent)[::-1][:self.queries]
 *   amg_test.py:451-452, :479-480   the same two lines on the hc / mixed frames
 *   amg_test.py:69-78   get_quadrant(arousal, valence)
 *   amg_test.py:109-115 per-song quadrant Counter -> np.round(count / n_votes, 3)
 *
 * The arithmetic lives in numpy / scipy (pinned numpy==1.19.5, scipy==1.5.4 at
 * requirements.txt:19,37; numpy 2.2.6 / scipy 1.15.3 in this image -- same
 * algorithms for these calls).  Their published algorithms, restated here:
 *   - np.mean over axis 0 of a C-contiguous [M,N,C] stack: output initialised to
 *     the add identity +0.0, then out += P[m] for m = 0..M-1 in member order
 *     (sequential, the reduced axis is the outer loop), then true_divide by M.
 *   - np.sum over the contiguous last axis (scipy's normaliser and final sum):
 *     out = +0.0 + pairwise_sum(row), numpy's pairwise summation
 *     (numpy/core/src/umath/loops_utils.h.src): n < 8 sequential; n <= 128 eight
 *     strided accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus a
 *     sequential tail; n > 128 split at n2 = n/2 - (n/2 % 8) and recurse.
 *   - scipy.stats.entropy: pk = 1.0*pk / sum(pk); vec = special.entr(pk);
 *     S = sum(vec).  entr(x) = NaN->NaN, x>0 -> -x*log(x), x==0 -> 0, x<0 -> -inf
 *     with the C library's log (scipy's xsf/cephes entr calls std::log).
 *   - np.round(x, 3) = rint(x * 1000.0) / 1000.0 (numpy PyArray_Round).
 *   - selection order: argsort ascending then reversed == entropy descending,
 *     NaN first.  numpy's tie order is unspecified; the engine's contract
 *     tightens it to "lowest index first" (BASELINE.json north_star), which is
 *     what this oracle implements (ce_ref_better below).
 *
 * Pinning: tests/golden/gen_golden.py runs the reference expressions verbatim
 * with numpy/scipy in this container and commits the outputs; tests/test_oracle.py
 * checks this file against them bit for bit.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CE_REF_F32 0
#define CE_REF_F64 1
#define CE_REF_BF16 2

/* numpy pairwise_sum (loops_utils.h.src), restated. */
static double pairwise(const double *a, int64_t n, int64_t stride) {
    if (n < 8) {
        double res = -0.0;
        for (int64_t i = 0; i < n; i++) res += a[i * stride];
        return res;
    } else if (n <= 128) {
        double r[8], res;
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j * stride];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[(i + j) * stride];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i * stride];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise(a, n2, stride) + pairwise(a + n2 * stride, n - n2, stride);
    }
}

/* np.add.reduce over a contiguous axis: identity +0.0, then pairwise. */
double ce_ref_row_sum(const double *a, int64_t n) { return 0.0 + pairwise(a, n, 1); }

/* scipy.special.entr */
double ce_ref_entr(double x) {
    if (isnan(x)) return x;
    if (x > 0) return -x * log(x);
    if (x == 0) return 0.0;
    return -INFINITY;
}

static double load_elem(const void *p, int dtype, int64_t off) {
    if (dtype == CE_REF_F64) return ((const double *)p)[off];
    if (dtype == CE_REF_F32) return (double)((const float *)p)[off];
    /* bf16: the upper 16 bits of an IEEE f32 */
    uint32_t u = (uint32_t)((const uint16_t *)p)[off] << 16;
    float f;
    memcpy(&f, &u, 4);
    return (double)f;
}

/* scipy.stats.entropy on one row of C probabilities (amg_test.py:443). */
double ce_ref_entropy_row(const double *row, int32_t C, double *scratch) {
    double s = ce_ref_row_sum(row, C);
    for (int32_t c = 0; c < C; c++) scratch[c] = ce_ref_entr(1.0 * row[c] / s);
    return ce_ref_row_sum(scratch, C);
}

/*
 * amg_test.py:441-443 for N items.  Element (n, m, c) is at p[n*sN + m*sM + c*sC]
 * (strides in elements), so both the reference's member-major [M,N,C] stack and
 * the item-major [N,M,C] tensor are covered.  mean_out (optional) gets [N,C].
 */
int ce_ref_committee_entropy(const void *p, int dtype, int64_t N, int32_t M, int32_t C,
                             int64_t sN, int64_t sM, int64_t sC, double *mean_out,
                             double *ent) {
    if (N < 0 || M <= 0 || C <= 0) return -1;
    double *acc = (double *)malloc(sizeof(double) * (size_t)C * 2);
    if (!acc) return -2;
    double *tmp = acc + C;
    for (int64_t n = 0; n < N; n++) {
        for (int32_t c = 0; c < C; c++) acc[c] = 0.0; /* add identity */
        for (int32_t m = 0; m < M; m++)
            for (int32_t c = 0; c < C; c++) acc[c] += load_elem(p, dtype, n * sN + m * sM + c * sC);
        for (int32_t c = 0; c < C; c++) acc[c] = acc[c] / (double)M; /* true_divide */
        if (mean_out)
            for (int32_t c = 0; c < C; c++) mean_out[n * C + c] = acc[c];
        ent[n] = ce_ref_entropy_row(acc, C, tmp);
    }
    free(acc);
    return 0;
}

/* Entropy of each row of an [N,C] f64 table (hc frame, amg_test.py:451). */
int ce_ref_table_entropy(const double *tab, int64_t N, int32_t C, int64_t ld, double *ent) {
    double *tmp = (double *)malloc(sizeof(double) * (size_t)C);
    if (!tmp) return -2;
    for (int64_t n = 0; n < N; n++) ent[n] = ce_ref_entropy_row(tab + n * ld, C, tmp);
    free(tmp);
    return 0;
}

/* amg_test.py:69-78.  Returns class 0..3 (Q1..Q4) or -1 when a value is NaN
 * (such votes are removed by dropna() at amg_test.py:101 before the rule runs). */
int ce_ref_quadrant(double arousal, double valence) {
    if (isnan(arousal) || isnan(valence)) return -1;
    if (arousal >= 0 && valence >= 0) return 0;
    if (arousal > 0 && valence < 0) return 1;
    if (arousal <= 0 && valence <= 0) return 2;
    if (arousal < 0 && valence > 0) return 3;
    return -1; /* unreachable for non-NaN input */
}

static void freq_from_counts(const int64_t *cnt, int32_t C, double *frow) {
    int64_t n = 0;
    for (int32_t c = 0; c < C; c++) n += cnt[c];
    for (int32_t c = 0; c < C; c++) {
        double x = (double)cnt[c] / (double)n; /* Python int / int */
        frow[c] = rint(x * 1000.0) / 1000.0;  /* np.round(x, 3) */
    }
}

/*
 * amg_test.py:109-117 on an int8 vote matrix: votes[n*ld + a] in 0..C-1 is a
 * class vote, anything else (e.g. -1) is a missing vote.  freq [N,C] and, if
 * ent != NULL, the per-row entropy of the frequency table (amg_test.py:451).
 */
int ce_ref_vote_table(const int8_t *votes, int64_t N, int32_t A, int32_t C, int64_t ld,
                      double *freq, double *ent) {
    int64_t *cnt = (int64_t *)malloc(sizeof(int64_t) * (size_t)C);
    double *tmp = (double *)malloc(sizeof(double) * (size_t)C);
    if (!cnt || !tmp) { free(cnt); free(tmp); return -2; }
    for (int64_t n = 0; n < N; n++) {
        for (int32_t c = 0; c < C; c++) cnt[c] = 0;
        for (int32_t a = 0; a < A; a++) {
            int v = votes[n * ld + a];
            if (v >= 0 && v < C) cnt[v]++;
        }
        freq_from_counts(cnt, C, freq + n * C);
        if (ent) ent[n] = ce_ref_entropy_row(freq + n * C, C, tmp);
    }
    free(cnt);
    free(tmp);
    return 0;
}

/*
 * amg_test.py:93-117 from raw annotations: va[(n*A + a)*2 + {0,1}] = (valence,
 * arousal) as in the AMG1608 'song_label' array, NaN = missing.  4 classes.
 */
int ce_ref_va_table(const double *va, int64_t N, int32_t A, double *freq, double *ent) {
    int64_t cnt[4];
    double tmp[4];
    for (int64_t n = 0; n < N; n++) {
        cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0;
        for (int32_t a = 0; a < A; a++) {
            double v = va[(n * A + a) * 2 + 0], ar = va[(n * A + a) * 2 + 1];
            int q = ce_ref_quadrant(ar, v);
            if (q >= 0) cnt[q]++;
        }
        freq_from_counts(cnt, 4, freq + n * 4);
        if (ent) ent[n] = ce_ref_entropy_row(freq + n * 4, 4, tmp);
    }
    return 0;
}

/* Total order of the selection: NaN first, then larger entropy, then lower
 * index.  -0.0 == +0.0 as in numpy's comparisons. */
int ce_ref_better(double va, int64_t ia, double vb, int64_t ib) {
    int na = isnan(va), nb = isnan(vb);
    if (na != nb) return na;
    if (!na && va != vb) return va > vb;
    return ia < ib;
}

/* Bounded selection of the best q of N (val, idx = base + i) by ce_ref_better,
 * output sorted best-first.  Returns the number written, min(q, N). */
int64_t ce_ref_topq(const double *ent, int64_t N, int32_t q, int64_t base, double *val_out,
                    int64_t *idx_out) {
    if (q <= 0 || N <= 0) return 0;
    int64_t k = 0; /* current list length, kept sorted best-first (insertion) */
    for (int64_t i = 0; i < N; i++) {
        double v = ent[i];
        int64_t id = base + i;
        if (k == q && !ce_ref_better(v, id, val_out[k - 1], idx_out[k - 1])) continue;
        int64_t pos = (k < q) ? k : q - 1;
        while (pos > 0 && ce_ref_better(v, id, val_out[pos - 1], idx_out[pos - 1])) {
            val_out[pos] = val_out[pos - 1];
            idx_out[pos] = idx_out[pos - 1];
            pos--;
        }
        val_out[pos] = v;
        idx_out[pos] = id;
        if (k < q) k++;
    }
    return k;
}

/* Merge of candidate lists (val, idx); entries with idx < 0 are padding. */
int64_t ce_ref_topq_merge(const double *vals, const int64_t *idx, int64_t L, int32_t q,
                          double *val_out, int64_t *idx_out) {
    if (q <= 0) return 0;
    int64_t k = 0;
    for (int64_t i = 0; i < L; i++) {
        if (idx[i] < 0) continue;
        double v = vals[i];
        int64_t id = idx[i];
        if (k == q && !ce_ref_better(v, id, val_out[k - 1], idx_out[k - 1])) continue;
        int64_t pos = (k < q) ? k : q - 1;
        while (pos > 0 && ce_ref_better(v, id, val_out[pos - 1], idx_out[pos - 1])) {
            val_out[pos] = val_out[pos - 1];
            idx_out[pos] = idx_out[pos - 1];
            pos--;
        }
        val_out[pos] = v;
        idx_out[pos] = id;
        if (k < q) k++;
    }
    return k;
}

/* ---------------------------------------------------------------------------
 * XGBClassifier.predict_proba (the 'classifier_xgb' member:
 * amg_test.py:435/:467 -> xgboost/sklearn.py:991-1029 -> libxgboost 1.3.3,
 * requirements.txt:50).  The C++ core is not in /root/reference and xgboost is
 * not installed here: this restates its published CPU predictor (PARITY
 * UNPINNED against xgboost itself; the engine is pinned to this restatement):
 *   - DMatrix from the f64 array: values cast to float32; NaN = missing;
 *   - preds[row][g] = base margin; for every tree t in MODEL order:
 *     walk from node 0 -- missing -> default child, else
 *     fvalue < split_cond ? left : right (RegTree::GetNext) -- until a leaf,
 *     then preds[row][tree_info[t]] += leaf (float32)  (PredictByAllTrees);
 *   - multi:softprob: common::Softmax (src/common/math.h: wmax = fmaxf over
 *     the row; e = expf(m - wmax); `double wsum = 0.0f` accumulates the float
 *     e's in double; each e /= static_cast<float>(wsum));
 *     binary:logistic: 1/(1+expf(-m)) -> [1-p, p] (sklearn.py:1025-1029).
 * The trees are the model's own node arrays (xgboost JSON: left_children,
 * right_children, split_indices, split_conditions -- the leaf value at a leaf
 * --, default_left), tree t's nodes at [node_off[t], node_off[t+1]).
 * expf: glibc's algorithm (e_expf.c, 32-entry exp2 table) as the x86-64 FMA
 * variant evaluates it; ce_ref_expf_mismatches compares it with libm's expf.
 * ------------------------------------------------------------------------- */
static const uint64_t kExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

static uint32_t f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

float ce_ref_expf(float x) {
    const uint32_t abstop = (f32_bits(x) >> 20) & 0x7ff;
    if (abstop >= (f32_bits(88.0f) >> 20)) {
        if (f32_bits(x) == f32_bits(-INFINITY)) return 0.0f;
        if (abstop >= (f32_bits(INFINITY) >> 20)) return x + x;
        if (x > 0x1.62e42ep6f) return INFINITY;
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    const double N = 32.0, inv_ln2_n = 0x1.71547652b82fep+0 * N;
    const double c0 = 0x1.c6af84b912394p-5 / N / N / N, c1 = 0x1.ebfce50fac4f3p-3 / N / N,
                 c2 = 0x1.62e42ff0c52d6p-1 / N, shift = 0x1.8p+52;
    const double xd = x, z = inv_ln2_n * xd;
    double kd = z + shift;
    uint64_t ki;
    memcpy(&ki, &kd, 8);
    kd -= shift;
    const double r = fma(inv_ln2_n, xd, -kd);
    uint64_t t = kExp2fTab[ki % 32] + (ki << (52 - 5));
    double s;
    memcpy(&s, &t, 8);
    const double zz = fma(c0, r, c1), r2 = r * r;
    double y = fma(c2, r, 1.0);
    y = fma(zz, r2, y);
    return (float)(y * s);
}

/* bit patterns start, start+stride, ... (count of them): how many differ from libm expf */
int64_t ce_ref_expf_mismatches(uint32_t start, uint32_t stride, int64_t count) {
    int64_t bad = 0;
    uint32_t u = start;
    for (int64_t i = 0; i < count; ++i, u += stride) {
        float x;
        memcpy(&x, &u, 4);
        const float ref = expf(x), got = ce_ref_expf(x);
        if (isnan(ref) ? !isnan(got) : f32_bits(ref) != f32_bits(got)) ++bad;
    }
    return bad;
}

int ce_ref_xgb_predict_proba(const double *X, int64_t F, int32_t D, int64_t ld, const int64_t *node_off,
                             const int32_t *left, const int32_t *right, const int32_t *split_idx,
                             const float *split_cond, const uint8_t *default_left, const int32_t *tree_info,
                             int32_t T, int32_t G, int32_t C, float base_margin, float *out) {
    if (G < 1 || G > 64 || !(G == C || (G == 1 && C == 2))) return -1;
    float preds[64];
    for (int64_t r = 0; r < F; ++r) {
        const double *x = X + r * ld;
        for (int g = 0; g < G; ++g) preds[g] = base_margin;
        for (int t = 0; t < T; ++t) {
            const int64_t o = node_off[t];
            int32_t nid = 0;
            while (left[o + nid] != -1) {
                const int32_t f = split_idx[o + nid];
                if (f < 0 || f >= D) return -2;
                const double v = x[f];
                if (isnan(v)) nid = default_left[o + nid] ? left[o + nid] : right[o + nid];
                else nid = ((float)v < split_cond[o + nid]) ? left[o + nid] : right[o + nid];
            }
            preds[tree_info[t]] += split_cond[o + nid];
        }
        float *p = out + r * C;
        if (G == 1) {
            const float p1 = 1.0f / (1.0f + ce_ref_expf(-preds[0]));
            p[0] = 1.0f - p1;
            p[1] = p1;
        } else {
            float mx = preds[0];
            for (int g = 1; g < G; ++g) mx = fmaxf(preds[g], mx);
            double wsum = 0.0; /* common::Softmax: double accumulator, one float cast */
            for (int g = 0; g < G; ++g) {
                p[g] = ce_ref_expf(preds[g] - mx);
                wsum += p[g];
            }
            const float ws = (float)wsum;
            for (int g = 0; g < G; ++g) p[g] /= ws;
        }
    }
    return 0;
}

/* got[k] = an implementation's expf of bit pattern start + k: how many differ from libm's expf */
int64_t ce_ref_expf_check(const float *got, uint32_t start, int64_t count) {
    int64_t bad = 0;
    for (int64_t k = 0; k < count; ++k) {
        const uint32_t u = start + (uint32_t)k;
        float x;
        memcpy(&x, &u, 4);
        const float ref = expf(x);
        if (isnan(ref) ? !isnan(got[k]) : f32_bits(ref) != f32_bits(got[k])) ++bad;
    }
    return bad;
}

/* -------------------------------------------------------------------------
 * The C library's log is what scipy.special.entr calls (amg_test.py:443 via
 * scipy.stats.entropy).  got[i] = an implementation's log(x[i]): how many
 * differ from libm's log bit for bit (NaN matches any NaN).
 * ------------------------------------------------------------------------- */
/* This libm's exp / log over a vector: numpy 1.19.5 (the reference's pin)
 * evaluates float64 np.exp / np.log with them; the installed numpy 2.x uses its
 * own SIMD routines, so the restatements of the members call these instead. */
void ce_ref_libm_exp(const double *x, int64_t n, double *y) {
    for (int64_t i = 0; i < n; ++i) y[i] = exp(x[i]);
}
void ce_ref_libm_log(const double *x, int64_t n, double *y) {
    for (int64_t i = 0; i < n; ++i) y[i] = log(x[i]);
}

/* Mismatches (bit for bit, NaN == NaN) between got[i] and this libm's exp(x[i])
 * -- the exp numpy 1.19.5 calls for float64 (GaussianNB's logsumexp). */
int64_t ce_ref_exp_check(const double *x, const double *got, int64_t n) {
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double ref = exp(x[i]);
        uint64_t a, b;
        memcpy(&a, &ref, 8);
        memcpy(&b, &got[i], 8);
        if (isnan(ref) ? !isnan(got[i]) : a != b) ++bad;
    }
    return bad;
}

int64_t ce_ref_log_check(const double *x, const double *got, int64_t n) {
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double ref = log(x[i]);
        uint64_t a, b;
        memcpy(&a, &ref, 8);
        memcpy(&b, &got[i], 8);
        if (isnan(ref) ? !isnan(got[i]) : a != b) ++bad;
    }
    return bad;
}
