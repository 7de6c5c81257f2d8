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
