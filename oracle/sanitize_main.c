/*
 * sanitize_main.c -- host ASan/UBSan driver for the CPU restatement (SURVEY.md
 * §5: "host ASan/UBSan for the C++ CPU restatement").  TEST INFRASTRUCTURE
 * ONLY (tests/test_oracle.py::test_oracle_under_sanitizers builds and runs it).
 *
 * Calls every ce_ref_* entry point on seeded inputs covering the edge cases the
 * reference path meets: N = 0 / 1, q > N, q = 1, C = 1 / 4 / 8 / 129 / 1000
 * (numpy pairwise leaves and recursion), NaN / zero / negative / -0.0 rows,
 * f32 / f64 / bf16 stacks in both layouts, votes with missing entries and a row
 * with no vote, raw valence/arousal with NaN, list merges with padding.  Any
 * out-of-bounds access, leak or undefined operation aborts (exit status != 0).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int ce_ref_committee_entropy(const void *p, int dtype, int64_t N, int32_t M, int32_t C, int64_t sN, int64_t sM,
                             int64_t sC, double *mean_out, double *ent);
int ce_ref_table_entropy(const double *tab, int64_t N, int32_t C, int64_t ld, double *ent);
int ce_ref_vote_table(const int8_t *votes, int64_t N, int32_t A, int32_t C, int64_t ld, double *freq, double *ent);
int ce_ref_va_table(const double *va, int64_t N, int32_t A, double *freq, double *ent);
int64_t ce_ref_topq(const double *ent, int64_t N, int32_t q, int64_t base, double *val_out, int64_t *idx_out);
int64_t ce_ref_topq_merge(const double *vals, const int64_t *idx, int64_t L, int32_t q, double *val_out,
                          int64_t *idx_out);
int64_t ce_ref_log_check(const double *x, const double *got, int64_t n);
float ce_ref_expf(float x);

static uint64_t s = 1987;
static double urand(void) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return (double)(s >> 11) * 0x1p-53;
}

static void mc_case(int64_t N, int32_t M, int32_t C, int dtype, int layout, int32_t q) {
    const int eb = dtype == 1 ? 8 : (dtype == 0 ? 4 : 2);
    const size_t n = (size_t)N * M * C;
    void *p = malloc(n * eb + 1);
    for (size_t i = 0; i < n; i++) {
        double v = urand();
        if (i % 97 == 0) v = 0.0;
        if (i % 211 == 0) v = -0.0;
        if (i % 389 == 0) v = NAN;
        if (i % 401 == 0) v = -urand();
        if (dtype == 1) ((double *)p)[i] = v;
        else if (dtype == 0) ((float *)p)[i] = (float)v;
        else { float f = (float)v; uint32_t u; memcpy(&u, &f, 4); ((uint16_t *)p)[i] = (uint16_t)(u >> 16); }
    }
    /* layout 0: member-major [M,N,C]; 1: item-major [N,M,C] */
    const int64_t sN = layout ? (int64_t)M * C : C, sM = layout ? C : N * C, sC = 1;
    double *mean = malloc(sizeof(double) * (size_t)(N * C + 1)), *ent = malloc(sizeof(double) * (size_t)(N + 1));
    if (ce_ref_committee_entropy(p, dtype, N, M, C, sN, sM, sC, mean, ent)) exit(2);
    double *v = malloc(sizeof(double) * (size_t)q);
    int64_t *ix = malloc(sizeof(int64_t) * (size_t)q);
    const int64_t k = ce_ref_topq(ent, N, q, 5, v, ix);
    if (k != (N < q ? N : q)) exit(3);
    if (ce_ref_table_entropy(mean, N, C, C, ent)) exit(4);
    free(p); free(mean); free(ent); free(v); free(ix);
}

int main(void) {
    const int32_t Cs[] = {1, 4, 8, 129, 1000};
    for (int ci = 0; ci < 5; ci++)
        for (int dt = 0; dt < 3; dt++)
            for (int lay = 0; lay < 2; lay++) {
                mc_case(0, 3, Cs[ci], dt, lay, 10);
                mc_case(1, 1, Cs[ci], dt, lay, 10);
                mc_case(Cs[ci] >= 129 ? 300 : 5000, 4, Cs[ci], dt, lay, 64);
                mc_case(37, 20, Cs[ci], dt, lay, 1);
            }
    /* votes: missing (-1) and out-of-range labels, one row without any vote */
    const int64_t N = 1608;
    const int32_t A = 665;
    int8_t *votes = malloc((size_t)N * A);
    for (int64_t i = 0; i < N * A; i++) votes[i] = (int8_t)((int)(urand() * 6.0) - 1);
    memset(votes, -1, A);
    double *freq = malloc(sizeof(double) * N * 4), *ent = malloc(sizeof(double) * N);
    if (ce_ref_vote_table(votes, N, A, 4, A, freq, ent)) return 5;
    double *va = malloc(sizeof(double) * N * 40 * 2);
    for (int64_t i = 0; i < N * 40 * 2; i++) va[i] = (i % 17 == 0) ? NAN : urand() * 2.0 - 1.0;
    if (ce_ref_va_table(va, N, 40, freq, ent)) return 6;
    /* merge of lists with padding */
    double vals[60];
    int64_t idx[60];
    for (int i = 0; i < 60; i++) { vals[i] = (i % 7 == 0) ? NAN : urand(); idx[i] = (i % 5 == 0) ? -1 : i; }
    double ov[10];
    int64_t oi[10];
    ce_ref_topq_merge(vals, idx, 60, 10, ov, oi);
    /* log check and expf over edge arguments */
    double x[6] = {0.0, -1.0, INFINITY, NAN, 5e-324, 1.0}, y[6];
    for (int i = 0; i < 6; i++) y[i] = log(x[i]);
    if (ce_ref_log_check(x, y, 6) != 0) return 7;
    volatile float f = ce_ref_expf(-104.0f) + ce_ref_expf(88.8f) + ce_ref_expf(NAN);
    (void)f;
    free(votes); free(freq); free(ent); free(va);
    puts("sanitized oracle run: ok");
    return 0;
}
