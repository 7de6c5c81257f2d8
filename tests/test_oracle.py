"""Pin the CPU oracle (oracle/ce_oracle.c) against the golden fixtures produced by
the reference's own numpy/scipy expressions (tests/golden/gen_golden.py).

Bar: bit-exact entropies and frequencies; selected indices equal to the
canonical order (NaN first, entropy descending, lowest index first); and the
reference's own argsort picks carry the same entropies position by position
(numpy's tie order among equal entropies is unspecified)."""
import glob
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from oracle import ce_oracle as O

ORACLE_DIR = os.path.dirname(os.path.abspath(O.__file__))

MC_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "mc_*.npz")))


def same_bits(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def check_selection(ent_ref, q_ind_ref, canon, idx):
    assert np.array_equal(idx, canon)
    # the reference's own picks have the same entropies in the same slots
    e_ref = ent_ref[q_ind_ref]
    e_new = ent_ref[idx]
    assert same_bits(e_ref, e_new)


def test_paper_examples():
    g = golden("paper_examples")
    assert g["ent_full"][0] == pytest.approx(1.386, abs=5e-4)       # paper p.3
    assert g["ent_full"][0] == 1.3862943611198906 == math.log(4)
    assert g["ent_six"][0] == 1.0116348139339553
    assert np.array_equal(g["freq_six"][0], [0.167, 0.333, 0.5, 0.0])
    assert g["ent_unanimous"][0] == 0.0
    full = np.eye(4)[:, None, :]  # [M=4, N=1, C=4]
    assert O.oracle_committee_entropy(full)[0] == g["ent_full"][0]
    freq, ent = O.oracle_vote_table(np.array([[0, 1, 1, 2, 2, 2]], np.int8))
    assert np.array_equal(freq, g["freq_six"]) and ent[0] == g["ent_six"][0]


@pytest.mark.parametrize("case", MC_CASES)
def test_committee_entropy_bit_exact(case):
    g = golden(case)
    ent, mean = O.oracle_committee_entropy(g["P"], "MNC", want_mean=True)
    assert same_bits(ent, g["ent"])
    if "mean" in g:
        assert same_bits(mean, g["mean"])
    _, idx = O.oracle_topq(ent, int(g["q"]))
    check_selection(g["ent"], g["q_ind"], g["canon"], idx)


@pytest.mark.parametrize("case", MC_CASES)
def test_committee_entropy_item_major(case):
    g = golden(case)
    P = np.ascontiguousarray(np.transpose(g["P"], (1, 0, 2)))  # [N, M, C]
    assert same_bits(O.oracle_committee_entropy(P, "NMC"), g["ent"])


def test_bf16_bits():
    g = golden("mc_m8_bf16")
    assert same_bits(O.oracle_committee_entropy(g["P_bits"]), g["ent"])


def test_f32_input_matches_f64_upcast():
    g = golden("mc_m16_f32")
    P32 = g["P"].astype(np.float32)
    assert np.array_equal(P32.astype(np.float64), g["P"])
    assert same_bits(O.oracle_committee_entropy(P32), g["ent"])


@pytest.mark.parametrize("tag", ["d03", "d100"])
def test_vote_table(tag):
    g = golden(f"hc_votes_{tag}")
    freq, ent = O.oracle_vote_table(g["votes"])
    assert same_bits(freq, g["freq"])
    assert same_bits(ent, g["ent"])
    _, idx = O.oracle_topq(ent, int(g["q"]))
    check_selection(g["ent"], g["q_ind"], g["canon"], idx)
    assert same_bits(O.oracle_table_entropy(g["freq"]), g["ent"])


def test_va_raw_quadrants():
    g = golden("hc_va_raw")
    freq, ent = O.oracle_va_table(g["va"])
    assert same_bits(freq, g["freq"])
    assert same_bits(ent, g["ent"])
    # quadrant rule (amg_test.py:69-78) vote by vote, boundaries included
    va = g["va"]
    lib = O.lib()
    for n in range(0, va.shape[0], 7):
        for a in range(va.shape[1]):
            assert lib.ce_ref_quadrant(float(va[n, a, 1]), float(va[n, a, 0])) == g["quad"][n, a]


def test_mix():
    g = golden("mix_m4")
    ent_mc = O.oracle_committee_entropy(g["P"])
    ent_hc = O.oracle_table_entropy(g["hc"])
    ent = np.concatenate([ent_mc, ent_hc])
    assert same_bits(ent, g["ent"])
    _, idx = O.oracle_select_mix(g["P"], g["hc"], int(g["q"]))
    check_selection(g["ent"], g["q_ind"], g["canon"], idx)


def test_batched():
    g = golden("batched_u8")
    offs, q = g["offsets"], int(g["q"])
    for u in range(len(offs) - 1):
        seg = g["P"][:, offs[u]:offs[u + 1], :]
        ent = O.oracle_committee_entropy(seg)
        assert same_bits(ent, g["ent"][offs[u]:offs[u + 1]])
        _, idx = O.oracle_topq(ent, q)
        exp = g["canon"][u]
        assert np.array_equal(idx, exp[exp >= 0])


def test_topq_merge_equals_global():
    rng = np.random.default_rng(5)
    ent = rng.random(10000)
    ent[rng.integers(0, 10000, 50)] = np.nan
    ent[rng.integers(0, 10000, 300)] = 0.5  # ties
    q = 25
    gv, gi = O.oracle_topq(ent, q)
    vals, idxs = [], []
    for s in range(0, 10000, 1237):
        v, i = O.oracle_topq(ent[s:s + 1237], q, base=s)
        pad = q - len(v)
        vals.append(np.concatenate([v, np.zeros(pad)]))
        idxs.append(np.concatenate([i, -np.ones(pad, np.int64)]))
    mv, mi = O.oracle_topq_merge(np.concatenate(vals), np.concatenate(idxs), q)
    assert np.array_equal(mi, gi) and same_bits(mv, gv)
    assert np.array_equal(gi, O.canonical_order(ent, q))


def test_topq_q_larger_than_n():
    v, i = O.oracle_topq(np.array([0.1, np.nan, 0.3]), 10)
    assert list(i) == [1, 2, 0]


def test_group_mean_restatement_vs_pandas():
    """The pandas-1.1.5 group_mean restatement against the installed pandas on
    the reference's own expression (amg_test.py:437).  Values are dyadic
    (multiples of 2**-12, few per group) so every partial sum is exact: the
    installed pandas' compensated sums and 1.1.5's plain sums then agree bit
    for bit, and so must the restatement.  NaN cells and unsorted keys too."""
    import pandas as pd

    from oracle.ce_oracle import ref_group_mean

    rng = np.random.default_rng(437)
    F, C = 3000, 4
    s_id = rng.integers(0, 200, F) * 7 + 3
    vals = rng.integers(0, 4096, (F, C)) / 4096.0
    vals[rng.random((F, C)) < 0.01] = np.nan
    for dt in (np.float64, np.float32):
        v = vals.astype(dt)
        exp = pd.DataFrame(v, index=pd.Index(s_id, name="s_id")).groupby(["s_id"]).mean()
        got, keys = ref_group_mean(v, s_id)
        assert np.array_equal(keys, exp.index.values)
        assert got.dtype == exp.values.dtype
        assert np.array_equal(got, exp.values, equal_nan=True)


def test_member_restatements_vs_sklearn():
    """The restated predict_proba of the GaussianNB and SGD(log) members
    against the installed sklearn on fitted models.  The restatement uses the
    pinned scipy 1.5.4 logsumexp; the installed scipy's rewritten one and
    BLAS's dot order differ by rounding only: rtol 1e-9 (stated)."""
    from conftest import fitted_members
    from oracle.ce_oracle import ref_gnb_predict_proba, ref_sgd_predict_proba

    gnb, sgd, Xt = fitted_members()
    p = ref_gnb_predict_proba(Xt, gnb.theta_, gnb.var_, gnb.class_prior_)
    np.testing.assert_allclose(p, gnb.predict_proba(Xt), rtol=1e-9, atol=1e-300)
    p = ref_sgd_predict_proba(Xt, sgd.coef_, sgd.intercept_)
    np.testing.assert_allclose(p, sgd.predict_proba(Xt), rtol=1e-9, atol=1e-300)


def test_oracle_under_sanitizers():
    """the C restatement under host ASan + UBSan (oracle/Makefile
    `sanitize`: every ce_ref_* entry point on edge-case inputs; any finding
    aborts)."""
    import shutil
    import subprocess

    if shutil.which("gcc") is None and shutil.which("cc") is None:
        pytest.skip("no C compiler")
    r = subprocess.run(["make", "-s", "-C", ORACLE_DIR, "sanitize"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "sanitized oracle run: ok" in r.stdout


def test_full_order_matches_insertion_oracle():
    """canonical_order (the whole pool in the total order, used for q >
    CE_MAX_Q where the insertion oracle's O(N q) is too slow) agrees with
    ce_ref_topq on tie-heavy pools with NaN, -inf, -0.0 / +0.0 and for q beyond N."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(5)
    for n in (1, 7, 3000):
        ent = np.floor(rng.random(n) * 16) / 16
        ent[rng.random(n) < 0.05] = np.nan
        ent[rng.random(n) < 0.05] = -np.inf
        ent[rng.random(n) < 0.05] = -0.0
        ent[rng.random(n) < 0.05] = 0.0
        for q in (1, n // 2 + 1, n, n + 5):
            assert np.array_equal(O.canonical_order(ent, q), O.oracle_topq(ent, q)[1]), (n, q)
