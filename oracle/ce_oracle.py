"""CPU oracle for the consensus-entropy selection path -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  It is the checker, never the thing measured or shipped: the
product (``consensus-entropy_amd/ce_amd``) never imports it.

Two layers:

* ``ref_*`` -- the reference's own expressions, verbatim, on numpy/scipy
  (``amg_test.py:441-445`` mc, ``:451-452`` hc, ``:473-480`` mix,
  ``:109-117`` hc table).  Used to generate the golden fixtures
  (tests/golden/gen_golden.py) and as bench.py's CPU baseline.
* ``oracle_*`` -- thin ctypes wrappers over ``ce_oracle.c``, the C restatement
  of those expressions (see its header for the algorithm and citations), with
  the engine's total order (NaN first, entropy descending, lowest index first).
  tests/test_oracle.py pins it bit for bit against the golden fixtures.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libce_oracle.so")
_lib = None

F32, F64, BF16 = 0, 1, 2


# ---------------------------------------------------------------------------
# Reference expressions, verbatim (numpy / scipy), amg_test.py
# ---------------------------------------------------------------------------
def ref_mc(pred_prob, q):
    """amg_test.py:441-445 verbatim.  ``pred_prob`` is the list of M [N,C] member
    frames/arrays.  Returns (q_ind, ent, consensus_prob)."""
    from scipy.stats import entropy

    consensus_prob = np.mean(np.array(pred_prob), axis=0)
    ent = entropy(consensus_prob, axis=1)
    q_ind = np.argsort(ent)[::-1][:q]
    return q_ind, ent, consensus_prob


def ref_mc_shard_time(args):
    """One worker of bench.py's multi-core CPU baseline: builds its own shard
    of a mixed f64/f32 committee (seeded) and times ref_mc on it (median of
    `reps` after a warm-up), single-threaded.  Returns (seconds, items)."""
    import statistics
    import time

    n, M, C, q, seed, reps = args
    rng = np.random.default_rng(seed)
    members = []
    for m in range(M):
        e = -np.log(rng.random((n, C)))
        p = e / e.sum(-1, keepdims=True)
        members.append(p if m < M // 2 else p.astype(np.float32))
    ref_mc(members, q)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ref_mc(members, q)
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), n


def ref_hc(consensus_hc, q):
    """amg_test.py:451-452 verbatim on an [N_h, C] frequency table."""
    from scipy.stats import entropy

    ent_hc = entropy(consensus_hc, axis=1)
    q_ind = np.argsort(ent_hc)[::-1][:q]
    return q_ind, ent_hc


def ref_mix(pred_prob, consensus_hc, q):
    """amg_test.py:473-480: ROW-stack [mc mean; hc table], entropy, top-q."""
    from scipy.stats import entropy

    consensus_prob_mc = np.mean(np.array(pred_prob), axis=0)
    mix_consensus = np.concatenate([consensus_prob_mc, np.asarray(consensus_hc)], axis=0)
    ent_mix = entropy(mix_consensus, axis=1)
    q_ind = np.argsort(ent_mix)[::-1][:q]
    return q_ind, ent_mix


def ref_group_mean(values, s_id):
    """amg_test.py:437 ``pd.DataFrame(y_probs, index=X_train.index)
    .groupby(['s_id']).mean()`` restated with pandas 1.1.5's group_mean (the
    reference pins pandas==1.1.5; the installed pandas compensates its sums,
    1.1.5 does not): values upcast to float64 (ensure_float64), per (group,
    column) a sequential sum in row order skipping NaN (np.add.at applies the
    additions in index order), divided by the non-NaN count, NaN for none; the
    result is cast back to float32 for float32 input.  Groups in sorted key
    order.  Returns (means [N, C], sorted keys)."""
    v = np.asarray(values)
    keys, labels = np.unique(np.asarray(s_id), return_inverse=True)
    labels = labels.reshape(-1)
    x = v.astype(np.float64)
    N, C = len(keys), x.shape[1]
    sumx = np.zeros((N, C))
    nobs = np.zeros((N, C), np.int64)
    for j in range(C):
        ok = ~np.isnan(x[:, j])
        np.add.at(sumx[:, j], labels[ok], x[ok, j])
        np.add.at(nobs[:, j], labels[ok], 1)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = np.where(nobs > 0, sumx / np.maximum(nobs, 1), np.nan)
    if v.dtype == np.float32:
        out = out.astype(np.float32)
    return out, keys


def libm_exp(a):
    """np.exp as numpy 1.19.5 evaluates float64 (the C library's exp, element by
    element) -- the installed numpy uses its own SIMD exp."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    y = np.empty_like(a)
    lib().ce_ref_libm_exp(_ptr(a), a.size, _ptr(y))
    return y


def libm_log(a):
    """np.log as numpy 1.19.5 evaluates float64 (the C library's log)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    y = np.empty_like(a)
    lib().ce_ref_libm_log(_ptr(a), a.size, _ptr(y))
    return y


def ref_gnb_predict_proba(X, theta, var, class_prior, exp=None, log=None):
    """GaussianNB.predict_proba as the reference's pinned sklearn 0.24.1 +
    scipy 1.5.4 + numpy 1.19.5 compute it (amg_test.py:435 on the
    'classifier_gnb' member, deam_classifier.py:211): _joint_log_likelihood
    (np.log of the prior, -0.5 * np.sum(np.log(2 pi var)), -0.5 *
    np.sum((X - theta)**2 / var, 1)), then predict_log_proba with scipy 1.5.4's
    logsumexp (amax, non-finite max -> 0, exp, sum, log, + max), then np.exp.
    exp / log default to the C library's (libm_exp / libm_log: numpy 1.19.5
    calls them for float64; the installed numpy's SIMD exp / log differ by an
    ulp here and there).  The installed scipy >= 1.14 rewrote logsumexp; tests
    pin this restatement to the installed sklearn within a stated tolerance."""
    exp = libm_exp if exp is None else exp
    log = libm_log if log is None else log
    X = np.asarray(X, np.float64)
    jll = []
    for i in range(len(class_prior)):
        jointi = log(np.array([class_prior[i]], np.float64))[0]
        n_ij = -0.5 * np.sum(log(2.0 * np.pi * var[i, :]))
        n_ij -= 0.5 * np.sum(((X - theta[i, :]) ** 2) / (var[i, :]), 1)
        jll.append(jointi + n_ij)
    jll = np.array(jll).T
    a_max = np.amax(jll, axis=1, keepdims=True)
    a_max[~np.isfinite(a_max)] = 0
    s = np.sum(exp(jll - a_max), axis=1)
    log_prob_x = log(s) + np.squeeze(a_max, axis=1)
    return exp(jll - np.atleast_2d(log_prob_x).T)


def ref_sgd_predict_proba(X, coef, intercept):
    """SGDClassifier(loss='log').predict_proba (sklearn 0.24.1
    _predict_proba_lr; deam_classifier.py:214): expit(X coef^T + intercept),
    then OvR normalisation, or [1 - p, p] for a binary model (numpy @ for the
    dot products -- BLAS order, as the reference)."""
    from scipy.special import expit

    d = np.asarray(X, np.float64) @ np.asarray(coef, np.float64).T + intercept
    if d.shape[1] == 1:
        p = expit(d[:, 0])
        return np.vstack([1 - p, p]).T
    p = expit(d)
    return p / p.sum(axis=1).reshape((p.shape[0], -1))


def ref_vote_table(votes, C=4):
    """amg_test.py:109-115 on an int8 vote matrix (-1 = missing): per row,
    Counter over classes, then ``np.round(v / num_anno, 3)``.  Pure-Python loop
    (small cases only)."""
    from collections import Counter

    votes = np.asarray(votes)
    out = np.empty((votes.shape[0], C), dtype=np.float64)
    for n in range(votes.shape[0]):
        row = [int(v) for v in votes[n] if 0 <= v < C]
        cnt = Counter({c: 0 for c in range(C)})
        cnt.update(row)
        num_anno = len(row)
        for c in range(C):
            out[n, c] = np.round(cnt[c] / num_anno, 3) if num_anno else np.nan
    return out


def ref_quadrant(arousal, valence):
    """amg_test.py:69-78 verbatim (returns 'Q1'..'Q4')."""
    if arousal >= 0 and valence >= 0:
        quad = "Q1"
    elif arousal > 0 and valence < 0:
        quad = "Q2"
    elif arousal <= 0 and valence <= 0:
        quad = "Q3"
    elif arousal < 0 and valence > 0:
        quad = "Q4"
    return quad


def canonical_order(ent, q):
    """The engine's total order on a numpy entropy vector: NaN first, then
    entropy descending, then lowest index.  (numpy's own argsort tie order is
    unspecified; this is the tightened rule.)"""
    ent = np.asarray(ent, dtype=np.float64)
    n = ent.shape[0]
    isn = np.isnan(ent)
    key = np.where(isn, 0.0, ent)
    key = np.where(key == 0.0, 0.0, key)  # -0.0 == +0.0
    order = np.lexsort((np.arange(n), -key, ~isn))
    return order[:q]


# ---------------------------------------------------------------------------
# C restatement (ce_oracle.c) via ctypes
# ---------------------------------------------------------------------------
def build():
    """Compile ce_oracle.c (gcc) in place."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, i32, dp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        L.ce_ref_committee_entropy.argtypes = [vp, ctypes.c_int, i64, i32, i32, i64, i64, i64, vp, vp]
        L.ce_ref_committee_entropy.restype = ctypes.c_int
        L.ce_ref_table_entropy.argtypes = [vp, i64, i32, i64, vp]
        L.ce_ref_vote_table.argtypes = [vp, i64, i32, i32, i64, vp, vp]
        L.ce_ref_va_table.argtypes = [vp, i64, i32, vp, vp]
        L.ce_ref_topq.argtypes = [vp, i64, i32, i64, vp, vp]
        L.ce_ref_topq.restype = i64
        L.ce_ref_topq_merge.argtypes = [vp, vp, i64, i32, vp, vp]
        L.ce_ref_topq_merge.restype = i64
        L.ce_ref_quadrant.argtypes = [dp, dp]
        L.ce_ref_entr.argtypes = [dp]
        L.ce_ref_entr.restype = dp
        L.ce_ref_row_sum.argtypes = [vp, i64]
        L.ce_ref_row_sum.restype = dp
        L.ce_ref_libm_exp.argtypes = [vp, i64, vp]
        L.ce_ref_libm_log.argtypes = [vp, i64, vp]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _dtype_code(a):
    if a.dtype == np.float32:
        return F32
    if a.dtype == np.float64:
        return F64
    if a.dtype == np.uint16:  # bf16 bit patterns
        return BF16
    raise TypeError(f"unsupported dtype {a.dtype}")


def oracle_committee_entropy(P, layout="MNC", want_mean=False):
    """Entropy per item of a committee tensor ([M,N,C] if layout == 'MNC', else
    [N,M,C]); bf16 is passed as uint16 bit patterns."""
    P = np.ascontiguousarray(P)
    if layout == "MNC":
        M, N, C = P.shape
        sN, sM, sC = C, N * C, 1
    else:
        N, M, C = P.shape
        sN, sM, sC = M * C, C, 1
    ent = np.empty(N, dtype=np.float64)
    mean = np.empty((N, C), dtype=np.float64) if want_mean else None
    rc = lib().ce_ref_committee_entropy(_ptr(P), _dtype_code(P), N, M, C, sN, sM, sC,
                                        _ptr(mean) if want_mean else None, _ptr(ent))
    assert rc == 0
    return (ent, mean) if want_mean else ent


def oracle_table_entropy(T):
    T = np.ascontiguousarray(T, dtype=np.float64)
    N, C = T.shape
    ent = np.empty(N, dtype=np.float64)
    lib().ce_ref_table_entropy(_ptr(T), N, C, C, _ptr(ent))
    return ent


def oracle_vote_table(votes, C=4):
    votes = np.ascontiguousarray(votes, dtype=np.int8)
    N, A = votes.shape
    freq = np.empty((N, C), dtype=np.float64)
    ent = np.empty(N, dtype=np.float64)
    lib().ce_ref_vote_table(_ptr(votes), N, A, C, A, _ptr(freq), _ptr(ent))
    return freq, ent


def oracle_va_table(va):
    """va: [N, A, 2] float64 (valence, arousal), NaN = missing."""
    va = np.ascontiguousarray(va, dtype=np.float64)
    N, A, _ = va.shape
    freq = np.empty((N, 4), dtype=np.float64)
    ent = np.empty(N, dtype=np.float64)
    lib().ce_ref_va_table(_ptr(va), N, A, _ptr(freq), _ptr(ent))
    return freq, ent


def oracle_topq(ent, q, base=0):
    ent = np.ascontiguousarray(ent, dtype=np.float64)
    vals = np.empty(max(q, 1), dtype=np.float64)
    idx = np.empty(max(q, 1), dtype=np.int64)
    k = lib().ce_ref_topq(_ptr(ent), ent.shape[0], q, base, _ptr(vals), _ptr(idx))
    return vals[:k], idx[:k]


def oracle_topq_merge(vals, idx, q):
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    ov = np.empty(max(q, 1), dtype=np.float64)
    oi = np.empty(max(q, 1), dtype=np.int64)
    k = lib().ce_ref_topq_merge(_ptr(vals), _ptr(idx), vals.shape[0], q, _ptr(ov), _ptr(oi))
    return ov[:k], oi[:k]


def oracle_select_mc(P, q, layout="MNC"):
    ent = oracle_committee_entropy(P, layout)
    return oracle_topq(ent, q)


def oracle_select_mix(P, hc_table, q, layout="MNC"):
    ent_mc = oracle_committee_entropy(P, layout)
    ent_hc = oracle_table_entropy(hc_table)
    return oracle_topq(np.concatenate([ent_mc, ent_hc]), q)


# ---------------------------------------------------------------------------
# XGBClassifier.predict_proba (xgboost 1.3.3 predictor,
# restated -- see the ce_oracle.c section for the algorithm and why parity is
# unpinned against xgboost itself, which is absent from this image)
# ---------------------------------------------------------------------------
def _xgb_trees(model):
    """(node_off, left, right, split, cond, default_left, tree_info, G, C, base_margin)
    from an xgboost JSON model dict, the model's own node arrays concatenated."""
    lrn = model["learner"]
    m = lrn["gradient_booster"]["model"]
    objective = lrn.get("objective", {}).get("name", "multi:softprob")
    nc = int(lrn["learner_model_param"].get("num_class", "0"))
    G, C = (1, 2) if objective == "binary:logistic" else (nc, nc)
    bs = np.float32(float(lrn["learner_model_param"]["base_score"]))
    if objective == "binary:logistic":
        base = np.float32(-_libm_logf(np.float32(np.float32(1.0) / bs - np.float32(1.0))))
    else:
        base = bs
    trees = m["trees"]
    sizes = [len(t["left_children"]) for t in trees]
    node_off = np.zeros(len(trees) + 1, dtype=np.int64)
    node_off[1:] = np.cumsum(sizes)
    cat = lambda key, dt: np.ascontiguousarray(  # noqa: E731
        np.concatenate([np.asarray(t[key], dtype=dt) for t in trees]) if trees else np.zeros(0, dt))
    return (node_off, cat("left_children", np.int32), cat("right_children", np.int32),
            cat("split_indices", np.int32), cat("split_conditions", np.float32),
            np.ascontiguousarray(np.concatenate([[bool(v) for v in t["default_left"]] for t in trees]).astype(np.uint8)),
            np.ascontiguousarray(m["tree_info"], dtype=np.int32), G, C, base)


_LIBM = None


def _libm():
    global _LIBM
    if _LIBM is None:
        import ctypes.util
        _LIBM = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        for fn in ("expf", "logf"):
            getattr(_LIBM, fn).restype = ctypes.c_float
            getattr(_LIBM, fn).argtypes = [ctypes.c_float]
    return _LIBM


def _libm_logf(x):
    return np.float32(_libm().logf(ctypes.c_float(x)))


def libm_expf(x):
    """The host C library's expf (what libxgboost calls)."""
    return np.float32(_libm().expf(ctypes.c_float(x)))


def oracle_xgb_predict_proba(X, model):
    """ce_oracle.c's restated predictor on X [F, D] (f64 or f32) -> [F, C] float32."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    F, D = X.shape
    node_off, left, right, split, cond, dl, tinfo, G, C, base = _xgb_trees(model)
    out = np.empty((F, C), dtype=np.float32)
    L = lib()
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    L.ce_ref_xgb_predict_proba.argtypes = [vp, i64, i32, i64, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32,
                                           ctypes.c_float, vp]
    rc = L.ce_ref_xgb_predict_proba(_ptr(X), F, D, D, _ptr(node_off), _ptr(left), _ptr(right), _ptr(split),
                                    _ptr(cond), _ptr(dl), _ptr(tinfo), len(tinfo), G, C, float(base), _ptr(out))
    assert rc == 0, rc
    return out


def oracle_expf(x):
    """The restated glibc expf (ce_ref_expf) elementwise."""
    L = lib()
    L.ce_ref_expf.restype = ctypes.c_float
    L.ce_ref_expf.argtypes = [ctypes.c_float]
    return np.array([L.ce_ref_expf(ctypes.c_float(v)) for v in np.asarray(x, np.float32).ravel()], np.float32)


def oracle_expf_mismatches(start, stride, count):
    """How many float bit patterns start + k*stride (k < count) the restated expf
    gets different from libm's expf."""
    L = lib()
    L.ce_ref_expf_mismatches.restype = ctypes.c_int64
    L.ce_ref_expf_mismatches.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64]
    return int(L.ce_ref_expf_mismatches(start, stride, count))


def ref_xgb_predict_proba_py(X, model):
    """Pure-Python walk of the JSON model with numpy float32 arithmetic and the
    host's libm expf (small cases only): an independent check of ce_oracle.c."""
    lrn = model["learner"]
    m = lrn["gradient_booster"]["model"]
    _, _, _, _, _, _, tinfo, G, C, base = _xgb_trees(model)
    X32 = np.asarray(X, dtype=np.float64).astype(np.float32)
    out = np.empty((X32.shape[0], C), dtype=np.float32)
    for r in range(X32.shape[0]):
        preds = [np.float32(base)] * G
        for t, tr in enumerate(m["trees"]):
            nid = 0
            while tr["left_children"][nid] != -1:
                v = X32[r, tr["split_indices"][nid]]
                if np.isnan(v):
                    nid = tr["left_children"][nid] if tr["default_left"][nid] else tr["right_children"][nid]
                elif v < np.float32(tr["split_conditions"][nid]):
                    nid = tr["left_children"][nid]
                else:
                    nid = tr["right_children"][nid]
            g = tinfo[t]
            preds[g] = np.float32(preds[g] + np.float32(tr["split_conditions"][nid]))
        if G == 1:
            p1 = np.float32(np.float32(1.0) / np.float32(np.float32(1.0) + libm_expf(-preds[0])))
            out[r] = [np.float32(1.0) - p1, p1]
        else:
            mx = preds[0]
            for v in preds[1:]:
                mx = np.float32(max(v, mx))  # fmaxf (margins are finite)
            e = [libm_expf(np.float32(v - mx)) for v in preds]
            ws = 0.0  # common::Softmax: `double wsum`; Python floats are IEEE doubles
            for v in e:
                ws += float(v)
            out[r] = [np.float32(v / np.float32(ws)) for v in e]
    return out


def oracle_expf_check(got, start):
    """Mismatches of got[k] (an expf of bit pattern start + k) against libm's expf."""
    got = np.ascontiguousarray(got, dtype=np.float32)
    L = lib()
    L.ce_ref_expf_check.restype = ctypes.c_int64
    L.ce_ref_expf_check.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64]
    return int(L.ce_ref_expf_check(_ptr(got), start, got.size))


def oracle_log_check(x, got):
    """Mismatches (bit for bit, NaN == NaN) between got and libm's log(x) --
    the log scipy.special.entr calls (amg_test.py:443)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    got = np.ascontiguousarray(got, dtype=np.float64)
    assert x.shape == got.shape
    L = lib()
    L.ce_ref_log_check.restype = ctypes.c_int64
    L.ce_ref_log_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    return int(L.ce_ref_log_check(_ptr(x), _ptr(got), x.size))


def oracle_exp_check(x, got):
    """Mismatches (bit for bit, NaN == NaN) between got and libm's exp(x) --
    the exp numpy 1.19.5 uses for float64 (GaussianNB's logsumexp, §8(f)4)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    got = np.ascontiguousarray(got, dtype=np.float64)
    assert x.shape == got.shape
    L = lib()
    L.ce_ref_exp_check.restype = ctypes.c_int64
    L.ce_ref_exp_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    return int(L.ce_ref_exp_check(_ptr(x), _ptr(got), x.size))


def exp_test_arguments(n, seed):
    """n f64 arguments covering every branch of glibc's exp: the log-probability
    range of logsumexp (jll - max <= 0), uniform over the finite range, near 0
    and tiny (|x| < 2^-54), |x| >= 512 (the rescaled special case, subnormal
    results included), the overflow / underflow edges, random bit patterns,
    inf / -inf / NaN / -0."""
    rng = np.random.default_rng(seed)
    k = n // 6
    parts = [
        -rng.random(k) * 800.0,
        rng.uniform(-745.2, 709.8, k),
        rng.standard_normal(k) * 2.0 ** rng.integers(-60, 4, k),
        rng.uniform(-746.0, -512.0, k // 2),
        rng.uniform(512.0, 709.8, k // 2),
        (rng.integers(0, 1 << 63, k, dtype=np.uint64) | (rng.integers(0, 2, k, dtype=np.uint64) << np.uint64(63))).view(np.float64),
    ]
    edges = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 709.782712893384, 709.7827128933841, -708.3964185322641,
                      -744.4400719213812, -745.1332191019411, -745.1332191019412, 512.0, -512.0, 1024.0, -1024.0,
                      2.0 ** -54, -(2.0 ** -54), 2.0 ** -55, 1.0, -1.0])
    rest = n - sum(len(p) for p in parts) - len(edges)
    parts += [edges, rng.uniform(-40.0, 0.0, max(rest, 0))]
    return np.concatenate(parts)


def log_test_arguments(n, seed):
    """n f64 arguments covering every branch of glibc's log: uniform (0, 1)
    (entropy terms), [0.5, 1) bit patterns, the near-1 window [1-2^-4,
    1+0x1.09p-4), subnormals, all positive bit patterns, the values 1, 0, -0,
    inf, NaN, negatives, and every table boundary z = 0x1.6p-1 * (1 + i/128)."""
    rng = np.random.default_rng(seed)
    k = n // 6
    parts = [
        rng.random(k),
        (np.uint64(0x3FE0000000000000) + (rng.integers(0, 1 << 52, k, dtype=np.uint64))).view(np.float64),
        1.0 - 2.0 ** -4 + rng.random(k) * (2.0 ** -4 + float.fromhex("0x1.09p-4")),
        (rng.integers(1, 1 << 52, k, dtype=np.uint64)).view(np.float64),
        (rng.integers(1, 0x7FF0000000000000, k, dtype=np.uint64)).view(np.float64),
    ]
    edges = np.array([1.0, 0.0, -0.0, np.inf, np.nan, -1.0, -np.inf, 5e-324, 2.2250738585072014e-308,
                      1.0 - 2.0 ** -4, 1.0 + float.fromhex("0x1.09p-4"), np.nextafter(1.0, 0), np.nextafter(1.0, 2)])
    zb = (np.uint64(0x3FE6000000000000) + (np.arange(256, dtype=np.uint64) << np.uint64(44)))
    bnd = np.concatenate([zb - np.uint64(1), zb, zb + np.uint64(1)]).view(np.float64)
    rest = n - sum(len(p) for p in parts) - len(edges) - len(bnd)
    parts += [edges, bnd, rng.random(max(rest, 0)) * 2.0 ** rng.integers(-1074, 1, max(rest, 0))]
    return np.concatenate(parts)
