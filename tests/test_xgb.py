"""CPU checks of the XGBoost member ('classifier_xgb'):
the C restatement of the xgboost 1.3.3 predictor (oracle/ce_oracle.c) against
an independent pure-Python walk of the JSON model that calls the host's libm
expf; the restated glibc expf against libm; the device packing (perfect
trees, group-major) evaluated in numpy against the oracle; model parsing and
argument checks.

Parity status: xgboost is not installed here and its C++ core is not in the
reference, so the predictor is a restatement of the published algorithm --
parity UNPINNED against xgboost itself; the device kernel is
pinned bit for bit to this restatement (tests/test_gpu_parity.py)."""
import json

import numpy as np
import pytest

from ce_amd.xgb import XgbForest, synthetic_model
from oracle import ce_oracle as O


def eval_packed(X, forest):
    """The device layout walked in numpy: margins [F, G] in the kernel's order."""
    nodes, leaves, goff, d = forest.pack()
    NI = (1 << d) - 1
    X32 = np.asarray(X, np.float64).astype(np.float32)
    F, G = X32.shape[0], forest.n_groups
    marg = np.full((F, G), forest.base_margin, np.float32)
    rows = np.arange(F)
    for g in range(G):
        for k in range(goff[g], goff[g + 1]):
            idx = np.zeros(F, np.int64)
            for _ in range(d):
                nd = nodes[k, idx]
                x = X32[rows, (nd[:, 0] & 0x7FFFFFFF).astype(np.int64)]
                right = np.where(np.isnan(x), (nd[:, 0] >> 31) == 0, ~(x < nd[:, 1].view(np.float32)))
                idx = 2 * idx + 1 + right
            marg[:, g] = marg[:, g] + leaves[k, idx - NI]
    return marg


def transform(marg, G):
    if G == 1:
        p1 = np.array([np.float32(1) / np.float32(np.float32(1) + O.libm_expf(-m)) for m in marg[:, 0]], np.float32)
        return np.stack([np.float32(1) - p1, p1], 1)
    out = np.empty_like(marg)
    for r, row in enumerate(marg):
        mx = row[0]
        for v in row[1:]:
            mx = v if v > mx else mx
        e = [O.libm_expf(np.float32(v - mx)) for v in row]
        ws = 0.0  # xgboost common::Softmax: `double wsum`, Python float = IEEE double
        for v in e:
            ws += float(v)
        out[r] = [np.float32(v / np.float32(ws)) for v in e]
    return out


def frames(F, D, seed, nan=0.05, ties_from=None):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(F, D))
    X[rng.random(X.shape) < nan] = np.nan
    if ties_from is not None:  # features exactly on split thresholds
        m = ties_from["learner"]["gradient_booster"]["model"]["trees"]
        for r in range(0, F, 3):
            t = m[r % len(m)]
            X[r, t["split_indices"][0]] = t["split_conditions"][0]
    return X


MODELS = {
    "softprob4_d5": dict(n_rounds=12, num_class=4, max_depth=5, num_feature=260, seed=1),
    "softprob3_d3": dict(n_rounds=10, num_class=3, max_depth=3, num_feature=40, seed=2),
    "softprob8_d6": dict(n_rounds=4, num_class=8, max_depth=6, num_feature=50, seed=3, p_stop=0.3),
    "binary_d4": dict(n_rounds=25, num_class=2, max_depth=4, num_feature=30, seed=4),
    "stumps_d1": dict(n_rounds=30, num_class=4, max_depth=1, num_feature=10, seed=5),
    "leaves_d0": dict(n_rounds=5, num_class=4, max_depth=0, num_feature=10, seed=6),
}


@pytest.mark.parametrize("name", sorted(MODELS))
def test_oracle_vs_python_walk(name):
    kw = MODELS[name]
    model = synthetic_model(**kw)
    X = frames(60, kw["num_feature"], seed=len(name), ties_from=model)
    a = O.oracle_xgb_predict_proba(X, model)
    b = O.ref_xgb_predict_proba_py(X, model)
    assert a.dtype == np.float32 and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    np.testing.assert_allclose(a.sum(1), 1.0, rtol=1e-5)


@pytest.mark.parametrize("name", sorted(MODELS))
def test_packed_layout_vs_oracle(name):
    kw = MODELS[name]
    model = synthetic_model(**kw)
    f = XgbForest.from_json(json.dumps(model))
    nodes, leaves, goff, d = f.pack()
    assert d == f.depth() <= kw["max_depth"]
    assert goff[-1] == len(f.trees) and nodes.shape[0] == leaves.shape[0] == len(f.trees)
    X = frames(300, kw["num_feature"], seed=7, ties_from=model)
    got = transform(eval_packed(X, f), f.n_groups)
    exp = O.oracle_xgb_predict_proba(X, model)
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_base_margin_binary():
    model = synthetic_model(**MODELS["binary_d4"])
    model["learner"]["learner_model_param"]["base_score"] = "2.5E-1"
    f = XgbForest.from_json(model)
    assert f.base_margin == np.float32(-O._libm_logf(np.float32(3.0)))
    X = frames(40, 30, seed=9)
    got = transform(eval_packed(X, f), 1)
    assert np.array_equal(got.view(np.uint32), O.oracle_xgb_predict_proba(X, model).view(np.uint32))


def test_restated_expf_matches_libm():
    """glibc expf restated (the FMA ifunc variant): a dense stride over all 2^32
    bit patterns plus the two inputs where the non-FMA evaluation differs.
    (The full 2^32 sweep was run once by hand: 0 mismatches.)"""
    assert O.oracle_expf_mismatches(0, 251, (1 << 32) // 251) == 0
    assert O.oracle_expf_mismatches(0xC2000000, 1, 1 << 20) == 0  # [-32, ...) dense
    hard = np.array([float.fromhex("0x1.04845ep+5"), float.fromhex("-0x1.f8cbb2p+5")], np.float32)
    assert np.array_equal(O.oracle_expf(hard).view(np.uint32), np.array([O.libm_expf(v) for v in hard]).view(np.uint32))


def test_softmax_accumulator_discriminates():
    """xgboost's common::Softmax sums the float32 exps in a DOUBLE and divides by
    its float32 cast; a float32 running sum rounds differently on some rows, so
    the walk above (double) and the oracle/device (double) are checked against
    a choice that matters."""
    rng = np.random.default_rng(3)
    differ = 0
    for row in rng.normal(0, 3, (4000, 4)).astype(np.float32):
        mx = max(row)
        e = [O.libm_expf(np.float32(v - mx)) for v in row]
        wf = np.float32(0)
        for v in e:
            wf = np.float32(wf + v)
        wd = np.float32(sum(float(v) for v in e))
        differ += wf != wd
    assert differ > 0


def test_model_errors():
    model = synthetic_model(n_rounds=2, num_class=4, max_depth=3, num_feature=8, seed=0)
    bad = json.loads(json.dumps(model))
    bad["learner"]["objective"]["name"] = "reg:squarederror"
    with pytest.raises(ValueError, match="objective"):
        XgbForest.from_json(bad)
    bad = json.loads(json.dumps(model))
    bad["learner"]["objective"]["name"] = "multi:softmax"  # predict_proba would be [1 - label, label]
    with pytest.raises(ValueError, match="objective"):
        XgbForest.from_json(bad)
    bad = json.loads(json.dumps(model))
    bad["learner"]["gradient_booster"]["model"]["tree_info"][0] = 7
    with pytest.raises(ValueError, match="tree_info"):
        XgbForest.from_json(bad).pack()
    with pytest.raises(ValueError, match="depth"):
        XgbForest.from_json(synthetic_model(n_rounds=1, num_class=4, max_depth=11, num_feature=8, p_stop=0.0)).pack()
    bad = json.loads(json.dumps(model))
    bad["learner"]["gradient_booster"]["model"]["trees"][0]["split_indices"][0] = 8
    with pytest.raises(ValueError, match="feature"):
        XgbForest.from_json(bad).pack()


def test_abi_argument_checks():
    import ctypes

    from ce_amd import _lib

    lib = _lib.load()
    p = ctypes.c_void_p(16)
    f = ctypes.c_float(0.5)
    assert lib.ce_xgb_predict_proba(p, 1, 10, 513, 513, p, p, p, 4, 5, f, 4, p, 0, 4, None) == _lib.CE_EINVAL
    assert lib.ce_xgb_predict_proba(p, 1, 10, 260, 260, p, p, p, 4, 11, f, 4, p, 0, 4, None) == _lib.CE_EINVAL
    assert lib.ce_xgb_predict_proba(p, 1, 10, 260, 260, p, p, p, 3, 5, f, 4, p, 0, 4, None) == _lib.CE_EINVAL
    assert lib.ce_xgb_predict_proba(p, 2, 10, 260, 260, p, p, p, 4, 5, f, 4, p, 0, 4, None) == _lib.CE_EINVAL
    assert lib.ce_xgb_predict_proba(p, 1, 0, 260, 260, p, p, p, 1, 5, f, 2, p, 0, 2, None) == _lib.CE_OK
    assert lib.ce_xgb_expf(None, 5, p, None) == _lib.CE_EINVAL
    assert lib.ce_xgb_lds_bytes(260, 4) == 260 * 64 * 4 + 4 * 64 * 4 + 64


def test_ops_guard_without_gpu():
    torch = pytest.importorskip("torch")
    from ce_amd import ops

    with pytest.raises(ValueError, match="HIP device"):
        ops.xgb_predict_proba(torch.zeros((4, 10), dtype=torch.float64), synthetic_model(n_rounds=1, num_feature=10))

