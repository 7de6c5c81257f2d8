"""The device members on the reference's SHIPPED committee weights
(models/pretrained/classifier_{gnb,sgd,xgb}.it_{0..4}.pkl, amg_test.py:347-351 /
:435), read without unpickling into tests/golden/pretrained_members.npz
(gen_pretrained.py): GaussianNB bit-identical to the restated sklearn 0.24.1
math, SGD within rtol 1e-10 (BLAS dot order), XGB bit-exact to the restated
xgboost 1.3.3 predictor -- on the real 400-tree forests with their actual
default_left and early-leaf patterns.  Parity against xgboost itself stays
unpinned (not installed; the reference holds no predictions).  Then the
15-member committee (GNB/SGD f64, XGB f32, as np.array(pred_prob) stacks them)
through the fused selection against the oracle."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import ce_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ce():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ce_amd
    import ce_amd.ops

    ce_amd.load()
    return ce_amd


@pytest.fixture(scope="module")
def fx():
    with np.load(os.path.join(ROOT, "tests", "golden", "pretrained_members.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def frames(F, seed, models=(), nan=0.0):
    """Standardised frames (the reference scales its features, amg_test.py:64-65);
    every fourth frame puts one feature exactly on a real split threshold."""
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(F, 260))
    for k, m in enumerate(models):
        trees = m["learner"]["gradient_booster"]["model"]["trees"]
        for r in range(k, F, 4 * max(1, len(models))):
            t = trees[(r * 7) % len(trees)]
            n = (r // 3) % len(t["left_children"])
            if t["left_children"][n] != -1:
                X[r, t["split_indices"][n]] = t["split_conditions"][n]
    if nan:
        X[rng.random(X.shape) < nan] = np.nan
    return X


def bits(a, dt):
    return np.ascontiguousarray(a, dtype=dt).view(np.uint32 if dt == np.float32 else np.uint64)


def xgb_models(fx):
    return [json.loads(fx[f"xgb_model_{k}"].tobytes()) for k in range(5)]


def test_shipped_gnb_bit_exact(ce, fx):
    X = frames(20_000, 1)
    Xd = torch.from_numpy(X).cuda()
    for k in range(5):
        th, va, pr = fx["gnb_theta"][k], fx["gnb_var"][k], fx["gnb_prior"][k]
        want = O.ref_gnb_predict_proba(X, th, va, pr)
        got = ce.ops.gnb_predict_proba(Xd, th, va, pr).cpu().numpy()
        assert np.array_equal(bits(got, np.float64), bits(want, np.float64)), k


def test_shipped_sgd_within_1e10(ce, fx):
    X = frames(20_000, 2)
    Xd = torch.from_numpy(X).cuda()
    for k in range(5):
        want = O.ref_sgd_predict_proba(X, fx["sgd_coef"][k], fx["sgd_intercept"][k])
        got = ce.ops.sgd_predict_proba(Xd, fx["sgd_coef"][k], fx["sgd_intercept"][k]).cpu().numpy()
        np.testing.assert_allclose(got, want, rtol=1e-10, atol=1e-300)


@pytest.mark.parametrize("nan", [0.0, 0.001], ids=["dense", "missing"])
def test_shipped_xgb_bit_exact(ce, fx, nan):
    from ce_amd.xgb import XgbForest

    models = xgb_models(fx)
    X = frames(20_000 + 37, 3, models, nan)
    Xd = torch.from_numpy(X).cuda()
    for k, m in enumerate(models):
        want = O.oracle_xgb_predict_proba(X, m)
        got = ce.ops.xgb_predict_proba(Xd, XgbForest.from_json(m)).cpu().numpy()
        assert np.array_equal(bits(got, np.float32), bits(want, np.float32)), (k, np.argwhere(got != want)[:3])


def test_shipped_committee_selection(ce, fx):
    """The 15 shipped members' device outputs, stacked as np.array(pred_prob)
    stacks them (amg_test.py:441: GNB/SGD f64, XGB f32 -> f64), selected on the
    device: equal to the oracle's selection over the restated members."""
    from ce_amd.xgb import XgbForest

    models = xgb_models(fx)
    X = frames(8_000, 4, models)
    Xd = torch.from_numpy(X).cuda()
    dev_members, ref_members = [], []
    for k in range(5):
        a = (fx["gnb_theta"][k], fx["gnb_var"][k], fx["gnb_prior"][k])
        dev_members.append(ce.ops.gnb_predict_proba(Xd, *a))
        ref_members.append(O.ref_gnb_predict_proba(X, *a))
    for k in range(5):
        a = (fx["sgd_coef"][k], fx["sgd_intercept"][k])
        dev_members.append(ce.ops.sgd_predict_proba(Xd, *a))
        ref_members.append(dev_members[-1].cpu().numpy())  # SGD: BLAS order -> take the device's (within 1e-10)
        np.testing.assert_allclose(ref_members[-1], O.ref_sgd_predict_proba(X, *a), rtol=1e-10, atol=1e-300)
    for m in models:
        dev_members.append(ce.ops.xgb_predict_proba(Xd, XgbForest.from_json(m), out_dtype=torch.float64))
        ref_members.append(O.oracle_xgb_predict_proba(X, m))
    P = torch.stack(dev_members)  # [15, F, 4] f64 (the XGB rows are exact upcasts)
    vals, idx = ce.ops.select_mc(P, 10, "MNC")
    vo, io = O.oracle_select_mc(ref_members, 10)
    assert np.array_equal(idx.cpu().numpy(), io)
    assert np.array_equal(bits(vals.cpu().numpy(), np.float64), bits(vo, np.float64))
