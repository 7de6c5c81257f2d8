"""The reference's shipped committee members (models/pretrained/*.pkl) as
fixtures, read without unpickling (tests/golden/pickle_walk.py): the walker
imports and calls nothing from a pickle, the committed fixture equals what it
reads from the reference's files, and the 15 members' weights run through the
CPU restatements (the GPU run is tests/test_gpu_pretrained.py)."""
import builtins
import os
import pickle
import sys

import numpy as np
import pytest

from conftest import ROOT

REF = "/root/reference"
HERE = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, HERE)
import pickle_walk as W  # noqa: E402

has_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "models", "pretrained")),
                             reason="the reference's pickles exist only in the build container")


def fixture():
    with np.load(os.path.join(HERE, "pretrained_members.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@has_ref
def test_walker_imports_and_calls_nothing(monkeypatch):
    """Reading all 15 pickles imports no module a pickle names (sklearn,
    joblib, xgboost, ...) and never reaches pickle's unpickler."""
    import gen_pretrained

    def refuse(*a, **k):
        raise AssertionError("the unpickler was called")

    for name in ("load", "loads", "Unpickler", "_load", "_loads"):
        if hasattr(pickle, name):
            monkeypatch.setattr(pickle, name, refuse)
    seen = []
    real_import = builtins.__import__

    def spy(name, *a, **k):
        seen.append(name)
        return real_import(name, *a, **k)

    before = set(sys.modules)
    monkeypatch.setattr(builtins, "__import__", spy)
    arrs = gen_pretrained.extract(REF)
    monkeypatch.setattr(builtins, "__import__", real_import)
    new = set(sys.modules) - before
    assert not any(m.split(".")[0] in ("sklearn", "joblib", "xgboost", "scipy", "pandas") for m in new), new
    named = {"sklearn", "joblib", "xgboost", "os", "subprocess", "builtins"}  # what the pickles' GLOBALs name
    assert not {m.split(".")[0] for m in seen} & named, set(seen)
    assert arrs["gnb_theta"].shape == (5, 4, 260)


@has_ref
def test_fixture_equals_the_reference_files():
    import gen_pretrained

    arrs = gen_pretrained.extract(REF)
    fx = fixture()
    assert set(arrs) == set(fx)
    for k in arrs:
        assert np.array_equal(arrs[k], fx[k]), k


def test_walker_leaves_globals_inert(tmp_path):
    """A pickle that would run os.system under pickle.loads is only a record
    here: the command never runs."""
    marker = tmp_path / "ran"
    evil = f"cos\nsystem\n(S'touch {marker}'\ntR.".encode()
    out = W.walk(evil)
    assert isinstance(out, W.Call) and out.func.is_("os", "system")
    assert not marker.exists()
    assert isinstance(W.walk(b"\x80\x02cos\nsystem\nq\x00."), W.Global)  # a bare GLOBAL stays a name
    with pytest.raises(ValueError):
        W.walk(b"\x80\x02\xff")  # unknown opcode
    with pytest.raises(ValueError):
        W.walk(b"\x80\x04\x95")  # truncated


def test_pretrained_members_through_the_restatements():
    """Each shipped member on standardised synthetic frames (the reference
    scales its features, amg_test.py:64-65): GaussianNB and SGD through the
    restated sklearn 0.24.1 math, XGB through the restated xgboost 1.3.3
    predictor -- probability rows, and the committee's selection."""
    from ce_amd.xgb import XgbForest
    from oracle import ce_oracle as O

    fx = fixture()
    rng = np.random.default_rng(1987)
    X = rng.normal(size=(400, 260))
    members = []
    for k in range(5):
        p = O.ref_gnb_predict_proba(X, fx["gnb_theta"][k], fx["gnb_var"][k], fx["gnb_prior"][k])
        assert p.shape == (400, 4) and np.allclose(p.sum(1), 1.0)
        members.append(p)
    for k in range(5):
        p = O.ref_sgd_predict_proba(X, fx["sgd_coef"][k], fx["sgd_intercept"][k])
        assert np.allclose(p.sum(1), 1.0)
        members.append(p)
    for k in range(5):
        model = __import__("json").loads(fx[f"xgb_model_{k}"].tobytes())
        forest = XgbForest.from_json(model)
        assert forest.n_groups == 4 and forest.n_classes == 4 and forest.max_feature() < 260
        assert forest.depth() <= 5 and len(forest.trees) == 400
        p = O.oracle_xgb_predict_proba(X, model)
        assert p.dtype == np.float32 and np.allclose(p.sum(1), 1.0, atol=1e-6)
        members.append(p)
    _, idx = O.oracle_select_mc(members, 10)
    assert len(set(idx.tolist())) == 10
