"""GPU parity of the XGBoost member: ce_xgb_predict_proba
through the C-ABI against the C restatement of the xgboost 1.3.3 predictor
(oracle/ce_oracle.c).  Bar: BIT-EXACT float32 probabilities -- the traversal is
comparisons, the margins are the same float32 chain in model order, and the
device evaluates the same glibc expf (checked exhaustively here against the
host's libm).  Parity against xgboost itself is unpinned."""
import numpy as np
import pytest

from ce_amd.xgb import XgbForest, synthetic_model
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


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def frames(F, D, seed, nan=0.03, model=None):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(F, D))
    X[rng.random(X.shape) < nan] = np.nan
    if model is not None:  # every third frame sits exactly on a root threshold
        trees = model["learner"]["gradient_booster"]["model"]["trees"]
        for r in range(0, F, 3):
            t = trees[r % len(trees)]
            if t["left_children"][0] != -1:
                X[r, t["split_indices"][0]] = t["split_conditions"][0]
    return X


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


CASES = [
    # (name, model kwargs, F)
    ("reference_member", dict(n_rounds=100, num_class=4, max_depth=5, num_feature=260, seed=1987), 20_000),
    ("ragged_tail", dict(n_rounds=7, num_class=4, max_depth=5, num_feature=260, seed=11), 1_000 * 64 + 37),
    ("one_frame", dict(n_rounds=9, num_class=4, max_depth=5, num_feature=260, seed=12), 1),
    ("three_class", dict(n_rounds=30, num_class=3, max_depth=4, num_feature=77, seed=13), 4_099),
    ("eight_class_d7", dict(n_rounds=6, num_class=8, max_depth=7, num_feature=512, seed=14, p_stop=0.25), 3_000),
    ("binary", dict(n_rounds=60, num_class=2, max_depth=5, num_feature=100, seed=15), 5_000),
    ("stumps", dict(n_rounds=50, num_class=4, max_depth=1, num_feature=9, seed=16), 2_000),
    ("leaves_only", dict(n_rounds=5, num_class=4, max_depth=0, num_feature=9, seed=17), 500),
    ("deep_d10", dict(n_rounds=2, num_class=4, max_depth=10, num_feature=64, seed=18, p_stop=0.05), 1_500),
    # depth 5 with an odd feature count: the LDS-staged walk's tree slots sit past an odd-sized tile
    ("odd_features_d5", dict(n_rounds=12, num_class=4, max_depth=5, num_feature=259, seed=19), 2_000),
    # the lane-table kernel's staging widths (ce_xgb_predict_proba_lanes: 64-feature chunks 2 / 4 / 5 / 8)
    ("d200_chunks4", dict(n_rounds=10, num_class=4, max_depth=5, num_feature=200, seed=20), 1_000),
    ("d400_chunks8", dict(n_rounds=10, num_class=3, max_depth=5, num_feature=400, seed=21), 1_000),
]


@pytest.mark.parametrize("nan", [0.03, 0.0], ids=["missing", "dense"])
@pytest.mark.parametrize("name,kw,F", CASES, ids=[c[0] for c in CASES])
def test_xgb_bit_exact(ce, name, kw, F, nan):
    """With missing values (every tile takes the default-direction path) and
    without (the single-compare path)."""
    model = synthetic_model(**kw)
    forest = XgbForest.from_json(model)
    X = frames(F, kw["num_feature"], seed=F, nan=nan, model=model)
    exp = O.oracle_xgb_predict_proba(X, model)
    got = ce.ops.xgb_predict_proba(dev(X), forest).cpu().numpy()
    assert got.dtype == np.float32
    assert np.array_equal(bits(got), bits(exp)), (np.argwhere(bits(got) != bits(exp))[:5], name)


def test_xgb_sparse_missing_tiles(ce):
    """A few NaN frames scattered over many tiles: tiles with and without a
    missing value in one launch."""
    kw = dict(n_rounds=40, num_class=4, max_depth=5, num_feature=260, seed=31)
    model = synthetic_model(**kw)
    X = frames(64 * 300 + 5, 260, seed=9, nan=0.0, model=model)
    X[np.arange(7, X.shape[0], 997), np.arange(7, X.shape[0], 997) % 260] = np.nan
    exp = O.oracle_xgb_predict_proba(X, model)
    got = ce.ops.xgb_predict_proba(dev(X), XgbForest.from_json(model)).cpu().numpy()
    assert np.array_equal(bits(got), bits(exp))


def test_xgb_dtypes_and_strides(ce):
    """f32 input (cast is the identity), f64 output (exact upcast), ld > D
    (a column slice of a wider frame matrix), out row stride > C."""
    kw = dict(n_rounds=20, num_class=4, max_depth=5, num_feature=260, seed=21)
    model = synthetic_model(**kw)
    forest = XgbForest.from_json(model)
    X = frames(3_333, 260, seed=5, model=model)
    exp = O.oracle_xgb_predict_proba(X, model)
    X32 = X.astype(np.float32)
    got = ce.ops.xgb_predict_proba(dev(X32), forest).cpu().numpy()
    assert np.array_equal(bits(got), bits(O.oracle_xgb_predict_proba(X32.astype(np.float64), model)))
    assert np.array_equal(bits(got), bits(exp))  # DMatrix's f64 -> f32 cast is the same rounding
    wide = dev(np.concatenate([X, np.full((X.shape[0], 9), 7.0)], 1))[:, :260]
    got64 = ce.ops.xgb_predict_proba(wide, forest, out_dtype=torch.float64).cpu().numpy()
    assert got64.dtype == np.float64 and np.array_equal(got64, exp.astype(np.float64))
    out = torch.full((X.shape[0], 6), -1.0, dtype=torch.float32, device="cuda")
    ce.ops.xgb_predict_proba(dev(X), forest, out=out)
    o = out.cpu().numpy()
    assert np.array_equal(bits(o[:, :4]), bits(exp)) and np.all(o[:, 4:] == -1.0)


def test_xgb_zero_frames(ce):
    forest = XgbForest.from_json(synthetic_model(n_rounds=2, num_feature=10))
    out = ce.ops.xgb_predict_proba(torch.empty((0, 10), dtype=torch.float64, device="cuda"), forest)
    assert tuple(out.shape) == (0, 4)


def test_device_expf_exhaustive(ce):
    """The device's glibc expf over ALL 2^32 float bit patterns vs the host
    libm expf (chunks of 2^28; the compare runs in C)."""
    from ce_amd._lib import call
    import ctypes

    n = 1 << 28
    y = torch.empty(n, dtype=torch.float32, device="cuda")
    bad = 0
    for c in range(16):
        start = c * n
        x = (torch.arange(n, dtype=torch.int64, device="cuda") + start).to(torch.int32).view(torch.float32)
        call("ce_xgb_expf", ctypes.c_void_p(x.data_ptr()), n, ctypes.c_void_p(y.data_ptr()),
             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        bad += O.oracle_expf_check(y.cpu().numpy(), start)
        print(f"expf chunk {c}: {bad} mismatches so far", flush=True)
    assert bad == 0


def test_xgb_member_in_committee(ce):
    """amg_test.py:426-445 with an xgb member on the device: frames -> xgb
    predict_proba (float32, as xgboost returns) -> per-song mean (pandas
    float32 groupby semantics) -> stack with a GaussianNB member -> selection,
    against the oracle on the same member outputs."""
    from conftest import fitted_members
    from oracle.ce_oracle import ref_group_mean

    gnb, _, Xt = fitted_members(n_test=16_080)
    model = synthetic_model(n_rounds=100, num_class=4, max_depth=5, num_feature=260, seed=1987)
    forest = XgbForest.from_json(model)
    s_id = np.repeat(np.arange(1608) * 3, 10)
    Xd = dev(Xt)
    fr_xgb = ce.ops.xgb_predict_proba(Xd, forest)
    assert np.array_equal(bits(fr_xgb.cpu().numpy()), bits(O.oracle_xgb_predict_proba(Xt, model)))
    fr_gnb = ce.ops.gnb_predict_proba(Xd, gnb.theta_, gnb.var_, gnb.class_prior_)
    _, offsets, _ = ce.song_groups(s_id)
    stack = torch.empty((2, 1608, 4), dtype=torch.float64, device="cuda")
    ce.ops.segment_mean(fr_xgb, dev(offsets), out=stack[0])
    ce.ops.segment_mean(fr_gnb, dev(offsets), out=stack[1])
    P = np.array([ref_group_mean(fr_xgb.cpu().numpy(), s_id)[0], ref_group_mean(fr_gnb.cpu().numpy(), s_id)[0]])
    assert np.array_equal(stack.cpu().numpy(), P)
    _, idx = ce.ops.select_mc(stack, 10, "MNC")
    assert np.array_equal(idx.cpu().numpy(), O.oracle_select_mc(P, 10, "MNC")[1])


@pytest.mark.parametrize("nan", [0.03, 0.0], ids=["missing", "dense"])
@pytest.mark.parametrize("name", ["reference_member", "ragged_tail", "three_class", "binary", "stumps",
                                  "leaves_only", "odd_features_d5", "d200_chunks4", "d400_chunks8"])
def test_xgb_lane_paths_agree(ce, name, nan):
    """The three walks of a depth <= 5 forest through the C-ABI directly:
    ce_xgb_predict_proba (per-tile tables built on the fly) and
    ce_xgb_predict_proba_lanes over the ce_xgb_lane_table tables (what
    ops.xgb_predict_proba runs) -- bit-identical to each other and to the
    restated predictor; the lane ABI refuses a deeper forest."""
    from ce_amd import _lib
    from ce_amd.ops import _p, _stream

    kw, F = {c[0]: (c[1], c[2]) for c in CASES}[name]
    model = synthetic_model(**kw)
    forest = XgbForest.from_json(model)
    D = kw["num_feature"]
    X = dev(frames(F, D, seed=F + 1, nan=nan, model=model))
    exp = bits(O.oracle_xgb_predict_proba(X.cpu().numpy(), model))
    lib = _lib.load()
    nodes, leaves, goff, depth = forest.device_arrays(X.device)
    G, C = forest.n_groups, forest.n_classes
    outs = []
    for lanes in (False, True):
        out = torch.empty((F, C), dtype=torch.float32, device="cuda")
        if lanes:
            table = forest.lane_table(X.device, D)
            rc = lib.ce_xgb_predict_proba_lanes(_p(X), 1, F, D, X.stride(0), _p(table), table.shape[1], _p(goff), G,
                                                depth, float(forest.base_margin), C, _p(out), 0, out.stride(0),
                                                _stream(X.device))
        else:
            rc = lib.ce_xgb_predict_proba(_p(X), 1, F, D, X.stride(0), _p(nodes), _p(leaves), _p(goff), G, depth,
                                          float(forest.base_margin), C, _p(out), 0, out.stride(0), _stream(X.device))
        assert rc == 0
        outs.append(bits(out.cpu().numpy()))
    assert np.array_equal(outs[0], exp) and np.array_equal(outs[1], exp), name
    assert lib.ce_xgb_lane_table(_p(nodes), _p(leaves), 1, 6, D, _p(X), _stream(X.device)) != 0
