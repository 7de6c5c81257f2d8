"""Host logic that needs no GPU: the groupby geometry, the C-ABI's argument
checks for the newer entry points, and the Python validation in front of them."""
import ctypes

import numpy as np
import pytest


def test_song_groups_matches_pandas_groupby():
    import pandas as pd

    from ce_amd import song_groups

    rng = np.random.default_rng(3)
    for grouped in (True, False):
        s_id = rng.integers(0, 50, 2000) * 3 + 11
        if grouped:
            s_id = np.sort(s_id)
        uniq, offsets, perm = song_groups(s_id)
        exp = pd.Series(np.arange(len(s_id)), index=s_id).groupby(level=0)
        assert np.array_equal(uniq, np.array(sorted(exp.groups)))
        assert (perm is None) == grouped
        order = np.arange(len(s_id)) if perm is None else perm
        for g, key in enumerate(uniq):
            rows = order[offsets[g]:offsets[g + 1]]
            assert np.array_equal(rows, np.flatnonzero(s_id == key))  # row order kept (stable)
    uniq, offsets, perm = song_groups(["b", "a", "b", "c"])
    assert list(uniq) == ["a", "b", "c"] and offsets.tolist() == [0, 1, 3, 4] and perm.tolist() == [1, 0, 2, 3]


def test_new_entry_points_validate_without_gpu():
    from ce_amd import _lib

    lib = _lib.load()
    p = ctypes.c_void_p(16)
    assert lib.ce_excl_words(0) == 0 and lib.ce_excl_words(33) == 2
    # q > 64 with an exclusion bitmap / candidate records: unsupported
    rc = lib.ce_select_mc_excl(p, 0, 100, 4, 4, 16, 4, 1, p, 65, 0, p, 1 << 20, p, p, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_select_finish_cands(100, 65, p, 1 << 20, p, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_select_finish_cands(100, 10, p, 1 << 20, ctypes.c_void_p(24), None)  # misaligned records
    assert rc == _lib.CE_EINVAL
    rc = lib.ce_merge_cands(None, 8, 10, p, p, None)
    assert rc == _lib.CE_EINVAL
    # segment mean: bad dtype, bad strides
    rc = lib.ce_segment_mean(p, 2, 10, 4, 4, None, p, 3, p, 1, 4, None)
    assert rc == _lib.CE_EUNSUPPORTED
    rc = lib.ce_segment_mean(p, 1, 10, 4, 3, None, p, 3, p, 1, 4, None)
    assert rc == _lib.CE_EINVAL
    # member inference: too many features / classes, inconsistent K
    rc = lib.ce_gnb_predict_proba(p, 10, 513, 513, p, p, p, 4, p, 4, None)
    assert rc == _lib.CE_EINVAL
    for D in range(1, 8):  # fewer than 8 features: numpy's sequential sum, not the 8-lane plan
        assert lib.ce_gnb_predict_proba(p, 10, D, D, p, p, p, 4, p, 4, None) == _lib.CE_EUNSUPPORTED
    rc = lib.ce_sgd_predict_proba(p, 10, 260, 260, p, p, 3, 4, p, 4, None)
    assert rc == _lib.CE_EINVAL
    assert lib.ce_mark_selected(None, 10, p, 1, 0, None) == _lib.CE_EINVAL
    # one-launch records: q > 64 unsupported, misaligned output rejected
    assert lib.ce_select_mc_cands(p, 0, 100, 4, 4, 16, 4, 1, 65, 0, p, 1 << 20, p, None) == _lib.CE_EUNSUPPORTED
    assert lib.ce_select_mc_cands(p, 0, 100, 4, 4, 16, 4, 1, 10, 0, p, 1 << 20, ctypes.c_void_p(24),
                                  None) == _lib.CE_EINVAL
    assert lib.ce_row_div_f64(p, p, -1, p, None) == _lib.CE_EINVAL


def test_frames_entry_validates_without_gpu():
    """ce_select_frames: member count, class count, dtype, q and workspace are
    checked on the host before anything launches."""
    from ce_amd import _lib
    from ce_amd.ops import _Member

    lib = _lib.load()
    p = ctypes.c_void_p(256)
    ws = lib.ce_select_frames_workspace_bytes(1000, 10)
    assert ws >= 65536 + 16 * 10
    mem = (_Member * 2)(_Member(256, 0, 0, 4), _Member(256, 1, 1, 4))
    args = lambda M, C, q, wsb, m=mem: (ctypes.cast(m, ctypes.c_void_p), M, C, p, None, 1000, q, 0, p, wsb, p, p,
                                        None)
    assert lib.ce_select_frames(*args(0, 4, 10, ws)) == _lib.CE_EINVAL          # no member
    assert lib.ce_select_frames(*args(33, 4, 10, ws)) == _lib.CE_EINVAL         # too many
    assert lib.ce_select_frames(*args(2, 5, 10, ws)) == _lib.CE_EUNSUPPORTED    # C = 5
    assert lib.ce_select_frames(*args(2, 4, 65, ws)) == _lib.CE_EUNSUPPORTED    # q > 64
    assert lib.ce_select_frames(*args(2, 4, 10, 64)) == _lib.CE_EWORKSPACE      # workspace
    bad = (_Member * 1)(_Member(256, 2, 0, 4))                                   # bf16 member
    assert lib.ce_select_frames(*args(1, 4, 10, ws, bad)) == _lib.CE_EUNSUPPORTED
    short = (_Member * 1)(_Member(256, 0, 0, 3))                                 # row stride < C
    assert lib.ce_select_frames(*args(1, 4, 10, ws, short)) == _lib.CE_EINVAL


def test_python_guards_without_gpu():
    torch = pytest.importorskip("torch")
    from ce_amd import ops

    with pytest.raises(ValueError, match="HIP device"):
        ops.segment_mean(torch.zeros((4, 4), dtype=torch.float64), torch.zeros(2, dtype=torch.int64))
    with pytest.raises(ValueError, match="HIP device"):
        ops.gnb_predict_proba(torch.zeros((4, 4), dtype=torch.float64), np.zeros((2, 4)), np.ones((2, 4)), [0.5, 0.5])
    with pytest.raises(ValueError, match="HIP device"):
        ops.merge_cands(torch.zeros((10, 2), dtype=torch.int64), 10)


def test_select_queries_guards_without_gpu():
    from ce_amd import select_queries
    from ce_amd.select import ConsensusEntropySelector

    with pytest.raises(ValueError, match="CE_MAX_Q"):
        select_queries("mc", 2049, committee=[np.zeros((3, 4))])
    with pytest.raises(ValueError, match="mode"):
        ConsensusEntropySelector(10, "qbc")
    sel = ConsensusEntropySelector(10, "mc")
    for empty in (None, [], np.zeros((0, 5, 4))):
        with pytest.raises(ValueError, match="pred_prob"):
            sel.select(pred_prob=empty)
