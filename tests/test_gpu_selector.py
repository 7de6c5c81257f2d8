"""The drop-in selector on the reference's own data structures: pandas frames
indexed by song id, as AMG_Tester.run holds them (amg_test.py:425-489).  Each
test restates the reference lines it checks with the oracle's arithmetic and
the lowest-position tie rule (tests/test_gpu_parity.py covers the kernels)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pd = pytest.importorskip("pandas")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ce():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ce_amd

    ce_amd.load()
    return ce_amd


def member_frames(rng, ids, dtypes, quant=None):
    """pred_prob as amg_test.py:437 builds it: one DataFrame per member, index =
    the sorted s_id of groupby, columns = the 4 quadrants."""
    out = []
    for dt in dtypes:
        e = -np.log(rng.random((len(ids), 4)))
        p = e / e.sum(1, keepdims=True)
        if quant:
            p = np.floor(p * quant) / quant + 1e-3
        out.append(pd.DataFrame(p.astype(dt), index=pd.Index(ids, name="s_id"), columns=["Q1", "Q2", "Q3", "Q4"]))
    return out


def ref_positions(P, q):
    from oracle import ce_oracle as O

    return O.oracle_select_mc(np.asarray(P), q, "MNC")[1]


def test_mc_ids_through_last_member_index(ce):
    """amg_test.py:441-447: q_ind over the stacked members, q_songs from the
    LAST member frame's index (y_probs.iloc[q_ind].index)."""
    rng = np.random.default_rng(447)
    ids = np.sort(rng.choice(100_000, 1608, replace=False))
    pred_prob = member_frames(rng, ids, [np.float64, np.float64, np.float32, np.float32], quant=16)
    sel = ce.ConsensusEntropySelector(queries=10, mode="mc")
    q_songs, hc_after = sel.select(pred_prob=pred_prob)
    q_ind = ref_positions(np.array([m.values for m in pred_prob]), 10)  # np.array upcasts to f64 (:441)
    assert q_songs == pred_prob[-1].iloc[q_ind].index.tolist()
    assert hc_after is None


def test_hc_select_and_shrink(ce):
    """amg_test.py:451-455 over two epochs: entropy of the remaining hc rows (in
    annotation order, not sorted), ids through the hc frame's index, the picks
    dropped with ~index.isin(q_songs)."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(455)
    ids = rng.permutation(np.arange(3000, 4608))  # annotation order
    votes = rng.integers(-1, 4, size=(1608, 30)).astype(np.int8)
    votes[:, 0] = rng.integers(0, 4, 1608)
    freq, _ = O.oracle_vote_table(votes)
    hc = pd.DataFrame(freq, index=ids, columns=["Q1", "Q2", "Q3", "Q4"])
    sel = ce.ConsensusEntropySelector(queries=10, mode="hc")
    cur = hc
    for _ in range(2):
        q_songs, nxt = sel.select(consensus_hc=cur)
        _, q_ind = O.oracle_topq(O.oracle_table_entropy(cur.values), 10)
        assert q_songs == cur.iloc[q_ind].index.tolist()
        exp = cur[~cur.index.isin(q_songs)]
        assert nxt.index.equals(exp.index) and np.array_equal(nxt.values, exp.values)
        cur = nxt
    assert len(cur) == 1608 - 20


def test_mix_duplicate_song_and_shrink(ce):
    """amg_test.py:473-484: the ROW stack [mc (sorted s_id); hc (annotation
    order)], one top-q over the union; a song whose mc row and hc row both rank
    is picked twice (fewer unique ids), and the hc frame drops it once."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(484)
    ids = np.sort(rng.choice(50_000, 1608, replace=False))
    pred_prob = member_frames(rng, ids, [np.float64, np.float32, np.float64, np.float32])
    dup = ids[700]
    for m in pred_prob:  # song `dup`: maximal entropy in the committee ...
        m.loc[dup] = 0.25
    hc_ids = rng.permutation(ids)
    freq = np.round(rng.dirichlet(np.ones(4) * 0.3, 1608), 3)
    hc = pd.DataFrame(freq, index=hc_ids, columns=["Q1", "Q2", "Q3", "Q4"])
    hc.loc[dup] = 0.25  # ... and in the crowd's table
    sel = ce.ConsensusEntropySelector(queries=10, mode="mix")
    q_songs, hc_after = sel.select(pred_prob=pred_prob, consensus_hc=hc)
    P = np.array([m.values for m in pred_prob])
    ent = np.concatenate([O.oracle_committee_entropy(P, "MNC"), O.oracle_table_entropy(hc.values)])
    _, q_ind = O.oracle_topq(ent, 10)
    stack_index = list(pred_prob[-1].index) + list(hc.index)
    assert q_songs == [stack_index[i] for i in q_ind]
    assert q_songs.count(dup) == 2 and len(set(q_songs)) < len(q_songs)
    exp = hc[~hc.index.isin(q_songs)]
    assert hc_after.index.equals(exp.index) and len(hc_after) == 1608 - len(set(q_songs) & set(hc.index))


def test_rand_matches_seeded_global_rng(ce):
    """amg_test.py:55 + :486-489: np.random.seed(1987) (the constructor), then
    np.random.shuffle of X_train.index.unique().tolist(), first q -- the global
    legacy MT19937 stream, so the selector must draw from it in the same way."""
    rng = np.random.default_rng(489)
    frames_index = pd.Index(np.repeat(rng.permutation(np.arange(1608)), 5), name="s_id")  # frame rows
    np.random.seed(1987)
    exp_pool = frames_index.unique().tolist()
    np.random.shuffle(exp_pool)
    exp = exp_pool[:10]
    np.random.seed(1987)
    sel = ce.ConsensusEntropySelector(queries=10, mode="rand")
    got, _ = sel.select(pool_ids=frames_index)
    assert got == exp
    # a second epoch continues the same stream
    np.random.seed(1987)
    a = frames_index.unique().tolist()
    np.random.shuffle(a)
    b = frames_index.unique().tolist()
    np.random.shuffle(b)
    np.random.seed(1987)
    sel.select(pool_ids=frames_index)
    assert sel.select(pool_ids=frames_index)[0] == b[:10]


def test_all_f32_committee_contract(ce):
    """Documented contract (DESIGN.md 'Numerics'): an all-float32 committee is
    accumulated in float64 (north star: fp32 load, fp64 accumulate).  numpy
    would stack it as float32 and average in float32, so the engine equals the
    reference on the float64 upcast of the same members -- the reference's
    real committee is mixed (GNB/SGD f64 + XGB/CNN f32) and upcast anyway."""
    rng = np.random.default_rng(32)
    ids = np.arange(1608)
    pred_prob = member_frames(rng, ids, [np.float32] * 4)
    assert np.array([m.values for m in pred_prob]).dtype == np.float32  # what numpy would average in
    sel = ce.ConsensusEntropySelector(queries=10, mode="mc")
    q_songs, _ = sel.select(pred_prob=pred_prob)
    q_ind = ref_positions(np.array([m.values for m in pred_prob]).astype(np.float64), 10)
    assert q_songs == pred_prob[-1].iloc[q_ind].index.tolist()
