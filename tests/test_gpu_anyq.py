"""The reference's q on every entry point (amg_test.py:445, :452, :480, :489;
`-q` any integer at :547-553): argsort(ent)[::-1][:q] returns min(q, N)
positions and none for q = 0.  Every path is held to the oracle at q in
{0, 65, 2049, N + 5}: q <= 64 runs on the streaming / single-block kernels,
64 < q <= CE_MAX_Q (2048) on the block lists, q > CE_MAX_Q on the device radix
sort (csrc/ce_launch_sort.hip).  Pools are tie-heavy so the lowest-position
rule decides many places.  The oracle is the C restatement's entropies with
canonical_order (the total order as a stable lexsort, pinned to the insertion
oracle in tests/test_oracle.py)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

QS = ("0", "65", "2049", "N+5")


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


def idx_np(t):
    i = t.cpu().numpy()
    return i[i >= 0]


def qval(kind, n):
    return n + 5 if kind == "N+5" else int(kind)


def committee(rng, N, M=4, C=4, quant=16, dtype=np.float64):
    e = -np.log(rng.random((M, N, C)))
    P = np.floor(e / e.sum(-1, keepdims=True) * quant) / quant + 1e-3  # coarse: exact ties everywhere
    return P.astype(dtype)


def hc_table(rng, N):
    votes = rng.integers(-1, 4, (N, 30)).astype(np.int8)  # ~24 votes per song: few distinct tables
    from oracle import ce_oracle as O

    return O.oracle_vote_table(votes)[0]


def expected(ent, q):
    from oracle import ce_oracle as O

    return O.canonical_order(ent, q)


@pytest.mark.parametrize("kind", QS)
def test_select_queries_any_q(ce, kind):
    """mc / hc / mix through the drop-in select_queries and the device ops."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(7)
    N, Nh = 3000, 2500
    P = committee(rng, N)
    H = hc_table(rng, Nh)
    ent_mc = O.oracle_committee_entropy(P, "MNC")
    ent_hc = O.oracle_table_entropy(H)
    members = [P[m] for m in range(P.shape[0])]
    q = qval(kind, N)
    assert np.array_equal(ce.select_queries("mc", q, committee=members), expected(ent_mc, q))
    q = qval(kind, Nh)
    assert np.array_equal(ce.select_queries("hc", q, hc=H), expected(ent_hc, q))
    q = qval(kind, N + Nh)
    assert np.array_equal(ce.select_queries("mix", q, committee=members, hc=H),
                          expected(np.concatenate([ent_mc, ent_hc]), q))
    # the device ops keep q slots (padding past the pool), item-major too
    q = qval(kind, N)
    v, i = ce.ops.select_mc(dev(P.transpose(1, 0, 2)), q, "NMC")
    assert i.shape == (q,) and v.shape == (q,)
    assert np.array_equal(idx_np(i), expected(ent_mc, q))
    assert (i.cpu().numpy()[N:] == -1).all()
    _, i = ce.ops.topq(dev(ent_mc), q, base_idx=100)
    assert np.array_equal(idx_np(i), expected(ent_mc, q) + 100)


@pytest.mark.parametrize("q", [2048, 2049, 5000])
def test_large_pool_any_q(ce, q):
    """A 600K-item f32 pool: the list kernels at q = 2048 and the sort path
    above, the same total order, entropies bit-identical."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(q)
    N = 600_000
    e = -np.log(rng.random((N, 16, 4)))
    P = (np.floor(e / e.sum(-1, keepdims=True) * 32) / 32).astype(np.float32)
    P[rng.random(N) < 0.001] = 0.0  # zero rows: NaN entropy, ranked first
    ent = O.oracle_committee_entropy(P, "NMC")
    Pd = dev(P)
    v, i = ce.ops.select_mc(Pd, q, "NMC")
    exp = expected(ent, q)
    assert np.array_equal(idx_np(i), exp)
    got, want = v.cpu().numpy(), ent[exp]  # bit-identical entropies (NaN: any payload)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    ok = ~np.isnan(want)
    assert np.array_equal(got[ok].view(np.int64), want[ok].view(np.int64))
    # member-major stack, and an exclusion bitmap dropping every third item
    _, i = ce.ops.select_mc(Pd.permute(1, 0, 2).contiguous(), q, "MNC")
    assert np.array_equal(idx_np(i), exp)
    ex = ce.ops.excl_bitmap(N, "cuda")
    drop = torch.arange(0, N, 3, device="cuda")
    ce.ops.mark_selected(ex, N, drop)
    _, i = ce.ops.select_mc(Pd, q, "NMC", excl=ex)
    keep = np.flatnonzero(np.arange(N) % 3 != 0)
    assert np.array_equal(idx_np(i), keep[expected(ent[keep], q)])


@pytest.mark.parametrize("kind", QS)
def test_batched_any_q(ce, kind):
    """Ragged users (empty, 1 item, shorter and longer than q) in one call."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(11)
    sizes = [3000, 0, 1, 70, 2100, 4500, 65]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    P = committee(rng, int(offs[-1]), dtype=np.float32)
    ent = O.oracle_committee_entropy(P, "MNC")
    q = qval(kind, max(sizes))
    v, i = ce.ops.select_batched(dev(P), dev(offs), q, "MNC")
    assert i.shape == (len(sizes), q)
    got = i.cpu().numpy()
    for u in range(len(sizes)):
        exp = expected(ent[offs[u]:offs[u + 1]], q)
        assert np.array_equal(got[u][got[u] >= 0], exp), (u, q)
        assert (got[u][len(exp):] == -1).all()


@pytest.mark.parametrize("kind", QS)
@pytest.mark.parametrize("grouped", [True, False])
def test_frames_any_q(ce, kind, grouped):
    """select_from_frames (one pass for q <= 64; the per-song entropies beyond)
    against the restated groupby mean + oracle."""
    from oracle import ce_oracle as O
    from oracle.ce_oracle import ref_group_mean

    rng = np.random.default_rng(5 + grouped)
    F, C = 40_000, 4
    s_id = rng.integers(0, 3000, F) * 3 + 1
    if grouped:
        s_id = np.sort(s_id)
    frame_members = []
    for dt in (np.float64, np.float32):
        e = -np.log(rng.random((F, C)))
        frame_members.append((np.floor(e / e.sum(-1, keepdims=True) * 8) / 8 + 1e-3).astype(dt))
    n_songs = len(np.unique(s_id))
    cnn = (np.floor(rng.random((n_songs, C)) * 4) / 4 + 0.1).astype(np.float32)
    P = np.array([ref_group_mean(m, s_id)[0] for m in frame_members] + [cnn])
    ent = O.oracle_committee_entropy(P, "MNC")
    q = qval(kind, n_songs)
    got, _ = ce.select_from_frames(frame_members + [cnn], s_id, q)
    assert np.array_equal(got, expected(ent, q))


@pytest.mark.parametrize("q", [65, 2049])
def test_chunked_job_any_q(ce, q):
    """MCChunkJob: >= 5 chunks into a running list of q records (list merges
    for q <= CE_MAX_Q, the sort path + a rank merge above), chunks handed in
    out of order too, ties across every boundary."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(q)
    N, chunk = 50_000, 9_000
    e = -np.log(rng.random((N, 16, 4)))
    P = (np.floor(e / e.sum(-1, keepdims=True) * 16) / 16).astype(np.float32)
    for b in range(chunk, N, chunk):
        P[b - 2:b + 2] = 0.25
    ent = O.oracle_committee_entropy(P, "NMC")
    Pd = dev(P)
    job = ce.ops.MCChunkJob(q, "NMC")
    for lo in range(0, N, chunk):
        job.add(Pd[lo:lo + chunk])
    _, i = job.result()
    assert np.array_equal(idx_np(i), expected(ent, q))
    _, i = ce.ops.select_mc_chunks([(Pd[lo:lo + chunk], lo) for lo in range(0, N, chunk)][::-1], q, "NMC")
    assert np.array_equal(idx_np(i), expected(ent, q))


@pytest.mark.parametrize("q", [65, 2049])
@pytest.mark.parametrize("world", [2, 3])
def test_record_exchange_any_q(ce, q, world):
    """The multi-GPU exchange on one device at q > 64: each 'rank' writes q
    candidate records of its shard (ce_select_mc_cands), the records are
    concatenated rank-major as the all-gather leaves them, ce_merge_cands
    merges them (list merge, or the rank merge above CE_MAX_Q); the (val, idx)
    lists of ce_topq_merge too."""
    from ce_amd import dist as cdist
    from oracle import ce_oracle as O

    rng = np.random.default_rng(world * q)
    N = 40_001
    e = -np.log(rng.random((N, 16, 4)))
    P = (np.floor(e / e.sum(-1, keepdims=True) * 16) / 16).astype(np.float32)
    ent = O.oracle_committee_entropy(P, "NMC")
    Pd = dev(P)
    recs, vals, idxs = [], [], []
    for r in range(world):
        lo, hi = cdist.shard_range(N, r, world)
        recs.append(ce.ops.MCPlan(Pd[lo:hi], q, "NMC", base_idx=lo).step_cands())
        v, i = ce.ops.select_mc(Pd[lo:hi], q, "NMC", base_idx=lo)
        vals.append(v)
        idxs.append(i)
    _, i = ce.ops.merge_cands(torch.cat(recs), q)
    assert np.array_equal(idx_np(i), expected(ent, q))
    _, i = ce.ops.topq_merge(torch.cat(vals), torch.cat(idxs), q)
    assert np.array_equal(idx_np(i), expected(ent, q))


@pytest.mark.parametrize("mode", ["mc", "mix"])
@pytest.mark.parametrize("q", [65, 2049])
def test_session_any_q(ce, mode, q):
    """SelectionSession at q > 64, epoch after epoch, against the reference's
    shrinking-pool loop (amg_test.py:455, :484, :521-531)."""
    from oracle import ce_oracle as O

    rng = np.random.default_rng(q + len(mode))
    N, epochs = 3000, 3
    committees = [committee(rng, N, quant=64) for _ in range(epochs)]
    hc = np.round(rng.dirichlet(np.ones(4), N), 2)
    alive = np.ones(N, bool)
    sess = ce.SelectionSession(q, mode, N, hc=hc if mode == "mix" else None)
    for e in range(epochs):
        pos = np.flatnonzero(alive)
        ent = O.oracle_committee_entropy(committees[e][:, pos], "MNC")
        if mode == "mix":
            ent = np.concatenate([ent, O.oracle_table_entropy(hc[pos])])
        i = expected(ent, q)
        n = len(pos)
        exp = np.where(i < n, pos[np.minimum(i, n - 1)], N + pos[np.maximum(i - n, 0)]) if mode == "mix" else pos[i]
        got = sess.select(committee=dev(committees[e]))
        assert np.array_equal(got, exp), (mode, e)
        alive[np.where(exp >= N, exp - N, exp)] = False
    assert sess.remaining == alive.sum()
