"""The N>1 path on CPU: world_size-2 gloo process groups run the real sharding,
packing and all-gather code of ce_amd.dist; the per-rank selection and the
merge are the oracle's (no GPU here).  The sharded answer must equal the
single-process global top-q."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ce_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_local(P, q, base):
    v, i = O.oracle_select_mc(P.numpy(), q, layout="NMC")
    vals = np.full(q, np.nan)
    idx = np.full(q, -1, np.int64)
    vals[:len(v)] = v
    idx[:len(i)] = i + base
    return torch.from_numpy(vals), torch.from_numpy(idx)


def _oracle_merge(vals, idx, q):
    v, i = O.oracle_topq_merge(vals.numpy(), idx.numpy(), q)
    return torch.from_numpy(v), torch.from_numpy(i)


def _order_key(h):
    """The engine's order key (ce_device.hpp order_key) restated in numpy for
    the record-exchange test: NaN -> max, -0.0 -> +0.0, monotone in the order."""
    h = np.asarray(h, np.float64) + 0.0
    b = h.view(np.uint64)
    k = np.where(b >> np.uint64(63), ~b, b | np.uint64(1 << 63))
    return np.where(np.isnan(h), np.uint64(0xFFFFFFFFFFFFFFFF), k)


def _key_to_val(k):
    k = np.asarray(k, np.uint64)
    b = np.where(k >> np.uint64(63), k & np.uint64(0x7FFFFFFFFFFFFFFF), ~k)
    v = b.view(np.float64).copy()
    v[k == np.uint64(0xFFFFFFFFFFFFFFFF)] = np.nan
    return v


def _oracle_local_records(P, q, base):
    v, i = _oracle_local(P, q, base)
    rec = np.zeros((q, 2), np.int64)
    ok = i.numpy() >= 0
    rec[:, 0] = np.where(ok, _order_key(v.numpy()), 0).view(np.int64)
    rec[:, 1] = i.numpy()
    return torch.from_numpy(rec)


def _oracle_merge_records(rec, q):
    r = rec.numpy()
    vals = _key_to_val(r[:, 0].view(np.uint64))
    return _oracle_merge(torch.from_numpy(vals), torch.from_numpy(r[:, 1].copy()), q)


def _worker_records(rank, world, port, N, q, seed, out):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "consensus-entropy_amd"))
    from ce_amd import dist as cdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P = _pool(N, seed)
    lo, hi = cdist.shard_range(N, rank, world)
    v, i = cdist.sharded_select_mc_records(torch.from_numpy(P[lo:hi]), q, global_offset=lo,
                                           local_records=_oracle_local_records,
                                           merge_records=_oracle_merge_records)
    out[rank] = (v.numpy().tolist(), i.numpy().tolist())
    dist.destroy_process_group()


def _pool(N, seed):
    rng = np.random.default_rng(seed)
    e = -np.log(rng.random((N, 8, 4)))
    P = (e / e.sum(-1, keepdims=True)).astype(np.float32)
    P[::50] = np.floor(P[::50] * 4) / 4  # ties across shard boundaries
    return P


@pytest.mark.parametrize("world,N,q", [(2, 5000, 10), (2, 7, 10), (3, 4001, 25), (2, 5000, 65), (3, 3001, 2049)])
def test_sharded_records_equal_global(world, N, q):
    """The record exchange (ce_cand all-gather, rank-major receive buffer)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_records, args=(world, _free_port(), N, q, 7, out), nprocs=world, join=True)
    vg, ig = O.oracle_select_mc(_pool(N, 7), q, layout="NMC")
    for r in range(world):
        v, i = out[r]
        assert list(i)[:len(ig)] == ig.tolist()
        assert all(x == -1 for x in list(i)[len(ig):])


def _worker_dead_rank(rank, world, port, out):
    import sys
    import time

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "consensus-entropy_amd"))
    from ce_amd import dist as cdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    cdist.init("gloo", timeout_s=5)
    if rank == 1:  # this rank dies before the exchange (no destroy: it just vanishes)
        os._exit(0)
    rec = torch.zeros((10, 2), dtype=torch.int64)
    t0 = time.time()
    try:
        cdist.allgather_cands(rec)
        out[rank] = ("no error", time.time() - t0)
    except Exception as e:  # noqa: BLE001 -- any failure is the point
        out[rank] = (type(e).__name__, time.time() - t0)


def test_dead_rank_fails_fast():
    """SURVEY.md section 5 fail-fast: with ce_amd.dist.init's timeout a survivor's
    collective raises instead of hanging on a rank that died (torch's default
    would wait 10 minutes)."""
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker_dead_rank, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode is not None for p in procs), "a rank hung"
    err, dt = out[0]
    assert err != "no error" and dt < 60, (err, dt)


def test_order_key_roundtrip():
    h = np.array([np.nan, 1.5, -0.0, 0.0, -np.inf, np.inf, 1e-300, -2.0])
    k = _order_key(h)
    back = _key_to_val(k)
    assert np.array_equal(np.isnan(back), np.isnan(h))
    assert np.array_equal(back[~np.isnan(h)], (h + 0.0)[~np.isnan(h)])
    fin = ~np.isnan(h)
    order = np.argsort(k[fin])
    assert np.all(np.diff((h[fin] + 0.0)[order]) >= 0)


def _worker(rank, world, port, N, q, seed, out):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "consensus-entropy_amd"))
    from ce_amd import dist as cdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(seed)
    e = -np.log(rng.random((N, 8, 4)))
    P = (e / e.sum(-1, keepdims=True)).astype(np.float32)
    P[::50] = np.floor(P[::50] * 4) / 4  # ties across shard boundaries
    lo, hi = cdist.shard_range(N, rank, world)
    v, i = cdist.sharded_select_mc(torch.from_numpy(P[lo:hi]), q, global_offset=lo,
                                   local_select=_oracle_local, merge=_oracle_merge)
    out[rank] = (v.numpy().tolist(), i.numpy().tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,N,q", [(2, 5000, 10), (2, 7, 10), (3, 4001, 25), (2, 5000, 65)])
def test_sharded_equals_global(world, N, q):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), N, q, 1987, out), nprocs=world, join=True)
    rng = np.random.default_rng(1987)
    e = -np.log(rng.random((N, 8, 4)))
    P = (e / e.sum(-1, keepdims=True)).astype(np.float32)
    P[::50] = np.floor(P[::50] * 4) / 4
    vg, ig = O.oracle_select_mc(P, q, layout="NMC")
    for r in range(world):
        v, i = out[r]
        assert list(i)[:len(ig)] == ig.tolist()
        assert all(x == -1 for x in list(i)[len(ig):])


def test_shard_range_covers():
    from ce_amd.dist import shard_range

    for n in (0, 1, 7, 100, 100_000_001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[k][1] == spans[k + 1][0] for k in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_pack_roundtrip():
    from ce_amd.dist import pack, unpack

    v = torch.tensor([np.nan, 1.5, -0.0, 0.25], dtype=torch.float64)
    i = torch.tensor([3, 1, -1, 9], dtype=torch.int64)
    buf = torch.cat([pack(v, i), pack(v * 2, i + 100)])
    vv, ii = unpack(buf, 4, 2)
    assert torch.equal(ii, torch.cat([i, i + 100]))
    assert torch.allclose(vv, torch.cat([v, v * 2]), equal_nan=True)


class _OracleChunkJob:
    """MCChunkJob's contract restated with the oracle: a running list of q
    records folded with each chunk's top-q (the CPU stand-in for the HIP job)."""

    def __init__(self, q):
        self.q = q
        self.rec = None

    def add(self, P, base):
        r = _oracle_local_records(P, self.q, base)
        if self.rec is not None:
            v, i = _oracle_merge_records(torch.cat([self.rec, r]), self.q)
            r = torch.from_numpy(np.stack([np.where(i.numpy() >= 0, _order_key(v.numpy()), 0).view(np.int64)
                                           if len(i) else np.zeros(0, np.int64), i.numpy()], 1))
            pad = self.q - r.shape[0]
            if pad:
                r = torch.cat([r, torch.tensor([[0, -1]] * pad, dtype=torch.int64)])
        self.rec = r

    def running_records(self):
        if self.rec is None:
            return torch.tensor([[0, -1]] * self.q, dtype=torch.int64)
        return self.rec


def _worker_chunks(rank, world, port, N, chunk, q, seed, out):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "consensus-entropy_amd"))
    from ce_amd import dist as cdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P = _pool(N, seed)
    mine = [(torch.from_numpy(P[lo:lo + chunk]), lo) for c, lo in enumerate(range(0, N, chunk)) if c % world == rank]
    v, i = cdist.sharded_select_mc_chunks(mine, q, job=_OracleChunkJob(q), merge_records=_oracle_merge_records)
    out[rank] = (v.numpy().tolist(), i.numpy().tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,N,chunk,q", [(2, 9000, 1000, 10), (3, 2500, 1000, 16), (3, 2000, 1000, 10),
                                             (2, 9000, 1000, 65)])
def test_sharded_chunks_equal_global(world, N, chunk, q):
    """Pools larger than HBM over several GPUs: chunk c streams on rank
    c % world into that rank's running list; one all-gather of the running
    lists + a merge equals the global selection (a rank may get no chunk)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_chunks, args=(world, _free_port(), N, chunk, q, 11, out), nprocs=world, join=True)
    vg, ig = O.oracle_select_mc(_pool(N, 11), q, layout="NMC")
    for r in range(world):
        v, i = out[r]
        assert list(i)[:len(ig)] == ig.tolist()


def _mix_inputs(N, Nh, seed):
    rng = np.random.default_rng(seed)
    e = -np.log(rng.random((4, N, 4)))
    P = e / e.sum(-1, keepdims=True)
    P[:, ::7] = np.floor(P[:, ::7] * 8) / 8  # exact ties inside and across shards
    votes = rng.integers(0, 4, size=(Nh, 12))
    hc = np.stack([np.round((votes == c).sum(1) / 12, 3) for c in range(4)], 1)  # tie-heavy, amg_test.py:115
    return P, hc


def _oracle_local_any(P, q, base, layout="MNC"):
    v, i = O.oracle_select_mc(P.numpy(), q, layout=layout)
    vals = np.full(q, np.nan)
    idx = np.full(q, -1, np.int64)
    vals[:len(v)] = v
    idx[:len(i)] = i + base
    return torch.from_numpy(vals), torch.from_numpy(idx)


def _worker_mix(rank, world, port, N, Nh, q, seed, out):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "consensus-entropy_amd"))
    from ce_amd import dist as cdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, hc = _mix_inputs(N, Nh, seed)
    lo, hi = cdist.shard_range(N, rank, world)
    lh, hh = cdist.shard_range(Nh, rank, world)
    v, i = cdist.sharded_select_mix(torch.from_numpy(P[:, lo:hi]), torch.from_numpy(hc[lh:hh]), q, n_items=N,
                                    item_offset=lo, row_offset=lh, local_select=_oracle_local_any,
                                    merge=_oracle_merge)
    out[rank] = i.numpy().tolist()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,N,Nh,q", [(2, 1608, 1608, 10), (3, 500, 97, 16), (2, 5, 3, 10), (2, 1608, 1608, 65)])
def test_sharded_mix_equals_global(world, N, Nh, q):
    """mix (amg_test.py:473-480) sharded over the concatenated [mc; hc] index
    space: the merged answer is the single-process mix, hc positions >= N."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_mix, args=(world, _free_port(), N, Nh, q, 5, out), nprocs=world, join=True)
    P, hc = _mix_inputs(N, Nh, 5)
    _, ig = O.oracle_select_mix(P, hc, q)
    for r in range(world):
        got = out[r]
        assert got[:len(ig)] == ig.tolist()
        assert all(x == -1 for x in got[len(ig):])


def _batched_inputs(U, seed):
    rng = np.random.default_rng(seed)
    n = rng.integers(1, 300, size=U)
    n[0] = 11
    offs = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    e = -np.log(rng.random((4, int(offs[-1]), 4)))
    P = (e / e.sum(-1, keepdims=True)).astype(np.float32)
    P[:, ::9] = np.floor(P[:, ::9] * 4) / 4
    return P, offs


def _oracle_batched(P, offs, q):
    Pn, o = P.numpy(), offs.numpy()
    vals = np.full((len(o) - 1, q), np.nan)
    idx = np.full((len(o) - 1, q), -1, np.int64)
    for u in range(len(o) - 1):
        v, i = O.oracle_select_mc(np.ascontiguousarray(Pn[:, o[u]:o[u + 1]]), q)
        vals[u, :len(v)] = v
        idx[u, :len(i)] = i
    return torch.from_numpy(vals), torch.from_numpy(idx)


def _worker_batched(rank, world, port, U, q, seed, out):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "consensus-entropy_amd"))
    from ce_amd import dist as cdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, offs = _batched_inputs(U, seed)
    ulo, uhi = cdist.shard_range(U, rank, world)
    a, b = offs[ulo], offs[uhi]
    v, i = cdist.sharded_select_batched(torch.from_numpy(np.ascontiguousarray(P[:, a:b])),
                                        torch.from_numpy(offs[ulo:uhi + 1] - a), q, n_users=U,
                                        local_select=_oracle_batched)
    out[rank] = (v.numpy().tolist(), i.numpy().tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,U,q", [(2, 37, 10), (3, 8, 5), (3, 2, 10), (2, 37, 65)])
def test_sharded_batched_equals_global(world, U, q):
    """Batched users sharded over ranks, one final gather: every rank holds
    the [U, q] answer of one launch over all users (a rank may hold none)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_batched, args=(world, _free_port(), U, q, 3, out), nprocs=world, join=True)
    P, offs = _batched_inputs(U, 3)
    vg, ig = _oracle_batched(torch.from_numpy(P), torch.from_numpy(offs), q)
    for r in range(world):
        v, i = out[r]
        assert np.array_equal(np.array(i), ig.numpy())
        assert np.array_equal(np.array(v), vg.numpy(), equal_nan=True)
