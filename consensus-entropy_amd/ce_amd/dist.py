"""Multi-GPU selection: the pool's N axis sharded over ranks (one process per GPU).

Each rank scores its contiguous shard [lo, hi) of the pool with the fused
kernel (positions reported globally: base_idx = lo), the ranks exchange their
local top-q with ONE all-gather of q x (f64 entropy, i64 position) = 16q bytes
per rank (RCCL over xGMI when the backend is "nccl"; latency-bound at q = 10),
and every rank runs the same deterministic merge.  Exact: the global top-q is a
subset of the union of the local top-qs, and the merge uses the same total
order (NaN first, entropy descending, lowest position).

Two exchange formats: (f64 entropy, i64 position) pairs packed into one i64
tensor, or -- what bench.py uses -- the engine's 16-byte
candidate records (ce_cand), written by stage 2 straight into the all-gather
send buffer and merged from the receive buffer as is (no pack/unpack kernels).
The local-select and merge steps are injectable so the collective logic can be
exercised on CPU with the gloo backend (tests/test_dist.py); by default they
are the HIP operators.

Validation status: every sharded path is tested against the CPU restatement on the gloo
backend at world 2 and 3 (tests/test_dist.py) and through the HIP kernels with
RCCL at world 1 (tests/test_gpu_dist.py); RCCL with more than one rank runs
only in the driver's multi-GPU bench (bench.py), so multi-rank exactness is
validated on gloo.

The other sharded configs of SURVEY.md §8(e): the mix stack [mc; hc] sharded
over its concatenated index space (sharded_select_mix), batched users sharded
over ranks with only a final gather (sharded_select_batched), and pools larger
than HBM streamed per rank (sharded_select_mc_chunks).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from . import ops

DEFAULT_TIMEOUT_S = 120.0


def init(backend="nccl", *, device=None, timeout_s=None):
    """Join the process group (one process per GPU; RANK / WORLD_SIZE /
    MASTER_* from the environment, as torchrun sets them) with FAIL-FAST
    error handling: every collective, the rendezvous included,
    gives up after ``timeout_s`` (default CE_AMD_DIST_TIMEOUT_S or 120 s;
    torch's own default is 10 minutes), and on the RCCL backend a failed or
    timed-out collective tears the process down (TORCH_NCCL_ASYNC_ERROR_HANDLING
    = 1) instead of leaving the survivors blocked on a dead rank.  The selection
    exchanges 16q bytes per rank per step (microseconds), so any wait of that
    order means a lost rank."""
    if timeout_s is None:
        timeout_s = float(os.environ.get("CE_AMD_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = {"timeout": datetime.timedelta(seconds=float(timeout_s))}
    if device is not None and backend == "nccl":
        kw["device_id"] = torch.device(device)
    dist.init_process_group(backend, **kw)


def shard_range(n, rank, world):
    """Contiguous shard of n items for `rank` (sizes differ by at most 1)."""
    base, rem = divmod(int(n), int(world))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def pack(vals, idx):
    """(f64 [q], i64 [q]) -> one i64 [2q] tensor (f64 bits viewed as i64)."""
    return torch.cat([vals.contiguous().view(torch.int64), idx.contiguous()])


def unpack(buf, q, world):
    b = buf.view(world, 2 * q)
    return b[:, :q].contiguous().view(torch.float64).reshape(-1), b[:, q:].contiguous().reshape(-1)


def allgather_topq(vals, idx, q, group=None):
    """All-gather every rank's best-first (vals, idx) list: returns the
    concatenated [world*q] lists, rank-major."""
    world = dist.get_world_size(group)
    send = pack(vals, idx)
    recv = torch.empty(world * send.numel(), dtype=send.dtype, device=send.device)
    dist.all_gather_into_tensor(recv, send, group=group)
    return unpack(recv, q, world)


def allgather_cands(cands, group=None, out=None):
    """All-gather every rank's q candidate records (int64 [q, 2] = ce_cand
    {order key, position}, from MCPlan.finish_cands): returns [world*q, 2],
    rank-major -- one RCCL collective of 16q bytes per rank and no pack/unpack
    kernels; ops.merge_cands reads the receive buffer as is."""
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty((world * cands.shape[0], 2), dtype=cands.dtype, device=cands.device)
    dist.all_gather_into_tensor(out, cands.contiguous(), group=group)
    return out


def sharded_select_mc_records(P_local, q, *, global_offset, layout="NMC", group=None, local_records=None,
                              merge_records=None):
    """sharded_select_mc over the record exchange (any q): stage 1 + stage 2
    write this rank's q records straight into the all-gather send buffer, and
    the merge reads the receive buffer.

    local_records  f(P_local, q, base_idx) -> int64 [q, 2] records; default
                   the HIP selection in one launch (ops.MCPlan.step_cands)
    merge_records  f(records [world*q, 2], q) -> (vals, idx); default
                   ops.merge_cands (HIP)
    """
    if local_records is None:
        def local_records(P, qq, base):
            return ops.MCPlan(P, qq, layout, base_idx=base).step_cands()
    if merge_records is None:
        merge_records = ops.merge_cands
    rec = local_records(P_local, q, int(global_offset))
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        rec = allgather_cands(rec, group)
    return merge_records(rec, q)


def sharded_select_mc(P_local, q, *, global_offset, layout="NMC", group=None, local_select=None, merge=None):
    """Global top-q over the union of every rank's shard.

    P_local        this rank's committee shard (items [global_offset, +n))
    local_select   f(P_local, q, base_idx) -> (vals [q], idx [q]); default the
                   fused HIP kernel ops.select_mc
    merge          f(vals [world*q], idx [world*q], q) -> (vals, idx);
                   default ops.topq_merge (HIP)
    """
    if local_select is None:
        def local_select(P, qq, base):
            return ops.select_mc(P, qq, layout, base_idx=base)
    if merge is None:
        merge = ops.topq_merge
    vals, idx = local_select(P_local, q, int(global_offset))
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return vals, idx
    all_vals, all_idx = allgather_topq(vals, idx, q, group)
    return merge(all_vals, all_idx, q)


def sharded_select_mix(P_local, hc_local, q, *, n_items, item_offset, row_offset, layout="MNC", group=None,
                       local_select=None, merge=None):
    """The mix of amg_test.py:473-480 with the row stack [mc (N items); hc
    (N_h rows)] sharded over ranks ("mix shards the
    concatenated index space"): this rank holds committee items
    [item_offset, +n) and hc rows [row_offset, +n_h).  Its two local top-q
    lists carry global stack positions (item i -> i, row j -> n_items + j),
    ONE all-gather moves 2q (entropy, position) pairs per rank, and the merge
    over the 2*world lists equals ops.select_mix on the whole stack.

    local_select  f(P, q, base_idx) -> (vals [q], idx [q]) for a committee
                  (the hc rows are passed as a one-member f64 committee
                  [1, n_h, C], "MNC"); default the fused HIP kernel
    merge         f(vals, idx, q) -> (vals, idx); default ops.topq_merge
    """
    if local_select is None:
        def local_select(P, qq, base, lay=layout):
            return ops.select_mc(P, qq, lay, base_idx=base)
    if merge is None:
        merge = ops.topq_merge
    v_mc, i_mc = local_select(P_local, q, int(item_offset))
    hc1 = hc_local.to(torch.float64).unsqueeze(0)  # M = 1: the hc rows' entropy (amg_test.py:479)
    v_hc, i_hc = local_select(hc1, q, int(n_items) + int(row_offset), "MNC")
    vals, idx = torch.cat([v_mc, v_hc]), torch.cat([i_mc, i_hc])
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        vals, idx = allgather_topq(vals, idx, 2 * q, group)
    return merge(vals, idx, q)


def sharded_select_batched(P_local, offsets_local, q, *, n_users, layout="MNC", group=None, local_select=None):
    """Batched users (BASELINE configs[2], the per-user loop of amg_test.py:345)
    sharded over ranks with no collective but the final gather (SURVEY.md
    §8(e)): rank r holds users shard_range(n_users, r, world) -- their items
    in P_local, user u's at offsets_local[u]:offsets_local[u+1] -- selects
    them in one launch, and ONE all-gather of the padded [ceil(U/world), q]
    (entropy, position) blocks gives every rank the full (vals [U, q],
    idx [U, q]), user-local positions, as one select_batched over all users.

    local_select  f(P, offsets, q) -> (vals [U_r, q], idx [U_r, q]); default
                  ops.select_batched (HIP)
    """
    if local_select is None:
        def local_select(P, off, qq):
            return ops.select_batched(P, off, qq, layout)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = shard_range(n_users, rank, world)
    if offsets_local.numel() != hi - lo + 1:
        raise ValueError(f"rank {rank} holds users [{lo}, {hi}): offsets_local needs {hi - lo + 1} entries")
    if hi > lo:
        vals, idx = local_select(P_local, offsets_local, q)
    else:  # more ranks than users
        vals = torch.empty((0, q), dtype=torch.float64, device=offsets_local.device)
        idx = torch.empty((0, q), dtype=torch.int64, device=offsets_local.device)
    if world == 1:
        return vals, idx
    umax = -(-int(n_users) // world)
    send = torch.zeros((umax, 2 * q), dtype=torch.int64, device=vals.device)
    send[:hi - lo, :q] = vals.contiguous().view(torch.int64)
    send[:hi - lo, q:] = idx
    recv = torch.empty((world * umax, 2 * q), dtype=torch.int64, device=vals.device)
    dist.all_gather_into_tensor(recv, send, group=group)
    spans = [shard_range(n_users, r, world) for r in range(world)]
    rows = torch.cat([torch.arange(r * umax, r * umax + (b - a), device=vals.device)
                      for r, (a, b) in enumerate(spans)])
    out = recv.index_select(0, rows)
    return out[:, :q].contiguous().view(torch.float64), out[:, q:].contiguous()


def sharded_select_mc_chunks(chunks, q, *, layout="NMC", group=None, job=None, merge_records=None):
    """A pool larger than HBM (BASELINE configs[4]) over several GPUs: this
    rank streams ITS chunks -- ``chunks`` yields (device tensor, global
    base_idx) pairs, e.g. chunk c on rank c % world -- into a running top-q
    (ops.MCChunkJob, any q), then ONE all-gather of every rank's q running
    records and the same merge on every rank.  A rank with no chunk contributes
    an empty list.  ``job``/``merge_records`` are injectable for CPU tests."""
    if job is None:
        job = ops.MCChunkJob(q, layout)
    if merge_records is None:
        merge_records = ops.merge_cands
    for P, base in chunks:
        job.add(P, base)
    rec = job.running_records()
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        rec = allgather_cands(rec, group)
    return merge_records(rec, q)
