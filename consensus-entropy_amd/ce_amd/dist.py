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


class ShardedStep:
    """One rank's step of the sharded mc selection, as bench.py runs it every
    step: stage 1 with stage 2 folded in (ONE kernel writing this rank's q
    records into the all-gather send buffer), the all-gather of every rank's
    records, and the merge of the receive buffer.

    The step runs eagerly: the host enqueues the all-gather and the merge while
    the stage-1 kernel runs, so on the GPU they follow it within ~5 us at the
    8-GPU shard size (profiles/r05_scale_proxy.json, world-1 RCCL).  capture()
    records the step as one HIP graph instead (RCCL collectives are
    graph-capturable; gloo's are not: it declines on any other backend); it is
    kept as an option and tested, but measured SLOWER on MI355X -- a replay
    added ~24 us over the kernel against the eager step's ~5 us -- so bench.py
    does not use it.

    Output: (vals [q], idx [q]) tensors (the graph's outputs when captured,
    overwritten by every replay)."""

    def __init__(self, P_local, q, *, global_offset, layout="NMC", group=None):
        if not 1 <= int(q) <= 64:
            raise ValueError("ShardedStep takes 1 <= q <= 64 (the one-launch record path); "
                             "use sharded_select_mc for larger q")
        self.q = int(q)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.plan = ops.MCPlan(P_local, self.q, layout, base_idx=int(global_offset))
        self.device = P_local.device
        self.send = torch.empty((self.q, 2), dtype=torch.int64, device=self.device)
        self.recv = torch.empty((self.world * self.q, 2), dtype=torch.int64, device=self.device)
        self.graph = None
        self.out = None

    def eager(self, ev=None):
        """The step without a graph; ev = (e0, e1) HIP events around the stage-1 kernel."""
        if ev is not None:
            ev[0].record()
        self.plan.step_cands(self.send)
        if ev is not None:
            ev[1].record()
        if self.world > 1:
            dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
            return ops.merge_cands(self.recv, self.q)
        return ops.merge_cands(self.send, self.q)

    def capture(self, warmup=2):
        """Capture the step as one HIP graph, after `warmup` eager steps on a
        side stream (torch's capture rules).  Returns False -- the step stays
        eager -- when the backend's collective cannot be captured."""
        if self.world > 1 and dist.get_backend(self.group) != "nccl":
            return False
        cur = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.eager()
        cur.wait_stream(s)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.out = self.eager()
        self.graph = g
        return True

    def __call__(self, ev=None):
        if self.graph is not None:
            self.graph.replay()
            return self.out
        return self.eager(ev)


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
