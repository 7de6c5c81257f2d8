"""The RCCL exchange itself on one GPU: a world-size-1 "nccl" process group
(RCCL on ROCm) runs sharded_select_mc_records / allgather_cands end to end --
stage 1, stage 2 into ce_cand records, the RCCL all-gather, ce_merge_cands --
and must equal the single-call selection.  (N > 1 ranks need N GPUs; their
exchange logic is covered by tests/test_dist.py on gloo.)"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_record_exchange_world1():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.distributed as dist

    import ce_amd
    from ce_amd import dist as cdist
    from ce_amd import ops
    from oracle import ce_oracle as O

    ce_amd.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        rng = np.random.default_rng(4)
        e = -np.log(rng.random((200_003, 16, 4)))
        P = (e / e.sum(-1, keepdims=True)).astype(np.float32)
        Pd = torch.from_numpy(P).cuda()
        plan = ops.MCPlan(Pd, 10, "NMC")
        plan.partial()
        rec = plan.finish_cands()
        recv = cdist.allgather_cands(rec)
        assert torch.equal(recv, rec)
        vals, idx = ops.merge_cands(recv, 10)
        exp = O.oracle_select_mc(P, 10, "NMC")[1]
        assert np.array_equal(idx.cpu().numpy(), exp)
        # the packed (entropy, position) exchange too
        v2, i2 = plan.finish()
        av, ai = cdist.allgather_topq(v2, i2, 10)
        v3, i3 = ops.topq_merge(av, ai, 10)
        assert np.array_equal(i3.cpu().numpy(), exp)
        # pools larger than HBM: this rank's chunks -> running list -> RCCL all-gather -> merge
        chunks = [(Pd[lo:lo + 40_000], lo) for lo in range(0, P.shape[0], 40_000)]
        _, i4 = cdist.sharded_select_mc_chunks(chunks, 10)
        assert np.array_equal(i4.cpu().numpy(), exp)
    finally:
        dist.destroy_process_group()


def test_rccl_step_graph_world1():
    """bench.py's N > 1 step (ce_amd.dist.ShardedStep: stage 1 with stage 2
    folded into this rank's records, the RCCL all-gather, the merge) on a
    world-1 RCCL group, eager and captured as a HIP graph: every replay equals
    the eager step and the oracle, also after the pool changes in place."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.distributed as dist

    import ce_amd
    from ce_amd import dist as cdist
    from oracle import ce_oracle as O

    ce_amd.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        rng = np.random.default_rng(6)
        e = -np.log(rng.random((300_007, 16, 4)))
        P = (e / e.sum(-1, keepdims=True)).astype(np.float32)
        Pd = torch.from_numpy(P).cuda()
        step = cdist.ShardedStep(Pd, 10, global_offset=5)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        v0, i0 = step(ev)
        torch.cuda.synchronize()
        assert ev[0].elapsed_time(ev[1]) > 0
        exp = O.oracle_select_mc(P, 10, "NMC")[1] + 5
        assert np.array_equal(i0.cpu().numpy(), exp)
        v0, i0 = v0.clone(), i0.clone()
        assert step.capture()
        for _ in range(4):
            v, i = step()
            torch.cuda.synchronize()
            assert torch.equal(i, i0) and torch.equal(v.view(torch.int64), v0.view(torch.int64))
        e2 = -np.log(rng.random(P.shape))
        P2 = (e2 / e2.sum(-1, keepdims=True)).astype(np.float32)
        Pd.copy_(torch.from_numpy(P2))
        _, i2 = step()
        torch.cuda.synchronize()
        assert np.array_equal(i2.cpu().numpy(), O.oracle_select_mc(P2, 10, "NMC")[1] + 5)
    finally:
        dist.destroy_process_group()


def test_bench_contract_small():
    """bench.py's JSON line (the driver's contract) on a small pool: the
    required keys, roofline / cpu_baseline objects, and a selection that
    equals the oracle's on the same synthetic pool."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--n-items", "2000000", "--steps", "3",
                        "--warmup", "1", "--cpu-sample", "200000"], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 3 and line["value"] > 0
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1.2
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] in ("port", "reference")
    assert len(line["selected"]) == 10
    assert line["ranks"] == 1 and line["selected_equal_n1"] is True
    assert line["selected_check"]["n1_rechecked"] is True and line["selected_check"]["n1_record"] is None
    assert cb["kind"] == "reference"


def test_rccl_sharded_mix_and_batched_world1():
    """sharded_select_mix / sharded_select_batched through the HIP kernels and
    an RCCL world-1 group: equal to ops.select_mix / ops.select_batched and
    to the oracle (the N > 1 exchange is covered on gloo)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.distributed as dist

    import ce_amd
    from ce_amd import dist as cdist
    from ce_amd import ops
    from oracle import ce_oracle as O

    ce_amd.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        rng = np.random.default_rng(8)
        e = -np.log(rng.random((4, 1608, 4)))
        P = e / e.sum(-1, keepdims=True)
        P[:, ::5] = np.floor(P[:, ::5] * 8) / 8
        votes = rng.integers(0, 4, size=(1608, 20))
        hc = np.stack([np.round((votes == c).sum(1) / 20, 3) for c in range(4)], 1)
        Pd, hd = torch.from_numpy(P).cuda(), torch.from_numpy(hc).cuda()
        _, i1 = cdist.sharded_select_mix(Pd, hd, 10, n_items=1608, item_offset=0, row_offset=0)
        _, i2 = ops.select_mix(Pd, hd, 10)
        exp = O.oracle_select_mix(P, hc, 10)[1]
        assert np.array_equal(i1.cpu().numpy(), exp) and np.array_equal(i2.cpu().numpy(), exp)
        n = rng.integers(100, 1608, size=40)
        offs = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
        e = -np.log(rng.random((4, int(offs[-1]), 4)))
        Pb = (e / e.sum(-1, keepdims=True)).astype(np.float32)
        Pbd, od = torch.from_numpy(Pb).cuda(), torch.from_numpy(offs).cuda()
        v3, i3 = cdist.sharded_select_batched(Pbd, od, 10, n_users=40)
        v4, i4 = ops.select_batched(Pbd, od, 10)
        assert torch.equal(i3, i4) and torch.equal(v3.view(torch.int64), v4.view(torch.int64))
        for u in range(40):
            eu = O.oracle_select_mc(np.ascontiguousarray(Pb[:, offs[u]:offs[u + 1]]), 10)[1]
            assert np.array_equal(i3[u].cpu().numpy(), eu)
    finally:
        dist.destroy_process_group()


def test_bench_world2_rehearsal():
    """bench.py's multi-GPU path end to end (shard generation, stage 1, stage 2
    into ce_cand records, the all-gather, the merge, max-over-ranks timing, the
    JSON line) with two ranks sharing the one GPU over gloo
    (CE_AMD_REHEARSAL=1): it must select what the single-process run selects
    on the same pool.  The real N-GPU run (RCCL, one rank per GPU) is the
    driver's."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    args = ["bench.py", "--steps", "3", "--warmup", "1", "--n-items", "3000001", "--no-cpu-baseline"]
    one = subprocess.run([sys.executable] + args, cwd=root, capture_output=True, text=True, timeout=600, env=env)
    assert one.returncode == 0, one.stderr[-2000:]
    env2 = dict(env, CE_AMD_REHEARSAL="1")
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args[:1] +
                         ["--gpus", "2"] + args[1:], cwd=root, capture_output=True, text=True, timeout=600, env=env2)
    assert two.returncode == 0, two.stderr[-2000:]
    l1 = json.loads(one.stdout.strip().splitlines()[-1])
    l2 = json.loads(two.stdout.strip().splitlines()[-1])
    assert l2["n_gpus"] == 2 and l2["config"]["items_per_gpu"] == 1500001
    assert l2["rehearsal"]["backend"] == "gloo" and l2["value"] is None  # never a valid-looking multi-GPU figure
    assert "rehearsal" not in l1 and l1["value"] > 0
    assert l1["selected"] == l2["selected"] and len(l1["selected"]) == 10
    assert l2["ranks"] == 2 and l2["backend"] == "gloo" and l2["selected_equal_n1"] is True
    assert l1["ranks"] == 1 and l1["backend"] is None and l1["selected_equal_n1"] is True
    # the same without torchrun: a plain `bench.py --gpus 2` starts both ranks itself
    three = subprocess.run([sys.executable] + args[:1] + ["--gpus", "2"] + args[1:], cwd=root, capture_output=True,
                           text=True, timeout=600, env=env2)
    assert three.returncode == 0, three.stderr[-2000:]
    lines = [ln for ln in three.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0's line only
    l3 = json.loads(lines[0])
    assert l3["n_gpus"] == 2 and l3["ranks"] == 2 and l3["config"]["items_per_gpu"] == 1500001
    assert l3["selected"] == l1["selected"] and l3["selected_equal_n1"] is True
    assert l3["selected_check"]["n1_rechecked"] is True and l3["value"] is None
