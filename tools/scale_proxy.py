"""Single-GPU proxies for the 1/2/4/8-GPU scaling of bench.py (BASELINE
configs[3]: the 100M x 16 x 4 fp32 pool, strong scaling) -- VERDICT r02 item 4.

On ONE MI355X it measures what one rank of an N-GPU run does per step:
  local(N)    the rank's selection kernel on its shard of 100M / N items
              (ops.MCPlan.step_cands: stage 1 with stage 2 folded in, writing
              the rank's q candidate records -- exactly bench.py's N > 1 path)
  merge(N)    ops.merge_cands over the N ranks' q records (the receive buffer)
  gather1     one RCCL all_gather_into_tensor of 16q bytes at world size 1
              (the communicator's fixed cost on this box; xGMI hops at N > 1
              are NOT measured here)
and prints a PREDICTED step time per N = local(N) + merge(N) + gather(N), with
gather(N) = gather1 + (N - 1) x hop_us (hop_us an assumed per-hop xGMI
latency, stated in the output), and the predicted speed-up vs N = 1.
Everything predicted is labelled so; the driver's SCALE run is the measurement.
  python tools/scale_proxy.py [--hop-us 8] > profiles/r03_scale_proxy.json"""
import argparse
import json
import os
import socket
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ce_amd.ops as ops  # noqa: E402
from bench import make_pool  # noqa: E402
from ce_amd import dist as cdist  # noqa: E402


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    st = torch.cuda.current_stream()
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) * 1e3 for a, b in ev]  # us
    return {"median_us": statistics.median(ts), "mean_us": statistics.mean(ts), "min_us": min(ts)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-items", type=int, default=100_000_000)
    ap.add_argument("--q", type=int, default=10)
    ap.add_argument("--hop-us", type=float, default=8.0, help="assumed xGMI latency per ring hop (not measured)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N, M, C, q = a.n_items, 16, 4, a.q
    out = {"what": "single-GPU proxies of one rank of bench.py at N GPUs (strong scaling of configs[3])",
           "local": {}, "merge": {}, "predicted": {}}
    P = make_pool(0, N, M, C, dev)
    for world in (1, 2, 4, 8):
        lo, hi = cdist.shard_range(N, 0, world)
        plan = ops.MCPlan(P[lo:hi], q, "NMC", base_idx=lo)
        rec = torch.empty((q, 2), dtype=torch.int64, device=dev)
        out["local"][world] = dict(timed(lambda: plan.step_cands(rec)), items=hi - lo,
                                   kernel="stage 1 + folded stage 2 -> records")
        recs = torch.cat([rec] * world)
        out["merge"][world] = timed(lambda: ops.merge_cands(recs, q), reps=50)
        del plan
    del P
    torch.cuda.empty_cache()
    os.environ.update(MASTER_ADDR="127.0.0.1", RANK="0", WORLD_SIZE="1")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    cdist.init("nccl", device=dev)
    send = torch.zeros((q, 2), dtype=torch.int64, device=dev)
    recv = torch.empty((q, 2), dtype=torch.int64, device=dev)
    g1 = timed(lambda: dist.all_gather_into_tensor(recv, send), reps=100)
    out["gather_world1"] = g1
    # the whole rank step at the 8-GPU shard (12.5M items) on the world-1 RCCL
    # group: eager (three launches from the host) vs one HIP graph per step
    # (ce_amd.dist.ShardedStep, what bench.py replays); overhead = step - local
    lo, hi = cdist.shard_range(N, 0, 8)
    P8 = make_pool(lo, hi, M, C, dev)
    sstep = cdist.ShardedStep(P8, q, global_offset=lo)
    loc = timed(lambda: sstep.plan.step_cands(sstep.send), reps=50)
    eager = timed(lambda: sstep.eager(), reps=50)
    sstep.capture()
    graph = timed(lambda: sstep(), reps=50)
    out["step_world1_at_8gpu_shard"] = {
        "items": hi - lo, "local_us": loc, "eager_step_us": eager, "graph_step_us": graph,
        "exchange_overhead_eager_us": eager["median_us"] - loc["median_us"],
        "exchange_overhead_graph_us": graph["median_us"] - loc["median_us"],
        "note": "world-1 RCCL: the all-gather is the communicator's local copy; xGMI hops at N > 1 not measured; "
                "bench.py runs the eager step (the HIP graph replay measured slower)"}
    del sstep, P8
    dist.destroy_process_group()
    # bench.py runs the step eagerly (the graph measured slower): predict with the eager overhead
    ovh = out["step_world1_at_8gpu_shard"]["exchange_overhead_eager_us"]
    base = None
    for world in (1, 2, 4, 8):
        # N > 1: the rank's kernel + the measured world-1 graph exchange overhead
        # (all-gather + merge inside the graph) + the assumed extra xGMI hops
        extra = 0.0 if world == 1 else ovh + (world - 1) * a.hop_us
        step = out["local"][world]["median_us"] + extra
        base = base or step
        out["predicted"][world] = {"step_us": step, "speedup_vs_1": base / step, "exchange_us": extra,
                                   "assumption": f"exchange = measured world-1 eager overhead ({ovh:.1f} us: RCCL "
                                                 f"all-gather + merge) + {a.hop_us} us per extra hop "
                                                 "(hop latency assumed, not measured)"}
    out["target"] = ">= 6x at 8 GPUs (BASELINE.json north_star)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
