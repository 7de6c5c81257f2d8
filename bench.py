#!/usr/bin/env python3
"""Benchmark of the consensus-entropy selection path on MI355X.

Metric (BASELINE.json): pool items scored+ranked/sec (M=16, C=4), whole job.
Workload: BASELINE.json configs[3] -- a 100M-item pool x 16 members x 4 classes,
fp32 probabilities in the item-major [N, M, C] layout (25.6 GB), q = 10.  It
fits one MI355X (288 GB), so N=1 runs the whole pool on one GPU; with N GPUs
the SAME pool is sharded over the ranks (strong scaling, as the north star's
"6x at 8 GPUs on the 100M-item pool" asks) and the ranks exchange their local
top-q with one RCCL all-gather before an identical merge on every rank.

One step = the full selection: ONE kernel per rank -- fused score + per-block
top-q over the resident shard (the streaming stage 1) whose last block merges
the blocks' candidates (stage 2 folded in) -- and for N > 1 the all-gather of
every rank's q candidate records (16 B each) + the merge
(ce_amd.dist.ShardedStep).  Inputs are synthetic
Dirichlet(1) member rows (1% un-normalised, like sigmoid CNN members), seed
1987, generated on the device before timing.

Ranks: under torchrun (WORLD_SIZE set) this process is one rank.  A plain
`python3 bench.py --gpus N` (N > 1) starts the N ranks itself -- N fresh child
processes with torchrun's environment, started before the parent makes any GPU
call -- and exits with the worst rank's status; rank 0's line is the output.
A --gpus that disagrees with WORLD_SIZE, or more ranks than visible GPUs
(outside a CE_AMD_REHEARSAL=1 rehearsal), exits 2 without a line.

Also reported:
  ranks / backend  the process group's size and backend (None at N=1)
  selected_equal_n1  the merged selection equals the N=1 selection of the same
                pool: rank 0 re-selects the whole pool after the timed region
                on its GPU by the chunked single-GPU path (ops.MCChunkJob), and
                compares with the committed 1-GPU record (profiles/
                selected_n1.json) when there is one; a mismatch exits 3
  roofline      the selection kernel (stage 1 + folded stage 2): algorithmic
                bytes (N_local x 256 B) / its mean duration from HIP events on
                the launch stream, vs 8 TB/s;
                traffic = HBM bytes per launch from the committed rocprofv3 PMC
                pass (profiles/traffic.json) of the kernel this run launched
                (ce_last_kernel()), or null when that record names another
  cpu_baseline  the reference's own expressions (amg_test.py:441-445, numpy +
                scipy) on a bounded sample, rank 0 at N=1 only
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "consensus-entropy_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "pool items scored+ranked/sec (M=16,C=4) at 1/2/4/8 GPUs; % HBM roofline"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")
# what the stage-1 kernel each layout launches at M=16, C=4, f32, q <= 64 does
# (csrc/ce_launch_stream.hip); the exact symbol comes from ce_last_kernel()
STAGE1_ROLE = {
    "NMC": "item-major [N,M,C], LDS-DMA tiles; stage 2 folded into the last block",
    "MNC": "member-major [M,N,C], LDS-DMA tiles of one 1 KiB run per member; stage 2 folded",
}


def kernel_symbol(name):
    """rocprofv3's kernel name without the return type and argument list
    ("void ce::k<0, 4>(ce::StreamArgs, ...)" -> "ce::k<0, 4>"), the form
    ce_last_kernel() reports."""
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def recorded_traffic(key, launched):
    """HBM bytes per launch from profiles/traffic.json for this workload key,
    only when the profiled kernel is the one this run launched; else None and
    the reason."""
    try:
        with open(TRAFFIC_FILE) as f:
            entry = json.load(f).get(key)
    except (OSError, ValueError) as e:
        return None, f"no traffic record ({e!r})"
    if not entry:
        return None, f"no traffic record for {key}"
    if not launched or kernel_symbol(entry["kernel"]) != launched:
        return None, f"traffic record is for {kernel_symbol(entry['kernel'])}, this run launched {launched or '?'}"
    return entry["hbm_bytes_per_launch"], entry.get("source")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


POOL_CHUNK = 4_000_000


def make_pool(lo, hi, M, C, device, seed=1987):
    """Items [lo, hi) of the synthetic pool: Dirichlet(1) rows per (item,
    member), 1% of member rows scaled by U(0.5, 2).  Generated in fixed global
    chunks seeded by chunk number, so every world size sees the SAME pool and
    the selected positions must agree across N."""
    P = torch.empty((hi - lo, M, C), dtype=torch.float32, device=device)
    for c in range(lo // POOL_CHUNK, (hi + POOL_CHUNK - 1) // POOL_CHUNK):
        c0, c1 = c * POOL_CHUNK, (c + 1) * POOL_CHUNK
        g = torch.Generator(device=device).manual_seed(seed * 100_003 + c)
        e = -torch.log(torch.rand((POOL_CHUNK, M, C), device=device, generator=g).clamp_min_(1e-30))
        e /= e.sum(-1, keepdim=True)
        scale = torch.where(torch.rand((POOL_CHUNK, M, 1), device=device, generator=g) < 0.01,
                            torch.rand((POOL_CHUNK, M, 1), device=device, generator=g) * 1.5 + 0.5,
                            torch.ones((), device=device))
        e *= scale
        a, b = max(lo, c0), min(hi, c1)
        P[a - lo:b - lo] = e[a - c0:b - c0]
        del e, scale
    return P


def cpu_baseline(n_items, M, C, q, seed=1987):
    """amg_test.py:441-445 verbatim (numpy/scipy) on n_items; mixed member
    dtypes like the reference committee (GNB/SGD f64, XGB/CNN f32)."""
    import numpy as np

    from oracle.ce_oracle import ref_mc

    rng = np.random.default_rng(seed)
    members = []
    for m in range(M):
        e = -np.log(rng.random((n_items, C)))
        p = e / e.sum(-1, keepdims=True)
        members.append(p if m < M // 2 else p.astype(np.float32))
    ref_mc(members, q)  # warm-up
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        ref_mc(members, q)
        ts.append(time.perf_counter() - t0)
    t = statistics.median(ts)
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    multicore = None
    try:
        multicore = cpu_baseline_multicore(n_items, M, C, q, seed)
    except Exception as e:  # the single-core figure stands on its own
        log(f"multi-core CPU baseline skipped: {e!r}")
    return {
        "value": n_items / t,
        "unit": "items/s",
        "cores": 1,
        "kind": "reference",
        "multicore": multicore,
        "sample": (f"reference expressions amg_test.py:441-445 verbatim (np.mean(np.array(pred_prob),0), "
                   f"scipy.stats.entropy(axis=1), np.argsort()[::-1][:{q}]) on {n_items} items x {M} mixed "
                   f"f64/f32 members x {C} classes; median of 5 after 1 warm-up = {t:.3f} s; numpy "
                   f"single-threaded; host: {cpu}, {os.cpu_count()} logical cpus visible"),
    }


def cpu_baseline_multicore(n_items, M, C, q, seed=1987, procs=None):
    """The same expressions on `procs` host cores at once: one spawned
    single-threaded worker per core, each on its own shard (n_items // 4 items),
    throughput = all shards' items / the slowest worker's median time (the
    shards' top-q lists would merge exactly, as the GPU ranks' do)."""
    import multiprocessing as mp

    from oracle.ce_oracle import ref_mc_shard_time

    share = host_cpu_share()
    procs = procs or share["usable"]
    n = max(1, n_items // 4)
    env_old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"  # inherited by the spawned workers
    pool = None
    try:
        pool = mp.get_context("spawn").Pool(procs)
        res = pool.map(ref_mc_shard_time, [(n, M, C, q, seed + 1 + r, 3) for r in range(procs)])
        # close + join: the workers exit on their own (Pool.__exit__ would
        # terminate() them, and under rocprofv3 every SIGTERM'd worker prints
        # an abort-looking stack)
        pool.close()
        pool.join()
        pool = None
    finally:
        if pool is not None:  # an exception on the way: do not leave workers behind
            pool.terminate()
            pool.join()
        if env_old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = env_old
    t = max(r[0] for r in res)
    rate = sum(r[1] for r in res) / t
    out = {"value": rate, "unit": "items/s", "cores": procs,
           "sample": f"{procs} spawned single-threaded workers x {n} items each, median of 3 per worker",
           "host": share}
    if share["physical_cores"]:
        # the job's CPU share is `usable` cores; the whole machine's physical cores, at
        # the measured per-core rate (numpy here is per-core compute-bound), would give:
        out["extrapolated_all_physical_cores"] = {"value": rate / procs * share["physical_cores"],
                                                  "cores": share["physical_cores"], "kind": "linear extrapolation"}
    return out


def host_cpu_share():
    """CPUs this job may use: the affinity mask, the cgroup CPU quota, and the
    GPU pool's rule of 16 host CPUs per GPU; plus the machine's physical cores
    (sockets x cores per socket from /proc/cpuinfo) for the record."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    phys = set()
    try:
        pid = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                pid = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
                phys.add((pid, core))
    except OSError:
        pass
    usable = min(x for x in (affinity, quota or affinity, 16) if x)
    return {"usable": usable, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "logical_cpus": os.cpu_count(), "physical_cores": len(phys) or None,
            "rule": "GPU pool: 16 host CPUs per GPU job"}


class LaunchError(SystemExit):
    """A --gpus request bench.py must refuse (exit status 2, no JSON line)."""

    def __init__(self, msg):
        log(f"bench.py: {msg}")
        super().__init__(2)


def launch_plan(gpus, env, visible):
    """What bench.py does for `--gpus gpus` given the environment and the
    number of visible GPUs (torch.cuda.device_count(), which does not
    initialise the GPU on this image):
      ("run", world)   run this process as one rank of `world` (torchrun, or
                       the launcher's child, set WORLD_SIZE), or alone at N=1
      ("spawn", n)     start n ranks as child processes and wait for them
    Refuses (LaunchError): --gpus < 1, a --gpus that disagrees with an
    explicit WORLD_SIZE, or more ranks than visible GPUs outside a one-GPU
    rehearsal (CE_AMD_REHEARSAL=1) -- never a 1-GPU line for --gpus N."""
    if gpus < 1:
        raise LaunchError(f"--gpus {gpus} must be >= 1")
    rehearsal = env.get("CE_AMD_REHEARSAL") == "1"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise LaunchError(f"WORLD_SIZE={world} disagrees with --gpus {gpus}")
        if not rehearsal and world > 1 and world > visible:
            raise LaunchError(f"{world} ranks but {visible} visible GPU(s)")
        return ("run", world)
    if not rehearsal and gpus > 1 and gpus > visible:
        raise LaunchError(f"--gpus {gpus} but {visible} visible GPU(s) (CE_AMD_REHEARSAL=1 shares them over gloo)")
    return ("run", 1) if gpus == 1 else ("spawn", gpus)


def free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(env, rank, world, port):
    """The environment of child rank `rank` (what torchrun would set)."""
    out = dict(env)
    out.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    out.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL needs dmabuf IPC on this pool
    return out


def spawn_ranks(cmd, n, env=None, poll_s=0.2):
    """Run `cmd` as n ranks (fresh child processes, each with its rank's
    environment; the parent never touches the GPU) and return the worst exit
    status: the first failing rank's, 128 + signal for a killed one.  When one
    rank fails, the others get SIGTERM after a grace period (the fail-fast
    collective timeout would end them anyway).  Rank 0's stdout is the
    parent's stdout: the JSON line."""
    import signal
    import subprocess

    env = dict(os.environ if env is None else env)
    port = free_port()
    procs = [subprocess.Popen(cmd, env=rank_env(env, r, n, port)) for r in range(n)]
    rcs = [None] * n
    failed_at = None
    try:
        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None and p.poll() is not None:
                    rcs[r] = p.returncode
                    if p.returncode != 0 and failed_at is None:
                        failed_at = time.monotonic()
            if failed_at is not None and time.monotonic() - failed_at > 30:
                for r, p in enumerate(procs):
                    if rcs[r] is None:
                        p.send_signal(signal.SIGTERM)
                failed_at = float("inf")
            time.sleep(poll_s)
    finally:
        for r, p in enumerate(procs):
            if p.poll() is None:
                p.kill()
                p.wait()
    worst = 0
    for rc in rcs:
        rc = 128 - rc if rc is not None and rc < 0 else rc
        if rc and not worst:
            worst = rc
    return worst


SELECTED_FILE = os.path.join(ROOT, "profiles", "selected_n1.json")


def recorded_selection(key):
    """The committed N=1 selection of a workload (profiles/selected_n1.json:
    the driver's own 1-GPU line), or None."""
    try:
        with open(SELECTED_FILE) as f:
            return json.load(f).get(key)
    except (OSError, ValueError):
        return None


def n1_selection(N, M, C, q, layout, device):
    """The N=1 selection of the whole generated pool on THIS GPU by another
    code path: the pool regenerated chunk by chunk (make_pool's global
    chunks) in the OTHER stack layout and streamed through one running top-q
    (ops.MCChunkJob).  The other layout runs another stage-1 kernel, so the
    re-selection is independent of the timed kernel and adds no dispatch of
    its symbol to a rocprofv3 --stats summary of this command.  Outside the
    timed region; ~1 s at 100M items."""
    from ce_amd import ops

    other = "MNC" if layout == "NMC" else "NMC"
    job = ops.MCChunkJob(q, other, device)
    for lo in range(0, N, POOL_CHUNK):
        hi = min(N, lo + POOL_CHUNK)
        P = make_pool(lo, hi, M, C, device)
        if other == "MNC":
            P = P.permute(1, 0, 2).contiguous()
        job.add(P, lo)
        del P
    _, idx = job.result()
    return idx.cpu().tolist()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n-items", type=int, default=100_000_000)
    ap.add_argument("--members", type=int, default=16)
    ap.add_argument("--classes", type=int, default=4)
    ap.add_argument("--q", type=int, default=10)
    ap.add_argument("--layout", default="NMC", choices=["NMC", "MNC"])
    ap.add_argument("--cpu-sample", type=int, default=6_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-n1-check", action="store_true", help="skip the N=1 re-selection of the pool")
    args = ap.parse_args()

    # before ANY GPU call: a plain `python3 bench.py --gpus N` starts N ranks itself
    mode, world = launch_plan(args.gpus, os.environ, torch.cuda.device_count())
    if mode == "spawn":
        log(f"bench.py: starting {world} ranks (one process per GPU)")
        sys.exit(spawn_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], world))

    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    # CE_AMD_REHEARSAL=1: several ranks share the visible GPUs over gloo (a
    # one-GPU rehearsal of the multi-GPU code path; never used for a bench line)
    rehearsal = os.environ.get("CE_AMD_REHEARSAL") == "1"
    if rehearsal:
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    import ce_amd
    from ce_amd import dist as cdist
    from ce_amd import ops

    if world > 1:  # fail fast: a dead rank ends the job within the timeout (ce_amd.dist.init)
        cdist.init("gloo" if rehearsal else "nccl", device=device)

    ce_amd.load()
    N, M, C, q = args.n_items, args.members, args.classes, args.q
    lo, hi = cdist.shard_range(N, rank, world)
    n_local = hi - lo
    t0 = time.time()
    P = make_pool(lo, hi, M, C, device)
    if args.layout == "MNC":
        P = P.permute(1, 0, 2).contiguous()
    torch.cuda.synchronize()
    log(f"[rank {rank}] pool shard {n_local} x {M} x {C} fp32 ({P.numel() * 4 / 1e9:.1f} GB) "
        f"generated in {time.time() - t0:.1f}s")
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world == 1 or q > 64:
        plan = ops.MCPlan(P, q, args.layout, base_idx=lo)

        def step(k):
            """N = 1: ONE launch (stage 2 folded into the streaming stage 1's
            last block) -> the final (vals, idx).  N > 1 with q > 64: the rank's
            list, then the packed (entropy, position) exchange and merge."""
            if k >= 0:
                ev[k][0].record(stream)
            loc = plan.step()
            if k >= 0:
                ev[k][1].record(stream)
            if world == 1:
                return loc
            return ops.topq_merge(*cdist.allgather_topq(*loc, q), q)
    else:
        # N > 1: stage 1 (stage 2 folded in) writes this rank's q candidate
        # records (ce_cand, 16 B each) straight into the all-gather send buffer,
        # one RCCL all-gather, the merge of the receive buffer (eager: a HIP
        # graph of the step measured slower, ce_amd.dist.ShardedStep)
        sstep = cdist.ShardedStep(P, q, global_offset=lo, layout=args.layout)

        def step(k):
            return sstep(ev[k] if k >= 0 else None)

    for _ in range(args.warmup):
        step(-1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        vals, idx = step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    kern_ms = statistics.mean(a.elapsed_time(b) for a, b in ev)
    picks = idx.cpu().tolist()
    launched = ce_amd._lib.load().ce_last_kernel().decode()  # the stage-1 kernel of the last step
    backend = dist.get_backend() if world > 1 else None

    bytes_per_launch = n_local * M * C * P.element_size()
    # release the pool before the checks below (the N=1 re-selection and the
    # CPU baseline): only the selected positions are needed from here on
    del step, P
    plan = sstep = None  # noqa: F841
    torch.cuda.empty_cache()

    check = None
    if rank == 0:
        # the ranks' merged selection vs the N=1 selection of the same pool
        # (after the timed region): the committed 1-GPU record when there is
        # one for this workload, and a re-selection on this GPU by the chunked
        # single-GPU path
        rec = recorded_selection(f"{args.layout}_{N}_{M}_{C}_q{q}")
        n1 = None if args.no_n1_check else n1_selection(N, M, C, q, args.layout, device)
        check = {"n1_rechecked": None if n1 is None else n1 == picks,
                 "n1_record": None if rec is None else rec == picks,
                 "record": os.path.relpath(SELECTED_FILE, ROOT) if rec is not None else None,
                 "method": "rank 0 regenerated the whole pool in 4M-item chunks in the other stack layout "
                           f"({'MNC' if args.layout == 'NMC' else 'NMC'}: another stage-1 kernel) and streamed it "
                           "through ops.MCChunkJob (one GPU, one running top-q), after the timed region"}

    if rank == 0:
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = recorded_traffic(f"{args.layout}_{N}_{M}_{C}_q{q}_w{world}", launched)
        line = {
            "metric": METRIC,
            "value": N * args.steps / elapsed,
            "unit": "items/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": (f"configs[3] large-ensemble pool: {N} items x {M} members x {C} classes fp32, "
                             f"[N,M,C] layout={args.layout}, q={q}, sharded over {world} GPU(s)"),
                "n_items": N, "members": M, "classes": C, "q": q, "input_dtype": "f32",
                "layout": args.layout, "items_per_gpu": n_local,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": launched,
                "kernel_role": STAGE1_ROLE[args.layout],
                "kernel_ms": kern_ms,
                "algorithmic_bytes_per_launch": bytes_per_launch,
            },
            "cpu_baseline": None,
            "ranks": world,
            "backend": backend,
            "selected": picks,
            "selected_equal_n1": (None if check["n1_rechecked"] is None and check["n1_record"] is None
                                  else check["n1_rechecked"] is not False and check["n1_record"] is not False),
            "selected_check": check,
        }
        if rehearsal:  # ranks sharing one GPU over gloo: a code-path rehearsal, not a multi-GPU figure
            line["rehearsal"] = {"backend": "gloo", "gpus_visible": torch.cuda.device_count(),
                                 "note": "NOT a multi-GPU measurement"}
            line["value"] = None
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_sample, M, C, q)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and line["selected_equal_n1"] is False:
        log("bench.py: the selection differs from the N=1 selection of the same pool")
        sys.exit(3)


if __name__ == "__main__":
    main()
