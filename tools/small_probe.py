"""Plain (graph-free) launches of one small-pool config, for rocprofv3 kernel
traces and --pmc passes (one config per run, so every rocprof row is one
kernel on one shape):
  c1    configs[0]  mc 4 x 1608 x 4 f64 (reference-sized pool)
  c2hc  configs[1]  hc select over a 1608 x 4 f64 table
  c2mix configs[1]  mix [4 x 1608 x 4 f32 ; 1608 x 4 hc]
  c3    configs[2]  500 users x 4 x 1608 x 4 f32, one launch (dense)
  c3r   configs[2]  the ragged variant (N_u in [128, 1608])
  c3cold configs[2] dense, rotating 8 distinct 51.5 MB pools between launches
        (412 MB > the 256 MiB Infinity Cache: each launch reads its pool from HBM)
  python tools/small_probe.py c3 [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402
from tools.bench_configs import dirichlet  # noqa: E402


def make(cfg, g):
    q = 10
    if cfg == "c1":
        P = dirichlet((4, 1608, 4), torch.float64, g)
        return lambda: ops.select_mc(P, q, "MNC")
    if cfg in ("c2hc", "c2mix"):
        freq = dirichlet((1608, 4), torch.float64, g)
        freq = torch.round(freq * 1000) / 1000
        if cfg == "c2hc":
            Hn = freq.unsqueeze(1)
            return lambda: ops.select_mc(Hn, q, "NMC")
        P = dirichlet((4, 1608, 4), torch.float32, g)
        return lambda: ops.select_mix(P, freq, q, "MNC")
    U, Nu = 500, 1608
    P = dirichlet((4, U * Nu, 4), torch.float32, g)
    if cfg == "c3":
        offs = torch.arange(0, U + 1, device="cuda", dtype=torch.int64) * Nu
        return lambda: ops.select_batched(P, offs, q, "MNC")
    if cfg == "c3cold":
        offs = torch.arange(0, U + 1, device="cuda", dtype=torch.int64) * Nu
        pools = [P] + [dirichlet((4, U * Nu, 4), torch.float32, g) for _ in range(7)]
        it = [0]

        def call():
            it[0] += 1
            return ops.select_batched(pools[it[0] % len(pools)], offs, q, "MNC")
        return call
    if cfg == "c3r":
        sizes = torch.randint(128, 1609, (U,), generator=torch.Generator().manual_seed(1987))
        offs = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(sizes, 0)]).cuda()
        Pr = P[:, :int(offs[-1])].contiguous()
        return lambda: ops.select_batched(Pr, offs, q, "MNC")
    raise SystemExit(f"unknown config {cfg}")


def main():
    cfg = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    g = torch.Generator(device="cuda").manual_seed(1987)
    fn = make(cfg, g)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("ok", cfg, reps)


if __name__ == "__main__":
    main()
