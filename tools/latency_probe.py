"""Latency probe of the small launches (single-block pools, stage-2 merges):
device time per call from HIP-graph replay, for several pool sizes, so the
per-iteration and fixed costs can be separated.  Prints one JSON line per case.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402
from tools.bench_configs import dirichlet, timed  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(1987)
    out = []
    z = torch.zeros(1, device="cuda")
    out.append(("trivial fill kernel", timed(lambda: z.fill_(1.0), 500)))
    for dt in (torch.float64, torch.float32):
        for n in (64, 256, 1024, 1608, 4096, 16384):
            P = dirichlet((4, n, 4), dt, g)
            out.append((f"select_mc MNC M=4 {dt} N={n}", timed(lambda: ops.select_mc(P, 10, "MNC"), 300)))
    for M in (1, 16):
        P = dirichlet((M, 1608, 4), torch.float32, g)
        out.append((f"select_mc MNC M={M} f32 N=1608", timed(lambda: ops.select_mc(P, 10, "MNC"), 300)))
    for nl in (1, 8, 64, 1024):
        v = torch.rand(nl * 10, device="cuda", generator=g, dtype=torch.float64)
        v = v.view(nl, 10).sort(dim=1, descending=True).values.contiguous()
        i = torch.arange(nl * 10, device="cuda", dtype=torch.int64).view(nl, 10)
        out.append((f"topq_merge nlists={nl} q=10", timed(lambda: ops.topq_merge(v, i, 10), 300)))
    for U in (1, 64, 500):
        P = dirichlet((4, U * 1608, 4), torch.float32, g)
        offs = torch.arange(0, U + 1, device="cuda", dtype=torch.int64) * 1608
        out.append((f"select_batched U={U} x 1608 f32", timed(lambda: ops.select_batched(P, offs, 10, "MNC"), 100)))
    for name, t in out:
        print(json.dumps({"case": name, "us": t * 1e6}), flush=True)


if __name__ == "__main__":
    main()
