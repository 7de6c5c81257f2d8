"""Host-inclusive latency of one selection call (Python -> ctypes -> kernels ->
result on the host), the way the reference's per-epoch loop would see it:
eager ops vs a replayed HIP graph of the same call."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402
from tools.bench_configs import dirichlet  # noqa: E402


def lat(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e6


def main():
    g = torch.Generator(device="cuda").manual_seed(1987)
    P = dirichlet((4, 1608, 4), torch.float64, g)
    out = {}
    out["eager select_mc + idx.cpu()"] = lat(lambda: ops.select_mc(P, 10, "MNC")[1].cpu())
    out["eager select_mc (launch only)"] = lat(lambda: ops.select_mc(P, 10, "MNC"))
    static_idx = {}
    gr = torch.cuda.CUDAGraph()
    ops.select_mc(P, 10, "MNC")
    torch.cuda.synchronize()
    with torch.cuda.graph(gr):
        static_idx["i"] = ops.select_mc(P, 10, "MNC")[1]
    out["graph replay + idx.cpu()"] = lat(lambda: (gr.replay(), static_idx["i"].cpu()))
    for k, v in out.items():
        print(json.dumps({"case": k, "median_us": v}), flush=True)


if __name__ == "__main__":
    main()
