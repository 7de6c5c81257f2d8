"""Probe of the batched-users path (configs[2]): layout / size / dtype variants,
device time per call from HIP-graph replay."""
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
    for U, Nu, M, dt, lay in [(500, 1608, 4, torch.float32, "MNC"), (500, 1608, 4, torch.float32, "NMC"),
                              (500, 512, 4, torch.float32, "MNC"), (2000, 402, 4, torch.float32, "MNC"),
                              (500, 1608, 4, torch.float64, "MNC"), (500, 1608, 1, torch.float32, "MNC"),
                              (125, 1608, 4, torch.float32, "MNC"), (250, 1608, 4, torch.float32, "MNC"),
                              (1000, 1608, 4, torch.float32, "MNC"), (4000, 1608, 4, torch.float32, "MNC")]:
        shape = (M, U * Nu, 4) if lay == "MNC" else (U * Nu, M, 4)
        P = dirichlet(shape, dt, g)
        offs = torch.arange(0, U + 1, device="cuda", dtype=torch.int64) * Nu
        t = timed(lambda: ops.select_batched(P, offs, 10, lay), 100)
        out.append({"U": U, "Nu": Nu, "M": M, "dtype": str(dt), "layout": lay, "us": t * 1e6,
                    "GBps": P.numel() * P.element_size() / t / 1e9})
        del P
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
