"""Per-block phase timing of k_select_tiles on the small-pool configs, from the
diagnostic build's stamps (make -C consensus-entropy_amd phase; run with
CE_AMD_LIB=tools/_diag/ce_amd_phase.so):
  c3  BASELINE configs[2]: 500 users x 4 x 1608 x 4 f32, one launch -> 500 blocks
  c3cold  the same, 8 distinct pools rotated between launches (each launch reads HBM)
  c1  configs[0]: one 4 x 1608 x 4 f64 pool -> one block; 5 samples, each the
      last of 200 back-to-back launches
The shader clock over a block = shader-clock ticks / wall-clock (100 MHz) time
between the block's first and last stamps.
  python tools/phase_probe.py [c3|c3cold|c1]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "consensus-entropy_amd"))
import ce_amd  # noqa: E402
from ce_amd import ops  # noqa: E402

L = ce_amd._lib.load()


def stamps(n):
    buf = np.zeros((n, 16), np.uint64)
    assert L.ce_debug_phase(buf.ctypes.data_as(ctypes.c_void_p), n) == 0
    return buf.astype(np.int64)


def pct(x, p=(0, 50, 100)):
    return np.percentile(x, p).tolist()


def reduce(b):
    t = (b[:, :14] - int(b[:, 0].min())) * 10  # ns
    mhz = (b[:, 15] - b[:, 14]) / ((b[:, 4] - b[:, 0]) * 10) * 1e3
    return {"start_ns": pct(t[:, 0], [0, 25, 50, 75, 100]),
            "keys_ns": pct(t[:, 1] - t[:, 0]),
            "floor_ns": pct(t[:, 2] - t[:, 1]),
            "append_ns": pct(t[:, 3] - t[:, 2]),
            "exact_ns": pct(t[:, 5] - t[:, 3]),  # survivors' exact entropies (wave 0's share)
            "rank_ns": pct(t[:, 4] - t[:, 5]),
            "end_ns": pct(t[:, 4]),
            # per-wave key ends (waves 0..7): the block's slowest / fastest wave, and the intra-block skew
            "wave_keys_last_ns": pct(t[:, 6:14].max(1) - t[:, 0]),
            "wave_keys_first_ns": pct(t[:, 6:14].min(1) - t[:, 0]),
            "wave_skew_ns": pct(t[:, 6:14].max(1) - t[:, 6:14].min(1)),
            "floor_after_last_wave_ns": pct(t[:, 2] - t[:, 6:14].max(1)),
            "shader_clock_mhz": pct(mhz)}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    g = torch.Generator(device="cuda").manual_seed(1)
    if cfg in ("c3", "c3cold"):
        U, Nu = 500, 1608
        pools = [torch.rand((4, U * Nu, 4), device="cuda", generator=g) for _ in range(8 if cfg == "c3cold" else 1)]
        offs = torch.arange(U + 1, device="cuda", dtype=torch.int64) * Nu
        for it in range(20):  # c3cold: 8 pools rotated (412 MB > the 256 MiB Infinity Cache), stamps of the last
            ops.select_batched(pools[it % len(pools)], offs, 10, "MNC")
        torch.cuda.synchronize()
        out = reduce(stamps(U))
    else:
        P = torch.rand((4, 1608, 4), device="cuda", generator=g, dtype=torch.float64)
        rows = []
        for _ in range(5):
            for _ in range(200):
                ops.select_mc(P, 10, "MNC")
            torch.cuda.synchronize()
            rows.append(stamps(1)[0])
        out = reduce(np.array(rows))
    out.update(config=cfg, percentiles="[min, median, max] over the blocks (c1: over 5 samples); "
               "start_ns: 0/25/50/75/100; relative to the first block's start")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
