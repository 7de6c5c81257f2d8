"""Per-block phase timing of k_select_small on BASELINE configs[2] (500 users x
4 x 1608 x 4 f32).  Needs the diagnostic build: make -C consensus-entropy_amd
phase; run with CE_AMD_LIB=tools/_diag/ce_amd_phase.so."""
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
U, Nu = 500, 1608
g = torch.Generator(device="cuda").manual_seed(1)
P = torch.rand((4, U * Nu, 4), device="cuda", generator=g)
offs = torch.arange(U + 1, device="cuda", dtype=torch.int64) * Nu
for _ in range(20):
    ops.select_batched(P, offs, 10, "MNC")
torch.cuda.synchronize()
buf = np.zeros((U, 16), np.uint64)
assert L.ce_debug_phase(buf.ctypes.data_as(ctypes.c_void_p), U) == 0
t = (buf.astype(np.int64) - int(buf[:, 0].min())) * 10  # ns
out = {"start_ns": np.percentile(t[:, 0], [0, 25, 50, 75, 100]).tolist(),
       "keys_ns": np.percentile(t[:, 1] - t[:, 0], [0, 50, 100]).tolist(),
       "floor_ns": np.percentile(t[:, 2] - t[:, 1], [0, 50, 100]).tolist(),
       "append_ns": np.percentile(t[:, 3] - t[:, 2], [0, 50, 100]).tolist(),
       "rank_ns": np.percentile(t[:, 4] - t[:, 3], [0, 50, 100]).tolist(),
       "end_ns": np.percentile(t[:, 4], [0, 50, 100]).tolist(),
       "start_hist": np.histogram(t[:, 0], bins=10)[0].tolist(),
       # per-wave key ends (waves 0..7): the block's slowest / fastest wave, and the intra-block skew
       "wave_keys_last_ns": np.percentile(t[:, 6:14].max(1) - t[:, 0], [0, 50, 100]).tolist(),
       "wave_keys_first_ns": np.percentile(t[:, 6:14].min(1) - t[:, 0], [0, 50, 100]).tolist(),
       "wave_skew_ns": np.percentile(t[:, 6:14].max(1) - t[:, 6:14].min(1), [0, 50, 100]).tolist(),
       "floor_after_last_wave_ns": np.percentile(t[:, 2] - t[:, 6:14].max(1), [0, 50, 100]).tolist()}
print(json.dumps(out))
