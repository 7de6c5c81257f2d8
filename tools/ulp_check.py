"""How often do device entropies differ from the glibc-log oracle, and by how
many ulps?  (Diagnostic for DESIGN.md 'Numerics'; needs the GPU.)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402
from oracle import ce_oracle as O  # noqa: E402

rng = np.random.default_rng(11)
for (N, M, C, dt) in [(2_000_000, 16, 4, np.float32), (1_000_000, 4, 4, np.float64), (20_000, 3, 1000, np.float32)]:
    e = -np.log(rng.random((N, M, C)))
    P = (e / e.sum(-1, keepdims=True)).astype(dt)
    g = ops.committee_entropy(torch.from_numpy(P).cuda(), "NMC").cpu().numpy()
    o = O.oracle_committee_entropy(P, "NMC")
    same = g == o
    ulp = np.abs(g.view(np.int64) - o.view(np.int64))
    print(f"N={N} M={M} C={C} {np.dtype(dt).name}: exact {same.mean():.6f}  max ulp {ulp.max()}  "
          f"ulp hist {np.bincount(np.minimum(ulp, 5))}")
