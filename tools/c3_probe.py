"""BASELINE configs[2] alone (500 users x 4 members x 1608 x 4 f32, member-major,
q = 10): `reps` select_batched calls, for rocprofv3 kernel traces / PMC passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402
from tools.bench_configs import dirichlet  # noqa: E402

U, Nu = 500, 1608
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
g = torch.Generator(device="cuda").manual_seed(1987)
P = dirichlet((4, U * Nu, 4), torch.float32, g)
offs = torch.arange(0, U + 1, device="cuda", dtype=torch.int64) * Nu
for _ in range(reps):
    ops.select_batched(P, offs, 10, "MNC")
torch.cuda.synchronize()
print("ok")
