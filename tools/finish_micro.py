"""Time the stage-2 merge alone (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402

torch.manual_seed(0)
N = 2_000_000
e = -torch.log(torch.rand((N, 16, 4), device="cuda").clamp_min_(1e-30))
P = e / e.sum(-1, keepdim=True)
plan = ops.MCPlan(P, 10, "NMC")
plan.partial()
torch.cuda.synchronize()
def t(fn, n=50):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3
print(os.environ.get("CE_AMD_FINISH_DEBUG", "0"), "finish us:", t(plan.finish), "partial us:", t(plan.partial, 10))
v = torch.rand(8 * 10, device="cuda", dtype=torch.float64).view(8, 10).sort(dim=1, descending=True).values.reshape(-1)
i = torch.randperm(1000, device="cuda")[:80].to(torch.int64)
print("merge 8 lists us:", t(lambda: ops.topq_merge(v, i, 10)))

