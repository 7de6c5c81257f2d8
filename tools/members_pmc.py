"""Plain (graph-free) launches of the §8(f)4 member kernels at the bench size
(4M frames x 260 f64 features, C = 4; XGB 400 trees of depth 5), for
rocprofv3 --pmc passes (a counter pass per run; tools/gpu_round.sh PHASE=mpmc):
  python tools/members_pmc.py [--reps 5]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402
from ce_amd.xgb import XgbForest, synthetic_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--frames", type=int, default=4_000_000)
    ap.add_argument("--only", default="gnb,sgd,xgb", help="comma list of members to launch")
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(1987)
    D, C, F = 260, 4, a.frames
    theta = torch.randn((C, D), device="cuda", dtype=torch.float64, generator=g)
    var = torch.rand((C, D), device="cuda", dtype=torch.float64, generator=g) + 0.5
    prior = torch.full((C,), 0.25, device="cuda", dtype=torch.float64)
    coef = torch.randn((C, D), device="cuda", dtype=torch.float64, generator=g) * 0.05
    icpt = torch.zeros(C, device="cuda", dtype=torch.float64)
    X = torch.randn((F, D), device="cuda", dtype=torch.float64, generator=g)
    forest = XgbForest.from_json(synthetic_model(n_rounds=100, num_class=4, max_depth=5, num_feature=D))
    only = set(a.only.split(","))
    for _ in range(a.reps):
        if "gnb" in only:
            ops.gnb_predict_proba(X, theta, var, prior)
        if "sgd" in only:
            ops.sgd_predict_proba(X, coef, icpt)
        if "xgb" in only:
            ops.xgb_predict_proba(X, forest)
    torch.cuda.synchronize()
    print("ok", F, a.reps)


if __name__ == "__main__":
    main()
