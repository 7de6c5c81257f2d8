"""Per-config measurements for BASELINE.json configs[0..4] (bench.py's JSON line
is configs[3]; this prints one JSON line per config for DESIGN.md).

Timing: HIP events on the launch stream around `reps` back-to-back calls of
the op with inputs resident in HBM; algorithmic bytes per SURVEY.md §8(d).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402

PEAK = 8000.0


def timed(fn, reps, graph=True, per_graph=20):
    """Seconds per call.  graph=True: `per_graph` back-to-back calls captured
    in one HIP graph and replayed, so Python/ctypes launch overhead and the
    graph-launch cost (~10 us per replay) are amortised: the figure is device
    time of the call's kernels plus the gaps between them."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(per_graph):
                fn()
        run = g.replay
        n_run = max(1, reps // per_graph)
        calls = n_run * per_graph
    else:
        run = fn
        n_run = calls = reps
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n_run):
        run()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / calls * 1e-3


def dirichlet(shape, dtype=torch.float32, gen=None):
    e = -torch.log(torch.rand(shape, device="cuda", generator=gen).clamp_min_(1e-30))
    return (e / e.sum(-1, keepdim=True)).to(dtype)


def report(name, items, bytes_, t, extra=None):
    d = {"config": name, "items": items, "s_per_call": t, "items_per_s": items / t,
         "GB_per_s": bytes_ / t / 1e9, "frac_hbm": bytes_ / t / 1e9 / PEAK}
    d.update(extra or {})
    print(json.dumps(d), flush=True)


def cpu_reference(only, reps=5):
    """The reference's own expressions (amg_test.py:441-445 mc, :109-117 +
    :451-452 hc, :473-480 mix, the per-user loop for configs[2]) timed on the
    host, numpy single-threaded, same shapes -- median of `reps` after a
    warm-up.  Restated here (not imported from oracle/, which only tests and
    bench.py's cpu_baseline may use)."""
    import statistics

    import numpy as np
    import pandas as pd
    from scipy.stats import entropy

    rng = np.random.default_rng(1987)

    def dir_(shape, dt=np.float64):
        e = -np.log(rng.random(shape))
        return (e / e.sum(-1, keepdims=True)).astype(dt)

    def med(fn, reps=reps):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    def mc(pred_prob, q=10):
        consensus_prob = np.mean(np.array(pred_prob), axis=0)
        ent = entropy(consensus_prob, axis=1)
        return np.argsort(ent)[::-1][:q]

    out = {}
    if 0 in only:
        members = [dir_((1608, 4)), dir_((1608, 4)), dir_((1608, 4), np.float32), dir_((1608, 4), np.float32)]
        out["configs[0] mc 4x1608x4"] = med(lambda: mc(members))
    if 1 in only:
        votes = rng.integers(0, 4, (1608, 665))
        votes[rng.random((1608, 665)) >= 0.03] = -1
        votes[:, 0] = 1

        def table():  # amg_test.py:109-117 (per-song Counter + np.round(c/n, 3)) on the vote matrix
            rows = []
            for r in votes:
                v = r[r >= 0]
                n = len(v)
                rows.append([np.round(np.count_nonzero(v == c) / n, 3) for c in range(4)])
            return pd.DataFrame(rows, columns=["Q1", "Q2", "Q3", "Q4"])

        hc = table()
        out["configs[1] hc table 1608x665 (3%)"] = med(table)
        out["configs[1] hc select 1608x4"] = med(lambda: np.argsort(entropy(hc, axis=1))[::-1][:10])
        members = [pd.DataFrame(dir_((1608, 4)), columns=hc.columns) for _ in range(4)]

        def mix():
            consensus_prob = pd.DataFrame(np.mean(np.array(members), axis=0), columns=hc.columns)
            this = pd.concat([consensus_prob, hc])
            return np.argsort(entropy(this, axis=1))[::-1][:10]

        out["configs[1] mix [4x1608x4 ; 1608x4]"] = med(mix)
    if 2 in only:
        users = [[dir_((1608, 4), np.float32) for _ in range(4)] for _ in range(500)]
        out["configs[2] batched 500 users (per-user loop)"] = med(lambda: [mc(u) for u in users], reps=3)
    if 4 in only:
        n = 2000
        members = [dir_((n, 1000), np.float32) for _ in range(32)]
        t = med(lambda: mc(members), reps=3)
        out["configs[4] wide 32x1000 (per item)"] = t / n
    if 5 in only:  # amg_test.py:437 groupby mean of one member, 1608 songs x 40 frames and 1M songs x 40 frames
        for songs in (1608, 1_000_000):
            F = songs * 40
            s_id = np.repeat(np.arange(songs), 40)
            vals = rng.random((F, 4))
            out[f"(f) segment mean {songs} songs x 40 frames (pandas groupby)"] = med(
                lambda: pd.DataFrame(vals, index=pd.Index(s_id, name="s_id")).groupby(["s_id"]).mean(), reps=3)
    if 6 in only:  # deam_classifier.py:211-218 members' predict_proba on 64,320 frames x 260 features
        from sklearn.linear_model import SGDClassifier
        from sklearn.naive_bayes import GaussianNB

        Xf = rng.normal(0, 1, (4000, 260))
        yf = rng.integers(0, 4, 4000)
        gnb = GaussianNB().fit(Xf, yf)
        sgd = SGDClassifier(loss="log_loss", max_iter=5, tol=None).fit(Xf, yf)
        X = rng.normal(0, 1, (64_320, 260))
        out["(f)4 GaussianNB predict_proba 64320 frames (sklearn)"] = med(lambda: gnb.predict_proba(X), reps=3)
        out["(f)4 SGD(log) predict_proba 64320 frames (sklearn)"] = med(lambda: sgd.predict_proba(X), reps=3)
    for k, v in out.items():
        print(json.dumps({"cpu_reference": k, "s": v, "threads": 1}), flush=True)


def cpu_reference_1thread(only):
    """cpu_reference with BLAS / OpenMP pools limited to one thread (the box
    exports OMP_NUM_THREADS=16; the sklearn members' predict_proba uses BLAS)."""
    from threadpoolctl import threadpool_limits

    with threadpool_limits(limits=1):
        cpu_reference(only)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="0,1,2,4,5,6,7,8")
    ap.add_argument("--cpu", action="store_true", help="also time the reference expressions on the host")
    args = ap.parse_args()
    only = {int(x) for x in args.only.split(",")}
    if args.cpu:
        cpu_reference_1thread(only)
    g = torch.Generator(device="cuda").manual_seed(1987)
    q = 10
    if 0 in only:  # configs[0]: 4-member committee x 1608 x 4, mixed f32/f64 -> f64 stack
        P = dirichlet((4, 1608, 4), torch.float64, g)
        t = timed(lambda: ops.select_mc(P, q, "MNC"), 200)
        report("configs[0] mc 4x1608x4 f64 (latency)", 1608, P.numel() * 8, t)
    if 1 in only:  # configs[1]: hc votes 1608 x 665 int8 + mix with a 4x1608x4 committee
        for dens in (0.03, 1.0):
            v = torch.randint(0, 4, (1608, 665), device="cuda", generator=g, dtype=torch.int64).to(torch.int8)
            miss = torch.rand((1608, 665), device="cuda", generator=g) >= dens
            v[miss] = -1
            v[:, 0] = 1
            t = timed(lambda: ops.vote_table(v), 200)
            report(f"configs[1] hc table 1608x665 int8 density {dens}", 1608, v.numel(), t)
            freq, _ = ops.vote_table(v)
            Hn = freq.unsqueeze(1)
            t = timed(lambda: ops.select_mc(Hn, q, "NMC"), 200)
            report("configs[1] hc select over the 1608x4 table", 1608, freq.numel() * 8, t)
            P = dirichlet((4, 1608, 4), torch.float32, g)
            t = timed(lambda: ops.select_mix(P, freq, q, "MNC"), 200)
            report("configs[1] mix [4x1608x4 f32 ; 1608x4 hc]", 3216, P.numel() * 4 + freq.numel() * 8, t)
    if 2 in only:  # configs[2]: 500 users x 4 members x 1608 x 4, q per user, one launch
        U, Nu = 500, 1608
        P = dirichlet((4, U * Nu, 4), torch.float32, g)
        offs = torch.arange(0, U + 1, device="cuda", dtype=torch.int64) * Nu
        t = timed(lambda: ops.select_batched(P, offs, q, "MNC"), 50)
        report("configs[2] batched 500 users x 4 x 1608 x 4 f32", U * Nu, P.numel() * 4, t)
        sizes = torch.randint(128, 1609, (U,), generator=torch.Generator().manual_seed(1987))
        offs_r = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(sizes, 0)]).cuda()
        n = int(offs_r[-1])
        Pr = P[:, :n].contiguous()
        t = timed(lambda: ops.select_batched(Pr, offs_r, q, "MNC"), 50)
        report("configs[2] batched ragged 500 users (N_u in [128,1608])", n, Pr.numel() * 4, t)
    if 4 in only:  # configs[4]: 50M x 32 x 1000 bf16 (3.2 TB) streamed in chunks; here the first 5M items
        from tools.bench_c5 import run as c5_run

        print(json.dumps(c5_run(items=5_000_000, chunk=1_000_000, log=False)), flush=True)  # full job: tools/bench_c5.py
    if 5 in only:
        segment_mean_configs(g, report)
    if 6 in only:  # §8(f)4: member inference over 260-feature frames (GNB, SGD log), C = 4
        D, C = 260, 4
        theta = torch.randn((C, D), device="cuda", dtype=torch.float64, generator=g)
        var = torch.rand((C, D), device="cuda", dtype=torch.float64, generator=g) + 0.5
        prior = torch.full((C,), 0.25, device="cuda", dtype=torch.float64)
        coef = torch.randn((C, D), device="cuda", dtype=torch.float64, generator=g) * 0.05
        icpt = torch.zeros(C, device="cuda", dtype=torch.float64)
        for F in (64_320, 4_000_000):
            X = torch.randn((F, D), device="cuda", dtype=torch.float64, generator=g)
            reps = 200 if F < 100_000 else 20
            t = timed(lambda: ops.gnb_predict_proba(X, theta, var, prior), reps)
            report(f"(f)4 GaussianNB predict_proba {F} frames x {D} f64", F, F * D * 8, t)
            t = timed(lambda: ops.sgd_predict_proba(X, coef, icpt), reps)
            report(f"(f)4 SGD(log) predict_proba {F} frames x {D} f64", F, F * D * 8, t)
            del X
    if 7 in only:  # §8(f)4: the xgb member, XGBClassifier(max_depth=5) x 100 rounds x 4 classes over 260 features
        import numpy as np

        from ce_amd.xgb import XgbForest, synthetic_model

        D = 260
        forest = XgbForest.from_json(synthetic_model(n_rounds=100, num_class=4, max_depth=5, num_feature=D))
        depth, T = forest.pack()[3], len(forest.trees)
        for F in (64_320, 4_000_000):
            X = torch.randn((F, D), device="cuda", dtype=torch.float64, generator=g)
            reps = 100 if F < 100_000 else 10
            for miss in (False, True):
                if miss:  # one missing value per ~100 frames: most tiles take the default-direction path
                    X[torch.rand((F, D), device="cuda", generator=g) < 1e-4] = float("nan")
                t = timed(lambda: ops.xgb_predict_proba(X, forest), reps)
                report(f"(f)4 XGB predict_proba {F} frames x {D} f64, {T} trees depth {depth}, "
                       f"{'with' if miss else 'no'} missing values", F, F * D * 8, t,
                       {"node_steps_per_s": F * T * depth / t})
            del X
    if 8 in only:
        frames_selection_configs(g, report)


def frames_selection_configs(g, report_fn, q=10):
    """SURVEY.md §8(f)1 end to end: three frame-level members (gnb, sgd, xgb:
    [F, 4] f64 frame rows, amg_test.py:435-437) and one song-level member (the
    CNN's [N, 4]) -> groupby mean -> member-sequential mean -> entropy -> top-q
    (:437-445).  Fused: ce_select_frames (one pass, the [M, N, C] stack never
    written).  Two-step: ce_segment_mean of each frame member into its row of a
    preallocated [M, N, C] stack + ce_select_mc over the stack.  Frames grouped
    (CSR) and shuffled (permutation gather)."""
    for songs, fps in ((1608, 40), (1_000_000, 40)):
        F, C = songs * fps, 4
        fr = [dirichlet((F, C), torch.float64, g) for _ in range(3)]
        cnn = dirichlet((songs, C), torch.float64, g)
        offs = torch.arange(0, songs + 1, device="cuda", dtype=torch.int64) * fps
        stack = torch.empty((4, songs, C), device="cuda", dtype=torch.float64)
        stack[3].copy_(cnn)
        reps = 200 if songs < 10_000 else 40
        for perm in (None, torch.randperm(F, device="cuda", generator=g)):
            kind = "grouped" if perm is None else "permuted"
            byts = 3 * F * C * 8 + songs * C * 8 + (F * 8 if perm is not None else 0)  # the permutation read once

            def two_step():
                for m in range(3):
                    ops.segment_mean(fr[m], offs, perm, out=stack[m])
                return ops.select_mc(stack, q, "MNC")

            fused = lambda: ops.select_frames(fr + [cnn], offs, q, perm=perm)  # noqa: E731
            a, b = fused(), two_step()
            same = bool(torch.equal(a[1], b[1]) and torch.equal(a[0].view(torch.int64), b[0].view(torch.int64)))
            t_f = timed(fused, reps)
            t_2 = timed(two_step, reps)
            report_fn(f"(f)1 frames -> selection {songs} songs x {fps} frames, 3 frame + 1 song member, {kind}: fused",
                      songs, byts, t_f, {"same_selection_as_two_step": same})
            report_fn(f"(f)1 frames -> selection {songs} songs x {fps} frames, 3 frame + 1 song member, {kind}: two-step",
                      songs, byts, t_2, {"speedup_fused": t_2 / t_f})


def segment_mean_configs(g, report_fn):
    """the frame -> song groupby mean (amg_test.py:437) per
    member, frames grouped (CSR) and shuffled (permutation gather)."""
    for songs, fps in ((1608, 40), (1_000_000, 40)):
        F, C = songs * fps, 4
        fr = torch.rand((F, C), device="cuda", generator=g, dtype=torch.float64)
        offs = torch.arange(0, songs + 1, device="cuda", dtype=torch.int64) * fps
        t = timed(lambda: ops.segment_mean(fr, offs), 200 if songs < 10_000 else 40)
        report_fn(f"(f) segment mean {songs} songs x {fps} frames x {C} f64, grouped", F, F * C * 8 + songs * C * 8, t)
        perm = torch.randperm(F, device="cuda", generator=g)
        t = timed(lambda: ops.segment_mean(fr, offs, perm), 200 if songs < 10_000 else 40)
        report_fn(f"(f) segment mean {songs} songs x {fps} frames x {C} f64, permuted", F,
                  F * (C * 8 + 8) + songs * C * 8, t)


if __name__ == "__main__":
    main()
