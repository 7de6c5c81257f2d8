"""The wide stream (BASELINE configs[4]: 32 members x 1000 classes bf16) on
pools that make the approximate prefilter skip (i.i.d. uniform members: after
a wave's first 64 items nearly every item is below its threshold) and pools
that make it fail (entropies rising with the position: every item beats the
threshold, so every item takes its exact entropy), for A/B runs of library
builds (CE_AMD_LIB).  One JSON line of per-case kernel times (HIP events, median
of the reps) and fractions of the 8 TB/s HBM peak:
  iid_single     ops.select_mc over one 2M-item i.i.d. pool (one launch)
  iid_job        ops.MCChunkJob over 4 chunks of 2M: the first chunk and the
                 seeded ones timed apart
  rising_single  select_mc over a 2M-item pool whose item i has K_i = 1 +
                 999 i / N classes at 1.0 and the rest at 2^-10 in every member
                 (entropy non-decreasing in i)
  rising_job     the chunked job over 3 chunks of such a pool (rising across
                 the whole pool: the running list never filters)
  python tools/c5_probe.py [--items 2000000] [--reps 3] [--cases iid_single,...]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd  # noqa: E402
import ce_amd.ops as ops  # noqa: E402

M, C = 32, 1000
PEAK = 8000.0


def fill_iid(buf, seed):
    buf.uniform_(0.0, 1.0, generator=torch.Generator(device="cuda").manual_seed(seed))


def fill_rising(buf, lo, total):
    """Item lo + i: K = 1 + 999 (lo + i) // total classes at 1.0, the rest at 2^-10."""
    n = buf.shape[0]
    step = 250_000
    cls = torch.arange(C, device="cuda")
    for a in range(0, n, step):
        b = min(n, a + step)
        k = 1 + (999 * (torch.arange(lo + a, lo + b, device="cuda", dtype=torch.int64))) // total
        row = torch.where(cls[None, :] < k[:, None], 1.0, 2.0 ** -10).to(torch.bfloat16)
        buf[a:b].copy_(row[:, None, :].expand(b - a, M, C))


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    return e0, e1


def frac(n_items, ms):
    return n_items * M * C * 2 / (ms * 1e-3) / 1e9 / PEAK


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cases", default="iid_single,iid_job,rising_single,rising_job")
    a = ap.parse_args()
    ce_amd.load()
    lib = ce_amd._lib.load()
    n = a.items
    buf = torch.empty((n, M, C), dtype=torch.bfloat16, device="cuda")
    out = {"lib": os.path.basename(ce_amd._lib.LIB_PATH), "items_per_chunk": n}
    fill_iid(buf, 7)
    ops.select_mc(buf, 10, "NMC")  # warm-up
    torch.cuda.synchronize()
    for case in a.cases.split(","):
        res = {}
        if case in ("iid_single", "rising_single"):
            if case == "iid_single":
                fill_iid(buf, 11)
            else:
                fill_rising(buf, 0, n)
            evs = []
            for _ in range(a.reps):
                evs.append(timed(lambda: ops.select_mc(buf, 10, "NMC")))
            torch.cuda.synchronize()
            ms = statistics.median(e0.elapsed_time(e1) for e0, e1 in evs)
            res = {"ms": ms, "frac": frac(n, ms), "kernel": lib.ce_last_kernel().decode()}
        else:
            nch = 4 if case == "iid_job" else 3
            first, later, kern = [], [], []
            for _ in range(a.reps):
                job = ops.MCChunkJob(10, "NMC")
                for c in range(nch):
                    if case == "iid_job":
                        fill_iid(buf, 100 + c)
                    else:
                        fill_rising(buf, c * n, nch * n)
                    e = timed(lambda: job.add(buf, c * n))
                    torch.cuda.synchronize()
                    (first if c == 0 else later).append(e[0].elapsed_time(e[1]))
                    if len(kern) < nch:
                        kern.append(lib.ce_last_kernel().decode())
                job.result()
            res = {"first_ms": statistics.median(first), "first_frac": frac(n, statistics.median(first)),
                   "later_ms": statistics.median(later), "later_frac": frac(n, statistics.median(later)),
                   "kernels": kern}
        out[case] = res
        print(f"{case}: {res}", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
