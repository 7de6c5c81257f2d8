"""The random-row ceiling for SURVEY.md §8(f)1's shuffled frames (VERDICT r04
Next #7): how fast can ANY kernel on this box read 32-B rows through a random
permutation?  Times, on the configuration of tools/bench_configs.py --only 8
(1M songs x 40 frames, 3 frame-level f64 members of C = 4 + 1 song-level):
  torch_gather   torch.index_select of each member's [F, 4] f64 rows by the
                 permutation (torch's own gather kernel; reads perm + rows,
                 writes the gathered copy)
  fused          ops.select_frames(..., perm=perm) (k_frames_lanes, one pass)
  fused_grouped  the same frames already grouped (no perm, LDS-DMA tiles)
and prints the useful bytes per second of each (rows read once + perm once).
  python tools/gather_probe.py [--songs N] [--mixed] [--pmc]
  (--mixed: the third frame member float32, as an XGB member's predict_proba;
   --pmc: only 5 fused shuffled calls, for a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE pass)"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "consensus-entropy_amd")]
import torch  # noqa: E402

import ce_amd.ops as ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev) * 1e-3


def main():
    g = torch.Generator(device="cuda").manual_seed(1987)
    songs = int(sys.argv[sys.argv.index("--songs") + 1]) if "--songs" in sys.argv else 1_000_000
    fps, C = 40, 4
    F = songs * fps
    mixed = "--mixed" in sys.argv
    dts = [torch.float64, torch.float64, torch.float32 if mixed else torch.float64]
    fr = [torch.rand((F, C), dtype=dt, device="cuda", generator=g) for dt in dts]
    cnn = torch.rand((songs, C), dtype=torch.float64, device="cuda", generator=g)
    offs = torch.arange(0, F + 1, fps, device="cuda", dtype=torch.int64)
    perm = torch.randperm(F, device="cuda", generator=g)
    rows = sum(f.numel() * f.element_size() for f in fr)
    if "--pmc" in sys.argv:
        for _ in range(5):
            ops.select_frames(fr + [cnn], offs, 10, perm=perm)
        torch.cuda.synchronize()
        print(json.dumps({"pmc_run": "fused shuffled x5", "useful_bytes_per_call": rows + F * 8 + songs * C * 8}))
        return
    out = {"config": f"{songs} songs x {fps} frames, 3 frame-level members ({'f64, f64, f32' if mixed else 'f64'}; C={C}) + 1 song-level"}
    reps = 200 if songs < 100_000 else 20
    t = timed(lambda: [torch.index_select(f, 0, perm) for f in fr], reps)
    out["torch_gather"] = {"s": t, "useful_GB_per_s": (rows + 3 * F * 8) / t / 1e9,
                           "note": "perm read per member; the gathered copy is also written (not counted)"}
    t = timed(lambda: ops.select_frames(fr + [cnn], offs, 10, perm=perm), reps)
    out["fused_shuffled"] = {"s": t, "useful_GB_per_s": (rows + F * 8 + songs * C * 8) / t / 1e9}
    t = timed(lambda: ops.select_frames(fr + [cnn], offs, 10), reps)
    out["fused_grouped"] = {"s": t, "useful_GB_per_s": (rows + songs * C * 8) / t / 1e9}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
