"""Reduce a PHASE=c5 visit (tools/gpu_round.sh: rocprofv3 kernel trace of the
full tools/bench_c5.py job + PMC passes of k_stream_wide2 at 12M items) to
one JSON: the job line, per-kernel trace stats, per-dispatch counters
averaged over dispatches 2.. (the first is a warm-up chunk), and derived
fractions (FETCH_SIZE x 2 per the gfx950 rule; VALU busy per SIMD; waves
waiting; LDS bank-conflict share; TA busy).
  python tools/c5_summary.py gpurun_out profiles/r04_c5_job_prefilter.json"""
import csv
import glob
import json
import os
import statistics
import sys

CUS, SIMDS, XCDS = 256, 4, 8


def stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[r["Name"][:120]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                "total_ms": float(r["TotalDurationNs"]) / 1e6}
    return out


def counters(d, kernel="k_stream_wide2"):
    """Per-dispatch counters of `kernel`, averaged over the dispatches that did
    the work: since round 6 every chunk launches BOTH wide grids and the one the
    grid vote does not pick exits at once (counters ~0: dropped, < 1 % of the
    pass's largest dispatch), and the first working dispatch is a warm-up."""
    per = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if kernel not in r["Kernel_Name"]:
            continue
        disp = int(r["Dispatch_Id"])
        per.setdefault(disp, {}).setdefault(r["Counter_Name"], 0.0)
        per[disp][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        return {}
    size = {k: sum(v.values()) for k, v in per.items()}
    big = max(size.values())
    keys = sorted(k for k in per if size[k] >= 0.01 * big)
    keys = keys[1:] if kernel == "k_stream_wide2" and len(keys) > 1 else keys
    names = set().union(*(per[k] for k in keys)) if keys else set()
    return {n: statistics.mean(per[k][n] for k in keys if n in per[k]) for n in names}


def main(gout, dst):
    prof = os.path.join(gout, "prof")
    job = json.loads(open(os.path.join(gout, "c5_job.json")).read().strip().splitlines()[-1])
    st = stats(glob.glob(os.path.join(prof, "c5_job", "**", "*kernel_stats.csv"), recursive=True)[0])
    pmc, seed = {}, {}
    for g in ("c5_fetch", "c5_write", "c5_sq", "c5_lds"):
        d = glob.glob(os.path.join(prof, g, "**", "run_counter_collection.csv"), recursive=True)
        if d:
            pmc.update(counters(os.path.dirname(d[0])))
            seed.update(counters(os.path.dirname(d[0]), "k_wide_seed<"))
    items = 12_000_000 / 6  # per dispatch at the PMC size (12M items, 6 chunks)
    der = {}
    if "FETCH_SIZE" in pmc:
        der["hbm_bytes_per_dispatch (FETCH_SIZE KiB x 1024 x 2, gfx950 rule)"] = pmc["FETCH_SIZE"] * 1024 * 2
        der["algorithmic_bytes_per_dispatch"] = items * 64000
    if "SQ_INSTS_VALU" in pmc and "SQ_WAVES" in pmc:
        der["valu_instructions_per_item (wave-level)"] = pmc["SQ_INSTS_VALU"] / items
    if "SQ_ACTIVE_INST_VALU" in pmc and "GRBM_GUI_ACTIVE" in pmc:
        der["valu_busy_per_simd"] = pmc["SQ_ACTIVE_INST_VALU"] * 4 / (pmc["GRBM_GUI_ACTIVE"] / XCDS) / (CUS * SIMDS)
    if "SQ_WAIT_ANY" in pmc and "SQ_WAVE_CYCLES" in pmc:
        der["wave_time_waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES)"] = pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in seed:
        der["k_wide_seed_hbm_bytes_per_dispatch"] = seed["FETCH_SIZE"] * 1024 * 2
    json.dump({"what": "BASELINE configs[4] full job (50M x 32 x 1000 bf16, 25 chunks of 2M items) under rocprofv3 "
                       "kernel trace, and PMC passes of k_stream_wide2 at 12M items (6 chunks; per-dispatch values "
                       "averaged over the working dispatches 2..6 -- the grid the vote did not pick exits at once)",
               "pmc_k_wide_seed_per_dispatch": seed,
               "command": "gpurun -- 'PHASE=c5 bash tools/gpu_round.sh' ; python tools/c5_summary.py gpurun_out " + dst,
               "job_line": job, "kernel_stats": st, "pmc_per_dispatch": pmc, "derived": der},
              open(dst, "w"), indent=1)
    print(json.dumps(der, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
