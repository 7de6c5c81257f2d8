"""Reduce a PHASE=smallab visit (tools/gpu_round.sh: rocprofv3 --kernel-trace of
tools/small_probe.py <config> 200 per library build, builds alternating, two
rounds) to median / min device microseconds of the selection kernels per
(build, config, round).
  python tools/ab_summary.py gpurun_out/prof [out.json]"""
import csv
import glob
import json
import os
import sys


def durations(path):
    out = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Name", "")
        if "ce::" in name:
            out.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return sorted(out)


def main(prof, out=None):
    res = {}
    for d in sorted(glob.glob(os.path.join(prof, "ab_*"))):
        _, lib, cfg, rep = os.path.basename(d).split("_", 3)
        tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if not tr:
            continue
        v = durations(tr[0])
        if v:
            res.setdefault(cfg, {}).setdefault(lib, {})[rep] = {
                "calls": len(v), "median_us": v[len(v) // 2] / 1e3, "min_us": v[0] / 1e3}
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
