"""Reduce the small-pool visit (tools/gpu_round.sh PHASE=small, one rocprofv3
kernel trace per config and library) to one JSON: per config, the selection
kernels' mean / min / max device time over the 200 calls, per tag (''=this
round's kernels, 'r02_' = the round-2 library, other tags = A/B knobs), plus
the PMC reduction of the dense configs[2] passes when present.
  python tools/small_summary.py gpurun_out/prof profiles/r03_small.json"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def kernel_rows(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"] if "Kernel_Name" in r else r["Name"]
        if "ce::" not in name:
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        rows.setdefault(name.split("(")[0].replace("void ", ""), []).append(dur)
    return rows


def main(prof, out):
    res = {"what": "rocprofv3 --kernel-trace of tools/small_probe.py <config> 200 (plain launches), device ns",
           "configs": {}}
    for d in sorted(glob.glob(os.path.join(prof, "*small_*"))):
        tag, cfg = os.path.basename(d).split("small_")
        tr = glob.glob(os.path.join(d, "*kernel_trace.csv"))
        if not tr:
            continue
        for k, v in kernel_rows(tr[0]).items():
            v = sorted(v)
            ent = res["configs"].setdefault(cfg, {}).setdefault(tag or "r03", {})
            ent[k[:140]] = {"calls": len(v), "mean_us": sum(v) / len(v) / 1e3, "median_us": v[len(v) // 2] / 1e3,
                            "min_us": v[0] / 1e3, "max_us": v[-1] / 1e3}
    try:
        from pmc_reduce import main as pmc_main
        tags = sorted({os.path.basename(d)[:-len("pmc_fetch")] for d in glob.glob(os.path.join(prof, "*pmc_fetch"))})
        for tag in tags:
            passes = [p for p in (f"{tag}pmc_fetch", f"{tag}pmc_write", f"{tag}pmc_sq", f"{tag}pmc_ta")
                      if os.path.isdir(os.path.join(prof, p))]
            if passes:
                tmp = out + f".{tag or 'r03'}.pmc.json"
                pmc_main(prof, tmp, passes)
                res.setdefault("pmc_configs2_dense", {})[tag or "r03"] = json.load(open(tmp))["kernels"]
                os.remove(tmp)
    except Exception as e:  # noqa: BLE001
        res["pmc_error"] = repr(e)
    json.dump(res, open(out, "w"), indent=1)
    for cfg, tags in res["configs"].items():
        for tag, ks in tags.items():
            for k, v in ks.items():
                print(f"{cfg:6s} {tag:6s} {v['median_us']:8.2f} us  {k[:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
