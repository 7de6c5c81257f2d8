"""Reduce rocprofv3 --pmc passes (run_counter_collection.csv under
<prof>/<pass>/) to per-kernel means per launch plus derived figures:
  python tools/pmc_reduce.py <prof dir> <out.json> <pass> [<pass> ...]
Derived (MI355X_MICROARCH.md units: SQ cycle counters in quad-cycles,
GRBM_GUI_ACTIVE summed over the 8 XCDs; FETCH_SIZE x 2 on gfx950):
  hbm_bytes     (FETCH_SIZE x 2 + WRITE_SIZE) x 1024
  valu_busy     SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  ta_busy       TA_TA_BUSY_sum / (256 CUs x GRBM_GUI_ACTIVE / 8)
  wait_any      SQ_WAIT_ANY / SQ_WAVE_CYCLES, valu_insts_per_wave, ..."""
import csv
import json
import os
import statistics
import sys


def main(prof, out, passes):
    per = {}
    for sub in passes:
        path = os.path.join(prof, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            print("missing", path, file=sys.stderr)
            continue
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if "ce::" not in k:
                continue
            name = k.split("(")[0].replace("void ce::", "")
            per.setdefault(name, {}).setdefault(r["Counter_Name"], {}).setdefault((sub, r["Dispatch_Id"]), 0.0)
            per[name][r["Counter_Name"]][(sub, r["Dispatch_Id"])] += float(r["Counter_Value"])
    res = {}
    for name, cs in per.items():
        m = {c: statistics.mean(v.values()) for c, v in cs.items()}
        d = {}
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            d["hbm_bytes"] = (m.get("FETCH_SIZE", 0) * 2 + m.get("WRITE_SIZE", 0)) * 1024
        g = m.get("GRBM_GUI_ACTIVE")
        if g:
            if "SQ_ACTIVE_INST_VALU" in m:
                d["valu_busy"] = m["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * g / 8)
            if "TA_TA_BUSY_sum" in m:
                d["ta_busy"] = m["TA_TA_BUSY_sum"] / (256 * g / 8)
            if "SQ_LDS_BANK_CONFLICT" in m:
                d["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / (256 * g / 8)
            d["gpu_cycles"] = g / 8
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            d["wait_any"] = m.get("SQ_WAIT_ANY", 0) / wc
            d["wait_inst_any"] = m.get("SQ_WAIT_INST_ANY", 0) / wc
        if m.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if c in m:
                    d[c.lower().replace("sq_insts_", "") + "_insts_per_wave"] = m[c] / m["SQ_WAVES"]
        res[name] = {"per_launch_mean": m, "derived": d, "launches": max(len(v) for v in cs.values())}
    json.dump({"passes": passes, "kernels": res}, open(out, "w"), indent=1)
    for n, v in res.items():
        print(n[:100], json.dumps(v["derived"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
