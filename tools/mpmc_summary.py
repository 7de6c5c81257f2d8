"""Reduce the member-kernel PMC passes (gpu_round.sh PHASE=mpmc) to
profiles/<tag>_members_pmc.json: per kernel, the mean per launch of every
counter and the derived occupancy / stall / VALU / gather figures.
  python tools/mpmc_summary.py gpurun_out/prof r02"""
import csv
import json
import os
import statistics
import sys

prof, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
per = {}
for sub in ("mpmc_sq", "mpmc_ta", "mpmc_sq2", "mpmc_lds"):
    path = os.path.join(prof, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if not k.startswith("void ce::"):
            continue
        name = k.split("(")[0].replace("void ce::", "")
        per.setdefault(name, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        per[name][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
out = {}
for name, cs in per.items():
    m = {c: statistics.mean(v.values()) for c, v in cs.items()}
    d = {}
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        d["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / wc  # parked on s_waitcnt / barrier
        d["wait_inst_any_frac"] = m.get("SQ_WAIT_INST_ANY", 0) / wc  # issue stalls
        d["active_valu_frac_of_wave_cycles"] = m.get("SQ_ACTIVE_INST_VALU", 0) / wc
    if m.get("SQ_BUSY_CYCLES") and m.get("GRBM_GUI_ACTIVE"):
        # VALU busy per SIMD: ACTIVE_INST_VALU (quad-cycles x 4) / (1024 SIMDs x GPU cycles / 8 XCDs)
        d["valu_busy_frac"] = m["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    if m.get("SQ_WAVES"):
        d["valu_insts_per_wave"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_WAVES"]
        d["vmem_rd_insts_per_wave"] = m.get("SQ_INSTS_VMEM_RD", 0) / m["SQ_WAVES"]
    if m.get("GRBM_GUI_ACTIVE"):
        d["ta_busy_frac"] = m.get("TA_TA_BUSY_sum", 0) / (256 * m["GRBM_GUI_ACTIVE"] / 8)
        d["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / (256 * m["GRBM_GUI_ACTIVE"] / 8)
    out[name] = {"per_launch_mean": m, "derived": d, "launches": len(next(iter(cs.values())))}
path = os.path.join(root, "profiles", f"{tag}_members_pmc.json")
json.dump({"commands": ["rocprofv3 --pmc <pass> -- python3 tools/members_pmc.py (4M frames x 260 f64, 5 reps; "
                        "passes: tools/gpu_round.sh PHASE=mpmc)"],
           "units": "SQ_*CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles (MI355X_MICROARCH.md); "
                    "GRBM_GUI_ACTIVE summed over the 8 XCDs",
           "kernels": out}, open(path, "w"), indent=1)
for n, v in out.items():
    print(n, json.dumps(v["derived"]))
