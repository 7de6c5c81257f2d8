"""Reduce rocprofv3 outputs (gpurun_out/prof) to the committed evidence under profiles/.

  python tools/pmc_summary.py <prof_dir> <round_tag>

Writes profiles/<tag>_<layout>_kernel_stats.csv (the --stats summary, ce kernels
first), profiles/<tag>_<layout>_pmc.json (per-kernel FETCH_SIZE / WRITE_SIZE
averages) and updates profiles/traffic.json, which bench.py reads for its
roofline.traffic field.  HBM bytes per launch follow MI355X_MICROARCH.md HBM:
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts exactly half
the bytes of a 16-B/lane streaming read (global_load and LDS-DMA alike), so the
read side is doubled; WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import shutil
import statistics
import sys

prof, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_dir = os.path.join(root, "profiles")
os.makedirs(out_dir, exist_ok=True)
traffic_path = os.path.join(out_dir, "traffic.json")
traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}

for layout in ("NMC", "MNC"):
    tdir = os.path.join(prof, f"trace_{layout}")
    if not os.path.isdir(tdir):
        continue
    rows = list(csv.reader(open(os.path.join(tdir, "run_kernel_stats.csv"))))
    head, body = rows[0], rows[1:]
    body.sort(key=lambda r: (not r[0].startswith("void ce::"), -float(r[2])))
    with open(os.path.join(out_dir, f"{tag}_{layout}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(head)
        w.writerows(body)
    pmc = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        cdir = os.path.join(prof, f"{counter.split('_')[0].lower()}_{layout}")
        path = os.path.join(cdir, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        vals = {}
        for r in csv.DictReader(open(path)):
            if not r["Kernel_Name"].startswith("void ce::"):
                continue
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
        for k, v in vals.items():
            pmc.setdefault(k, {})[counter + "_KiB_mean"] = statistics.mean(v)
            pmc[k]["dispatches"] = len(v)
    stage1 = [k for k in pmc if "k_stream" in k or "k_partial" in k]
    for k in pmc:
        f = pmc[k].get("FETCH_SIZE_KiB_mean", 0.0) * 1024 * 2
        wr = pmc[k].get("WRITE_SIZE_KiB_mean", 0.0) * 1024
        pmc[k]["hbm_bytes_per_launch"] = f + wr
    json.dump(pmc, open(os.path.join(out_dir, f"{tag}_{layout}_pmc.json"), "w"), indent=1)
    if stage1:
        k = stage1[0]
        key = f"{layout}_100000000_16_4_q10_w1"
        traffic[key] = {"kernel": k, "hbm_bytes_per_launch": pmc[k]["hbm_bytes_per_launch"],
                        "fetch_bytes": pmc[k].get("FETCH_SIZE_KiB_mean", 0.0) * 1024 * 2,
                        "write_bytes": pmc[k].get("WRITE_SIZE_KiB_mean", 0.0) * 1024,
                        "source": f"profiles/{tag}_{layout}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"}
    print(layout, json.dumps(pmc, indent=1)[:1500])
# secondary configs (tools/bench_configs.py): stats of every kernel, PMC of the wide stream
cdir = os.path.join(prof, "configs")
if os.path.isdir(cdir):
    rows = list(csv.reader(open(os.path.join(cdir, "run_kernel_stats.csv"))))
    head, body = rows[0], rows[1:]
    body.sort(key=lambda r: (not r[0].startswith("void ce::"), -float(r[2])))
    with open(os.path.join(out_dir, f"{tag}_configs_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(head)
        w.writerows(body)
pmc = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    path = os.path.join(prof, f"{counter.split('_')[0].lower()}_wide", "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith("void ce::"):
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    for k, v in vals.items():
        pmc.setdefault(k, {})[counter + "_KiB_mean"] = statistics.mean(v)
        pmc[k]["dispatches"] = len(v)
for k in pmc:
    pmc[k]["hbm_bytes_per_launch"] = (pmc[k].get("FETCH_SIZE_KiB_mean", 0.0) * 1024 * 2
                                      + pmc[k].get("WRITE_SIZE_KiB_mean", 0.0) * 1024)
if pmc:
    json.dump(pmc, open(os.path.join(out_dir, f"{tag}_wide_pmc.json"), "w"), indent=1)
    print("wide", json.dumps(pmc, indent=1)[:800])
json.dump(traffic, open(traffic_path, "w"), indent=1)
# the XGB member (tools/bench_configs.py --only 7, PHASE=xgb): per-dispatch-size
# kernel time from the trace, FETCH_SIZE per launch (x2, gfx950 rule above)
xdir = os.path.join(prof, "xgb")
if os.path.isdir(xdir):
    rows = list(csv.reader(open(os.path.join(xdir, "run_kernel_stats.csv"))))
    head, body = rows[0], [r for r in rows[1:] if r[0].startswith("void ce::")]
    with open(os.path.join(out_dir, f"{tag}_xgb_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(head)
        w.writerows(body)
    by_grid = {}
    for r in csv.DictReader(open(os.path.join(xdir, "run_kernel_trace.csv"))):
        if "k_xgb_walk" in r["Kernel_Name"]:
            frames = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) * 64
            by_grid.setdefault(frames, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    fetch = {}
    path = os.path.join(prof, "fetch_xgb", "run_counter_collection.csv")
    if os.path.exists(path):
        for r in csv.DictReader(open(path)):
            if "k_xgb_walk" in r["Kernel_Name"]:
                frames = int(r["Grid_Size"]) // int(r["Workgroup_Size"]) * 64
                fetch.setdefault(frames, []).append(float(r["Counter_Value"]) * 1024 * 2)
    summary = {str(k): {"dispatches": len(v), "mean_ms": statistics.mean(v), "min_ms": min(v),
                        "hbm_fetch_bytes_per_launch": statistics.mean(fetch[k]) if k in fetch else None,
                        "algorithmic_bytes_per_launch": k * 260 * 8}
               for k, v in sorted(by_grid.items())}
    json.dump(summary, open(os.path.join(out_dir, f"{tag}_xgb_summary.json"), "w"), indent=1)
    print("xgb", json.dumps(summary, indent=1))
