"""Reduce the rocprofv3 evidence of ONE bench.py command (gpu_round.sh
PHASE=benchprof: `rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1
--steps 20 --warmup 5`, then FETCH_SIZE / WRITE_SIZE passes) to committed files:
  profiles/<tag>_bench_exact.json      the bench JSON line of the traced run, and
      per ce kernel: all dispatches (warm-up included) and the TIMED dispatches
      only (the last `steps` ones), mean/min/max duration, and the roofline
      fraction recomputed from the timed mean; HBM bytes per launch from the
      PMC passes (FETCH_SIZE x 2 per the gfx950 rule + WRITE_SIZE, KiB units)
  profiles/<tag>_bench_exact_kernel_stats.csv   the --stats table (ce kernels first)
  python tools/trace_summary.py gpurun_out/prof gpurun_out/bench_exact.json r02"""
import csv
import json
import os
import statistics
import sys

prof, bench_path, tag = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_dir = os.path.join(root, "profiles")
bench = json.loads(open(bench_path).read().strip().splitlines()[-1])
steps, warmup = bench["steps"], bench["warmup"]
tdir = os.path.join(prof, "bench_exact")
trace = list(csv.DictReader(open(os.path.join(tdir, "run_kernel_trace.csv"))))
per = {}
for r in sorted(trace, key=lambda r: int(r["Start_Timestamp"])):
    if not r["Kernel_Name"].startswith("void ce::"):
        continue
    per.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
PEAK = 8000.0
alg = bench["roofline"]["algorithmic_bytes_per_launch"]
kern = {}
for name, ds in per.items():
    timed = ds[-steps:] if len(ds) >= steps else ds
    d = {"dispatches": len(ds), "all_mean_ms": statistics.mean(ds), "all_min_ms": min(ds), "all_max_ms": max(ds),
         "timed_dispatches": len(timed), "timed_mean_ms": statistics.mean(timed), "timed_min_ms": min(timed),
         "timed_max_ms": max(timed)}
    if "k_stream" in name:
        d["roofline_frac_from_timed_mean"] = alg / (d["timed_mean_ms"] * 1e-3) / 1e9 / PEAK
    kern[name] = d
pmc = {}
for counter, sub in (("FETCH_SIZE", "fetch_NMC"), ("WRITE_SIZE", "write_NMC")):
    path = os.path.join(prof, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith("void ce::"):
            pmc.setdefault(r["Kernel_Name"], {}).setdefault(counter, []).append(float(r["Counter_Value"]))
for name, c in pmc.items():
    f = statistics.mean(c.get("FETCH_SIZE", [0.0])) * 1024 * 2
    w = statistics.mean(c.get("WRITE_SIZE", [0.0])) * 1024
    kern.setdefault(name, {})["hbm_bytes_per_launch_pmc"] = f + w
    kern[name]["fetch_bytes_per_launch_pmc"] = f
    kern[name]["write_bytes_per_launch_pmc"] = w
out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5",
       "bench_line": bench, "ms_per_step": bench["ms_per_step"], "kernels": kern,
       "note": "timed_* = the last `steps` dispatches (the timed region); all_* include the warm-up dispatches"}
json.dump(out, open(os.path.join(out_dir, f"{tag}_bench_exact.json"), "w"), indent=1)
# bench.py's roofline.traffic: the PMC of the stage-1 kernel this command launched
stage1 = [k for k in kern if "k_stream" in k and "hbm_bytes_per_launch_pmc" in kern[k]]
if stage1:
    k = stage1[0]
    traffic_path = os.path.join(out_dir, "traffic.json")
    traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
    cfg = bench["config"]
    key = f"{cfg['layout']}_{cfg['n_items']}_{cfg['members']}_{cfg['classes']}_q{cfg['q']}_w{bench['n_gpus']}"
    traffic[key] = {"kernel": k, "hbm_bytes_per_launch": kern[k]["hbm_bytes_per_launch_pmc"],
                    "fetch_bytes": kern[k]["fetch_bytes_per_launch_pmc"],
                    "write_bytes": kern[k]["write_bytes_per_launch_pmc"],
                    "source": f"profiles/{tag}_bench_exact.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
                              f"bench.py; FETCH x 2 per the gfx950 rule + WRITE)"}
    json.dump(traffic, open(traffic_path, "w"), indent=1)
rows = list(csv.reader(open(os.path.join(tdir, "run_kernel_stats.csv"))))
head, body = rows[0], rows[1:]
body.sort(key=lambda r: (not r[0].startswith("void ce::"), -float(r[2])))
for r in body:
    r[0] = r[0][:160]
with open(os.path.join(out_dir, f"{tag}_bench_exact_kernel_stats.csv"), "w", newline="") as f:
    wr = csv.writer(f)
    wr.writerow(head)
    wr.writerows(body)
for name, d in kern.items():
    print(name[:70], {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items()})
