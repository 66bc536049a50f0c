"""Cross-check a bench line's roofline against the rocprofv3 kernel summary
of the same run: the average duration rocprof reports for the dominant
kernel (spmv_tiles_batch<double, ...>) against the line's avg_launch_us, and
frac recomputed from each.

    python scripts/check_roofline.py --stats DIR_OR_CSV --bench bench_prof.json
"""
import argparse
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("--stats", required=True)
ap.add_argument("--bench", required=True)
ap.add_argument("--kernel", default="spmv_tiles_batch<double")
ap.add_argument("--fp32", action="store_true", help="check the line's fp32.roofline (kernel spmv_tiles_batch<float)")
args = ap.parse_args()
path = args.stats
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)[0]
kernel = "spmv_tiles_batch<float" if args.fp32 else args.kernel
row = next(r for r in csv.DictReader(open(path)) if kernel in r["Name"])
b = json.loads(open(args.bench).read().strip().splitlines()[-1])
rf = b["fp32"]["roofline"] if args.fp32 else b["roofline"]
prof_us = float(row["AverageNs"]) / 1e3
bytes_ = rf["bytes_per_launch_avg"]
frac_prof = bytes_ / (prof_us * 1e3) / rf["peak"]
print(json.dumps({"kernel": row["Name"][:80], "calls": int(row["Calls"]), "rocprof_avg_us": round(prof_us, 3),
                  "bench_avg_launch_us": rf["avg_launch_us"],
                  "rel_diff": round(prof_us / rf["avg_launch_us"] - 1, 4),
                  "frac_bench": rf["frac"], "frac_from_rocprof": round(frac_prof, 4),
                  "bench_value": b["value"]}))
