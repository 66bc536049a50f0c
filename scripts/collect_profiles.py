"""Copy one profiling session's summaries (scripts/round_check.sh / profile.sh
output under gpurun_out/<tag>) into profiles/ under a round prefix.

    python scripts/collect_profiles.py gpurun_out/r01j r01
"""
import csv
import json
import os
import shutil
import sys

src, prefix = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(ROOT, "profiles")
tag = os.path.basename(src.rstrip("/"))
shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"{prefix}_kernel_stats.csv"))
shutil.copy(os.path.join(src, "bench_prof.json"), os.path.join(dst, f"{prefix}_bench_under_rocprof.json"))
shutil.copy(os.path.join(src, f"{tag}_pmc.json"), os.path.join(dst, f"{prefix}_pmc.json"))
if os.path.exists(os.path.join(src, f"{tag}_pmc_f32.json")):
    shutil.copy(os.path.join(src, f"{tag}_pmc_f32.json"), os.path.join(dst, f"{prefix}_pmc_f32.json"))
if os.path.exists(os.path.join(src, "roofline_check.txt")):
    shutil.copy(os.path.join(src, "roofline_check.txt"), os.path.join(dst, f"{prefix}_roofline_check.txt"))
with open(os.path.join(src, "stats", "run_kernel_trace.csv")) as f, \
        open(os.path.join(dst, f"{prefix}_spmv_dispatches.csv"), "w", newline="") as g:
    w = csv.writer(g)
    w.writerow(["dispatch", "kernel", "grid_wg", "duration_ns", "vgpr", "sgpr", "lds"])
    for r in csv.DictReader(f):
        if "spmv_tiles" in r["Kernel_Name"]:
            w.writerow([r["Dispatch_Id"], r["Kernel_Name"].split("(")[0],
                        int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1),
                        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                        r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"]])
for name in ("bench.out", "bench_moderate.out", "ilu.out"):
    p = os.path.join(src, name)
    if os.path.exists(p):
        out = {"bench.out": f"{prefix}_bench_big.json", "bench_moderate.out": f"{prefix}_bench_moderate.json",
               "ilu.out": f"{prefix}_ilu_config3.txt"}[name]
        shutil.copy(p, os.path.join(dst, out))
if os.path.exists(os.path.join(src, "ilu.json")):
    shutil.copy(os.path.join(src, "ilu.json"), os.path.join(dst, f"{prefix}_ilu_config3.json"))
print("copied", tag, "->", prefix)
