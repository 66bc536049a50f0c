"""Per-call SpMV floor, dissected (verdict r03 item 8): from a rocprofv3
--kernel-trace of scripts/spmv_ab.py --mode hot (back-to-back rsp_spmv calls
of one matrix), per matrix the median kernel duration and the median gap
between the end of one dispatch and the start of the next (the launch / CP
part of a call).

    python scripts/percall_trace.py DIR   # DIR holds *kernel_trace.csv
"""
import csv
import glob
import statistics
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows = [r for r in rows if "spmv_tiles<" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
runs = []  # consecutive dispatches of one grid size = one matrix's hot calls
for r in rows:
    g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if runs and runs[-1]["grid"] == g and s - runs[-1]["end"] < 50_000:
        runs[-1]["d"].append(e - s)
        runs[-1]["gap"].append(s - runs[-1]["end"])
        runs[-1]["end"] = e
    else:
        runs.append({"grid": g, "d": [e - s], "gap": [], "end": e})
print(f"{'grid':>9s} {'calls':>5s} {'kernel us':>10s} {'gap us':>8s} {'call us':>8s}")
tk = tg = 0.0
for u in runs:
    if len(u["d"]) < 5:
        continue
    d = statistics.median(u["d"]) / 1e3
    gp = statistics.median(u["gap"]) / 1e3 if u["gap"] else 0.0
    tk += d
    tg += gp
    print(f"{u['grid']:9d} {len(u['d']):5d} {d:10.2f} {gp:8.2f} {d + gp:8.2f}")
print(f"sum of medians: kernel {tk:.1f} us, gap {tg:.1f} us")
