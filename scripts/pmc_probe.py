"""Summarise diagnostic rocprofv3 --pmc passes (scripts/pmc_probe.sh): the
per-dispatch counter values of the kernels named on the command line,
averaged over their dispatches (first dispatch of each kernel skipped), with
the busy fractions the counters imply (MI355X: 256 CUs, 8 XCDs;
GRBM_GUI_ACTIVE is summed over the XCDs, per-CU blocks over the CUs).

    python scripts/pmc_probe.py DIR [DIR ...] --kernels 'spmv_tiles_batch<double,spmv_tiles_batch<float'
"""
import argparse
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--kernels", default="spmv_tiles_batch<double,spmv_tiles_batch<float")
ap.add_argument("--out", default="")
ap.add_argument("--by-grid", action="store_true",
                help="one entry per kernel and grid size (one matrix each, e.g. --set cage13,Si87H76)")
args = ap.parse_args()
kern = args.kernels.split(",")
vals = {k: {} for k in kern}  # kernel -> counter -> {dispatch: value}
for d in args.dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            for k in kern:
                if k in name:
                    kk = k
                    if args.by_grid:
                        kk = f"{k} grid={r.get('Grid_Size', r.get('Grid_Size_X', ''))}"
                        vals.setdefault(kk, {})
                    c = vals[kk].setdefault(r["Counter_Name"], {})
                    disp = (f, int(r["Dispatch_Id"]))
                    c[disp] = c.get(disp, 0.0) + float(r["Counter_Value"])
out = {}
for k, cs in vals.items():
    if not cs:
        continue
    avg = {}
    for c, dv in cs.items():
        xs = [dv[key] for key in sorted(dv)][1:] or list(dv.values())
        avg[c] = sum(xs) / len(xs)
    g = avg.get("GRBM_GUI_ACTIVE")
    derived = {}
    if g:
        cyc = g / 8.0  # per-XCD GPU cycles of the dispatch
        for c in ("TA_TA_BUSY", "TD_TD_BUSY", "TA_ADDR_STALLED_BY_TC_CYCLES", "TD_TC_STALL",
                  "TCP_TCP_TA_DATA_STALL_CYCLES", "TCP_PENDING_STALL_CYCLES", "SQ_BUSY_CYCLES"):
            if c in avg:
                derived[c + "/cu_cycle"] = round(avg[c] / (256.0 * cyc), 4)
    if "SQ_WAVE_CYCLES" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"):
            if c in avg:
                derived[c + "/wave_cycle"] = round(avg[c] / w, 4)
    out[k] = {"avg": {c: round(v) for c, v in sorted(avg.items())}, "derived": derived}
print(json.dumps(out, indent=1))
if args.out:
    json.dump(out, open(args.out, "w"), indent=1)
