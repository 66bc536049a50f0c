"""Summarise the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
scripts/pmc_run.py into profiles/<tag>_pmc.json (read by bench.py as
roofline.traffic).

    python scripts/pmc_summary.py --fetch DIR1 --write DIR2 --meta meta.json --out profiles/r01_pmc.json

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE under-counts wide
streaming reads (128-B requests tallied at 64 B); other widths are
uncalibrated. We calibrate on the diagonal-matrix SpMV launched first by
pmc_run.py, whose bytes are exactly known and which uses the same kernel and
load widths, and apply its bytes-per-counted-byte to the workload launches.
Both raw and corrected numbers are recorded.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys


def load(dirname, counter, kernel="spmv_tiles<double"):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and kernel in r.get("Kernel_Name", ""):
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    rows.sort()
    # one value per dispatch (sum over XCD/agent instances if split)
    agg = {}
    for d, v in rows:
        agg[d] = agg.get(d, 0.0) + v
    return [agg[d] for d in sorted(agg)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--meta", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--workload", default="big")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--commit", default=os.environ.get("RSP_COMMIT"),
                    help="git commit the profiled tree was taken from (the GPU box has no .git)")
    args = ap.parse_args()
    meta = json.load(open(args.meta))
    if args.dtype == "f32":
        meta = meta["f32"]
    tn = "double" if args.dtype == "f64" else "float"
    fetch = load(args.fetch, "FETCH_SIZE", f"spmv_tiles<{tn}")
    write = load(args.write, "WRITE_SIZE", f"spmv_tiles<{tn}")
    nc = meta["calibration"]["launches"]
    nm = len(meta["matrices"])
    cal = meta["calibration"]
    f_cal = sum(fetch[:nc]) / nc * 1024.0
    w_cal = sum(write[:nc]) / nc * 1024.0
    rf = cal["read_bytes"] / f_cal if f_cal else None
    wf = cal["write_bytes"] / w_cal if w_cal else None
    fw, ww = fetch[nc:], write[nc:]
    launches = min(len(fw), len(ww))
    alg = [m["alg_bytes"] for m in meta["matrices"]]
    per = []
    for i in range(launches):
        per.append({"matrix": meta["matrices"][i % nm]["name"], "fetch_raw": fw[i] * 1024.0,
                    "write_raw": ww[i] * 1024.0,
                    "hbm_bytes": fw[i] * 1024.0 * rf + ww[i] * 1024.0 * wf,
                    "alg_bytes": alg[i % nm]})
    # skip the first pass (cold TLB / first touch), average the rest
    steady = per[nm:] if launches > nm else per
    hbm = sum(p["hbm_bytes"] for p in steady) / len(steady)
    algb = sum(p["alg_bytes"] for p in steady) / len(steady)
    per_matrix = {"kernel": f"rsp_k::spmv_tiles<{tn},true,false>",
                  "hbm_bytes_per_launch": round(hbm), "algorithmic_bytes_per_launch": round(algb),
                  "traffic_over_algorithmic": round(hbm / algb, 4)}
    # batched launches (one per <= 32 matrices per pass): same correction
    fb = load(args.fetch, "FETCH_SIZE", f"spmv_tiles_batch<{tn}")
    wb = load(args.write, "WRITE_SIZE", f"spmv_tiles_batch<{tn}")
    batch = None
    nb = min(len(fb), len(wb))
    lpp = meta.get("batch_launches_per_pass", 1)
    if nb >= 2 * lpp and lpp == 1:
        hb = [fb[i] * 1024.0 * rf + wb[i] * 1024.0 * wf for i in range(nb)][1:]  # skip the cold pass
        hbm_b = sum(hb) / len(hb)
        alg_b = float(sum(alg))
        e16 = meta.get("batch_entries_16bit")  # the batch tiles the matrices itself
        if e16 is None:
            e16 = sum(m.get("entries_16bit", 0) for m in meta["matrices"])
        moved_b = alg_b - 2.0 * e16
        batch = {"kernel": f"rsp_k::spmv_tiles_batch<{tn},true,false,true>",
                 "hbm_bytes_per_launch": round(hbm_b), "algorithmic_bytes_per_launch": round(alg_b),
                 "traffic_over_algorithmic": round(hbm_b / alg_b, 4),
                 "moved_bytes_per_launch": round(moved_b), "traffic_over_moved": round(hbm_b / moved_b, 4),
                 "launches": nb}
    top = batch or per_matrix
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import spmv_kernel_sha  # the build bench.py accepts this summary for
    out = {
        "workload": args.workload,
        "dtype": args.dtype,
        "kernel_sha": spmv_kernel_sha(),
        "commit": args.commit,
        "kernel": top["kernel"],
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; corrected by a "
                  "diagonal-matrix calibration launch of the same tile code with exactly known bytes",
        "calibration": {"read_bytes_per_counted_byte": rf, "write_bytes_per_counted_byte": wf,
                        "rows": cal["rows"]},
        "hbm_bytes_per_launch": top["hbm_bytes_per_launch"],
        "algorithmic_bytes_per_launch": top["algorithmic_bytes_per_launch"],
        "traffic_over_algorithmic": top["traffic_over_algorithmic"],
        "batch": batch,
        "per_matrix": per_matrix,
        "per_matrix_last_pass": {p["matrix"]: {"hbm_bytes": round(p["hbm_bytes"]),
                                               "alg_bytes": p["alg_bytes"],
                                               "ratio": round(p["hbm_bytes"] / p["alg_bytes"], 3)}
                                 for p in per[-nm:]},
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "algorithmic_bytes_per_launch",
                                          "traffic_over_algorithmic", "calibration")}))


if __name__ == "__main__":
    main()
