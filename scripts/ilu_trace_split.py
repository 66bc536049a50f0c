"""Per matrix and kernel: launches and summed duration from a rocprofv3
kernel trace of scripts/bench_ilu0.py --fp64-only --reps 1 (diagnostics).
Matrices are told apart by the trsv_stream launches that open each solve."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    path = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    names = sys.argv[2].split(",")
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # each matrix: analysis kernels, then 2 reps (warm-up + 1) of factor + 2 solves
    # split on the analysis kernel (ilu_an_rows) that opens each matrix
    seg, cur = [], None
    for r in rows:
        k = r["Kernel_Name"]
        if "::an_rows(" in k:
            cur = []
            seg.append(cur)
        if cur is not None:
            cur.append(r)
    for name, rs in zip(names, seg):
        agg = defaultdict(lambda: [0, 0.0])
        for r in rs:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k][0] += 1
            agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"== {name} (2 factor + 4 solve calls incl. warm-up)")
        for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
            print(f"  {us / 1e3:9.3f} ms {n:6d} launches  {k[:110]}")


if __name__ == "__main__":
    main()
