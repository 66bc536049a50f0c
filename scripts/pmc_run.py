"""Workload for the rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE are
collected in separate runs, guide §rocprofv3).

1. calibration: y = D x with a 32 M-row DIAGONAL matrix (fp64). Every byte
   is streamed exactly once (vals 8 B + column index 2 B (16-bit offsets) or
   4 B + rowptr 4 B + x 8 B read, y 8 B written per row), so its FETCH_SIZE/WRITE_SIZE give the counter's
   bytes-per-unit for this kernel's access pattern (the gfx950 FETCH_SIZE
   under-count of wide loads, MI355X_MICROARCH.md §HBM);
2. the bench workload: `--passes` cycles of fp64 SpMV over every matrix of
   the set, one launch per matrix (the same order as bench.py, so no matrix
   is cache-resident);
3. `--passes` batched launches over the whole set (rsp_spmv_batch, the
   bench's default step);
then the same three in fp32 (own calibration; the kernel names carry the
value type, so scripts/pmc_summary.py --dtype f32 separates them).
scripts/pmc_summary.py turns the two CSVs into profiles/<tag>_pmc.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from respasol_amd import csr  # noqa: E402
from respasol_amd.sparse import Handle, SpMat, SpmvBatch, upload_csr  # noqa: E402


def run_dtype(h, args, dt):
    """Calibration + per-matrix passes + batched passes in one dtype; returns
    the meta record of this dtype."""
    elem = 8 if dt == torch.float64 else 4
    n = args.calib_rows
    rp = torch.arange(n + 1, dtype=torch.int32, device="cuda")
    ci = torch.arange(n, dtype=torch.int32, device="cuda")
    va = torch.rand(n, dtype=dt, device="cuda")
    x = torch.rand(n, dtype=dt, device="cuda")
    y = torch.empty(n, dtype=dt, device="cuda")
    D = SpMat(h, rp, ci, va, n)
    for _ in range(3):
        D.spmv(x, y)
    torch.cuda.synchronize()
    # vals + rowptr 4 + x per row, plus the column index: 2 B where the
    # schedule reads 16-bit offsets (rsp_spmv_plan_info), else 4 B
    e16 = D.plan_info()["entries_16bit"]
    calib = {"rows": n, "read_bytes": n * (elem + 4 + 4 + elem) - 2 * e16 + 4, "write_bytes": n * elem,
             "launches": 3, "entries_16bit": e16}
    del D, rp, ci, va, x, y
    names = (csr.surrogate_names(1 if args.set == "big" else 0) if args.set in ("big", "moderate")
             else args.set.split(","))
    mats = []
    for name in names:
        A = csr.surrogate(name)
        d = upload_csr(A.rowptr, A.colidx, A.values, dt)
        xx = torch.from_numpy(csr.dlarnv(1, [0, 0, 0, 1], A.n)[0]).to(dt).cuda()
        mats.append((name, A.spmv_bytes(elem), SpMat(h, *d, A.n), xx,
                     torch.empty(A.m, dtype=dt, device="cuda")))
        del A
    for _ in range(args.passes):
        for name, b, M, xx, yy in mats:
            M.spmv(xx, yy)
    torch.cuda.synchronize()
    B = SpmvBatch(h, [q[2] for q in mats], [q[3] for q in mats], [q[4] for q in mats])
    for _ in range(args.passes):
        B.run()
    torch.cuda.synchronize()
    meta = {"calibration": calib, "set": args.set, "passes": args.passes,
            "batch_launches_per_pass": -(-len(mats) // 32),
            "batch_entries_16bit": B.info()["entries_16bit"],
            "matrices": [{"name": n_, "grid": int(M.buffer.numel()), "alg_bytes": b,
                          "entries_16bit": M.plan_info()["entries_16bit"]}
                         for n_, b, M, _, _ in mats]}
    del B, mats
    torch.cuda.synchronize()
    return meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="big")
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--calib-rows", type=int, default=32 << 20)
    ap.add_argument("--dtypes", default="f64,f32", help="f64 first, then f32 (each its own calibration)")
    ap.add_argument("--meta", default="")
    args = ap.parse_args()
    h = Handle()
    meta = {}
    for d in args.dtypes.split(","):
        m = run_dtype(h, args, torch.float64 if d == "f64" else torch.float32)
        if d == "f64":
            meta.update(m)  # the round-1..3 layout: fp64 at the top level
        else:
            meta[d] = m
    if args.meta:
        with open(args.meta, "w") as f:
            json.dump(meta, f)


if __name__ == "__main__":
    main()
