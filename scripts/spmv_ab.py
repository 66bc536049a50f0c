"""Interleaved A/B timing of SpMV kernel variants in ONE process (guide §5.4
rule 24), plus a device-copy bandwidth reference.

    python scripts/spmv_ab.py [--variants 0,1] [--set big] [--rounds 5] [--dtype f64]

Variants are RSP_SPMV_VARIANT values (bit 0: non-temporal vals/colidx loads).
For each round, every matrix is run with every variant (20 back-to-back calls
between one event pair, the whole set cycled so no matrix stays in the
Infinity Cache); reported: median us and algorithmic GB/s per matrix and the
set aggregate.
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from respasol_amd import csr  # noqa: E402
from respasol_amd.sparse import Handle, SpMat, upload_csr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--set", default="big")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--mode", default="cycled", choices=["cycled", "hot"],
                    help="cycled: one call per matrix per pass over the set (cache-cold, like "
                         "bench.py); hot: --reps back-to-back calls of one matrix")
    args = ap.parse_args()
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    elem = 8 if dt == torch.float64 else 4
    variants = [int(v) for v in args.variants.split(",")]
    handles = {}
    for v in variants:
        os.environ["RSP_SPMV_VARIANT"] = str(v)
        handles[v] = Handle()
    names = csr.surrogate_names({"big": 1, "moderate": 0}[args.set]) if args.set in ("big", "moderate") \
        else args.set.split(",")
    mats = []
    for n in names:
        A = csr.surrogate(n)
        d = upload_csr(A.rowptr, A.colidx, A.values, dt)
        x = torch.from_numpy(csr.dlarnv(1, [0, 0, 0, 1], A.n)[0]).to(dt).cuda()
        y = torch.empty(A.m, dtype=dt, device="cuda")
        per = {v: SpMat(handles[v], *d, A.n) for v in variants}
        mats.append((n, A.spmv_bytes(elem), 2 * A.nnz_stored, per, x, y))
        del A
    # device copy reference: read + write of a 2 GiB buffer
    src = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dst.copy_(src)
    e0.record()
    for _ in range(5):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    copy_gbs = 2 * src.numel() * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    times = {(n, v): [] for n, *_ in mats for v in variants}
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in mats]
    for _ in range(args.rounds):
        for v in variants:
            if args.mode == "hot":
                for n, _b, _f, per, x, y in mats:
                    per[v].spmv(x, y)
                    e0.record()
                    for _ in range(args.reps):
                        per[v].spmv(x, y)
                    e1.record()
                    torch.cuda.synchronize()
                    times[(n, v)].append(e0.elapsed_time(e1) / args.reps * 1e3)
            else:
                for _ in range(args.reps):
                    for (n, _b, _f, per, x, y), (a, b) in zip(mats, evs):
                        a.record()
                        per[v].spmv(x, y)
                        b.record()
                    torch.cuda.synchronize()
                    for (n, *_), (a, b) in zip(mats, evs):
                        times[(n, v)].append(a.elapsed_time(b) * 1e3)
    print(f"device copy (read+write) {copy_gbs:.0f} GB/s")
    tot = {v: 0.0 for v in variants}
    totb = sum(b for _, b, *_ in mats)
    for n, b, f, *_ in mats:
        row = [f"{n:18s}"]
        for v in variants:
            t = statistics.median(times[(n, v)])
            tot[v] += t
            row.append(f"v{v}: {t:8.2f} us {b / t / 1e3:7.0f} GB/s")
        print("  ".join(row))
    for v in variants:
        print(f"variant {v}: set {tot[v]:.1f} us  {totb / tot[v] / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
