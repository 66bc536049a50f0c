"""What sets the per-call SpMV time of the moderate circuits (diagnostics):
each matrix is timed as given and as structural variants of itself, hot
(20 back-to-back rsp_spmv calls between one event pair, median of rounds).

    python scripts/percall_probe.py [names] [--rounds 5]

Variants: "orig"; "short" = rows longer than 1024 entries cut to their first
64 (no long-row chunks); "band" = every row keeps its length but its columns
become a contiguous run around the diagonal (gathers local, no L1 misses).
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


def variant(A, kind):
    rp = np.asarray(A.rowptr[:A.m + 1], np.int64)
    ci = np.asarray(A.colidx[:A.nnz_stored], np.int32)
    va = np.asarray(A.values[:A.nnz_stored], np.float64)
    if kind == "orig":
        return rp.astype(np.int32), ci, va
    lens = np.diff(rp)
    if kind.startswith("cap") and kind.endswith("band"):  # rows cut to N entries, banded
        cap = int(kind[3:-4])
        lens = np.diff(rp)
        keep = np.minimum(lens, cap)
        idx = np.concatenate([np.arange(s, s + k) for s, k in zip(rp[:-1], keep)])
        nrp = np.concatenate([[0], np.cumsum(keep)])
        return variant_band(nrp, ci[idx], va[idx], A.n)
    if kind == "shortband":
        return variant_band(*variant(A, "short"), A.n)
    if kind == "short":
        keep = np.minimum(lens, np.where(lens > 1024, 64, lens))
        starts = rp[:-1]
        idx = np.concatenate([np.arange(s, s + k) for s, k in zip(starts, keep)]) if len(keep) else np.zeros(0, np.int64)
        nrp = np.concatenate([[0], np.cumsum(keep)])
        return nrp.astype(np.int32), ci[idx], va[idx]
    if kind == "band":
        return variant_band(rp, ci, va, A.n)
    raise ValueError(kind)


def variant_band(rp, ci, va, n):
    rp = np.asarray(rp, np.int64)
    m = len(rp) - 1
    if True:
        lens = np.minimum(np.diff(rp), n)
        first = np.clip(np.arange(m) - lens // 2, 0, n - lens)
        nrp = np.concatenate([[0], np.cumsum(lens)])
        row = np.repeat(np.arange(m), lens)
        nci = (first[row] + (np.arange(nrp[-1]) - nrp[row])).astype(np.int32)
        return nrp.astype(np.int32), nci, va[:nrp[-1]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="?", default="ASIC_320ks,ss1,dc1,G2_circuit,matrix-new_3,Baumann,2cubes_sphere")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="orig,short,band,shortband")
    ap.add_argument("--floor", action="store_true",
                    help="also time a one-element kernel and device copies of 4-64 MB the same way")
    ap.add_argument("--spmv-variants", default="0", help="RSP_SPMV_VARIANT per handle (16: no spreading)")
    args = ap.parse_args()
    hs = {}
    for v in args.spmv_variants.split(","):
        os.environ["RSP_SPMV_VARIANT"] = v
        hs[v] = Handle()
    kinds = args.variants.split(",")
    rows = []
    if args.floor:
        def timed(fn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(args.rounds):
                fn()
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / args.reps)
            return statistics.median(ts)
        one = torch.zeros(1, device="cuda")
        print(f"floor one-element add_   {timed(lambda: one.add_(1.0)):7.2f} us", flush=True)
        for mb in (4, 8, 16, 32, 64):
            src = torch.empty(mb << 19, dtype=torch.uint8, device="cuda")  # read mb/2 + write mb/2
            dst = torch.empty_like(src)
            t = timed(lambda: dst.copy_(src))
            print(f"floor copy {mb:3d} MB moved   {t:7.2f} us {mb * (1 << 20) / t / 1e6:6.2f} TB/s", flush=True)
            del src, dst
    for name in args.names.split(","):
        A = csr.surrogate(name)
        x = torch.from_numpy(csr.dlarnv(1, [0, 0, 0, 1], A.n)[0]).cuda()
        y = torch.empty(A.m, dtype=torch.float64, device="cuda")
        for k, (v, h) in [(k, vh) for k in kinds for vh in hs.items()]:
            rp, ci, va = variant(A, k)
            mat = SpMat(h, *upload_csr(rp, ci, va, torch.float64), A.n)
            call = mat.bind(x, y)
            nnz = int(rp[-1])
            byts = 12 * nnz + 4 * (A.m + 1) + 8 * (A.n + A.m)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(args.rounds):
                call()
                e0.record()
                for _ in range(args.reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / args.reps)
            t = statistics.median(ts)
            rows.append((name, k, nnz, byts, t, mat.plan_info()["tiles"]))
            print(f"{name:14s} {k:9s} v{v:3s} nnz {nnz:8d} {byts / 1e6:6.1f} MB tiles {rows[-1][5]:6d} "
                  f"{t:7.2f} us {byts / t / 1e6:6.2f} TB/s", flush=True)
            del mat


if __name__ == "__main__":
    main()
