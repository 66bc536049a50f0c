"""Bisect the slow SpMV on circuit surrogates: time the kernel on variants of
the same matrix (hub rows truncated, only hub rows, far columns localised)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from respasol_amd import csr  # noqa: E402
from respasol_amd.sparse import Handle, SpMat, upload_csr  # noqa: E402


def timeit(h, rp, ci, va, n, dt=torch.float64, reps=20):
    M = SpMat(h, *upload_csr(rp, ci, va, dt), n)
    x = torch.ones(n, dtype=dt, device="cuda")
    y = torch.empty(len(rp) - 1, dtype=dt, device="cuda")
    M.spmv(x, y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        M.spmv(x, y)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def rebuild(rows):
    rp = np.zeros(len(rows) + 1, np.int32)
    rp[1:] = np.cumsum([len(c) for c, _ in rows])
    ci = np.concatenate([c for c, _ in rows]).astype(np.int32)
    va = np.concatenate([v for _, v in rows])
    return rp, ci, va


def main():
    h = Handle()
    for name in sys.argv[1:] or ["G2_circuit", "ASIC_320ks"]:
        A = csr.surrogate(name)
        rows = [(A.colidx[A.rowptr[i]:A.rowptr[i + 1]], A.values[A.rowptr[i]:A.rowptr[i + 1]])
                for i in range(A.m)]
        lens = np.diff(A.rowptr)
        print(name, "m", A.m, "nnz", A.nnz_stored, "max row", lens.max(), "rows>64", (lens > 64).sum(),
              "rows>2047", (lens > 2047).sum())
        print("  original        ", round(timeit(h, A.rowptr, A.colidx, A.values, A.n), 2), "us")
        t = [(c[:64], v[:64]) for c, v in rows]
        print("  rows cut to 64  ", round(timeit(h, *rebuild(t), A.n), 2), "us")
        t = [(c, v) if len(c) > 64 else (c[:0], v[:0]) for c, v in rows]
        print("  only rows > 64  ", round(timeit(h, *rebuild(t), A.n), 2), "us")
        t = [(np.sort(np.unique(np.clip(c, max(i - 40, 0), min(i + 40, A.n - 1)))),
              v[:len(np.unique(np.clip(c, max(i - 40, 0), min(i + 40, A.n - 1))))]) for i, (c, v) in enumerate(rows)]
        print("  cols localised  ", round(timeit(h, *rebuild(t), A.n), 2), "us")
        for cap in (256, 1024, 2047):
            t = [(c[:cap], v[:cap]) for c, v in rows]
            print(f"  rows cut to {cap:5d}", round(timeit(h, *rebuild(t), A.n), 2), "us")


if __name__ == "__main__":
    main()
