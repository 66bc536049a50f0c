"""Runs the ILU factor + L / L^T solves a few times on named surrogates (for
rocprofv3 --kernel-trace --stats: per-kernel time of one configuration).
    python scripts/ilu_kernel_probe.py dc1 offshore [--reps 3] [--fp32]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from respasol_amd import csr  # noqa: E402
from respasol_amd.sparse import Handle, Ilu0, upload_csr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("names", nargs="+")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--fp32", action="store_true")
a = ap.parse_args()
dt = torch.float32 if a.fp32 else torch.float64
h = Handle()
for name in a.names:
    A = csr.surrogate(name)
    rp, ci, va0 = upload_csr(A.rowptr, A.colidx, A.values, dt)
    il = Ilu0(h, rp, ci)
    il.analysis()
    x = torch.ones(A.n, dtype=dt, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for r in range(a.reps):
        va = va0.clone()
        torch.cuda.synchronize()
        ev[0].record()
        il.factor(va)
        ev[1].record()
        z = il.solve_lower(va, x)
        il.solve_lower(va, z, transpose=True)
        ev[2].record()
        torch.cuda.synchronize()
        print(f"{name} rep {r}: factor {ev[0].elapsed_time(ev[1]):.3f} ms solve {ev[1].elapsed_time(ev[2]):.3f} ms",
              flush=True)
