"""Per-level cost of the level-scheduled solves and factor on synthetic DAGs
of fixed shape (diagnostics only): W interleaved chains (row i depends on
rows i-W, i-2W, ..., i-T*W), so every level holds W rows of T terms.

    python scripts/ilu_levelcost.py [--n 60000]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from respasol_amd.sparse import Handle, Ilu0, upload_csr  # noqa: E402


def chains(n, W, T):
    rows = []
    for i in range(n):
        cols = [i - k * W for k in range(T, 0, -1) if i - k * W >= 0] + [i]
        rows.append(cols)
    rp = np.zeros(n + 1, np.int32)
    np.cumsum([len(r) for r in rows], out=rp[1:])
    ci = np.concatenate([np.array(r, np.int32) for r in rows])
    rng = np.random.default_rng(1)
    va = rng.uniform(-0.1, 0.1, len(ci))
    va[rp[1:] - 1] = 1.0 + T * 0.1  # diagonal last in each row
    return rp, ci, va


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=60000)
    args = ap.parse_args()
    h = Handle()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for W, T in ((1, 1), (10, 1), (10, 2), (10, 4), (10, 6), (30, 3), (64, 3), (100, 3)):
        rp, ci, va = chains(args.n, W, T)
        drp, dci, dva = upload_csr(rp, ci, va)
        il = Ilu0(h, drp, dci)
        il.analysis()
        lv = il.levels()[0]
        x = torch.ones(args.n, dtype=torch.float64, device="cuda")
        best_f, best_s = 1e9, 1e9
        for _ in range(3):
            v = dva.clone()
            torch.cuda.synchronize()
            e[0].record()
            il.factor(v)
            e[1].record()
            z = il.solve_lower(v, x)
            e[2].record()
            torch.cuda.synchronize()
            best_f = min(best_f, e[0].elapsed_time(e[1]))
            best_s = min(best_s, e[1].elapsed_time(e[2]))
        print(f"W={W:3d} T={T}: levels {lv:6d}  factor {best_f:7.3f} ms = {best_f * 1e6 / lv:6.0f} ns/level   "
              f"L solve {best_s:7.3f} ms = {best_s * 1e6 / lv:6.0f} ns/level", flush=True)
        il.close()


if __name__ == "__main__":
    main()
