"""Per-chunk timing of the prefetching thin solve kernel (diagnostics only):
runs L and L^T solves of the named surrogates with RSP_ILU_TRACE set and
summarises the wall-clock (100 MHz) stamps: the wait at each chunk switch,
the LDS staging, the chunk's levels.

    python scripts/ilu_trace.py ecology2,dc1
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    names = sys.argv[1].split(",")
    out = os.path.join(ROOT, "gpurun_out", "ilu_trace")
    os.makedirs(out, exist_ok=True)
    import torch
    from respasol_amd import csr
    from respasol_amd.sparse import Handle, Ilu0, upload_csr
    for name in names:
        path = os.path.join(out, name + ".txt")
        if os.path.exists(path):
            os.remove(path)
        A = csr.surrogate(name)
        h = Handle()
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, torch.float64)
        il = Ilu0(h, rp, ci)
        il.analysis()
        il.factor(va)
        x = torch.ones(A.n, dtype=torch.float64, device="cuda")
        z = il.solve_lower(va, x)  # warm
        torch.cuda.synchronize()
        os.environ["RSP_ILU_TRACE"] = path
        z = il.solve_lower(va, x)
        il.solve_lower(va, z, transpose=True)
        torch.cuda.synchronize()
        del os.environ["RSP_ILU_TRACE"]
        blocks, cur, levs, curl = [], [], [], []
        for line in open(path):
            if line.startswith("#"):
                if cur:
                    blocks.append(np.array(cur, np.int64))
                    levs.append(np.array(curl, np.int64))
                cur, curl = [], []
                continue
            if line.startswith("L "):
                curl.append([int(v) for v in line.split()[1:]])
                continue
            cur.append([int(v) for v in line.split()])
        if cur:
            blocks.append(np.array(cur, np.int64))
            levs.append(np.array(curl, np.int64))
        for bi, L in enumerate(levs):
            if len(L) > 2:
                clk = os.environ.get("RSP_ILU_TRACE_CLK", "0") != "0"
                d = np.diff(L[:, 1]) * (1.0 if clk else 10.0)
                print(f"{name} solve {bi}: level-to-level {'cycles' if clk else 'ns'}: median {np.median(d):.0f} "
                      f"p10 {np.percentile(d, 10):.0f} p90 {np.percentile(d, 90):.0f} (n={len(d)})")
        for bi, b in enumerate(blocks):
            t = b[:, 1:]
            ok = (t > 0).all(axis=1)
            t = t[ok]
            if len(t) == 0:
                continue
            wait = (t[:, 1] - t[:, 0]) * 10.0  # ns
            stg = (t[:, 2] - t[:, 1]) * 10.0
            lev = (t[:, 3] - t[:, 2]) * 10.0
            gap = np.diff(t[:, 0]) * 10.0
            if t.shape[1] >= 6:  # prefetch issued by wave 0 / the last wave, after the stage
                i0 = (t[:, 4] - t[:, 2]) * 10.0
                i1 = (t[:, 5] - t[:, 2]) * 10.0
                print(f"{name} solve {bi}: prefetch issue ns: wave0 mean {i0.mean():.0f} last wave mean {i1.mean():.0f}")
            print(f"{name} solve {bi}: chunks {len(t)}  mean ns: wait {wait.mean():.0f} "
                  f"stage {stg.mean():.0f} levels {lev.mean():.0f} chunk-to-chunk "
                  f"{gap.mean() if len(gap) else 0:.0f}; total {(wait.sum() + stg.sum() + lev.sum()) / 1e6:.3f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
