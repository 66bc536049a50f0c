"""Per-chunk timing of the thin-run factor kernel (diagnostics only): factors
the named surrogates with RSP_ILU_FTRACE set and summarises the shader-clock
stamps per chunk: LDS staging (incl. the wait for the prefetch), the chunk's
rounds, and cycles per round.

    python scripts/ilu_ftrace.py dc1,G2_circuit
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from respasol_amd import csr
    from respasol_amd.sparse import Handle, Ilu0, upload_csr
    out = os.path.join(ROOT, "gpurun_out", "ilu_ftrace")
    os.makedirs(out, exist_ok=True)
    for name in sys.argv[1].split(","):
        path = os.path.join(out, name + ".txt")
        if os.path.exists(path):
            os.remove(path)
        A = csr.surrogate(name)
        h = Handle()
        rp, ci, va0 = upload_csr(A.rowptr, A.colidx, A.values, torch.float64)
        il = Ilu0(h, rp, ci)
        il.analysis()
        va = va0.clone()
        il.factor(va)  # warm
        torch.cuda.synchronize()
        os.environ["RSP_ILU_FTRACE"] = path
        va = va0.clone()
        il.factor(va)
        torch.cuda.synchronize()
        del os.environ["RSP_ILU_FTRACE"]
        rows = [list(map(int, l.split())) for l in open(path) if not l.startswith("#")]
        t = np.array(rows, dtype=np.float64)
        if not len(t):
            print(name, "no thin chunks")
            continue
        stage, rnd = t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
        nr, ni = t[:, 4], t[:, 5]
        print(f"{name}: {len(t)} chunks, {int(nr.sum())} rounds, {int(ni.sum())} items; cycles: staging "
              f"{stage.sum():.3g} ({stage.mean():.0f}/chunk), rounds {rnd.sum():.3g} "
              f"({rnd.sum() / max(nr.sum(), 1):.0f}/round); rounds/chunk median {np.median(nr):.0f}, "
              f"items/chunk median {np.median(ni):.0f}")


if __name__ == "__main__":
    main()
