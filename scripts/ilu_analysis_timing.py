"""Wall time of the ILU(0) analysis phases (RSP_ILU_TIMING) on named
surrogates (diagnostics only).

    python scripts/ilu_analysis_timing.py ecology2,xenon2
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ.setdefault("RSP_ILU_TIMING", "1")
    import torch
    from respasol_amd import csr
    from respasol_amd.sparse import Handle, Ilu0, upload_csr
    h = Handle()
    for name in sys.argv[1].split(","):
        A = csr.surrogate(name)
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, torch.float64)
        il = Ilu0(h, rp, ci)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        il.analysis()
        print(f"{name}: analysis {1e3 * (time.perf_counter() - t0):.1f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
