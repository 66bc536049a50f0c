"""Wall time of the ILU(0) analysis phases (RSP_ILU_TIMING) on named
surrogates (diagnostics only).

    python scripts/ilu_analysis_timing.py ecology2,xenon2 [reps]
    python scripts/ilu_analysis_timing.py moderate [reps]

Each matrix is analysed `reps` times (default 2); the line of every call is
printed, so the later calls show the steady state.
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
    names = csr.surrogate_names(0) if sys.argv[1] == "moderate" else sys.argv[1].split(",")
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    total = [0.0] * reps
    for name in names:
        A = csr.surrogate(name)
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, torch.float64)
        for r in range(reps):
            il = Ilu0(h, rp, ci)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            il.analysis()
            t = 1e3 * (time.perf_counter() - t0)
            total[r] += t
            print(f"{name}: analysis {t:.1f} ms", file=sys.stderr, flush=True)
            del il
    print("total per rep: " + " ".join(f"{t:.1f}" for t in total), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
