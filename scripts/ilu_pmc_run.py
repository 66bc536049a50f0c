"""Workload for rocprofv3 --pmc passes over the ILU solves of one surrogate
(diagnostics only): analysis + factor once, then 3 L and L^T solves.

    rocprofv3 --pmc SQ_... -- python3 scripts/ilu_pmc_run.py ecology2
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from respasol_amd import csr
    from respasol_amd.sparse import Handle, Ilu0, upload_csr
    A = csr.surrogate(sys.argv[1])
    h = Handle()
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, torch.float64)
    il = Ilu0(h, rp, ci)
    il.analysis()
    il.factor(va)
    x = torch.ones(A.n, dtype=torch.float64, device="cuda")
    for _ in range(3):
        z = il.solve_lower(va, x)
        il.solve_lower(va, z, transpose=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
