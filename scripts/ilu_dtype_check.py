import sys, os, torch, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from respasol_amd import csr
from respasol_amd.sparse import Handle, Ilu0, upload_csr
A = csr.surrogate(sys.argv[1])
h = Handle()
for dt, ftz in ((torch.float64, False), (torch.float32, False), (torch.float32, True)):
    h.set_ftz(ftz)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dt)
    il = Ilu0(h, rp, ci); il.analysis(); il.factor(va)
    x = torch.ones(A.n, dtype=dt, device="cuda")
    for _ in range(2): z = il.solve_lower(va, x); il.solve_lower(va, z, transpose=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5): z = il.solve_lower(va, x); il.solve_lower(va, z, transpose=True)
    e1.record(); torch.cuda.synchronize()
    print(sys.argv[1], dt, "ftz" if ftz else "", round(e0.elapsed_time(e1) / 5, 3), "ms")
