"""Randomised GPU parity of ILU(0) + the L / L^T solves (seeded,
reproducible): random patterns — banded, random, clustered, with hub rows
and columns and with deep chains — and strictly diagonally dominant values;
the factor, the L solve and the L^T solve are checked bit for bit against
the oracle (reference operation order), fp64 and fp32, under the shipped
schedule and with every level forced fat (flow launches everywhere)."""
import numpy as np
import pytest
import torch

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.sparse import Handle, Ilu0, upload_csr

pytestmark = pytest.mark.gpu
NP = {torch.float64: np.float64, torch.float32: np.float32}
SEEDS = range(8)


def random_matrix(seed, lower=False):
    """lower: only the stored lower triangle (the symmetric matrices'
    storage): no update pairs, so the factor runs as one level."""
    rng = np.random.default_rng(2000 + seed)
    n = int(rng.choice([5, 400, 6000, 30000]))
    kind = seed % 4
    per = int(rng.integers(2, 9))
    row = np.repeat(np.arange(n), per)
    if kind == 0:  # banded
        col = np.clip(row + rng.integers(-40, 41, row.size), 0, n - 1)
    elif kind == 1:  # random
        col = rng.integers(0, n, row.size)
    elif kind == 2:  # deep chains: mostly i-1, i-2 (thousands of narrow levels)
        col = np.clip(row - rng.integers(0, 3, row.size), 0, n - 1)
    else:  # clustered, with a few hub rows and columns
        centers = rng.integers(0, n, max(1, n // 50))
        col = np.clip(centers[rng.integers(0, centers.size, row.size)] + rng.integers(-16, 17, row.size), 0, n - 1)
        hubs = rng.choice(n, min(n, 3), replace=False)
        row = np.concatenate([row, np.repeat(hubs, min(n, 600)), rng.integers(0, n, 800)])
        col = np.concatenate([col, rng.integers(0, n, hubs.size * min(n, 600)), np.full(800, hubs[0])])
    row = np.concatenate([row, np.arange(n)])  # the diagonal
    col = np.concatenate([col, np.arange(n)])
    key = np.unique(row.astype(np.int64) * n + col)
    row, col = key // n, key % n
    if lower:
        row, col = row[col <= row], col[col <= row]
    rp = np.zeros(n + 1, np.int32)
    np.add.at(rp, row + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    vals = rng.uniform(-1, 1, col.size)
    offsum = np.zeros(n)
    np.add.at(offsum, row, np.where(row != col, np.abs(vals), 0.0))
    vals = np.where(row == col, 1.0 + offsum[row], vals)  # strictly diagonally dominant
    return csr.CsrMatrix(0, n, n, int(col.size), rp, col.astype(np.int32), vals)


@pytest.mark.parametrize("lower", [0, 1, 2])
@pytest.mark.parametrize("fat", [False, True])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_random_patterns_bitwise(monkeypatch, dtype, fat, lower):
    """lower 1 / 2: stored lower triangles (no update pairs), factored in
    one launch (ilu0_scale_lower, 1) or as ONE level of the factor plan
    (RSP_ILU_FAC_SCALE=0, 2: a row's divisor u_kk may be in the same level —
    thin runs stage its input, fat levels read it while its row rewrites the
    same bits)."""
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    if lower == 2:
        monkeypatch.setenv("RSP_ILU_FAC_SCALE", "0")
    if fat:
        monkeypatch.setenv("RSP_ILU_THIN_FACTOR", "0")
        monkeypatch.setenv("RSP_ILU_THIN_SOLVE", "0")
    h = Handle()
    for seed in SEEDS:
        A = random_matrix(seed, lower > 0)
        v, sz, zp = ob.ilu0(A.rowptr, A.colidx, A.values.astype(NP[dtype]))
        assert sz == -1 and zp == -1
        x = np.random.default_rng(seed).uniform(-1, 1, A.n).astype(NP[dtype])
        rz = ob.trsv("lower_n", A.rowptr, A.colidx, v, x)
        ry = ob.trsv("lower_t", A.rowptr, A.colidx, v, rz)
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
        il = Ilu0(h, rp, ci, nnz=A.nnz)
        il.analysis()
        il.factor(va)
        assert il.zero_pivot() == -1
        z = il.solve_lower(va, torch.from_numpy(x).cuda())
        y = il.solve_lower(va, z, transpose=True)
        assert il.solve_zero_pivot(il.TRSV_L) == -1 and il.solve_zero_pivot(il.TRSV_LT) == -1
        assert np.array_equal(va.cpu().numpy(), v), (seed, "factor")
        assert np.array_equal(z.cpu().numpy(), rz), (seed, "L")
        assert np.array_equal(y.cpu().numpy(), ry), (seed, "L^T")
        del il
    h.close()
