"""GPU parity of the block-inverse L / L^T solves of deep DAGs (round 6;
trsv_blocks.hip, plan ilu_blocks.cpp) through the C-ABI.

The kernels follow the oracle's restatement of the block order
(oracle_trsv_blocks_*, rsp_oracle.c) bit for bit; against the reference's
own order (L column ascending, L^T the column sweep) the results differ by
rounding only, asserted within SURVEY 8c's solve tolerance (normwise 1e-12
fp64, 1e-4 fp32)."""
import os

import numpy as np
import pytest
import torch

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.sparse import Ilu0, upload_csr

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NP = {torch.float64: np.float64, torch.float32: np.float32}
STOL = {torch.float64: 1e-12, torch.float32: 1e-4}


@pytest.fixture(scope="module")
def handle():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from respasol_amd.sparse import Handle
    h = Handle()
    yield h
    h.close()


def solve_both(handle, A, dtype, x, ftz=False, alpha=1.0):
    """GPU factor then L and L^T solves; the oracle's factor values (bitwise
    equal to the GPU's, test_gpu_ilu0.py) feed the oracle solves."""
    handle.set_ftz(ftz)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
    il = Ilu0(handle, rp, ci, nnz=A.nnz)
    il.analysis()
    il.factor(va)
    xx = torch.from_numpy(np.ascontiguousarray(x, NP[dtype])).cuda()
    z = il.solve_lower(va, xx, alpha=alpha)
    y = il.solve_lower(va, z, transpose=True, alpha=alpha)
    torch.cuda.synchronize()
    handle.set_ftz(False)
    rv, sz, _ = ob.ilu0(A.rowptr, A.colidx, A.values.astype(NP[dtype]), ftz=ftz)
    assert sz == -1
    assert np.array_equal(va.cpu().numpy(), rv)
    return il, rv, z.cpu().numpy(), y.cpu().numpy()


def check(A, rv, x, z, y, dtype, ftz=False, alpha=1.0):
    xx = np.ascontiguousarray(x, NP[dtype])
    rz = ob.trsv("lower_n_blocks", A.rowptr, A.colidx, rv, xx, alpha=alpha, ftz=ftz)
    ry = ob.trsv("lower_t_blocks", A.rowptr, A.colidx, rv, rz, alpha=alpha, ftz=ftz)
    # the reference's order, for the tolerance
    fz = ob.trsv("lower_n_ref", A.rowptr, A.colidx, rv, xx, alpha=alpha, ftz=ftz).astype(np.float64)
    fy = ob.trsv("lower_t_ref", A.rowptr, A.colidx, rv, z, alpha=alpha, ftz=ftz).astype(np.float64)
    tol = STOL[dtype]
    assert np.linalg.norm(z.astype(np.float64) - fz) <= tol * max(np.linalg.norm(fz), 1e-300)
    assert np.linalg.norm(y.astype(np.float64) - fy) <= tol * max(np.linalg.norm(fy), 1e-300)
    assert np.array_equal(z, rz), f"L solve: {np.count_nonzero(z != rz)} of {z.size} differ"
    assert np.array_equal(y, ry), f"L^T solve: {np.count_nonzero(y != ry)} of {y.size} differ"


@pytest.mark.parametrize("dtype,ftz", [(torch.float64, False), (torch.float32, False), (torch.float32, True)])
@pytest.mark.parametrize("name", ["dc1", "G2_circuit", "matrix-new_3"])
def test_deep_circuits_full_size(handle, name, dtype, ftz):
    """The config-3 deep DAGs at full size take the block solve by default
    (<= 32 rows per level) and match the block-order oracle bit for bit."""
    A = csr.surrogate(name)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    il, rv, z, y = solve_both(handle, A, dtype, x, ftz)
    bl, bt = il.solve_blocks()
    assert bl > 0 and bt > 0
    assert ob.blocks_wanted(0, A.rowptr, A.colidx) and ob.blocks_wanted(1, A.rowptr, A.colidx)
    check(A, rv, x, z, y, dtype, ftz)


@pytest.mark.parametrize("name,scale", [("xenon2", 0.05), ("offshore", 0.05), ("ss1", 0.1), ("cfd2", 0.05),
                                        ("ASIC_320ks", 0.1), ("thermomech_TK", 0.2), ("para-10", 0.1)])
def test_forced_on_other_families(handle, monkeypatch, name, scale):
    """RSP_ILU_BLOCKS=1: every family through the block solve (wide levels:
    full blocks without in-block dependencies; hub rows: long blocks), fp64
    and fp32, a random right-hand side and alpha != 1."""
    monkeypatch.setenv("RSP_ILU_BLOCKS", "1")
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [1, 2, 3, 5], A.n)
    for dtype in (torch.float64, torch.float32):
        il, rv, z, y = solve_both(handle, A, dtype, x, alpha=-0.75)
        assert min(il.solve_blocks()) > 0
        check(A, rv, x, z, y, dtype, alpha=-0.75)


@pytest.mark.parametrize("fixture", ["bcspwr01.mtx", "one.mtx", "random_300.mtx", "empty_rows.mtx"])
def test_small_fixtures(handle, monkeypatch, fixture):
    """The reference's and the edge-case fixtures, forced through blocks."""
    monkeypatch.setenv("RSP_ILU_BLOCKS", "1")
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", fixture))
    rv, sz, _ = ob.ilu0(A.rowptr, A.colidx, A.values)
    if sz >= 0:
        pytest.skip("structural zero: no factor")
    x = np.linspace(-1.0, 2.0, A.n)
    _, rv, z, y = solve_both(handle, A, torch.float64, x)
    check(A, rv, x, z, y, torch.float64)


def test_level_path_still_selectable(handle, monkeypatch):
    """RSP_ILU_BLOCKS=0 at analysis: no block plan, the level-scheduled solve
    in the reference's order (bitwise its oracle)."""
    monkeypatch.setenv("RSP_ILU_BLOCKS", "0")
    A = csr.surrogate("G2_circuit", 0.2)
    x = np.ones(A.n)
    il, rv, z, y = solve_both(handle, A, torch.float64, x)
    assert il.solve_blocks() == (0, 0)
    assert np.array_equal(z, ob.trsv("lower_n", A.rowptr, A.colidx, rv, x))
    assert np.array_equal(y, ob.trsv("lower_t", A.rowptr, A.colidx, rv, z))


def test_solve_reads_the_values_it_is_given(handle):
    """The coefficients are built by each solve from its own values argument:
    a second factor of changed values, then the solves, use the new ones."""
    A = csr.surrogate("dc1", 0.2)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
    il = Ilu0(handle, rp, ci, nnz=A.nnz)
    il.analysis()
    ones = torch.ones(A.n, dtype=torch.float64, device="cuda")
    for scale in (1.0, 1.5):
        vals = A.values * scale
        va.copy_(torch.from_numpy(vals))
        il.factor(va)
        z = il.solve_lower(va, ones)
        y = il.solve_lower(va, z, transpose=True)
        rv, _, _ = ob.ilu0(A.rowptr, A.colidx, vals)
        rz = ob.trsv("lower_n_blocks", A.rowptr, A.colidx, rv, np.ones(A.n))
        assert np.array_equal(z.cpu().numpy(), rz)
        assert np.array_equal(y.cpu().numpy(), ob.trsv("lower_t_blocks", A.rowptr, A.colidx, rv, rz))
