"""GPU parity of the level-scheduled ILU(0) factor and unit-lower triangular
solves (librsp.so) against the CPU oracle and the SURVEY §8c known answers.
The kernels use the oracle's operation order with explicit fma, so factor
values and solves match bitwise; tolerances (rel 1e-13 / 1e-5 per entry,
normwise 1e-12 / 1e-4 for solves) are asserted as the stated contract."""
import json
import os

import numpy as np
import pytest
import torch

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.sparse import Handle, Ilu0, upload_csr

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat.json")))
NP = {torch.float64: np.float64, torch.float32: np.float32}
TOL = {torch.float64: (1e-13, 1e-12), torch.float32: (1e-5, 1e-4)}


@pytest.fixture(autouse=True)
def level_scheduled_solves(monkeypatch):
    """This file holds the level-scheduled kernels (thin runs, flow launches,
    fat levels) to the reference-order oracle: every analysis here plans
    level-scheduled solves (RSP_ILU_BLOCKS=0). The block-inverse solves of
    deep DAGs, the default there since round 6, are tests/test_gpu_blocks.py."""
    monkeypatch.setenv("RSP_ILU_BLOCKS", "0")


@pytest.fixture(scope="module")
def handle():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    h = Handle()
    yield h
    h.close()


def gpu_ilu(handle, A, dtype, ftz=False, x=None, true_lu=False):
    handle.set_ftz(ftz)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
    il = Ilu0(handle, rp, ci, nnz=A.nnz)
    il.analysis()
    sz = il.zero_pivot()
    if sz >= 0:
        handle.set_ftz(False)
        return None, sz, None, None, il
    il.factor(va)
    zp = il.zero_pivot()
    xx = torch.from_numpy(np.ascontiguousarray(x if x is not None else np.ones(A.n), NP[dtype])).cuda()
    z = il.solve_lower(va, xx)
    y = il.solve_upper(va, z) if true_lu else il.solve_lower(va, z, transpose=True)
    torch.cuda.synchronize()
    assert il.zero_pivot() == zp  # (raises if the factor's flow launch gave up waiting)
    assert il.solve_zero_pivot(il.TRSV_L) == -1  # (raise if a solve's flow launch gave up)
    il.solve_zero_pivot(il.TRSV_U if true_lu else il.TRSV_LT)
    handle.set_ftz(False)
    return va.cpu().numpy(), zp, z.cpu().numpy(), y.cpu().numpy(), il


def oracle_ilu(A, dtype, ftz=False, x=None, true_lu=False):
    v, sz, zp = ob.ilu0(A.rowptr, A.colidx, A.values.astype(NP[dtype]), ftz=ftz)
    xx = np.ascontiguousarray(x if x is not None else np.ones(A.n), NP[dtype])
    z = ob.trsv("lower_n", A.rowptr, A.colidx, v, xx, ftz=ftz)
    y = ob.trsv("upper" if true_lu else "lower_t", A.rowptr, A.colidx, v, z, ftz=ftz)
    return v, sz, zp, z, y


def compare(A, dtype, handle, ftz=False, x=None, true_lu=False):
    v, zp, z, y, il = gpu_ilu(handle, A, dtype, ftz, x, true_lu)
    rv, rsz, rzp, rz, ry = oracle_ilu(A, dtype, ftz, x, true_lu)
    assert rsz == -1 and zp == rzp
    ftol, stol = TOL[dtype]
    scale = np.maximum(np.abs(rv.astype(np.float64)), 1e-300)
    assert np.all(np.abs(v.astype(np.float64) - rv) <= ftol * scale)
    for got, ref in ((z, rz), (y, ry)):
        assert np.linalg.norm(got.astype(np.float64) - ref) <= stol * max(np.linalg.norm(ref), 1e-300)
    # bitwise: same operation order, explicit fma on both sides
    assert np.array_equal(v, rv) and np.array_equal(z, rz) and np.array_equal(y, ry)
    return il


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_bcspwr01_kat(handle, dtype):
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "bcspwr01.mtx"))
    v, zp, z, y, _ = gpu_ilu(handle, A, dtype)
    k = KAT["bcspwr01"]
    assert zp == -1
    assert y[:4].tolist() == k["ilu_LLt_solve_x1_first4"]
    assert np.abs(y).max() == k["ilu_LLt_solve_x1_maxabs"]


def test_b1_ss_structural_zero(handle):
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "b1_ss.mtx"))
    _, sz, _, _, _ = gpu_ilu(handle, A, torch.float64)
    assert sz == KAT["b1_ss"]["structural_zero"]


def test_identity(handle):
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "one.mtx"))
    _, zp, _, y, _ = gpu_ilu(handle, A, torch.float64)
    assert zp == -1 and np.all(y == 1.0)


@pytest.mark.parametrize("fat", [False, True])
def test_numerical_zero_pivot(handle, monkeypatch, fat):
    """u_11 = 0 after the update; with every level forced fat the three
    one-row levels form a flow run (ilu0_flow) that still reports it."""
    if fat:
        monkeypatch.setenv("RSP_ILU_THIN_FACTOR", "0")
        monkeypatch.setenv("RSP_ILU_THIN_SOLVE", "0")
    A = csr.CsrMatrix(0, 3, 3, 7, np.array([0, 2, 4, 7], np.int32),
                      np.array([0, 1, 0, 1, 0, 1, 2], np.int32), np.array([1, 1, 1, 1, 1, 1, 1.0]))
    v, zp, _, _, _ = gpu_ilu(handle, A, torch.float64)
    assert zp == 1


@pytest.mark.parametrize("scale_kernel", [1, 0])
@pytest.mark.parametrize("dtype,ftz,u11", [(torch.float64, False, 0.0), (torch.float32, False, 0.0),
                                           (torch.float32, True, 1e-40), (torch.float32, False, 1e-40)])
def test_lower_triangle_factor_zero_pivot(handle, monkeypatch, scale_kernel, dtype, ftz, u11):
    """A stored lower triangle (no update pairs: the one-launch factor,
    ilu0_scale_lower, or the one-level plan with RSP_ILU_FAC_SCALE=0) whose
    u_11 is 0 (or a denormal, flushed under FTZ): the zero pivot is reported
    and l_21 = a_21 / u_11 has the oracle's bits (inf, or the denormal
    quotient without FTZ)."""
    monkeypatch.setenv("RSP_ILU_FAC_SCALE", str(scale_kernel))
    A = csr.CsrMatrix(0, 3, 3, 6, np.array([0, 1, 3, 6], np.int32), np.array([0, 0, 1, 0, 1, 2], np.int32),
                      np.array([2.0, 1.0, u11, 1.0, 1.0, 1.0]))
    v, zp, _, _, _ = gpu_ilu(handle, A, dtype, ftz=ftz)
    rv, _, rzp = ob.ilu0(A.rowptr, A.colidx, A.values.astype(NP[dtype]), ftz=ftz)
    assert zp == rzp == (1 if (u11 == 0.0 or ftz) else -1)
    assert np.array_equal(v.view(np.uint8), rv.view(np.uint8))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("name,scale", [
    ("2cubes_sphere", 0.1), ("ASIC_320ks", 0.05), ("Baumann", 0.1), ("crashbasis", 0.1),
    ("dc1", 0.1), ("FEM_3D_thermal2", 0.05), ("G2_circuit", 0.1), ("para-10", 0.05),
    ("tmt_unsym", 0.02), ("xenon2", 0.05)])
def test_surrogates(handle, name, scale, dtype):
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, dtype, handle, x=x)


def test_fp32_ftz(handle):
    from respasol_amd._lib import SURR_FTZ_STRESS
    A = csr.surrogate("Goodwin_095", 0.05, flags=SURR_FTZ_STRESS)
    compare(A, torch.float32, handle, ftz=True)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_true_lu_extension(handle, dtype):
    A = csr.surrogate("stomach", 0.05)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, dtype, handle, x=x, true_lu=True)


def _levels(rowptr, colidx, transpose):
    n = len(rowptr) - 1
    lev = np.zeros(n, np.int64)
    order = range(n - 1, -1, -1) if transpose else range(n)
    for i in order:
        row = colidx[rowptr[i]:rowptr[i + 1]]
        low = row[row < i]
        if transpose:
            if low.size:
                np.maximum.at(lev, low, lev[i] + 1)
        elif low.size:
            lev[i] = lev[low].max() + 1
    return int(lev.max()) + 1


def test_levels_reported(handle):
    A = csr.surrogate("ecology2", 0.01)
    il = compare(A, torch.float64, handle)
    lo, up = il.levels()
    assert lo == _levels(A.rowptr, A.colidx, False)
    assert up == _levels(A.rowptr, A.colidx, True)


@pytest.mark.parametrize("name", ["FEM_3D_thermal2", "dc1", "ecology2"])
def test_full_size_moderate(handle, name):
    """Full moderate-set surrogates (config 3 size) fp64, bitwise vs oracle:
    fat levels (FEM), ~10^4 narrow levels with staged long-range terms (dc1),
    thin runs of single-level chunks (ecology2)."""
    A = csr.surrogate(name)
    compare(A, torch.float64, handle)


@pytest.mark.parametrize("group", [2, 4])
@pytest.mark.parametrize("name,scale", [("dc1", 0.2), ("ecology2", 0.05), ("stomach", 0.05),
                                        ("ASIC_320ks", 0.1)])
def test_term_group_variants(handle, monkeypatch, group, name, scale):
    """Thin-run rows padded to term groups of 2 or 4 (pads are exact no-op
    fmas) give the same bits, for L, L^T and the U extension."""
    monkeypatch.setenv("RSP_ILU_GROUP", str(group))
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x, true_lu=True)


@pytest.mark.parametrize("thin_solve,thin_factor", [(0, 0), (1024, 1 << 30), (1, 1)])
@pytest.mark.parametrize("name,scale", [("G2_circuit", 0.2), ("stomach", 0.05), ("ss1", 0.05)])
def test_schedule_variants(handle, monkeypatch, thin_solve, thin_factor, name, scale):
    """Every launch schedule gives the same bits: all levels launched one by
    one (0), all levels in single-workgroup thin runs (max), and mixed."""
    monkeypatch.setenv("RSP_ILU_THIN_SOLVE", str(thin_solve))
    monkeypatch.setenv("RSP_ILU_THIN_FACTOR", str(thin_factor))
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x, true_lu=True)


@pytest.mark.parametrize("waves", [1, 2, 4, 16])
@pytest.mark.parametrize("name,scale", [("dc1", 0.3), ("matrix-new_3", 0.2), ("G2_circuit", 0.3),
                                        ("thermomech_TK", 0.2)])
def test_factor_narrow_waves(handle, monkeypatch, waves, name, scale):
    """Narrow factor runs shared by 1, 2, 4 or 16 waves (a level's rounds on
    one wave, levels round-robin, an LDS counter between them): same bits."""
    monkeypatch.setenv("RSP_ILU_FNARROW_WAVES", str(waves))
    A = csr.surrogate(name, scale)
    compare(A, torch.float64, handle)
    compare(A, torch.float32, handle)


@pytest.mark.parametrize("piece", [1, 700, 1 << 30])
@pytest.mark.parametrize("name,scale", [("dc1", 0.2), ("parabolic_fem", 0.05), ("crashbasis", 0.05)])
def test_factor_plan_pieces(handle, monkeypatch, piece, name, scale):
    """The thin factor runs planned in pieces (in parallel on the host) and
    joined by an empty chunk — one piece per level (1), pieces of ~700
    positions, one piece per run — give the same bits."""
    monkeypatch.setenv("RSP_ILU_PIECE_ITEMS", str(piece))
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x)


@pytest.mark.parametrize("slot,lds,pad,wlds,flong", [(0, 1, 0, 0, 3), (0, 0, 1, 1, 8), (1, 1, 1, 1, 8),
                                                     (1, 1, 1, 0, 3), (1, 1, 0, 1, 1)])
@pytest.mark.parametrize("name,scale", [("FEM_3D_thermal2", 0.1), ("Goodwin_095", 0.1), ("crashbasis", 0.1),
                                        ("ASIC_320ks", 0.1)])
def test_fat_level_paths(handle, monkeypatch, slot, lds, pad, wlds, flong, name, scale):
    """Every level forced fat, through each row kernel: factor rows in the
    slot layout (one round trip for a row's structure), the FacRow + LDS
    kernel and the global-memory path; solve short rows with padded flat terms
    (values loaded with the task; the padded layout needs the 8-term short-row
    cut) or unpadded, rows past 1 / 3 (default) / 8 terms a wave each; wave
    rows chained on LDS broadcast operands or on readlanes — the same bits."""
    monkeypatch.setenv("RSP_ILU_FAT_LONG", str(flong))
    monkeypatch.setenv("RSP_ILU_WAVE_LDS", str(wlds))
    monkeypatch.setenv("RSP_ILU_FAT_SLOT", str(slot))
    monkeypatch.setenv("RSP_ILU_FAT_LDS", str(lds))
    monkeypatch.setenv("RSP_ILU_FAT_PAD", str(pad))
    monkeypatch.setenv("RSP_ILU_THIN_FACTOR", "0")
    monkeypatch.setenv("RSP_ILU_THIN_SOLVE", "0")
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_tiny_and_diagonal(handle, dtype):
    """1x1, a pure diagonal (one level, no terms) and a 2x2 lower-only chain."""
    for rp, ci, va in (([0, 1], [0], [4.0]),
                       (list(range(6)), list(range(5)), [1.0, 2.0, 3.0, 4.0, 5.0]),
                       ([0, 1, 3], [0, 0, 1], [2.0, -1.0, 3.0])):
        n = len(rp) - 1
        A = csr.CsrMatrix(0, n, n, len(ci), np.array(rp, np.int32), np.array(ci, np.int32),
                          np.array(va, np.float64))
        compare(A, dtype, handle, x=np.arange(1, n + 1, dtype=np.float64))
        compare(A, dtype, handle, x=np.arange(1, n + 1, dtype=np.float64), true_lu=True)


def test_empty_matrix(handle):
    """n = 0: analysis, factor and solves are no-ops that succeed."""
    A = csr.CsrMatrix(0, 0, 0, 0, np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0))
    rp = torch.zeros(1, dtype=torch.int32, device="cuda")
    ci = torch.zeros(1, dtype=torch.int32, device="cuda")
    va = torch.zeros(1, dtype=torch.float64, device="cuda")
    il = Ilu0(handle, rp, ci, nnz=0)
    il.analysis()
    assert il.zero_pivot() == -1
    il.factor(va)
    assert il.zero_pivot() == -1
    assert A.n == 0


def test_trsv_analysis_lifecycle(handle):
    """Round 6: rsp_ilu0_analysis leaves the solve plans running on a worker
    thread; rsp_trsv_analysis joins them (either op, repeatable), the first
    solve does it otherwise, and destroying or re-analysing the info while
    they still run is safe. Bad arguments are INVALID_VALUE."""
    from respasol_amd import _lib
    from respasol_amd._lib import rsp
    A = csr.surrogate("dc1", 0.3)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
    # destroyed with the plans still running (the destructor joins them)
    for _ in range(3):
        il = Ilu0(handle, rp, ci, nnz=A.nnz)
        il.analysis()
        del il
    il = Ilu0(handle, rp, ci, nnz=A.nnz)
    # not analysed yet / a bad op
    assert rsp.rsp_trsv_analysis(handle.ptr, _lib.OP_N, il._info) == _lib.STATUS_INVALID_VALUE
    il.analysis()
    assert rsp.rsp_trsv_analysis(handle.ptr, 7, il._info) == _lib.STATUS_INVALID_VALUE
    il.analysis()  # re-analysis while the first analysis' plans may still run
    il.trsv_analysis(transpose=True)
    il.trsv_analysis()  # (already done: returns at once)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    il.factor(va)
    xx = torch.from_numpy(x).cuda()
    z = il.solve_lower(va, xx)
    y = il.solve_lower(va, z, transpose=True)
    rv, _, _ = ob.ilu0(A.rowptr, A.colidx, A.values)
    assert np.array_equal(va.cpu().numpy(), rv)
    assert np.array_equal(z.cpu().numpy(), ob.trsv("lower_n", A.rowptr, A.colidx, rv, x))
    assert np.array_equal(y.cpu().numpy(), ob.trsv("lower_t", A.rowptr, A.colidx, rv, z.cpu().numpy()))
    # n = 0: both analyses succeed
    z0 = torch.zeros(1, dtype=torch.int32, device="cuda")
    e = Ilu0(handle, z0, z0, nnz=0)
    e.analysis()
    e.trsv_analysis()
    e.trsv_analysis(transpose=True)


@pytest.mark.parametrize("thin_solve", [1024, 0])
def test_fp32_fma_single_rounding(handle, monkeypatch, thin_solve):
    """fp32 solves fuse in fp32 (one rounding, fmaf), not in double: for
    a*b + c = 1 + 2^-23 + 2^-24 - 2^-60 (just below a float midpoint) fmaf
    gives 1 + 2^-23, a double fma rounded to float gives 1 + 2^-22."""
    monkeypatch.setenv("RSP_ILU_THIN_SOLVE", str(thin_solve))
    a = np.float32(2.0 ** -12 * (1 + 2.0 ** -18))
    b = np.float32(2.0 ** -12 * (1 - 2.0 ** -18))
    c = np.float32(1 + 2.0 ** -23)
    rp = np.array([0, 1, 3], np.int32)
    ci = np.array([0, 0, 1], np.int32)
    va_h = np.array([1.0, -float(a), 1.0], np.float64)  # L = [[1, 0], [-a, 1]]
    rpd, cid, va = upload_csr(rp, ci, va_h, torch.float32)
    il = Ilu0(handle, rpd, cid)
    il.analysis()
    il.factor(va)
    x = torch.tensor([b, c], dtype=torch.float32, device="cuda")
    z = il.solve_lower(va, x).cpu().numpy()
    assert z[1] == np.float32(1 + 2.0 ** -23), z[1]
    v, _, _ = ob.ilu0(rp, ci, va_h.astype(np.float32))
    assert np.array_equal(z, ob.trsv("lower_n", rp, ci, v, np.array([b, c], np.float32)))


def test_unsorted_or_duplicate_rows_rejected(handle):
    """rsp_ilu0_analysis needs strictly increasing columns per row (the
    diagonal search and the update pairs assume it; csrilu02 requires sorted,
    duplicate-free rows): an unsorted row or a repeated column is
    INVALID_VALUE, never a factor of the wrong pattern."""
    from respasol_amd import RspError
    rp = torch.tensor([0, 2, 4], dtype=torch.int32, device="cuda")
    # row 0 unsorted / duplicate column 0 / a column past n / a negative column
    for cols in ([1, 0, 0, 1], [0, 0, 0, 1], [0, 2, 0, 1], [-1, 0, 0, 1]):
        ci = torch.tensor(cols, dtype=torch.int32, device="cuda")
        il = Ilu0(handle, rp, ci)
        with pytest.raises(RspError) as e:
            il.analysis()
        assert e.value.status == 3
        il.close()
    # the reference fixture with duplicate coordinates (sorted by the loader)
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "unsorted_dups.mtx"))
    rp, ci, _ = upload_csr(A.rowptr, A.colidx, A.values)
    il = Ilu0(handle, rp, ci)
    with pytest.raises(RspError):
        il.analysis()
    il.close()
    # rowptr[n] past the declared nnz: rejected before colidx is read
    rp = torch.tensor([0, 1, 3], dtype=torch.int32, device="cuda")
    ci = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
    il = Ilu0(handle, rp, ci, nnz=2)
    with pytest.raises(RspError) as e:
        il.analysis()
    assert e.value.status == 3
    il.close()


@pytest.mark.parametrize("name,scale", [("ASIC_320ks", 1.0), ("dc1", 1.0), ("FEM_3D_thermal2", 0.2),
                                        ("ecology2", 0.2), ("Goodwin_095", 0.2), ("G2_circuit", 0.3),
                                        ("matrix-new_3", 1.0), ("thermomech_TK", 1.0), ("tmt_unsym", 0.1),
                                        ("crashbasis", 0.3), ("parabolic_fem", 0.2), ("para-10", 0.3)])
def test_device_analysis_same_plan_as_host(handle, monkeypatch, name, scale):
    """rsp_ilu0_analysis validates the pattern, finds the diagonals and builds
    the symbolic factor (update lists, stages, stage order, divisor positions)
    with MI355X kernels; rsp_ilu0_analysis_host builds everything on the
    host. Every array of the plan must be identical (64-bit digest over all of
    them), hub rows (ASIC_320ks: the long-row kernel classes) included — and
    so the per-term half of the L and L^T solve plans, which the device
    analysis builds with MI355X kernels (ilu_an_solve_terms)."""
    import ctypes as C
    from respasol_amd._lib import rsp
    monkeypatch.setenv("RSP_ILU_DIGEST", "1")
    A = csr.surrogate(name, scale)
    rp, ci, _ = upload_csr(A.rowptr, A.colidx, A.values)
    il = Ilu0(handle, rp, ci)
    il.analysis()
    dev = C.c_uint64()
    assert rsp.rsp_ilu0_plan_digest(il._info, C.byref(dev)) == 0
    lo, up, hst = C.c_int(), C.c_int(), C.c_uint64()
    r = np.ascontiguousarray(A.rowptr, np.int32)
    c = np.ascontiguousarray(A.colidx, np.int32)
    assert rsp.rsp_ilu0_analysis_host(A.n, r.ctypes.data, c.ctypes.data, C.byref(lo), C.byref(up),
                                      C.byref(hst), None) == 0
    assert dev.value == hst.value
    assert il.levels() == (lo.value, up.value)
    il.close()


@pytest.mark.parametrize("wave_row", ["0", "8"])
@pytest.mark.parametrize("name,scale", [("dc1", 0.5), ("stomach", 0.05), ("crashbasis", 0.2), ("G2_circuit", 0.2)])
def test_device_analysis_wave_stages(handle, monkeypatch, wave_row, name, scale):
    """The one-wave-per-row stages kernel (an_stages_wave: stages, stable
    stage order, group ends, divisors) forced onto every row longer than
    RSP_AN_WAVE_ROW entries: the plan digest equals the host analysis'."""
    import ctypes as C
    from respasol_amd._lib import rsp
    monkeypatch.setenv("RSP_ILU_DIGEST", "1")
    monkeypatch.setenv("RSP_AN_WAVE_ROW", wave_row)
    A = csr.surrogate(name, scale)
    rp, ci, _ = upload_csr(A.rowptr, A.colidx, A.values)
    il = Ilu0(handle, rp, ci)
    il.analysis()
    dev = C.c_uint64()
    assert rsp.rsp_ilu0_plan_digest(il._info, C.byref(dev)) == 0
    lo, up, hst = C.c_int(), C.c_int(), C.c_uint64()
    r = np.ascontiguousarray(A.rowptr, np.int32)
    c = np.ascontiguousarray(A.colidx, np.int32)
    assert rsp.rsp_ilu0_analysis_host(A.n, r.ctypes.data, c.ctypes.data, C.byref(lo), C.byref(up),
                                      C.byref(hst), None) == 0
    assert dev.value == hst.value
    il.close()


@pytest.mark.parametrize("knobs",[{"RSP_ILU_THIN_SOLVE": "0"}, {"RSP_ILU_THIN_SOLVE": "1"},
                                   {"RSP_ILU_GROUP": "2"}, {"RSP_ILU_FAT_PAD": "0"},
                                   {"RSP_ILU_THIN_TERMS": "64"}, {"RSP_ILU_FAT_LONG": "8"}])
@pytest.mark.parametrize("name,scale", [("dc1", 0.3), ("stomach", 0.05), ("ecology2", 0.05)])
def test_device_solve_terms_same_plan_under_schedule_knobs(handle, monkeypatch, knobs, name, scale):
    """The device-built per-term solve plan equals the host's whatever the
    segment structure: every level fat, single-row thin levels, term groups
    of 2, unpadded fat short rows, tiny thin chunks."""
    import ctypes as C
    from respasol_amd._lib import rsp
    monkeypatch.setenv("RSP_ILU_DIGEST", "1")
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    A = csr.surrogate(name, scale)
    rp, ci, _ = upload_csr(A.rowptr, A.colidx, A.values)
    il = Ilu0(handle, rp, ci)
    il.analysis()
    dev = C.c_uint64()
    assert rsp.rsp_ilu0_plan_digest(il._info, C.byref(dev)) == 0
    hst = C.c_uint64()
    r = np.ascontiguousarray(A.rowptr, np.int32)
    c = np.ascontiguousarray(A.colidx, np.int32)
    assert rsp.rsp_ilu0_analysis_host(A.n, r.ctypes.data, c.ctypes.data, None, None, C.byref(hst), None) == 0
    assert dev.value == hst.value
    il.close()


@pytest.mark.parametrize("waves,order,nsplit,group", [(1, 0, 0, 0), (2, 0, 0, 0), (3, 0, 0, 0), (8, 0, 0, 0),
                                                      (4, 0, 0, 0), (4, 0, 1, 2), (4, 1, 1, 0), (4, 1, 1, 2),
                                                      (4, 1, 0, 4), (4, 1, 0, 2)])
@pytest.mark.parametrize("name,scale", [("dc1", 1.0), ("G2_circuit", 0.5), ("thermomech_TK", 0.5),
                                        ("matrix-new_3", 0.5)])
def test_narrow_runs_on_several_waves(handle, monkeypatch, waves, order, nsplit, group, name, scale):
    """Narrow solve levels of L and L^T shared round-robin by 1-8 waves (an
    LDS counter of completed levels orders them), or on one wave with the
    late groups' y loaded together (RSP_ILU_NARROW_SPLIT, early sums under
    the late loads), in the reference's term order (default) or the split
    order (RSP_ILU_SPLIT=1), groups of 2 / 4 / the plan's choice (0):
    bitwise equal to the oracle in that order for L, L^T and the U
    extension, fp64 and fp32."""
    monkeypatch.setenv("RSP_ILU_NARROW_WAVES", str(waves))
    monkeypatch.setenv("RSP_ILU_SPLIT", str(order))
    monkeypatch.setenv("RSP_ILU_NARROW_SPLIT", str(nsplit))
    if group:
        monkeypatch.setenv("RSP_ILU_GROUP", str(group))
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x, true_lu=True)


@pytest.mark.parametrize("waves,group,pairs", [(4, 0, 1), (2, 0, 1), (3, 2, 1), (4, 4, 1), (4, 0, 0), (3, 4, 0)])
@pytest.mark.parametrize("name,scale", [("dc1", 1.0), ("G2_circuit", 0.5), ("thermomech_TK", 0.5)])
def test_narrow_runs_two_levels_per_turn(handle, monkeypatch, waves, group, pairs, name, scale):
    """Narrow solve runs with two consecutive levels per wave turn (the
    default, RSP_ILU_NARROW_PAIRS=1: the second level reads the first's y from
    the same wave's stores) or one (=0): bitwise equal to the oracle for L and
    L^T (U keeps the one-level turns), fp64 and fp32, odd and even run lengths."""
    monkeypatch.setenv("RSP_ILU_NARROW_PAIRS", str(pairs))
    monkeypatch.setenv("RSP_ILU_NARROW_WAVES", str(waves))
    if group:
        monkeypatch.setenv("RSP_ILU_GROUP", str(group))
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x, true_lu=True)


@pytest.mark.parametrize("flow,wpc,mode", [(0, 8, 0), (1, 4, 0), (1, 8, 0), (1, 16, 0), (1, 4, 1), (1, 16, 1),
                                           (1, 4, 2)])
@pytest.mark.parametrize("name,scale", [("xenon2", 0.3), ("offshore", 0.2), ("cfd2", 0.3), ("ss1", 0.2)])
def test_flow_segments(handle, monkeypatch, flow, wpc, mode, name, scale):
    """Fat solve segments and fat factor levels as one persistent launch each
    (trsv_flow: items start when the y they read exist, read from y itself;
    ilu0_flow: rows start when the u values they read exist, read from the
    values themselves) or a launch per level, 1-4 workgroups per CU, items
    walked statically (mode 0), claimed from the flow counter (mode 1) or by
    workgroup start tickets (mode 2, the default): bitwise equal to the
    oracle for the factor, L, L^T and U."""
    monkeypatch.setenv("RSP_ILU_FLOW", str(flow))
    monkeypatch.setenv("RSP_ILU_FLOW_WPC", str(wpc))
    monkeypatch.setenv("RSP_ILU_FLOW_MODE", str(mode))
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x, true_lu=True)


@pytest.mark.parametrize("exp2", [0, 70, -70, 100])
@pytest.mark.parametrize("name,scale", [("dc1", 0.05), ("xenon2", 0.1)])
def test_ftz_division_any_exponent(handle, exp2, name, scale):
    """FTZ build divisions (ilu0.hip qdiv): operands within [2^-60, 2^60] run
    the float Newton sequence without the denormal-mode switch, others the
    double quotient rounded once; with the matrix scaled by 2^exp2 both
    branches meet the oracle's DAZ/FTZ bits (factor and solves, fp32)."""
    import dataclasses
    A = csr.surrogate(name, scale)
    A = dataclasses.replace(A, values=A.values * (2.0 ** exp2))
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float32, handle, ftz=True, x=x)


@pytest.mark.parametrize("grid_x", [4, 16])
@pytest.mark.parametrize("name,scale", [("xenon2", 0.3), ("offshore", 0.2), ("ss1", 0.2)])
def test_flow_tickets_oversubscribed(handle, monkeypatch, grid_x, name, scale):
    """Start tickets with a flow grid grid_x times the resident one
    (RSP_ILU_FLOW_GRID_X, capped at 1024 workgroups): workgroups start only
    as others end, so the launches finish only through steals (a waiting
    workgroup claims the tickets of those not started) and the rerun of
    yielded items — with recovery off and the oracle's bits."""
    monkeypatch.setenv("RSP_ILU_FLOW", "1")
    monkeypatch.setenv("RSP_ILU_FLOW_MODE", "2")
    monkeypatch.setenv("RSP_ILU_FLOW_RECOVER", "0")
    monkeypatch.setenv("RSP_ILU_FLOW_GRID_X", str(grid_x))
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    compare(A, torch.float64, handle, x=x)
    compare(A, torch.float32, handle, x=x, true_lu=True)


def test_flow_give_up_is_reported(handle, monkeypatch):
    """A persistent (flow) launch whose dependency wait gives up is reported,
    not silent, when recovery is off
    (RSP_ILU_FLOW_RECOVER=0): forced with a zero wait bound
    (RSP_ILU_FLOW_TIMEOUT_US=0) and every level fat, so every level is in a
    flow run. The factor's zero_pivot and the solves' status then raise
    EXECUTION_FAILED; the next call with the normal bound starts clean,
    reports SUCCESS and gives the oracle's bits."""
    from respasol_amd._lib import STATUS_EXECUTION_FAILED, RspError
    monkeypatch.setenv("RSP_ILU_FLOW_RECOVER", "0")
    monkeypatch.setenv("RSP_ILU_THIN_FACTOR", "0")
    monkeypatch.setenv("RSP_ILU_THIN_SOLVE", "0")
    # (G2_circuit is a stored lower triangle: its factor is one level, no
    # flow run, unless it runs over L's levels)
    monkeypatch.setenv("RSP_ILU_FAC_ONE", "0")
    A = csr.surrogate("G2_circuit", 0.1)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
    va0 = va.clone()
    il = Ilu0(handle, rp, ci, nnz=A.nnz)
    il.analysis()
    assert il.zero_pivot() == -1
    ones = torch.ones(A.n, dtype=torch.float64, device="cuda")
    monkeypatch.setenv("RSP_ILU_FLOW_TIMEOUT_US", "0")
    il.factor(va)
    with pytest.raises(RspError) as e:
        il.zero_pivot()
    assert e.value.status == STATUS_EXECUTION_FAILED
    z = il.solve_lower(va, ones)
    il.solve_lower(va, z, transpose=True)
    for which in (il.TRSV_L, il.TRSV_LT):
        with pytest.raises(RspError) as e:
            il.solve_zero_pivot(which)
        assert e.value.status == STATUS_EXECUTION_FAILED
    monkeypatch.setenv("RSP_ILU_FLOW_TIMEOUT_US", "200000")
    va.copy_(va0)
    il.factor(va)
    assert il.zero_pivot() == -1
    z = il.solve_lower(va, ones)
    assert il.solve_zero_pivot(il.TRSV_L) == -1
    y = il.solve_lower(va, z, transpose=True)
    assert il.solve_zero_pivot(il.TRSV_LT) == -1
    _, _, _, rz, ry = oracle_ilu(A, torch.float64)
    rv, _, _ = ob.ilu0(A.rowptr, A.colidx, A.values)
    assert np.array_equal(va.cpu().numpy(), rv)
    assert np.array_equal(z.cpu().numpy(), rz) and np.array_equal(y.cpu().numpy(), ry)


@pytest.mark.parametrize("dtype,ftz", [(torch.float64, False), (torch.float32, False), (torch.float32, True)])
def test_flow_give_up_is_recovered(handle, monkeypatch, dtype, ftz):
    """The same forced give-ups with recovery on (the default): the zero-pivot
    calls restore the factor's input values (copied before every factor with
    flow runs) or keep the solve's x, re-run the call — and every solve made
    after it, whose input it produced — without flow launches, report
    SUCCESS, and the results are the oracle's bits."""
    monkeypatch.setenv("RSP_ILU_THIN_FACTOR", "0")
    monkeypatch.setenv("RSP_ILU_THIN_SOLVE", "0")
    monkeypatch.setenv("RSP_ILU_FLOW_TIMEOUT_US", "0")
    monkeypatch.setenv("RSP_ILU_FAC_ONE", "0")  # the factor's flow runs (see above)
    A = csr.surrogate("G2_circuit", 0.1)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
    il = Ilu0(handle, rp, ci, nnz=A.nnz)
    il.analysis()
    ones = torch.ones(A.n, dtype=dtype, device="cuda")
    handle.set_ftz(ftz)
    il.factor(va)
    handle.set_ftz(False)  # the recovery re-runs in the mode of the call, not the current one
    assert il.zero_pivot() == -1
    handle.set_ftz(ftz)
    # the reference's order: both solves, then their status (GPU/ilu0.cu:284-310):
    # recovering L re-runs the L^T solve that read L's y
    z = il.solve_lower(va, ones)
    y = il.solve_lower(va, z, transpose=True)
    handle.set_ftz(False)
    assert il.solve_zero_pivot(il.TRSV_L) == -1
    assert il.solve_zero_pivot(il.TRSV_LT) == -1
    rv, _, _, rz, ry = oracle_ilu(A, dtype, ftz=ftz)
    assert np.array_equal(va.cpu().numpy(), rv)
    assert np.array_equal(z.cpu().numpy(), rz) and np.array_equal(y.cpu().numpy(), ry)


TESTKIT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "respasol_amd", "lib",
                       "librsp_testkit.so")


@pytest.mark.parametrize("hog_us,bound_us,recover,mode", [(50000, 200000, 1, 2), (100000, 5000, 0, 2),
                                                        (100000, 5000, 1, 0), (100000, 5000, 0, 0)])
def test_flow_launches_beside_an_occupying_kernel(monkeypatch, hog_us, bound_us, recover, mode):
    """the factor and both solves (default
    schedule, flow runs included) beside a kernel on another stream that holds
    all but 8 CUs — one 1024-thread workgroup per CU with the CU's whole LDS,
    bounded by the wall clock (librsp_testkit.so, test-only).
    Start tickets (mode 2, the default): a flow workgroup waits only on
    workgroups that started before it, so the launch runs on the 8 free CUs:
    SUCCESS and the oracle's bits with recovery OFF, even with a 5 ms wait
    bound under a 100 ms occupant — nothing waits for the occupant.
    The static walk (mode 0) needs its whole grid resident: under the 100 ms
    occupant its waits give up past a 5 ms bound; with recovery the
    zero-pivot calls re-run the calls without flow launches (SUCCESS, the
    oracle's bits), without it the factor reports EXECUTION_FAILED — which
    shows the occupant really kept flow workgroups off the CUs."""
    import ctypes
    import time
    from respasol_amd._lib import STATUS_EXECUTION_FAILED, RspError
    tk = ctypes.CDLL(TESTKIT)
    tk.rsp_testkit_occupy.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong]
    monkeypatch.setenv("RSP_ILU_FLOW_TIMEOUT_US", str(bound_us))
    monkeypatch.setenv("RSP_ILU_FLOW_RECOVER", str(recover))
    monkeypatch.setenv("RSP_ILU_FLOW_MODE", str(mode))
    # offshore is a stored lower triangle: its factor runs over L's levels
    # here (RSP_ILU_FAC_ONE=0) so that it has flow runs to block
    monkeypatch.setenv("RSP_ILU_FAC_ONE", "0")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    main, side = torch.cuda.Stream(), torch.cuda.Stream()
    h = Handle(stream=main)
    A = csr.surrogate("offshore", 0.2)
    with torch.cuda.stream(main):
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
        il = Ilu0(h, rp, ci, nnz=A.nnz)
        il.analysis()
        ones = torch.ones(A.n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    assert tk.rsp_testkit_occupy(side.cuda_stream, ncu - 8, hog_us) == 0
    time.sleep(0.01)  # the occupant is resident before the factor's launches
    with torch.cuda.stream(main):
        il.factor(va)
        if mode == 0 and not recover:
            with pytest.raises(RspError) as e:
                il.zero_pivot()
            assert e.value.status == STATUS_EXECUTION_FAILED
            torch.cuda.synchronize()
            return
        assert il.zero_pivot() == -1
    torch.cuda.synchronize()
    assert tk.rsp_testkit_occupy(side.cuda_stream, ncu - 8, hog_us) == 0
    time.sleep(0.01)
    with torch.cuda.stream(main):  # both solves, then their status (the L^T solve reads L's y)
        z = il.solve_lower(va, ones)
        y = il.solve_lower(va, z, transpose=True)
        assert il.solve_zero_pivot(il.TRSV_L) == -1
        assert il.solve_zero_pivot(il.TRSV_LT) == -1
    torch.cuda.synchronize()
    rv, _, _, rz, ry = oracle_ilu(A, torch.float64)
    assert np.array_equal(va.cpu().numpy(), rv)
    assert np.array_equal(z.cpu().numpy(), rz) and np.array_equal(y.cpu().numpy(), ry)


def test_flow_recovery_refuses_overwritten_inputs(handle, monkeypatch):
    """a recovery re-runs the recorded solves from their recorded
    buffers, so it must not run when a later recorded solve wrote over one of
    them. The ping-pong pattern — L: r -> z, then L^T: z -> r — overwrites
    the L solve's x; with forced give-ups (static walk, zero bound) the L
    solve's status is EXECUTION_FAILED instead of a silently wrong re-run.
    With separate buffers the same sequence recovers (the oracle's bits)."""
    from respasol_amd._lib import STATUS_EXECUTION_FAILED, RspError
    monkeypatch.setenv("RSP_ILU_THIN_FACTOR", "0")
    monkeypatch.setenv("RSP_ILU_THIN_SOLVE", "0")
    monkeypatch.setenv("RSP_ILU_FAC_ONE", "0")
    monkeypatch.setenv("RSP_ILU_FLOW_MODE", "0")
    A = csr.surrogate("G2_circuit", 0.1)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
    il = Ilu0(handle, rp, ci, nnz=A.nnz)
    il.analysis()
    il.factor(va)
    assert il.zero_pivot() == -1
    monkeypatch.setenv("RSP_ILU_FLOW_TIMEOUT_US", "0")
    r = torch.ones(A.n, dtype=torch.float64, device="cuda")
    z = torch.empty_like(r)
    il.solve_lower(va, r, y=z)
    il.solve_lower(va, z, y=r, transpose=True)  # writes over the L solve's x
    with pytest.raises(RspError) as e:
        il.solve_zero_pivot(il.TRSV_L)
    assert e.value.status == STATUS_EXECUTION_FAILED
    r = torch.ones(A.n, dtype=torch.float64, device="cuda")
    z = il.solve_lower(va, r)
    y = il.solve_lower(va, z, transpose=True)
    assert il.solve_zero_pivot(il.TRSV_L) == -1
    assert il.solve_zero_pivot(il.TRSV_LT) == -1
    _, _, _, rz, ry = oracle_ilu(A, torch.float64)
    assert np.array_equal(z.cpu().numpy(), rz) and np.array_equal(y.cpu().numpy(), ry)
