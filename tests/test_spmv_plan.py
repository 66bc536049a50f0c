"""The SpMV schedule on the host (rsp_spmv_plan_host, no device): tiles,
16-bit column offsets and the staged tiles' column runs (spmv.hip
stream_products_staged) decode back to every entry's own column; staged
tiles appear where a tile's distinct columns are few (mesh / stencil), list
tiles (column list instead of runs, fp64) on random-band matrices, neither with
RSP_SPMV_STAGE_LIST=0; RSP_SPMV_STAGE_PCT moves the cut. The GPU tests
(tests/test_gpu_spmv.py) hold the kernels on these plans to the oracle."""
import ctypes as C

import numpy as np
import pytest

from respasol_amd import _lib, csr

R64, R32 = 0, 1  # RSP_R_64F / RSP_R_32F (include/rsp.h)


def plan(A, dt):
    rp = np.ascontiguousarray(A.rowptr, np.int32)
    ci = np.ascontiguousarray(A.colidx, np.int32)
    t, e16, est = C.c_int64(), C.c_int64(), C.c_int64()
    st = _lib.rsp.rsp_spmv_plan_host(A.m, rp.ctypes.data, ci.ctypes.data, int(max(A.nnz, A.nnz_stored)), dt,
                                     C.byref(t), C.byref(e16), C.byref(est))
    return st, t.value, e16.value, est.value


@pytest.mark.parametrize("dt", [R64, R32])
@pytest.mark.parametrize("name,scale,staged", [("Serena", 0.02, True), ("Hook_1498", 0.02, True),
                                               ("atmosmodd", 0.05, True), ("ecology2", 0.05, True),
                                               ("cage13", 1.0, "list"), ("ASIC_320ks", 0.2, None),
                                               ("dc1", 0.3, None)])
def test_plan_decodes(name, scale, staged, dt, monkeypatch):
    A = csr.surrogate(name, scale)
    st, tiles, e16, est = plan(A, dt)
    assert st == 0 and tiles > 0 and 0 <= est <= e16 <= A.nnz_stored
    if staged == "list" and dt == R32:  # list tiles are fp64 only (rsp_kernels.h kStageList)
        assert est == 0
    elif staged:
        assert est > 0.5 * A.nnz_stored
    if staged == "list":
        monkeypatch.setenv("RSP_SPMV_STAGE_LIST", "0")
        st, tiles, e16, est = plan(A, dt)
        assert st == 0 and est == 0


def test_stage_share_knob(monkeypatch):
    A = csr.surrogate("atmosmodd", 0.05)
    got = []
    for pct in (0, 30, 80, 100):
        monkeypatch.setenv("RSP_SPMV_STAGE_PCT", str(pct))
        st, _, e16, est = plan(A, R64)
        assert st == 0
        got.append(est)
    assert got[0] == 0 and got == sorted(got) and got[-1] > 0


def test_plan_odd_rows_and_bands():
    """Rows of 1-9 entries (tiles starting inside a 16-B vector) in a band
    wide enough for many short runs per tile, both dtypes."""
    rng = np.random.default_rng(7)
    n = 20000
    rows = [np.unique(np.clip(i + rng.integers(-700, 701, 1 + i % 9), 0, n - 1)) for i in range(n)]
    rp = np.zeros(n + 1, np.int32)
    np.cumsum([len(r) for r in rows], out=rp[1:])
    ci = np.concatenate(rows).astype(np.int32)
    A = csr.CsrMatrix(0, n, n, len(ci), rp, ci, np.ones(len(ci)))
    for dt in (R64, R32):
        st, tiles, e16, est = plan(A, dt)
        assert st == 0 and tiles > 0 and e16 == len(ci)


def test_plan_list_tiles_ragged_band(monkeypatch):
    """A random band of +-20000 columns with rows of 1-15 entries: every
    fp64 tile has more runs than the table holds, so the plan goes to list
    tiles (re-packed, and each list decodes back to the entries' columns);
    fp32 keeps gathered tiles; RSP_SPMV_STAGE_LIST=0 turns the lists off."""
    rng = np.random.default_rng(11)
    n = 60000
    rows = [np.unique(np.clip(i + rng.integers(-20000, 20001, 1 + i % 15), 0, n - 1)) for i in range(n)]
    rp = np.zeros(n + 1, np.int32)
    np.cumsum([len(r) for r in rows], out=rp[1:])
    ci = np.concatenate(rows).astype(np.int32)
    A = csr.CsrMatrix(0, n, n, len(ci), rp, ci, np.ones(len(ci)))
    st, tiles, e16, est = plan(A, R64)
    assert st == 0 and e16 == len(ci) and est > 0.9 * len(ci)
    assert tiles >= len(ci) // 1536
    st, _, _, est32 = plan(A, R32)
    assert st == 0 and est32 == 0
    monkeypatch.setenv("RSP_SPMV_STAGE_LIST", "0")
    st, _, _, est = plan(A, R64)
    assert st == 0 and est == 0


@pytest.mark.parametrize("shift,staged64,staged32", [(0, True, True), (300_000_000, False, True),
                                                    (600_000_000, False, False)])
def test_plan_no_staging_past_the_x_resource(shift, staged64, staged32):
    """Staged tiles load x through a buffer resource of 0x7ffffffc bytes with
    32-bit byte offsets (spmv.hip stream_products_staged): a tile whose
    columns reach past 0x7ffffffc / sizeof(T) (268 435 455 fp64, 536 870 910
    fp32) must not be staged; it keeps the plain 16-bit column offsets."""
    n = 20000
    rows = [np.arange(max(0, i - 3), min(n, i + 4)) + shift for i in range(n)]
    rp = np.zeros(n + 1, np.int32)
    np.cumsum([len(r) for r in rows], out=rp[1:])
    ci = np.concatenate(rows).astype(np.int32)
    A = csr.CsrMatrix(0, n, shift + n, len(ci), rp, ci, np.ones(len(ci)))
    for dt, want in ((R64, staged64), (R32, staged32)):
        st, tiles, e16, est = plan(A, dt)
        assert st == 0 and e16 == len(ci)
        assert (est > 0.9 * len(ci)) if want else est == 0
