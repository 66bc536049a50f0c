"""GPU parity of the HIP CSR SpMV (librsp.so through the C-ABI) against the
CPU oracle, on the reference fixtures, surrogates of every structural family
(including circuit matrices with rows longer than one tile), edge cases and
full BASELINE-size matrices.

Tolerance: |y_i - y_oracle_i| <= (len_i + 2) * u * sum_j |a_ij x_j|
with u = 2^-53 (fp64) / 2^-24 (fp32) against the column-order oracle, for
every row. In addition every row must equal the oracle's restatement of the
kernels' canonical summation order (oracle_spmv_canon_*) bit for bit, and
repeated calls must be bitwise identical."""
import os

import numpy as np
import pytest
import torch

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.sparse import Handle, SpMat, upload_csr

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mtx")
EPS = {torch.float64: 2.0 ** -53, torch.float32: 2.0 ** -24}
NP = {torch.float64: np.float64, torch.float32: np.float32}


@pytest.fixture(scope="module")
def handle():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    h = Handle()
    yield h
    h.close()


def run_gpu(handle, A, x, dtype, ftz=False, alpha=1.0, beta=0.0, y0=None):
    handle.set_ftz(ftz)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
    mat = SpMat(handle, rp, ci, va, A.n, nnz=max(A.nnz, A.nnz_stored))
    xd = torch.from_numpy(np.ascontiguousarray(x, NP[dtype])).cuda()
    y = torch.from_numpy(np.ascontiguousarray(y0, NP[dtype])).cuda() if y0 is not None else None
    out = mat.spmv(xd, y, alpha, beta)
    torch.cuda.synchronize()
    res = out.cpu().numpy()
    out2 = mat.spmv(xd, None, alpha, 0.0) if beta == 0.0 else None
    torch.cuda.synchronize()
    handle.set_ftz(False)
    return res, (out2.cpu().numpy() if out2 is not None else None), mat


def same_bits(a, b):
    """Bitwise equality that also treats matching NaNs as equal."""
    return np.array_equal(a.view(np.uint64 if a.dtype == np.float64 else np.uint32),
                          b.view(np.uint64 if b.dtype == np.float64 else np.uint32))


def check(A, x, dtype, handle, ftz=False):
    """GPU y vs the oracle: within the forward-error bound of the column-order
    sum everywhere, and bit-identical to the canonical order for every row;
    deterministic across calls."""
    y, y2, mat = run_gpu(handle, A, x, dtype, ftz)
    v = A.values.astype(NP[dtype])
    xx = x.astype(NP[dtype])
    ref = ob.spmv(A.rowptr, A.colidx, v, xx, ftz=ftz)
    bound = ob.spmv_bound(A.rowptr, A.colidx, v, xx, EPS[dtype])
    fin = np.isfinite(ref)
    err = np.abs(y.astype(np.float64) - ref.astype(np.float64))
    assert np.all(err[fin] <= bound[fin]), f"max excess {np.max(err[fin] - bound[fin])}"
    assert same_bits(y[~fin], ref[~fin]) or np.all(~np.isfinite(y[~fin]))
    canon = ob.spmv(A.rowptr, A.colidx, v, xx, ftz=ftz, order="canon")
    assert same_bits(y, canon), "canonical-order mismatch"
    assert same_bits(y, y2), "not deterministic"
    return y, ref


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("name", ["b1_ss", "bcspwr01", "one"] + [
    "sym_lower", "unsorted_dups", "empty_rows", "rect", "random_300", "pattern_general", "zero_based"])
def test_fixtures(handle, name, dtype):
    A = csr.load_matrix_market(os.path.join(GOLD, name + ".mtx"))
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    y, ref = check(A, x, dtype, handle)
    if name == "one":
        assert np.array_equal(y, x.astype(NP[dtype]))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("name,scale", [
    ("2cubes_sphere", 0.2), ("ASIC_320ks", 0.2), ("dc1", 0.3), ("G2_circuit", 0.3),
    ("ecology2", 0.05), ("crashbasis", 0.2), ("para-10", 0.2), ("ss1", 0.2), ("cage13", 0.05),
    ("ML_Laplace", 0.05), ("Si87H76", 0.1), ("matrix-new_3", 0.3)])
def test_surrogates(handle, name, scale, dtype):
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
    check(A, x, dtype, handle)


def test_long_rows_exercised(handle):
    """ASIC_320ks has hub rows far longer than one tile (fp64 2047 / fp32 4093
    entries): they take the chunked path (finished by the last-arriving chunk)."""
    A = csr.surrogate("ASIC_320ks")
    assert np.diff(A.rowptr).max() > 4093
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    for dt in (torch.float64, torch.float32):
        check(A, x, dt, handle)


def test_long_row_tickets_repeat(handle):
    """Chunked long rows are finished inside the tile kernel by the chunk that
    arrives last (agent-scope atomics; an arrival ticket per row that the last
    arriver resets). Many back-to-back calls, with beta = 0 and beta != 0,
    must give the oracle's bits every time: a ticket left non-zero or a stale
    partial would show up as a wrong or missing y[row]."""
    rng = np.random.default_rng(11)
    n, hub = 20000, 9000  # 5 fp64 chunks / 3 fp32 chunks per hub row
    rows, cols = [], []
    for i in range(n):
        if i % 997 == 0:  # hub rows
            c = np.sort(rng.choice(n, hub, replace=False)).astype(np.int32)
        else:
            c = np.unique(np.clip(i + rng.integers(-30, 31, 5), 0, n - 1)).astype(np.int32)
        cols.append(c)
        rows.append(len(c))
    rp = np.zeros(n + 1, np.int32)
    np.cumsum(rows, out=rp[1:])
    ci = np.concatenate(cols)
    A = csr.CsrMatrix(0, n, n, len(ci), rp, ci, rng.uniform(-1, 1, len(ci)))
    x = rng.uniform(-1, 1, n)
    y0 = rng.uniform(-1, 1, n)
    for dt in (torch.float64, torch.float32):
        v, xx, yy = A.values.astype(NP[dt]), x.astype(NP[dt]), y0.astype(NP[dt])
        canon = ob.spmv(A.rowptr, A.colidx, v, xx, order="canon")
        rp_d, ci_d, va_d = upload_csr(A.rowptr, A.colidx, A.values, dt)
        mat = SpMat(handle, rp_d, ci_d, va_d, n)
        xd = torch.from_numpy(xx).cuda()
        for rep in range(20):
            y = mat.spmv(xd).cpu().numpy()
            assert same_bits(y, canon), f"{dt} call {rep}"
        # beta != 0 on the same workspace: y = 2 A x + 0.5 y0 (hub rows included)
        yd = torch.from_numpy(yy.copy()).cuda()
        got = mat.spmv(xd, yd, 2.0, 0.5).cpu().numpy()
        hubs = np.arange(0, n, 997)
        t = (NP[dt](2.0) * canon + NP[dt](0.5) * yy).astype(NP[dt])
        assert same_bits(got[hubs], t[hubs])
        assert same_bits(mat.spmv(xd).cpu().numpy(), canon)


@pytest.mark.parametrize("pattern", ["random_mix", "alt_1_33", "alt_1_65", "alt_3_129", "alt_2_256"])
def test_heavy_rows_in_short_row_tiles(handle, pattern):
    """Rows of 33-256 entries packed into tiles of short rows are summed by
    the tile's second, eight-lanes-per-row pass (reduce_heavy_rows): the same
    canonical bits as every other row, with up to ~120 such rows in one fp32
    tile (alternating 1- and 33-entry rows) and at every lanes-per-row width."""
    rng = np.random.default_rng(sum(map(ord, pattern)))
    n = 30000
    if pattern == "random_mix":
        lens = np.where(rng.random(n) < 0.1, rng.integers(17, 257, n), rng.choice([0, 1, 2, 3, 5, 8], n))
    else:
        a, b = (int(t) for t in pattern.split("_")[1:])
        lens = np.where(np.arange(n) % 2 == 0, a, b)
    cols = [np.sort(rng.choice(n, int(k), replace=False)).astype(np.int32) for k in lens]
    rp = np.zeros(n + 1, np.int32)
    np.cumsum(lens, out=rp[1:])
    ci = np.concatenate(cols)
    A = csr.CsrMatrix(0, n, n, len(ci), rp, ci, rng.uniform(-1, 1, len(ci)))
    x = rng.uniform(-1, 1, n)
    for dt in (torch.float64, torch.float32):
        check(A, x, dt, handle)


def test_single_dense_row_and_column(handle):
    n = 10000
    rows = [np.arange(n, dtype=np.int32)]  # row 0 dense
    rp = [0, n]
    cols = [np.arange(n, dtype=np.int32)]
    for i in range(1, n):
        cols.append(np.array([0, i], np.int32))  # column 0 dense
        rp.append(rp[-1] + 2)
    ci = np.concatenate(cols)
    rng = np.random.default_rng(3)
    A = csr.CsrMatrix(0, n, n, len(ci), np.array(rp, np.int32), ci, rng.uniform(-1, 1, len(ci)))
    x = rng.uniform(-1, 1, n)
    for dt in (torch.float64, torch.float32):
        check(A, x, dt, handle)
    del rows


def test_empty_and_tiny(handle):
    # all-empty rows
    A = csr.CsrMatrix(0, 5, 5, 0, np.zeros(6, np.int32), np.zeros(0, np.int32), np.zeros(0))
    y, _, _ = run_gpu(handle, A, np.ones(5), torch.float64)
    assert np.array_equal(y, np.zeros(5))
    # 1 x 1
    A = csr.CsrMatrix(0, 1, 1, 1, np.array([0, 1], np.int32), np.array([0], np.int32), np.array([2.5]))
    y, _, _ = run_gpu(handle, A, np.array([4.0]), torch.float64)
    assert y.tolist() == [10.0]


def test_alpha_beta(handle):
    A = csr.surrogate("cfd2", 0.05)
    rng = np.random.default_rng(1)
    x = rng.uniform(-1, 1, A.n)
    y0 = rng.uniform(-1, 1, A.m)
    y, _, _ = run_gpu(handle, A, x, torch.float64, alpha=2.0, beta=-0.5, y0=y0)
    ref = 2.0 * ob.spmv(A.rowptr, A.colidx, A.values, x) - 0.5 * y0
    assert np.allclose(y, ref, rtol=1e-14, atol=1e-13)
    # beta == 0 must not read y (NaN in y is ignored, cuSPARSE semantics)
    y, _, _ = run_gpu(handle, A, x, torch.float64, beta=0.0, y0=np.full(A.m, np.nan))
    assert np.all(np.isfinite(y))


def test_unaligned_pointers_scalar_path(handle):
    """vals/colidx views starting at an odd element disable the 16-B vector
    loads; the scalar instantiation must give the same result."""
    A = csr.surrogate("offshore", 0.05)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    ci = torch.zeros(A.nnz_stored + 1, dtype=torch.int32, device="cuda")
    va = torch.zeros(A.nnz_stored + 1, dtype=torch.float64, device="cuda")
    ci[1:] = torch.from_numpy(A.colidx).cuda()
    va[1:] = torch.from_numpy(A.values).cuda()
    rp = torch.from_numpy(A.rowptr).cuda()
    mat = SpMat(handle, rp, ci[1:], va[1:], A.n)
    y = mat.spmv(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = ob.spmv(A.rowptr, A.colidx, A.values, x)
    assert np.all(np.abs(y - ref) <= ob.spmv_bound(A.rowptr, A.colidx, A.values, x, EPS[torch.float64]))


def test_ftz_flushes_subnormal_products(handle):
    """fp32 + FTZ (nvcc -ftz=true, GPU/Makefile:5): subnormal inputs/products
    are zero; without FTZ they survive. Both match the oracle bitwise."""
    rp = np.array([0, 2, 3], np.int32)
    ci = np.array([0, 1, 1], np.int32)
    vals = np.array([1e-39, 2e-39, 1e-20], np.float64)
    A = csr.CsrMatrix(0, 2, 2, 3, rp, ci, vals)
    x = np.array([1.0, 1e-20])
    y_ieee, _, _ = run_gpu(handle, A, x, torch.float32, ftz=False)
    y_ftz, _, _ = run_gpu(handle, A, x, torch.float32, ftz=True)
    v32, x32 = vals.astype(np.float32), x.astype(np.float32)
    assert np.array_equal(y_ieee, ob.spmv(rp, ci, v32, x32))
    assert np.array_equal(y_ftz, ob.spmv(rp, ci, v32, x32, ftz=True))
    assert y_ieee[0] != 0 and y_ftz[0] == 0 and y_ftz[1] == 0


def test_ftz_stress_surrogate(handle):
    from respasol_amd._lib import SURR_FTZ_STRESS
    A = csr.surrogate("cfd2", 0.1, flags=SURR_FTZ_STRESS)
    x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
    check(A, x, torch.float32, handle, ftz=True)


@pytest.mark.parametrize("name", ["Serena", "ML_Laplace", "Transport"])
def test_full_size_big_set(handle, name):
    """BASELINE config 4 sizes (full surrogate) fp64 against the oracle, plus
    linearity A(2x + z) = 2Ax + Az as a size-independent property."""
    A = csr.surrogate(name)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    y, ref = check(A, x, torch.float64, handle)
    z, _ = csr.dlarnv(1, [1, 2, 3, 5], A.n)
    yz, _, _ = run_gpu(handle, A, z, torch.float64)
    ylin, _, _ = run_gpu(handle, A, 2 * x + z, torch.float64)
    assert np.allclose(ylin, 2 * y + yz, rtol=1e-12, atol=1e-10)


def test_invalid_inputs_are_status_codes(handle):
    from respasol_amd import RspError
    rp = torch.tensor([0, 2], dtype=torch.int32, device="cuda")
    ci = torch.tensor([0, 7], dtype=torch.int32, device="cuda")  # column 7 >= n = 2
    va = torch.ones(2, dtype=torch.float64, device="cuda")
    with pytest.raises(RspError) as e:
        SpMat(handle, rp, ci, va, 2)
    assert e.value.status == 3
    # rowptr[m] past the declared nnz (the colidx / vals length): rejected
    # before any of it is read
    rp3 = torch.tensor([0, 3], dtype=torch.int32, device="cuda")
    ci2 = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
    with pytest.raises(RspError) as e:
        SpMat(handle, rp3, ci2, va, 2)
    assert e.value.status == 3


def test_column_offset_tiles(handle):
    """16-bit column offsets: tiles spanning < 65536 columns read them, wider
    tiles the int32 indices, in one matrix; a partial vector at a tile edge
    decodes its neighbour's offset against the wrong base (clamped to n - 1,
    never read). Rows of 3 put tile edges mid-vector."""
    n = 200003
    rows = []
    for i in range(3001):  # offsets up to 60000 from base 0
        rows.append([0, 30000 + i % 7, 60000])
    for i in range(2999):  # base n - 3
        rows.append([n - 3, n - 2, n - 1])
    for i in range(3000):  # span > 65535: int32 indices
        rows.append([i, 100000 + i, n - 1 - i])
    for i in range(n - len(rows)):  # short banded rows
        r = len(rows)
        rows.append(sorted({max(r - 1, 0), r, min(r + 1, n - 1)}))
    rp = np.zeros(n + 1, np.int32)
    np.cumsum([len(r) for r in rows], out=rp[1:])
    ci = np.concatenate([np.array(r, np.int32) for r in rows])
    rng = np.random.default_rng(11)
    A = csr.CsrMatrix(0, n, n, len(ci), rp, ci, rng.uniform(-1, 1, len(ci)))
    x = rng.uniform(-1, 1, n)
    for dt in (torch.float64, torch.float32):
        check(A, x, dt, handle)


@pytest.mark.parametrize("variant", [1, 16, 17, 32, 33, 64, 128, 80, 256, 257, 512, 1024])
def test_kernel_variants_same_bits(monkeypatch, variant):
    """Every kernel / plan variant (RSP_SPMV_VARIANT: default-policy instead of
    non-temporal loads; small plans not spread over the chip, or every small
    plan spread (bit 9, the round-2 rule); int32 column
    indices only, no 16-bit offsets; no staged tiles, bit 10) gives the same
    bits as the canonical-order oracle, on matrices with short rows, rows
    just above the 256 threshold and chunked hub rows."""
    monkeypatch.setenv("RSP_SPMV_VARIANT", str(variant))
    h = Handle()
    try:
        for name, scale in (("ecology2", 0.05), ("ASIC_320ks", 0.3), ("G2_circuit", 0.3),
                            ("Serena", 0.02), ("cage13", 0.05)):
            A = csr.surrogate(name, scale)
            x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
            for dt in (torch.float64, torch.float32):
                check(A, x, dt, h)
    finally:
        h.close()


@pytest.mark.parametrize("pct", [100, 80, 30])
def test_staged_tiles_same_bits(monkeypatch, pct):
    """Staged tiles (a tile's distinct columns loaded once into LDS as column
    runs, entries reading x by slot index; RSP_SPMV_STAGE_PCT = the largest
    distinct-column share of a tile's entries that is staged): every row
    bitwise the canonical-order oracle for mesh / stencil / random-band /
    circuit structures, odd row lengths (tiles starting inside a 16-B
    vector), a band just wide enough to hit the run cap, single calls and a
    batch, fp64 and fp32."""
    from respasol_amd.sparse import SpmvBatch
    monkeypatch.setenv("RSP_SPMV_STAGE_PCT", str(pct))
    h = Handle()
    try:
        mats = [csr.surrogate(nm, sc) for nm, sc in (("Serena", 0.02), ("atmosmodd", 0.05), ("Si87H76", 0.05),
                                                        ("ecology2", 0.05), ("CurlCurl_2", 0.05), ("G2_circuit", 0.2))]
        rng = np.random.default_rng(3)
        n = 30000  # 7 entries per row, columns in a +-600 band: many short runs per tile
        ci = np.sort(np.clip(np.arange(n)[:, None] + rng.integers(-600, 601, (n, 7)), 0, n - 1), axis=1)
        rows = [np.unique(r) for r in ci]
        rp = np.zeros(n + 1, np.int32)
        np.cumsum([len(r) for r in rows], out=rp[1:])
        cc = np.concatenate(rows).astype(np.int32)
        mats.append(csr.CsrMatrix(0, n, n, len(cc), rp, cc, rng.uniform(-1, 1, len(cc))))
        for dt in (torch.float64, torch.float32):
            xs, ys, ms, refs = [], [], [], []
            for A in mats:
                x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
                check(A, x, dt, h)
                M = SpMat(h, *upload_csr(A.rowptr, A.colidx, A.values, dt), A.n)
                ms.append(M)
                xs.append(torch.from_numpy(x.astype(NP[dt])).cuda())
                ys.append(torch.empty(A.m, dtype=dt, device="cuda"))
                refs.append(ob.spmv(A.rowptr, A.colidx, A.values.astype(NP[dt]), x.astype(NP[dt]), order="canon"))
            SpmvBatch(h, ms, xs, ys).run()
            torch.cuda.synchronize()
            for r, y in zip(refs, ys):
                assert same_bits(y.cpu().numpy(), r)
    finally:
        h.close()


@pytest.mark.parametrize("lst", ["1", "0"])
def test_list_staged_tiles_same_bits(monkeypatch, lst):
    """List-staged tiles (fp64 random-band tiles: an explicit column list
    instead of runs, the matrix re-packed with tiles of <= 1536 entries;
    RSP_SPMV_STAGE_LIST=0 turns them off): cage13 and Si87H76 at full size
    and a ragged random band (tiles starting inside a 16-B vector),
    the plan checked on the host to hold list tiles, then single calls and a
    batch bitwise the canonical-order oracle in both settings (fp32 keeps
    its plan and is covered by test_staged_tiles_same_bits)."""
    import ctypes as C
    from respasol_amd import _lib
    from respasol_amd.sparse import SpmvBatch
    monkeypatch.setenv("RSP_SPMV_STAGE_LIST", lst)
    h = Handle()
    try:
        mats = [csr.surrogate(nm, 1.0) for nm in ("cage13", "Si87H76")]
        rng = np.random.default_rng(11)  # ragged rows (1-15 entries) in a +-20000 band
        n = 60000
        rows = [np.unique(np.clip(i + rng.integers(-20000, 20001, 1 + i % 15), 0, n - 1)) for i in range(n)]
        rp = np.zeros(n + 1, np.int32)
        np.cumsum([len(r) for r in rows], out=rp[1:])
        cc = np.concatenate(rows).astype(np.int32)
        mats.append(csr.CsrMatrix(0, n, n, len(cc), rp, cc, rng.uniform(-1, 1, len(cc))))
        dt = torch.float64
        xs, ys, ms, refs = [], [], [], []
        for A in mats:
            rp = np.ascontiguousarray(A.rowptr, np.int32)
            ci = np.ascontiguousarray(A.colidx, np.int32)
            t, e16, est = C.c_int64(), C.c_int64(), C.c_int64()
            assert _lib.rsp.rsp_spmv_plan_host(A.m, rp.ctypes.data, ci.ctypes.data, int(A.nnz_stored), 0,
                                               C.byref(t), C.byref(e16), C.byref(est)) == 0
            # (with the lists off a few of Si87H76's tiles still qualify for runs)
            assert (est.value > 0.5 * A.nnz_stored) if lst == "1" else est.value < 0.1 * A.nnz_stored
            x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
            ref = ob.spmv(A.rowptr, A.colidx, A.values, x, order="canon")
            M = SpMat(h, *upload_csr(A.rowptr, A.colidx, A.values, dt), A.n)
            xd = torch.from_numpy(x).cuda()
            y = torch.empty(A.m, dtype=dt, device="cuda")
            M.spmv(xd, y)
            torch.cuda.synchronize()
            assert same_bits(y.cpu().numpy(), ref)
            ms.append(M)
            xs.append(xd)
            ys.append(torch.empty(A.m, dtype=dt, device="cuda"))
            refs.append(ref)
        SpmvBatch(h, ms, xs, ys).run()
        torch.cuda.synchronize()
        for r, y in zip(refs, ys):
            assert same_bits(y.cpu().numpy(), r)
    finally:
        h.close()


def test_shared_workspace_alternating(handle):
    """Several matrices may share one SpMV workspace (cusparseSpMV treats it
    as scratch). The schedule lives in each matrix (built at bufferSize), so
    calls alternating A, B, A, B on one shared workspace give the
    canonical-order bits without re-planning (plan generation unchanged)."""
    from respasol_amd import RspError
    from respasol_amd.sparse import SpmvBatch
    A = csr.surrogate("cfd2", 0.05)
    B = csr.surrogate("ASIC_320ks", 0.1)  # different shape, hub rows (long-row tickets)
    xa, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
    xb, _ = csr.dlarnv(2, [0, 0, 0, 1], B.n)
    ma = SpMat(handle, *upload_csr(A.rowptr, A.colidx, A.values), A.n)
    mb = SpMat(handle, *upload_csr(B.rowptr, B.colidx, B.values), B.n)
    shared = torch.empty(1, dtype=torch.uint8, device="cuda")
    ma.buffer = mb.buffer = shared
    info_a, info_b = ma.plan_info(), mb.plan_info()
    ref_a = ob.spmv(A.rowptr, A.colidx, A.values, xa, order="canon")
    ref_b = ob.spmv(B.rowptr, B.colidx, B.values, xb, order="canon")
    dxa, dxb = torch.from_numpy(xa).cuda(), torch.from_numpy(xb).cuda()
    for mat, dx, ref in ((ma, dxa, ref_a), (mb, dxb, ref_b), (ma, dxa, ref_a), (mb, dxb, ref_b)):
        y = mat.spmv(dx).cpu().numpy()
        assert same_bits(y, ref), "shared workspace changed the result"
    assert ma.plan_info() == info_a and mb.plan_info() == info_b
    ya, yb = torch.empty(A.m, dtype=torch.float64, device="cuda"), torch.empty(B.m, dtype=torch.float64, device="cuda")
    # one matrix twice in a batch (round 4: every member has its own long-row
    # tickets in the batch's memory) on the shared workspace: both y exact
    yb2 = torch.empty(B.m, dtype=torch.float64, device="cuda")
    SpmvBatch(handle, [mb, mb], [dxb, dxb], [yb, yb2]).run()
    assert same_bits(yb.cpu().numpy(), ref_b) and same_bits(yb2.cpu().numpy(), ref_b)
    bt = SpmvBatch(handle, [ma, mb], [dxa, dxb], [ya, yb])  # same shared workspace: fine
    bt.run()
    assert same_bits(ya.cpu().numpy(), ref_a) and same_bits(yb.cpu().numpy(), ref_b)
    mb.set_local_cols(B.n)  # B re-planned: the batch's copy of B is stale
    with pytest.raises(RspError) as e:
        bt.run()
    assert e.value.status == 3
    bt.close()


def test_reference_call_sequence_plans_nothing_in_rep0(handle):
    """GPU/spmv.cu:143-195 verbatim (create_csr -> bufferSize -> malloc ->
    SpMV, no preprocess): the schedule is built by bufferSize, so timed call 0
    costs what the later calls do (event pair per call, synchronised)."""
    from respasol_amd import _lib
    from respasol_amd._lib import check, rsp
    import ctypes as C
    A = csr.surrogate("Serena", 0.25)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
    mat = C.c_void_p()
    check(rsp.rsp_create_csr(C.byref(mat), A.m, A.n, A.nnz_stored, C.c_void_p(rp.data_ptr()),
                             C.c_void_p(ci.data_ptr()), C.c_void_p(va.data_ptr()), _lib.R_64F), "create")
    one, zero, size = C.c_double(1.0), C.c_double(0.0), C.c_size_t()
    check(rsp.rsp_spmv_buffer_size(handle.ptr, _lib.OP_N, C.byref(one), mat, C.byref(zero), _lib.R_64F,
                                   C.byref(size)), "bufferSize")
    buf = torch.empty(max(size.value, 1), dtype=torch.uint8, device="cuda")
    x = torch.ones(A.n, dtype=torch.float64, device="cuda")
    y = torch.empty(A.m, dtype=torch.float64, device="cuda")
    times = []
    for _ in range(20):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        check(rsp.rsp_spmv(handle.ptr, _lib.OP_N, C.byref(one), mat, C.c_void_p(x.data_ptr()),
                           C.byref(zero), C.c_void_p(y.data_ptr()), _lib.R_64F, C.c_void_p(buf.data_ptr())),
              "spmv")
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
    med = sorted(times)[len(times) // 2]
    assert times[0] <= 2.0 * med + 0.02, (times[0], med)
    ref = ob.spmv(A.rowptr, A.colidx, A.values, np.ones(A.n), order="canon")
    assert same_bits(y.cpu().numpy(), ref)
    rsp.rsp_destroy_spmat(mat)
