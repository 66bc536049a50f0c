"""Host-side product logic that needs no GPU: the C-ABI libraries load and
export every symbol declared in include/*.h, the surrogate generator's
contracts, the row partitioner, and the CPU reference-CLI driver."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_bind as ob
from respasol_amd import _lib, csr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
BIN = os.path.join(ROOT, "respasol_amd", "bin")


def header_functions(path):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return sorted(set(re.findall(r"\b([A-Za-z_]\w*)\s*\(", text)) - {
        "if", "sizeof", "defined", "return", "while", "for"} - {"extern"})


@pytest.mark.parametrize("header,lib,protos", [
    ("rsp.h", "rsp", _lib.RSP_PROTOS), ("rsp_host.h", "host", _lib.HOST_PROTOS)])
def test_every_declared_symbol_is_exported_and_bound(header, lib, protos):
    funcs = [f for f in header_functions(os.path.join(ROOT, "include", header))
             if f.startswith(("rsp_", "load"))]
    assert funcs, header
    L = getattr(_lib, lib)
    for f in funcs:
        assert hasattr(L, f), f"{f} declared in {header} but not exported"
        assert f in protos, f"{f} has no ctypes prototype"
    assert set(protos) <= set(funcs)


def test_native_version_and_error_strings():
    import respasol_amd
    assert respasol_amd.native_version() == 1
    assert _lib.rsp.rsp_get_error_string(9) == b"RSP_STATUS_ZERO_PIVOT"


def test_library_has_gfx950_code_object():
    so = os.path.join(_lib.LIB_DIR, "librsp.so")
    blob = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob  # gfx950 only


# ------------------------------------------------------------ surrogates

@pytest.mark.parametrize("name", ["Serena", "ASIC_320ks", "G2_circuit", "ecology2", "cage13",
                                  "ML_Laplace", "af_shell2", "Si87H76"])
def test_surrogate_contract(name):
    info = csr.surrogate_info(name)
    A = csr.surrogate(name, 0.02)
    rows = np.repeat(np.arange(A.m), np.diff(A.rowptr))
    # sorted, unique columns per row; diagonal present
    d = np.diff(A.colidx)
    newrow = np.diff(rows) != 0
    assert np.all((d > 0) | newrow)
    diag = A.colidx == rows
    assert np.bincount(rows[diag], minlength=A.m).min() == 1
    if info["symmetric"]:
        assert np.all(A.colidx <= rows)
    # strict row diagonal dominance over the stored row
    absrow = np.bincount(rows, weights=np.abs(A.values), minlength=A.m)
    assert np.all(A.values[diag] * 2 > absrow)
    # row-local: any slice equals the same rows of the whole matrix
    r0, r1 = A.m // 3, A.m // 3 + A.m // 4
    rp, ci, va = csr.surrogate_rows_csr(name, r0, r1, 0.02)
    s, e = A.rowptr[r0], A.rowptr[r1]
    assert np.array_equal(rp, A.rowptr[r0:r1 + 1] - s)
    assert np.array_equal(ci, A.colidx[s:e])
    assert np.array_equal(va, A.values[s:e])


def test_surrogate_sizes_match_catalog():
    for name in csr.surrogate_names():
        info = csr.surrogate_info(name)
        lens = csr.surrogate_rowlens(name)
        assert len(lens) == info["m"]
        assert abs(int(lens.sum()) - info["nnz_target"]) <= 1e-3 * info["nnz_target"], name
    assert len(csr.surrogate_names(0)) == 21 and len(csr.surrogate_names(1)) == 15


def test_surrogate_ftz_stress_has_fp32_subnormals():
    A = csr.surrogate("cfd2", 0.02, flags=_lib.SURR_FTZ_STRESS)
    v32 = A.values.astype(np.float32)
    sub = (v32 != 0) & (np.abs(v32) < np.finfo(np.float32).tiny)
    assert sub.sum() > 0


def test_custom_surrogate_spec():
    A = csr.surrogate("stencil3d:1000:7000:G")
    assert A.m == 1000 and abs(A.nnz_stored - 7000) < 100


# ------------------------------------------------------------ partition

def test_partition_rows_balanced():
    A = csr.surrogate("ASIC_320ks", 0.05)
    for P in (1, 2, 3, 4, 8):
        b = csr.partition_rows(A.rowptr, P)
        assert b[0] == 0 and b[-1] == A.m and np.all(np.diff(b) >= 0)
        nnz = A.rowptr[b[1:]] - A.rowptr[b[:-1]]
        assert nnz.sum() == A.nnz_stored
        assert nnz.max() <= A.nnz_stored / P + np.diff(A.rowptr).max()
    b = csr.partition_rows(np.array([0, 1, 2], np.int32), 4)  # P > m
    assert b.tolist()[0] == 0 and b.tolist()[-1] == 2


# ------------------------------------------------------------ CPU driver

def test_cpu_driver_csv_schema(tmp_path):
    out = tmp_path / "bench.csv"
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for f in ("b1_ss", "bcspwr01", "one"):
        r = subprocess.run([os.path.join(BIN, "test_spmv_cpu"), os.path.join(GOLD, "mtx", f + ".mtx"),
                            str(out)], env=env, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    r = subprocess.run([os.path.join(BIN, "test_spmv_cpu"),
                        os.path.join(tmp_path, "matrix-new_3.mtx"), str(out)], env=env,
                       capture_output=True, text=True)
    assert r.returncode != 0  # missing file exits non-zero (reference: exit(-1))
    lines = out.read_text().splitlines()
    assert len(lines) == 4
    for line, name in zip(lines, ("b1_ss", "bcspwr01", "one")):
        f = line.split(",")
        assert f[0] == "2" and f[1] == name and f[-1] == ""
        float(f[2]), float(f[3])
        assert float(f[4]) < 1e-6  # fp32-vs-fp64 mean difference
    # the missing-file run wrote only the thread field before exiting
    assert lines[3] == "2,"


def test_cpu_driver_name_regex(tmp_path):
    # (\w+)\.mtx keeps only the word run: matrix-new_3 -> new_3 (test_spmv.c:57-62)
    src = os.path.join(GOLD, "mtx", "one.mtx")
    dst = tmp_path / "matrix-new_3.mtx"
    dst.write_text(open(src).read())
    out = tmp_path / "o.csv"
    subprocess.run([os.path.join(BIN, "test_spmv_cpu"), str(dst), str(out)], check=True,
                   env=dict(os.environ, OMP_NUM_THREADS="1"), capture_output=True)
    assert out.read_text().split(",")[1] == "new_3"


def test_cpu_driver_error_matches_oracle(tmp_path):
    """err column = mean |y64 - y32| with x = dlarnv(1,{0,0,0,1}) (test_spmv.c:200-208)."""
    out = tmp_path / "o.csv"
    spec = "surrogate:cfd2@0.05"
    subprocess.run([os.path.join(BIN, "test_spmv_cpu"), spec, str(out)], check=True,
                   env=dict(os.environ, OMP_NUM_THREADS="3"), capture_output=True)
    err = float(out.read_text().split(",")[4])
    A = csr.surrogate("cfd2", 0.05)
    x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
    y64 = ob.spmv(A.rowptr, A.colidx, A.values, x)
    y32 = ob.spmv(A.rowptr, A.colidx, A.values.astype(np.float32), x.astype(np.float32))
    ref = np.abs(y64 - y32.astype(np.float64)).mean()
    assert err == pytest.approx(ref, rel=1e-5)


def test_gpu_drivers_usage_without_args():
    for exe in ("test_spmv", "test_ilu0", "spmv", "ilu0", "test_spmv_cpu"):
        r = subprocess.run([os.path.join(BIN, exe)], capture_output=True, text=True)
        assert r.returncode == 255 and "Usage examples" in r.stderr


def test_buffer_loader_stays_inside_len():
    """rsp_mm_load_buffer does not require a NUL at buf[len]: a number cut by
    `len` must parse only the bytes inside it (here '2.5', not '2.5e7')."""
    import ctypes as C
    text = b"%%MatrixMarket matrix coordinate real general\n1 1 1\n1 1 2.5"
    raw = C.create_string_buffer(text + b"e7 9 9 9", len(text) + 8)
    s = _lib.CSRStruct()
    st = _lib.host.rsp_mm_load_buffer(C.cast(raw, C.c_char_p), len(text), C.byref(s), 0, 0, _lib.MM_QUIET)
    assert st == 0
    A = csr._from_struct(s, 0)
    assert A.values.tolist() == [2.5]


def test_padded_allgather_layout_c_matches_python():
    """rsp_padded_chunk / rsp_remap_cols_padded (the C driver's --ngpu layout)
    equal dist.padded_layout / remap_columns, and an emulated equal-count
    all-gather of the slices through that layout reproduces the global x at
    every remapped column (the exchange logic, no GPU)."""
    import ctypes as C
    from respasol_amd import _lib
    from respasol_amd.dist import remap_columns
    A = csr.surrogate("G2_circuit", 0.3)
    x = np.random.default_rng(2).uniform(-1, 1, A.n)
    for P in (1, 2, 3, 8):
        bounds = csr.partition_rows(A.rowptr, P)
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
        chunk = _lib.host.rsp_padded_chunk(ip(bounds), P)
        ref_cols, ref_chunk = remap_columns(A.colidx, bounds)
        assert chunk == ref_chunk
        out = np.empty_like(A.colidx)
        assert _lib.host.rsp_remap_cols_padded(len(A.colidx), ip(A.colidx), ip(bounds), P, chunk, ip(out)) == 0
        assert np.array_equal(out, ref_cols)
        # every rank contributes its slice (count = chunk, padded); the gathered
        # buffer read at the remapped columns is x at the original columns
        xp = np.full(P * chunk, np.nan)
        for p in range(P):
            xp[p * chunk: p * chunk + bounds[p + 1] - bounds[p]] = x[bounds[p]:bounds[p + 1]]
        assert np.array_equal(xp[out], x[A.colidx])
        # row slices of the product reassemble A x exactly
        y = np.empty(A.m)
        for p in range(P):
            r0, r1 = bounds[p], bounds[p + 1]
            k0 = A.rowptr[r0]
            rp = A.rowptr[r0:r1 + 1] - k0
            y[r0:r1] = ob.spmv(rp, out[k0:A.rowptr[r1]], A.values[k0:A.rowptr[r1]], xp[: P * chunk])
        assert np.array_equal(y, ob.spmv(A.rowptr, A.colidx, A.values, x))
    bad = np.array([0, 5, A.n], np.int32)  # column n is out of range
    b = csr.partition_rows(A.rowptr, 2)
    assert _lib.host.rsp_remap_cols_padded(3, ip(bad), ip(b), 2, _lib.host.rsp_padded_chunk(ip(b), 2),
                                           ip(np.empty(3, np.int32))) == -1


def _py_levels(rowptr, colidx, transpose):
    n = len(rowptr) - 1
    lev = np.zeros(n, np.int64)
    for i in (range(n - 1, -1, -1) if transpose else range(n)):
        row = colidx[rowptr[i]:rowptr[i + 1]]
        low = row[row < i]
        if transpose:
            if low.size:
                np.maximum.at(lev, low, lev[i] + 1)
        elif low.size:
            lev[i] = lev[low].max() + 1
    return int(lev.max()) + 1 if n else 0


def _analysis_host(A):
    import ctypes as C
    lo, up, dg = C.c_int(), C.c_int(), C.c_uint64()
    ph = (C.c_double * 6)()
    rp = np.ascontiguousarray(A.rowptr, np.int32)
    ci = np.ascontiguousarray(A.colidx, np.int32)
    st = _lib.rsp.rsp_ilu0_analysis_host(A.n, rp.ctypes.data, ci.ctypes.data, C.byref(lo), C.byref(up),
                                         C.byref(dg), ph)
    return st, lo.value, up.value, dg.value, list(ph)


@pytest.mark.parametrize("name,scale", [("G2_circuit", 0.05), ("ASIC_320ks", 0.05), ("ecology2", 0.01),
                                        ("FEM_3D_thermal2", 0.02)])
def test_ilu_analysis_host_levels_and_digest(name, scale):
    """rsp_ilu0_analysis_host (the analysis' host phases, no device): the L and
    L^T level counts equal a direct restatement of the DAG's longest paths,
    and the plan digest is deterministic (threads and all)."""
    A = csr.surrogate(name, scale)
    st, lo, up, dg, ph = _analysis_host(A)
    assert st == 0
    assert lo == _py_levels(A.rowptr, A.colidx, False)
    assert up == _py_levels(A.rowptr, A.colidx, True)
    assert _analysis_host(A)[3] == dg and dg != 0
    assert all(v >= 0 for v in ph)


@pytest.mark.parametrize("name,scale", [("dc1", 0.3), ("parabolic_fem", 0.3), ("tmt_unsym", 0.05)])
def test_ilu_analysis_plan_thread_independent(monkeypatch, name, scale):
    """The plans are built by parallel phases (rows, levels, chunks and factor
    pieces as work items): the same plan on 1, 3 and 8 host threads, and with
    the thin factor runs cut into many small pieces the plan still differs
    from the one-piece plan only by construction (digests differ, both stable)."""
    A = csr.surrogate(name, scale)
    dg = set()
    for t in ("1", "3", "8"):
        monkeypatch.setenv("OMP_NUM_THREADS", t)
        st, _, _, d, _ = _analysis_host(A)
        assert st == 0
        dg.add(d)
    assert len(dg) == 1
    # (parabolic_fem is a stored lower triangle: its factor is one fat level
    # by default, no thin pieces; with its L levels it has them)
    monkeypatch.setenv("RSP_ILU_FAC_ONE", "0")
    dg = {_analysis_host(A)[3]}
    monkeypatch.setenv("RSP_ILU_PIECE_ITEMS", "500")
    small = {_analysis_host(A)[3] for t in ("1", "8") if not monkeypatch.setenv("OMP_NUM_THREADS", t)}
    assert len(small) == 1 and small != dg


@pytest.mark.parametrize("name,one", [("parabolic_fem", True), ("G2_circuit", True), ("dc1", False),
                                      ("tmt_unsym", False)])
def test_ilu_factor_one_level_without_update_pairs(monkeypatch, name, one):
    """A stored lower triangle (the symmetric matrices) has no update pairs:
    its factor plan is one level of every row, a different plan from the one
    over L's levels (RSP_ILU_FAC_ONE=0); a pattern with update pairs keeps
    L's levels either way (the same digest)."""
    A = csr.surrogate(name, 0.05)
    d1 = _analysis_host(A)[3]
    monkeypatch.setenv("RSP_ILU_FAC_ONE", "0")
    d0 = _analysis_host(A)[3]
    assert (d1 != d0) == one


def test_ilu_analysis_host_rejects_malformed():
    for rp, ci in (([0, 2, 4], [1, 0, 0, 1]), ([0, 2, 4], [0, 0, 0, 1]), ([0, 1, 2], [0, 5])):
        A = csr.CsrMatrix(0, 2, 2, len(ci), np.array(rp, np.int32), np.array(ci, np.int32), np.ones(len(ci)))
        assert _analysis_host(A)[0] == 3
