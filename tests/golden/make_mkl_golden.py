"""Golden vectors from the reference's own CPU math library (SURVEY §8c,
"Oracle the build uses" (1)). CONTAINER ONLY: it loads oneMKL 2021.4
(/opt/conda/lib/libmkl_rt.so.1, conda mkl-2021.4.0 — README.md:19 pins "MKL
2020 or recent") through ctypes; the GPU box has no MKL and never runs this.

    python tests/golden/make_mkl_golden.py        # writes tests/golden/mkl/*.npz + index.json

The calls are the ones the reference makes on its CPU path, with CORRECT
base-0 arrays (the reference hands base-1 arrays to MKL as base 0,
test_spmv.c:54-55,91-92 — a shifted product):
  * y64 = mkl_sparse_d_mv(NON_TRANSPOSE, 1, A, GENERAL, x, 0)   test_spmv.c:89-101,165-171
  * y32 = mkl_sparse_s_mv(...) on the fp32 demotion              test_spmv.c:112-158,174-180
    x = LAPACKE_dlarnv(1, {0,0,0,1}, n)                          test_spmv.c:75-76
and for ILU(0) (no MKL call in the reference's GPU driver; MKL's own
ILU(0) and triangular solve, the CPU counterparts SURVEY §8c names):
  * dcsrilu0 (1-based arrays, as the RCI ISS routines require)  -> factor
  * mkl_sparse_d_trsv(NON_TRANSPOSE, 1, LU, {TRIANGULAR, LOWER, UNIT}, 1)  -> z
  * mkl_sparse_d_trsv(TRANSPOSE, ...) on z                       -> y
    (the GPU driver's x = 1 and its L, then L^T solves, GPU/ilu0.cu:284-302)

Inputs: the reference's three Matrix-Market fixtures (tests/golden/mtx, via
the product loader, which is byte-identical to the reference loader) and
small seeded surrogates of each structure family (respasol_amd host
generator; each npz stores the CSR it was computed on, so the vectors stay
valid whatever the generator does later). Outputs only — no reference
source is copied.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
OUT = os.path.join(HERE, "mkl")
MKL = "/opt/conda/lib/libmkl_rt.so.1"

SPARSE_INDEX_BASE_ZERO = 0
SPARSE_OPERATION_NON_TRANSPOSE, SPARSE_OPERATION_TRANSPOSE = 10, 11
SPARSE_MATRIX_TYPE_GENERAL, SPARSE_MATRIX_TYPE_TRIANGULAR = 20, 23
SPARSE_FILL_MODE_LOWER, SPARSE_FILL_MODE_FULL = 40, 42
SPARSE_DIAG_NON_UNIT, SPARSE_DIAG_UNIT = 50, 51


class Descr(C.Structure):
    _fields_ = [("type", C.c_int), ("mode", C.c_int), ("diag", C.c_int)]


def load_mkl():
    m = C.CDLL(MKL)
    vp, ip = C.c_void_p, C.POINTER(C.c_int)
    m.MKL_Set_Interface_Layer.argtypes = [C.c_int]
    m.MKL_Set_Interface_Layer(0)  # LP64 (32-bit MKL_INT, as the reference's arrays)
    m.MKL_Set_Threading_Layer.argtypes = [C.c_int]
    m.MKL_Set_Threading_Layer(1)  # sequential: deterministic vectors
    for f in ("mkl_sparse_d_create_csr", "mkl_sparse_s_create_csr"):
        getattr(m, f).argtypes = [C.POINTER(vp), C.c_int, C.c_int, C.c_int, ip, ip, ip, vp]
        getattr(m, f).restype = C.c_int
    m.mkl_sparse_d_mv.argtypes = [C.c_int, C.c_double, vp, Descr, vp, C.c_double, vp]
    m.mkl_sparse_d_mv.restype = C.c_int
    m.mkl_sparse_s_mv.argtypes = [C.c_int, C.c_float, vp, Descr, vp, C.c_float, vp]
    m.mkl_sparse_s_mv.restype = C.c_int
    m.mkl_sparse_d_trsv.argtypes = [C.c_int, C.c_double, vp, Descr, vp, vp]
    m.mkl_sparse_d_trsv.restype = C.c_int
    m.mkl_sparse_destroy.argtypes = [vp]
    m.mkl_sparse_destroy.restype = C.c_int
    m.dcsrilu0.argtypes = [ip, vp, ip, ip, vp, ip, vp, ip]
    m.dcsrilu0.restype = None
    buf = C.create_string_buffer(256)
    m.MKL_Get_Version_String(buf, 256)
    return m, buf.value.decode()


def ptr_i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


class Csr:
    """An MKL CSR handle over base-0 arrays (kept alive with the handle)."""

    def __init__(self, m, rp, ci, va):
        self.mkl = m
        self.rp = np.ascontiguousarray(rp, np.int32)
        self.ci = np.ascontiguousarray(ci, np.int32)
        self.va = np.ascontiguousarray(va)
        self.h = C.c_void_p()
        n = len(self.rp) - 1
        create = m.mkl_sparse_d_create_csr if self.va.dtype == np.float64 else m.mkl_sparse_s_create_csr
        st = create(C.byref(self.h), SPARSE_INDEX_BASE_ZERO, n, n, ptr_i(self.rp[:-1]), ptr_i(self.rp[1:]),
                    ptr_i(self.ci), self.va.ctypes.data)
        assert st == 0, st

    def close(self):
        self.mkl.mkl_sparse_destroy(self.h)


def mkl_mv(m, rp, ci, va, x):
    A = Csr(m, rp, ci, va)
    y = np.zeros(len(rp) - 1, va.dtype)
    d = Descr(SPARSE_MATRIX_TYPE_GENERAL, SPARSE_FILL_MODE_FULL, SPARSE_DIAG_NON_UNIT)
    xx = np.ascontiguousarray(x, va.dtype)
    if va.dtype == np.float64:
        st = m.mkl_sparse_d_mv(SPARSE_OPERATION_NON_TRANSPOSE, 1.0, A.h, d, xx.ctypes.data, 0.0, y.ctypes.data)
    else:
        st = m.mkl_sparse_s_mv(SPARSE_OPERATION_NON_TRANSPOSE, 1.0, A.h, d, xx.ctypes.data, 0.0, y.ctypes.data)
    A.close()
    assert st == 0, st
    return y


def mkl_ilu0(m, rp, ci, va):
    """dcsrilu0 on 1-based copies; returns (factor values, ierr)."""
    n = C.c_int(len(rp) - 1)
    ia = np.ascontiguousarray(rp + 1, np.int32)
    ja = np.ascontiguousarray(ci + 1, np.int32)
    a = np.ascontiguousarray(va, np.float64)
    b = np.zeros_like(a)
    ipar = np.zeros(128, np.int32)
    dpar = np.zeros(128, np.float64)
    ipar[1] = 6      # ipar(2): messages to the screen
    ipar[5] = 1      # ipar(6): print errors
    ipar[30] = 0     # ipar(31): stop at a zero / too small diagonal
    dpar[30] = 1e-300  # dpar(31): "too small" only for an exact zero (cuSPARSE csrilu02 semantics)
    ierr = C.c_int(0)
    m.dcsrilu0(C.byref(n), a.ctypes.data, ptr_i(ia), ptr_i(ja), b.ctypes.data, ptr_i(ipar),
               dpar.ctypes.data, C.byref(ierr))
    return b, ierr.value


def mkl_trsv_lower_unit(m, rp, ci, lu, x, transpose):
    A = Csr(m, rp, ci, lu)
    y = np.zeros(len(rp) - 1, np.float64)
    d = Descr(SPARSE_MATRIX_TYPE_TRIANGULAR, SPARSE_FILL_MODE_LOWER, SPARSE_DIAG_UNIT)
    xx = np.ascontiguousarray(x, np.float64)
    st = m.mkl_sparse_d_trsv(SPARSE_OPERATION_TRANSPOSE if transpose else SPARSE_OPERATION_NON_TRANSPOSE, 1.0,
                             A.h, d, xx.ctypes.data, y.ctypes.data)
    A.close()
    assert st == 0, st
    return y


# (name, source, scale): the reference's fixtures, then one small surrogate
# per structure family of SURVEY App. A / §8d (3-D stencil, 2-D grid, FEM
# general, circuit with hub rows, random band) — symmetric ones stored as the
# reference loader keeps them (lower triangle only)
CASES = [
    ("b1_ss", "mtx", None), ("bcspwr01", "mtx", None), ("one", "mtx", None),
    ("2cubes_sphere", "surrogate", 0.02), ("ecology2", "surrogate", 0.004),
    ("xenon2", "surrogate", 0.01), ("G2_circuit", "surrogate", 0.02), ("dc1", "surrogate", 0.03),
    ("ASIC_320ks", "surrogate", 0.01), ("cage13", "surrogate", 0.005), ("Goodwin_095", "surrogate", 0.01),
]


def main():
    from respasol_amd import csr
    m, version = load_mkl()
    os.makedirs(OUT, exist_ok=True)
    index = {"mkl": version, "generator": "tests/golden/make_mkl_golden.py", "cases": []}
    for name, src, scale in CASES:
        if src == "mtx":
            A = csr.load_matrix_market(os.path.join(HERE, "mtx", name + ".mtx"))
        else:
            A = csr.surrogate(name, scale)
        nnz_s = int(A.rowptr[A.m])
        rp = np.ascontiguousarray(A.rowptr[: A.m + 1], np.int32)
        ci = np.ascontiguousarray(A.colidx[:nnz_s], np.int32)
        va = np.ascontiguousarray(A.values[:nnz_s], np.float64)
        x = csr.dlarnv(1, [0, 0, 0, 1], A.n)[0]
        out = {"rowptr": rp, "colidx": ci, "values": va, "x": x,
               "y64": mkl_mv(m, rp, ci, va, x),
               "y32": mkl_mv(m, rp, ci, va.astype(np.float32), x.astype(np.float32))}
        rec = {"name": name, "source": src, "scale": scale, "m": int(A.m), "nnz_stored": nnz_s,
               "symmetric": int(A.is_symmetric)}
        hasdiag = all(np.any(ci[rp[i]:rp[i + 1]] == i) for i in range(A.m))
        if hasdiag and A.m == A.n:
            lu, ierr = mkl_ilu0(m, rp, ci, va)
            rec["dcsrilu0_ierr"] = ierr
            if ierr == 0:
                ones = np.ones(A.n)
                z = mkl_trsv_lower_unit(m, rp, ci, lu, ones, False)
                y = mkl_trsv_lower_unit(m, rp, ci, lu, z, True)
                out.update({"ilu": lu, "z": z, "y": y})
        else:
            rec["ilu"] = "skipped: a diagonal entry is missing (csrilu02 reports a structural zero)"
        rec["arrays"] = sorted(out)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        index["cases"].append(rec)
        print(name, rec, flush=True)
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
