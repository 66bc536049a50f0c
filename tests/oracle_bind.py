"""ctypes binding of oracle/build/liboracle.so — the CPU restatement used as
the parity checker (TEST INFRASTRUCTURE ONLY; see oracle/rsp_oracle.h)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")
REF_DUMP = os.path.join(ORACLE_DIR, "_ref", "ref_dump")
FIXTURES = os.path.join(ROOT, "tests", "golden", "mtx")


def _load():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    lib = C.CDLL(ORACLE_SO)
    ip, vp = C.POINTER(C.c_int), C.c_void_p
    for name in ("oracle_spmv_f64", "oracle_spmv_f32", "oracle_spmv_f32_ftz", "oracle_spmv_f64_omp",
                 "oracle_spmv_f32_omp"):
        getattr(lib, name).argtypes = [C.c_int, ip, ip, vp, vp, vp]
        getattr(lib, name).restype = None
    for name in ("oracle_spmv_canon_f64", "oracle_spmv_canon_f32", "oracle_spmv_canon_f32_ftz"):
        getattr(lib, name).argtypes = [C.c_int, ip, ip, vp, vp, vp, C.c_int]
        getattr(lib, name).restype = None
    lib.oracle_num_threads.restype = C.c_int
    lib.oracle_set_threads.argtypes = [C.c_int]
    lib.oracle_set_threads.restype = None
    lib.oracle_ilu0_f64.argtypes = [C.c_int, ip, ip, vp, ip]
    lib.oracle_ilu0_f64.restype = C.c_int
    lib.oracle_ilu0_f32.argtypes = [C.c_int, ip, ip, vp, ip, C.c_int]
    lib.oracle_ilu0_f32.restype = C.c_int
    for n in ("lower_n", "lower_t", "upper", "lower_n_split", "lower_t_split"):
        f = getattr(lib, f"oracle_trsv_{n}_f64")
        f.argtypes = [C.c_int, ip, ip, vp, C.c_double, vp, vp]
        f.restype = None
        f = getattr(lib, f"oracle_trsv_{n}_f32")
        f.argtypes = [C.c_int, ip, ip, vp, C.c_float, vp, vp, C.c_int]
        f.restype = None
    lib.oracle_dag_levels.argtypes = [C.c_int, C.c_int, ip, ip]
    lib.oracle_dag_levels.restype = C.c_int
    lib.oracle_trsv_blocks_f64.argtypes = [C.c_int, C.c_int, ip, ip, vp, C.c_double, vp, vp, vp]
    lib.oracle_trsv_blocks_f64.restype = C.c_int
    lib.oracle_trsv_blocks_f32.argtypes = [C.c_int, C.c_int, ip, ip, vp, C.c_float, vp, vp, vp, C.c_int]
    lib.oracle_trsv_blocks_f32.restype = C.c_int
    lib.oracle_dlarnv.argtypes = [C.c_int, ip, C.c_int, vp]
    lib.oracle_dlarnv.restype = C.c_int
    return lib


lib = _load()


def _i(a):
    return np.ascontiguousarray(a, np.int32).ctypes.data_as(C.POINTER(C.c_int))


def spmv(rowptr, colidx, vals, x, ftz=False, threads=False, order="seq"):
    """order="seq": column order per row (the reference semantics);
    order="canon": the canonical order of the GPU kernels (bit-exact target)."""
    rp = np.ascontiguousarray(rowptr, np.int32)
    ci = np.ascontiguousarray(colidx, np.int32)
    v = np.ascontiguousarray(vals)
    xx = np.ascontiguousarray(x, v.dtype)
    m = rp.shape[0] - 1
    y = np.empty(m, v.dtype)
    if order == "canon":
        fn = (lib.oracle_spmv_canon_f64 if v.dtype == np.float64
              else (lib.oracle_spmv_canon_f32_ftz if ftz else lib.oracle_spmv_canon_f32))
        fn(m, rp.ctypes.data_as(C.POINTER(C.c_int)), ci.ctypes.data_as(C.POINTER(C.c_int)),
           v.ctypes.data, xx.ctypes.data, y.ctypes.data, TILE_CAP[v.dtype])
        return y
    if v.dtype == np.float64:
        fn = lib.oracle_spmv_f64_omp if threads else lib.oracle_spmv_f64
    else:
        fn = lib.oracle_spmv_f32_ftz if ftz else (lib.oracle_spmv_f32_omp if threads else lib.oracle_spmv_f32)
    fn(m, rp.ctypes.data_as(C.POINTER(C.c_int)), ci.ctypes.data_as(C.POINTER(C.c_int)),
       v.ctypes.data, xx.ctypes.data, y.ctypes.data)
    return y


def ilu0(rowptr, colidx, vals, ftz=False):
    """Returns (factored values, structural_zero or -1, zero_pivot or -1)."""
    rp = np.ascontiguousarray(rowptr, np.int32)
    ci = np.ascontiguousarray(colidx, np.int32)
    v = np.array(vals, copy=True)
    n = rp.shape[0] - 1
    zp = C.c_int(-1)
    if v.dtype == np.float64:
        s = lib.oracle_ilu0_f64(n, rp.ctypes.data_as(C.POINTER(C.c_int)),
                                ci.ctypes.data_as(C.POINTER(C.c_int)), v.ctypes.data, C.byref(zp))
    else:
        s = lib.oracle_ilu0_f32(n, rp.ctypes.data_as(C.POINTER(C.c_int)),
                                ci.ctypes.data_as(C.POINTER(C.c_int)), v.ctypes.data, C.byref(zp),
                                1 if ftz else 0)
    return v, s, zp.value


def dag_levels(kind, rowptr, colidx):
    """Levels of the L (kind 0) or L^T (kind 1) DAG."""
    rp = np.ascontiguousarray(rowptr, np.int32)
    ci = np.ascontiguousarray(colidx, np.int32)
    return lib.oracle_dag_levels(kind, rp.shape[0] - 1, rp.ctypes.data_as(C.POINTER(C.c_int)),
                                 ci.ctypes.data_as(C.POINTER(C.c_int)))


def blocks_wanted(kind, rowptr, colidx):
    """The product's rule for a block-inverse solve of that DAG
    (rsp_an::blocks_wanted, ilu_blocks.cpp): RSP_ILU_BLOCKS -1 (default) for
    DAGs of <= 32 rows per level on average, 1 always, 0 never."""
    mode = int(os.environ.get("RSP_ILU_BLOCKS", "-1") or "-1")
    n = len(rowptr) - 1
    if mode == 0 or n <= 0:
        return False
    return mode > 0 or n <= 32 * dag_levels(kind, rowptr, colidx)


def trsv(kind, rowptr, colidx, vals, x, alpha=1.0, ftz=False):
    """kind in {'lower_n', 'lower_t', 'upper', 'lower_n_ref', 'lower_t_ref',
    'lower_n_split', 'lower_t_split', 'lower_n_blocks', 'lower_t_blocks'}.
    '*_ref' is the reference's own order (L: column ascending; L^T: the
    column sweep), '*_split' the split order (a row's terms from the level
    just below it applied last, rsp_oracle.c ORACLE_TRSV_SPLIT), '*_blocks'
    the block-inverse order of the deep-DAG solve (ORACLE_BLOCKS, round 6);
    'lower_n' / 'lower_t' follow the product's plan order: the block order
    where the product plans blocks for that DAG (blocks_wanted), else the
    reference's, or the split one where RSP_ILU_SPLIT=1 is set (the analysis
    knobs)."""
    split = os.environ.get("RSP_ILU_SPLIT", "0") not in ("", "0")
    if kind in ("lower_n", "lower_t") and blocks_wanted(0 if kind == "lower_n" else 1, rowptr, colidx):
        kind += "_blocks"
    kind = {"lower_n": "lower_n_split" if split else "lower_n",
            "lower_t": "lower_t_split" if split else "lower_t",
            "lower_n_ref": "lower_n", "lower_t_ref": "lower_t"}.get(kind, kind)
    rp = np.ascontiguousarray(rowptr, np.int32)
    ci = np.ascontiguousarray(colidx, np.int32)
    v = np.ascontiguousarray(vals)
    xx = np.ascontiguousarray(x, v.dtype)
    n = rp.shape[0] - 1
    y = np.empty(n, v.dtype)
    if kind.endswith("_blocks"):
        bk = 0 if kind == "lower_n_blocks" else 1
        if v.dtype == np.float64:
            r = lib.oracle_trsv_blocks_f64(bk, n, rp.ctypes.data_as(C.POINTER(C.c_int)),
                                           ci.ctypes.data_as(C.POINTER(C.c_int)), v.ctypes.data, alpha,
                                           xx.ctypes.data, y.ctypes.data, None)
        else:
            r = lib.oracle_trsv_blocks_f32(bk, n, rp.ctypes.data_as(C.POINTER(C.c_int)),
                                           ci.ctypes.data_as(C.POINTER(C.c_int)), v.ctypes.data, alpha,
                                           xx.ctypes.data, y.ctypes.data, None, 1 if ftz else 0)
        if r < 0:
            raise ValueError("oracle_trsv_blocks: bad arguments")
        return y
    if v.dtype == np.float64:
        getattr(lib, f"oracle_trsv_{kind}_f64")(n, rp.ctypes.data_as(C.POINTER(C.c_int)),
                                                ci.ctypes.data_as(C.POINTER(C.c_int)), v.ctypes.data,
                                                alpha, xx.ctypes.data, y.ctypes.data)
    else:
        getattr(lib, f"oracle_trsv_{kind}_f32")(n, rp.ctypes.data_as(C.POINTER(C.c_int)),
                                                ci.ctypes.data_as(C.POINTER(C.c_int)), v.ctypes.data,
                                                alpha, xx.ctypes.data, y.ctypes.data, 1 if ftz else 0)
    return y


def dlarnv(idist, seed, n):
    s = (C.c_int * 4)(*seed)
    x = np.empty(n, np.float64)
    assert lib.oracle_dlarnv(idist, s, n, x.ctypes.data) == 0
    return x, list(s)


TILE_CAP = {np.dtype(np.float64): 2047, np.dtype(np.float32): 4093}  # SpmvTile<T>::kMaxNnz


def spmv_bound(rowptr, colidx, vals, x, eps):
    """|dy_i| <= (len_i + 2) * eps * sum_j |a_ij x_j|."""
    rp = np.asarray(rowptr, np.int64)
    lens = np.diff(rp)
    absprod = np.abs(np.asarray(vals, np.float64)[:rp[-1]]) * np.abs(np.asarray(x, np.float64)[colidx[:rp[-1]]])
    # a trailing 0 keeps reduceat's indices in range when the last rows are empty
    rowsum = np.add.reduceat(np.append(absprod, 0.0), rp[:-1]) if len(lens) else np.zeros(0)
    rowsum = np.where(lens > 0, rowsum, 0.0)
    return (lens + 2) * eps * rowsum


def read_ref_dump(path):
    b = open(path, "rb").read()
    h = np.frombuffer(b[:24], np.int32)
    ok, sym, m, n, nnz, stored = (int(v) for v in h)
    o = 24
    rp = np.frombuffer(b[o:o + 4 * (m + 1)], np.int32) if ok else None
    o += 4 * (m + 1) if ok else 0
    ci = np.frombuffer(b[o:o + 4 * stored], np.int32) if ok else None
    o += 4 * stored if ok else 0
    va = np.frombuffer(b[o:o + 8 * stored], np.float64) if ok else None
    return dict(ok=ok, sym=sym, m=m, n=n, nnz=nnz, stored=stored, rowptr=rp, colidx=ci, values=va)


def ref_load(path, base=0, transpose=0, tmpdir="/tmp"):
    """Run the reference loader (oracle/_ref/ref_dump) — container only."""
    out = os.path.join(tmpdir, f"refdump_{os.getpid()}.bin")
    subprocess.run([REF_DUMP, path, str(base), str(transpose), out], check=True,
                   capture_output=True)
    d = read_ref_dump(out)
    os.remove(out)
    return d
