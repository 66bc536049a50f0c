"""Host-side CSR matrices: the Matrix-Market loader (input side of the
drop-in boundary), the seeded SuiteSparse surrogates, dlarnv and the
nnz-balanced row partition — thin numpy wrappers over librsp_host.so.

Reference interface mirrored:
  ``CSR`` struct                  ReadMatrixMarket/loadMatrixMarket.h:17-25
  ``loadMatrixMarket``            ReadMatrixMarket/loadMatrixMarket.cpp:47-253
  ``LAPACKE_dlarnv``              test_spmv.c:75-76
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import CSRStruct, host

MM_STATUS = {
    0: "ok", 1: "open failed", 2: "bad banner", 3: "unsupported type", 4: "bad size line",
    5: "coordinate out of range", 6: "nnz mismatch", 7: "allocation failed",
}


class LoadError(RuntimeError):
    def __init__(self, status: int, path: str):
        self.status = status
        super().__init__(f"loadMatrixMarket({path!r}) failed: {MM_STATUS.get(status, status)}")


@dataclass
class CsrMatrix:
    """A loaded matrix with the reference's fields. ``nnz`` keeps the
    reference semantics (expanded count for symmetric files);
    ``nnz_stored`` = rowptr[m] - base is what every kernel computes on."""

    is_symmetric: int
    m: int
    n: int
    nnz: int
    rowptr: np.ndarray  # int32[m+1]
    colidx: np.ndarray  # int32[nnz_stored]
    values: np.ndarray  # float64[nnz_stored]
    base: int = 0

    @property
    def nnz_stored(self) -> int:
        return int(self.rowptr[self.m]) - self.base

    def to_base0(self) -> "CsrMatrix":
        if self.base == 0:
            return self
        return CsrMatrix(self.is_symmetric, self.m, self.n, self.nnz,
                         (self.rowptr - self.base).astype(np.int32),
                         (self.colidx - self.base).astype(np.int32), self.values.copy(), 0)

    def spmv_bytes(self, elem: int) -> int:
        """Algorithmic bytes of one y = A x."""
        return (elem + 4) * self.nnz_stored + 4 * (self.m + 1) + elem * (self.n + self.m)


def _from_struct(s: CSRStruct, base: int) -> CsrMatrix:
    m = s.m
    stored = s.rowptr[m] - base if m >= 0 and s.rowptr else 0
    rp = np.ctypeslib.as_array(s.rowptr, shape=(m + 1,)).copy() if s.rowptr else np.zeros(1, np.int32)
    ci = (np.ctypeslib.as_array(s.colidx, shape=(stored,)).copy()
          if stored > 0 else np.zeros(0, np.int32))
    va = (np.ctypeslib.as_array(s.values, shape=(stored,)).copy()
          if stored > 0 else np.zeros(0, np.float64))
    out = CsrMatrix(s.isSymmetric, s.m, s.n, s.nnz, rp.astype(np.int32), ci.astype(np.int32),
                    va.astype(np.float64), base)
    host.rsp_csr_free(C.byref(s))
    return out


def load_matrix_market(path: str, output_base: int = 0, transpose: int = 0,
                       full_symmetric: bool = False, quiet: bool = True,
                       serial: bool = False) -> CsrMatrix:
    """loadMatrixMarket (loadMatrixMarket.cpp:47-253); raises LoadError.
    Large files parse their entries on all OpenMP threads (same result);
    serial=True forces the one-thread parse."""
    s = CSRStruct()
    flags = ((_lib.MM_FULL_SYMMETRIC if full_symmetric else 0) | (_lib.MM_QUIET if quiet else 0)
             | (_lib.MM_SERIAL if serial else 0))
    st = host.rsp_mm_load(path.encode(), C.byref(s), output_base, transpose, flags)
    if st != 0:
        raise LoadError(st, path)
    return _from_struct(s, output_base)


def load_matrix_market_text(text: str | bytes, output_base: int = 0, transpose: int = 0,
                            full_symmetric: bool = False, serial: bool = False) -> CsrMatrix:
    buf = text.encode() if isinstance(text, str) else bytes(text)
    s = CSRStruct()
    flags = ((_lib.MM_FULL_SYMMETRIC if full_symmetric else 0) | _lib.MM_QUIET
             | (_lib.MM_SERIAL if serial else 0))
    st = host.rsp_mm_load_buffer(buf, len(buf), C.byref(s), output_base, transpose, flags)
    if st != 0:
        raise LoadError(st, "<buffer>")
    return _from_struct(s, output_base)


def dlarnv(idist: int, iseed: list[int] | tuple[int, ...], n: int) -> tuple[np.ndarray, list[int]]:
    """LAPACKE_dlarnv(idist, iseed, n, x): returns (x, advanced seed)."""
    seed = (C.c_int * 4)(*iseed)
    x = np.empty(n, np.float64)
    st = host.rsp_dlarnv(idist, seed, n, x.ctypes.data_as(C.POINTER(C.c_double)))
    if st != 0:
        raise ValueError("dlarnv: bad arguments")
    return x, list(seed)


def surrogate_names(set_id: int | None = None) -> list[str]:
    names = [host.rsp_surrogate_name(i).decode() for i in range(host.rsp_surrogate_count())]
    if set_id is None:
        return names
    return [n for n in names if surrogate_info(n)["set"] == set_id]


def surrogate_info(name: str) -> dict:
    m, nnz, sym, st, fam = C.c_int(), C.c_int64(), C.c_int(), C.c_int(), C.c_int()
    if host.rsp_surrogate_info(name.encode(), C.byref(m), C.byref(nnz), C.byref(sym), C.byref(st),
                               C.byref(fam)) != 0:
        raise KeyError(name)
    return {"m": m.value, "nnz_target": nnz.value, "symmetric": sym.value, "set": st.value,
            "family": ("stencil3d", "stencil2d", "circuit", "randband")[fam.value]}


def surrogate_rows(name: str, scale: float = 1.0) -> int:
    m = C.c_int()
    if host.rsp_surrogate_rows(name.encode(), scale, C.byref(m)) != 0:
        raise KeyError(name)
    return m.value


def surrogate_rowlens(name: str, scale: float = 1.0, flags: int = 0, r0: int = 0,
                      r1: int | None = None) -> np.ndarray:
    if r1 is None:
        r1 = surrogate_rows(name, scale)
    out = np.empty(max(r1 - r0, 0), np.int32)
    if host.rsp_surrogate_rowlens(name.encode(), scale, flags, r0, r1,
                                  out.ctypes.data_as(C.POINTER(C.c_int))) != 0:
        raise ValueError(f"surrogate_rowlens({name}) failed")
    return out


def surrogate_rows_csr(name: str, r0: int, r1: int, scale: float = 1.0,
                       flags: int = 0) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Rows [r0, r1) of a surrogate: (local rowptr from 0, global colidx, values)."""
    lens = surrogate_rowlens(name, scale, flags, r0, r1)
    rp = np.zeros(r1 - r0 + 1, np.int32)
    total = int(lens.sum(dtype=np.int64))
    if total > np.iinfo(np.int32).max:
        raise ValueError("slice too large for int32 offsets")
    ci = np.empty(max(total, 1), np.int32)
    va = np.empty(max(total, 1), np.float64)
    st = host.rsp_surrogate_fill(name.encode(), scale, flags, r0, r1,
                                 rp.ctypes.data_as(C.POINTER(C.c_int)),
                                 ci.ctypes.data_as(C.POINTER(C.c_int)),
                                 va.ctypes.data_as(C.POINTER(C.c_double)))
    if st != 0:
        raise ValueError(f"surrogate_fill({name}) failed")
    return rp, ci[:total], va[:total]


def surrogate(name: str, scale: float = 1.0, flags: int = 0) -> CsrMatrix:
    m = surrogate_rows(name, scale)
    rp, ci, va = surrogate_rows_csr(name, 0, m, scale, flags)
    sym = surrogate_info(name)["symmetric"]
    return CsrMatrix(sym, m, m, int(rp[-1]), rp, ci, va, 0)


def partition_rows(rowptr: np.ndarray, parts: int) -> np.ndarray:
    """nnz-balanced contiguous row ranges: bounds[p] = lower_bound(rowptr, p*nnz/P)."""
    rp = np.ascontiguousarray(rowptr, dtype=np.int32)
    m = rp.shape[0] - 1
    bounds = np.zeros(parts + 1, np.int32)
    if host.rsp_partition_rows(rp.ctypes.data_as(C.POINTER(C.c_int)), m, parts,
                               bounds.ctypes.data_as(C.POINTER(C.c_int))) != 0:
        raise ValueError("partition_rows: bad arguments")
    return bounds
