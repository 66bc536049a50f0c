"""Python host mirror of the operator boundary (include/rsp.h) on torch
device tensors. torch provides device memory, the stream and events —
plumbing only; every operation runs the HIP kernels of librsp.so.

Mapping to the reference's cuSPARSE usage:
  Handle                 cusparseCreate / cusparseDestroy   (GPU/spmv.cu:128,282)
  SpMat                  cusparseCreateCsr + SpMV_bufferSize (builds the
                         schedule) + the caller's workspace cudaMalloc
                                                             (GPU/spmv.cu:148-164)
  SpMat.spmv             cusparseSpMV                        (GPU/spmv.cu:184-186)
  SpmvBatch              cusparseSpMV over several matrices as one launch (no
                         cuSPARSE counterpart; bits equal to SpMat.spmv each)
  Ilu0.analysis          csrilu02_analysis + 2x csrsv2_analysis (GPU/ilu0.cu:203-252)
  Ilu0.zero_pivot        cusparseXcsrilu02_zeroPivot         (GPU/ilu0.cu:222,278)
  Ilu0.solve_zero_pivot  cusparseXcsrsv2_zeroPivot (the csrsv2 infos, GPU/ilu0.cu:143-150)
  Ilu0.factor            cusparse?csrilu02                   (GPU/ilu0.cu:264-268)
  Ilu0.solve_lower       cusparse?csrsv2_solve, desc_L, op N / op T (GPU/ilu0.cu:296-302)
Errors raise RspError carrying the rsp_status_t (numbered like cusparseStatus_t).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import RspError, check, rsp

_DT = {torch.float64: _lib.R_64F, torch.float32: _lib.R_32F}


def _ptr(t: torch.Tensor | None) -> C.c_void_p:
    return C.c_void_p(t.data_ptr() if t is not None and t.numel() > 0 else 0)


def _scalar(value: float, dtype: torch.dtype):
    return C.c_double(value) if dtype == torch.float64 else C.c_float(value)


class Handle:
    """rsp_handle_t bound to the current HIP device and a stream (default:
    torch's current stream, so torch events time the kernels)."""

    def __init__(self, stream: torch.cuda.Stream | None = None, ftz: bool = False):
        if not torch.cuda.is_available():
            raise RuntimeError("respasol_amd.sparse needs a HIP device (MI355X, gfx950)")
        self._h = C.c_void_p()
        check(rsp.rsp_create(C.byref(self._h)), "rsp_create")
        self.set_stream(stream if stream is not None else torch.cuda.current_stream())
        self.set_ftz(ftz)

    @property
    def ptr(self) -> C.c_void_p:
        return self._h

    def set_stream(self, stream: torch.cuda.Stream) -> None:
        self.stream = stream
        check(rsp.rsp_set_stream(self._h, C.c_void_p(stream.cuda_stream)), "rsp_set_stream")

    def set_ftz(self, on: bool) -> None:
        self.ftz = bool(on)
        check(rsp.rsp_set_ftz(self._h, 1 if on else 0), "rsp_set_ftz")

    def close(self) -> None:
        if self._h:
            rsp.rsp_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def upload_csr(rowptr: np.ndarray, colidx: np.ndarray, values: np.ndarray,
               dtype: torch.dtype = torch.float64, device: str | torch.device = "cuda"):
    """Host CSR arrays -> device tensors (values cast on the host with
    round-to-nearest, as the reference's fp32 demotion, GPU/spmv.cu:64-67)."""
    np_dt = np.float64 if dtype == torch.float64 else np.float32
    rp = torch.from_numpy(np.ascontiguousarray(rowptr, np.int32)).to(device)
    ci = torch.from_numpy(np.ascontiguousarray(colidx, np.int32)).to(device)
    va = torch.from_numpy(np.ascontiguousarray(values).astype(np_dt)).to(device)
    return rp, ci, va


class SpMat:
    """A device CSR matrix with its SpMV schedule (rsp_spmat_t + workspace)."""

    def __init__(self, handle: Handle, rowptr: torch.Tensor, colidx: torch.Tensor,
                 values: torch.Tensor, n_cols: int, nnz: int | None = None):
        if values.dtype not in _DT:
            raise TypeError("values must be float64 or float32")
        if rowptr.dtype != torch.int32 or colidx.dtype != torch.int32:
            raise TypeError("rowptr/colidx must be int32 (CUSPARSE_INDEX_32I)")
        self.handle = handle
        self.rowptr, self.colidx, self.values = rowptr, colidx, values
        self.m = rowptr.numel() - 1
        self.n = int(n_cols)
        self.dtype = values.dtype
        self.nnz = int(nnz if nnz is not None else colidx.numel())
        self._mat = C.c_void_p()
        check(rsp.rsp_create_csr(C.byref(self._mat), self.m, self.n, self.nnz, _ptr(rowptr),
                                 _ptr(colidx), _ptr(values), _DT[self.dtype]), "rsp_create_csr")
        one, zero = _scalar(1.0, self.dtype), _scalar(0.0, self.dtype)
        size = C.c_size_t()
        check(rsp.rsp_spmv_buffer_size(handle.ptr, _lib.OP_N, C.byref(one), self._mat,
                                       C.byref(zero), _DT[self.dtype], C.byref(size)),
              "rsp_spmv_buffer_size")
        # the reference's sequence (GPU/spmv.cu:159-164): bufferSize (which
        # builds the schedule inside the matrix) and the caller's workspace
        self.buffer = torch.empty(max(int(size.value), 1), dtype=torch.uint8, device=values.device)

    @property
    def nnz_stored(self) -> int:
        return int(self.colidx.numel())

    def spmv(self, x: torch.Tensor, y: torch.Tensor | None = None, alpha: float = 1.0,
             beta: float = 0.0) -> torch.Tensor:
        """y = alpha*A*x + beta*y on the handle's stream (cusparseSpMV)."""
        if x.dtype != self.dtype or x.numel() < self.n:
            raise ValueError("x has the wrong dtype or length")
        if y is None:
            y = torch.empty(self.m, dtype=self.dtype, device=x.device)
        a, b = _scalar(alpha, self.dtype), _scalar(beta, self.dtype)
        check(rsp.rsp_spmv(self.handle.ptr, _lib.OP_N, C.byref(a), self._mat, _ptr(x), C.byref(b),
                           _ptr(y), _DT[self.dtype], _ptr(self.buffer)), "rsp_spmv")
        return y

    def bind(self, x: torch.Tensor, y: torch.Tensor, alpha: float = 1.0, beta: float = 0.0):
        """The call y = alpha*A*x + beta*y with its C arguments converted once:
        returns a no-argument callable that issues exactly one rsp_spmv (the
        C driver's per-call cost, without the per-call Python argument
        conversion of spmv(); for timing loops of many short calls)."""
        if x.dtype != self.dtype or x.numel() < self.n or y.dtype != self.dtype or y.numel() < self.m:
            raise ValueError("x / y have the wrong dtype or length")
        a, b = _scalar(alpha, self.dtype), _scalar(beta, self.dtype)
        args = (self.handle.ptr, _lib.OP_N, C.byref(a), self._mat, _ptr(x), C.byref(b), _ptr(y),
                _DT[self.dtype], _ptr(self.buffer))
        keep = (a, b, x, y)  # the scalars and tensors the pointers refer to
        fn = rsp.rsp_spmv

        def call():
            st = fn(*args)
            if st:
                check(st, "rsp_spmv")
        call.keep = keep
        return call

    def set_local_cols(self, ncols_local: int) -> None:
        """Split the schedule for halo overlap (rsp_spmat_set_local_cols): tiles
        reading columns < ncols_local only (the rank's own x) run as part 1."""
        check(rsp.rsp_spmat_set_local_cols(self._mat, int(ncols_local)), "rsp_spmat_set_local_cols")
        one, zero = _scalar(1.0, self.dtype), _scalar(0.0, self.dtype)
        check(rsp.rsp_spmv_preprocess(self.handle.ptr, _lib.OP_N, C.byref(one), self._mat, None,
                                      C.byref(zero), None, _DT[self.dtype], _ptr(self.buffer)),
              "rsp_spmv_preprocess")

    def plan_info(self) -> dict:
        """{"tiles", "entries_16bit"} of the current schedule (rsp_spmv_plan_info)."""
        t, e = C.c_int64(), C.c_int64()
        check(rsp.rsp_spmv_plan_info(self._mat, C.byref(t), C.byref(e)), "rsp_spmv_plan_info")
        return {"tiles": t.value, "entries_16bit": e.value}

    def spmv_part(self, x: torch.Tensor, y: torch.Tensor, part: int, alpha: float = 1.0) -> torch.Tensor:
        """Part 1 (interior tiles) or 2 (the rest + fixup) of y = alpha*A*x (rsp_spmv_part)."""
        if x.dtype != self.dtype or x.numel() < self.n:
            raise ValueError("x has the wrong dtype or length")
        a, b = _scalar(alpha, self.dtype), _scalar(0.0, self.dtype)
        check(rsp.rsp_spmv_part(self.handle.ptr, C.byref(a), self._mat, _ptr(x), C.byref(b), _ptr(y),
                                _DT[self.dtype], _ptr(self.buffer), int(part)), "rsp_spmv_part")
        return y

    def close(self) -> None:
        if self._mat:
            rsp.rsp_destroy_spmat(self._mat)
            self._mat = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class SpmvBatch:
    """Several independent products y_j = alpha*A_j*x_j (+ beta*y_j) as one
    launch (rsp_spmv_batch_*): the same bits per matrix as SpMat.spmv /
    spmv_part, without one kernel ramp and drain per matrix. The x/y tensors
    are recorded: keep them (and the matrices) alive and in place."""

    def __init__(self, handle: Handle, mats: list[SpMat], xs: list[torch.Tensor],
                 ys: list[torch.Tensor], part: int = 0):
        if not (len(mats) == len(xs) == len(ys)):
            raise ValueError("mats, xs and ys must have the same length")
        dt = mats[0].dtype if mats else torch.float64
        for A, x, y in zip(mats, xs, ys):
            if A.dtype != dt or x.dtype != dt or y.dtype != dt:
                raise ValueError("one compute type per batch")
            if x.numel() < A.n or y.numel() < A.m:
                raise ValueError("x or y too short")
        self.handle, self.dtype, self.part = handle, dt, int(part)
        self._keep = (list(mats), list(xs), list(ys))
        n = len(mats)
        arr = C.c_void_p * max(n, 1)
        self._b = C.c_void_p()
        check(rsp.rsp_spmv_batch_create(
            handle.ptr, n, arr(*[A._mat.value for A in mats]), arr(*[x.data_ptr() for x in xs]),
            arr(*[y.data_ptr() for y in ys]), arr(*[A.buffer.data_ptr() for A in mats]),
            _DT[dt], self.part, C.byref(self._b)), "rsp_spmv_batch_create")

    def run(self, alpha: float = 1.0, beta: float = 0.0) -> None:
        a, b = _scalar(alpha, self.dtype), _scalar(beta, self.dtype)
        check(rsp.rsp_spmv_batch_run(self.handle.ptr, self._b, C.byref(a), C.byref(b)),
              "rsp_spmv_batch_run")

    def info(self) -> dict:
        """{"tiles", "entries_16bit"} of the batch's own schedule (rsp_spmv_batch_info)."""
        t, e = C.c_int64(), C.c_int64()
        check(rsp.rsp_spmv_batch_info(self._b, C.byref(t), C.byref(e)), "rsp_spmv_batch_info")
        return {"tiles": t.value, "entries_16bit": e.value}

    def close(self) -> None:
        if self._b:
            rsp.rsp_spmv_batch_destroy(self._b)
            self._b = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Ilu0:
    """ILU(0) + unit-lower triangular solves on one analysed pattern."""

    def __init__(self, handle: Handle, rowptr: torch.Tensor, colidx: torch.Tensor,
                 nnz: int | None = None):
        self.handle = handle
        self.rowptr, self.colidx = rowptr, colidx
        self.n = rowptr.numel() - 1
        self.nnz = int(nnz if nnz is not None else colidx.numel())
        self._info = C.c_void_p()
        check(rsp.rsp_create_ilu0_info(C.byref(self._info)), "rsp_create_ilu0_info")

    def analysis(self) -> None:
        """cusparse?csrilu02_analysis (rsp_ilu0_analysis): the solve plans
        are finished by trsv_analysis() or the first solve."""
        check(rsp.rsp_ilu0_analysis(self.handle.ptr, self.n, self.nnz, _ptr(self.rowptr),
                                    _ptr(self.colidx), self._info), "rsp_ilu0_analysis")

    def trsv_analysis(self, transpose: bool = False) -> None:
        """cusparse?csrsv2_analysis (rsp_trsv_analysis) for the L (or L^T) solve."""
        op = _lib.OP_T if transpose else _lib.OP_N
        check(rsp.rsp_trsv_analysis(self.handle.ptr, op, self._info), "rsp_trsv_analysis")

    def zero_pivot(self) -> int:
        """-1 if none, else the 0-based row (cusparseXcsrilu02_zeroPivot)."""
        pos = C.c_int(-1)
        st = rsp.rsp_ilu0_zero_pivot(self.handle.ptr, self._info, C.byref(pos))
        if st == _lib.STATUS_ZERO_PIVOT:
            return pos.value
        check(st, "rsp_ilu0_zero_pivot")
        return -1

    TRSV_L, TRSV_LT, TRSV_U = 0, 1, 2

    def solve_zero_pivot(self, which: int) -> int:
        """cusparseXcsrsv2_zeroPivot for the last solve of kind `which`
        (TRSV_L / TRSV_LT / TRSV_U): -1 if none, else the 0-based row (U
        only); raises RspError(EXECUTION_FAILED) if that solve's persistent
        launch gave up a dependency wait."""
        pos = C.c_int(-1)
        st = rsp.rsp_trsv_zero_pivot(self.handle.ptr, self._info, which, C.byref(pos))
        if st == _lib.STATUS_ZERO_PIVOT:
            return pos.value
        check(st, "rsp_trsv_zero_pivot")
        return -1

    def levels(self) -> tuple[int, int]:
        lo, up = C.c_int(), C.c_int()
        check(rsp.rsp_ilu0_levels(self._info, C.byref(lo), C.byref(up)), "rsp_ilu0_levels")
        return lo.value, up.value

    def solve_blocks(self) -> tuple[int, int]:
        """Blocks of the block-inverse L / L^T solves (0: level-scheduled)."""
        lo, up = C.c_int(), C.c_int()
        check(rsp.rsp_ilu0_solve_blocks(self._info, C.byref(lo), C.byref(up)), "rsp_ilu0_solve_blocks")
        return lo.value, up.value

    def factor(self, values: torch.Tensor) -> None:
        check(rsp.rsp_ilu0_factor(self.handle.ptr, self._info, _DT[values.dtype], _ptr(values)),
              "rsp_ilu0_factor")

    def solve_lower(self, values: torch.Tensor, x: torch.Tensor, y: torch.Tensor | None = None,
                    transpose: bool = False, alpha: float = 1.0) -> torch.Tensor:
        if y is None:
            y = torch.empty_like(x)
        a = _scalar(alpha, values.dtype)
        check(rsp.rsp_trsv_lower_unit(self.handle.ptr, _lib.OP_T if transpose else _lib.OP_N,
                                      C.byref(a), self._info, _DT[values.dtype], _ptr(values),
                                      _ptr(x), _ptr(y)), "rsp_trsv_lower_unit")
        return y

    def solve_upper(self, values: torch.Tensor, x: torch.Tensor, y: torch.Tensor | None = None,
                    alpha: float = 1.0) -> torch.Tensor:
        if y is None:
            y = torch.empty_like(x)
        a = _scalar(alpha, values.dtype)
        check(rsp.rsp_trsv_upper(self.handle.ptr, C.byref(a), self._info, _DT[values.dtype],
                                 _ptr(values), _ptr(x), _ptr(y)), "rsp_trsv_upper")
        return y

    def close(self) -> None:
        if self._info:
            rsp.rsp_destroy_ilu0_info(self._info)
            self._info = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def gather(handle: Handle, idx: torch.Tensor, src: torch.Tensor, dst: torch.Tensor) -> None:
    """dst[i] = src[idx[i]] (rsp_gather; idx int64, all on the device)."""
    if idx.dtype != torch.int64 or src.dtype != dst.dtype or dst.numel() < idx.numel():
        raise ValueError("gather: bad arguments")
    check(rsp.rsp_gather(handle.ptr, _DT[src.dtype], idx.numel(), _ptr(idx), _ptr(src), _ptr(dst)),
          "rsp_gather")


def scatter(handle: Handle, idx: torch.Tensor, src: torch.Tensor, dst: torch.Tensor) -> None:
    """dst[idx[i]] = src[i] (rsp_scatter; idx int64 without duplicates)."""
    if idx.dtype != torch.int64 or src.dtype != dst.dtype or src.numel() < idx.numel():
        raise ValueError("scatter: bad arguments")
    check(rsp.rsp_scatter(handle.ptr, _DT[src.dtype], idx.numel(), _ptr(idx), _ptr(src), _ptr(dst)),
          "rsp_scatter")


__all__ = ["Handle", "SpMat", "Ilu0", "upload_csr", "gather", "scatter", "RspError"]
