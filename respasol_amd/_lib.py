"""ctypes binding of the two C-ABI libraries built from respasol_amd/csrc.

* ``librsp.so``      — include/rsp.h: the HIP (gfx950) sparse operators that
  replace the cuSPARSE calls of GPU/spmv.cu and GPU/ilu0.cu.
* ``librsp_host.so`` — include/rsp_host.h: the Matrix-Market loader
  (ReadMatrixMarket/loadMatrixMarket.cpp semantics), dlarnv, surrogates and
  the row partitioner.

The libraries are built in-tree by ``__graft_entry__.build()`` (or ``make -C
respasol_amd/csrc``). There is no fallback: if a library is missing this
module raises at import time, so nothing can silently run on a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
BIN_DIR = os.path.join(_HERE, "bin")


class RspError(RuntimeError):
    """A non-success rsp_status_t (numbered like cusparseStatus_t)."""

    def __init__(self, status: int, where: str):
        self.status = int(status)
        super().__init__(f"{where}: {STATUS_NAMES.get(self.status, 'RSP_STATUS_UNKNOWN')} ({self.status})")


STATUS_SUCCESS = 0
STATUS_NOT_INITIALIZED = 1
STATUS_ALLOC_FAILED = 2
STATUS_INVALID_VALUE = 3
STATUS_ARCH_MISMATCH = 4
STATUS_EXECUTION_FAILED = 6
STATUS_INTERNAL_ERROR = 7
STATUS_MATRIX_TYPE_NOT_SUPPORTED = 8
STATUS_ZERO_PIVOT = 9
STATUS_NOT_SUPPORTED = 10
STATUS_NAMES = {
    0: "RSP_STATUS_SUCCESS", 1: "RSP_STATUS_NOT_INITIALIZED", 2: "RSP_STATUS_ALLOC_FAILED",
    3: "RSP_STATUS_INVALID_VALUE", 4: "RSP_STATUS_ARCH_MISMATCH", 6: "RSP_STATUS_EXECUTION_FAILED",
    7: "RSP_STATUS_INTERNAL_ERROR", 8: "RSP_STATUS_MATRIX_TYPE_NOT_SUPPORTED",
    9: "RSP_STATUS_ZERO_PIVOT", 10: "RSP_STATUS_NOT_SUPPORTED",
}

R_64F = 0
R_32F = 1
OP_N = 0
OP_T = 1

MM_FULL_SYMMETRIC = 0x1
MM_QUIET = 0x2
MM_SERIAL = 0x4
SURR_FTZ_STRESS = 0x1


class CSRStruct(C.Structure):
    """``CSR`` of ReadMatrixMarket/loadMatrixMarket.h:17-25 (same layout)."""

    _fields_ = [("isSymmetric", C.c_int), ("m", C.c_int), ("n", C.c_int), ("nnz", C.c_int),
                ("rowptr", C.POINTER(C.c_int)), ("colidx", C.POINTER(C.c_int)),
                ("values", C.POINTER(C.c_double))]


class COOStruct(C.Structure):
    """``COO`` of ReadMatrixMarket/loadMatrixMarket.h:28-36 (same layout)."""

    _fields_ = [("isSymmetric", C.c_int), ("m", C.c_int), ("n", C.c_int), ("nnz", C.c_int),
                ("Colidx", C.POINTER(C.c_int)), ("Rowidx", C.POINTER(C.c_int)),
                ("values", C.POINTER(C.c_double))]


vp = C.c_void_p
ip = C.POINTER(C.c_int)
i64 = C.c_int64
i32 = C.c_int

# name -> (restype, argtypes); the test suite checks this table against
# every function declared in include/*.h.
RSP_PROTOS = {
    "rsp_create": (i32, [C.POINTER(vp)]),
    "rsp_destroy": (i32, [vp]),
    "rsp_set_stream": (i32, [vp, vp]),
    "rsp_get_stream": (i32, [vp, C.POINTER(vp)]),
    "rsp_set_ftz": (i32, [vp, i32]),
    "rsp_get_ftz": (i32, [vp, ip]),
    "rsp_get_error_string": (C.c_char_p, [i32]),
    "rsp_get_version": (i32, []),
    "rsp_create_csr": (i32, [C.POINTER(vp), i64, i64, i64, vp, vp, vp, i32]),
    "rsp_csr_set_values": (i32, [vp, vp, i32]),
    "rsp_destroy_spmat": (i32, [vp]),
    "rsp_spmv_buffer_size": (i32, [vp, i32, vp, vp, vp, i32, C.POINTER(C.c_size_t)]),
    "rsp_spmv_preprocess": (i32, [vp, i32, vp, vp, vp, vp, vp, i32, vp]),
    "rsp_spmv": (i32, [vp, i32, vp, vp, vp, vp, vp, i32, vp]),
    "rsp_create_ilu0_info": (i32, [C.POINTER(vp)]),
    "rsp_destroy_ilu0_info": (i32, [vp]),
    "rsp_ilu0_buffer_size": (i32, [vp, i32, i32, i32, vp, C.POINTER(C.c_size_t)]),
    "rsp_ilu0_analysis": (i32, [vp, i32, i32, vp, vp, vp]),
    "rsp_ilu0_zero_pivot": (i32, [vp, vp, ip]),
    "rsp_trsv_zero_pivot": (i32, [vp, vp, i32, ip]),
    "rsp_ilu0_factor": (i32, [vp, vp, i32, vp]),
    "rsp_trsv_lower_unit": (i32, [vp, i32, vp, vp, i32, vp, vp, vp]),
    "rsp_trsv_upper": (i32, [vp, vp, vp, i32, vp, vp, vp]),
    "rsp_ilu0_levels": (i32, [vp, ip, ip]),
    "rsp_ilu0_solve_blocks": (i32, [vp, ip, ip]),
    "rsp_trsv_analysis": (i32, [vp, i32, vp]),
    "rsp_gather": (i32, [vp, i32, i64, vp, vp, vp]),
    "rsp_scatter": (i32, [vp, i32, i64, vp, vp, vp]),
    "rsp_spmat_set_local_cols": (i32, [vp, i64]),
    "rsp_spmv_part": (i32, [vp, vp, vp, vp, vp, vp, i32, vp, i32]),
    "rsp_spmv_batch_create": (i32, [vp, i32, vp, vp, vp, vp, i32, i32, vp]),
    "rsp_spmv_batch_run": (i32, [vp, vp, vp, vp]),
    "rsp_spmv_batch_destroy": (i32, [vp]),
    "rsp_spmv_batch_info": (i32, [vp, vp, vp]),
    "rsp_spmv_plan_info": (i32, [vp, vp, vp]),
    "rsp_ilu0_analysis_host": (i32, [i32, vp, vp, vp, vp, vp, vp]),
    "rsp_spmv_plan_host": (i32, [i32, vp, vp, C.c_int64, i32, vp, vp, vp]),
    "rsp_ilu0_plan_digest": (i32, [vp, vp]),
}

HOST_PROTOS = {
    "loadMatrixMarket": (i32, [C.c_char_p, C.POINTER(CSRStruct), i32, i32]),
    "loadCooMatrix": (i32, [C.c_char_p, C.POINTER(COOStruct), i32, i32]),
    "rsp_mm_load": (i32, [C.c_char_p, C.POINTER(CSRStruct), i32, i32, i32]),
    "rsp_mm_load_buffer": (i32, [C.c_char_p, C.c_size_t, C.POINTER(CSRStruct), i32, i32, i32]),
    "rsp_row_qsort": (None, [ip, C.POINTER(C.c_double), i32, i32]),
    "rsp_csr_free": (None, [C.POINTER(CSRStruct)]),
    "rsp_coo_free": (None, [C.POINTER(COOStruct)]),
    "rsp_csr_save": (i32, [C.c_char_p, C.POINTER(CSRStruct)]),
    "rsp_csr_load": (i32, [C.c_char_p, C.POINTER(CSRStruct)]),
    "rsp_dlarnv": (i32, [i32, ip, i64, C.POINTER(C.c_double)]),
    "rsp_set_cpu_ftz": (None, [i32]),
    "rsp_surrogate_count": (i32, []),
    "rsp_surrogate_name": (C.c_char_p, [i32]),
    "rsp_surrogate_info": (i32, [C.c_char_p, ip, C.POINTER(i64), ip, ip, ip]),
    "rsp_surrogate_rowlens": (i32, [C.c_char_p, C.c_double, i32, i32, i32, ip]),
    "rsp_surrogate_rows": (i32, [C.c_char_p, C.c_double, ip]),
    "rsp_surrogate_fill": (i32, [C.c_char_p, C.c_double, i32, i32, i32, ip, ip, C.POINTER(C.c_double)]),
    "rsp_surrogate_csr": (i32, [C.c_char_p, C.c_double, i32, C.POINTER(CSRStruct)]),
    "rsp_partition_rows": (i32, [ip, i32, i32, ip]),
    "rsp_padded_chunk": (i32, [ip, i32]),
    "rsp_remap_cols_padded": (i32, [i64, ip, ip, i32, i32, ip]),
    "rsp_host_spmv_f64": (None, [i32, ip, ip, vp, vp, vp]),
    "rsp_host_spmv_f32": (None, [i32, ip, ip, vp, vp, vp]),
}


def _load(name: str, protos: dict, path: str | None = None, probe: bool = False) -> C.CDLL:
    path = path or os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP/C libraries first "
            f"(python -c 'import __graft_entry__ as g; g.build()' or make -C respasol_amd/csrc)")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for fname, (res, args) in protos.items():
        if probe and not hasattr(lib, fname):  # an older diagnostic build (A/B runs)
            continue
        fn = getattr(lib, fname)
        fn.restype = res
        fn.argtypes = args
    return lib


host = _load("librsp_host.so", HOST_PROTOS)
# RSP_PROBE_LIB: a diagnostic build of librsp.so (scripts/spmv_probe.py only)
_RSP_PATH = os.environ.get("RSP_PROBE_LIB") or os.path.join(LIB_DIR, "librsp.so")
# RSP_HOST_ONLY=1: host library only (bench.py's CPU-baseline child process,
# which must not load the HIP runtime); the device operators are then absent
rsp = (None if os.environ.get("RSP_HOST_ONLY") == "1"
       else _load("librsp.so", RSP_PROTOS, _RSP_PATH, probe=bool(os.environ.get("RSP_PROBE_LIB"))))


def check(status: int, where: str) -> None:
    if status != STATUS_SUCCESS:
        raise RspError(status, where)


def loaded_paths() -> list[str]:
    """Absolute paths of the native libraries this package loaded."""
    return [os.path.join(LIB_DIR, "librsp_host.so"), _RSP_PATH]
