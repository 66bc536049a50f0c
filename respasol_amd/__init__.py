"""respasol_amd — MI355X-native (gfx950) implementation of ReSpaSol's
reduced-precision sparse hot path: CSR SpMV in fp64/fp32 (+FTZ) and the
ILU(0) factor + unit-lower triangular solves, behind the reference's driver
CLI (respasol_amd/bin/test_spmv, test_ilu0, test_spmv_cpu) and its
Matrix-Market -> CSR loader, through the C-ABI of include/rsp.h and
include/rsp_host.h.

Submodules:
  csr     host CSR: loader, surrogates, dlarnv, partition (librsp_host.so)
  sparse  device operators on torch tensors (librsp.so HIP kernels)
  dist    row-partitioned multi-GPU SpMV with an RCCL all-gather of x
"""
from . import _lib  # noqa: F401  (raises ImportError if the libraries are not built)
from ._lib import RspError, loaded_paths  # noqa: F401
from . import csr  # noqa: F401

__version__ = "0.1.0"


def native_version() -> int:
    return int(_lib.rsp.rsp_get_version())
