"""The oracle (oracle/rsp_oracle.c, the CPU restatement every GPU parity test
is bitwise against) checked against the reference's own CPU math library:
oneMKL 2021.4 outputs recorded by tests/golden/make_mkl_golden.py
(mkl_sparse_?_mv as test_spmv.c:89-101,147-158,165-183 calls it, with
correct base-0 arrays; dcsrilu0; mkl_sparse_d_trsv LOWER|UNIT, N then T) on
the reference's three Matrix-Market fixtures and seeded surrogates of each
structure family. Tolerances are SURVEY §8c's:
  SpMV  |dy_i| <= (len_i + 2) * u * sum_j |a_ij x_j|, u = 2^-53 (fp64), 2^-24 (fp32)
  ILU   relative <= 1e-13 (fp64) per row (largest |entry| of the row as the scale)
  trsv  normwise relative <= 1e-12 (fp64)
(cuSPARSE itself cannot run here; parity with it stays unpinned.)"""
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
from respasol_amd import csr

HERE = os.path.dirname(os.path.abspath(__file__))
MKL = os.path.join(HERE, "golden", "mkl")
if not os.path.exists(os.path.join(MKL, "index.json")):  # CPU-only vectors, not shipped to GPU boxes
    pytest.skip("MKL golden vectors not in this tree", allow_module_level=True)
INDEX = json.load(open(os.path.join(MKL, "index.json")))
CASES = [c["name"] for c in INDEX["cases"]]


def load(name):
    with np.load(os.path.join(MKL, name + ".npz")) as d:
        return {k: d[k] for k in d.files}


def spmv_bound(rp, ci, va, x, u):
    m = len(rp) - 1
    lens = np.diff(rp).astype(np.float64)
    rows = np.repeat(np.arange(m), np.diff(rp))
    s = np.zeros(m)
    np.add.at(s, rows, np.abs(va.astype(np.float64) * x.astype(np.float64)[ci]))
    return (lens + 2) * u * s


def test_index_names_the_library():
    assert "Math Kernel Library Version 2021.4" in INDEX["mkl"]
    assert {"b1_ss", "bcspwr01", "one"} <= set(CASES)


@pytest.mark.parametrize("name", [c["name"] for c in INDEX["cases"] if c["source"] == "mtx"])
def test_fixture_csr_is_the_loaders(name):
    """The golden CSR of the reference's fixtures is what the loader returns."""
    d = load(name)
    A = csr.load_matrix_market(os.path.join(HERE, "golden", "mtx", name + ".mtx"))
    nnz = int(A.rowptr[A.m])
    assert np.array_equal(A.rowptr[: A.m + 1], d["rowptr"])
    assert np.array_equal(A.colidx[:nnz], d["colidx"]) and np.array_equal(A.values[:nnz], d["values"])


@pytest.mark.parametrize("name", CASES)
def test_oracle_spmv_vs_mkl(name):
    d = load(name)
    rp, ci, va, x = d["rowptr"], d["colidx"], d["values"], d["x"]
    for order in ("seq", "canon"):  # the reference semantics, and the GPU kernels' order
        y = ob.spmv(rp, ci, va, x, order=order)
        assert np.all(np.abs(y - d["y64"]) <= spmv_bound(rp, ci, va, x, 2.0 ** -53)), order
        v32, x32 = va.astype(np.float32), x.astype(np.float32)
        y32 = ob.spmv(rp, ci, v32, x32, order=order)
        err = np.abs(y32.astype(np.float64) - d["y32"].astype(np.float64))
        assert np.all(err <= spmv_bound(rp, ci, v32, x32, 2.0 ** -24)), order


@pytest.mark.parametrize("name", [c["name"] for c in INDEX["cases"] if "ilu" in c.get("arrays", [])])
def test_oracle_ilu0_and_solves_vs_mkl(name):
    d = load(name)
    rp, ci, va = d["rowptr"], d["colidx"], d["values"]
    lu, sz, zp = ob.ilu0(rp, ci, va)
    assert sz == -1 and zp == -1
    ref = d["ilu"]
    # 1e-13 relative to the largest factor entry of the row: entry-wise
    # relative error is ill-posed where the update sum cancels (Goodwin_095:
    # an entry of 2.9e-7 left from terms of order 1 differs by 4.8e-19 =
    # 1.7e-12 relative, 1.8e-16 of its row); MKL's updates are not fused
    # (dcsrilu0) while the oracle's are (fma), so the bits differ slightly
    m = len(rp) - 1
    rows = np.repeat(np.arange(m), np.diff(rp))
    rmax, dmax = np.zeros(m), np.zeros(m)
    np.maximum.at(rmax, rows, np.abs(ref))
    np.maximum.at(dmax, rows, np.abs(lu - ref))
    assert np.all(dmax <= 1e-13 * np.maximum(rmax, 1e-300))
    n = len(rp) - 1
    z = ob.trsv("lower_n", rp, ci, lu, np.ones(n))
    y = ob.trsv("lower_t", rp, ci, lu, z)
    for got, want in ((z, d["z"]), (y, d["y"])):
        assert np.linalg.norm(got - want) <= 1e-12 * max(np.linalg.norm(want), 1e-300)


def test_bcspwr01_mkl_solve_is_the_integer_kat():
    """MKL's ILU(0) + L, L^T solve reproduces SURVEY §8c's integer-exact KAT,
    the same values the GPU test (test_gpu_ilu0.py) asserts."""
    kat = json.load(open(os.path.join(HERE, "golden", "kat.json")))["bcspwr01"]
    y = load("bcspwr01")["y"]
    assert y[:4].tolist() == kat["ilu_LLt_solve_x1_first4"]
    assert np.abs(y).max() == kat["ilu_LLt_solve_x1_maxabs"]
