"""The HIP kernels held DIRECTLY to the reference's CPU math library: oneMKL
2021.4 outputs (tests/golden/mkl/*.npz, recorded by
tests/golden/make_mkl_golden.py: mkl_sparse_?_mv as test_spmv.c:89-101,147-158
calls it with base-0 arrays, dcsrilu0, mkl_sparse_d_trsv LOWER|UNIT op N then
op T) on the reference's three Matrix-Market fixtures and seeded surrogates of
each structure family. Each case's own CSR and x go through librsp.so
(rsp_spmv fp64 / fp32, rsp_ilu0_analysis + rsp_ilu0_factor, rsp_trsv_lower_unit
N then T) on the GPU; the results must meet SURVEY §8c's bounds against MKL's:
  SpMV  |dy_i| <= (len_i + 2) * u * sum_j |a_ij x_j|, u = 2^-53 (fp64), 2^-24 (fp32)
  ILU   |d| <= 1e-13 * (largest |entry| of the row), fp64
  trsv  normwise relative <= 1e-12, fp64
— the same bounds tests/test_mkl_golden.py holds the oracle to on the CPU, so
GPU ≈ MKL holds on identical inputs, not only by transitivity through the
oracle."""
import json
import os

import numpy as np
import pytest
import torch

from respasol_amd.sparse import Handle, Ilu0, SpMat, upload_csr

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
MKL = os.path.join(HERE, "golden", "mkl")
INDEX = json.load(open(os.path.join(MKL, "index.json")))
CASES = [c["name"] for c in INDEX["cases"]]
ILU_CASES = [c["name"] for c in INDEX["cases"] if "ilu" in c.get("arrays", [])]


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


@pytest.fixture(scope="module")
def handle():
    h = Handle()
    yield h
    h.close()


@pytest.mark.parametrize("name", CASES)
def test_gpu_spmv_vs_mkl(name, handle):
    d = load(name)
    rp, ci, va, x = d["rowptr"], d["colidx"], d["values"], d["x"]
    n = len(x)
    for dt, npdt, want, u in ((torch.float64, np.float64, d["y64"], 2.0 ** -53),
                              (torch.float32, np.float32, d["y32"], 2.0 ** -24)):
        A = SpMat(handle, *upload_csr(rp, ci, va, dt), n)
        y = A.spmv(torch.from_numpy(x.astype(npdt)).cuda()).cpu().numpy()
        err = np.abs(y.astype(np.float64) - want.astype(np.float64))
        bound = spmv_bound(rp, ci, va.astype(npdt), x.astype(npdt), u)
        assert np.all(err <= bound), (name, str(dt), float((err - bound).max()))


@pytest.mark.parametrize("name", ILU_CASES)
def test_gpu_ilu0_and_solves_vs_mkl(name, handle):
    d = load(name)
    rp, ci, va = d["rowptr"], d["colidx"], d["values"]
    m = len(rp) - 1
    drp, dci, dva = upload_csr(rp, ci, va, torch.float64)
    il = Ilu0(handle, drp, dci)
    il.analysis()
    assert il.zero_pivot() == -1
    il.factor(dva)
    assert il.zero_pivot() == -1
    lu = dva.cpu().numpy()
    ref = d["ilu"]
    rows = np.repeat(np.arange(m), np.diff(rp))
    rmax, dmax = np.zeros(m), np.zeros(m)
    np.maximum.at(rmax, rows, np.abs(ref))
    np.maximum.at(dmax, rows, np.abs(lu - ref))
    assert np.all(dmax <= 1e-13 * np.maximum(rmax, 1e-300)), name
    ones = torch.ones(m, dtype=torch.float64, device="cuda")
    z = il.solve_lower(dva, ones)
    y = il.solve_lower(dva, z, transpose=True)
    for got, want in ((z.cpu().numpy(), d["z"]), (y.cpu().numpy(), d["y"])):
        assert np.linalg.norm(got - want) <= 1e-12 * max(np.linalg.norm(want), 1e-300), name


def test_gpu_bcspwr01_solve_is_the_integer_kat(handle):
    """MKL's and the GPU's L, L^T solves of bcspwr01 with x = 1 are both the
    integer-exact KAT."""
    d = load("bcspwr01")
    drp, dci, dva = upload_csr(d["rowptr"], d["colidx"], d["values"], torch.float64)
    il = Ilu0(handle, drp, dci)
    il.analysis()
    il.factor(dva)
    ones = torch.ones(len(d["x"]), dtype=torch.float64, device="cuda")
    y = il.solve_lower(dva, il.solve_lower(dva, ones), transpose=True).cpu().numpy()
    assert np.array_equal(y, d["y"])
