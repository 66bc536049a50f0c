"""Full-size parity of every single-GPU BASELINE config against the oracle
(VERDICT r02 "next" #1): each matrix of the sets the reference's run scripts
sweep (GPU/run_spmv.sh:3-5, GPU/run_ilu0.sh:3-5), at BASELINE size.

* config 4: all 15 "big" matrices, fp64 SpMV, one rsp_spmv each AND the
  bench's headline kernel (spmv_tiles_batch: the whole 15-matrix step as one
  launch), each compared directly with the oracle;
* config 2: all 21 "moderate" matrices, fp64 and fp32 SpMV, single calls and
  the 21-matrix batched launch, against the oracle;
* config 3: ILU(0) factor + L solve + L^T solve on all 21 moderate matrices
  in fp64, fp32 and fp32+FTZ, x = ones (GPU/ilu0.cu:63,74), bitwise against
  the oracle's IKJ restatement.

SpMV contract: every row bit-identical to the canonical-order
restatement (oracle_spmv_canon_*) and within
|dy_i| <= (len_i + 2) * u * sum_j |a_ij x_j| (u = 2^-53 / 2^-24) of the
column-order sum, the reference's own semantics (GPU/spmv.cu:221-260).
Inputs are the seeded surrogates of SURVEY App. A (no .mtx data offline)."""
import numpy as np
import pytest
import torch

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.sparse import Handle, Ilu0, SpMat, SpmvBatch, upload_csr

pytestmark = pytest.mark.gpu
NP = {torch.float64: np.float64, torch.float32: np.float32}
EPS = {torch.float64: 2.0 ** -53, torch.float32: 2.0 ** -24}
BIG = csr.surrogate_names(1)
MODERATE = csr.surrogate_names(0)


@pytest.fixture(scope="module")
def handle():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    h = Handle()
    yield h
    h.close()


_HOST = {}


def host_matrix(name):
    """Full-size surrogate + its x (dlarnv(1), the CPU test_spmv.c RHS), cached
    for the module (the big set is 3.2 GB of host CSR)."""
    if name not in _HOST:
        A = csr.surrogate(name)
        x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
        _HOST[name] = (A, x)
    return _HOST[name]


def same_bits(a, b):
    return np.array_equal(a.view(np.uint64 if a.dtype == np.float64 else np.uint32),
                          b.view(np.uint64 if b.dtype == np.float64 else np.uint32))


def check_rows(y, A, x, dtype):
    """y (GPU) against the oracle: canonical order bit for bit, column order
    within the forward-error bound; returns the number of rows checked."""
    v = A.values.astype(NP[dtype])
    xx = x.astype(NP[dtype])
    canon = ob.spmv(A.rowptr, A.colidx, v, xx, order="canon")
    bad = np.flatnonzero(y.view(np.uint64 if y.dtype == np.float64 else np.uint32)
                         != canon.view(np.uint64 if canon.dtype == np.float64 else np.uint32))
    assert bad.size == 0, f"{bad.size} rows differ from the canonical-order oracle, first {bad[:5]}"
    ref = ob.spmv(A.rowptr, A.colidx, v, xx, threads=True)
    bound = ob.spmv_bound(A.rowptr, A.colidx, v, xx, EPS[dtype])
    err = np.abs(y.astype(np.float64) - ref.astype(np.float64))
    assert np.all(err <= bound), f"max excess over the 8c bound {np.max(err - bound)}"
    return y.size


def gpu_mat(handle, A, dtype):
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
    return SpMat(handle, rp, ci, va, A.n, nnz=max(A.nnz, A.nnz_stored))


@pytest.mark.parametrize("name", BIG)
def test_config4_single_call(handle, name):
    A, x = host_matrix(name)
    M = gpu_mat(handle, A, torch.float64)
    y = M.spmv(torch.from_numpy(x).cuda()).cpu().numpy()
    check_rows(y, A, x, torch.float64)
    M.close()


def test_config4_batched_step(handle):
    """The bench step exactly as timed: the 15 big matrices as ONE
    spmv_tiles_batch launch, every y against the oracle (not only against the
    single-call bits), then repeated (no stale long-row tickets)."""
    mats, xs, ys, hosts = [], [], [], []
    for name in BIG:
        A, x = host_matrix(name)
        mats.append(gpu_mat(handle, A, torch.float64))
        xs.append(torch.from_numpy(x).cuda())
        ys.append(torch.full((A.m,), float("nan"), dtype=torch.float64, device="cuda"))
        hosts.append((A, x))
    B = SpmvBatch(handle, mats, xs, ys)
    B.run()
    torch.cuda.synchronize()
    first = [y.cpu().numpy() for y in ys]
    for y, (A, x) in zip(first, hosts):
        check_rows(y, A, x, torch.float64)
    for _ in range(3):
        B.run()
    torch.cuda.synchronize()
    for y, y0 in zip(ys, first):
        assert same_bits(y.cpu().numpy(), y0)
    B.close()
    for M in mats:
        M.close()


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_config2_moderate_set(handle, dtype):
    """All 21 moderate matrices at full size: one rsp_spmv each and the
    21-matrix batched launch, both against the oracle."""
    mats, xs, ys, hosts = [], [], [], []
    for name in MODERATE:
        A, x = host_matrix(name)
        M = gpu_mat(handle, A, dtype)
        xd = torch.from_numpy(x.astype(NP[dtype])).cuda()
        y = M.spmv(xd).cpu().numpy()
        check_rows(y, A, x, dtype)
        mats.append(M)
        xs.append(xd)
        ys.append(torch.full((A.m,), float("nan"), dtype=dtype, device="cuda"))
        hosts.append((A, x))
    B = SpmvBatch(handle, mats, xs, ys)
    B.run()
    torch.cuda.synchronize()
    for y, (A, x) in zip(ys, hosts):
        check_rows(y.cpu().numpy(), A, x, dtype)
    B.close()
    for M in mats:
        M.close()


@pytest.mark.parametrize("dtype,ftz", [(torch.float64, False), (torch.float32, False),
                                       (torch.float32, True)])
def test_config3_ilu0_moderate_set(handle, dtype, ftz):
    """Config 3 exactly as GPU/ilu0.cu runs it (analysis, zero-pivot checks,
    csrilu02, L solve, L^T solve with x = 1) on all 21 moderate matrices:
    factor values, z and y bit-identical to the oracle."""
    for name in MODERATE:
        A, _ = host_matrix(name)
        handle.set_ftz(ftz)
        try:
            rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
            il = Ilu0(handle, rp, ci, nnz=A.nnz)
            il.analysis()
            assert il.zero_pivot() == -1, name
            il.factor(va)
            zp = il.zero_pivot()
            ones = torch.ones(A.n, dtype=dtype, device="cuda")
            z = il.solve_lower(va, ones)
            y = il.solve_lower(va, z, transpose=True)
            torch.cuda.synchronize()
            v_gpu, z_gpu, y_gpu = va.cpu().numpy(), z.cpu().numpy(), y.cpu().numpy()
            il.close()
        finally:
            handle.set_ftz(False)
        rv, rsz, rzp = ob.ilu0(A.rowptr, A.colidx, A.values.astype(NP[dtype]), ftz=ftz)
        assert rsz == -1 and zp == rzp, name
        rz = ob.trsv("lower_n", A.rowptr, A.colidx, rv, np.ones(A.n, NP[dtype]), ftz=ftz)
        ry = ob.trsv("lower_t", A.rowptr, A.colidx, rv, rz, ftz=ftz)
        assert same_bits(v_gpu, rv), f"{name}: factor differs"
        assert same_bits(z_gpu, rz), f"{name}: L solve differs"
        assert same_bits(y_gpu, ry), f"{name}: L^T solve differs"
