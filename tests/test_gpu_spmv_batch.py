"""GPU tests of the batched SpMV (rsp_spmv_batch_*, respasol_amd.sparse.SpmvBatch):
every matrix of a batch gets exactly the bits of its own rsp_spmv /
rsp_spmv_part call (which test_gpu_spmv.py pins to the oracle), for batches
spanning several launches (> 32 matrices), long-row fixups, empty matrices,
alpha/beta, fp32 with and without FTZ, the halo split (part 1 + part 2) and
the kernel variants; a matrix re-planned after the batch was built is a
status code, not a stale launch."""
import numpy as np
import pytest
import torch

from respasol_amd import RspError, csr
from respasol_amd.sparse import Handle, SpMat, SpmvBatch, upload_csr

pytestmark = pytest.mark.gpu
NP = {torch.float64: np.float64, torch.float32: np.float32}

# short rows, rows just above the 256-thread threshold, chunked hub rows,
# scattered columns, banded stencils; repeated to pass 32 matrices per launch
NAMES = [("ecology2", 0.02), ("ASIC_320ks", 0.2), ("G2_circuit", 0.1), ("Serena", 0.01),
         ("cage13", 0.02), ("atmosmodd", 0.02), ("Si87H76", 0.05), ("af_shell10", 0.005)]


def same_bits(a, b):
    return np.array_equal(a.view(np.uint64 if a.dtype == np.float64 else np.uint32),
                          b.view(np.uint64 if b.dtype == np.float64 else np.uint32))


def build(handle, dtype, count=37, local_frac=None):
    mats, xs, hosts = [], [], []
    for k in range(count):
        if k == 3:  # all-empty rows
            A = csr.CsrMatrix(0, 7, 7, 0, np.zeros(8, np.int32), np.zeros(0, np.int32), np.zeros(0))
        elif k == 5:  # 1 x 1
            A = csr.CsrMatrix(0, 1, 1, 1, np.array([0, 1], np.int32), np.array([0], np.int32),
                              np.array([2.5]))
        else:
            name, scale = NAMES[k % len(NAMES)]
            A = csr.surrogate(name, scale * (1 + 0.1 * (k // len(NAMES))))
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
        M = SpMat(handle, rp, ci, va, A.n, nnz=max(A.nnz, A.nnz_stored))
        if local_frac is not None:
            M.set_local_cols(int(A.n * local_frac))
        x, _ = csr.dlarnv(1, [0, 0, k, 1], A.n)
        mats.append(M)
        xs.append(torch.from_numpy(x.astype(NP[dtype])).cuda())
        hosts.append(A)
    return mats, xs, hosts


@pytest.fixture(scope="module")
def handle():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    h = Handle()
    yield h
    h.close()


@pytest.mark.parametrize("dtype,ftz", [(torch.float64, False), (torch.float32, False),
                                       (torch.float32, True)])
def test_batch_equals_single_calls(handle, dtype, ftz):
    handle.set_ftz(ftz)
    try:
        mats, xs, _ = build(handle, dtype)
        for alpha, beta in ((1.0, 0.0), (-1.5, 0.0), (0.75, 0.5)):
            y0 = [torch.from_numpy(np.random.default_rng(k).uniform(-1, 1, M.m).astype(NP[dtype])).cuda()
                  for k, M in enumerate(mats)]
            ref = [M.spmv(x, y.clone(), alpha, beta) for M, x, y in zip(mats, xs, y0)]
            ys = [y.clone() for y in y0]
            B = SpmvBatch(handle, mats, xs, ys)
            B.run(alpha, beta)
            torch.cuda.synchronize()
            for k, (r, y) in enumerate(zip(ref, ys)):
                assert same_bits(r.cpu().numpy(), y.cpu().numpy()), (k, alpha, beta)
            if beta == 0.0:  # repeatable
                B.run(alpha, beta)
                torch.cuda.synchronize()
                for r, y in zip(ref, ys):
                    assert same_bits(r.cpu().numpy(), y.cpu().numpy())
            B.close()
    finally:
        handle.set_ftz(False)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_batch_parts_equal_whole(handle, dtype):
    """Interior tiles of every matrix (part 1) then the rest + fixups (part 2)
    as two batched launches == one whole SpMV per matrix."""
    mats, xs, _ = build(handle, dtype, count=18, local_frac=0.6)
    ref = [M.spmv(x) for M, x in zip(mats, xs)]
    ys = [torch.full((max(M.m, 1),), float("nan"), dtype=dtype, device="cuda") for M in mats]
    b1 = SpmvBatch(handle, mats, xs, ys, part=1)
    b2 = SpmvBatch(handle, mats, xs, ys, part=2)
    b1.run()
    b2.run()
    torch.cuda.synchronize()
    for k, (r, y) in enumerate(zip(ref, ys)):
        assert same_bits(r.cpu().numpy(), y[: mats[k].m].cpu().numpy()), k
    with pytest.raises(RspError) as e:  # beta must be 0 for a split
        b1.run(1.0, 1.0)
    assert e.value.status == 3


@pytest.mark.parametrize("names,split", [
    ([("ecology2", 0.02), ("G2_circuit", 0.1)], False),     # few tiles: spread by nnz share
    ([("ecology2", 1.0), ("ASIC_320ks", 1.0)], False),      # > 2048 tiles: full tiles
    ([("ecology2", 1.0), ("ASIC_320ks", 1.0)], True)])
def test_batch_own_tiling_same_bits(handle, names, split):
    """The batch plans its members itself (full tiles once the launch fills
    the chip, a per-matrix share of the slots otherwise) while a lone
    rsp_spmv spreads a small matrix over the whole chip: different tiles,
    the same bits (canonical summation order), whole and split."""
    mats, xs = [], []
    for k, (name, scale) in enumerate(names):
        A = csr.surrogate(name, scale)
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, torch.float64)
        M = SpMat(handle, rp, ci, va, A.n, nnz=max(A.nnz, A.nnz_stored))
        if split:
            M.set_local_cols(A.n // 2)
        x, _ = csr.dlarnv(1, [0, 0, k, 3], A.n)
        mats.append(M)
        xs.append(torch.from_numpy(x).cuda())
    ref = [M.spmv(x) for M, x in zip(mats, xs)]
    ys = [torch.full((M.m,), float("nan"), dtype=torch.float64, device="cuda") for M in mats]
    if split:
        b1, b2 = SpmvBatch(handle, mats, xs, ys, part=1), SpmvBatch(handle, mats, xs, ys, part=2)
        b1.run()
        b2.run()
        infos = [b1.info(), b2.info()]
    else:
        B = SpmvBatch(handle, mats, xs, ys)
        B.run()
        infos = [B.info()]
    torch.cuda.synchronize()
    nnz = sum(M.nnz for M in mats)
    tiles = sum(i["tiles"] for i in infos)
    assert tiles > 0 and all(0 <= i["entries_16bit"] for i in infos)
    if names[0][1] == 1.0:  # > 2048 full tiles: none spread, so never more than the lone plans
        assert tiles <= sum(M.plan_info()["tiles"] for M in mats)
    assert sum(i["entries_16bit"] for i in infos) <= nnz
    for k, (r, y) in enumerate(zip(ref, ys)):
        assert same_bits(r.cpu().numpy(), y.cpu().numpy()), k


@pytest.mark.parametrize("variant", [1, 8, 9, 16, 32, 64, 128, 256, 1024])
def test_batch_variants_same_bits(monkeypatch, variant):
    """Default-policy loads (bit 0), no per-matrix XCD swizzle (bit 3), no
    spreading (bit 4), int32 column indices only (bit 5), no staged tiles
    (bit 10)."""
    monkeypatch.setenv("RSP_SPMV_VARIANT", str(variant))
    h = Handle()
    try:
        mats, xs, _ = build(h, torch.float64, count=10)
        ref = [M.spmv(x) for M, x in zip(mats, xs)]
        ys = [torch.empty(max(M.m, 1), dtype=torch.float64, device="cuda") for M in mats]
        SpmvBatch(h, mats, xs, ys).run()
        torch.cuda.synchronize()
        for r, y in zip(ref, ys):
            assert same_bits(r.cpu().numpy(), y[: r.numel()].cpu().numpy())
    finally:
        h.close()


def test_batch_stale_and_empty(handle):
    mats, xs, _ = build(handle, torch.float64, count=4)
    ys = [torch.empty(max(M.m, 1), dtype=torch.float64, device="cuda") for M in mats]
    B = SpmvBatch(handle, mats, xs, ys)
    B.run()
    mats[1].set_local_cols(mats[1].n // 2)  # re-planned: the batch's copy is stale
    with pytest.raises(RspError) as e:
        B.run()
    assert e.value.status == 3
    SpmvBatch(handle, [], [], []).run()  # no matrices: nothing launched
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        SpmvBatch(handle, mats[:1], xs[:1], [ys[0][:0]])


@pytest.mark.parametrize("variant", [0, 8])
def test_batch_many_chunk_hub_rows(monkeypatch, variant):
    """Hub rows of 20-40 chunks (fp64 2047 / fp32 4093 entries each) finished
    by their last-arriving chunk (release ticket add, acquire fence in the
    last arriver), with and without the per-matrix XCD swizzle (variant bit
    3 off spreads a row's chunks over the XCDs): every repeat gives the
    canonical-order oracle's bits."""
    import oracle_bind as ob
    monkeypatch.setenv("RSP_SPMV_VARIANT", str(variant))
    h = Handle()
    try:
        rng = np.random.default_rng(5)
        n = 60000
        cols, lens = [], []
        for i in range(n):
            if i % 4999 == 0:
                c = np.sort(rng.choice(n, 40000 + (i % 7) * 3000, replace=False)).astype(np.int32)
            else:
                c = np.unique(np.clip(i + rng.integers(-40, 41, 6), 0, n - 1)).astype(np.int32)
            cols.append(c)
            lens.append(len(c))
        rp = np.zeros(n + 1, np.int32)
        np.cumsum(lens, out=rp[1:])
        ci = np.concatenate(cols)
        va = rng.uniform(-1, 1, len(ci))
        for dt in (torch.float64, torch.float32):
            x = rng.uniform(-1, 1, n).astype(NP[dt])
            canon = ob.spmv(rp, ci, va.astype(NP[dt]), x, order="canon")
            mats, xs, ys = [], [], []
            for k in range(3):  # three copies: chunks of several matrices in flight together
                M = SpMat(h, *upload_csr(rp, ci, va, dt), n)
                mats.append(M)
                xs.append(torch.from_numpy(x).cuda())
                ys.append(torch.empty(n, dtype=dt, device="cuda"))
            B = SpmvBatch(h, mats, xs, ys)
            for rep in range(10):
                B.run()
                torch.cuda.synchronize()
                for y in ys:
                    assert same_bits(y.cpu().numpy(), canon), (dt, rep)
            for M, xd in zip(mats, xs):
                assert same_bits(M.spmv(xd).cpu().numpy(), canon)
            B.close()
    finally:
        h.close()


def test_batch_repeats_a_matrix_with_own_tickets(handle):
    """The same matrix several times in one batch (one A, several right-hand
    sides) and in a second batch: each batch member has its own long-row
    partials and tickets, so every y carries the bits of a
    single rsp_spmv of that x — here on a circuit surrogate whose hub rows
    are chunked (last-arriving-chunk tickets)."""
    import oracle_bind as ob
    A = csr.surrogate("ASIC_320ks", 0.3)
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
    M = SpMat(handle, rp, ci, va, A.n)
    xs = [torch.from_numpy(csr.dlarnv(1, [0, 0, k, 1], A.n)[0]).cuda() for k in range(3)]
    ys = [torch.empty(A.m, dtype=torch.float64, device="cuda") for _ in range(3)]
    ys2 = [torch.empty(A.m, dtype=torch.float64, device="cuda") for _ in range(2)]
    B1 = SpmvBatch(handle, [M, M, M], xs, ys)
    B2 = SpmvBatch(handle, [M, M], xs[:2], ys2)
    for _ in range(4):  # tickets return to 0 after every launch
        B1.run()
        B2.run()
        M.spmv(xs[2])
    torch.cuda.synchronize()
    for k in range(3):
        ref = ob.spmv(A.rowptr, A.colidx, A.values, xs[k].cpu().numpy(), order="canon")
        assert same_bits(ref, ys[k].cpu().numpy()), k
        if k < 2:
            assert same_bits(ref, ys2[k].cpu().numpy()), k
