"""Randomised GPU parity of the CSR SpMV (seeded, reproducible): matrices
whose row-length mixtures and column patterns are drawn per seed — empty
rows, short rows, 33-256-entry rows among short ones (the reduce's
eight-lanes-per-row pass), rows longer than a tile (chunked, finished by
the last-arriving chunk), uniform, banded and clustered columns — each
checked bit for bit against the oracle's canonical order, fp64 and fp32, as
single calls and all together as one batched launch."""
import numpy as np
import pytest
import torch

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.sparse import Handle, SpMat, SpmvBatch, upload_csr

pytestmark = pytest.mark.gpu
NP = {torch.float64: np.float64, torch.float32: np.float32}
SEEDS = range(12)


def same_bits(a, b):
    return np.array_equal(a.view(np.uint64 if a.dtype == np.float64 else np.uint32),
                          b.view(np.uint64 if b.dtype == np.float64 else np.uint32))


def random_matrix(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([1, 7, 300, 5000, 40000]))
    # row lengths: a mixture of classes, weights drawn per seed
    w = rng.dirichlet(np.ones(4)) * np.array([1.0, 4.0, 1.0, 0.05 if n >= 5000 else 0.0])
    w /= w.sum()
    cls = rng.choice(4, n, p=w)
    lens = np.select([cls == 0, cls == 1, cls == 2, cls == 3],
                     [0, rng.integers(1, 9, n), rng.integers(17, 257, n), rng.integers(300, 9000, n)])
    lens = np.minimum(lens, n).astype(np.int64)
    pattern = seed % 3  # 0 uniform, 1 banded, 2 clustered
    row = np.repeat(np.arange(n), lens)
    if pattern == 0:
        col = rng.integers(0, n, row.size)
    elif pattern == 1:
        width = max(8, n // 50)
        col = np.clip(row + rng.integers(-width, width + 1, row.size), 0, n - 1)
    else:
        centers = rng.integers(0, n, max(1, n // 100))
        col = np.clip(centers[rng.integers(0, centers.size, row.size)] + rng.integers(-64, 65, row.size), 0, n - 1)
    key = np.unique(row.astype(np.int64) * n + col)
    row, col = key // n, key % n
    if n >= 5000:  # a few rows longer than a tile (fp64 2047 / fp32 4093 entries): chunked
        hubs = rng.choice(n, int(rng.integers(1, 6)), replace=False)
        keep = ~np.isin(row, hubs)
        row, col = row[keep], col[keep]
        extra_r = [np.full(int(k), h) for h, k in zip(hubs, rng.integers(2100, min(n, 12000), hubs.size))]
        extra_c = [np.sort(rng.choice(n, r.size, replace=False)) for r in extra_r]
        row = np.concatenate([row] + extra_r)
        col = np.concatenate([col] + extra_c)
        order = np.lexsort((col, row))
        row, col = row[order], col[order]
    rp = np.zeros(n + 1, np.int32)
    np.add.at(rp, row + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    vals = rng.uniform(-1, 1, col.size)
    return csr.CsrMatrix(0, n, n, int(col.size), rp, col.astype(np.int32), vals)


@pytest.mark.parametrize("variant", [0, 512, 1056])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_random_matrices_single_and_batched(monkeypatch, dtype, variant):
    """variant: RSP_SPMV_VARIANT of the handle — 0 the shipped schedule, 512
    small plans spread over every resident slot, 1056 = int32 column
    indices only (32) and no staged tiles (1024): the same bits every time."""
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    monkeypatch.setenv("RSP_SPMV_VARIANT", str(variant))
    handle = Handle()
    mats, xs, refs, ys = [], [], [], []
    for seed in SEEDS:
        A = random_matrix(seed)
        x = np.random.default_rng(seed).uniform(-1, 1, A.n)
        v, xx = A.values.astype(NP[dtype]), x.astype(NP[dtype])
        canon = ob.spmv(A.rowptr, A.colidx, v, xx, order="canon")
        rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values, dtype)
        M = SpMat(handle, rp, ci, va, A.n)
        xd = torch.from_numpy(xx).cuda()
        y = M.spmv(xd).cpu().numpy()
        assert same_bits(y, canon), (seed, A.n, A.nnz_stored)
        mats.append(M)
        xs.append(xd)
        refs.append(canon)
        ys.append(torch.empty(A.m, dtype=dtype, device="cuda"))
    B = SpmvBatch(handle, mats, xs, ys)
    B.run(1.0, 0.0)
    torch.cuda.synchronize()
    for seed, (r, y) in enumerate(zip(refs, ys)):
        assert same_bits(y.cpu().numpy(), r), seed
    B.close()
    handle.close()
