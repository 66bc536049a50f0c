"""Multi-rank SpMV logic on CPU with the gloo backend (world_size 2 and 3):
nnz-balanced row partition, rank-local surrogate generation, padded column
remap and the in-place all_gather of x. The local product is the oracle here
(standing in for the HIP kernel, which the GPU tests cover); the check is that
the gathered, partitioned result equals the single-process product bitwise."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.dist import RowPartitionedSpmv, remap_columns, unpad


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, scale, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = csr.surrogate_rows(name, scale)
        lens = csr.surrogate_rowlens(name, scale)
        rowptr = np.zeros(m + 1, np.int32)
        np.cumsum(lens, out=rowptr[1:])
        bounds = csr.partition_rows(rowptr, world)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        rp, ci, va = csr.surrogate_rows_csr(name, r0, r1, scale)  # only this rank's rows
        ci_pad, chunk = remap_columns(ci, bounds)

        def local(xf):
            return torch.from_numpy(ob.spmv(rp, ci_pad, va, xf.numpy()))

        part = RowPartitionedSpmv(bounds, rank, torch.float64, "cpu", local)
        x_global, _ = csr.dlarnv(2, [0, 0, 0, 1], m)
        part.set_local_x(torch.from_numpy(x_global[r0:r1]))
        y_local = part.step()
        y = part.gather_global(y_local)
        # the padded gather really delivered every rank's slice
        xg = unpad(part.x_full, bounds, chunk).numpy()
        q.put((rank, y.numpy(), np.array_equal(xg, x_global)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "Serena"), (3, "ASIC_320ks"), (2, "G2_circuit")])
def test_row_partitioned_spmv_gloo(world, name):
    scale = 0.01
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    ref = ob.spmv(A.rowptr, A.colidx, A.values, x)
    for rank, y, xok in res:
        assert xok
        assert np.array_equal(y, ref), rank


def _halo_worker(rank, world, port, names, scale, bucket, q, direct=False):
    from respasol_amd.dist import HaloExchange, HaloSlice
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        slices, hosts = [], []
        for name in names:
            m = csr.surrogate_rows(name, scale)
            lens = csr.surrogate_rowlens(name, scale)
            rowptr = np.zeros(m + 1, np.int32)
            np.cumsum(lens, out=rowptr[1:])
            bounds = csr.partition_rows(rowptr, world)
            r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
            rp, ci, va = csr.surrogate_rows_csr(name, r0, r1, scale)
            hs = HaloSlice(ci, bounds, rank)
            slices.append(hs)
            hosts.append((rp, va, csr.dlarnv(2, [0, 0, 0, 1], m)[0], r0, r1, ci))
        groups = [list(range(len(names)))] if bucket else [[i] for i in range(len(names))]
        out = {}
        for g in groups:
            ex = HaloExchange([slices[i] for i in g], rank, world, torch.float64, "cpu", direct=direct)
            for j, i in enumerate(g):
                rp, va, x, r0, r1, ci = hosts[i]
                ex.x_local(j).copy_(torch.from_numpy(x[r0:r1]))
            ex.exchange()
            for j, i in enumerate(g):
                rp, va, x, r0, r1, ci = hosts[i]
                xe = ex.x_ext(j).numpy()
                cols = ex.colidx(j)
                assert cols.dtype == np.int32 and (cols.size == 0 or cols.max() < ex.n_x(j))
                assert len(xe) == ex.n_x(j)
                # every entry the slice reads is the global x entry of its column
                ok_x = np.array_equal(xe[cols], x[ci])
                if not direct:
                    ok_x = ok_x and np.array_equal(xe[slices[i].m_local:],
                                                   x[np.concatenate(slices[i].recv_cols)])
                out[names[i]] = (r0, r1, ob.spmv(rp, cols, va, xe), ok_x, slices[i].H)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bucket,direct", [(2, True, False), (3, True, False), (2, False, False),
                                                 (2, True, True), (4, True, True), (3, False, True)])
def test_halo_exchange_gloo(world, bucket, direct):
    """Halo-only exchange (all_to_all with per-peer splits), bucketed over
    several matrices, in both arena layouts (halo unpacked into each slice's
    x, or received in place with the columns remapped): every rank's y slice
    equals the single-process y bitwise, and every x entry a slice reads is
    the global x entry of its column."""
    names, scale = ["Serena", "G2_circuit", "cage13", "ML_Laplace"], 0.01
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, names, scale, bucket, q, direct))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for name in names:
        A = csr.surrogate(name, scale)
        x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
        ref = ob.spmv(A.rowptr, A.colidx, A.values, x)
        got = np.concatenate([res[r][name][2] for r in range(world)])
        assert np.array_equal(got, ref), name
        assert all(res[r][name][3] for r in range(world))
        # the halo is a small fraction of x for the banded/mesh matrices
        if name in ("Serena", "ML_Laplace"):
            assert max(res[r][name][4] for r in range(world)) < 0.5 * A.n
