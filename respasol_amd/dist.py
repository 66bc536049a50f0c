"""Row-partitioned multi-GPU SpMV: one process per GPU,
torch.distributed over RCCL ("nccl" backend) on xGMI.

Rows are split into P contiguous nnz-balanced ranges (rsp_partition_rows:
bounds[p] = lower_bound(rowptr, p*nnz/P)). Rank p holds its row slice
(rebased rowptr, vals) and a replica of x. One step of the iterated product
is
    all_gather(x slices -> replicated x)   # the exchange step, RCCL over xGMI
    y_p = A_p x                            # local SpMV, librsp HIP kernels
after which a solver forms its next x slice from y_p (set_local_x).

Layout: the gather uses equal per-rank counts (chunk = max rows per rank) so
it is one in-place all_gather_into_tensor; the replicated x is therefore
"padded" (rank p's rows at [p*chunk, p*chunk + m_p)) and the slice's column
indices are remapped once at setup to that layout, so the kernel reads the
gathered buffer directly with no unpack copy.
The ILU(0) path does not shard (level dependencies cross any row split) and
stays single-GPU.
"""
from __future__ import annotations

from typing import Callable

import numpy as np
import torch
import torch.distributed as dist


def padded_layout(bounds: np.ndarray) -> tuple[int, np.ndarray]:
    """chunk and, for every global row, its position in the padded gather."""
    P = len(bounds) - 1
    sizes = np.diff(bounds)
    chunk = int(sizes.max()) if P > 0 else 0
    n = int(bounds[-1])
    owner = np.repeat(np.arange(P, dtype=np.int64), sizes)
    pos = owner * chunk + (np.arange(n, dtype=np.int64) - bounds[owner].astype(np.int64))
    return chunk, pos


def remap_columns(colidx: np.ndarray, bounds: np.ndarray) -> tuple[np.ndarray, int]:
    """Global column j -> its padded position (int32); returns (cols, chunk)."""
    chunk, pos = padded_layout(bounds)
    if len(bounds) - 1 > 0 and (len(bounds) - 1) * chunk > np.iinfo(np.int32).max:
        raise ValueError("padded x does not fit int32 indices")
    return pos[colidx].astype(np.int32), chunk


def unpad(x_full: torch.Tensor, bounds: np.ndarray, chunk: int) -> torch.Tensor:
    """Padded replicated vector -> dense global order."""
    parts = [x_full[p * chunk: p * chunk + int(bounds[p + 1] - bounds[p])]
             for p in range(len(bounds) - 1)]
    return torch.cat(parts) if parts else x_full[:0]


class RowPartitionedSpmv:
    """This rank's share of y = A x with an all-gathered x.

    ``local_spmv(x_full) -> y_local`` computes the slice's product on the
    padded x; the product path passes a librsp ``SpMat.spmv`` (HIP). The
    all-gather uses the default process group (nccl = RCCL on ROCm)."""

    def __init__(self, bounds: np.ndarray, rank: int, dtype: torch.dtype, device,
                 local_spmv: Callable[[torch.Tensor], torch.Tensor], group=None):
        self.bounds = np.asarray(bounds, dtype=np.int64)
        self.P = len(self.bounds) - 1
        self.rank = rank
        self.r0, self.r1 = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.m_local = self.r1 - self.r0
        self.chunk = int(np.diff(self.bounds).max()) if self.P else 0
        self.group = group
        self.local_spmv = local_spmv
        self.x_full = torch.zeros(max(self.P * self.chunk, 1), dtype=dtype, device=device)
        self.x_local = self.x_full[rank * self.chunk:(rank + 1) * self.chunk]

    def set_local_x(self, values: torch.Tensor) -> None:
        """Write this rank's rows of x (length m_local); the padding stays 0."""
        self.x_local[: self.m_local].copy_(values[: self.m_local])

    def exchange(self) -> None:
        """all_gather the x slices into the replicated x (in place)."""
        if self.P <= 1:
            return
        if self.x_full.is_cuda and dist.get_backend(self.group) == "gloo":
            # rehearsal path (gloo on a GPU box): stage through host memory
            host = self.x_full.cpu()
            dist.all_gather_into_tensor(host, host[self.rank * self.chunk:(self.rank + 1) * self.chunk].clone(),
                                        group=self.group)
            self.x_full.copy_(host)
            return
        dist.all_gather_into_tensor(self.x_full, self.x_local, group=self.group)

    def step(self, y_local: torch.Tensor | None = None) -> torch.Tensor:
        self.exchange()
        return self.local_spmv(self.x_full) if y_local is None else self.local_spmv(self.x_full, y_local)

    def gather_global(self, y_local: torch.Tensor) -> torch.Tensor:
        """Collect every rank's y slice into the dense global y (for checks)."""
        buf = torch.zeros(max(self.P * self.chunk, 1), dtype=y_local.dtype, device=y_local.device)
        pad = torch.zeros(max(self.chunk, 1), dtype=y_local.dtype, device=y_local.device)
        pad[: self.m_local].copy_(y_local[: self.m_local])
        if self.P > 1 and buf.is_cuda and dist.get_backend(self.group) == "gloo":
            host = buf.cpu()
            dist.all_gather_into_tensor(host, pad[: self.chunk].cpu(), group=self.group)
            buf.copy_(host)
        elif self.P > 1:
            dist.all_gather_into_tensor(buf, pad[: self.chunk], group=self.group)
        else:
            buf[: self.chunk].copy_(pad[: self.chunk])
        return unpad(buf, self.bounds, self.chunk)


# ----------------------------------------------------------------- halo exchange
#
# The all-gather above moves all of x to every rank: 8*n*(P-1)/P bytes per
# rank per SpMV, ~10 MB for Serena at P = 8 against ~11 us of kernel time.
# A row block of a banded / mesh matrix references only a thin "halo" of
# columns outside its own range, so each rank needs just those x entries
# (SURVEY §8f rank 2). Layout per slice: x_ext = [x_local (m_local) | halo (H)],
# halo ordered by (owner rank, column); the slice's column indices are remapped
# once (own column j -> j - r0, halo column -> m_local + position). One
# exchange = pack (gather the entries each peer asked for) -> all_to_all_single
# with per-peer split sizes -> unpack (scatter into each x_ext). Several slices
# (one per matrix) share ONE all_to_all per step ("bucketed": fewer, larger
# collectives — on xGMI the per-call latency, not bandwidth, dominates these
# small halos). pack/unpack are librsp kernels (rsp_gather / rsp_scatter) on
# the GPU; CPU tensors (gloo tests) use torch indexing.


class HaloSlice:
    """Halo analysis of one rank's row slice (global column indices)."""

    def __init__(self, colidx: np.ndarray, bounds: np.ndarray, rank: int):
        self.bounds = np.asarray(bounds, np.int64)
        self.P = len(self.bounds) - 1
        self.rank = rank
        self.r0, self.r1 = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.m_local = self.r1 - self.r0
        ci = np.asarray(colidx, np.int64)
        cols = np.unique(ci)
        remote = cols[(cols < self.r0) | (cols >= self.r1)]
        owner = np.searchsorted(self.bounds, remote, side="right") - 1
        self.recv_cols = [remote[owner == p] for p in range(self.P)]  # sorted per owner
        self.recv_counts = np.array([len(c) for c in self.recv_cols], np.int64)
        self.H = int(remote.size)
        local = (ci >= self.r0) & (ci < self.r1)
        ext = np.empty_like(ci)
        ext[local] = ci[local] - self.r0
        ext[~local] = self.m_local + np.searchsorted(remote, ci[~local])
        if self.m_local + self.H > np.iinfo(np.int32).max:
            raise ValueError("extended x does not fit int32 indices")
        self.colidx_ext = ext.astype(np.int32)
        self.n_ext = self.m_local + self.H
        self.send_local: list[np.ndarray] | None = None  # filled by HaloExchange

    def halo_offsets(self) -> np.ndarray:
        """Start of each owner's block inside the halo."""
        return np.concatenate([[0], np.cumsum(self.recv_counts)[:-1]]).astype(np.int64)


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group) -> None:
    if out.is_cuda and dist.get_backend(group) == "gloo":  # rehearsal path
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(host, inp.cpu(), list(out_splits), list(in_splits), group=group)
        out.copy_(host)
        return
    dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=group)


class HaloExchange:
    """Bucketed halo exchange for the slices of several matrices on one rank.

    Setup is collective (every rank constructs it with its slices in the same
    order). `exchange()` refreshes every halo with one all_to_all_single.

    Layouts of the arena that holds every slice's x:
    * packed (direct=False): slice i's x_ext = [own rows | halo] back to back,
      columns as HaloSlice.colidx_ext; the all-to-all lands in a receive
      buffer and an unpack kernel (rsp_scatter) copies it into the halos.
    * direct (direct=True): [own rows of slice 0 | ... of slice S-1 | receive
      region]; the all-to-all writes straight into the receive region (ordered
      by source rank, then slice, then column) and slice i's columns are
      remapped once (`colidx(i)`) to index the arena from its own part's
      start, so its halo entries point into the receive region. No unpack
      launch per step; own columns stay [0, m_local), so the interior/boundary
      tile split (rsp_spmat_set_local_cols) is unchanged.
    `x_ext(i)` is the vector slice i's SpMV reads (`n_x(i)` entries),
    `x_local(i)` its owned part."""

    def __init__(self, slices: list[HaloSlice], rank: int, world: int, dtype: torch.dtype,
                 device, handle=None, group=None, direct: bool = False):
        self.slices, self.rank, self.P, self.group = slices, rank, world, group
        self.dtype, self.device, self.handle = dtype, torch.device(device), handle
        self.direct = direct
        sizes = [s.m_local for s in slices] if direct else [s.n_ext for s in slices]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        n_recv_all = int(sum(int(s.recv_counts.sum()) for s in slices))
        self.recv_off = int(self.offsets[-1])
        total = self.recv_off + (n_recv_all if direct else 0)
        self.arena = torch.zeros(max(total, 1), dtype=dtype, device=self.device)
        # 1) who wants what: counts then the requested global columns
        idx_dev = self.device if (self.device.type == "cuda" and
                                  dist.get_backend(group) != "gloo") else torch.device("cpu")
        want = np.stack([s.recv_counts for s in slices], axis=0) if slices else np.zeros((0, world), np.int64)
        send_cnt = torch.empty(len(slices) * world, dtype=torch.int64, device=idx_dev)
        # element [i*P + p] on rank r = how many columns slice i of rank r wants from p;
        # transpose through all_to_all so rank p learns the counts it must send.
        req = torch.from_numpy(np.ascontiguousarray(want.T.reshape(-1))).to(idx_dev)  # [p][i]
        dist.all_to_all_single(send_cnt, req, [len(slices)] * world, [len(slices)] * world, group=group)
        send_counts = send_cnt.cpu().numpy().reshape(world, len(slices))  # [q][i]: q wants from me
        req_cols = np.concatenate([np.concatenate([s.recv_cols[p] for s in slices]) if slices
                                   else np.zeros(0, np.int64) for p in range(world)]).astype(np.int64)
        in_split = [int(want[:, p].sum()) for p in range(world)]
        out_split = [int(send_counts[q].sum()) for q in range(world)]
        asked = torch.empty(sum(out_split), dtype=torch.int64, device=idx_dev)
        dist.all_to_all_single(asked, torch.from_numpy(req_cols).to(idx_dev), out_split, in_split,
                               group=group)
        asked = asked.cpu().numpy()
        # 2) pack index: for dest q, slice i: positions of the asked columns in my arena
        pack, pos = [], 0
        for q in range(world):
            for i, s in enumerate(slices):
                c = int(send_counts[q, i])
                cols = asked[pos:pos + c]
                pos += c
                if c and (cols.min() < s.r0 or cols.max() >= s.r1):
                    raise RuntimeError("halo request outside the owner's rows")
                pack.append(self.offsets[i] + (cols - s.r0))
        self.send_split = out_split
        self.recv_split = in_split
        # 3) data from source p arrives ordered (slice i, column): where block
        # (p, i) starts in the receive stream
        self.recv_start = np.zeros((world, len(slices)), np.int64)
        pos = 0
        for p in range(world):
            for i, s in enumerate(slices):
                self.recv_start[p, i] = pos
                pos += int(s.recv_counts[p])
        self.n_recv = pos
        cat = lambda a: np.concatenate(a) if a else np.zeros(0, np.int64)  # noqa: E731
        self.pack_idx = torch.from_numpy(cat(pack)).to(self.device)
        self.sendbuf = torch.empty(max(self.pack_idx.numel(), 1), dtype=dtype, device=self.device)
        if direct:  # the all-to-all writes the arena's receive region itself
            self.unpack_idx = torch.zeros(0, dtype=torch.int64, device=self.device)
            self.recvbuf = self.arena[self.recv_off:self.recv_off + max(self.n_recv, 1)]
        else:  # unpack index: receive stream -> each slice's halo
            unpack = []
            for p in range(world):
                for i, s in enumerate(slices):
                    c = int(s.recv_counts[p])
                    start = self.offsets[i] + s.m_local + s.halo_offsets()[p]
                    unpack.append(np.arange(start, start + c, dtype=np.int64))
            self.unpack_idx = torch.from_numpy(cat(unpack)).to(self.device)
            self.recvbuf = torch.empty(max(self.unpack_idx.numel(), 1), dtype=dtype, device=self.device)
        self._work = None

    def colidx(self, i: int) -> np.ndarray:
        """Column indices of slice i into x_ext(i) (int32)."""
        s = self.slices[i]
        if not self.direct:
            return s.colidx_ext
        ext = s.colidx_ext.astype(np.int64)
        h = ext - s.m_local
        halo = h >= 0
        offs = s.halo_offsets()
        owner = np.searchsorted(offs, h[halo], side="right") - 1
        # several owners may hold no columns (equal offsets): side="right"
        # picks the last of them, the one whose block is non-empty
        base = self.recv_off - int(self.offsets[i])
        ext[halo] = base + self.recv_start[owner, i] + (h[halo] - offs[owner])
        if ext.size and int(ext.max()) > np.iinfo(np.int32).max:
            raise ValueError("arena does not fit int32 indices")
        return ext.astype(np.int32)

    def n_x(self, i: int) -> int:
        """Length of x_ext(i) (the column count of slice i's matrix)."""
        if self.direct:
            return max(int(self.arena.numel() - self.offsets[i]), self.slices[i].m_local)
        return self.slices[i].n_ext

    def x_ext(self, i: int) -> torch.Tensor:
        if self.direct:
            return self.arena[int(self.offsets[i]):]
        return self.arena[int(self.offsets[i]):int(self.offsets[i + 1])]

    def x_local(self, i: int) -> torch.Tensor:
        return self.arena[int(self.offsets[i]):int(self.offsets[i]) + self.slices[i].m_local]

    @property
    def bytes_per_exchange(self) -> int:
        """Halo bytes this rank sends plus receives per exchange."""
        return int(self.pack_idx.numel() + self.n_recv) * self.arena.element_size()

    def exchange(self) -> None:
        self.start()
        self.finish()

    def start(self) -> None:
        """Pack and launch the all-to-all (asynchronous on RCCL: the local,
        interior part of the SpMV can run meanwhile; finish() joins it)."""
        self._work = None
        if self.P <= 1:
            return
        n_send, n_recv = self.pack_idx.numel(), self.n_recv
        if self.device.type == "cuda":
            from .sparse import gather
            if n_send:
                gather(self.handle, self.pack_idx, self.arena, self.sendbuf)
            if dist.get_backend(self.group) == "gloo":  # rehearsal: synchronous, staged
                _a2a(self.recvbuf[:n_recv], self.sendbuf[:n_send], self.recv_split, self.send_split,
                     self.group)
            else:
                self._work = dist.all_to_all_single(self.recvbuf[:n_recv], self.sendbuf[:n_send],
                                                    list(self.recv_split), list(self.send_split),
                                                    group=self.group, async_op=True)
        else:  # CPU tensors: gloo tests of the host logic
            self.sendbuf[:n_send] = self.arena[self.pack_idx]
            dist.all_to_all_single(self.recvbuf[:n_recv], self.sendbuf[:n_send],
                                   list(self.recv_split), list(self.send_split), group=self.group)
        assert sum(self.recv_split) == n_recv

    def finish(self) -> None:
        """Wait for the all-to-all (on the current stream) and unpack the halos."""
        if self.P <= 1:
            return
        if self._work is not None:
            self._work.wait()
            self._work = None
        if self.direct:  # received in place
            return
        n_recv = self.unpack_idx.numel()
        if self.device.type == "cuda":
            from .sparse import scatter
            if n_recv:
                scatter(self.handle, self.unpack_idx, self.recvbuf, self.arena)
        else:
            self.arena[self.unpack_idx] = self.recvbuf[:n_recv]
