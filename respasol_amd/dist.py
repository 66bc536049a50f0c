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
