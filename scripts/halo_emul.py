"""One rank's overlapped halo step of the N-GPU bench, emulated on one GPU
(diagnostics only: kernels and launch gaps, no RCCL).

For world W and rank r, builds every rank's row slice of the big set on the
host (to know who asks r for what), then rank r's HaloExchange with a stand-in
for the two setup all-to-alls, and times the step's kernels back to back with
the all-to-all left out:
  packed : pack (rsp_gather) -> interior tiles -> unpack (rsp_scatter) -> boundary tiles
  direct : pack -> interior tiles -> boundary tiles   (halo received in place)
and, for reference, the slice's whole SpMV as one batched launch.

    python scripts/halo_emul.py [--worlds 2,4,8] [--steps 50]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from respasol_amd import csr, dist as rdist  # noqa: E402
from respasol_amd.sparse import Handle, SpMat, SpmvBatch, upload_csr  # noqa: E402


class _FakeDist:
    """Answers HaloExchange's two setup all-to-alls for rank r from every
    rank's HaloSlices; the per-step all-to-all returns at once."""

    def __init__(self, all_slices, r):
        self.all, self.r, self.calls = all_slices, r, 0

    def get_backend(self, group=None):
        return "nccl"

    def all_to_all_single(self, out, inp, out_splits, in_splits, group=None, async_op=False):
        P = len(self.all)
        if self.calls == 0:  # counts: [p][i] = how many columns slice i of p wants from r
            v = [self.all[p][i].recv_counts[self.r] for p in range(P) for i in range(len(self.all[p]))]
            out.copy_(torch.tensor(v, dtype=out.dtype))
        elif self.calls == 1:  # the columns every p asks r for, (p, slice) order
            cols = [self.all[p][i].recv_cols[self.r] for p in range(P) for i in range(len(self.all[p]))]
            out.copy_(torch.from_numpy(np.concatenate(cols).astype(np.int64)))
        self.calls += 1
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    h = Handle()
    names = csr.surrogate_names(1)
    for W in [int(w) for w in args.worlds.split(",")]:
        all_slices = [[] for _ in range(W)]
        mine = {}
        for n in names:
            m = csr.surrogate_rows(n)
            rp = np.zeros(m + 1, np.int64)
            np.cumsum(csr.surrogate_rowlens(n), out=rp[1:])
            b = csr.partition_rows(rp.astype(np.int32), W)
            for p in range(W):
                lrp, ci, va = csr.surrogate_rows_csr(n, int(b[p]), int(b[p + 1]))
                all_slices[p].append(rdist.HaloSlice(ci, b, p))
                if p in (0, W - 1):
                    mine.setdefault(p, []).append((lrp, va))
        for r in sorted({0, W - 1}):
            res = {}
            for direct in (False, True):
                real = rdist.dist
                rdist.dist = _FakeDist(all_slices, r)
                try:
                    ex = rdist.HaloExchange(all_slices[r], r, W, torch.float64, "cuda", h, direct=direct)
                finally:
                    rdist.dist = real
                mats, ys = [], []
                for i, (lrp, va) in enumerate(mine[r]):
                    M = SpMat(h, *upload_csr(lrp, ex.colidx(i), va, torch.float64), ex.n_x(i))
                    M.set_local_cols(all_slices[r][i].m_local)
                    mats.append(M)
                    ys.append(torch.empty(max(all_slices[r][i].m_local, 1), dtype=torch.float64,
                                          device="cuda"))
                xs = [ex.x_ext(i) for i in range(len(mats))]
                b1, b2, b0 = (SpmvBatch(h, mats, xs, ys, part) for part in (1, 2, 0))
                from respasol_amd.sparse import gather, scatter

                def step():
                    if ex.pack_idx.numel():
                        gather(h, ex.pack_idx, ex.arena, ex.sendbuf)
                    b1.run()
                    if not direct and ex.unpack_idx.numel():
                        scatter(h, ex.unpack_idx, ex.recvbuf, ex.arena)
                    b2.run()

                def timed(fn):
                    for _ in range(3):
                        fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record()
                    for _ in range(args.steps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    return e0.elapsed_time(e1) / args.steps

                res[direct] = (timed(step), timed(b0.run), ex.n_recv, b1.info()["entries_16bit"]
                               + b2.info()["entries_16bit"])
            (tp, wp, nr, e16p), (td, wd, _, e16d) = res[False], res[True]
            print(f"W={W} r={r}: step packed {tp * 1e3:.1f} us, direct {td * 1e3:.1f} us; whole-slice "
                  f"batch {wp * 1e3:.1f} / {wd * 1e3:.1f} us; halo {nr} entries; 16-bit entries "
                  f"{e16p} / {e16d}", flush=True)


if __name__ == "__main__":
    main()
