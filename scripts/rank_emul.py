"""Per-rank compute of the N-GPU bench, emulated on one GPU (diagnostics only).

For world W and a rank r, builds that rank's row slice of every big matrix
(nnz-balanced split, global column indices, full x) and times one step's 15
SpMVs three ways: eager Python launches (host wall + GPU events), and one HIP
graph replay per step. Shows whether a rank's step at N = 8 is bound by the
host's launch rate rather than the kernels.

    python scripts/rank_emul.py [--worlds 2,4,8] [--steps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from respasol_amd import csr  # noqa: E402
from respasol_amd.sparse import Handle, SpMat, SpmvBatch, upload_csr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--merged", action="store_true")
    args = ap.parse_args()
    h = Handle()
    stream = torch.cuda.current_stream()
    names = csr.surrogate_names(1)
    for W in [int(w) for w in args.worlds.split(",")]:
        for r in sorted({0, W - 1}):
            mats, hosts = [], []
            for n in names:
                m = csr.surrogate_rows(n)
                lens = csr.surrogate_rowlens(n)
                rp = np.zeros(m + 1, np.int64)
                np.cumsum(lens, out=rp[1:])
                b = csr.partition_rows(rp.astype(np.int32), W)
                r0, r1 = int(b[r]), int(b[r + 1])
                lrp, ci, va = csr.surrogate_rows_csr(n, r0, r1)
                if args.merged:
                    hosts.append((lrp, ci, va))
                M = SpMat(h, *upload_csr(lrp, ci, va, torch.float64), m)
                x = torch.ones(m, dtype=torch.float64, device="cuda")
                y = torch.empty(max(r1 - r0, 1), dtype=torch.float64, device="cuda")
                mats.append((M, x, y, int(lrp[-1])))

            def step():
                for M, x, y, _ in mats:
                    M.spmv(x, y)

            step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            for _ in range(args.steps):
                step()
            t_host = time.perf_counter() - t0
            e1.record(stream)
            torch.cuda.synchronize()
            eager_ms = e0.elapsed_time(e1) / args.steps
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                h.set_stream(torch.cuda.current_stream())
                step()
            h.set_stream(stream)
            g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(stream)
            for _ in range(args.steps):
                g.replay()
            t_host_g = time.perf_counter() - t0
            e1.record(stream)
            torch.cuda.synchronize()
            graph_ms = e0.elapsed_time(e1) / args.steps
            flops = 2.0 * sum(q[3] for q in mats)
            B = SpmvBatch(h, [q[0] for q in mats], [q[1] for q in mats], [q[2] for q in mats])
            B.run()
            torch.cuda.synchronize()
            e0.record(stream)
            for _ in range(args.steps):
                B.run()
            e1.record(stream)
            torch.cuda.synchronize()
            batch_ms = round(e0.elapsed_time(e1) / args.steps, 4)
            B.close()
            merged_ms = None
            if args.merged:  # the same 15 slices as one block-diagonal matrix, one launch
                rps, cis, vas, off, base = [np.zeros(1, np.int64)], [], [], 0, 0
                for n, (lrp, ci, va) in zip(names, hosts):
                    rps.append(lrp[1:].astype(np.int64) + base)
                    cis.append(ci.astype(np.int64) + off)
                    vas.append(va)
                    base += int(lrp[-1])
                    off += csr.surrogate_rows(n)
                rpm = np.concatenate(rps)
                Mm = SpMat(h, *upload_csr(rpm, np.concatenate(cis).astype(np.int32),
                                          np.concatenate(vas), torch.float64), off)
                xm = torch.ones(off, dtype=torch.float64, device="cuda")
                ym = torch.empty(len(rpm) - 1, dtype=torch.float64, device="cuda")
                Mm.spmv(xm, ym)
                torch.cuda.synchronize()
                e0.record(stream)
                for _ in range(args.steps):
                    Mm.spmv(xm, ym)
                e1.record(stream)
                torch.cuda.synchronize()
                merged_ms = round(e0.elapsed_time(e1) / args.steps, 4)
                del Mm, xm, ym
            print(json.dumps({"world": W, "rank": r, "eager_ms": round(eager_ms, 4),
                              "eager_host_ms": round(t_host * 1e3 / args.steps, 4),
                              "graph_ms": round(graph_ms, 4),
                              "graph_host_ms": round(t_host_g * 1e3 / args.steps, 4),
                              "graph_gflops": round(flops / graph_ms / 1e6, 1),
                              "batch_ms": batch_ms, "merged_ms": merged_ms}), flush=True)
            del mats, g
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
