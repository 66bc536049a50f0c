"""Tile-geometry / cost-breakdown probe of the SpMV kernel (diagnostics only).

Each probe is a separate build of librsp.so (respasol_amd/build/probe/<name>,
`make -C respasol_amd/csrc probe PROBE_NAME=<name> PROBE_DEFS=...`) loaded in
its own child process through RSP_PROBE_LIB. The child times the cycled big
set exactly like bench.py (one event pair around K passes, fp64 then fp32)
and prints one JSON line. The loadsonly probe (RSP_SPMV_PROBE_LOADS,
respasol_amd/csrc/spmv_probe.h) computes wrong results on purpose: the tile's
stream alone, the ceiling of the tile structure.

    python scripts/spmv_probe.py --build                  # here (CPU): build all probes
    python scripts/spmv_probe.py [--probes base,it8]      # on the GPU box
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBES = {  # (round 5: the gather / reduce / y-store / walk / policy probes measured in
    # rounds 2-4 were removed from spmv.hip with their macros; DESIGN.md §5 keeps the numbers)
    "base": "",
    "it6": "-DRSP_SPMV_ITER=6",
    "it8": "-DRSP_SPMV_ITER=8",
    "loadsonly": "-DRSP_SPMV_PROBE_LOADS",
    "nty": "-DRSP_NT_Y=1",
    "plainy": "-DRSP_NT_Y=0",
    "rows256": "-DRSP_SPMV_MAXROWS=256",
    "rows1024": "-DRSP_SPMV_MAXROWS=1024",
    "t512": "-DRSP_SPMV_THREADS=512",
    "t512r1k": "-DRSP_SPMV_THREADS=512 -DRSP_SPMV_MAXROWS=1024",
    "t512it2": "-DRSP_SPMV_THREADS=512 -DRSP_SPMV_ITER=2",
}


def lib_path(name):
    return os.path.join(ROOT, "respasol_amd", "build", "probe", name, "librsp.so")


def build(names):
    for n in names:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "respasol_amd", "csrc"), "probe",
                        f"PROBE_NAME={n}", f"PROBE_DEFS={PROBES[n]}"], check=True)
        print("built", lib_path(n))


def child(steps, workload):
    import torch
    sys.path.insert(0, ROOT)
    from respasol_amd import csr
    from respasol_amd.sparse import Handle, SpMat, upload_csr
    h = Handle()
    names = (csr.surrogate_names(1 if workload == "big" else 0) if workload in ("big", "moderate")
             else workload.split(","))
    out = {}
    for dt, elem in ((torch.float64, 8), (torch.float32, 4)):
        mats, nbytes, flops = [], 0, 0
        for n in names:
            A = csr.surrogate(n)
            M = SpMat(h, *upload_csr(A.rowptr, A.colidx, A.values, dt), A.n)
            x = torch.ones(A.n, dtype=dt, device="cuda")
            y = torch.empty(A.m, dtype=dt, device="cuda")
            mats.append((M, x, y))
            nbytes += (elem + 4) * A.nnz_stored + 4 * (A.m + 1) + elem * (A.n + A.m)
            flops += 2 * A.nnz_stored
        for M, x, y in mats:
            M.spmv(x, y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            for M, x, y in mats:
                M.spmv(x, y)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        key = "f64" if dt == torch.float64 else "f32"
        out[key] = {"ms_per_pass": round(ms, 4), "gflops": round(flops / ms / 1e6, 1),
                    "gbps": round(nbytes / ms / 1e6, 1)}
        del mats
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def stream_ref():
    """Device read bandwidth references: torch sum over 2 GiB, and a 2 GiB copy."""
    import torch
    a = torch.ones(2 ** 28, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    out = {}
    for name, fn, nbytes in (("sum_read", lambda: a.sum(), a.numel() * 8),
                             ("copy_rw", lambda: b.copy_(a), a.numel() * 16)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_gbps"] = round(nbytes * 10 / (e0.elapsed_time(e1) * 1e6), 1)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--probes", default=",".join(PROBES))
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--workload", default="big")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--stream-ref", action="store_true")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    names = args.probes.split(",")
    if args.build:
        build(names)
        return
    if args.stream_ref:
        stream_ref()
        return
    if args.child:
        child(args.steps, args.workload)
        return
    for rnd in range(args.rounds):  # interleaved rounds, to see the box noise
        for n in names:
            env = dict(os.environ, RSP_PROBE_LIB=lib_path(n))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--steps",
                                str(args.steps), "--workload", args.workload], env=env,
                               capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(n, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
                sys.exit(r.returncode)
            print(f"round {rnd} {n:10s} {r.stdout.strip()}", flush=True)


if __name__ == "__main__":
    main()
