"""BASELINE config 3: level-scheduled ILU(0) factor + L / L^T solves on the
21 moderate matrices (surrogates), fp64, fp32 (the parity configuration)
and fp32+FTZ (an extension: the reference's -ftz flag is commented out,
GPU/Makefile:5), on one MI355X, with
the oracle's sequential CPU time beside it and a bitwise parity check.

    python scripts/bench_ilu0.py [--set moderate] [--reps 3] [--json out.json]

Times (ms): analysis (rsp_ilu0_analysis = csrilu02_analysis, the
reference's timed "Symbolic", wall clock) and the two trsv analyses
(rsp_trsv_analysis = csrsv2_analysis, untimed in the reference, wall clock),
factor and solve (L then L^T, the reference's "Solve", GPU/ilu0.cu:284-310)
as HIP event pairs, median of --reps.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_bind as ob  # noqa: E402  (checker + CPU reference time)
from respasol_amd import csr  # noqa: E402
from respasol_amd.sparse import Handle, Ilu0, upload_csr  # noqa: E402


def run_one(h, A, dt, ftz, reps):
    npdt = np.float64 if dt == torch.float64 else np.float32
    h.set_ftz(ftz)
    rp, ci, va0 = upload_csr(A.rowptr, A.colidx, A.values, dt)
    il = Ilu0(h, rp, ci)
    t0 = time.perf_counter()
    il.analysis()  # csrilu02_analysis: the reference's timed "Symbolic" (GPU/ilu0.cu:196-217)
    t_an = (time.perf_counter() - t0) * 1e3
    assert il.zero_pivot() == -1
    t0 = time.perf_counter()
    il.trsv_analysis()  # the two csrsv2_analysis (:228-252), untimed there
    il.trsv_analysis(transpose=True)
    t_tan = (time.perf_counter() - t0) * 1e3
    lev = il.levels()
    x = torch.ones(A.n, dtype=dt, device="cuda")
    tf, ts = [], []
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for rep in range(reps + 1):  # rep 0: warm-up (first-call graph capture), not timed
        va = va0.clone()
        torch.cuda.synchronize()
        e[0].record()
        il.factor(va)
        e[1].record()
        z = il.solve_lower(va, x)
        y = il.solve_lower(va, z, transpose=True)
        e[2].record()
        torch.cuda.synchronize()
        if rep:
            tf.append(e[0].elapsed_time(e[1]))
            ts.append(e[1].elapsed_time(e[2]))
    zp = il.zero_pivot()
    # parity (bitwise) and the sequential CPU time of the same arithmetic
    t0 = time.perf_counter()
    rv, _, rzp = ob.ilu0(A.rowptr, A.colidx, A.values.astype(npdt), ftz=ftz)
    t_cf = (time.perf_counter() - t0) * 1e3
    # the CPU time is the reference's own sequential solves (L column
    # ascending, L^T column sweep); the parity check (untimed) follows the
    # plan's order, which is the reference's order unless RSP_ILU_SPLIT=1
    t0 = time.perf_counter()
    cz = ob.trsv("lower_n_ref", A.rowptr, A.colidx, rv, np.ones(A.n, npdt), ftz=ftz)
    ob.trsv("lower_t_ref", A.rowptr, A.colidx, rv, cz, ftz=ftz)
    t_cs = (time.perf_counter() - t0) * 1e3
    rz = ob.trsv("lower_n", A.rowptr, A.colidx, rv, np.ones(A.n, npdt), ftz=ftz)
    ry = ob.trsv("lower_t", A.rowptr, A.colidx, rv, rz, ftz=ftz)
    ok = (zp == rzp and np.array_equal(va.cpu().numpy(), rv) and np.array_equal(y.cpu().numpy(), ry))
    h.set_ftz(False)
    # SURVEY §8d (reporting only): factor >= 20 nnz_s + 4(m+1) + 4m bytes, each
    # trsv >= 12 nnz_L + 4(m+1) + 16m; graded on time, not roofline
    m, nnz_s = A.m, A.nnz_stored
    nnz_l = int(np.sum(A.colidx[:nnz_s] < np.repeat(np.arange(m), np.diff(A.rowptr))))
    fbytes = 20 * nnz_s + 4 * (m + 1) + 4 * m
    sbytes = 2 * (12 * nnz_l + 4 * (m + 1) + 16 * m)
    fac, sol = statistics.median(tf), statistics.median(ts)
    return {"analysis_ms": round(t_an, 3), "trsv_analysis_ms": round(t_tan, 3), "factor_ms": round(fac, 4),
            "solve_ms": round(sol, 4), "levels_L": lev[0], "levels_LT": lev[1],
            "factor_gbps": round(fbytes / (fac * 1e6), 1), "solve_gbps": round(sbytes / (sol * 1e6), 1),
            "cpu_factor_ms": round(t_cf, 3), "cpu_solve_ms": round(t_cs, 3), "bitwise_ok": bool(ok)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="moderate")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default="")
    ap.add_argument("--fp64-only", action="store_true", help="A/B runs: fp64 only (fp32 columns repeat it)")
    args = ap.parse_args()
    names = csr.surrogate_names(0 if args.set == "moderate" else 1) if args.set in ("moderate", "big") \
        else args.set.split(",")
    h = Handle()
    out = []
    print(f"{'matrix':16s} {'n':>8s} {'nnz_s':>9s} {'lvL':>5s} {'lvT':>5s} | "
          f"{'fp64 fac':>9s} {'solve':>8s} | {'fp32 fac':>9s} {'solve':>8s} | {'fp32ftz fac':>11s} {'solve':>8s} | "
          f"{'cpu fac':>8s} {'cpu slv':>8s} ok")
    for name in names:
        A = csr.surrogate(name)
        r64 = run_one(h, A, torch.float64, False, args.reps)
        r32p = r64 if args.fp64_only else run_one(h, A, torch.float32, False, args.reps)
        r32 = r64 if args.fp64_only else run_one(h, A, torch.float32, True, args.reps)
        row = {"matrix": name, "n": A.m, "nnz_s": A.nnz_stored, "fp64": r64, "fp32": r32p, "fp32_ftz": r32}
        out.append(row)
        print(f"{name:16s} {A.m:8d} {A.nnz_stored:9d} {r64['levels_L']:5d} {r64['levels_LT']:5d} | "
              f"{r64['factor_ms']:9.3f} {r64['solve_ms']:8.3f} | {r32p['factor_ms']:9.3f} {r32p['solve_ms']:8.3f} | "
              f"{r32['factor_ms']:11.3f} "
              f"{r32['solve_ms']:8.3f} | {r64['cpu_factor_ms']:8.2f} {r64['cpu_solve_ms']:8.2f} "
              f"{r64['bitwise_ok'] and r32p['bitwise_ok'] and r32['bitwise_ok']}", flush=True)
    tot = lambda k, p: sum(r[p][k] for r in out)  # noqa: E731
    gb = lambda k, p: statistics.median(r[p][k] for r in out)  # noqa: E731
    print(f"median algorithmic GB/s (SURVEY 8d, reporting only; 8000 = HBM peak): fp64 factor "
          f"{gb('factor_gbps', 'fp64'):.1f} solve {gb('solve_gbps', 'fp64'):.1f}")
    print(f"TOTAL fp64 factor {tot('factor_ms', 'fp64'):.2f} ms solve {tot('solve_ms', 'fp64'):.2f} ms; "
          f"fp32 factor {tot('factor_ms', 'fp32'):.2f} solve {tot('solve_ms', 'fp32'):.2f}; "
          f"fp32+ftz factor {tot('factor_ms', 'fp32_ftz'):.2f} solve {tot('solve_ms', 'fp32_ftz'):.2f}; "
          f"cpu(1 thread) factor {tot('cpu_factor_ms', 'fp64'):.1f} solve {tot('cpu_solve_ms', 'fp64'):.1f}")
    print(f"ANALYSIS fp64 ilu (Symbolic) {tot('analysis_ms', 'fp64'):.1f} ms; trsv (untimed in the reference) "
          f"{tot('trsv_analysis_ms', 'fp64'):.1f} ms")
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
