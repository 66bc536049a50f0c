"""CPU baseline leg of bench.py (TEST INFRASTRUCTURE: it times the oracle's
OpenMP CSR SpMV, the restated CPU path of the reference's test_spmv.c,
test_spmv.c:165-183). bench.py starts it as a child process so that the
OpenMP placement (OMP_NUM_THREADS, OMP_PROC_BIND=close, OMP_PLACES = one
logical CPU per physical core) is in the environment before the OpenMP
runtime starts; it prints one JSON object.

    python tests/cpu_baseline_run.py --workload big --method B --seconds 10
      B: steady state, repeated full passes over the workload for `seconds`
      A: the reference's methodology, ONE cold call per matrix
         (run_spmv.sh:45 OMP_NUM_THREADS=4 taskset -c 0-3; test_spmv.c:165-183)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def topology(cpus):
    """{cpu: (socket, core)} for the given logical CPUs (sysfs)."""
    topo = {}
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            sock = int(open(base + "physical_package_id").read())
            core = int(open(base + "core_id").read())
        except OSError:
            sock, core = 0, c
        topo[c] = (sock, core)
    return topo


def placement(max_threads):
    """One logical CPU per physical core of the socket holding most of this
    process's CPU set, at most max_threads of them. Returns (cpus, facts)."""
    mask = sorted(os.sched_getaffinity(0))
    topo = topology(mask)
    per_sock = {}
    for c in mask:
        s, k = topo[c]
        per_sock.setdefault(s, {}).setdefault(k, c)  # first logical CPU of each core
    sock = max(per_sock, key=lambda s: len(per_sock[s]))
    cores = sorted(per_sock[sock].values())
    use = cores[:max(1, min(max_threads, len(cores)))]
    facts = {"cpuset_cpus": len(mask), "sockets_in_cpuset": len(per_sock),
             "physical_cores_socket": len(cores), "socket": sock, "threads": len(use),
             "places": use}
    return use, facts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="big")
    ap.add_argument("--method", default="B", choices=["A", "B"])
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--threads", type=int, default=0,
                    help="B: threads (default: the physical cores of one socket in the CPU set, "
                         "capped by the CPU share the environment gives this job, OMP_NUM_THREADS)")
    args = ap.parse_args()
    if args.method == "A":
        want = 4
    elif args.threads > 0:
        want = args.threads
    else:
        share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        want = share if share > 0 else 1 << 30
    cpus, facts = placement(want)
    # before the OpenMP runtime starts (it starts when the libraries load)
    os.environ["OMP_NUM_THREADS"] = str(len(cpus))
    os.environ["OMP_PROC_BIND"] = "close"
    os.environ["OMP_PLACES"] = ",".join("{%d}" % c for c in cpus)
    os.environ["RSP_HOST_ONLY"] = "1"
    global ob, csr
    import oracle_bind as ob  # noqa: E402  (the checker's CPU restatement)
    from respasol_amd import csr  # noqa: E402
    names = csr.surrogate_names(1) if args.workload == "big" else (
        csr.surrogate_names(0) if args.workload == "moderate" else args.workload.split(","))
    mats = []
    for n in names:
        m = csr.surrogate_rows(n)
        rp, ci, va = csr.surrogate_rows_csr(n, 0, m)
        mats.append((rp, ci, va, csr.dlarnv(1, [0, 0, 0, 1], m)[0]))
    threads = ob.lib.oracle_num_threads()
    flops_pass = sum(2.0 * int(rp[-1]) for rp, *_ in mats)
    if args.method == "A":  # one cold call per matrix, summed
        t = 0.0
        for rp, ci, va, x in mats:
            t0 = time.perf_counter()
            ob.spmv(rp, ci, va, x, threads=True)
            t += time.perf_counter() - t0
        print(json.dumps({"gflops": flops_pass / t / 1e9, "seconds": t, "threads": threads, "placement": facts}))
        return
    for rp, ci, va, x in mats:  # page-in pass
        ob.spmv(rp, ci, va, x, threads=True)
    passes, t0 = 0, time.perf_counter()
    while True:
        for rp, ci, va, x in mats:
            ob.spmv(rp, ci, va, x, threads=True)
        passes += 1
        el = time.perf_counter() - t0
        if el >= args.seconds:
            break
    print(json.dumps({"gflops": flops_pass * passes / el / 1e9, "seconds": el, "passes": passes,
                      "threads": threads, "placement": facts}))


if __name__ == "__main__":
    main()
