"""Benchmark of the hot path: CSR SpMV on MI355X (BASELINE.json metric
"CSR SpMV GFLOP/s + achieved HBM GB/s (fp64 vs fp32), SuiteSparse set,
1/2/4/8 GPU").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload big|moderate|NAME]
    torchrun --nproc-per-node N ... bench.py --gpus N ...      (N > 1, RCCL)

With --gpus N > 1 and no WORLD_SIZE in the environment (a plain `python
bench.py --gpus N`), bench.py launches the N ranks itself: N child processes
(one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT set), spawned before anything loads the HIP runtime; the parent
relays rank 0's JSON line and exits non-zero if any rank fails. Under
torchrun the ranks come from the environment; --gpus must equal WORLD_SIZE,
and with the nccl backend every rank needs a GPU of its own.

Workload (default "big"): one step = one fp64 y = A x over EACH of the 15
"big" SuiteSparse matrices (BASELINE config 4; seeded surrogates of the same
m / stored nnz / structure, since no .mtx data exists offline). With N > 1
every matrix is row-partitioned (nnz-balanced) across the ranks; one bucketed
RCCL all_to_all_single per step moves each rank's halo of x over xGMI while
the interior tiles (own columns only) run, then the boundary tiles finish
(config 5 applied to the whole set; --no-overlap / --exchange allgather are
the simpler variants); total work is fixed => "scaling": "strong". A
step's SpMVs go out as one batched launch (rsp_spmv_batch; --no-batch: one
launch per matrix, also timed and reported as "per_matrix_calls"). Cycling
through 3.4 GB of matrices per step also keeps the 256 MB Infinity Cache
from serving any matrix twice, so the rate is an HBM rate.

value = total GFLOP of all ranks / max-over-ranks wall time of the K steps.
roofline = the dominant kernel (spmv_tiles_batch: the step's one launch over
all 15 matrices; spmv_tiles per matrix with --no-batch) timed
with one HIP event pair on the stream it runs on around the K steps (N = 1:
the timed region itself; N > 1: a kernel-only repeat of the K steps):
algorithmic bytes / average launch duration against 8 TB/s. cpu_baseline = the oracle's OpenMP CSR SpMV (the reference's
test_spmv.c CPU path, restated) on a bounded sample, rank 0, N = 1 only.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# product modules (they map librsp.so) and torch: imported by _import_product()
# once this process is known to be a rank, never in the launcher parent
np = torch = dist = csr = None
HaloExchange = HaloSlice = RowPartitionedSpmv = remap_columns = None
Handle = SpMat = SpmvBatch = upload_csr = None


def _import_product():
    global np, torch, dist, csr, HaloExchange, HaloSlice, RowPartitionedSpmv, remap_columns
    global Handle, SpMat, SpmvBatch, upload_csr
    import numpy as np_
    import torch as torch_
    import torch.distributed as dist_
    from respasol_amd import csr as csr_
    from respasol_amd import dist as rd
    from respasol_amd import sparse as sp
    np, torch, dist, csr = np_, torch_, dist_, csr_
    HaloExchange, HaloSlice, RowPartitionedSpmv, remap_columns = (rd.HaloExchange, rd.HaloSlice,
                                                                  rd.RowPartitionedSpmv, rd.remap_columns)
    Handle, SpMat, SpmvBatch, upload_csr = sp.Handle, sp.SpMat, sp.SpmvBatch, sp.upload_csr


# ---------------------------------------------------------------- launcher
def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, base_env, port, addr="127.0.0.1"):
    """The environment of each of the n ranks a single-node launch starts (the
    variables torch.distributed.run sets that bench.py and init_process_group
    read)."""
    envs = []
    for r in range(n):
        e = dict(base_env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "NODE_RANK": "0",
                  "MASTER_ADDR": addr, "MASTER_PORT": str(port),
                  "HSA_ENABLE_IPC_MODE_LEGACY": base_env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
                  "PYTHONUNBUFFERED": "1"})
        envs.append(e)
    return envs


def launch_ranks(n, child_argv, base_env=None, timeout=None, out=None):
    """Start n rank processes (child_argv each, environments from rank_envs),
    relay rank 0's stdout to `out` (default sys.stdout; the other ranks'
    stdout goes to stderr), wait for all of them. If one fails, the others are
    terminated. Returns the exit code: 0 only if every rank exited 0."""
    base_env = dict(os.environ if base_env is None else base_env)
    out = sys.stdout if out is None else out
    procs = []
    for r, env in enumerate(rank_envs(n, base_env, free_port())):
        procs.append(subprocess.Popen(child_argv, env=env, stdout=subprocess.PIPE if r == 0 else 2,
                                      start_new_session=True, text=True))
    # rank 0's stdout is drained on a thread, so a full pipe never blocks it
    import threading

    def pump():
        for line in procs[0].stdout:
            out.write(line)
            out.flush()
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    t0 = time.time()
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0:
                print(f"bench.py launcher: rank {r} exited with {c}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                rc = rc or (c if c > 0 else 1)
                for q in live:
                    try:
                        os.killpg(procs[q].pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        if timeout is not None and time.time() - t0 > timeout and live:
            print("bench.py launcher: time limit reached; stopping the ranks", file=sys.stderr, flush=True)
            for q in live:
                try:
                    os.killpg(procs[q].pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
            rc = rc or 124
            timeout = None
        time.sleep(0.05)
    th.join(timeout=10)
    return rc


def visible_gpus():
    """GPUs this process could use, counted without initialising the HIP
    runtime (torch.cuda.device_count() does not on this image)."""
    import torch as torch_
    return int(torch_.cuda.device_count())


def check_world(args, world, n_visible):
    """None if this rank may run, else the reason it must not: --gpus must
    equal the launched world, and the nccl backend needs one GPU per rank."""
    if args.gpus != world:
        return (f"--gpus {args.gpus} but WORLD_SIZE is {world}: the JSON line would name the wrong "
                f"number of GPUs")
    if world > 1 and args.dist_backend == "nccl" and n_visible < world:
        return (f"--gpus {world} with the nccl backend needs {world} GPUs, {n_visible} visible "
                f"(use --dist-backend gloo only to rehearse N > 1 ranks sharing one GPU)")
    return None


METRIC = "CSR SpMV GFLOP/s + achieved HBM GB/s (fp64 vs fp32), SuiteSparse set, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


class Slice:
    """One matrix's share on this rank: its rows [r0, r1) (nnz-balanced split),
    generated locally, with the column layout of the chosen exchange."""

    def __init__(self, name, rank, world, handle, device, exchange, overlap=False, meta=None):
        self.name = name
        m, self.nnz_global, self.bounds = meta if meta is not None else partition_meta([name], world)[0]
        self.m, self.n = m, m
        r0, r1 = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.r0, self.r1 = r0, r1
        self.m_local = r1 - r0
        rp, ci, va = csr.surrogate_rows_csr(name, r0, r1)
        self.nnz_local = int(rp[-1])
        self.x_global_slice = csr.dlarnv(1, [0, 0, 0, 1], m)[0][r0:r1]
        self.mode = exchange if world > 1 else "none"
        self.ci_global = ci
        self.handle, self.device, self.overlap = handle, device, overlap
        if self.mode == "halo":  # matrices uploaded by bind_halo, in the exchange's column layout
            self.halo = HaloSlice(ci, self.bounds, rank)
            self.n_x = self.halo.n_ext  # x entries the slice reads (algorithmic bytes)
            self.host = (rp, None, va)
        else:
            if self.mode == "allgather":
                ci_dev, chunk = remap_columns(ci, self.bounds)
                self.n_x = world * chunk
            else:
                ci_dev, self.n_x = ci, m
            self.host = (rp, ci_dev, va)
            self._upload(ci_dev, self.n_x)
        self.y64 = torch.empty(max(self.m_local, 1), dtype=torch.float64, device=device)
        self.y32 = torch.empty(max(self.m_local, 1), dtype=torch.float32, device=device)
        if self.mode != "halo":  # replicated x (padded layout for the all-gather)
            self.part64 = RowPartitionedSpmv(self.bounds, rank, torch.float64, device, None)
            self.part32 = RowPartitionedSpmv(self.bounds, rank, torch.float32, device, None)
            self.part64.set_local_x(torch.from_numpy(self.x_global_slice).to(device))
            self.part32.set_local_x(torch.from_numpy(self.x_global_slice.astype(np.float32)).to(device))
            self.part64.exchange()
            self.part32.exchange()

    def _upload(self, ci_dev, ncols):
        rp, _, va = self.host
        self.mat64 = SpMat(self.handle, *upload_csr(rp, ci_dev, va, torch.float64, self.device), ncols)
        self.mat32 = SpMat(self.handle, *upload_csr(rp, ci_dev, va, torch.float32, self.device), ncols)
        if self.mode == "halo" and self.overlap:  # interior tiles (own columns only) run under the exchange
            self.mat64.set_local_cols(self.m_local)
            self.mat32.set_local_cols(self.m_local)

    def bind_halo(self, i, ex64, ex32):
        self.i, self.ex64, self.ex32 = i, ex64, ex32
        ci_dev = ex64.colidx(i)  # same layout in both arenas
        self.host = (self.host[0], ci_dev, self.host[2])
        self._upload(ci_dev, ex64.n_x(i))
        ex64.x_local(i).copy_(torch.from_numpy(self.x_global_slice))
        ex32.x_local(i).copy_(torch.from_numpy(self.x_global_slice.astype(np.float32)))

    def x64(self):
        return self.ex64.x_ext(self.i) if self.mode == "halo" else self.part64.x_full

    def x32(self):
        return self.ex32.x_ext(self.i) if self.mode == "halo" else self.part32.x_full

    def bytes_local(self, elem):
        """Algorithmic bytes of this rank's SpMV: vals+colidx,
        rowptr, one read of the x the slice references (n at N = 1, the
        replicated x for the all-gather, local + halo for the halo exchange),
        y write."""
        return (elem + 4) * self.nnz_local + 4 * (self.m_local + 1) + elem * self.n_x + elem * self.m_local


def partition_meta(names, world, rank=0, device=None):
    """Per matrix (m, stored nnz, nnz-balanced row bounds for `world` ranks).
    The bounds need every row's length: rank 0 generates them and broadcasts
    the result (world > 1), so the ranks' setup does not repeat the
    whole-matrix pass — each rank then generates only its own rows (Slice)."""
    meta = None
    if rank == 0:
        meta = []
        for name in names:
            m = csr.surrogate_rows(name)
            rowptr = np.zeros(m + 1, np.int64)
            np.cumsum(csr.surrogate_rowlens(name), out=rowptr[1:])
            meta.append((m, int(rowptr[-1]), csr.partition_rows(rowptr.astype(np.int32), world)))
    if world == 1 or not dist.is_initialized():
        return meta
    flat = torch.zeros(len(names) * (world + 3), dtype=torch.int64)
    if rank == 0:
        flat.copy_(torch.tensor([v for m, nnz, b in meta for v in (m, nnz, *map(int, b))], dtype=torch.int64))
    on = flat.to(device) if dist.get_backend() == "nccl" else flat
    dist.broadcast(on, 0)
    rows = on.cpu().view(len(names), world + 3).numpy()
    return [(int(r[0]), int(r[1]), r[2:].astype(np.int32)) for r in rows]


def workload_names(w):
    if w == "big":
        return csr.surrogate_names(1)
    if w == "moderate":
        return csr.surrogate_names(0)
    return w.split(",")


def host_cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(workload, seconds, threads=0):
    """The reference's CPU path (test_spmv.c's CSR SpMV, restated by the
    oracle as an OpenMP row-parallel loop) on the same matrices, two ways
    (BASELINE.md §4), each in a child process (tests/cpu_baseline_run.py) so
    the OpenMP placement is set before the OpenMP runtime starts:
      B (value): one thread per physical core of one socket of this
        process's CPU set, OMP_PROC_BIND=close, capped by the CPU share the
        job is given (OMP_NUM_THREADS; the GPU pool sets 16 per GPU box) or
        --cpu-threads; steady-state mean over `seconds` of full passes;
      A (method_a): the reference's own methodology - 4 threads on 4 cores
        (run_spmv.sh:45 OMP_NUM_THREADS=4 taskset -c 0-3), ONE cold call per
        matrix (test_spmv.c:165-183)."""
    import subprocess
    runner = os.path.join(ROOT, "tests", "cpu_baseline_run.py")

    def run(*extra):
        r = subprocess.run([sys.executable, runner, "--workload", workload, *extra],
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"cpu baseline child failed: {r.stderr[-2000:]}")
        return json.loads(r.stdout.strip().splitlines()[-1])

    a = run("--method", "A")
    b = run("--method", "B", "--seconds", str(seconds), *(["--threads", str(threads)] if threads else []))
    pl = b["placement"]
    cap = ("--cpu-threads" if threads else
           f"OMP_NUM_THREADS={os.environ['OMP_NUM_THREADS']} (this job's CPU share)"
           if os.environ.get("OMP_NUM_THREADS") else "none")
    return {"value": round(b["gflops"], 3), "unit": "GFLOP/s", "cores": b["threads"],
            "kind": "port",
            "sample": f"method B: {b['passes']} full fp64 passes over the {workload} set ({b['seconds']:.1f} s), "
                      f"OpenMP row-parallel CSR, {b['threads']} threads pinned one per physical core "
                      f"(OMP_PROC_BIND=close) on socket {pl['socket']} of {pl['sockets_in_cpuset']} in a "
                      f"CPU set of {pl['cpuset_cpus']} logical CPUs ({pl['physical_cores_socket']} physical "
                      f"cores on that socket; thread cap: {cap}), x=dlarnv(1,{{0,0,0,1}})",
            "host": {"model": host_cpu_model(), "cpuset_cpus": pl["cpuset_cpus"],
                     "sockets_in_cpuset": pl["sockets_in_cpuset"],
                     "physical_cores_socket": pl["physical_cores_socket"], "threads": b["threads"],
                     "places": pl["places"]},
            "method_a": {"value": round(a["gflops"], 3), "unit": "GFLOP/s", "threads": a["threads"],
                         "places": a["placement"]["places"],
                         "note": "the reference's methodology: OMP_NUM_THREADS=4 on 4 physical cores, one cold "
                                 "call per matrix (run_spmv.sh:45, test_spmv.c:165-183), summed over the set"}}


def spmv_kernel_sha():
    """sha256 (16 hex) of the SpMV kernel sources — spmv.hip and the SpMV
    part of rsp_kernels.h (schedule records, tile geometry, batch records: up
    to the ILU level-schedule section) — the build a PMC summary must have been
    recorded for. (The ILU declarations further down the header do not change
    the SpMV kernel.)"""
    import hashlib
    hsh = hashlib.sha256()
    src = os.path.join(ROOT, "respasol_amd", "csrc")
    with open(os.path.join(src, "spmv.hip"), "rb") as fh:
        hsh.update(fh.read())
    with open(os.path.join(src, "rsp_kernels.h"), "rb") as fh:
        head = fh.read()
    cut = head.find(b"// Level schedule of one dependency DAG.")
    hsh.update(head if cut < 0 else head[:cut])
    return hsh.hexdigest()[:16]


def pmc_traffic(workload, batched, dtype="f64"):
    """HBM bytes per dominant-kernel launch (the batched launch, or one
    per-matrix launch with --no-batch) from a committed rocprofv3 --pmc
    summary (profiles/*pmc*.json written by scripts/pmc_summary.py) recorded
    for THIS kernel build (its kernel_sha equals spmv_kernel_sha()); a summary
    of another build is refused. Returns (bytes or None, source dict)."""
    sha = spmv_kernel_sha()
    best, src, seen = None, None, []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") != workload or d.get("dtype", "f64") != dtype:
            continue
        seen.append(os.path.relpath(p, ROOT))
        if d.get("kernel_sha") != sha:
            continue
        part = d.get("batch") if batched else d.get("per_matrix", d)
        if part and "hbm_bytes_per_launch" in part:
            best = part["hbm_bytes_per_launch"]
            src = {"file": os.path.relpath(p, ROOT), "kernel_sha": sha, "commit": d.get("commit"),
                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs), calibrated"}
    if src is None:
        src = {"file": None, "kernel_sha": sha,
               "note": "no PMC summary recorded for this kernel build (refused: "
                       + (", ".join(seen) if seen else "none found") + ")"}
    return best, src


class Workload:
    """One bench step over a set of matrices on this rank: the slices, the
    RCCL halo exchange (N > 1), the batched launches and the step itself."""

    def __init__(self, names, rank, world, handle, device, args, batch=True):
        self.world, self.device = world, device
        self.overlap = overlap = world > 1 and args.exchange == "halo" and not args.no_overlap
        meta = partition_meta(names, world, rank, device)
        self.slices = slices = [Slice(n, rank, world, handle, device, args.exchange, overlap, mt)
                                for n, mt in zip(names, meta)]
        self.exchanges64, self.exchanges32 = [], []
        if world > 1 and args.exchange == "halo":
            groups = [[i] for i in range(len(slices))] if args.no_bucket else [list(range(len(slices)))]
            for g in groups:
                direct = not args.halo_unpack
                ex64 = HaloExchange([slices[i].halo for i in g], rank, world, torch.float64, device, handle,
                                    direct=direct)
                ex32 = HaloExchange([slices[i].halo for i in g], rank, world, torch.float32, device, handle,
                                    direct=direct)
                for j, i in enumerate(g):
                    slices[i].bind_halo(j, ex64, ex32)
                ex64.exchange()
                ex32.exchange()
                self.exchanges64.append((g, ex64))
                self.exchanges32.append((g, ex32))
        torch.cuda.synchronize()
        self.stream = torch.cuda.current_stream()
        # part -> one batched launch over every matrix (rsp_spmv_batch): a
        # step's SpMVs cost one kernel ramp and drain instead of one per
        # matrix (--no-batch: one rsp_spmv per matrix)
        self.batches = {}
        if batch and not args.no_batch:
            for part in ((0, 1, 2) if overlap else (0,)):
                self.batches[part] = SpmvBatch(handle, [s.mat64 for s in slices], [s.x64() for s in slices],
                                               [s.y64 for s in slices], part)

    def spmv_all(self, part):
        for s in self.slices:
            if part:
                s.mat64.spmv_part(s.x64(), s.y64, part)
            else:
                s.mat64.spmv(s.x64(), s.y64[: s.m_local] if s.m_local else s.y64)

    def run(self, part):
        b = self.batches.get(part)
        if b is not None:
            b.run()
        else:
            self.spmv_all(part)

    def step(self, exchange=True, events=None):
        stream = self.stream
        if events is not None:  # instrumented pass: kernels only, one event pair per matrix
            # one whole step first keeps the stream busy while the host queues
            # the pairs, so the first pair does not time the host submission
            # gap after the previous synchronise
            self.run(0)
            for i, s in enumerate(self.slices):
                events[i][0].record(stream)
                s.mat64.spmv(s.x64(), s.y64[: s.m_local] if s.m_local else s.y64)
                events[i][1].record(stream)
            return
        if exchange and self.overlap:
            # halo overlap: start every exchange, interior tiles of every matrix
            # (own columns only), join the exchanges, then the boundary tiles
            for _, ex in self.exchanges64:
                ex.start()
            self.run(1)
            for _, ex in self.exchanges64:
                ex.finish()
            self.run(2)
            return
        if exchange and self.world > 1:  # every matrix's x is independent: exchange all, then compute
            for s in self.slices:
                if s.mode == "allgather":
                    s.part64.exchange()
            for _, ex in self.exchanges64:
                ex.exchange()
        self.run(0)

    def ramp(self, ramp_ms, device):
        """The GPU's clocks ramp up over the first tens of ms of load: 5
        warm-up steps (3 ms) leave 20 timed ones 5-8 % below steady state
        (measured 882-902 vs 933-957 GFLOP/s on one box). So setup runs the
        step until ramp_ms of GPU time have passed (untimed, reported in the
        JSON); returns the step count (equal on every rank)."""
        steps = 0
        if ramp_ms > 0:
            t_r = time.perf_counter()
            while True:
                for _ in range(5):
                    self.step()
                steps += 5
                torch.cuda.synchronize()
                more = torch.tensor([1.0 if (time.perf_counter() - t_r) * 1e3 < ramp_ms else 0.0],
                                    device=device)
                if self.world > 1:  # every rank runs the same number of steps (collectives inside)
                    dist.all_reduce(more, op=dist.ReduceOp.MAX)
                if more.item() == 0.0:
                    break
        return steps

    def timed(self, steps, warmup):
        """W warm-up steps, then exactly K steps between barrier + synchronize,
        one HIP event pair on the kernels' stream around the loop (an event
        pair per launch would insert ~10 us of marker gap between kernels).
        Returns (max-over-ranks wall seconds, start event, end event)."""
        for _ in range(warmup):
            self.step()
        torch.cuda.synchronize()
        e_start, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e_start.record(self.stream)
        for _ in range(steps):
            self.step()
        e_end.record(self.stream)
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if self.world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, e_start, e_end

    def totals(self):
        """(FLOPs, algorithmic fp64 bytes) of one step summed over ranks."""
        tot = torch.tensor([float(sum(2.0 * s.nnz_local for s in self.slices)),
                            float(sum(s.bytes_local(8) for s in self.slices))],
                           dtype=torch.float64, device=self.device)
        if self.world > 1:
            dist.all_reduce(tot)
        return float(tot[0]), float(tot[1])


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="big")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: physical cores of one socket, capped by "
                         "OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--ramp-ms", type=float, default=200.0,
                    help="untimed clock ramp before the warm-up steps (ms of repeated steps)")
    ap.add_argument("--fp32-reps", type=int, default=20)
    ap.add_argument("--exchange", default="halo", choices=["halo", "allgather"],
                    help="N>1 x exchange: halo-only all_to_all (default) or full all-gather")
    ap.add_argument("--no-bucket", action="store_true",
                    help="halo mode: one exchange per matrix instead of one per step")
    ap.add_argument("--halo-unpack", action="store_true",
                    help="halo mode: receive into a buffer and unpack it into each slice's x "
                         "(one more launch per step) instead of receiving in place")
    ap.add_argument("--no-overlap", action="store_true",
                    help="halo mode: finish the exchange before any SpMV instead of running the "
                         "interior tiles under it")
    ap.add_argument("--no-batch", action="store_true",
                    help="one rsp_spmv launch per matrix instead of one batched launch per step")
    ap.add_argument("--nccl-normal-priority", action="store_true",
                    help="RCCL on a normal-priority stream (default: high priority, so the "
                         "overlapped exchange is not queued behind the interior tiles)")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip the Serena-only step (BASELINE config 5) reported beside the big set")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the product path); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--launch-timeout", type=float, default=0.0,
                    help="launcher mode: stop every rank after this many seconds (0: no limit)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # plain `python bench.py --gpus N`: launch the N ranks here, before
        # anything in this process touches the GPU
        why = check_world(args, args.gpus, visible_gpus())
        if why:
            print(f"bench.py: {why}", file=sys.stderr, flush=True)
            sys.exit(2)
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                              timeout=args.launch_timeout or None))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    why = check_world(args, world, visible_gpus())
    if why:
        print(f"bench.py (rank {rank}): {why}", file=sys.stderr, flush=True)
        sys.exit(2)
    _import_product()
    dev = local % max(torch.cuda.device_count(), 1)  # == local on a full node
    torch.cuda.set_device(dev)
    device = torch.device("cuda", dev)
    if world > 1:
        if args.dist_backend == "nccl":
            # the halo all_to_all runs beside the interior SpMV tiles, which fill
            # every CU: a high-priority RCCL stream gets its kernel dispatched as
            # soon as slots free instead of behind the remaining tiles
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = not args.nccl_normal_priority
            dist.init_process_group("nccl", device_id=device, pg_options=opts)
        else:
            dist.init_process_group(args.dist_backend)
    handle = Handle()
    names = workload_names(args.workload)

    t_setup = time.perf_counter()
    W = Workload(names, rank, world, handle, device, args)
    slices, batches, overlap, exchanges64 = W.slices, W.batches, W.overlap, W.exchanges64
    step, spmv_all, stream = W.step, W.spmv_all, W.stream
    log(f"setup {time.perf_counter() - t_setup:.1f}s: {len(slices)} matrices, "
        f"{sum(s.nnz_global for s in slices) / 1e6:.1f} M stored nnz, world={world}")

    ramp_steps = W.ramp(args.ramp_ms, device)
    elapsed, e_start, e_end = W.timed(args.steps, args.warmup)
    big = max(slices, key=lambda s: s.nnz_global)
    y_step_t = big.y64.clone()  # checked against a whole SpMV below

    # dominant kernel, this rank: algorithmic bytes / average launch duration.
    # N = 1: the timed region is nothing but back-to-back launches of it; N > 1:
    # the same K steps again without the exchange (kernel-only), same stream.
    per_step = -(-len(slices) // 32) if batches else len(slices)  # 32 matrices per batch launch
    launches = args.steps * per_step
    if world == 1:
        kern_ms = e_start.elapsed_time(e_end)
    else:
        k0_, k1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k0_.record(stream)
        for _ in range(args.steps):
            step(exchange=False)
        k1_.record(stream)
        torch.cuda.synchronize()
        kern_ms = k0_.elapsed_time(k1_)
    bytes64 = sum(s.bytes_local(8) for s in slices)
    achieved = bytes64 * args.steps / (kern_ms * 1e-3) / 1e9
    # the schedule reads 16-bit column offsets for tiles spanning < 65536
    # columns: 2 B of the CSR's 4-B index per such entry are never moved (the
    # batch tiles the matrices itself: its own count)
    if batches:
        saved64 = 2 * sum(b.info()["entries_16bit"] for p, b in batches.items() if (p != 0) == overlap)
    else:
        saved64 = 2 * sum(s.mat64.plan_info()["entries_16bit"] for s in slices)
    moved_achieved = (bytes64 - saved64) * args.steps / (kern_ms * 1e-3) / 1e9
    # the same K steps as one rsp_spmv launch per matrix (kernel-only), for
    # comparison with the batched launch: what a caller doing one SpMV at a
    # time sees (calls bound once: the loop issues one rsp_spmv per matrix and
    # step, as a C caller would, without per-call Python argument conversion)
    calls = [s.mat64.bind(s.x64(), s.y64) for s in slices] if world == 1 else None
    for c in calls or []:
        c()
    p0_, p1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    p0_.record(stream)
    for _ in range(args.steps):
        if calls:
            for c in calls:
                c()
        else:
            spmv_all(0)
    p1_.record(stream)
    torch.cuda.synchronize()
    pm_ms = p0_.elapsed_time(p1_) / args.steps
    per_matrix_calls = {"ms_per_step_rank0": round(pm_ms, 4),
                        "gbps_rank0": round(bytes64 / (pm_ms * 1e6), 1),
                        "frac_rank0": round(bytes64 / (pm_ms * 1e6) / HBM_PEAK_GBS, 4)}
    # informative per-matrix split (one instrumented pass, outside the timing)
    ev = [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in slices]
    step(exchange=False, events=ev)
    torch.cuda.synchronize()
    per_matrix = {s.name: round(ev[i][0].elapsed_time(ev[i][1]) * 1e3, 2) for i, s in enumerate(slices)}

    # totals over ranks
    tot = torch.tensor([float(sum(2.0 * s.nnz_local for s in slices)), float(bytes64)],
                       dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(tot)
    flops_step, bytes_step = float(tot[0]), float(tot[1])
    value = flops_step * args.steps / elapsed / 1e9
    hbm_gbs = bytes_step * args.steps / elapsed / 1e9

    # fp32 companion measurement (outside the timed region), launched as the fp64 step
    b32 = (SpmvBatch(handle, [s.mat32 for s in slices], [s.x32() for s in slices],
                     [s.y32 for s in slices]) if batches else None)

    def pass32():
        if b32 is not None:
            b32.run()
            return
        for s in slices:
            s.mat32.spmv(s.x32(), s.y32[: s.m_local] if s.m_local else s.y32)

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pass32()
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(args.fp32_reps):
        pass32()
    e1.record(stream)
    torch.cuda.synchronize()
    ms32 = e0.elapsed_time(e1) / args.fp32_reps
    bytes32 = sum(s.bytes_local(4) for s in slices)
    fp32 = {"kernel_gflops_rank0": round(sum(2.0 * s.nnz_local for s in slices) / (ms32 * 1e6), 2),
            "kernel_gbps_rank0": round(bytes32 / (ms32 * 1e6), 1),
            "ms_per_pass_rank0": round(ms32, 4)}
    # fp32 roofline of its dominant kernel (the fp32 batched launch; one
    # launch per matrix with --no-batch), as the fp64 one below: algorithmic
    # bytes (8 B per stored entry + 4(m+1) + 4 n + 4 m) per launch
    # over the average launch duration from the event pair around the reps
    per32 = per_step
    avg32_ms = ms32 / per32
    b32_launch = bytes32 / per32
    if b32 is not None:
        saved32 = 2 * b32.info()["entries_16bit"]
    else:
        saved32 = 2 * sum(s.mat32.plan_info()["entries_16bit"] for s in slices)
    ach32 = b32_launch / (avg32_ms * 1e6)
    moved32 = (bytes32 - saved32) / per32 / (avg32_ms * 1e6)
    tr32, tr32_src = (pmc_traffic(args.workload, bool(batches), "f32") if world == 1
                      else (None, {"file": None, "note": "PMC summaries are recorded at N = 1"}))
    fp32["roofline"] = {
        "bound": "hbm",
        "kernel": ("rsp_k::spmv_tiles_batch<float,true,false,true>" if b32 is not None
                   else "rsp_k::spmv_tiles<float,true,false>"),
        "achieved": round(ach32, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(ach32 / HBM_PEAK_GBS, 4), "traffic": tr32, "traffic_source": tr32_src,
        "avg_launch_us": round(avg32_ms * 1e3, 3), "bytes_per_launch_avg": int(b32_launch),
        "index_bytes_saved_per_launch": int(saved32 / per32),
        "entries_16bit_share_rank0": round(saved32 / 2 / max(1, sum(s.nnz_local for s in slices)), 4),
        "moved_achieved": round(moved32, 1), "moved_frac": round(moved32 / HBM_PEAK_GBS, 4),
        "launches": args.fp32_reps * per32,
        "note": "fp32 companion of the fp64 roofline: same workload in fp32 (fp32 accumulation, "
                "the reference's CUDA_R_32F SpMV); event pair on the kernels' stream around the reps"}

    # parity spot check of this rank's slice of the largest matrix vs the oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob
    xf = big.x64().cpu().numpy()
    rp, ci_dev, va = big.host
    ref = ob.spmv(rp, ci_dev, va, xf, threads=True)
    y_step = y_step_t.cpu().numpy()[: big.m_local]  # as the last timed step left it
    got = big.mat64.spmv(big.x64()).cpu().numpy()[: big.m_local]
    bound = ob.spmv_bound(rp, ci_dev, va, xf, 2.0 ** -53)
    # the exchanged x must hold exactly the global x entries the slice references
    ok_x = True
    if big.mode == "halo":  # every entry the slice reads is the global x entry of its column
        xg = csr.dlarnv(1, [0, 0, 0, 1], big.n)[0]
        ok_x = np.array_equal(xf[ci_dev], xg[big.ci_global])
    # the step's y (overlapped split at N > 1) equals one whole SpMV bit for bit
    ok_step = np.array_equal(y_step, got) if big.m_local else True
    check_ok = bool(np.all(np.abs(got - ref) <= bound)) and ok_x and ok_step

    # config 5 (BASELINE.json): row-partitioned fp64 SpMV on the largest
    # matrix alone (Serena), measured like the headline step at the same N —
    # the hard case for scaling (about 11 us of compute per GPU at N = 8)
    config5 = None
    if args.workload == "big" and not args.no_config5:
        # one matrix: rsp_spmv / rsp_spmv_part launches (spmv_tiles), so the
        # batched kernel's rocprof average covers the headline step alone
        W5 = Workload(["Serena"], rank, world, handle, device, args, batch=False)
        W5.ramp(20.0, device)
        el5, _, _ = W5.timed(args.steps, args.warmup)
        f5, b5 = W5.totals()
        backend = "RCCL" if args.dist_backend == "nccl" else f"{args.dist_backend} (rehearsal)"
        config5 = {"workload": "Serena only, CSR SpMV fp64"
                               + (f", row-partitioned x{world} + {backend} {args.exchange} exchange of x"
                                  if world > 1 else ", 1 GPU"),
                   "value": round(f5 * args.steps / el5 / 1e9, 2), "unit": "GFLOP/s",
                   "ms_per_step": round(el5 / args.steps * 1e3, 4),
                   "hbm_gbps": round(b5 * args.steps / el5 / 1e9, 1),
                   "nnz_stored": int(W5.slices[0].nnz_global), "steps": args.steps}
        del W5

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.workload, args.cpu_seconds, args.cpu_threads)

    if rank == 0:
        traffic, traffic_src = (pmc_traffic(args.workload, bool(batches)) if world == 1  # PMC run was N = 1
                                else (None, {"file": None, "note": "PMC summaries are recorded at N = 1"}))
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: seeded surrogates of the SuiteSparse matrices (same m, stored nnz, "
                    "structure family; SURVEY App. A) - no .mtx data offline",
            "config": {
                "workload": f"{args.workload}-set CSR SpMV fp64, {len(slices)} matrices per step"
                            + (f", row-partitioned + RCCL {args.exchange} exchange of x" if world > 1 else ""),
                "matrices": len(slices),
                "nnz_stored_total": int(sum(s.nnz_global for s in slices)),
                "parallelism": f"row-partition x{world}" if world > 1 else "1 GPU",
                "launch": "one rsp_spmv per matrix" if args.no_batch else
                          (f"rsp_spmv_batch ({per_step} launch(es) of <= 32 matrices per step part): "
                           + ("interior, then boundary" if overlap else "whole step")),
                "collective": (("halo all_to_all_single" + ("" if args.halo_unpack else ", received in place")
                                 + ("" if args.no_bucket else
                                 " (one per step, bucketed over the matrices)")
                                 + (", interior tiles overlapped" if overlap else "")
                                 if args.exchange == "halo" else "all_gather_into_tensor")
                               + f" over {args.dist_backend}"
                               + (" (RCCL, xGMI)" if args.dist_backend == "nccl" else " (rehearsal)"))
                if world > 1 else None,
                "halo_bytes_per_step_rank0": (sum(ex.bytes_per_exchange for _, ex in exchanges64)
                                              if exchanges64 else None),
            },
            "setup_ramp": {"ms": args.ramp_ms, "steps": ramp_steps,
                           "note": "untimed steps before the warm-up so the GPU clocks reach steady "
                                   "state; the timed region is exactly `steps` full steps"},
            "hbm_gbps": round(hbm_gbs, 1),
            "roofline": {
                "bound": "hbm",
                "kernel": ("rsp_k::spmv_tiles_batch<double,true,false,true>" if batches
                           else "rsp_k::spmv_tiles<double,true,false>"),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_launch_us": round(kern_ms / launches * 1e3, 3),
                "bytes_per_launch_avg": int(bytes64 / per_step),
                "note": "achieved/frac count the CSR's algorithmic bytes (SURVEY 8d: 12 B per stored "
                        "entry fp64); the kernel reads 16-bit column offsets where a tile spans < 65536 "
                        "columns, so it moves index_bytes_saved fewer: moved_* below",
                "index_bytes_saved_per_launch": int(saved64 / per_step),
                # share of stored entries read as 16-bit offsets (rank 0; halo layouts at N > 1
                # lose it on boundary tiles whose columns span the receive region)
                "entries_16bit_share_rank0": round(saved64 / 2 / max(1, sum(s.nnz_local for s in slices)), 4),
                "moved_achieved": round(moved_achieved, 1),
                "moved_frac": round(moved_achieved / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": cpu,
            "config5_serena": config5,
            "fp32": fp32,
            "per_matrix_calls": per_matrix_calls,
            "per_matrix_us_rank0": per_matrix,
            "parity_check": "ok" if check_ok else "FAILED",
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not check_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
