"""The reference-CLI drivers on the GPU (respasol_amd/bin): output format of
GPU/spmv.cu:202-207,260 and GPU/ilu0.cu:221-226,312-317, results checked
against the oracle; plus the multi-partition SpMV on one GPU (the N>1
data path without the collective: every rank's slice computed by the HIP
kernel on the padded x must reassemble the single-GPU y bitwise)."""
import json
import os
import re
import subprocess

import numpy as np
import pytest
import torch

import oracle_bind as ob
from respasol_amd import csr
from respasol_amd.dist import padded_layout, remap_columns, unpad
from respasol_amd.sparse import Handle, SpMat, upload_csr

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "respasol_amd", "bin")
MTX = os.path.join(ROOT, "tests", "golden", "mtx")
FLOAT = r"[-+]?\d+\.\d+"


def run(*args):
    r = subprocess.run([os.path.join(BIN, args[0]), *args[1:]], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.parametrize("name", ["b1_ss", "bcspwr01", "one"])
def test_spmv_driver_reference_format(name):
    out = run("test_spmv", os.path.join(MTX, name + ".mtx"))
    lines = out.splitlines()
    assert re.fullmatch(rf"DOUBLE PRECISION SPMV solve time \(microseconds\) = {FLOAT}", lines[0])
    m = re.fullmatch(r"Error= (\S+)", lines[1])
    assert m and float(m.group(1)) == 0.0  # GPU y == host y on the fixtures
    assert len(lines) == 2


def test_spmv_driver_fp32_ftz_both_and_stats():
    out = run("spmv", "surrogate:Serena@0.05", "--prec=both", "--ftz", "--batched", "--stats",
              "--reps=20")
    assert "DOUBLE PRECISION SPMV solve time (microseconds) = " in out
    assert "SINGLE PRECISION SPMV solve time (microseconds) = " in out
    assert "batched time" in out and "STATS" in out
    for e in re.findall(r"Error= (\S+)", out):
        assert float(e) < 1e-5


def test_spmv_driver_ref_sequence_serena():
    """--ref-sequence (the default): GPU/spmv.cu:143-195 verbatim, no
    preprocess call before the 50 timed calls. Timed call 0 must cost no more
    than 2x the median, and the 50-rep mean must be no more than 5 % above
    the mean with an explicit preprocess (full-size Serena surrogate)."""
    def reps(*extra):
        out = run("test_spmv", "surrogate:Serena", "--rep-times", *extra)
        m = re.search(rf"REPS first_us=({FLOAT}) median_us=({FLOAT}) mean_us=({FLOAT})", out)
        assert m, out
        return [float(v) for v in m.groups()]
    first, med, mean = reps("--ref-sequence")
    assert first <= 2.0 * med, (first, med)
    _, _, mean_pre = reps("--preprocess")
    assert mean <= 1.05 * mean_pre, (mean, mean_pre)  # (one-sided: two processes, box noise either way)


def test_spmv_driver_ngpu_rccl():
    """--ngpu=N: the C driver's row-partitioned SpMV over an RCCL clique
    (ncclCommInitAll + grouped in-place ncclAllGather of the padded x, then
    the local SpMV). On a one-GPU box N = 1 is the run that exercises RCCL from
    C; Error= over the reassembled y (mean |host - GPU|, host in column order)
    must be at rounding level, and asking for more GPUs than visible is a
    clean error."""
    out = run("test_spmv", "surrogate:Serena@0.05", "--ngpu=1", "--prec=both", "--reps=10")
    assert re.search(rf"DOUBLE PRECISION SPMV solve time \(microseconds\) = {FLOAT}", out), out
    assert re.search(rf"NGPU=1 exchange=allgather chunk=\d+ allgather_us={FLOAT} spmv_us={FLOAT}", out), out
    errs = [float(e) for e in re.findall(r"Error= (\S+)", out)]
    assert len(errs) == 2 and errs[0] < 1e-10 and errs[1] < 1e-4, out
    n = torch.cuda.device_count()
    r = subprocess.run([os.path.join(BIN, "test_spmv"), "surrogate:Serena@0.01", f"--ngpu={n + 1}"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr


def _bench(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run(["python3", os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_bench_launches_n_ranks_itself():
    """`python bench.py --gpus 2` (no torchrun: the driver's scaling command)
    starts two ranks itself. On a one-GPU box the rehearsal backend (gloo)
    lets both ranks share cuda:0; the line must name 2 GPUs, the row-partitioned
    step's y must pass the oracle check, and with the product backend (nccl =
    RCCL) and too few GPUs bench.py must exit non-zero without a line."""
    r = _bench("--gpus", "2", "--dist-backend", "gloo", "--workload", "Serena", "--steps", "3",
               "--warmup", "1", "--ramp-ms", "20", "--no-cpu", "--fp32-reps", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["parity_check"] == "ok" and d["value"] > 0
    assert "row-partition x2" == d["config"]["parallelism"] and "gloo" in d["config"]["collective"]
    if torch.cuda.device_count() < 2:
        r = _bench("--gpus", "2", "--workload", "Serena", "--steps", "3", "--no-cpu", timeout=120)
        assert r.returncode != 0 and not r.stdout.strip() and "nccl" in r.stderr


def test_ilu0_driver_reference_format():
    out = run("test_ilu0", os.path.join(MTX, "bcspwr01.mtx"))
    pat = (rf"DOUBLE PRECISION SOLVE IN  MILLISECONDS\n Symbolic = {FLOAT}\n Numeric = {FLOAT} \n"
           rf" Symbolic\+ Numeric = {FLOAT}\n Solve = {FLOAT}\n")
    assert re.fullmatch(pat, out), out


def test_ilu0_driver_structural_zero_exit0():
    out = run("ilu0", os.path.join(MTX, "b1_ss.mtx"))
    assert out == "A(0,0) is missing\n"


def test_ilu0_driver_dump_matches_oracle(tmp_path):
    dump = tmp_path / "y.bin"
    out = run("test_ilu0", "surrogate:thermomech_TK@0.2", "--prec=fp32", "--ftz", f"--dump={dump}")
    assert out.startswith("SINGLE PRECISION SOLVE IN  MILLISECONDS\n")
    y = np.fromfile(dump, np.float32)
    A = csr.surrogate("thermomech_TK", 0.2)
    v, _, _ = ob.ilu0(A.rowptr, A.colidx, A.values.astype(np.float32), ftz=True)
    z = ob.trsv("lower_n", A.rowptr, A.colidx, v, np.ones(A.n, np.float32), ftz=True)
    ref = ob.trsv("lower_t", A.rowptr, A.colidx, v, z, ftz=True)
    assert np.array_equal(y, ref)


@pytest.mark.parametrize("P", [2, 3, 8])
def test_partitioned_spmv_single_gpu(P):
    """Each of P row slices (rank-local surrogate rows, padded column remap)
    through the HIP kernel; reassembled y == single-GPU y, bitwise."""
    name, scale = "Hook_1498", 0.05
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    h = Handle()
    rp, ci, va = upload_csr(A.rowptr, A.colidx, A.values)
    y_full = SpMat(h, rp, ci, va, A.n).spmv(torch.from_numpy(x).cuda()).cpu().numpy()
    bounds = csr.partition_rows(A.rowptr, P)
    chunk, pos = padded_layout(bounds)
    x_pad = np.zeros(P * chunk)
    x_pad[pos] = x
    xd = torch.from_numpy(x_pad).cuda()
    ys = []
    for p in range(P):
        r0, r1 = int(bounds[p]), int(bounds[p + 1])
        lrp, lci, lva = csr.surrogate_rows_csr(name, r0, r1, scale)
        lci_pad, _ = remap_columns(lci, bounds)
        d = upload_csr(lrp, lci_pad, lva)
        yp = SpMat(h, *d, P * chunk).spmv(xd)
        buf = torch.zeros(chunk, dtype=torch.float64, device="cuda")
        buf[: r1 - r0] = yp
        ys.append(buf)
    y = unpad(torch.cat(ys), bounds, chunk).cpu().numpy()
    assert np.array_equal(y, y_full)
    h.close()


@pytest.mark.parametrize("P", [2, 4, 8])
def test_halo_partitioned_spmv_single_gpu(P):
    """Halo layout (x_ext = [own rows | referenced remote columns], remapped
    column indices) through the HIP kernel for each of P slices: the
    concatenated y equals the single-GPU y bitwise; pack/unpack via
    rsp_gather / rsp_scatter reproduce the host-built x_ext."""
    from respasol_amd.dist import HaloSlice
    from respasol_amd.sparse import gather, scatter
    name, scale = "Serena", 0.05
    A = csr.surrogate(name, scale)
    x, _ = csr.dlarnv(1, [0, 0, 0, 1], A.n)
    h = Handle()
    y_full = SpMat(h, *upload_csr(A.rowptr, A.colidx, A.values), A.n).spmv(
        torch.from_numpy(x).cuda()).cpu().numpy()
    bounds = csr.partition_rows(A.rowptr, P)
    xd = torch.from_numpy(x).cuda()
    ys = []
    for p in range(P):
        r0, r1 = int(bounds[p]), int(bounds[p + 1])
        rp, ci, va = csr.surrogate_rows_csr(name, r0, r1, scale)
        hs = HaloSlice(ci, bounds, p)
        cols = np.concatenate([np.arange(r0, r1)] + hs.recv_cols).astype(np.int64)
        idx = torch.from_numpy(cols).cuda()
        x_ext = torch.empty(hs.n_ext, dtype=torch.float64, device="cuda")
        gather(h, idx, xd, x_ext)                      # pack: global x -> x_ext
        back = torch.zeros_like(xd)
        scatter(h, idx, x_ext, back)                   # unpack: x_ext -> global slots
        assert np.array_equal(back.cpu().numpy()[cols], x[cols])
        assert np.array_equal(x_ext.cpu().numpy(), x[cols])
        M = SpMat(h, *upload_csr(rp, hs.colidx_ext, va), hs.n_ext)
        ys.append(M.spmv(x_ext).cpu().numpy())
        # overlap split: interior tiles (own columns) with a poisoned halo, then
        # the boundary tiles after the halo is restored — same bits
        M.set_local_cols(hs.m_local)
        y2 = torch.full((max(r1 - r0, 1),), float("nan"), dtype=torch.float64, device="cuda")
        saved = x_ext[hs.m_local:].clone()
        x_ext[hs.m_local:] = float("nan")
        M.spmv_part(x_ext, y2, 1)
        x_ext[hs.m_local:] = saved
        M.spmv_part(x_ext, y2, 2)
        assert np.array_equal(y2.cpu().numpy()[: r1 - r0], ys[-1])
    assert np.array_equal(np.concatenate(ys), y_full)
    h.close()


class _AllRanks:
    """Stands in for torch.distributed in HaloExchange's setup: answers the two
    setup all-to-alls of rank r from every rank's HaloSlices (one process)."""

    def __init__(self, all_slices, r):
        self.all, self.r, self.calls = all_slices, r, 0

    def get_backend(self, group=None):
        return "nccl"

    def all_to_all_single(self, out, inp, out_splits, in_splits, group=None, async_op=False):
        P = len(self.all)
        if self.calls == 0:
            v = [self.all[p][i].recv_counts[self.r] for p in range(P) for i in range(len(self.all[p]))]
            out.copy_(torch.tensor(v, dtype=out.dtype))
        else:
            cols = [self.all[p][i].recv_cols[self.r] for p in range(P) for i in range(len(self.all[p]))]
            out.copy_(torch.from_numpy(np.concatenate(cols).astype(np.int64)))
        self.calls += 1


@pytest.mark.parametrize("P", [3, 8])
def test_halo_direct_layout_single_gpu(P):
    """Halo received in place (HaloExchange(direct=True): arena = own parts of
    every slice + one receive region, columns remapped) for several matrices
    bucketed into one exchange, every rank emulated on one GPU: the receive
    region is filled as the all-to-all would (source rank, slice, column), the
    interior tiles run with it poisoned, the boundary tiles after it is
    restored — one-matrix calls and the batched parts — and every rank's y
    equals the single-GPU y bit for bit."""
    from respasol_amd import dist as rdist
    from respasol_amd.sparse import SpmvBatch
    names, scale = ["Serena", "G2_circuit", "cage13"], 0.02
    h = Handle()
    mats = {n: csr.surrogate(n, scale) for n in names}
    xs = {n: csr.dlarnv(1, [0, 0, 0, 1], mats[n].n)[0] for n in names}
    y_full = {n: SpMat(h, *upload_csr(mats[n].rowptr, mats[n].colidx, mats[n].values), mats[n].n).spmv(
        torch.from_numpy(xs[n]).cuda()).cpu().numpy() for n in names}
    bounds = {n: csr.partition_rows(mats[n].rowptr, P) for n in names}
    hosts = {(n, p): csr.surrogate_rows_csr(n, int(bounds[n][p]), int(bounds[n][p + 1]), scale)
             for n in names for p in range(P)}
    all_slices = [[rdist.HaloSlice(hosts[(n, p)][1], bounds[n], p) for n in names] for p in range(P)]
    ys = {n: [] for n in names}
    for r in range(P):
        real = rdist.dist
        rdist.dist = _AllRanks(all_slices, r)
        try:
            ex = rdist.HaloExchange(all_slices[r], r, P, torch.float64, "cuda", h, direct=True)
        finally:
            rdist.dist = real
        recv = np.concatenate([xs[n][all_slices[r][i].recv_cols[p]] for p in range(P)
                               for i, n in enumerate(names)] + [np.zeros(0)])
        for i, n in enumerate(names):
            r0, r1 = int(bounds[n][r]), int(bounds[n][r + 1])
            ex.x_local(i).copy_(torch.from_numpy(xs[n][r0:r1]))
        region = ex.arena[ex.recv_off:ex.recv_off + ex.n_recv]
        Ms, outs = [], []
        for i, n in enumerate(names):
            rp, ci, va = hosts[(n, r)]
            M = SpMat(h, *upload_csr(rp, ex.colidx(i), va), ex.n_x(i))
            M.set_local_cols(all_slices[r][i].m_local)
            Ms.append(M)
            outs.append(torch.full((max(all_slices[r][i].m_local, 1),), float("nan"), dtype=torch.float64,
                                   device="cuda"))
        b1 = SpmvBatch(h, Ms, [ex.x_ext(i) for i in range(len(names))], outs, 1)
        b2 = SpmvBatch(h, Ms, [ex.x_ext(i) for i in range(len(names))], outs, 2)
        for batched in (False, True):
            for o in outs:
                o.fill_(float("nan"))
            region.fill_(float("nan"))  # the exchange has not landed yet
            if batched:
                b1.run()
            else:
                for i, M in enumerate(Ms):
                    M.spmv_part(ex.x_ext(i), outs[i], 1)
            region.copy_(torch.from_numpy(recv))
            if batched:
                b2.run()
            else:
                for i, M in enumerate(Ms):
                    M.spmv_part(ex.x_ext(i), outs[i], 2)
            for i, n in enumerate(names):
                m_loc = all_slices[r][i].m_local
                got = outs[i].cpu().numpy()[:m_loc]
                if batched:
                    assert np.array_equal(got, ys[n][-1]), (n, r)
                else:
                    ys[n].append(got)
    for n in names:
        assert np.array_equal(np.concatenate(ys[n]), y_full[n]), n
    h.close()


def test_ilu0_driver_flow_give_up_exits_nonzero():
    """test_ilu0 treats a failed factor / solve as an error (exit 1), also on
    the reference call sequence: a flow wait forced to give up
    (RSP_ILU_FLOW_TIMEOUT_US=0, every level fat) with recovery off
    (RSP_ILU_FLOW_RECOVER=0) is caught by the zero-pivot check after the
    factor; with recovery on (default) the zero-pivot check re-runs the call
    without flow launches and the driver succeeds; the normal bound runs clean."""
    # (RSP_ILU_FAC_ONE=0: G2_circuit's factor over L's levels, with flow runs)
    # (RSP_ILU_BLOCKS=0: the solves level-scheduled too, with flow launches)
    env = dict(os.environ, RSP_ILU_THIN_FACTOR="0", RSP_ILU_THIN_SOLVE="0", RSP_ILU_FAC_ONE="0",
               RSP_ILU_BLOCKS="0")
    exe = os.path.join(BIN, "test_ilu0")
    r = subprocess.run([exe, "surrogate:G2_circuit@0.1"], capture_output=True, text=True, timeout=300,
                       env=dict(env, RSP_ILU_FLOW_TIMEOUT_US="0", RSP_ILU_FLOW_RECOVER="0"))
    assert r.returncode == 1 and "RSP_STATUS_EXECUTION_FAILED" in r.stderr, (r.returncode, r.stderr)
    r = subprocess.run([exe, "surrogate:G2_circuit@0.1"], capture_output=True, text=True, timeout=300,
                       env=dict(env, RSP_ILU_FLOW_TIMEOUT_US="0"))
    assert r.returncode == 0 and "Solve = " in r.stdout, r.stderr
    r = subprocess.run([exe, "surrogate:G2_circuit@0.1"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "Solve = " in r.stdout, r.stderr
