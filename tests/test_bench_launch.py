"""bench.py's own N-rank launcher (`python bench.py --gpus N` without
torchrun): environment plumbing, rank-0 relay, failure propagation and the
world/GPU-count guards. CPU only: the ranks here are tiny Python children."""
import io
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (stdlib-only at import: the product loads in the ranks)


def test_bench_import_loads_no_product():
    assert bench.torch is None and bench.csr is None


def test_rank_envs():
    envs = bench.rank_envs(4, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29511)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["PATH"] == "/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # the dmabuf IPC setting is kept (set when absent)
    assert bench.rank_envs(1, {}, 1)[0]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


CHILD = ("import json, os, sys, time\n"
         "r = int(os.environ['RANK'])\n"
         "mode = sys.argv[1]\n"
         "if mode == 'fail' and r == 1: sys.exit(5)\n"
         "if mode == 'fail': time.sleep(60)\n"
         "print(json.dumps({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR',"
         " 'MASTER_PORT')}), flush=True)\n")


def test_launch_relays_rank0_only():
    out = io.StringIO()
    rc = bench.launch_ranks(3, [sys.executable, "-c", CHILD, "ok"], out=out)
    assert rc == 0
    lines = [json.loads(s) for s in out.getvalue().splitlines() if s.strip()]
    assert len(lines) == 1 and lines[0]["RANK"] == "0" and lines[0]["WORLD_SIZE"] == "3"
    assert lines[0]["MASTER_ADDR"] == "127.0.0.1" and int(lines[0]["MASTER_PORT"]) > 0


def test_launch_failure_stops_the_others():
    t0 = time.time()
    rc = bench.launch_ranks(3, [sys.executable, "-c", CHILD, "fail"], out=io.StringIO())
    assert rc == 5
    assert time.time() - t0 < 30  # ranks 0 and 2 (sleeping 60 s) were stopped


def test_launch_timeout():
    rc = bench.launch_ranks(2, [sys.executable, "-c", "import time; time.sleep(60)"], out=io.StringIO(),
                            timeout=1.0)
    assert rc == 124


class _A:
    def __init__(self, gpus, backend="nccl"):
        self.gpus, self.dist_backend = gpus, backend


def test_check_world():
    assert bench.check_world(_A(1), 1, 0) is None
    assert bench.check_world(_A(8), 8, 8) is None
    assert "WORLD_SIZE" in bench.check_world(_A(8), 1, 8)  # torchrun world != --gpus
    assert "nccl" in bench.check_world(_A(2), 2, 1)  # one GPU for two RCCL ranks
    assert bench.check_world(_A(2, "gloo"), 2, 1) is None  # rehearsal: ranks share a GPU


def test_bench_refuses_nccl_without_gpus():
    """`python bench.py --gpus 2` where fewer than 2 GPUs are visible exits
    non-zero before starting any rank (here: none visible)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    if r.returncode == 0:
        pytest.fail("bench.py --gpus 2 ran without 2 GPUs")
    assert r.returncode == 2 and "nccl" in r.stderr and r.stdout.strip() == ""


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE is 1" in r.stderr


def _meta_worker(rank, world, port, names, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bench._import_product()
        q.put((rank, bench.partition_meta(names, world, rank)))
    finally:
        dist.destroy_process_group()


def test_partition_meta_is_rank0s_broadcast():
    """the whole-matrix row-length pass runs on rank 0 only;
    every rank receives the same (m, nnz, bounds) as a single process computes
    (gloo, world 2, small surrogate matrices)."""
    import socket
    import numpy as np
    import torch.multiprocessing as mp
    from respasol_amd import csr
    names = ["ASIC_320ks", "ecology2"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_meta_worker, args=(r, 2, port, names, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for name, *per_rank in zip(names, got[0], got[1]):
        m = csr.surrogate_rows(name)
        rowptr = np.zeros(m + 1, np.int64)
        np.cumsum(csr.surrogate_rowlens(name), out=rowptr[1:])
        want = csr.partition_rows(rowptr.astype(np.int32), 2)
        for mm, nnz, b in per_rank:
            assert mm == m and nnz == int(rowptr[-1]) and np.array_equal(b, want)
