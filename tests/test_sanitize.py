"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5:
the reference has no sanitizer runs). `make -C respasol_amd/csrc asan` builds
the CPU driver `test_spmv_cpu` from the host sources it links (Matrix-Market
loader, dlarnv, surrogates, the OpenMP CSR SpMV) with
-fsanitize=address,undefined into respasol_amd/build/asan/ (never shipped).
It then runs over every golden .mtx fixture, the malformed ones included, and
over a small surrogate. Pass = no sanitizer report, exit 0 (loaded) or 1
(rejected by the loader)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "respasol_amd", "csrc")
EXE = os.path.join(ROOT, "respasol_amd", "build", "asan", "test_spmv_cpu")
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def asan_exe():
    if shutil.which("gcc") is None or shutil.which("make") is None:
        pytest.skip("gcc/make not available")
    r = subprocess.run(["make", "-s", "-C", CSRC, "asan"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return EXE


def _run(exe, arg, out):
    env = dict(os.environ, OMP_NUM_THREADS="2",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return subprocess.run([exe, arg, str(out)], env=env, capture_output=True, text=True, timeout=120)


def _clean(p):
    err = p.stdout + p.stderr
    return "Sanitizer" not in err and "runtime error" not in err, err[-4000:]


def test_host_code_clean_on_golden_files(asan_exe, tmp_path):
    files = sorted(glob.glob(os.path.join(GOLDEN, "mtx", "*.mtx")))
    assert len(files) > 10
    codes = {}
    for path in files:
        p = _run(asan_exe, path, tmp_path / "out.csv")
        ok, err = _clean(p)
        assert ok, (path, err)
        assert p.returncode in (0, 1), (path, p.returncode, err)
        codes[os.path.basename(path)] = p.returncode
    assert codes["bcspwr01.mtx"] == 0 and codes["bad_banner.mtx"] == 1


def test_host_code_clean_on_surrogate(asan_exe, tmp_path):
    out = tmp_path / "out.csv"
    p = _run(asan_exe, "surrogate:dc1@0.01", out)
    ok, err = _clean(p)
    assert ok, err
    assert p.returncode == 0, err
    row = out.read_text().strip().split(",")
    assert row[0] == "2" and row[1] == "dc1"


AN_TSAN = os.path.join(ROOT, "respasol_amd", "build", "asan", "an_host_check_tsan")
AN_ASAN = os.path.join(ROOT, "respasol_amd", "build", "asan", "an_host_check_asan")


@pytest.fixture(scope="module")
def an_exes():
    """The ILU analysis' host half (worker pool, concurrent L / L^T / factor
    plans, the factor pieces' shared position table, the block cache) under
    ThreadSanitizer and under ASan + UBSan (respasol_amd/drivers/an_host_check.cpp)."""
    if shutil.which("g++") is None or shutil.which("make") is None:
        pytest.skip("g++/make not available")
    r = subprocess.run(["make", "-s", "-C", CSRC, "tsan", "asan-an"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return AN_TSAN, AN_ASAN


@pytest.mark.parametrize("name,scale", [("dc1", 0.3), ("ecology2", 0.05), ("ASIC_320ks", 0.1),
                                        ("FEM_3D_thermal2", 0.05)])
def test_analysis_host_clean_under_tsan_and_asan(an_exes, name, scale):
    """Plans built twice per run must agree (digest) and no sanitizer may
    report; small factor pieces (RSP_ILU_PIECE_ITEMS) so several pieces are
    planned concurrently, 4 worker threads."""
    env = dict(os.environ, OMP_NUM_THREADS="4", RSP_ILU_PIECE_ITEMS="4096",
               TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    digests = set()
    for exe in an_exes:
        p = subprocess.run([exe, name, str(scale)], env=env, capture_output=True, text=True, timeout=300)
        ok, err = _clean(p)
        assert ok and "ThreadSanitizer" not in err, err
        assert p.returncode == 0, err
        digests.add(p.stdout.split()[-1])
    assert len(digests) == 1  # the same plan from both builds
