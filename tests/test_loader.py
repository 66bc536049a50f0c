"""Loader parity: respasol_amd's Matrix-Market loader vs the REFERENCE loader
(ReadMatrixMarket/loadMatrixMarket.cpp:47-253), byte for byte.

* committed dumps of the reference loader (tests/golden/ref_csr, made by
  tests/golden/make_golden.py from oracle/_ref/ref_dump) — always run;
* a live differential run against oracle/_ref/ref_dump on randomly generated
  files — runs where the reference build exists (the build container).
"""
import json
import os
import random

import numpy as np
import pytest

import oracle_bind as ob
from respasol_amd import csr

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))


def _same(A, d):
    return ((A.is_symmetric, A.m, A.n, A.nnz) == (d["sym"], d["m"], d["n"], d["nnz"])
            and np.array_equal(A.rowptr, d["rowptr"]) and np.array_equal(A.colidx, d["colidx"])
            and np.array_equal(A.values.view(np.uint64), d["values"].view(np.uint64)))


@pytest.mark.parametrize("entry", MANIFEST, ids=lambda e: f"{e['file']}-b{e['base']}-t{e['transpose']}")
def test_loader_matches_reference_dump(entry):
    d = ob.read_ref_dump(os.path.join(GOLD, entry["dump"]))
    path = os.path.join(GOLD, "mtx", entry["file"])
    if not d["ok"]:
        with pytest.raises(csr.LoadError):
            csr.load_matrix_market(path, entry["base"], entry["transpose"])
        return
    A = csr.load_matrix_market(path, entry["base"], entry["transpose"])
    assert _same(A, d)


def test_symmetric_quirk_bcspwr01():
    """stored triangle only in the CSR, nnz = expanded count."""
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "bcspwr01.mtx"))
    assert (A.m, A.nnz, A.nnz_stored) == (39, 131, 85)
    rows = np.repeat(np.arange(A.m), np.diff(A.rowptr))
    assert np.all(A.colidx <= rows)  # no upper entries
    assert np.all(A.values == 1.0)   # pattern -> 1.0


def test_b1_ss_rows():
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "b1_ss.mtx"))
    kat = json.load(open(os.path.join(GOLD, "kat.json")))["b1_ss"]
    r0 = list(zip(A.colidx[A.rowptr[0]:A.rowptr[1]].tolist(), A.values[A.rowptr[0]:A.rowptr[1]].tolist()))
    r1 = list(zip(A.colidx[A.rowptr[1]:A.rowptr[2]].tolist(), A.values[A.rowptr[1]:A.rowptr[2]].tolist()))
    assert r0 == [tuple(p) for p in kat["row0"]]
    assert r1 == [tuple(p) for p in kat["row1"]]


def test_full_symmetric_extension():
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "bcspwr01.mtx"), full_symmetric=True)
    assert A.nnz_stored == A.nnz == 131
    dense = np.zeros((A.m, A.n))
    for i in range(A.m):
        dense[i, A.colidx[A.rowptr[i]:A.rowptr[i + 1]]] = A.values[A.rowptr[i]:A.rowptr[i + 1]]
    assert np.array_equal(dense, dense.T)


def test_loader_errors_and_buffer():
    with pytest.raises(csr.LoadError) as e:
        csr.load_matrix_market("/nonexistent/file.mtx")
    assert e.value.status == 1
    A = csr.load_matrix_market_text("%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 3\n2 2 4\n")
    assert A.rowptr.tolist() == [0, 1, 2] and A.values.tolist() == [3.0, 4.0]


def test_row_qsort_matches_reference_order():
    """Duplicate columns keep the order the reference's quicksort leaves
    (loadMatrixMarket.cpp:5-26) — pinned through the unsorted_dups dump."""
    d = ob.read_ref_dump(os.path.join(GOLD, "ref_csr", "unsorted_dups_b0_t0.bin"))
    A = csr.load_matrix_market(os.path.join(GOLD, "mtx", "unsorted_dups.mtx"))
    assert np.array_equal(A.values, d["values"])
    assert np.any(np.diff(A.colidx) == 0)  # the file really has duplicates


def _random_mtx(rnd: random.Random) -> str:
    m, n = rnd.randint(1, 40), rnd.randint(1, 40)
    field = rnd.choice(["real", "pattern", "integer", "complex"])
    sym = rnd.choice(["general", "symmetric"]) if field != "complex" else "general"
    if sym == "symmetric":
        n = m
    k = rnd.randint(m + 1, 4 * m + 8)
    lines = []
    for _ in range(k):
        i, j = rnd.randint(1, m), rnd.randint(1, n)
        if sym == "symmetric" and rnd.random() < 0.85 and j > i:
            i, j = j, i
        if field == "pattern":
            lines.append(f"{i} {j}")
        elif field == "integer":
            lines.append(f"{i} {j} {rnd.randint(-999, 999)}")
        elif field == "complex":
            lines.append(f"{i} {j} {rnd.uniform(-5, 5):.6e} {rnd.uniform(-1, 1)}")
        else:
            lines.append(f"{i} {j} {rnd.uniform(-1e3, 1e3):.17g}")
    return f"%%MatrixMarket matrix coordinate {field} {sym}\n% random\n{m} {n} {k}\n" + "\n".join(lines) + "\n"


@pytest.mark.skipif(not os.path.exists(ob.REF_DUMP), reason="reference loader build (oracle/_ref) not present")
def test_loader_differential_vs_reference_build(tmp_path):
    rnd = random.Random(20241218)
    for t in range(60):
        p = tmp_path / f"r{t}.mtx"
        p.write_text(_random_mtx(rnd))
        for base in (0, 1):
            tr = t % 2
            d = ob.ref_load(str(p), base, tr, str(tmp_path))
            assert d["ok"] == 1
            A = csr.load_matrix_market(str(p), base, tr)
            assert _same(A, d), (t, base)


def test_binary_cache_roundtrip(tmp_path):
    import ctypes as C
    from respasol_amd._lib import CSRStruct, host
    path = os.path.join(GOLD, "mtx", "bcspwr01.mtx")
    s = CSRStruct()
    assert host.rsp_mm_load(path.encode(), C.byref(s), 0, 0, 2) == 0
    out = str(tmp_path / "c.bin").encode()
    assert host.rsp_csr_save(out, C.byref(s)) == 0
    t = CSRStruct()
    assert host.rsp_csr_load(out, C.byref(t)) == 0
    assert (t.m, t.n, t.nnz, t.isSymmetric) == (s.m, s.n, s.nnz, s.isSymmetric)
    assert [t.rowptr[i] for i in range(t.m + 1)] == [s.rowptr[i] for i in range(s.m + 1)]
    host.rsp_csr_free(C.byref(s))
    host.rsp_csr_free(C.byref(t))


# --------------------------------------------------- parallel entry parse

def _big_text(n_rows=60000, per_row=30, sym=False, seed=7, pattern=False, split_lines=False):
    """A > 8 MB coordinate file (the parallel-parse threshold)."""
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(1, n_rows + 1), per_row)
    cols = rng.integers(1, n_rows + 1, rows.size)
    if sym:
        lo = np.minimum(rows, cols)
        hi = np.maximum(rows, cols)
        rows, cols = hi, lo
    vals = rng.standard_normal(rows.size) * 10.0 ** rng.integers(-30, 30, rows.size)
    field = "pattern" if pattern else "real"
    head = f"%%MatrixMarket matrix coordinate {field} {'symmetric' if sym else 'general'}\n% c\n"
    head += f"{n_rows} {n_rows} {rows.size}\n"
    sep = "\n" if split_lines else " "
    if pattern:
        body = "".join(f"{r} {c}\n" for r, c in zip(rows.tolist(), cols.tolist()))
    else:
        body = "".join(f"{r} {c}{sep}{v!r}\n" for r, c, v in zip(rows.tolist(), cols.tolist(), vals.tolist()))
    return head + body


def _same_csr(a, b):
    return (a.m == b.m and a.n == b.n and a.nnz == b.nnz and np.array_equal(a.rowptr, b.rowptr)
            and np.array_equal(a.colidx, b.colidx) and np.array_equal(a.values.view(np.uint64), b.values.view(np.uint64)))


@pytest.mark.parametrize("sym,pattern,split", [(False, False, False), (True, False, False),
                                               (False, True, False), (False, False, True)])
def test_parallel_parse_identical(sym, pattern, split):
    """Large files: the OpenMP entry parse gives the same CSR as the serial
    parse (incl. entries split over lines, where it falls back)."""
    text = _big_text(sym=sym, pattern=pattern, split_lines=split)
    assert len(text) > (8 << 20)
    a = csr.load_matrix_market_text(text)
    b = csr.load_matrix_market_text(text, serial=True)
    assert _same_csr(a, b)


@pytest.mark.parametrize("bad", ["garbage", "range", "extra"])
def test_parallel_parse_errors_identical(bad):
    """Malformed / out-of-range / surplus entries: same status as the serial parse."""
    text = _big_text()
    lines = text.split("\n")
    k = len(lines) // 2
    if bad == "garbage":
        lines[k] = "12 x7 1.0"
    elif bad == "range":
        lines[k] = "999999999 1 1.0"
    else:
        lines.insert(k, "1 1 1.0")
    text = "\n".join(lines)
    errs = []
    for serial in (False, True):
        try:
            csr.load_matrix_market_text(text, serial=serial)
            errs.append(None)
        except csr.LoadError as e:
            errs.append(e.status)
    assert errs[0] == errs[1] and errs[0] is not None
