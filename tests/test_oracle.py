"""The oracle pinned against the known answers recorded in SURVEY §0.7/§8c
(tests/golden/kat.json) and cross-checked against independent restatements,
plus the product's host-side dlarnv against the oracle's DLARUV-limb version."""
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
from respasol_amd import csr

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat.json")))


def fixture(name):
    return csr.load_matrix_market(os.path.join(GOLD, "mtx", name + ".mtx"))


def test_dlarnv_known_answers():
    x1, _ = ob.dlarnv(1, [0, 0, 0, 1], 3)
    x2, _ = ob.dlarnv(2, [0, 0, 0, 1], 3)
    assert x1.tolist() == KAT["dlarnv1_seed0001_first3"]
    assert x2.tolist() == KAT["dlarnv2_seed0001_first3"]
    p1, _ = csr.dlarnv(1, [0, 0, 0, 1], 3)
    assert p1.tolist() == KAT["dlarnv1_seed0001_first3"]


@pytest.mark.parametrize("idist", [1, 2])
def test_dlarnv_product_vs_oracle_long_stream(idist):
    # crosses DLARNV's 64-value DLARUV batches and several seeds
    for seed in ([0, 0, 0, 1], [1, 2, 3, 5], [4095, 4095, 4095, 4095]):
        a, sa = ob.dlarnv(idist, seed, 1000)
        b, sb = csr.dlarnv(idist, seed, 1000)
        assert np.array_equal(a, b) and sa == sb
        # the stream continues across calls exactly
        c1, s1 = csr.dlarnv(idist, seed, 300)
        c2, _ = csr.dlarnv(idist, s1, 700)
        assert np.array_equal(np.concatenate([c1, c2]), b)


def test_bcspwr01_ilu_solve_integer_exact():
    """ILU(0) + L + L^T solve with x = 1 on bcspwr01 is integer-exact."""
    A = fixture("bcspwr01")
    k = KAT["bcspwr01"]
    for dt in (np.float64, np.float32):
        v, sz, zp = ob.ilu0(A.rowptr, A.colidx, A.values.astype(dt))
        assert sz == -1 and zp == -1
        x = np.ones(A.n, dt)
        z = ob.trsv("lower_n", A.rowptr, A.colidx, v, x)
        y = ob.trsv("lower_t", A.rowptr, A.colidx, v, z)
        assert y[:4].tolist() == k["ilu_LLt_solve_x1_first4"]
        assert np.abs(y).max() == k["ilu_LLt_solve_x1_maxabs"]
        assert np.array_equal(y, np.round(y))


def test_b1_ss_structural_zero():
    A = fixture("b1_ss")
    _, sz, _ = ob.ilu0(A.rowptr, A.colidx, A.values)
    assert sz == KAT["b1_ss"]["structural_zero"]


def test_identity():
    A = fixture("one")
    x = np.arange(1, 8, dtype=np.float64) / 3
    assert np.array_equal(ob.spmv(A.rowptr, A.colidx, A.values, x), x)
    v, sz, zp = ob.ilu0(A.rowptr, A.colidx, A.values)
    z = ob.trsv("lower_n", A.rowptr, A.colidx, v, np.ones(7))
    y = ob.trsv("lower_t", A.rowptr, A.colidx, v, z)
    assert np.all(y == KAT["one"]["ilu_solve_x1"])


def _dense(A, vals=None):
    D = np.zeros((A.m, A.n))
    v = A.values if vals is None else vals
    for i in range(A.m):
        s, e = A.rowptr[i], A.rowptr[i + 1]
        np.add.at(D[i], A.colidx[s:e], v[s:e])
    return D


def test_spmv_oracle_vs_sequential_python():
    A = csr.surrogate("dc1", 0.01)
    x, _ = csr.dlarnv(2, [0, 0, 0, 1], A.n)
    y = ob.spmv(A.rowptr, A.colidx, A.values, x)
    ref = np.empty(A.m)
    for i in range(A.m):
        s = 0.0
        for k in range(A.rowptr[i], A.rowptr[i + 1]):
            s += A.values[k] * x[A.colidx[k]]
        ref[i] = s
    assert np.array_equal(y, ref)
    assert np.array_equal(ob.spmv(A.rowptr, A.colidx, A.values, x, threads=True), y)
    # fp32 storage + accumulation
    y32 = ob.spmv(A.rowptr, A.colidx, A.values.astype(np.float32), x.astype(np.float32))
    bound = ob.spmv_bound(A.rowptr, A.colidx, A.values, x, 2.0 ** -23)
    assert np.all(np.abs(y32 - y) <= bound + 1e-30)


def test_ilu0_oracle_reproduces_LU():
    """ILU(0) on a pattern that is closed under the elimination is exact LU:
    L*U reproduces A on a tridiagonal (no fill) matrix."""
    n = 50
    rows, cols, vals = [], [], []
    rng = np.random.default_rng(0)
    for i in range(n):
        for j in (i - 1, i, i + 1):
            if 0 <= j < n:
                rows.append(i)
                cols.append(j)
                vals.append(4.0 if i == j else rng.uniform(-1, 1))
    rp = np.searchsorted(rows, np.arange(n + 1)).astype(np.int32)
    ci = np.array(cols, np.int32)
    va = np.array(vals)
    v, sz, zp = ob.ilu0(rp, ci, va)
    assert sz == -1 and zp == -1
    L = np.eye(n)
    U = np.zeros((n, n))
    for i in range(n):
        for k in range(rp[i], rp[i + 1]):
            if ci[k] < i:
                L[i, ci[k]] = v[k]
            else:
                U[i, ci[k]] = v[k]
    A = np.zeros((n, n))
    A[np.array(rows), ci] = va
    assert np.allclose(L @ U, A, rtol=1e-13, atol=1e-13)
    x = rng.uniform(-1, 1, n)
    z = ob.trsv("lower_n", rp, ci, v, x)
    assert np.allclose(L @ z, x)
    y = ob.trsv("lower_t", rp, ci, v, x)
    assert np.allclose(L.T @ y, x)
    u = ob.trsv("upper", rp, ci, v, x)
    assert np.allclose(U @ u, x)


def test_ilu0_numerical_zero_pivot():
    # [[1, 1], [1, 1]] -> u_11 = 1 - 1*1 = 0
    rp = np.array([0, 2, 4], np.int32)
    ci = np.array([0, 1, 0, 1], np.int32)
    v, sz, zp = ob.ilu0(rp, ci, np.ones(4))
    assert sz == -1 and zp == 1


def test_fp32_solve_fuses_with_one_rounding():
    """The oracle's fp32 solve fuses with fmaf (one rounding); the HIP kernels
    mirror it (tests/test_gpu_ilu0.py::test_fp32_fma_single_rounding). For
    a*b + c = 1 + 2^-23 + 2^-24 - 2^-60, just below a float midpoint, one
    rounding gives 1 + 2^-23; a double fma rounded to float gives 1 + 2^-22."""
    a = np.float32(2.0 ** -12 * (1 + 2.0 ** -18))
    b = np.float32(2.0 ** -12 * (1 - 2.0 ** -18))
    c = np.float32(1 + 2.0 ** -23)
    rp = np.array([0, 1, 3], np.int32)
    ci = np.array([0, 0, 1], np.int32)
    v = np.array([1.0, -a, 1.0], np.float32)  # L = [[1, 0], [-a, 1]]
    z = ob.trsv("lower_n_ref", rp, ci, v, np.array([b, c], np.float32))
    assert z[0] == b
    assert z[1] == np.float32(1 + 2.0 ** -23)
    assert np.float32(np.float64(c) + np.float64(a) * np.float64(b)) == np.float32(1 + 2.0 ** -22)


def test_ftz_oracle_flushes_subnormals():
    rp = np.array([0, 2], np.int32)
    ci = np.array([0, 1], np.int32)
    vals = np.array([1e-39, 2e-39], np.float32)  # fp32 subnormals
    x = np.array([1.0, 1.0], np.float32)
    assert ob.spmv(rp, ci, vals, x)[0] != 0.0
    assert ob.spmv(rp, ci, vals, x, ftz=True)[0] == 0.0


@pytest.mark.parametrize("name,scale", [("dc1", 0.1), ("G2_circuit", 0.1), ("xenon2", 0.03), ("ecology2", 0.02)])
def test_split_order_solves_within_tolerance(name, scale):
    """The split solve order (RSP_ILU_SPLIT=1: a row's terms from the level
    just below it last) against the reference's own order
    (L column ascending, L^T column sweep): same terms, different summation
    order only — normwise within SURVEY 8c's 1e-12 (fp64) and 1e-4 (fp32),
    most entries bitwise."""
    A = csr.surrogate(name, scale)
    v, _, _ = ob.ilu0(A.rowptr, A.colidx, A.values)
    x = csr.dlarnv(2, [0, 0, 0, 1], A.n)[0]
    for dt, tol in ((np.float64, 1e-12), (np.float32, 1e-4)):
        vv, xx = v.astype(dt), x.astype(dt)
        for k in ("lower_n", "lower_t"):
            a = ob.trsv(k + "_split", A.rowptr, A.colidx, vv, xx).astype(np.float64)
            b = ob.trsv(k + "_ref", A.rowptr, A.colidx, vv, xx).astype(np.float64)
            assert np.linalg.norm(a - b) <= tol * np.linalg.norm(b)
            assert np.mean(a == b) > 0.5


@pytest.mark.parametrize("name,scale", [("dc1", 0.2), ("G2_circuit", 0.2), ("matrix-new_3", 0.2), ("xenon2", 0.03),
                                        ("ASIC_320ks", 0.05), ("ecology2", 0.02)])
def test_block_order_solves_within_tolerance(name, scale):
    """The block-inverse order of the deep-DAG solves (round 6,
    oracle_trsv_blocks_*: each block's unknowns as combinations of its
    right-hand sides and of earlier blocks' unknowns) against the reference's
    own order: same unknowns, rounding only — normwise within SURVEY 8c's
    1e-12 (fp64) and 1e-4 (fp32), for L and L^T, alpha = 1 and a scaled
    alpha."""
    A = csr.surrogate(name, scale)
    v, _, _ = ob.ilu0(A.rowptr, A.colidx, A.values)
    x = csr.dlarnv(2, [0, 0, 0, 1], A.n)[0]
    for dt, tol in ((np.float64, 1e-12), (np.float32, 1e-4)):
        vv, xx = v.astype(dt), x.astype(dt)
        for k in ("lower_n", "lower_t"):
            for alpha in (1.0, -2.5):
                a = ob.trsv(k + "_blocks", A.rowptr, A.colidx, vv, xx, alpha=alpha).astype(np.float64)
                b = ob.trsv(k + "_ref", A.rowptr, A.colidx, vv, xx, alpha=alpha).astype(np.float64)
                assert np.isfinite(a).all()
                assert np.linalg.norm(a - b) <= tol * np.linalg.norm(b)


def test_block_order_kat_bcspwr01():
    """The bcspwr01 L L^T solve with x = 1 is integer-exact (SURVEY 8c KAT):
    the block order reproduces it exactly (every coefficient and partial sum
    is a small integer)."""
    import json
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    kat = json.load(open(os.path.join(gold, "kat.json")))["bcspwr01"]
    A = csr.load_matrix_market(os.path.join(gold, "mtx", "bcspwr01.mtx"))
    v, _, _ = ob.ilu0(A.rowptr, A.colidx, A.values)
    z = ob.trsv("lower_n_blocks", A.rowptr, A.colidx, v, np.ones(A.n))
    y = ob.trsv("lower_t_blocks", A.rowptr, A.colidx, v, z)
    assert y[:4].tolist() == kat["ilu_LLt_solve_x1_first4"]
    assert np.abs(y).max() == kat["ilu_LLt_solve_x1_maxabs"]


def test_block_rule_matches_the_product():
    """oracle_bind.blocks_wanted restates the product's rule
    (rsp_an::blocks_wanted): deep DAGs (<= 32 rows per level) only."""
    deep = csr.surrogate("dc1", 0.2)
    wide = csr.surrogate("xenon2", 0.03)
    assert ob.blocks_wanted(0, deep.rowptr, deep.colidx) and ob.blocks_wanted(1, deep.rowptr, deep.colidx)
    assert not ob.blocks_wanted(0, wide.rowptr, wide.colidx)
