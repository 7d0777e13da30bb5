"""IC(0)-preconditioned block CG.

Setup (IncompleteCholesky, work_2025/cg/incomplete_cholesky_decomp.hpp:84-201) runs on the host in
the reference and here.  That header includes <mkl.h>, absent from this image, so the reference
cannot be built: the factorization is checked bit for bit against the oracle's restatement
(oracle/mspmv_oracle.c orc_ic0_factor, same sequential operation order) -- **parity pinned to the
restatement only**.  The solve (PCGSolveMultiple, work_2025/main/incomplete_cholesky.hpp:33-199)
runs on the GPU with sync-free triangular solves; it is compared with the oracle's restatement
(orc_pcg_ic0_multi) under the CG tolerances of test_gpu_cg.py.
"""
import numpy as np
import pytest

import mspmv


def spd_small():
    return {
        "fem2d": lambda: mspmv.CsrMatrix.synth_stencil(0, 900, 30),
        "stencil27": lambda: mspmv.CsrMatrix.synth_stencil(1, 8 * 9 * 10, 8, 9, 10),
        "fem2d_partial_row": lambda: mspmv.CsrMatrix.synth_stencil(0, 1003, 41),
    }


@pytest.mark.parametrize("name", list(spd_small()))
def test_ic0_factor_bitexact_with_oracle(orc, name):
    a = spd_small()[name]()
    l, shift = mspmv.ic0_factor(a)
    lro, lci, lva, sh = orc.ic0_factor(a)
    assert shift == sh
    np.testing.assert_array_equal(l.row_offsets, lro)
    np.testing.assert_array_equal(l.column_indices, lci)
    np.testing.assert_array_equal(l.values, lva)


def test_ic0_factor_shift_retries(orc):
    """[[1, 2], [2, 1]] is indefinite: pivots fail until the diagonal shift (1e-3, 1e-2, 0.1,
    1, ... -- incomplete_cholesky_decomp.hpp:150-225) makes them positive; the product and the
    oracle agree on the shift and on every value."""
    a = mspmv.CsrMatrix.from_arrays(2, [0, 2, 4], [0, 1, 0, 1], [1.0, 2.0, 2.0, 1.0])
    l, shift = mspmv.ic0_factor(a)
    lro, lci, lva, sh = orc.ic0_factor(a)
    assert shift == sh and shift >= 0.1
    np.testing.assert_array_equal(l.values, lva)
    r = mspmv.CsrMatrix.from_arrays(3, [0, 1], [2], [1.0])
    with pytest.raises(mspmv.MspmvError):
        mspmv.ic0_factor(r)


def test_oracle_pcg_ic0_beats_cg(orc):
    a = spd_small()["fem2d"]()
    lro, lci, lva, _ = orc.ic0_factor(a)
    B = np.random.default_rng(3).uniform(0, 1, (a.num_rows, 2))
    _, itp, hp = orc.pcg_ic0_multi(a, lro, lci, lva, B, 1000, 1e-10, hist_cap=1000)
    _, itc, _ = orc.cg_multi(a, B, 1000, 1e-10, hist_cap=1000)
    assert hp[-1] < 1e-10 and itp < itc


def _iter_match(it_g, it_o, hist_o, tol):
    if it_g == it_o:
        return True
    if abs(it_g - it_o) == 1 and len(hist_o):
        k = min(it_g, it_o) - 1
        return abs(hist_o[k] - tol) <= 1e-9 * tol
    return False


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(spd_small()))
@pytest.mark.parametrize("L", [1, 4, 8, 32])
def test_gpu_pcg_ic0_vs_oracle(gpu_available, orc, name, L):
    a = spd_small()[name]()
    l, _ = mspmv.ic0_factor(a)
    B = np.random.default_rng(11 + L).uniform(0, 1, (a.num_rows, L))
    tol = 1e-9
    Xo, it_o, ho = orc.pcg_ic0_multi(a, l.row_offsets, l.column_indices, l.values, B, 2000, tol, hist_cap=2000)
    with mspmv.GpuCsr(a) as ga, mspmv.GpuIc0(l) as ic:
        X, it, h, st = mspmv.pcg_ic0(ga, ic, B, 2000, tol, hist_cap=2000)
        X2, it2, h2, _ = mspmv.pcg_ic0(ga, ic, B, 2000, tol, hist_cap=2000)
    assert st == 0 and _iter_match(it, it_o, ho, tol)
    k = min(len(h), len(ho))
    np.testing.assert_allclose(h[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(X - Xo) <= 1e-8 * np.linalg.norm(Xo)
    # the sync-free solves fold each row in a fixed order: a repeat is bitwise identical
    assert it2 == it
    np.testing.assert_array_equal(X2, X)
    np.testing.assert_array_equal(h2, h)


@pytest.mark.gpu
def test_gpu_ic0_facade_names(gpu_available, orc):
    a = spd_small()["stencil27"]()
    l = mspmv.IncompleteCholesky(a)
    L = 8
    B = np.random.default_rng(12).uniform(0, 1, a.num_rows * L)
    X = np.zeros_like(B)
    errs = []
    it = mspmv.PCGSolveMultiple(a, l, None, B, X, L, 1000, 1e-8, mspmv.MERGE, errs)
    _, it_o, _ = orc.pcg_ic0_multi(a, l.row_offsets, l.column_indices, l.values, B.reshape(-1, L), 1000, 1e-8)
    assert abs(it - it_o) <= 1 and len(errs) == it and errs[-1] < 1e-8
