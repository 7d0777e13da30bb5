"""GPU parity of the register-resident CGSolveSingle (csrc/mspmv_cg_resident.hip: the whole solve
as one launch of one workgroup per CU, matrix values in registers, columns in LDS, two in-launch hand-offs
per iteration) against the oracle's restatement of CGSolveSingle (single_strategy.hpp:102-170) and
against the pipelined two-kernel path (MSPMV_CG_RESIDENT=0) on the same inputs.

Tolerances as tests/test_gpu_cg.py (north_star "CG residual match within 1e-10 rel"): iteration
counts equal, every ||r_k||/||b|| within 1e-10, x within 1e-8 relative.
"""
import os

import numpy as np
import pytest

import mspmv
from test_gpu_cg import csr_matvec, iter_match

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


FORMS = ["classic", "single_reduction"]  # the resident kernel's iteration (MSPMV_CG_RESIDENT_FORM)


def solve(a, b, max_iters, tol, resident, hist_cap=None, form=None):
    old = {k: os.environ.get(k) for k in ("MSPMV_CG_RESIDENT", "MSPMV_CG_RESIDENT_FORM")}
    os.environ["MSPMV_CG_RESIDENT"] = "1" if resident else "0"
    if form:
        os.environ["MSPMV_CG_RESIDENT_FORM"] = form
    try:
        with mspmv.GpuCsr(a) as g:
            out = g.cg_single(b, max_iters, tol, hist_cap=hist_cap or max_iters)
            name = g.cg_kernel_name()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if resident and form and name.startswith("k_cg_resident"):
        assert f",{form}>" in name, name
    return out + (name,)


CASES = {
    "fem2d": lambda: mspmv.CsrMatrix.synth_stencil(0, 4000, 64),
    "fem2d_partial_row": lambda: mspmv.CsrMatrix.synth_stencil(0, 5003, 71),
    "stencil27": lambda: mspmv.CsrMatrix.synth_stencil(1, 14 * 15 * 16, 14, 15, 16),  # 27 > 16: pipelined
    # 3 rows per thread on some workgroups (m > 256 x 2048): the (3, 7) shape of configs[3]
    "fem2d_3rows": lambda: mspmv.CsrMatrix.synth_stencil(0, 540000, 600, diag_shift=5e-2),
}


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("name", list(CASES))
def test_resident_cg_vs_oracle(orc, name, form):
    a = CASES[name]()
    b = orc.glibc_rand(42, a.num_rows)
    tol = 1e-8
    xo, it_o, ho = orc.cg_single(a, b, 3000, tol, hist_cap=3000)
    xg, it_g, hg, st, kname = solve(a, b, 3000, tol, True, form=form)
    assert st == 0
    if name == "stencil27":
        assert not kname.startswith("k_cg_resident"), kname   # rows of 27 nonzeros: no resident shape
    else:
        assert kname.startswith("k_cg_resident"), kname
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho), it_g)
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)


@pytest.mark.parametrize("form", FORMS)
def test_resident_matches_pipelined_full_size(orc, form):
    """configs[3]'s parabolic_fem shape and RHS (m = 525,825: 3 rows per thread on some
    workgroups, 447 iterations).  The two GPU paths sum their dot products in different fixed
    orders, and at this size the reference does not reproduce itself to 1e-10 past iteration ~115
    (test_gpu_fullsize.py::test_cg_single_full_size holds the resident path to the reference's own
    thread-count envelope over the whole solve).  Here: the first 100 residuals within 1e-10 of each
    other, iterations within one, both true residuals below the stop threshold's order."""
    a = mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)
    b = orc.glibc_rand(42, a.num_rows)
    tol = orc.calculate_threshold(b, a.num_rows, 1e-5)   # cpu_singlecg.cpp:22-34 quirk
    xr, it_r, hr, st_r, kr = solve(a, b, 10000, tol, True, form=form)
    xp, it_p, hp, st_p, kp = solve(a, b, 10000, tol, False)
    assert kr.startswith("k_cg_resident<3,7,"), kr
    assert kp.startswith("pipelined"), kp
    assert st_r == 0 and st_p == 0
    assert abs(it_r - it_p) <= 1, (it_r, it_p)
    np.testing.assert_allclose(hr[:100], hp[:100], rtol=0, atol=1e-10)
    for x in (xr, xp):
        assert np.linalg.norm(b - orc.spmv_gold(a, x)) / np.linalg.norm(b) < 2 * tol


@pytest.mark.parametrize("form", FORMS)
def test_resident_max_iters_repeat_and_breakdown(orc, form):
    a = CASES["fem2d"]()
    n = a.num_rows
    b = orc.glibc_rand(42, n)
    # max_iters caps the count; the history holds every iteration; repeated solves are bitwise equal
    x1, it1, h1, st1, k1 = solve(a, b, 7, 1e-14, True, form=form)
    x2, it2, h2, st2, _ = solve(a, b, 7, 1e-14, True, form=form)
    assert k1.startswith("k_cg_resident") and st1 == 0 and it1 == 7 and len(h1) == 7
    np.testing.assert_array_equal(x1, x2)
    np.testing.assert_array_equal(h1, h2)
    xo, ito, ho = orc.cg_single(a, b, 7, 1e-14, hist_cap=7)
    np.testing.assert_allclose(h1, ho[:7], rtol=0, atol=1e-10)
    # max_iters = 0: x = 0, no iterations
    x0, it0, h0, st0, _ = solve(a, b, 0, 1e-8, True, form=form)
    assert st0 == 0 and it0 == 0 and not np.any(x0)
    # b = 0: p.Ap = 0 -> alpha = 0/0 at the first iteration -> breakdown (status 4), x stays 0
    xb, itb, hb, stb, kb = solve(a, np.zeros(n), 10, 1e-8, True, form=form)
    assert kb.startswith("k_cg_resident") and stb == 4 and itb == 1 and not np.any(xb)


def test_resident_follows_cu_limit(orc):
    """The resident layout is one workgroup per CU of the whole device: after set_cu_limit(64) the
    next single-RHS solve runs the pipelined CG (not a grid that cannot be co-resident), and after
    the limit is lifted the resident path is rebuilt and runs again -- same results every time."""
    a = CASES["fem2d"]()
    b = orc.glibc_rand(42, a.num_rows)
    with mspmv.GpuCsr(a) as g:
        x0, it0, h0, st0 = g.cg_single(b, 3000, 1e-8, hist_cap=3000)
        k0 = g.cg_kernel_name()
        g.set_cu_limit(64)
        x1, it1, h1, st1 = g.cg_single(b, 3000, 1e-8, hist_cap=3000)
        k1 = g.cg_kernel_name()
        g.set_cu_limit(0)
        x2, it2, h2, st2 = g.cg_single(b, 3000, 1e-8, hist_cap=3000)
        k2 = g.cg_kernel_name()
    assert k0.startswith("k_cg_resident") and k2.startswith("k_cg_resident"), (k0, k2)
    assert k1.startswith("pipelined"), k1
    assert st0 == st1 == st2 == 0
    np.testing.assert_array_equal(x0, x2)
    assert abs(it1 - it0) <= 1
    k = min(len(h0), len(h1))
    np.testing.assert_allclose(h1[:k], h0[:k], rtol=0, atol=1e-10)


@pytest.mark.parametrize("form", FORMS)
def test_resident_nan_rhs_reports_breakdown(orc, form):
    """b holding the all-ones NaN pattern (the hand-off slots' 'empty' marker) must end in a breakdown
    (or a NaN result) promptly, never in a stalled hand-off (MSPMV_ERR_STALL, status 8)."""
    a = CASES["fem2d"]()
    b = orc.glibc_rand(42, a.num_rows)
    b[17] = np.frombuffer(np.uint64(0xFFFFFFFFFFFFFFFF).tobytes(), np.float64)[0]
    x, it, h, st, kname = solve(a, b, 50, 1e-8, True, form=form)
    assert kname.startswith("k_cg_resident"), kname
    assert st in (0, 4), st


def test_resident_phase_stamps(orc):
    """mspmv_cg_resident_stamps: the same iterations and x as the plain solve, and stamps that are
    monotone within every workgroup's iteration (start <= Ap done <= p.Ap total <= r done <= r.r
    total) and across iterations."""
    a = CASES["fem2d"]()
    b = orc.glibc_rand(42, a.num_rows)
    with mspmv.GpuCsr(a) as g:
        db = mspmv.DeviceBuffer.from_array(b)
        dx = mspmv.DeviceBuffer(8 * a.num_rows)
        it, _, st = g.cg_dev(db, dx, 1, 3000, 1e-8)
        x_plain = dx.download(a.num_rows)
        its, stamps = g.cg_resident_stamps(db, dx, 3000, 1e-8, 64)
        x_st = dx.download(a.num_rows)
        db.free()
        dx.free()
    assert st == 0 and its == it
    np.testing.assert_array_equal(x_st, x_plain)
    k = min(its, 64)
    s = stamps[:k].astype(np.int64)
    assert s.shape[1] >= 8 and np.all(s > 0)
    assert np.all(np.diff(s, axis=2) >= 0)
    assert np.all(s[1:, :, 0] >= s[:-1, :, 4])


def test_resident_stall_falls_back_to_pipelined(orc, monkeypatch):
    """A resident solve whose hand-off stalls (its grid not co-resident: CUs held by other work) is run
    again on the pipelined kernels instead of failing (MSPMV_CG_RESIDENT_STALL=1 starts the launch with
    the abort word raised); the result is the pipelined solve's, held to the oracle as above."""
    a = CASES["fem2d"]()
    b = orc.glibc_rand(42, a.num_rows)
    tol = 1e-8
    xo, it_o, ho = orc.cg_single(a, b, 3000, tol, hist_cap=3000)
    monkeypatch.setenv("MSPMV_CG_RESIDENT_STALL", "1")
    xg, it_g, hg, st, kname = solve(a, b, 3000, tol, True)
    assert st == 0
    assert "after a resident-CG stall" in kname, kname
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)
    monkeypatch.delenv("MSPMV_CG_RESIDENT_STALL")
    _, _, _, st2, kname2 = solve(a, b, 3000, tol, True)   # the switch is read per solve
    assert st2 == 0 and kname2.startswith("k_cg_resident"), kname2
