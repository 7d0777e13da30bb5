"""GPU parity: fused CG (single and multi-RHS) vs the oracle's restatement of CGSolveSingle
(single_strategy.hpp:102-170) and CGSolveMultiple (no_pretreatment.hpp:32-197).

Tolerances (north_star "CG residual match within 1e-10 rel", read relative to ||b||):
  * iteration counts equal (the stop test compares a value ~tol against tol; a +-1 slack is
    allowed only when the oracle's deciding residual lies within 1e-9 relative of tol);
  * every recorded residual ||r_k||/||b|| within 1e-10 of the oracle's;
  * final x within 1e-8 relative, and the true residual ||b - A x||/||b|| of the same order
    as the oracle's.
"""
import os

import numpy as np
import pytest

import mspmv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


def spd_cases():
    return {
        "fem2d": lambda: mspmv.CsrMatrix.synth_stencil(0, 4000, 64),
        "fem2d_partial_row": lambda: mspmv.CsrMatrix.synth_stencil(0, 5003, 71),
        "stencil27": lambda: mspmv.CsrMatrix.synth_stencil(1, 14 * 15 * 16, 14, 15, 16),
    }


def csr_matvec(a, x):
    lens = np.diff(a.row_offsets)
    rows = np.repeat(np.arange(a.num_rows), lens)
    y = np.zeros((a.num_rows,) + x.shape[1:])
    np.add.at(y, rows, a.values.reshape((-1,) + (1,) * (x.ndim - 1)) * x[a.column_indices])
    return y


def iter_match(it_g, it_o, hist_o, tol):
    if it_g == it_o:
        return True
    if abs(it_g - it_o) == 1 and len(hist_o):
        k = min(it_g, it_o) - 1
        return abs(hist_o[k] - tol) <= 1e-9 * tol
    return False


@pytest.mark.parametrize("name", list(spd_cases()))
@pytest.mark.parametrize("tol", [1e-6, 1e-10])
def test_cg_single_vs_oracle(orc, name, tol):
    a = spd_cases()[name]()
    b = orc.glibc_rand(42, a.num_rows)   # cpu_singlecg.cpp:87-90
    xo, it_o, ho = orc.cg_single(a, b, 5000, tol, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        xg, it_g, hg, st = g.cg_single(b, 5000, tol, hist_cap=5000)
    assert st == 0
    assert it_o < 5000
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)
    res_g = np.linalg.norm(b - csr_matvec(a, xg)) / np.linalg.norm(b)
    res_o = np.linalg.norm(b - csr_matvec(a, xo)) / np.linalg.norm(b)
    assert res_g <= max(10 * res_o, 1e-13)


@pytest.mark.parametrize("L", [1, 2, 4, 8, 16])
def test_cg_multi_vs_oracle(orc, L):
    a = spd_cases()["fem2d"]()
    n = a.num_rows
    flat = orc.glibc_rand(42, n * L)
    B = flat.reshape(n, L)                               # interleaved n x L (utils_multiple.hpp:17)
    tol = orc.calculate_threshold(flat, n, 1e-5)         # the cpu_multicg.cpp:168 quirk
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, tol, kernel=1, P=8, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 5000, tol, hist_cap=5000)
    assert st == 0
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(Xg - Xo) <= 1e-8 * np.linalg.norm(Xo)


@pytest.mark.parametrize("L", [3, 32])
def test_cg_multi_any_width_vs_oracle(orc, L):
    """num_vectors outside {1, 2, 4, 8, 16} (preconditioner_benchmark.cpp:401 runs 32): column
    groups of native widths; iteration count, max-over-all-columns history and X as the oracle's
    single L-wide solve."""
    a = spd_cases()["fem2d"]()
    n = a.num_rows
    flat = orc.glibc_rand(42, n * L)
    B = flat.reshape(n, L)
    tol = orc.calculate_threshold(flat, n, 1e-5)
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, tol, kernel=1, P=8, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 5000, tol, hist_cap=5000)
    assert st == 0
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    for j in range(L):
        assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j])


def test_cg_multi_masks_columns_converge_at_different_iterations(orc):
    """Columns of very different difficulty: converged columns freeze (alpha = beta = 0)
    while the rest continue (no_pretreatment.hpp:109-120, 163-176)."""
    a = spd_cases()["fem2d"]()
    n, L = a.num_rows, 4
    rng = np.random.default_rng(0)
    B = np.empty((n, L))
    B[:, 0] = csr_matvec(a, np.ones(n))          # smooth: converges fast
    B[:, 1] = rng.uniform(0, 1, n)
    B[:, 2] = rng.standard_normal(n)
    B[:, 3] = np.sin(np.arange(n) * 0.37)
    tol = 1e-9
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, tol, kernel=1, P=8, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 5000, tol, hist_cap=5000)
    assert st == 0 and iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    np.testing.assert_allclose(hg[: min(len(hg), len(ho))], ho[: min(len(hg), len(ho))], rtol=0, atol=1e-10)
    for j in range(L):
        assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j])


def test_cg_multi_L1_equals_single():
    a = spd_cases()["stencil27"]()
    b = np.random.default_rng(3).uniform(0, 1, a.num_rows)
    with mspmv.GpuCsr(a) as g:
        x1, it1, h1, _ = g.cg_single(b, 3000, 1e-9, hist_cap=3000)
        xm, itm, hm, _ = g.cg_multi(b[:, None], 3000, 1e-9, hist_cap=3000)
    assert it1 == itm
    assert x1.tobytes() == xm[:, 0].tobytes()
    assert h1.tobytes() == hm.tobytes()


def test_cg_max_iters_and_repeatability(orc):
    a = spd_cases()["fem2d"]()
    b = orc.glibc_rand(7, a.num_rows)
    xo, it_o, _ = orc.cg_single(a, b, 37, 1e-30)
    with mspmv.GpuCsr(a) as g:
        xg, it_g, _, st = g.cg_single(b, 37, 1e-30)
        xg2, _, _, _ = g.cg_single(b, 37, 1e-30)
        x0, it0, _, _ = g.cg_single(b, 0, 1e-30)
    assert it_g == it_o == 37 and st == 0
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)
    assert xg.tobytes() == xg2.tobytes()       # deterministic run to run
    assert it0 == 0


def test_cg_breakdown_reported():
    a = spd_cases()["fem2d"]()
    with mspmv.GpuCsr(a) as g:
        x, it, _, st = g.cg_single(np.zeros(a.num_rows), 100, 1e-8)
    assert st == 4  # MSPMV_ERR_BREAKDOWN: p.Ap = 0 -> non-finite alpha; the reference has no guard


def test_cg_facade_names(orc):
    a = spd_cases()["fem2d"]()
    b = orc.glibc_rand(42, a.num_rows)
    x = np.empty(a.num_rows)
    it = mspmv.CGSolveSingle(a, b, x, 5000, 1e-8)
    _, it_o, _ = orc.cg_single(a, b, 5000, 1e-8)
    assert it == it_o
    L = 2
    B = orc.glibc_rand(42, a.num_rows * L)
    X = np.empty_like(B)
    errs = []
    it = mspmv.CGSolveMultiple(a, B, X, L, 5000, 1e-8, mspmv.NONZERO_SPLIT, errs)
    assert len(errs) == it and errs[-1] < 1e-8


def test_cg_multi_breakdown_reported_split_path():
    """L >= 2 runs the split iteration (p update pass, SpMM MODE 2, update): a zero RHS gives
    p.Ap = 0 -> non-finite alpha, caught by the SpMM's last block before x and r change."""
    a = spd_cases()["fem2d"]()
    with mspmv.GpuCsr(a) as g:
        X, it, _, st = g.cg_multi(np.zeros((a.num_rows, 4)), 100, 1e-8)
    assert st == 4 and it == 1
    assert np.all(X == 0.0)


_SPLIT_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import mspmv
a = mspmv.CsrMatrix.synth_stencil(0, 4000, 64)
B = np.random.default_rng(11).uniform(0, 1, (a.num_rows, 4))
with mspmv.GpuCsr(a) as g:
    X, it, h, st = g.cg_multi(B, 5000, 1e-9, hist_cap=5000)
    x1, it1, h1, st1 = g.cg_single(B[:, 0].copy(), 5000, 1e-9, hist_cap=5000)
np.savez(sys.argv[2], X=X, it=it, h=h, st=st, x1=x1, it1=it1, h1=h1, st1=st1)
"""


@pytest.mark.parametrize("split", ["0", "1"])
def test_cg_pipelined_and_split_iterations_match_oracle(orc, tmp_path, split):
    """Both iteration forms reproduce the oracle: single RHS pipelined (MSPMV_CG_SPLIT=0: stop
    test and beta summed by every SpMV workgroup, alpha by every update workgroup) or split
    (=1: p update pass, SpMV MODE 2, update); multi-RHS always split.  Run in a child so the
    environment is read fresh."""
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "sparse-matrix-linear-equations_amd")
    out = str(tmp_path / "r.npz")
    env = dict(os.environ, MSPMV_CG_SPLIT=split)
    r = subprocess.run([sys.executable, "-c", _SPLIT_CHILD, pkg, out], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = np.load(out)
    a = mspmv.CsrMatrix.synth_stencil(0, 4000, 64)
    B = np.random.default_rng(11).uniform(0, 1, (a.num_rows, 4))
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, 1e-9, kernel=1, P=8, hist_cap=5000)
    assert int(d["st"]) == 0 and iter_match(int(d["it"]), it_o, ho, 1e-9)
    k = min(len(d["h"]), len(ho))
    np.testing.assert_allclose(d["h"][:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(d["X"] - Xo) <= 1e-8 * np.linalg.norm(Xo)
    xo, it1_o, h1o = orc.cg_single(a, B[:, 0].copy(), 5000, 1e-9, hist_cap=5000)
    assert int(d["st1"]) == 0 and iter_match(int(d["it1"]), it1_o, h1o, 1e-9)
    k = min(len(d["h1"]), len(h1o))
    np.testing.assert_allclose(d["h1"][:k], h1o[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(d["x1"] - xo) <= 1e-8 * np.linalg.norm(xo)


@pytest.mark.parametrize("L", [8, 16])
@pytest.mark.parametrize("name", ["fem2d", "stencil27"])
def test_cg_multi_vs_oracle_nonzero_split(orc, name, L):
    """cpu_multicg.cpp:202 runs TestCGMultipleRHS with SpmmKernel NONZERO_SPLIT
    (nonzero_splitting.hpp:49-150, behind no_pretreatment.hpp:93's memset(AP, 0)): the oracle
    restated that way, with the reference's g_omp_threads = 8 partition (hyper_parameters.hpp:11),
    against the GPU (which always runs its merge-path SpMM; the kernels differ only in how split
    rows round)."""
    a = spd_cases()[name]()
    n = a.num_rows
    flat = orc.glibc_rand(42, n * L)
    B = flat.reshape(n, L)
    tol = orc.calculate_threshold(flat, n, 1e-5)                  # cpu_multicg.cpp:168 quirk
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, tol, kernel=mspmv.NONZERO_SPLIT, P=8, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 5000, tol, kernel=mspmv.NONZERO_SPLIT, hist_cap=5000)
    assert st == 0 and it_o < 5000
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    for j in range(L):
        assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j])


@pytest.mark.parametrize("L,zero_cols", [(4, [1]), (8, [0, 5]), (32, [3, 17])])
def test_cg_multi_zero_column_breaks_down_alone(orc, L, zero_cols):
    """A zero RHS column gives p.Ap = 0 and alpha = 0/0 in that column only.  The reference
    (no_pretreatment.hpp:109-161) turns the column into NaN, skips it in the max-error history
    (std::max) and never converges it; here the column is frozen at x = 0 (its exact solution),
    reported as MSPMV_ERR_BREAKDOWN, and every other column is solved exactly as the oracle
    solves it: the history matches the oracle's on the GPU's iterations, the other columns'
    X within 1e-8.  L = 32 runs as column groups: every group is solved, the broken ones too."""
    a = spd_cases()["fem2d"]()
    n = a.num_rows
    B = orc.glibc_rand(42, n * L).reshape(n, L).copy()
    B[:, zero_cols] = 0.0
    tol = 1e-9
    Xo, it_o, ho = orc.cg_multi(a, B, 3000, tol, kernel=1, P=8, hist_cap=3000)
    assert it_o == 3000                          # the reference never converges the NaN column
    assert np.all(np.isnan(Xo[:, zero_cols]))
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 3000, tol, hist_cap=3000)
    assert st == 4 and 0 < it_g < 3000
    assert np.all(Xg[:, zero_cols] == 0.0)
    np.testing.assert_allclose(hg, ho[:it_g], rtol=0, atol=1e-10)
    assert hg[-1] < tol
    for j in range(L):
        if j not in zero_cols:
            assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j]), j


def test_cg_multi_breakdown_warns_in_facade(orc):
    a = spd_cases()["fem2d"]()
    n, L = a.num_rows, 2
    B = orc.glibc_rand(42, n * L).reshape(n, L).copy()
    B[:, 1] = 0.0
    X = np.empty(n * L)
    with pytest.warns(RuntimeWarning, match="breakdown"):
        it = mspmv.CGSolveMultiple(a, B.reshape(-1), X, L, 3000, 1e-9)
    assert 0 < it < 3000 and np.all(X.reshape(n, L)[:, 1] == 0.0)


_KNOB_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import mspmv
from test_gpu_cg import spd_cases
a = spd_cases()[sys.argv[4]]()
L = int(sys.argv[5])
B = np.random.default_rng(11).uniform(0, 1, (a.num_rows, L))
with mspmv.GpuCsr(a) as g:
    X, it, h, st = g.cg_multi(B, 5000, 1e-9, hist_cap=5000)
np.save(sys.argv[3] + "/X.npy", X)
np.save(sys.argv[3] + "/h.npy", h)
np.save(sys.argv[3] + "/m.npy", np.array([it, st]))
print("KNOB OK")
"""


@pytest.mark.parametrize("env", [{"MSPMV_CG_DOT": "fused"}, {"MSPMV_CG_REV": "0"},
                                 {"MSPMV_CG_DOT": "fused", "MSPMV_CG_REV": "0"}])
@pytest.mark.parametrize("name,L", [("stencil27", 8), ("fem2d", 4), ("fem2d", 1)])
def test_cg_split_forms_vs_oracle(tmp_path, orc, env, name, L):
    """The split CG's alternative forms kept as knobs -- p.Ap from the SpMM's dot mode
    (MSPMV_CG_DOT=fused) instead of the separate pass, forward-only sweeps (MSPMV_CG_REV=0) --
    against the oracle's CGSolveMultiple like the default form (L = 1 runs split with
    MSPMV_CG_SPLIT=1).  Each variant in its own process (the knobs are read once)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, **env)
    if L == 1:
        e["MSPMV_CG_SPLIT"] = "1"
    r = subprocess.run([sys.executable, "-c", _KNOB_CHILD, os.path.join(root, "sparse-matrix-linear-equations_amd"),
                        os.path.join(root, "tests"), str(tmp_path), name, str(L)], env=e, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "KNOB OK" in r.stdout, r.stdout + r.stderr[-3000:]
    a = spd_cases()[name]()
    B = np.random.default_rng(11).uniform(0, 1, (a.num_rows, L))
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, 1e-9, kernel=1, P=8, hist_cap=5000)
    it, st = np.load(tmp_path / "m.npy")
    assert st == 0 and iter_match(int(it), it_o, ho, 1e-9), (it, it_o)
    hg = np.load(tmp_path / "h.npy")
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    Xg = np.load(tmp_path / "X.npy")
    for j in range(L):
        assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j])


_PIPE_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import mspmv
from test_gpu_cg import spd_cases, big_window_case, perturbed_spd
name, tol, cap = sys.argv[4], float(sys.argv[5]), int(sys.argv[6])
a = big_window_case() if name == "big2d" else perturbed_spd() if name == "perturbed27" else spd_cases()[name]()
b = np.random.default_rng(5).uniform(-1, 1, a.num_rows)
with mspmv.GpuCsr(a) as g:
    x, it, h, st = g.cg_single(b, cap, tol, hist_cap=cap)
    kern = g.cg_kernel_name()
np.savez(sys.argv[3], x=x, it=it, h=h, st=st, kern=np.array(kern))
"""


def perturbed_spd():
    """The 27-point stencil with off-pattern columns, symmetrised and made diagonally dominant (SPD): its
    windows carry a remainder (2,276 entries at this size), which k_cg1_dia sums after each row's offsets."""
    import scipy.sparse as sp
    a = mspmv.CsrMatrix.synth_stencil_perturbed((24, 22, 20), seed=2, extra_frac=0.02, long_frac=0.01)
    A = sp.csr_matrix((a.values, a.column_indices, a.row_offsets), shape=(a.num_rows, a.num_cols))
    S = (abs(A) + abs(A).T) * 0.5
    S = sp.csr_matrix(-S + sp.diags(np.asarray(abs(S).sum(axis=1)).ravel() * 2 + 1.0))
    S.sort_indices()
    return mspmv.CsrMatrix.from_arrays(S.shape[1], S.indptr.astype(np.int32), S.indices.astype(np.int32), S.data)


def big_window_case():
    # 1,100,000 rows of the 7-point triangle stencil: 4,297 window workgroups, past kConsumeTile = 4,096, so
    # the p.Ap partials go through one ticket-folded level before k_cg1_update sums them
    return mspmv.CsrMatrix.synth_stencil(0, 1_100_000, 1000)


@pytest.mark.parametrize("tiles", [False, True])
@pytest.mark.parametrize("name,tol,cap", [("fem2d", 1e-10, 5000), ("fem2d_partial_row", 1e-10, 5000),
                                          ("stencil27", 1e-10, 5000), ("perturbed27", 1e-10, 5000),
                                          ("big2d", 1e-30, 150)])
def test_cg_pipelined_on_windows_vs_oracle(orc, tmp_path, tiles, name, tol, cap):
    """The two-kernel pipelined single-RHS CG (MSPMV_CG_RESIDENT=0) with its SpMV on the offset windows
    (k_cg1_dia: p = r + beta p_old formed at each {r, p} load, Ap, p.Ap per workgroup; MSPMV_DIA=1 puts even
    the small cases' boundary-heavy grids on windows) -- or, MSPMV_DIA=0, on the merge tiles -- against
    CGSolveSingle.  big2d runs 150 iterations (tol 1e-30: none converges)
    with its partials past the consumer limit; its whole history is compared."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "p.npz")
    e = dict(os.environ, MSPMV_CG_RESIDENT="0", MSPMV_DIA="0" if tiles else "1")  # =1: windows at any fill
    r = subprocess.run([sys.executable, "-c", _PIPE_CHILD, os.path.join(root, "sparse-matrix-linear-equations_amd"),
                        os.path.join(root, "tests"), out, name, str(tol), str(cap)], env=e, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = np.load(out)
    kern = str(d["kern"])
    assert ("k_spmv_tile MODE 1" if tiles else "k_cg1_dia") in kern, kern
    a = big_window_case() if name == "big2d" else perturbed_spd() if name == "perturbed27" else spd_cases()[name]()
    if name == "perturbed27" and not tiles:
        assert mspmv.offset_windows(a)["remainder"] > 0  # the windows' remainder path is exercised
    b = np.random.default_rng(5).uniform(-1, 1, a.num_rows)
    xo, it_o, ho = orc.cg_single(a, b, cap, tol, hist_cap=cap)
    it_g, st = int(d["it"]), int(d["st"])
    assert st == 0
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(d["h"]), len(ho))
    np.testing.assert_allclose(d["h"][:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(d["x"] - xo) <= 1e-8 * np.linalg.norm(xo)
