"""Offset windows (csrc/mspmv_dia.hip): 64-row windows whose rows list their columns at <= 32 common
offsets col - row, values stored lane-major per window, one wave per window with lane = row.

Every row is summed from 0.0 in its CSR order (the planner requires ascending columns), mul then
add, so every row -- and every column of an SpMM -- is bit-identical to the oracle's SpmvGold
(cpu_spmv.cpp:241-265) / row-by-row CsrSpmm; the plan reports every window as mode 1 and check_parity
demands exactly that.  Shapes: 27-point and 2-D stencils (the nlpkkt120 and parabolic_fem shapes,
windows straddling grid lines: presence masks), a tridiagonal band (every window full), a partial last
window, rectangular panels, empty rows and rows missing offsets (forced with MSPMV_DIA=1), an x holding
inf where no row reads it.  The L-wide products take the windows too (MSPMV_DIA_SPMM=0 opts them out),
and the block CG runs its SpMM on the windows, held to the oracle's CGSolveMultiple
(no_pretreatment.hpp:32-197) like the tile path.
"""
import re

import numpy as np
import pytest

import mspmv
from gpu_common import check_parity, check_parity_chunked
from test_gpu_cg import iter_match
from test_gpu_slab import scatter_band

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


@pytest.fixture(autouse=True)
def _windows_every_width(monkeypatch):
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    monkeypatch.delenv("MSPMV_DIA_SPMM", raising=False)


def is_dia(name, L=None):
    """The offset-window kernel k_spmm_dia<L, ...> (one window per wave)."""
    m = re.match(r"k_spmm_dia<(\d+),", name)
    return m is not None and (L is None or int(m.group(1)) == L)


def band(m, offsets, seed, n=None, drop=0.0):
    """m x n, row r holding columns r + d (d in offsets, inside [0, n)); a fraction `drop` of the
    entries removed at random (rows missing offsets)."""
    n = m if n is None else n
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for d in sorted(offsets):
        r = np.arange(m)
        c = r + d
        ok = (c >= 0) & (c < n)
        rows.append(r[ok])
        cols.append(c[ok])
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    if drop > 0:
        keep = rng.random(r.size) >= drop
        r, c = r[keep], c[keep]
    order = np.lexsort((c, r))
    r, c = r[order], c[order]
    ro = np.zeros(m + 1, np.int64)
    np.add.at(ro, r + 1, 1)
    ro = np.cumsum(ro)
    return mspmv.CsrMatrix.from_arrays(n, ro.astype(np.int32), c.astype(np.int32), rng.uniform(-1, 1, c.size))


CASES = {
    "stencil27": lambda: mspmv.CsrMatrix.synth_stencil(1, 33 * 30 * 29, 33, 30, 29, seed=1, diag_shift=1e-2),
    "fem2d": lambda: mspmv.CsrMatrix.synth_stencil(0, 100003, 301),
    "tridiag": lambda: band(64 * 500, [-1, 0, 1], 2),                 # every window full
    "partial": lambda: band(64 * 77 + 13, [-70, -3, 0, 2, 9, 70], 3),  # a 13-row last window
    "rect": lambda: band(20000, [0, 5, 17000, 30000], 4, n=50001),    # n > m, far offsets
    # shapes the windows were not designed on (round 6, windows plus a remainder): off-pattern columns and
    # rows of 35 entries; a KKT saddle point whose upper rows hold 34 offsets
    "perturbed27": lambda: mspmv.CsrMatrix.synth_stencil_perturbed((33, 30, 29), seed=2, extra_frac=0.02,
                                                                   long_frac=0.01),
    "kkt": lambda: mspmv.CsrMatrix.synth_kkt((20, 21, 22), seed=3),
}
REMAINDER = {"perturbed27"}  # cases with entries off the windows' offset lists (the KKT's 34 offsets fit whole)
# windows whose rows miss offsets and empty rows: taken only when forced (fill below kDiaAutoFill)
FORCED = {
    "holes": lambda: band(40000, [-200, -1, 0, 1, 200], 5, drop=0.3),
    "empty_rows": lambda: band(30000, [0, 3], 6, drop=0.6),
}


def _check_product(a, g, L, orc):
    rng = np.random.default_rng(L)
    if L == 1:
        x = rng.uniform(-1, 1, a.num_cols)
        y = g.spmv(x)
        gold = orc.spmv_gold(a, x)
        assert is_dia(g.kernel_name(), 1), g.kernel_name()
        plan = g.tile_plan(1)
        n_exact, n = check_parity(a, y, gold, x, plan, 1)
        assert n_exact == _exact_rows(plan)
        assert g.spmv(x).tobytes() == y.tobytes()
        return
    X = rng.uniform(-1, 1, (a.num_cols, L))
    Y = g.spmm(X)
    assert is_dia(g.spmm_kernel_name(L), L), g.spmm_kernel_name(L)
    plan = g.tile_plan(L)
    n_exact, n = check_parity(a, Y, orc.csr_spmm_t(a, X), X, plan, L)
    assert n_exact == _exact_rows(plan)
    assert g.spmm(X).tobytes() == Y.tobytes()


def _exact_rows(plan):
    """Rows of windows in mode 1 (summed in CSR order: bit-identical); windows holding remainder entries
    report 255 (their rows within the reordering bound).  No other mode occurs on the windows."""
    modes, b = plan["modes"], plan["bounds"]
    assert np.all((modes == 1) | (modes == 255)), np.unique(modes)
    rows = np.diff(b[:, 0])
    return int(rows[modes == 1].sum())


@pytest.mark.parametrize("L", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("name", list(CASES))
def test_dia_parity(orc, monkeypatch, name, L):
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = CASES[name]()
    w = mspmv.offset_windows(a)
    assert w is not None and (w["remainder"] > 0) == (name in REMAINDER), (name, w and w["remainder"])
    with mspmv.GpuCsr(a) as g:
        _check_product(a, g, L, orc)


@pytest.mark.parametrize("L", [1, 8])
@pytest.mark.parametrize("name", list(FORCED))
def test_dia_forced_parity(orc, monkeypatch, name, L):
    a = FORCED[name]()
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    with mspmv.GpuCsr(a) as g:  # fill below the automatic threshold: the tiles
        assert not is_dia(g.spmm_kernel_name(L))
    monkeypatch.setenv("MSPMV_DIA", "1")
    with mspmv.GpuCsr(a) as g:
        _check_product(a, g, L, orc)


def test_dia_cu_limit_and_inf(orc, monkeypatch):
    """A CU limit drops and rebuilds the plan (same bits); an inf in x where no row of a masked window
    reads it stays out of every row (absent entries are skipped, not multiplied by 0)."""
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = CASES["partial"]()
    x = np.random.default_rng(9).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        y0 = g.spmv(x)
        g.set_cu_limit(32)
        y1 = g.spmv(x)
        assert is_dia(g.kernel_name(), 1)
        g.set_cu_limit(0)
        assert y0.tobytes() == y1.tobytes()
        x[0] = np.inf  # column 0: read by rows 0, 3 and 70 only (offsets 0, -3, -70)
        y2 = g.spmv(x)
    gold = orc.spmv_gold(a, x)
    assert np.array_equal(np.isfinite(y2), np.isfinite(gold))
    fin = np.isfinite(gold)
    assert y2[fin].tobytes() == gold[fin].tobytes()


@pytest.mark.parametrize("L", [1, 2, 8, 16])
@pytest.mark.parametrize("name", ["partial", "stencil27"])
def test_dia_nonfinite_x_exact_fallback(orc, monkeypatch, name, L):
    """Masked windows are summed first as if every row held every offset (an absent entry's 0.0 adds +-0.0)
    and again with the absent entries selected out when a row comes out non-finite.  Inf and NaN in x/X --
    at columns read only through absent entries of masked windows and at columns rows do read -- give the
    oracle's rows exactly: the same non-finite rows (NaN where it has NaN) and every finite row bit-equal."""
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = CASES[name]()
    rng = np.random.default_rng(17 + L)
    X = rng.uniform(-1, 1, (a.num_cols, L))
    bad = rng.choice(a.num_cols, 6, replace=False)
    X[bad[:2]] = np.inf
    X[bad[2:4]] = -np.inf
    X[bad[4:]] = np.nan
    X[0] = np.inf  # the partial band: column 0 is read by rows 0, 3 and 70 only
    with mspmv.GpuCsr(a) as g:
        if L == 1:
            Y = g.spmv(X[:, 0].copy())
            gold = orc.spmv_gold(a, X[:, 0].copy())
            assert is_dia(g.kernel_name(), 1), g.kernel_name()
        else:
            Y = g.spmm(X)
            gold = orc.csr_spmm_t(a, X)
            assert is_dia(g.spmm_kernel_name(L), L), g.spmm_kernel_name(L)
    assert np.array_equal(np.isnan(Y), np.isnan(gold))
    assert np.array_equal(np.isfinite(Y), np.isfinite(gold))
    fin = np.isfinite(gold)
    assert fin.sum() > 0.9 * fin.size
    assert np.array_equal(Y[~fin & ~np.isnan(gold)], gold[~fin & ~np.isnan(gold)])  # the infinities' signs
    if name in REMAINDER:
        return
    assert Y[fin].tobytes() == gold[fin].tobytes()


@pytest.mark.parametrize("L", [24, 12, 5])
def test_dia_column_chunks(orc, monkeypatch, L):
    """Widths outside {1, 2, 4, 8, 16}: column chunks (odd L on a zero-padded panel) on the same
    windows, panel stride L."""
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = CASES["stencil27"]()
    X = np.random.default_rng(2).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity_chunked(a, g, Y, orc.csr_spmm_t(a, X), X, L)
        assert is_dia(g.spmm_kernel_name(L))


def test_dia_device_buffers(orc, monkeypatch):
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = CASES["fem2d"]()
    L = 8
    X = np.random.default_rng(3).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        dX, dY = mspmv.DeviceBuffer.from_array(X), mspmv.DeviceBuffer(8 * a.num_rows * L)
        g.spmm_dev(dX, dY, L)
        Y = dY.download((a.num_rows, L))
        n_exact, n = check_parity(a, Y, orc.csr_spmm_t(a, X), X, g.tile_plan(L), L)
        assert n_exact == n
        dX.free()
        dY.free()


@pytest.mark.parametrize("L", [2, 8, 16])
def test_dia_cg_multi_vs_oracle(orc, monkeypatch, L):
    """CGSolveMultiple with its plain SpMM on the offset windows (configs[4]'s iteration shape)."""
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = mspmv.CsrMatrix.synth_stencil(1, 24 * 25 * 26, 24, 25, 26)
    n = a.num_rows
    flat = orc.glibc_rand(42, n * L)
    B = flat.reshape(n, L)
    tol = orc.calculate_threshold(flat, n, 1e-5)
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, tol, kernel=1, P=8, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 5000, tol, hist_cap=5000)
        assert is_dia(g.spmm_kernel_name(L), L)
        Xg2, it_g2, hg2, st2 = g.cg_multi(B, 5000, tol, hist_cap=5000)  # cached graph: bitwise repeat
    assert st == 0 and st2 == 0
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(Xg - Xo) <= 1e-8 * np.linalg.norm(Xo)
    assert it_g2 == it_g and Xg.tobytes() == Xg2.tobytes() and hg.tobytes() == hg2.tobytes()


def test_dia_default_choice(monkeypatch):
    """Stencils take the windows; FEM node blocks, scattered bands, power-law rows, rows with unsorted
    columns (forced or not) and MSPMV_DIA=0 keep the tile plans."""
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    rng = np.random.default_rng(4)
    tri = band(64 * 40, [-1, 0, 1], 7)
    ci = tri.column_indices.copy()
    ci[tri.row_offsets[5]:tri.row_offsets[6]] = ci[tri.row_offsets[5]:tri.row_offsets[6]][::-1]
    unsorted = mspmv.CsrMatrix.from_arrays(tri.num_cols, tri.row_offsets, ci, rng.uniform(-1, 1, ci.size))
    want = {
        "stencil27": (CASES["stencil27"], True),
        "fem2d": (CASES["fem2d"], True),
        "fem_blocked": (lambda: mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3), False),
        "cant": (lambda: scatter_band(62451, 64, 2000, 1), False),
        "powerlaw": (lambda: mspmv.CsrMatrix.synth_powerlaw(40000, 40000, 600000, exponent=1.2, seed=5), False),
        "unsorted": (lambda: unsorted, False),
    }
    for name, (make, dia) in want.items():
        with mspmv.GpuCsr(make()) as g:
            for L in (1, 8):
                assert is_dia(g.spmm_kernel_name(L)) == dia, (name, L, g.spmm_kernel_name(L))
    monkeypatch.setenv("MSPMV_DIA_SPMM", "0")  # the L-wide products opted out: only the SpMV takes the windows
    with mspmv.GpuCsr(CASES["stencil27"]()) as g:
        assert is_dia(g.kernel_name(), 1)
        assert not is_dia(g.spmm_kernel_name(8))
        assert not is_dia(g.spmm_kernel_name(2))
    monkeypatch.setenv("MSPMV_DIA", "1")
    with mspmv.GpuCsr(unsorted) as g:
        assert not is_dia(g.kernel_name())
    monkeypatch.setenv("MSPMV_DIA", "0")
    with mspmv.GpuCsr(CASES["stencil27"]()) as g:
        assert not is_dia(g.kernel_name())
        assert not is_dia(g.spmm_kernel_name(8))
