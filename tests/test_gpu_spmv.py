"""GPU parity: merge-path SpMV/SpMM through the C-ABI vs the oracle and the reference's own
golden outputs.  Unsplit rows must be bit-identical; split rows within 2(len+1)eps(|A||x|)."""
import os

import numpy as np
import pytest

import mspmv
from gpu_common import check_parity, check_parity_chunked
from test_oracle_pinning import G, MATS, csr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


def synth_cases():
    return {
        "cant_small": lambda: mspmv.CsrMatrix.synth_banded(6000, 380000, 2000, seed=1),
        "rma10_small": lambda: mspmv.CsrMatrix.synth_banded(4700, 240000, 3000, seed=2),
        "powerlaw": lambda: mspmv.CsrMatrix.synth_powerlaw(20000, 20000, 600000, exponent=1.3, seed=3),
        "powerlaw_rect": lambda: mspmv.CsrMatrix.synth_powerlaw(3000, 70000, 400000, exponent=1.6, seed=4),
        "fem2d": lambda: mspmv.CsrMatrix.synth_stencil(0, 10007, 101),
        "stencil27": lambda: mspmv.CsrMatrix.synth_stencil(1, 12 * 13 * 14, 12, 13, 14),
    }


# --- against the reference's own outputs (golden fixtures) ---------------------------------
@pytest.mark.parametrize("key", MATS)
def test_spmv_vs_reference_gold(key):
    a = csr("m_" + key)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(G[f"m_{key}_x"])
        nb, n = check_parity(a, y, G[f"m_{key}_gold"], G[f"m_{key}_x"], g.tile_plan(1), 1)
        yc = g.spmv(np.full(a.num_cols, 0.0019))
        check_parity(a, yc, G[f"m_{key}_gold_const"], np.full(a.num_cols, 0.0019), g.tile_plan(1), 1)


@pytest.mark.parametrize("key", MATS)
@pytest.mark.parametrize("L", [8, 16])
def test_spmm_vs_reference_rowsplit(key, L):
    a = csr("m_" + key)
    X = G[f"m_{key}_X{L}"]
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity(a, Y, G[f"m_{key}_rowsplit{L}"], X, g.tile_plan(L), L)


def test_kats():
    with mspmv.GpuCsr(csr("fig")) as g:
        assert g.spmv(np.ones(4)).tolist() == [2.0, 0.0, 2.0, 4.0]
        for P in (2, 3, 4, 12):
            np.testing.assert_array_equal(g.merge_coords(P), G[f"fig_coords_P{P}"])
    with mspmv.GpuCsr(csr("lat")) as g:
        assert g.spmv(np.ones(9)).tolist() == [2, 3, 2, 3, 4, 3, 2, 3, 2]


# --- merge coordinates: bit-exact with MergePathSearch -------------------------------------
@pytest.mark.parametrize("key", MATS)
def test_merge_coords_vs_reference(key):
    a = csr("m_" + key)
    with mspmv.GpuCsr(a) as g:
        for P in (1, 2, 3, 4, 8, 64, 256):
            np.testing.assert_array_equal(g.merge_coords(P), G[f"m_{key}_coords_P{P}"])


@pytest.mark.parametrize("name", ["cant_small", "powerlaw", "fem2d"])
def test_merge_coords_vs_oracle_many_parts(orc, name):
    a = synth_cases()[name]()
    with mspmv.GpuCsr(a) as g:
        for P in (1, 7, 256, 4096, 100000):
            np.testing.assert_array_equal(g.merge_coords(P), orc.merge_coords(a, P))


# --- synthetic shapes vs the oracle --------------------------------------------------------
@pytest.mark.parametrize("name", list(synth_cases()))
def test_spmv_synthetic(orc, name):
    a = synth_cases()[name]()
    x = np.random.default_rng(5).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(x)
        plan = g.tile_plan(1)
        nb, n = check_parity(a, y, orc.spmv_gold(a, x), x, plan, 1)
        if name.startswith("powerlaw"):
            assert plan["num_carries"] > 0, "power-law case should exercise cross-tile carries"
        # the reference merge CsrMV at P=256 (within the same bound)
        check_parity(a, y, orc.merge_csrmv(a, x, 256), x, {"bounds": np.array([[0, 0]]), "num_tiles": 0}, 1)
    if name == "fem2d":   # ~7 nnz per row: most rows are not split between walkers
        assert nb > 0.3 * n


def test_tile_modes_cover_both_reductions(orc):
    """k_tile_modes: short uniform rows -> one row per thread (mode 1, bit-exact whole rows);
    long uniform rows -> wider row groups; skewed tiles -> the merge walk (mode 0); SpMM
    plans always walk.  Parity holds on every mix."""
    fem = mspmv.CsrMatrix.synth_stencil(0, 40000, 200, 0, 0, seed=3)
    blk = mspmv.CsrMatrix.synth_fem_blocked(20000, 1000000, 6, 300, seed=2)
    skew = mspmv.CsrMatrix.synth_powerlaw(50000, 50000, 1500000, exponent=1.8, seed=4)
    for a, want in ((fem, {1}), (blk, None), (skew, None)):
        x = np.random.default_rng(8).uniform(-1, 1, a.num_cols)
        with mspmv.GpuCsr(a) as g:
            plan = g.tile_plan(1)
            modes = set(np.unique(plan["modes"]).tolist())
            if want is not None:
                assert modes == want, modes
            if a is blk:
                assert min(modes) >= 3, modes     # ~50 nnz rows: groups of >= 4 lanes
            if a is skew:
                assert 0 in modes, modes          # hub rows: merge walk
            m4 = g.tile_plan(4)["modes"]
            if a is skew:
                assert 0 in set(m4.tolist())
            if a is blk:
                assert m4.min() >= 2          # SpMM row groups: 2 column-pair lanes x >= 2
            X = np.random.default_rng(9).uniform(-1, 1, (a.num_cols, 4))
            check_parity(a, g.spmm(X), orc.csr_spmm_t(a, X), X, g.tile_plan(4), 4)
            nb, n = check_parity(a, g.spmv(x), orc.spmv_gold(a, x), x, plan, 1)
            if a is fem:
                assert nb >= n - 2 * plan["num_tiles"]   # all rows held whole by a tile


def test_skewed_rows_run_one_wave_tiles(orc):
    """Plain SpMV plan choice (spmv_plan): a power-law matrix, whose workgroup tiles are mostly
    merge walks, runs one-wave tiles (64 lanes, 512 merge items); a banded one keeps 256-thread
    tiles.  Parity with 64 walkers per walk tile, and the CG on the skewed handle still runs its
    own workgroup plan."""
    skew = mspmv.CsrMatrix.synth_powerlaw(60000, 60000, 1800000, exponent=1.2, seed=7)
    band = mspmv.CsrMatrix.synth_banded(20000, 1000000, 800, seed=5)
    for a, lanes in ((skew, 64), (band, 256)):
        x = np.random.default_rng(11).uniform(-1, 1, a.num_cols)
        with mspmv.GpuCsr(a) as g:
            y = g.spmv(x)
            plan = g.tile_plan(1)
            assert plan["lanes"] == lanes, (plan["lanes"], lanes)
            assert (",64," in g.kernel_name()) == (lanes == 64), g.kernel_name()
            if lanes == 64:
                assert (plan["modes"] == 0).any()
            check_parity(a, y, orc.spmv_gold(a, x), x, plan, 1)
            # the L = 2 SpMM shares the workgroup single-RHS tile size: unaffected by the choice
            X = np.random.default_rng(12).uniform(-1, 1, (a.num_cols, 2))
            check_parity(a, g.spmm(X), orc.csr_spmm_t(a, X), X, g.tile_plan(2), 2)


@pytest.mark.parametrize("name", ["cant_small", "powerlaw", "fem2d", "powerlaw_rect"])
@pytest.mark.parametrize("L", [1, 2, 4, 8, 16])
def test_spmm_synthetic(orc, name, L):
    a = synth_cases()[name]()
    X = np.random.default_rng(6 + L).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity(a, Y, orc.csr_spmm_t(a, X), X, g.tile_plan(L), L)


@pytest.mark.parametrize("name", ["powerlaw", "fem2d"])
@pytest.mark.parametrize("L", [3, 6, 12, 24, 32, 40, 128])
def test_spmm_any_width(orc, name, L):
    """num_vectors outside {1, 2, 4, 8, 16} (OmpMergeCsrmm takes any; cpu_spmm_v2 defaults to
    32, eval_vectors.sh sweeps 1..1024): column chunks of the native widths with panel stride L,
    odd L through a zero-padded panel."""
    a = synth_cases()[name]()
    X = np.random.default_rng(60 + L).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity_chunked(a, g, Y, orc.csr_spmm_t(a, X), X, L)


def test_column_dictionary_tiles(orc):
    """Scattered-band tiles gather x through sorted per-tile column dictionaries (k_build_dict);
    FEM / stencil tiles keep the direct gathers (power-law tiles: either, by their line counts).
    Either way the products are val * x[col]: unsplit rows bit-identical to SpmvGold."""
    cases = synth_cases()
    for name, want in (("cant_small", True), ("fem2d", False), ("stencil27", False), ("powerlaw", None)):
        a = cases[name]()
        x = np.random.default_rng(4).uniform(-1, 1, a.num_cols)
        with mspmv.GpuCsr(a) as g:
            _, nd = g.tile_streams()
            nt = g.tile_plan(1)["num_tiles"]
            assert want is None or (nd > 0 if want else nd <= max(1, nt // 100)), (name, nd, nt)
            check_parity(a, g.spmv(x), orc.spmv_gold(a, x), x, g.tile_plan(1), 1)


def test_spmm16_column_dictionary_tiles(orc):
    """L = 16 tiles that park their distinct panel rows in LDS (k_spmm_tile DICT): the same
    products in the same order as direct gathers, so the same parity rule; a FEM-blocked shape
    (6 rows per node share their columns, 5 nodes per row in a +-3-node band) lets nearly
    every tile take one (<= 64 distinct columns per 512-item tile)."""
    a = mspmv.CsrMatrix.synth_fem_blocked(6000, 180000, 6, 3, seed=4)
    X = np.random.default_rng(8).uniform(-1, 1, (a.num_cols, 16))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        plan = g.tile_plan(16)
        assert g.dict_tiles(16) > plan["num_tiles"] // 2, (g.dict_tiles(16), plan["num_tiles"])
        assert g.dict_tiles(8) == 0
        check_parity(a, Y, orc.csr_spmm_t(a, X), X, plan, 16)


def test_deterministic_repeat():
    a = mspmv.CsrMatrix.synth_powerlaw(30000, 30000, 900000, exponent=1.4, seed=9)
    x = np.random.default_rng(1).uniform(-1, 1, a.num_cols)
    X = np.random.default_rng(2).uniform(-1, 1, (a.num_cols, 8))
    with mspmv.GpuCsr(a) as g:
        y0, Y0 = g.spmv(x), g.spmm(X)
        for _ in range(3):
            assert g.spmv(x).tobytes() == y0.tobytes()
            assert g.spmm(X).tobytes() == Y0.tobytes()


# --- edge cases --------------------------------------------------------------------------
def _mk(m, n, lens, seed=0):
    rng = np.random.default_rng(seed)
    ro = np.zeros(m + 1, np.int32)
    ro[1:] = np.cumsum(lens)
    ci = np.concatenate([np.sort(rng.choice(n, int(k), replace=False)) for k in lens] or [np.zeros(0)]).astype(np.int32)
    return mspmv.CsrMatrix(m, n, int(ro[-1]), ro, ci, rng.uniform(-1, 1, len(ci)))


@pytest.mark.parametrize("case", ["all_empty", "one_long_row", "long_rows_many_tiles", "single_entry",
                                  "leading_empty", "trailing_empty", "dense_rows", "one_row_matrix"])
def test_edge_cases(orc, case):
    if case == "all_empty":
        a = _mk(5000, 100, np.zeros(5000, int))
    elif case == "one_long_row":
        a = _mk(1, 200000, [150000])
    elif case == "long_rows_many_tiles":
        lens = np.ones(3000, int)
        lens[[10, 1500, 2999]] = [40000, 9000, 25000]
        a = _mk(3000, 60000, lens)
    elif case == "single_entry":
        a = _mk(1, 1, [1])
    elif case == "leading_empty":
        a = _mk(9000, 500, np.r_[np.zeros(8000, int), np.full(1000, 7)])
    elif case == "trailing_empty":
        a = _mk(9000, 500, np.r_[np.full(1000, 7), np.zeros(8000, int)])
    elif case == "dense_rows":
        a = _mk(64, 4096, np.full(64, 4096))
    else:
        a = _mk(1, 10, [10])
    x = np.random.default_rng(3).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(x)
        check_parity(a, y, orc.spmv_gold(a, x), x, g.tile_plan(1), 1)
        X = np.random.default_rng(4).uniform(-1, 1, (a.num_cols, 4))
        check_parity(a, g.spmm(X), orc.csr_spmm_t(a, X), X, g.tile_plan(4), 4)


def test_empty_matrix():
    a = mspmv.CsrMatrix(0, 0, 0, np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0))
    with mspmv.GpuCsr(a) as g:
        assert g.spmv(np.zeros(0)).shape == (0,)


def test_invalid_inputs_fail_loudly():
    bad = mspmv.CsrMatrix(2, 2, 2, np.array([0, 1, 2], np.int32), np.array([0, 5], np.int32), np.ones(2))
    with pytest.raises(mspmv.MspmvError):
        mspmv.GpuCsr(bad)
    bad2 = mspmv.CsrMatrix(2, 2, 2, np.array([0, 2, 1], np.int32), np.array([0, 1], np.int32), np.ones(2))
    with pytest.raises(mspmv.MspmvError):
        mspmv.GpuCsr(bad2)
    a = csr("m_grid3d6")
    with mspmv.GpuCsr(a) as g:
        with pytest.raises(mspmv.MspmvError):
            g.spmm(np.zeros((a.num_cols, 0)))  # L = 0


def test_facade_reference_names(orc):
    a = csr("m_skew300")
    x = G["m_skew300_x"]
    y = np.empty(a.num_rows)
    mspmv.OmpMergeCsrmv(8, a, a.row_offsets[1:], a.column_indices, a.values, x, y)
    check_parity(a, y, G["m_skew300_gold"], x, mspmv._gpu(a).tile_plan(1), 1)
    X = G["m_skew300_X8"]
    Y = np.empty(a.num_rows * 8)
    mspmv.OmpMergeCsrmm(8, a, a.row_offsets[1:], a.column_indices, a.values, X.reshape(-1), Y, 8)
    check_parity(a, Y, G["m_skew300_rowsplit8"], X, mspmv._gpu(a).tile_plan(8), 8)
