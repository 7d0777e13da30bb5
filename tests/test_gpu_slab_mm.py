"""Column-slab SpMM (mspmv_slab.hip k_spmm_slab, L = 8 and 16): merge-path blocks of rows, each block's
nonzeros reordered by column segment (<= cfg.cols consecutive panel rows, staged in LDS once per block
and segment), rows accumulated in LDS in segment order -- the reference's OmpMergeCsrmm
(work_2025/spmm/merge_based.hpp:46-153) computes the same Y = A X.

Forced with MSPMV_SPMM_SLAB=1 (read when a handle first decides its plain L-wide plan) on banded,
stencil, scattered, skewed, split, empty and rectangular shapes; checked against the oracle's
OmpCsrSpmmT (row-by-row CSR-order sums) within the reordering bound (the slab order is a reordered CSR
sum: mspmv_tile_modes reports every block as 255), bit-identical on repeats and under a CU limit's
rebuilt plan against the oracle again.  Widths outside {8, 16} run column chunks with panel stride L;
the block CG runs its plain SpMM on the slab plan and is held to the oracle's CGSolveMultiple like the
tile path (iterations, history within 1e-10, X within 1e-8).
"""
import numpy as np
import pytest

import mspmv
from gpu_common import check_parity, check_parity_chunked
from test_gpu_cg import iter_match
from test_gpu_slab import scatter_band, with_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


@pytest.fixture
def slab_mm_on(monkeypatch):
    monkeypatch.setenv("MSPMV_SPMM_SLAB", "1")


CASES = {
    "band": lambda: scatter_band(30000, 40, 2000, 3),                        # cant-like banded
    "stencil27": lambda: mspmv.CsrMatrix.synth_stencil(1, 40 * 30 * 30, 40, 30, 30, seed=1, diag_shift=1e-2),
    "scatter": lambda: scatter_band(60000, 40, 10000, 3),                    # wide band: many segments
    "powerlaw": lambda: mspmv.CsrMatrix.synth_powerlaw(40000, 40000, 600000, exponent=1.2, seed=5),
    # a hub row over many blocks (split rows, carries), empty rows, a rectangular X (n > m)
    "hub_rect": lambda: with_rows(20000, 70001, [0 if i % 7 == 0 else (60000 if i == 11 else 9) for i in range(20000)], 6),
    # more short rows than one block may hold: the plan adds blocks
    "short_rows": lambda: with_rows(200000, 5000, [1 if i % 3 else 0 for i in range(200000)], 7),
}
# shapes whose blocks need more segments x chunks than a block's table holds may keep the tiles
MAY_DECLINE = {"powerlaw", "scatter", "hub_rect"}


@pytest.mark.parametrize("L", [8, 16])
@pytest.mark.parametrize("name", list(CASES))
def test_slab_mm_parity(orc, slab_mm_on, name, L):
    a = CASES[name]()
    X = np.random.default_rng(1).uniform(-1, 1, (a.num_cols, L))
    gold = orc.csr_spmm_t(a, X)
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        kname = g.spmm_kernel_name(L)
        if name not in MAY_DECLINE:
            assert kname.startswith("k_spmm_slab<"), kname
        plan = g.tile_plan(L)
        if kname.startswith("k_spmm_slab<"):
            assert np.all(plan["modes"] == 255)
        check_parity(a, Y, gold, X, plan, L)
        Y2 = g.spmm(X)
        g.set_cu_limit(32)  # a rebuilt plan (blocks sized for 32 CUs): parity again, repeats identical
        Y3 = g.spmm(X)
        Y4 = g.spmm(X)
        check_parity(a, Y3, gold, X, g.tile_plan(L), L)
        g.set_cu_limit(0)
    assert Y.tobytes() == Y2.tobytes()
    assert Y3.tobytes() == Y4.tobytes()


@pytest.mark.parametrize("L", [24, 12])
def test_slab_mm_column_chunks(orc, slab_mm_on, L):
    """Even widths outside {8, 16}: chunks of 16 / 8 (and 4) columns of the same panels, stride L."""
    a = CASES["band"]()
    X = np.random.default_rng(2).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity_chunked(a, g, Y, orc.csr_spmm_t(a, X), X, L)
        assert g.spmm_kernel_name(L).startswith("k_spmm_slab<")


def test_slab_mm_device_buffers(orc, slab_mm_on):
    a = CASES["stencil27"]()
    L = 8
    X = np.random.default_rng(3).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        dX, dY = mspmv.DeviceBuffer.from_array(X), mspmv.DeviceBuffer(8 * a.num_rows * L)
        g.spmm_dev(dX, dY, L)
        Y = dY.download((a.num_rows, L))
        check_parity(a, Y, orc.csr_spmm_t(a, X), X, g.tile_plan(L), L)
        dX.free()
        dY.free()


@pytest.mark.parametrize("L", [8, 16])
def test_slab_mm_cg_multi_vs_oracle(orc, slab_mm_on, L):
    """CGSolveMultiple (no_pretreatment.hpp:32-197) with its plain SpMM on the slab plan."""
    a = mspmv.CsrMatrix.synth_stencil(1, 24 * 25 * 26, 24, 25, 26)
    n = a.num_rows
    flat = orc.glibc_rand(42, n * L)
    B = flat.reshape(n, L)
    tol = orc.calculate_threshold(flat, n, 1e-5)
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, tol, kernel=1, P=8, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 5000, tol, hist_cap=5000)
        assert g.spmm_kernel_name(L).startswith("k_spmm_slab<")
        Xg2, it_g2, hg2, st2 = g.cg_multi(B, 5000, tol, hist_cap=5000)  # cached graph: bitwise repeat
    assert st == 0 and st2 == 0
    assert iter_match(it_g, it_o, ho, tol), (it_g, it_o)
    k = min(len(hg), len(ho))
    np.testing.assert_allclose(hg[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(Xg - Xo) <= 1e-8 * np.linalg.norm(Xo)
    assert it_g2 == it_g and Xg.tobytes() == Xg2.tobytes() and hg.tobytes() == hg2.tobytes()


def test_slab_mm_default_choice(monkeypatch):
    """Without MSPMV_SPMM_SLAB the L-wide products keep their tiles (FEM node-block matrices k_spmm_blk):
    the slab plan is opt-in until it measures faster on the BASELINE shapes."""
    monkeypatch.delenv("MSPMV_SPMM_SLAB", raising=False)
    want = {
        "cant": lambda: scatter_band(62451, 64, 2000, 1),
        "stencil": lambda: mspmv.CsrMatrix.synth_stencil(1, 60 * 50 * 50, 60, 50, 50, seed=1, diag_shift=1e-2),
        "fem": lambda: mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3),
    }
    for name, make in want.items():
        with mspmv.GpuCsr(make()) as g:
            for L in (8, 16):
                assert not g.spmm_kernel_name(L).startswith("k_spmm_slab<"), (name, L, g.spmm_kernel_name(L))
