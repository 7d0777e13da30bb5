"""Column-slab SpMV (mspmv_slab.hip): blocks of a CU's share of the merge path, each block's nonzeros
reordered by 4,096-column slab of x (staged in LDS), rows accumulated in LDS in slab order.

Forced with MSPMV_SPMV_SLAB=1 (merge-path blocks), =2 (column-group blocks whose partial row sums the
row block's last group folds) and =4 (the column-group blocks in sliced-ELL form, k_spmv_sell; read when a
handle first decides its plain-SpMV plan) on shapes with
scattered, skewed, split, empty and rectangular rows; checked against the oracle's SpmvGold
(cpu_spmv.cpp:241-265) within the reordering bound (the slab order is a reordered CSR sum:
mspmv_tile_modes reports every block as 255), bit-identical on repeats and under a CU limit's
rebuilt plan against the oracle again.  The default choice (scattered band: sliced-ELL with one column
group; large power-law: sliced-ELL with four; FEM, stencil, cant, small power-law: tiles) is checked on its
own.
"""
import numpy as np
import pytest

import mspmv
from gpu_common import check_parity

pytestmark = pytest.mark.gpu


# sell: <NT, PACK>, PACK (short runs packed per lane) on exactly when the plan has more than one column group --
# a matrix narrower than one slab gets one group even when four are asked for
SLAB_KERNEL = {"1": "k_spmv_slab<{nt},0>", "2": "k_spmv_slab<{nt},1>", "4": "k_spmv_sell<{nt},",
               "4g1": "k_spmv_sell<{nt},false>"}


@pytest.fixture(params=["1", "2", "4", "4g1"], ids=["band", "groups", "sell", "sell_one_group"])
def slab_on(monkeypatch, request):
    """1: merge-path blocks (kSlabCfgs[0]); 2: column-group blocks (kSlabCfgs[1], partials folded);
    4: the column-group blocks in sliced-ELL form (k_spmv_sell, 4 groups); 4g1: the same with one column
    group (whole-row blocks staging their own slabs: the default for line-bound bands, round 6)."""
    monkeypatch.setenv("MSPMV_SPMV_SLAB", request.param[0])
    if request.param == "4g1":
        monkeypatch.setenv("MSPMV_SLAB_GROUPS", "1")
    else:
        monkeypatch.delenv("MSPMV_SLAB_GROUPS", raising=False)
    return request.param


def slab_kernel_ok(name, mode):
    want = (SLAB_KERNEL[mode].format(nt="true"), SLAB_KERNEL[mode].format(nt="false"))
    if want[0].endswith(","):
        return name.startswith(want) and name[len(want[0]) if name.startswith(want[0]) else len(want[1]):] in ("true>", "false>")
    return name in want


def scatter_band(m, per_row, band, seed):
    return mspmv.CsrMatrix.synth_banded(m, m * per_row, band, seed=seed)


def with_rows(m, n, lens, seed):
    """m x n with the given row lengths (random sorted distinct columns)."""
    rng = np.random.default_rng(seed)
    lens = np.minimum(np.asarray(lens, np.int64), n)
    ro = np.zeros(m + 1, np.int64)
    ro[1:] = np.cumsum(lens)
    ci = np.empty(int(ro[-1]), np.int32)
    for i in np.flatnonzero(lens):
        ci[ro[i]:ro[i + 1]] = np.sort(rng.choice(n, int(lens[i]), replace=False))
    return mspmv.CsrMatrix.from_arrays(n, ro.astype(np.int32), ci, rng.uniform(-1, 1, ci.size))


CASES = {
    "scatter_band": lambda: scatter_band(60000, 40, 10000, 3),
    "narrow_band": lambda: scatter_band(30000, 30, 500, 4),
    "powerlaw": lambda: mspmv.CsrMatrix.synth_powerlaw(40000, 40000, 1200000, exponent=1.2, seed=5),
    # a hub row over ~20 blocks, empty rows, a rectangular x (n > m) reaching past the last slab edge
    "hub_rect": lambda: with_rows(20000, 70001, [0 if i % 7 == 0 else (60000 if i == 11 else 9) for i in range(20000)], 6),
    # more short rows than one block may hold (rows per block <= 2,047): the plan adds blocks
    "short_rows": lambda: with_rows(200000, 5000, [1 if i % 3 else 0 for i in range(200000)], 7),
}


@pytest.mark.parametrize("name", list(CASES))
def test_slab_parity(orc, slab_on, name):
    a = CASES[name]()
    x = np.random.default_rng(1).uniform(-1, 1, a.num_cols)
    gold = orc.spmv_gold(a, x)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(x)
        assert slab_kernel_ok(g.kernel_name(), slab_on), g.kernel_name()
        plan = g.tile_plan(1)
        assert np.all(plan["modes"] == 255)
        check_parity(a, y, gold, x, plan, 1)
        y2 = g.spmv(x)
        g.set_cu_limit(32)  # a rebuilt plan (blocks sized for 32 CUs): parity again, repeats identical
        y3 = g.spmv(x)
        y4 = g.spmv(x)
        check_parity(a, y3, gold, x, g.tile_plan(1), 1)
        g.set_cu_limit(0)
    assert y.tobytes() == y2.tobytes()
    assert y3.tobytes() == y4.tobytes()



@pytest.mark.parametrize("name", ["scatter_band", "powerlaw", "hub_rect"])
def test_slab_nonfinite_x(orc, slab_on, name):
    """Inf and NaN in x, column 0 among them (the sliced-ELL pad slots hold value 0 at column 0 and are
    selected out by their run's length): the oracle's non-finite rows exactly (NaN where it has NaN, the
    infinities' signs), and every other row bit-equal to the same plan's product with the bad columns
    zeroed, itself within the reordering bound."""
    a = CASES[name]()
    rng = np.random.default_rng(21)
    x = rng.uniform(-1, 1, a.num_cols)
    bad = rng.choice(a.num_cols, 6, replace=False)
    x[bad[:2]] = np.inf
    x[bad[2:4]] = -np.inf
    x[bad[4:]] = np.nan
    x[0] = np.inf
    clean = np.where(np.isfinite(x), x, 0.0)
    gold = orc.spmv_gold(a, x)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(x)
        assert slab_kernel_ok(g.kernel_name(), slab_on), g.kernel_name()
        yc = g.spmv(clean)
        check_parity(a, yc, orc.spmv_gold(a, clean), clean, g.tile_plan(1), 1)
    assert np.array_equal(np.isnan(y), np.isnan(gold))
    assert np.array_equal(np.isfinite(y), np.isfinite(gold))
    inf = ~np.isfinite(gold) & ~np.isnan(gold)
    assert np.array_equal(y[inf], gold[inf])
    fin = np.isfinite(gold)
    assert 0 < (~fin).sum() and fin.sum() > 0.5 * fin.size
    assert y[fin].tobytes() == yc[fin].tobytes()

def test_slab_device_buffers_and_cg_unaffected(orc, slab_on):
    """The slab plan serves the plain product only: the CG on the same handle runs its tile plan."""
    a = scatter_band(20000, 12, 3000, 8)
    import scipy.sparse as sp
    A = sp.csr_matrix((a.values, a.column_indices, a.row_offsets), shape=(a.num_rows, a.num_cols))
    S = (abs(A) + abs(A).T) * 0.5
    S = sp.csr_matrix(S + sp.diags(np.asarray(S.sum(axis=1)).ravel() + 1.0))
    S.sort_indices()
    spd = mspmv.CsrMatrix.from_arrays(S.shape[1], S.indptr.astype(np.int32), S.indices.astype(np.int32), S.data)
    x = np.random.default_rng(2).uniform(-1, 1, spd.num_cols)
    with mspmv.GpuCsr(spd) as g:
        dx, dy = mspmv.DeviceBuffer.from_array(x), mspmv.DeviceBuffer(8 * spd.num_rows)
        g.spmm_dev(dx, dy, 1)
        y = dy.download(spd.num_rows)
        assert slab_kernel_ok(g.kernel_name(), slab_on), g.kernel_name()
        check_parity(spd, y, orc.spmv_gold(spd, x), x, g.tile_plan(1), 1)
        b = np.random.default_rng(3).uniform(-1, 1, spd.num_rows)
        xs, it, _, st = g.cg_single(b, 400, 1e-10)
        assert st == 0
        r = b - orc.spmv_gold(spd, xs)
        assert np.linalg.norm(r) <= 1e-8 * np.linalg.norm(b)
        dx.free()
        dy.free()


def test_slab_default_choice(orc, monkeypatch):
    """The default plain-SpMV choice: scattered band at >= 12,288 nonzeros per CU -> the sliced-ELL kernel
    with one column group (round 6; the slab blocks before); power-law rows at >= 12,288 nonzeros per CU ->
    the sliced-ELL column groups (both checked against the oracle here too); a smaller power-law matrix ->
    one-wave tiles; FEM, stencil, cant -> tiles."""
    monkeypatch.delenv("MSPMV_SPMV_SLAB", raising=False)
    monkeypatch.delenv("MSPMV_SLAB_GROUPS", raising=False)
    want = {
        "scatter": (lambda: scatter_band(217918, 53, 10000, 77), "k_spmv_sell<"),
        "powerlaw": (lambda: mspmv.CsrMatrix.synth_powerlaw(120000, 120000, 4000000, exponent=1.2, seed=9),
                     "k_spmv_sell<"),
        "powerlaw_small": (lambda: mspmv.CsrMatrix.synth_powerlaw(60000, 60000, 1800000, exponent=1.2, seed=7),
                           "k_spmv_tile<"),
        "fem": (lambda: mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3), None),
        "stencil": (lambda: mspmv.CsrMatrix.synth_stencil(1, 40 * 30 * 30, 40, 30, 30, seed=1, diag_shift=1e-2), None),
        "cant": (lambda: scatter_band(62451, 64, 2000, 1), None),  # small blocks: tiles win (r04x)
    }
    for name, (make, prefix) in want.items():
        a = make()
        with mspmv.GpuCsr(a) as g:
            k = g.kernel_name()
            if prefix is None:
                assert not k.startswith(("k_spmv_slab<", "k_spmv_sell<")), (name, k)
            else:
                assert k.startswith(prefix), (name, k)
            if name in ("powerlaw", "scatter"):
                x = np.random.default_rng(4).uniform(-1, 1, a.num_cols)
                y = g.spmv(x)
                check_parity(a, y, orc.spmv_gold(a, x), x, g.tile_plan(1), 1)
                assert y.tobytes() == g.spmv(x).tobytes()
