"""GPU: node-block staging (k_build_blocks / blk_stage) -- FEM rows of one mesh node
share their column list, so a tile stages each run's list once (16-bit offsets of its longest
row) and gathers each x once for all the run's rows.

Runs at most 64 columns wide are summed in registers by a fixed lane tree (tile mode 255): those
rows are within the reordering bound 2 (len+1) eps (|A||x|)_i of the oracle's SpmvGold
(cpu_spmv.cpp:241-265) and reproducible bit for bit.  Wider runs keep the striped path's LDS
slots and reduction: every row outside register tiles must be BIT-IDENTICAL to the run with node
blocks switched off (MSPMV_SPMV_BLOCKS=0, in a child process since the tuning is read once per
process).  Covered: equal-length node rows,
prefix runs (rows of one node 52 and 53 long, as the pwtk-shaped generator makes them), rows
wider than 64 columns (pattern chunks), runs longer than 8 rows (split), empty rows inside runs,
a Kronecker FEM matrix solved by the pipelined single-RHS CG (blocks in the fused CG SpMV), the
full pwtk shape, and imperfect FEM plans: nodes of 5 / 7 unknowns, rows with an off-pattern column,
long rows split between tiles and stencil rows mixed in -- a plan whose tiles are mostly register run
tiles runs the column-pair kernel whole (k_spmv_blk), its register fallback taking the other tiles
(every tile reported 255: all rows within the reordering bound)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import mspmv
from gpu_common import check_parity

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sparse-matrix-linear-equations_amd")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


def kron_fem(nx, ny, dof, empty_every=0):
    """SPD K = kron(S, B): S a 5-point M-matrix on an nx x ny node grid (diag 4.2), B = I + 0.2 J
    (dof x dof); every row of a node lists the same columns.  empty_every > 0 clears every
    empty_every-th node's rows (empty rows inside a tile's runs; the matrix is then singular)."""
    import scipy.sparse as sp
    n = nx * ny
    main = np.full(n, 4.2)
    ex = -np.ones(n - 1)
    ex[np.arange(1, n) % nx == 0] = 0.0
    ey = -np.ones(n - nx)
    S = sp.diags([main, ex, ex, ey, ey], [0, 1, -1, nx, -nx], format="csr")
    B = np.eye(dof) + 0.2 * np.ones((dof, dof))
    K = sp.kron(S, sp.csr_matrix(B), format="csr")
    if empty_every:
        keep = np.ones(K.shape[0])
        for node in range(0, n, empty_every):
            keep[node * dof:(node + 1) * dof] = 0.0
        K = sp.diags(keep) @ K
        K = K.tocsr()
    K.eliminate_zeros()
    K.sort_indices()
    return mspmv.CsrMatrix.from_arrays(K.shape[1], K.indptr.astype(np.int32), K.indices.astype(np.int32),
                                       K.data.astype(np.float64))


def kron_fem9(nx, ny, dof):
    """kron(S9, B): a 9-point node stencil (3-D-like FEM coupling, 9 nodes per row), dof unknowns
    per node -> 9 dof columns per row (pwtk-like widths: 54 at dof 6)."""
    import scipy.sparse as sp
    n = nx * ny
    rows, cols = [], []
    for i in range(ny):
        for j in range(nx):
            for di in (-1, 0, 1):
                for dj in (-1, 0, 1):
                    if 0 <= i + di < ny and 0 <= j + dj < nx:
                        rows.append(i * nx + j)
                        cols.append((i + di) * nx + j + dj)
    vals = np.where(np.array(rows) == np.array(cols), 9.5, -1.0)
    S = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    B = np.eye(dof) + 0.2 * np.ones((dof, dof))
    K = sp.kron(S, sp.csr_matrix(B), format="csr")
    K.sort_indices()
    return mspmv.CsrMatrix.from_arrays(K.shape[1], K.indptr.astype(np.int32), K.indices.astype(np.int32),
                                       K.data.astype(np.float64))


def cases():
    """Matrices whose tiles take node blocks (whole-row tiles, runs >= 32 columns wide on average,
    <= 8 run chunks per tile -- one round for the tile's 4 waves)."""
    return {
        "pwtk_small": lambda: mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3),
        "kron9_6": lambda: kron_fem9(60, 50, 6),            # 54 columns per row
        "kron9_7": lambda: kron_fem9(50, 40, 7),            # 63 columns per row
        "kron12_wide": lambda: kron_fem(30, 30, 12),        # 60 columns per row: one chunk
        "kron9_8_wider": lambda: kron_fem9(25, 20, 8),      # 72 columns per row: two chunks (LDS path)
        "kron9_6_empty": lambda: kron_fem9(50, 40, 6),      # (see test_blocks_empty_rows)
    }


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import mspmv
d = np.load(sys.argv[2])
a = mspmv.CsrMatrix.from_arrays(int(d["n"]), d["ro"], d["ci"], d["va"])
with mspmv.GpuCsr(a) as g:
    y = g.spmv(d["x"])
    nb = g.plan_block_tiles(1)
np.savez(sys.argv[3], y=y, nb=nb)
"""


def spmv_in_child(tmp_path, a, x, blocks):
    inp, out = str(tmp_path / f"in{blocks}.npz"), str(tmp_path / f"out{blocks}.npz")
    np.savez(inp, n=a.num_cols, ro=a.row_offsets, ci=a.column_indices, va=a.values, x=x)
    env = dict(os.environ, MSPMV_SPMV_BLOCKS=str(blocks))
    r = subprocess.run([sys.executable, "-c", _CHILD, PKG, inp, out], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = np.load(out)
    return d["y"], int(d["nb"])


def register_rows(a, plan):
    """Rows of tiles the kernel reduces in registers (tile mode 255)."""
    mask = np.zeros(a.num_rows, bool)
    for t in np.flatnonzero(plan["modes"][: plan["num_tiles"]] == 255):
        mask[plan["bounds"][t][0]:plan["bounds"][t + 1][0]] = True
    return mask


def test_blocks_empty_rows(orc):
    """Empty rows inside runs (an empty row is a prefix of any list: it joins the run)."""
    a = kron_fem9(50, 40, 6)
    ro = a.row_offsets.copy()
    keep = np.ones(a.num_rows, bool)
    keep[::37] = False
    keep[1::37] = False
    lens = np.diff(ro) * keep
    mask = np.repeat(keep, np.diff(ro))
    e = mspmv.CsrMatrix.from_arrays(a.num_cols, np.concatenate([[0], np.cumsum(lens)]).astype(np.int32),
                                    a.column_indices[mask], a.values[mask])
    x = np.random.default_rng(3).uniform(-1, 1, e.num_cols)
    with mspmv.GpuCsr(e) as g:
        assert g.plan_block_tiles(1) > 0
        y = g.spmv(x)
        check_parity(e, y, orc.spmv_gold(e, x), x, g.tile_plan(1), 1)
        Y = g.spmm(np.stack([x, 2 * x], axis=1))
    assert np.all(y[~keep] == 0.0) and np.all(Y[~keep] == 0.0)


@pytest.mark.parametrize("name", [k for k in cases() if k != "kron9_6_empty"])
def test_blocks_parity(orc, tmp_path, name):
    a = cases()[name]()
    x = np.random.default_rng(7).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        nb = g.plan_block_tiles(1)
        plan = g.tile_plan(1)
        y = g.spmv(x)
        y2 = g.spmv(x)
        check_parity(a, y, orc.spmv_gold(a, x), x, plan, 1)
    assert nb > 0, "no tile took the node-block staging"
    assert y.tobytes() == y2.tobytes()  # fixed reduction order: run-to-run reproducible
    y_off, nb_off = spmv_in_child(tmp_path, a, x, 0)
    assert nb_off == 0
    keep = ~register_rows(a, plan)  # LDS-path rows: the striped staging's bits exactly
    assert y[keep].tobytes() == y_off[keep].tobytes(), "node-block staging changed LDS-path result bits"


def test_blocks_not_taken_where_they_lose():
    """Stencils and random bands have no two rows with one column list; 5-point node stencils with
    3 or 6 unknowns per node (15 / 30 columns, 11-20 runs per tile) measured slower on node blocks:
    striped staging for all four."""
    for a in (mspmv.CsrMatrix.synth_stencil(0, 10007, 101), mspmv.CsrMatrix.synth_banded(6000, 380000, 2000, seed=1),
              kron_fem(90, 80, 3), kron_fem(60, 50, 6)):
        with mspmv.GpuCsr(a) as g:
            assert g.plan_block_tiles(1) == 0


@pytest.mark.parametrize("dof", [6, 7])
def test_blocks_in_pipelined_cg(orc, dof):
    """The fused CG SpMV (MODE 1: p = r + beta p_old gathered as {r, p} pairs) stages node blocks
    too; the solve must match the oracle's CGSolveSingle as every single-RHS CG does.  dof 7: runs
    of 6 + 1 rows, column pairs broken at every node boundary."""
    a = kron_fem9(60, 50, dof)
    b = orc.glibc_rand(42, a.num_rows)
    xo, it_o, ho = orc.cg_single(a, b, 5000, 1e-10, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        assert g.plan_block_tiles(1) > 0
        xg, it_g, hg, st = g.cg_single(b, 5000, 1e-10, hist_cap=5000)
    assert st == 0 and it_g == it_o
    np.testing.assert_allclose(hg, ho[: len(hg)], rtol=0, atol=1e-10)
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)


def test_blocks_full_pwtk_shape(orc, tmp_path):
    a = mspmv.CsrMatrix.synth_fem_blocked(217918, 11524432, 6, 1700, seed=1)
    x = np.random.default_rng(11).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        nb = g.plan_block_tiles(1)
        nt = g.tile_plan(1)["num_tiles"]
        y = g.spmv(x)
        check_parity(a, y, orc.spmv_gold(a, x), x, g.tile_plan(1), 1)
    assert nb >= 0.9 * nt, (nb, nt)


# ---- node-block SpMM (k_spmm_blk: one panel-row gather per (run, column)) -------------------
_SPMM_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import mspmv
d = np.load(sys.argv[2])
a = mspmv.CsrMatrix.from_arrays(int(d["n"]), d["ro"], d["ci"], d["va"])
with mspmv.GpuCsr(a) as g:
    Y = g.spmm(d["X"])
np.savez(sys.argv[3], Y=Y)
"""


@pytest.mark.parametrize("name", ["pwtk_small", "kron9_6", "kron9_7", "kron12_wide"])
@pytest.mark.parametrize("L", [2, 4, 8, 16, 3, 32])
def test_blocks_spmm_parity(orc, tmp_path, name, L):
    """Y = A X on the node-block plan (every single-RHS tile a register run tile) against the
    oracle's row-split OmpCsrSpmmT (row_splitting.hpp:15-54) within the reordering bound, for the
    native widths, an odd width (zero-padded panel) and a chunked width (panel stride 32)."""
    from gpu_common import check_parity_chunked
    a = cases()[name]()
    X = np.random.default_rng(L).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        Y2 = g.spmm(X)
        check_parity_chunked(a, g, Y, orc.csr_spmm_t(a, X), X, L)
        reg = g.tile_plan(1)["modes"]
    assert Y.tobytes() == Y2.tobytes()
    if name == "pwtk_small":  # all tiles register tiles -> the SpMM ran k_spmm_blk
        assert np.all(reg == 255)


def test_blocks_spmm_vs_merge_tiles(orc, tmp_path):
    """The node-block SpMM against the L-wide merge tiles (MSPMV_SPMM_BLK=0, in a child process):
    both within the reordering bound of the same sequential sums, so within twice it of each other."""
    a = cases()["pwtk_small"]()
    X = np.random.default_rng(5).uniform(-1, 1, (a.num_cols, 16))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
    inp, out = str(tmp_path / "in.npz"), str(tmp_path / "out.npz")
    np.savez(inp, n=a.num_cols, ro=a.row_offsets, ci=a.column_indices, va=a.values, X=X)
    r = subprocess.run([sys.executable, "-c", _SPMM_CHILD, PKG, inp, out],
                       env=dict(os.environ, MSPMV_SPMM_BLK="0"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    Yo = np.load(out)["Y"]
    from gpu_common import EPS, abs_bound
    bound, lens = abs_bound(a, X)
    assert np.all(np.abs(Y - Yo) <= 4.0 * (lens[:, None] + 1) * EPS * bound + 1e-300)


@pytest.mark.parametrize("L", [4, 8, 16])
def test_blocks_cg_multi(orc, L):
    """CGSolveMultiple's split iteration runs the node-block SpMM in dot mode (x.(Ax) partials
    per tile, k_fold_dot): the whole solve against the oracle (NONZERO_SPLIT, as cpu_multicg)."""
    a = kron_fem9(60, 50, 6)
    n = a.num_rows
    flat = orc.glibc_rand(42, n * L)
    B = flat.reshape(n, L)
    tol = orc.calculate_threshold(flat, n, 1e-5)
    Xo, it_o, ho = orc.cg_multi(a, B, 5000, tol, kernel=mspmv.NONZERO_SPLIT, P=8, hist_cap=5000)
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 5000, tol, hist_cap=5000)
    assert st == 0 and it_g == it_o
    np.testing.assert_allclose(hg, ho[: len(hg)], rtol=0, atol=1e-10)
    for j in range(L):
        assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j])


def test_blocks_spai_pcg(orc):
    """SPAI-PCG: both SpMMs (A P and M R, M on A's pattern) on node-block plans in dot mode."""
    a = kron_fem9(40, 30, 6)
    m_vals = mspmv.spai_values(a)
    B = orc.glibc_rand(7, a.num_rows * 8).reshape(a.num_rows, 8)
    Xo, it_o, ho = orc.pcg_spai_multi(a, m_vals, B, 3000, 1e-9, kernel=1, P=8, hist_cap=3000)
    m = mspmv.CsrMatrix.from_arrays(a.num_cols, a.row_offsets, a.column_indices, m_vals)
    with mspmv.GpuCsr(a) as g, mspmv.GpuCsr(m) as gm:
        Xg, it_g, hg, st = g.pcg_spai(gm, B, 3000, 1e-9, hist_cap=3000)
    assert st == 0 and it_g == it_o
    np.testing.assert_allclose(hg, ho[: len(hg)], rtol=0, atol=1e-10)
    assert np.linalg.norm(Xg - Xo) <= 1e-8 * np.linalg.norm(Xo)


# ---- imperfect FEM: mixed plans (k_spmv_blk's register fallback, per-chunk pair flags) ----------
def fem_with_long_rows(a, rows, length, seed=5):
    """`a` with the given rows replaced by `length` random sorted columns: rows longer than the snap
    distance (tile / 8) are split between tiles, so the plan carries (closed by the completing tiles) and those tiles are
    not node blocks."""
    rng = np.random.default_rng(seed)
    ro, ci, va = a.row_offsets, a.column_indices, a.values
    new_ro, new_ci, new_va = [0], [], []
    rows = set(rows)
    for i in range(a.num_rows):
        if i in rows:
            c = np.sort(rng.choice(a.num_cols, length, replace=False)).astype(np.int32)
            v = rng.uniform(0.5, 1.5, length)
        else:
            c, v = ci[ro[i]:ro[i + 1]], va[ro[i]:ro[i + 1]]
        new_ci.append(c)
        new_va.append(v)
        new_ro.append(new_ro[-1] + len(c))
    return mspmv.CsrMatrix.from_arrays(a.num_cols, np.array(new_ro, np.int32), np.concatenate(new_ci),
                                       np.concatenate(new_va))


def stack_rows(a, b):
    """Rows of a, then rows of b (same column count)."""
    ro = np.concatenate([a.row_offsets, a.row_offsets[-1] + b.row_offsets[1:]]).astype(np.int32)
    return mspmv.CsrMatrix.from_arrays(a.num_cols, ro, np.concatenate([a.column_indices, b.column_indices]),
                                       np.concatenate([a.values, b.values]))


def mixed_cases():
    base = lambda: mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3)  # noqa: E731
    return {
        "perturbed_small": lambda: mspmv.CsrMatrix.synth_fem_perturbed(21792, 1152443, 6, 170, 0.02, 0.01, seed=4),
        "perturbed_heavy": lambda: mspmv.CsrMatrix.synth_fem_perturbed(21792, 1152443, 6, 170, 0.2, 0.1, seed=5),
        "long_rows": lambda: fem_with_long_rows(base(), [100, 5000, 5001, 17000], 1500),
        # a stencil block beside the FEM rows: its tiles have no runs (the register fallback, G = 2)
        "fem_plus_stencil": lambda: stack_rows(base(), _stencil_rows(21792, 3000)),
    }


def _stencil_rows(ncols, m):
    """m rows of 7 nonzeros in a narrow band, num_cols = ncols."""
    rng = np.random.default_rng(9)
    ro = np.arange(0, 7 * m + 1, 7, dtype=np.int32)
    base = rng.integers(0, ncols - 40, m)
    ci = (base[:, None] + np.arange(0, 35, 5)[None, :]).astype(np.int32).reshape(-1)
    va = rng.uniform(0.5, 1.5, 7 * m)
    return mspmv.CsrMatrix.from_arrays(ncols, ro, ci, va)


@pytest.mark.parametrize("name", list(mixed_cases()))
def test_blocks_mixed_plan(orc, name):
    a = mixed_cases()[name]()
    x = np.random.default_rng(17).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        plan = g.tile_plan(1)
        nb = g.plan_block_tiles(1)
        y = g.spmv(x)
        y2 = g.spmv(x)
        kname = g.kernel_name()
        check_parity(a, y, orc.spmv_gold(a, x), x, plan, 1)
    assert y.tobytes() == y2.tobytes()
    assert kname.startswith("k_spmv_blk<0,"), kname
    assert np.all(plan["modes"] == 255)
    assert 0 < nb <= plan["num_tiles"]
    if name == "long_rows":
        assert plan["num_carries"] > 0


def test_blocks_perturbed_full_size(orc):
    """The bench's imperfect pwtk leg (m = 217,918; 2 % odd nodes, 1 % off-pattern rows) at full size."""
    a = mspmv.CsrMatrix.synth_fem_perturbed(217918, 11524432, 6, 1700, 0.02, 0.01, seed=11)
    x = np.random.default_rng(12).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        plan = g.tile_plan(1)
        y = g.spmv(x)
        kname = g.kernel_name()
        check_parity(a, y, orc.spmv_gold(a, x), x, plan, 1)
        nb = g.plan_block_tiles(1)
    assert kname.startswith("k_spmv_blk<0,"), kname
    assert nb >= 0.9 * plan["num_tiles"], (nb, plan["num_tiles"])


@pytest.mark.parametrize("name", ["perturbed_small", "long_rows"])
@pytest.mark.parametrize("L", [1, 8])
def test_blocks_mixed_plan_spmm(orc, name, L):
    """Mixed plans under the SpMM (k_spmm_blk when every tile is a register run tile, else the L-wide
    merge tiles) against the oracle's row-split SpMM."""
    from gpu_common import check_parity_chunked
    a = mixed_cases()[name]()
    X = np.random.default_rng(L).uniform(-1, 1, (a.num_cols, L))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity_chunked(a, g, Y, orc.csr_spmm_t(a, X), X, L)


@pytest.mark.parametrize("runs", ["0", "1", "auto"])
@pytest.mark.parametrize("name", ["regular", "perturbed_small", "perturbed_heavy"])
def test_blocks_run_plan(orc, monkeypatch, name, runs):
    """The run-balanced node-block plan (mspmv_api.hip spmv_runs_decide: tiles cut at run starts, <= 8
    run chunks each, so k_spmv_blk takes every tile in one round of its half-wave slots): automatic on
    every all-register node-block plan, off with MSPMV_SPMV_RUNS=0.  Parity against SpmvGold under the
    plan the product ran on, and the L = 16 node-block SpMM on it against OmpCsrSpmmT; bitwise repeats;
    its boundaries are row starts."""
    if runs == "auto":
        monkeypatch.delenv("MSPMV_SPMV_RUNS", raising=False)
    else:
        monkeypatch.setenv("MSPMV_SPMV_RUNS", runs)
    make = mixed_cases().get(name) or (lambda: mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3))
    a = make()
    x = np.random.default_rng(21).uniform(-1, 1, a.num_cols)
    X = np.random.default_rng(22).uniform(-1, 1, (a.num_cols, 16))
    with mspmv.GpuCsr(a) as g:
        plan = g.tile_plan(1)
        y = g.spmv(x)
        y2 = g.spmv(x)
        kname = g.kernel_name()
        check_parity(a, y, orc.spmv_gold(a, x), x, plan, 1)
        Y = g.spmm(X)
        check_parity(a, Y, orc.csr_spmm_t(a, X), X, g.tile_plan(16), 16)
        mname = g.spmm_kernel_name(16)
        assert g.tile_plan(16)["num_tiles"] == plan["num_tiles"] or name.startswith("perturbed") or runs == "0"
    assert y.tobytes() == y2.tobytes()
    assert kname.startswith("k_spmv_blk<0,"), kname
    b = plan["bounds"]
    on_rows = np.array_equal(a.row_offsets[b[:, 0]], b[:, 1])
    if runs != "0":  # automatic on every all-register node-block plan
        assert on_rows and plan["num_carries"] == 0
