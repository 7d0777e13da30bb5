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
a Kronecker FEM matrix solved by the pipelined single-RHS CG (blocks in the fused CG SpMV), and
the full pwtk shape."""
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


def cases():
    return {
        "pwtk_small": lambda: mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3),
        "kron6": lambda: kron_fem(60, 50, 6),
        "kron3": lambda: kron_fem(90, 80, 3),
        "kron12_wide": lambda: kron_fem(30, 30, 12),     # 60 columns per row: one chunk
        "kron16_wider": lambda: kron_fem(25, 20, 16),    # 80 columns per row: two chunks
        "kron10_empty": lambda: kron_fem(50, 40, 10, empty_every=7),
        "wide_runs": lambda: mspmv.CsrMatrix.synth_fem_blocked(12000, 1320000, 12, 60, seed=4),  # runs of 12 > 8
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


@pytest.mark.parametrize("name", list(cases()))
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


def test_blocks_not_taken_without_shared_columns():
    """Stencils and random bands have no two rows with one column list: striped staging."""
    for a in (mspmv.CsrMatrix.synth_stencil(0, 10007, 101), mspmv.CsrMatrix.synth_banded(6000, 380000, 2000, seed=1)):
        with mspmv.GpuCsr(a) as g:
            assert g.plan_block_tiles(1) == 0


def test_blocks_in_pipelined_cg(orc):
    """The fused CG SpMV (MODE 1: p = r + beta p_old gathered as {r, p} pairs) stages node blocks
    too; the solve must match the oracle's CGSolveSingle as every single-RHS CG does."""
    a = kron_fem(60, 50, 6)
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
