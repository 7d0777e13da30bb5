"""Rows split between tiles, closed inside the tile kernels (close_split_rows, mspmv_kernels.hip).

A row longer than the snap distance spans consecutive tiles: the tiles ending inside it store carries,
the tile where it ends stores the row's own part, and whichever of them finishes last adds the carries in
tile order (one ticket per row; no fix-up launch).  Checked here against the oracle (cpu_spmv.cpp
SpmvGold / the row-split SpMM, within the reordering bound of gpu_common.check_parity), for
bit-identical repeats (the tickets reset themselves every launch and the closing order is fixed
whichever tile closes), under a CU limit (fewer resident workgroups, so another tile tends to finish
last), and through the CG paths whose Ap products split rows.
"""
import numpy as np
import pytest

import mspmv
from gpu_common import check_parity, check_parity_chunked

pytestmark = pytest.mark.gpu


def hub_matrix(m=200000, short=12, hubs=((7, 180000), (120000, 60000)), long_rows=40, long_len=9000, seed=3):
    """m x m: rows of `short` random columns, two hub rows (the first spans ~90 tiles of the default
    plan) and `long_rows` rows of `long_len` columns -- split rows everywhere, including across the XCD
    ranges of the tile mapping."""
    rng = np.random.default_rng(seed)
    lens = np.full(m, short, np.int64)
    special = {int(r): long_len for r in rng.choice(m, long_rows, replace=False)}
    special.update({r: n for r, n in hubs})
    for r, n in special.items():
        lens[r] = n
    ro = np.zeros(m + 1, np.int64)
    ro[1:] = np.cumsum(lens)
    ci = np.empty(int(ro[-1]), np.int32)
    base = np.sort(rng.integers(0, m, (m, short)), axis=1).astype(np.int32)
    plain = lens == short
    starts = ro[:-1][plain]
    ci[(starts[:, None] + np.arange(short)[None, :]).ravel()] = base[plain].ravel()
    for r, n in special.items():
        ci[ro[r]:ro[r + 1]] = np.sort(rng.choice(m, n, replace=False))
    va = rng.uniform(-1.0, 1.0, ci.size)
    return mspmv.CsrMatrix.from_arrays(m, ro.astype(np.int32), ci, va)


@pytest.fixture(scope="module")
def hub():
    return hub_matrix()


def test_split_rows_spmv(orc, hub):
    a = hub
    x = np.random.default_rng(1).uniform(-1, 1, a.num_cols)
    gold = orc.spmv_gold(a, x)
    with mspmv.GpuCsr(a) as g:
        plan = g.tile_plan(1)
        assert plan["num_carries"] > 200, plan["num_carries"]
        ys = [g.spmv(x) for _ in range(3)]
        check_parity(a, ys[0], gold, x, plan, 1)
        # fewer resident workgroups: other tiles finish last.  (The single-RHS plan is rebuilt for the
        # CU count -- its tiles are stretched to whole generations of resident workgroups -- so its
        # sums are compared with each other and with the oracle, not with the full-device bits.)
        g.set_cu_limit(16)
        yl = [g.spmv(x) for _ in range(2)]
        check_parity(a, yl[0], gold, x, g.tile_plan(1), 1)
        g.set_cu_limit(0)
        ys.append(g.spmv(x))
    for y in ys[1:]:
        assert y.tobytes() == ys[0].tobytes()
    assert yl[1].tobytes() == yl[0].tobytes()


@pytest.mark.parametrize("L", [2, 4, 8, 16])
def test_split_rows_spmm(orc, hub, L):
    a = hub
    X = np.random.default_rng(L).uniform(-1, 1, (a.num_cols, L))
    ref = orc.csr_spmm_t(a, X)
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        Y2 = g.spmm(X)
        check_parity_chunked(a, g, Y, ref, X, L)
        g.set_cu_limit(8)  # (L = 2 shares the single-RHS plan, rebuilt for the CU count: see above)
        Y3 = g.spmm(X)
        Y4 = g.spmm(X)
        check_parity_chunked(a, g, Y3, ref, X, L)
        g.set_cu_limit(0)
    assert Y.tobytes() == Y2.tobytes()
    assert Y3.tobytes() == Y4.tobytes()


def test_split_rows_one_wave_plan(orc):
    """The skewed-rows plan (one-wave tiles) splits its hub rows over hundreds of tiles."""
    a = mspmv.CsrMatrix.synth_powerlaw(60000, 60000, 2400000, exponent=1.2, seed=3)
    x = np.random.default_rng(2).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(x)
        y2 = g.spmv(x)
        plan = g.tile_plan(1)
        check_parity(a, y, orc.spmv_gold(a, x), x, plan, 1)
    assert y.tobytes() == y2.tobytes()


def spd_with_long_rows(m=20000, seed=4):
    """SPD (diagonally dominant, symmetric) with a few dense-ish rows/columns: the CG's Ap splits rows."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for i in range(m):
        for d in (1, 2, 7):
            if i + d < m:
                rows.append(i)
                cols.append(i + d)
    for h in (5, 9000, 15000):
        others = rng.choice(m, 6000, replace=False)
        others = others[others != h]
        rows += [h] * others.size
        cols += others.tolist()
    r = np.array(rows)
    c = np.array(cols)
    v = rng.uniform(-0.5, 0.5, r.size)
    i = np.concatenate([r, c, np.arange(m)])
    j = np.concatenate([c, r, np.arange(m)])
    w = np.concatenate([v, v, np.zeros(m)])
    import scipy.sparse as sp
    A = sp.csr_matrix((w, (i, j)), shape=(m, m))
    A.sum_duplicates()
    absrow = np.asarray(abs(A).sum(axis=1)).ravel()
    A = A + sp.diags(absrow + 1.0)
    A = sp.csr_matrix(A)
    A.sort_indices()
    return mspmv.CsrMatrix.from_arrays(m, A.indptr.astype(np.int32), A.indices.astype(np.int32), A.data)


@pytest.mark.parametrize("L", [1, 4])
def test_split_rows_cg(orc, L):
    """L = 1 under a CU limit: the pipelined CG (k_spmv_tile MODE 1 closes Ap's split rows); L = 4: the
    split iteration (plain SpMM, then the p.Ap pass)."""
    a = spd_with_long_rows()
    B = np.random.default_rng(6).uniform(-1, 1, (a.num_rows, L))
    with mspmv.GpuCsr(a) as g:
        assert g.tile_plan(1)["num_carries"] > 0
        if L == 1:
            g.set_cu_limit(128)
            x, it, _, st = g.cg_single(B[:, 0], 500, 1e-10)
            X = x[:, None]
        else:
            X, it, _, st = g.cg_multi(B, 500, 1e-10)
    assert st == 0 and it < 500
    R = B - np.column_stack([orc.spmv_gold(a, np.ascontiguousarray(X[:, j])) for j in range(L)])
    rel = np.linalg.norm(R, axis=0) / np.linalg.norm(B, axis=0)
    assert np.all(rel < 1e-8), rel
