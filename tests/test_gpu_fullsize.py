"""GPU parity at BASELINE.json's full configuration sizes (SURVEY 8(d) synthetic stand-ins for
the SuiteSparse matrices, which are not available offline), through the C-ABI.

* SpMV (configs[0..1]: cant, pwtk, rma10 shapes; the parabolic_fem and nlpkkt120 sizes of
  configs[3..4]) against the oracle's SpmvGold restatement (cpu_spmv.cpp:241-265): rows the
  kernel sums sequentially bit-identical, all others within 2 (len+1) eps (|A||x|)_i; merge
  coordinates at P = 256 bit-exact with MergePathSearch (cpu_spmv.cpp:208-235).
* SpMM, 16-column panel (configs[2]) on the cant and pwtk shapes against the row-split
  OmpCsrSpmmT (row_splitting.hpp:15-54), same bound.
* Single CG (configs[3], parabolic_fem shape, the cpu_singlecg tol = 1e-5 ||b|| quirk) against
  the oracle's CGSolveSingle, within the reference's own thread-count envelope (see the test).
* Multi CG (configs[4], nlpkkt120 size, L = 8): the whole solve against the oracle's
  CGSolveMultiple run with NONZERO_SPLIT as cpu_multicg.cpp:202 runs it (history within 1e-10
  wherever the reference reproduces itself across thread counts, X within 1e-8 relative), plus
  a size-independent property: every column's true residual ||b_j - A x_j|| / ||b_j|| below the
  threshold the solve stopped on.
"""
import numpy as np
import pytest

import mspmv
from gpu_common import check_parity

pytestmark = pytest.mark.gpu

PWTK = dict(m=217918, nnz=11524432, block=6, half_band_nodes=1700)   # bench.py's pwtk shape


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


def full_cases():
    return {
        "cant": lambda: mspmv.CsrMatrix.synth_banded(62451, 4007383, 2000, seed=1),
        "pwtk": lambda: mspmv.CsrMatrix.synth_fem_blocked(PWTK["m"], PWTK["nnz"], PWTK["block"],
                                                          PWTK["half_band_nodes"], seed=1),
        "rma10": lambda: mspmv.CsrMatrix.synth_banded(46835, 2374001, 3000, seed=2),
        "parabolic_fem": lambda: mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4),
        "nlpkkt120": lambda: mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2),
    }


@pytest.mark.parametrize("name", list(full_cases()))
def test_spmv_full_size(orc, name):
    a = full_cases()[name]()
    x = np.random.default_rng(11).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(x)
        check_parity(a, y, orc.spmv_gold(a, x), x, g.tile_plan(1), 1)
        np.testing.assert_array_equal(g.merge_coords(256), orc.merge_coords(a, 256))


@pytest.mark.parametrize("name", ["cant", "pwtk"])
def test_spmm16_full_size(orc, name):
    a = full_cases()[name]()
    X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, 16))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity(a, Y, orc.csr_spmm_t(a, X), X, g.tile_plan(16), 16)


def test_cg_single_full_size(orc):
    """At this size (447 iterations, diag shift 1e-4) the reference's CG does not reproduce
    itself to 1e-10: its OpenMP dot order depends on the thread count, and the oracle at 1 vs
    8 threads already differs by > 1e-10 from iteration ~115 on and by ~1.3e-3 (1.8 %) at the
    end (measured in the build container).  The bar here is therefore the reference's own
    run-to-run envelope: the GPU history within 4x the oracle(1 thread) vs oracle(8 threads)
    difference at every iteration prefix, iterations within one, and the final true residual of
    the same order as the oracle's.  The 1e-10 match itself is tested where the reference does
    reproduce itself (test_gpu_cg.py, up to ~700 iterations on smaller grids)."""
    a = full_cases()["parabolic_fem"]()
    b = orc.glibc_rand(42, a.num_rows)
    tol = orc.calculate_threshold(b, a.num_rows, 1e-5)   # cpu_singlecg.cpp:22-34 quirk
    # The envelope is sampled over several thread counts: OpenMP's reduction combine order (and so
    # the reference's own history) also varies from run to run at a fixed count, so a single
    # 1-vs-8 pair under-samples it (one such pair left 37 of 447 iterations just outside 4x).
    hist, n0 = {}, orc.lib.orc_max_threads()
    try:
        for t in (1, 2, 4, 8, 16):
            orc.lib.orc_set_threads(t)
            hist[t] = orc.cg_single(a, b, 10000, tol, hist_cap=10000)
    finally:
        orc.lib.orc_set_threads(n0)
    xo, it_o, ho = hist[8]
    with mspmv.GpuCsr(a) as g:
        xg, it_g, hg, st = g.cg_single(b, 10000, tol, hist_cap=10000)
    assert st == 0 and it_o < 10000
    assert abs(it_g - it_o) <= 1 and all(abs(h[1] - it_o) <= 1 for h in hist.values()), (it_g, it_o)
    k = min([len(hg)] + [len(h[2]) for h in hist.values()])
    spread = np.max([np.abs(h[2][:k] - ho[:k]) for h in hist.values()], axis=0)
    env = np.maximum.accumulate(spread)   # the reference's own spread so far
    dev = np.abs(hg[:k] - ho[:k])
    np.testing.assert_array_less(dev, 4 * env + 1e-10)
    res = [np.linalg.norm(b - orc.spmv_gold(a, x)) / np.linalg.norm(b) for x in (xg, xo)]
    assert res[0] <= max(10 * res[1], tol), res


def test_cg_multi_full_size(orc):
    """configs[4] at its full size, compared over the WHOLE solve against the oracle run as
    cpu_multicg runs it: SpmmKernel NONZERO_SPLIT (cpu_multicg.cpp:202) with the partition and
    OpenMP reductions of T threads (g_omp_threads).  The reference's rounding depends on T, so the
    oracle is run at two thread counts first: on the prefix where those two agree to 1e-10 (the
    reference reproduces itself there) the GPU history must match to 1e-10 too; past it (if any)
    it must stay within 4x the oracle's own spread.  Iterations within one, every column's X
    within 1e-8 relative of the oracle's where the prefix covers the whole solve, and every
    column's true residual below the threshold the solve stopped on."""
    a = full_cases()["nlpkkt120"]()
    n, L = a.num_rows, 8
    B = np.random.default_rng(42).uniform(0, 1, (n, L))
    thr = orc.calculate_threshold(B.reshape(-1), n, 1e-5)   # cpu_multicg.cpp:168 quirk
    runs, t0 = {}, orc.lib.orc_max_threads()
    try:
        for t in sorted({max(2, min(8, t0)), max(2, t0)} | {4}):
            orc.lib.orc_set_threads(t)
            runs[t] = orc.cg_multi(a, B, 50000, thr, kernel=mspmv.NONZERO_SPLIT, P=t, hist_cap=50000)
    finally:
        orc.lib.orc_set_threads(t0)
    ts = sorted(runs)
    Xo, it_o, ho = runs[ts[-1]]
    assert 3 < it_o < 50000
    k = min(len(r[2]) for r in runs.values())
    spread = np.max([np.abs(runs[t][2][:k] - ho[:k]) for t in ts[:-1]], axis=0)
    agree = int(np.argmax(spread > 1e-10)) if np.any(spread > 1e-10) else k   # reproducible prefix
    with mspmv.GpuCsr(a) as g:
        Xg, it_g, hg, st = g.cg_multi(B, 50000, thr, kernel=mspmv.NONZERO_SPLIT, hist_cap=50000)
    assert st == 0 and abs(it_g - it_o) <= 1, (it_g, it_o)
    k = min(k, len(hg))
    np.testing.assert_allclose(hg[:agree], ho[:agree], rtol=0, atol=1e-10)
    env = np.maximum.accumulate(spread[:k])
    np.testing.assert_array_less(np.abs(hg[:k] - ho[:k]), 4 * env + 1e-10)
    if agree >= min(it_g, it_o):
        assert it_g == it_o
        for j in range(L):
            assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j]), j
    assert hg[-1] < thr <= hg[-2]
    R = B - orc.csr_spmm_t(a, Xg)
    rel = np.linalg.norm(R, axis=0) / np.linalg.norm(B, axis=0)
    assert np.all(rel < thr), rel
