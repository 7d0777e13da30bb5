"""GPU parity at BASELINE.json's full configuration sizes (SURVEY 8(d) synthetic stand-ins for
the SuiteSparse matrices, which are not available offline), through the C-ABI.

* SpMV (configs[0..1]: cant, pwtk, rma10 shapes; the parabolic_fem and nlpkkt120 sizes of
  configs[3..4]; the power-law variant at pwtk size) against the oracle's SpmvGold restatement (cpu_spmv.cpp:241-265): rows the
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
        # SURVEY 8(d)'s skewed variant, bench.py's spmv_shapes power-law leg (the sliced-ELL SpMV)
        "powerlaw": lambda: mspmv.CsrMatrix.synth_powerlaw(PWTK["m"], PWTK["m"], PWTK["nnz"], 1.2, 3),
        # bench.py's window_shapes legs (round 6): the nlpkkt120-size stencil with off-pattern columns (the
        # windows plus a remainder) and the KKT saddle point of nlpkkt120's block structure (34 offsets)
        "stencil27_perturbed": lambda: mspmv.CsrMatrix.synth_stencil_perturbed(
            (160, 135, 164), seed=5, diag_shift=1e-2, extra_frac=0.01, long_frac=0.001),
        "kkt": lambda: mspmv.CsrMatrix.synth_kkt((120, 120, 123), seed=6, eps=1e-2),
    }


@pytest.mark.parametrize("name", list(full_cases()))
def test_spmv_full_size(orc, name):
    a = full_cases()[name]()
    x = np.random.default_rng(11).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        y = g.spmv(x)
        check_parity(a, y, orc.spmv_gold(a, x), x, g.tile_plan(1), 1)
        np.testing.assert_array_equal(g.merge_coords(256), orc.merge_coords(a, 256))
        if name == "powerlaw":
            assert g.kernel_name().startswith("k_spmv_sell<"), g.kernel_name()
            assert y.tobytes() == g.spmv(x).tobytes()  # fixed order: repeats bit-identical
        if name in ("stencil27_perturbed", "kkt"):  # both on the offset windows
            assert g.kernel_name().startswith("k_spmm_dia<1,"), g.kernel_name()
            assert y.tobytes() == g.spmv(x).tobytes()


@pytest.mark.parametrize("name", ["cant", "pwtk"])
def test_spmm16_full_size(orc, name):
    a = full_cases()[name]()
    X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, 16))
    with mspmv.GpuCsr(a) as g:
        Y = g.spmm(X)
        check_parity(a, Y, orc.csr_spmm_t(a, X), X, g.tile_plan(16), 16)


_SINGLE_ORACLE = {}


@pytest.mark.parametrize("form", ["classic", "single_reduction"])
def test_cg_single_full_size(orc, form, monkeypatch):
    """At this size (447 iterations, diag shift 1e-4) the reference's CG does not reproduce
    itself to 1e-10: its OpenMP dot order depends on the thread count, and the oracle at 1 vs
    8 threads already differs by > 1e-10 from iteration ~115 on and by ~1.3e-3 (1.8 %) at the
    end (measured in the build container).  The bar here is therefore the reference's own
    run-to-run envelope: the GPU history within 4x the oracle(1 thread) vs oracle(8 threads)
    difference at every iteration prefix, iterations within one, and the final true residual of
    the same order as the oracle's.  The 1e-10 match itself is tested where the reference does
    reproduce itself (test_gpu_cg.py, up to ~700 iterations on smaller grids).  Both iteration forms
    of the register-resident kernel (MSPMV_CG_RESIDENT_FORM) are held to it."""
    a = full_cases()["parabolic_fem"]()
    b = orc.glibc_rand(42, a.num_rows)
    tol = orc.calculate_threshold(b, a.num_rows, 1e-5)   # cpu_singlecg.cpp:22-34 quirk
    # The envelope is sampled over several thread counts: OpenMP's reduction combine order (and so
    # the reference's own history) also varies from run to run at a fixed count, so a single
    # 1-vs-8 pair under-samples it (one such pair left 37 of 447 iterations just outside 4x).
    if not _SINGLE_ORACLE:
        n0 = orc.lib.orc_max_threads()
        try:
            for t in (1, 2, 4, 8, 16):
                orc.lib.orc_set_threads(t)
                _SINGLE_ORACLE[t] = orc.cg_single(a, b, 10000, tol, hist_cap=10000)
        finally:
            orc.lib.orc_set_threads(n0)
    hist = _SINGLE_ORACLE
    xo, it_o, ho = hist[8]
    monkeypatch.setenv("MSPMV_CG_RESIDENT_FORM", form)
    with mspmv.GpuCsr(a) as g:
        xg, it_g, hg, st = g.cg_single(b, 10000, tol, hist_cap=10000)
        assert g.cg_kernel_name().startswith("k_cg_resident<3,7," + form), g.cg_kernel_name()
    assert st == 0 and it_o < 10000
    assert abs(it_g - it_o) <= 1 and all(abs(h[1] - it_o) <= 1 for h in hist.values()), (it_g, it_o)
    k = min([len(hg)] + [len(h[2]) for h in hist.values()])
    spread = np.max([np.abs(h[2][:k] - ho[:k]) for h in hist.values()], axis=0)
    env = np.maximum.accumulate(spread)   # the reference's own spread so far
    dev = np.abs(hg[:k] - ho[:k])
    np.testing.assert_array_less(dev, 4 * env + 1e-10)
    res = [np.linalg.norm(b - orc.spmv_gold(a, x)) / np.linalg.norm(b) for x in (xg, xo)]
    assert res[0] <= max(10 * res[1], tol), res


_MULTI_ORACLE = {}


def multi_oracle(orc):
    """configs[4]'s oracle runs, computed once per session: the nlpkkt120-size matrix, its 8-column
    RHS and threshold, and CGSolveMultiple run as cpu_multicg runs it (NONZERO_SPLIT,
    cpu_multicg.cpp:202) at two or three OpenMP thread counts (the reference's rounding depends on
    the count).  Returns (a, B, thr, runs, ho, Xo, it_o, spread, agree): `agree` is the prefix where
    the thread counts agree to 1e-10 (the reference reproduces itself there), `spread` their
    per-iteration disagreement."""
    if not _MULTI_ORACLE:
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
        k = min(len(r[2]) for r in runs.values())
        spread = np.max([np.abs(runs[t][2][:k] - ho[:k]) for t in ts[:-1]], axis=0)
        agree = int(np.argmax(spread > 1e-10)) if np.any(spread > 1e-10) else k
        _MULTI_ORACLE.update(a=a, B=B, thr=thr, ho=ho, Xo=Xo, it_o=it_o, spread=spread, agree=agree)
    return _MULTI_ORACLE


def check_multi_full(orc, Xg, it_g, hg, st):
    """test_cg_multi_full_size's bars for a configs[4] solve (Xg, it_g, hg, st)."""
    o = multi_oracle(orc)
    a, B, thr, ho, Xo, it_o, spread, agree = (o[k] for k in ("a", "B", "thr", "ho", "Xo", "it_o", "spread", "agree"))
    assert 3 < it_o < 50000
    assert st == 0 and abs(it_g - it_o) <= 1, (it_g, it_o)
    k = min(len(spread), len(hg))
    np.testing.assert_allclose(hg[:agree], ho[:agree], rtol=0, atol=1e-10)
    env = np.maximum.accumulate(spread[:k])
    np.testing.assert_array_less(np.abs(hg[:k] - ho[:k]), 4 * env + 1e-10)
    if agree >= min(it_g, it_o):
        assert it_g == it_o
        for j in range(B.shape[1]):
            assert np.linalg.norm(Xg[:, j] - Xo[:, j]) <= 1e-8 * np.linalg.norm(Xo[:, j]), j
    assert hg[-1] < thr <= hg[-2]
    R = B - orc.csr_spmm_t(a, Xg)
    rel = np.linalg.norm(R, axis=0) / np.linalg.norm(B, axis=0)
    assert np.all(rel < thr), rel


def test_cg_multi_full_size(orc):
    """configs[4] at its full size, compared over the WHOLE solve against the oracle run as
    cpu_multicg runs it: SpmmKernel NONZERO_SPLIT (cpu_multicg.cpp:202) with the partition and
    OpenMP reductions of T threads (g_omp_threads).  The reference's rounding depends on T, so the
    oracle is run at two thread counts first: on the prefix where those two agree to 1e-10 (the
    reference reproduces itself there) the GPU history must match to 1e-10 too; past it (if any)
    it must stay within 4x the oracle's own spread.  Iterations within one, every column's X
    within 1e-8 relative of the oracle's where the prefix covers the whole solve, and every
    column's true residual below the threshold the solve stopped on."""
    o = multi_oracle(orc)
    with mspmv.GpuCsr(o["a"]) as g:
        Xg, it_g, hg, st = g.cg_multi(o["B"], 50000, o["thr"], kernel=mspmv.NONZERO_SPLIT, hist_cap=50000)
    check_multi_full(orc, Xg, it_g, hg, st)


_DIST_FULL_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import mspmv
a = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2)
n, L = a.num_rows, 8
B = np.random.default_rng(42).uniform(0, 1, (n, L))
thr = float(sys.argv[4])
rb = mspmv.dist_partition(a, 1)
d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))
dB, dX = mspmv.DeviceBuffer.from_array(B), mspmv.DeviceBuffer(8 * n * L)
it, hist, st = d.cg_dev(dB, dX, L, 50000, thr, hist_cap=50000)
np.save(sys.argv[3] + "/X.npy", dX.download((n, L)))
np.save(sys.argv[3] + "/h.npy", hist)
np.save(sys.argv[3] + "/m.npy", np.array([it, st]))
d.close()
print("DIST FULL OK")
"""


@pytest.mark.parametrize("graph", ["0", "1"])
def test_dist_cg_multi_full_size(tmp_path, orc, graph):
    """configs[4]'s sharded path at its full size on one GPU: the nlpkkt120-size L = 8 solve through
    DistCsr (mspmv_dist_cg_dev: RCCL communicator, request exchange, pack, both all-reduces) at world
    1 with the overlapped iteration forced (MSPMV_DIST_FORCE_SPLIT=1: head | interior | tail, the
    interior's dot-mode SpMM on its own stream), batches eager and replayed from a captured hipGraph --
    the code an 8-GPU run executes first, held to test_cg_multi_full_size's bars."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    o = multi_oracle(orc)
    env = dict(os.environ, MSPMV_DIST_FORCE_SPLIT="1", MSPMV_DIST_GRAPH=graph)
    r = subprocess.run([sys.executable, "-c", _DIST_FULL_CHILD, os.path.join(root, "sparse-matrix-linear-equations_amd"),
                        os.path.join(root, "tests"), str(tmp_path), repr(o["thr"])], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0 and "DIST FULL OK" in r.stdout, r.stdout + r.stderr[-3000:]
    it, st = (int(v) for v in np.load(tmp_path / "m.npy"))
    check_multi_full(orc, np.load(tmp_path / "X.npy"), it, np.load(tmp_path / "h.npy"), st)
