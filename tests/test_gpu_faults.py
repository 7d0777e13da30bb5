"""GPU: the fold tickets' overrun guard (ticket_arrive, csrc/mspmv_device.h) and the round-5 failure
it explains.

Round 5 recorded one sharded CG at L = 3 on the offset windows' dot mode running 70 iterations
against the oracle's 43 (profiles/r05at_gpu_tests_flaky.txt).  The fold tickets of a fresh object were
zeroed by a null-stream memset that was not ordered before the folds on the object's non-blocking
stream (fixed in a46d710), so the first folds could meet recycled, non-zero tickets.  These tests make
that state deterministic through the test hook (mspmv_test_poison_tickets /
mspmv_dist_test_poison_tickets: the next solve's tickets start at a chosen value, optionally zeroed
again after the first iteration -- the late memset) and check:

* the guard: a ticket that draws past its group raises the fault word and the solve returns
  MSPMV_ERR_FAULT (single GPU and sharded), and the next solve on the same object is clean again;
* the mechanism: with the guard told not to stop, dirty tickets at the first folds alone turn the
  oracle's iteration count into another one -- the silent wrong result round 5 saw.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

L3_TOL, L3_ITERS = 1e-9, 3000


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


def _stencil():
    import mspmv
    return mspmv.CsrMatrix.synth_stencil(1, 16 * 17 * 18, 16, 17, 18)


def _dist(a):
    import mspmv
    rb = mspmv.dist_partition(a, 1)
    return mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))


def _check_clean(orc, a, B, it, hist, X):
    Xo, it_o, ho = orc.cg_multi(a, B, L3_ITERS, L3_TOL, kernel=1, P=8, hist_cap=L3_ITERS)
    assert abs(it - it_o) <= 1, (it, it_o)
    k = min(len(hist), len(ho))
    np.testing.assert_allclose(hist[:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(X - Xo) <= 1e-8 * np.linalg.norm(Xo)
    return it_o


@pytest.mark.parametrize("plan", ["tiles", "windows"])
@pytest.mark.parametrize("value", [32, 0x7FFFFFFF, 0xFFFFFFFF])
def test_poisoned_tickets_single_gpu(orc, monkeypatch, plan, value):
    """mspmv_dcg_multi (L = 8, the split iteration: p update, SpMM, p.Ap fold, update) with every fold
    ticket at `value` when the solve starts.  32 and 2^31 - 1: no arrival of a group (<= 32 arrivals)
    draws its last value, so no fold runs and the consumer would read a stale total; 2^32 - 1: the
    first arrival draws it and the counter wraps, so a later arrival folds early.  Each time an
    arrival draws past its group, and the solve stops with MSPMV_ERR_FAULT.  The next solve on the
    handle starts from re-zeroed tickets and matches the oracle."""
    import mspmv
    if plan == "windows":
        monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = _stencil()
    B = np.random.default_rng(8).uniform(0, 1, (a.num_rows, 8))
    with mspmv.GpuCsr(a, device=0) as g:
        g.test_poison_tickets(value, mspmv.POISON_FILL)
        with pytest.raises(mspmv.MspmvError) as ei:
            g.cg_multi(B, L3_ITERS, L3_TOL, hist_cap=L3_ITERS)
        assert ei.value.status == mspmv.FAULT
        X, it, hist, st = g.cg_multi(B, L3_ITERS, L3_TOL, hist_cap=L3_ITERS)
        assert st == 0
        _check_clean(orc, a, B, it, hist, X)


@pytest.mark.parametrize("value", [32, 0x7FFFFFFF])
def test_poisoned_tickets_dist(orc, monkeypatch, value):
    """The sharded CG (world 1, the offset windows' dot mode, L = 3: column groups of 2 and 1 -- the
    round-5 case) with dirty fold tickets: every rank stops at the same batch on the all-reduced fault
    word and returns MSPMV_ERR_FAULT; the next solve on the object is clean."""
    import mspmv
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = _stencil()
    d = _dist(a)
    B = np.random.default_rng(3).uniform(0, 1, (a.num_rows, 3))
    dB = mspmv.DeviceBuffer.from_array(B)
    dX = mspmv.DeviceBuffer(8 * a.num_rows * 3)
    d.test_poison_tickets(value, mspmv.POISON_FILL)
    with pytest.raises(mspmv.MspmvError) as ei:
        d.cg_dev(dB, dX, 3, L3_ITERS, L3_TOL, hist_cap=L3_ITERS)
    assert ei.value.status == mspmv.FAULT
    it, hist, st = d.cg_dev(dB, dX, 3, L3_ITERS, L3_TOL, hist_cap=L3_ITERS)
    assert st == 0
    _check_clean(orc, a, B, it, hist, dX.download((a.num_rows, 3)))
    d.close()


@pytest.mark.parametrize("value", [32, 0x7FFFFFFF])
def test_dirty_tickets_mechanism(orc, monkeypatch, value, capsys):
    """Round 5's failure, made deterministic: the sharded CG at L = 3 on the windows with its fold
    tickets dirty for the FIRST iteration only (filled after the init, zeroed right after the first
    iteration is enqueued -- the unordered memset landing late) and the guard recording instead of
    stopping.  No fold of that iteration completes, so its alpha comes from a stale p.Ap and its stop
    test and beta from a stale r.r (the init's b.b); CG loses conjugacy and recovers slowly, running to
    its own stop test with a wrong iteration count or history -- and the fault word reports it."""
    import mspmv
    monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = _stencil()
    d = _dist(a)
    B = np.random.default_rng(3).uniform(0, 1, (a.num_rows, 3))
    dB = mspmv.DeviceBuffer.from_array(B)
    dX = mspmv.DeviceBuffer(8 * a.num_rows * 3)
    d.test_poison_tickets(value, mspmv.POISON_FILL | mspmv.POISON_LATE_ZERO | mspmv.POISON_NO_STOP)
    it, hist, st = d.cg_dev(dB, dX, 3, L3_ITERS, L3_TOL, hist_cap=L3_ITERS, allow_fault=True)
    assert st == mspmv.FAULT
    Xo, it_o, ho = orc.cg_multi(a, B, L3_ITERS, L3_TOL, kernel=1, P=8, hist_cap=L3_ITERS)
    k = min(len(hist), len(ho))
    dev = float(np.max(np.abs(hist[:k] - ho[:k]))) if k else float("inf")
    with capsys.disabled():
        print(f"\n[mechanism] poison {value:#x}: {it} iterations vs the oracle's {it_o}, "
              f"max history deviation {dev:.3e}")
    assert it != it_o or dev > 1e-10
    d.close()


_PIPE_FAULT_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import mspmv
from test_gpu_cg import big_window_case
a = big_window_case()
b = np.random.default_rng(5).uniform(-1, 1, a.num_rows)
with mspmv.GpuCsr(a) as g:
    g.test_poison_tickets(int(sys.argv[4]), mspmv.POISON_FILL)
    try:
        g.cg_single(b, 150, 1e-30, hist_cap=150)
        status = 0
    except mspmv.MspmvError as e:
        status = e.status
    kern = g.cg_kernel_name()
    x, it, h, st = g.cg_single(b, 150, 1e-30, hist_cap=150)
np.savez(sys.argv[3], status=status, x=x, it=it, h=h, st=st, kern=np.array(kern))
"""


@pytest.mark.parametrize("value", [32, 0x7FFFFFFF])
def test_poisoned_tickets_pipelined_windows(orc, tmp_path, value):
    """The pipelined single-RHS CG on the offset windows past the consumer limit (1.1 M rows: 4,297 window
    workgroups, so k_cg1_dia folds its p.Ap partials one level by group tickets before k_cg1_update sums
    them) with every fold ticket dirty: MSPMV_ERR_FAULT, then a clean solve equal to the oracle's.  In a child
    process (MSPMV_CG_RESIDENT=0 and MSPMV_DIA=1 read fresh)."""
    import os
    import subprocess
    import sys
    import mspmv
    from test_gpu_cg import big_window_case, iter_match
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "f.npz")
    e = dict(os.environ, MSPMV_CG_RESIDENT="0", MSPMV_DIA="1")
    r = subprocess.run([sys.executable, "-c", _PIPE_FAULT_CHILD, os.path.join(root, "sparse-matrix-linear-equations_amd"),
                        os.path.join(root, "tests"), out, str(value)], env=e, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = np.load(out)
    assert "k_cg1_dia" in str(d["kern"]), str(d["kern"])
    assert int(d["status"]) == mspmv.FAULT
    a = big_window_case()
    b = np.random.default_rng(5).uniform(-1, 1, a.num_rows)
    xo, it_o, ho = orc.cg_single(a, b, 150, 1e-30, hist_cap=150)
    assert int(d["st"]) == 0 and iter_match(int(d["it"]), it_o, ho, 1e-30)
    k = min(len(d["h"]), len(ho))
    np.testing.assert_allclose(d["h"][:k], ho[:k], rtol=0, atol=1e-10)
    assert np.linalg.norm(d["x"] - xo) <= 1e-8 * np.linalg.norm(xo)
