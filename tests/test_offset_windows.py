"""Offset-window planning on the host (mspmv_offset_windows; csrc/mspmv_dia.hip dia_plan_host), no GPU:
the library's decision and per-window offset counts against a numpy restatement of the rules --
64-row windows, each window's offsets col - row taken as the union over its rows (sorted), every row's
columns strictly ascending, K <= 32, nonzeros >= min_window_fill x rows x K in each window and >=
min_fill x 64 x sum K overall; a window is masked when some row lacks one of its offsets or it holds
fewer than 64 rows.
"""
import numpy as np
import pytest

import mspmv
from test_gpu_dia import band


def restate(a, min_fill=0.85, min_window_fill=0.3, kmax=32):
    m = a.num_rows
    ro = a.row_offsets.astype(np.int64)
    ci = a.column_indices.astype(np.int64)
    if m == 0 or a.num_nonzeros == 0 or np.diff(ro).max() > kmax:
        return None
    ks, masked = [], 0
    for r0 in range(0, m, 64):
        r1 = min(m, r0 + 64)
        offs = []
        for r in range(r0, r1):
            o = ci[ro[r]:ro[r + 1]] - r
            if o.size > 1 and np.any(np.diff(o) <= 0):
                return None
            offs.append(o)
        D = np.unique(np.concatenate(offs)) if any(o.size for o in offs) else np.zeros(0, np.int64)
        K = D.size
        nz = int(ro[r1] - ro[r0])
        if K < 1 or K > kmax or nz < min_window_fill * (r1 - r0) * K:
            return None
        ks.append(K)
        masked += not (r1 - r0 == 64 and nz == 64 * K)
    if a.num_nonzeros < min_fill * 64 * sum(ks):
        return None
    return {"windows": len(ks), "sum_offsets": sum(ks), "masked_windows": masked, "k": np.array(ks)}


def unsorted_tridiag():
    t = band(64 * 10, [-1, 0, 1], 7)
    ci = t.column_indices.copy()
    ci[t.row_offsets[5]:t.row_offsets[6]] = ci[t.row_offsets[5]:t.row_offsets[6]][::-1]
    return mspmv.CsrMatrix.from_arrays(t.num_cols, t.row_offsets, ci, t.values)


CASES = {
    "stencil27": (lambda: mspmv.CsrMatrix.synth_stencil(1, 17 * 12 * 9, 17, 12, 9, seed=1), True),
    "fem2d": (lambda: mspmv.CsrMatrix.synth_stencil(0, 20003, 141), True),
    "tridiag": (lambda: band(64 * 50, [-1, 0, 1], 2), True),
    "partial": (lambda: band(64 * 7 + 13, [-70, -3, 0, 2, 9, 70], 3), True),
    "rect": (lambda: band(2000, [0, 5, 1700, 3000], 4, n=5001), True),
    "holes": (lambda: band(4000, [-200, -1, 0, 1, 200], 5, drop=0.3), False),   # fill 0.7 < 0.85
    "unsorted": (unsorted_tridiag, False),
    "fem_blocked": (lambda: mspmv.CsrMatrix.synth_fem_blocked(2400, 126000, 6, 60, seed=3), False),  # rows > 32
    "banded_random": (lambda: mspmv.CsrMatrix.synth_banded(3000, 3000 * 8, 400, seed=2), False),     # K > 32
}


@pytest.mark.parametrize("name", list(CASES))
def test_offset_windows_plan(name):
    make, fits = CASES[name]
    a = make()
    got = mspmv.offset_windows(a)
    want = restate(a)
    assert (got is not None) == fits == (want is not None), (name, got, want)
    if want is not None:
        assert got["windows"] == want["windows"]
        assert got["sum_offsets"] == want["sum_offsets"]
        assert got["masked_windows"] == want["masked_windows"]
        np.testing.assert_array_equal(got["k"], want["k"])


def test_offset_windows_thresholds():
    """Forced thresholds (MSPMV_DIA=1 plans at fill 0): windows with missing offsets and empty rows fit;
    a window whose nonzeros fall below min_window_fill does not."""
    a = CASES["holes"][0]()
    assert mspmv.offset_windows(a, 0.0, 0.0) is not None
    assert mspmv.offset_windows(a, 0.6, 0.3) is not None
    assert mspmv.offset_windows(a, 0.8, 0.3) is None
    e = band(3000, [0, 3], 6, drop=0.6)
    got, want = mspmv.offset_windows(e, 0.0, 0.0), restate(e, 0.0, 0.0)
    assert got is not None and got["masked_windows"] == want["masked_windows"] == got["windows"]
    assert mspmv.offset_windows(e, 0.0, 0.5) is None


def test_offset_windows_rejects_bad_input():
    t = band(200, [0, 1], 1)
    bad = mspmv.CsrMatrix.from_arrays(t.num_cols, t.row_offsets, t.column_indices.copy(), t.values)
    bad.column_indices[3] = t.num_cols + 5
    with pytest.raises(RuntimeError):
        mspmv.offset_windows(bad)
