"""Offset-window planning on the host (mspmv_offset_windows; csrc/mspmv_dia.hip dia_plan_host), no GPU:
the library's decision, per-window offset counts and remainder against a numpy restatement of the rules
(round 6, windows plus a remainder) -- 64-row windows; every row's columns strictly ascending; first
every window keeping its whole offset list with no remainder (the exact plan), else a window keeps the
offsets col - row that >= min(8, its rows) of its rows hold, the 64 most frequent (ties: the
smaller offset), and drops its rarest kept offsets while they fill < min_window_fill of rows x K; every
other entry is remainder; the plan holds when sum K > 0, the kept entries fill >= min_fill x 64 x sum K
and the remainder is <= 5 % of the nonzeros (any share when min_fill is 0); a window is masked when some
row lacks one of its kept offsets or it holds fewer than 64 rows.
"""
import numpy as np
import pytest

import mspmv
from test_gpu_dia import band


def restate(a, min_fill=0.85, min_window_fill=0.3, kmax=64, keep_rows=8, max_rem=0.05):
    """Two passes, as dia_plan_host: every window's whole offset list (no remainder allowed), then the
    frequency rule with the remainder."""
    if min_fill <= 0:
        max_rem = 1.0
    return (restate_pass(a, min_fill, min_window_fill, kmax, 1, 0.0, True)
            or restate_pass(a, min_fill, min_window_fill, kmax, keep_rows, max_rem, False))


def restate_pass(a, min_fill, min_window_fill, kmax, keep_rows, max_rem, exact):
    m = a.num_rows
    ro = a.row_offsets.astype(np.int64)
    ci = a.column_indices.astype(np.int64)
    if m == 0 or a.num_nonzeros == 0:
        return None
    ks, masked, kept_total = [], 0, 0
    for r0 in range(0, m, 64):
        r1 = min(m, r0 + 64)
        nr = r1 - r0
        offs = []
        for r in range(r0, r1):
            o = ci[ro[r]:ro[r + 1]] - r
            if o.size > 1 and np.any(np.diff(o) <= 0):
                return None
            offs.append(o)
        allo = np.concatenate(offs) if offs else np.zeros(0, np.int64)
        vals, counts = np.unique(allo, return_counts=True)  # ascending offsets
        sel = counts >= min(keep_rows, nr)
        cand = list(zip(vals[sel].tolist(), counts[sel].tolist()))
        cand.sort(key=lambda t: -t[1])  # stable: equal counts keep the smaller offset first
        cand = cand[:kmax]
        kept = sum(c for _, c in cand)
        while cand and kept < min_window_fill * nr * len(cand):
            kept -= cand.pop()[1]
        K = len(cand)
        ks.append(K)
        kept_total += kept
        masked += not (nr == 64 and kept == 64 * K)
    rem = a.num_nonzeros - kept_total
    if sum(ks) == 0 or kept_total < min_fill * 64 * sum(ks) or rem > max_rem * a.num_nonzeros:
        return None
    return {"windows": len(ks), "sum_offsets": sum(ks), "masked_windows": masked, "k": np.array(ks),
            "remainder": rem}


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
    "fem_blocked": (lambda: mspmv.CsrMatrix.synth_fem_blocked(2400, 126000, 6, 60, seed=3), False),  # no offsets
    "banded_random": (lambda: mspmv.CsrMatrix.synth_banded(3000, 3000 * 8, 400, seed=2), False),     # kept
    "perturbed27": (lambda: mspmv.CsrMatrix.synth_stencil_perturbed((17, 12, 9), seed=1, extra_frac=0.02,
                                                                    long_frac=0.01), True),        # remainder
    "perturbed_heavy": (lambda: mspmv.CsrMatrix.synth_stencil_perturbed((17, 12, 9), seed=1, extra_frac=0.5,
                                                                        long_frac=0.1), False),    # > 5 %
    "kkt": (lambda: mspmv.CsrMatrix.synth_kkt((17, 12, 9), seed=4), True),                         # K 34
    "wide": (lambda: band(64 * 9, list(range(-20, 21)) + [100, 200], 8), True),                   # K 43
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
        assert got["remainder"] == want["remainder"]
        np.testing.assert_array_equal(got["k"], want["k"])


def test_offset_windows_thresholds():
    """Forced thresholds (MSPMV_DIA=1 plans at fill 0): windows with missing offsets and empty rows fit;
    a window whose kept entries fall below min_window_fill drops its rarest offsets to the remainder
    (round 5 rejected the whole plan), which the forced plan takes in any amount."""
    a = CASES["holes"][0]()
    assert mspmv.offset_windows(a, 0.0, 0.0) is not None
    assert mspmv.offset_windows(a, 0.6, 0.3) is not None
    assert mspmv.offset_windows(a, 0.8, 0.3) is None
    e = band(3000, [0, 3], 6, drop=0.6)
    got, want = mspmv.offset_windows(e, 0.0, 0.0), restate(e, 0.0, 0.0)
    assert got is not None and got["masked_windows"] == want["masked_windows"] == got["windows"]
    got, want = mspmv.offset_windows(e, 0.0, 0.5), restate(e, 0.0, 0.5)
    assert got is not None and got["remainder"] == want["remainder"] > 0
    np.testing.assert_array_equal(got["k"], want["k"])
    assert np.any(got["k"] == 0)  # whole windows left to the remainder


def test_offset_windows_rejects_bad_input():
    t = band(200, [0, 1], 1)
    bad = mspmv.CsrMatrix.from_arrays(t.num_cols, t.row_offsets, t.column_indices.copy(), t.values)
    bad.column_indices[3] = t.num_cols + 5
    with pytest.raises(RuntimeError):
        mspmv.offset_windows(bad)
