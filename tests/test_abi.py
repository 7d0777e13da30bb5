"""The C-ABI boundary: libmspmv.so loads (no GPU needed) and exports every symbol that
include/*.h declares; host-only pieces (synthetic generators) behave."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("mspmv.h", "mspmv_synth.h", "mspmv_dist.h", "mspmv_io.h")]


def declared():
    names = set()
    for h in HEADERS:
        names |= set(re.findall(r"MSPMV_API\s+[\w\s\*]*?\b(mspmv_\w+)\s*\(", open(h).read()))
    return sorted(names)


def test_every_declared_symbol_is_exported(mspmv):
    names = declared()
    assert len(names) >= 30
    lib = ctypes.CDLL(mspmv.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding declares exactly that set
    assert set(mspmv._SIGS) == set(names)


def test_no_compute_without_device(mspmv):
    if mspmv.device_count() > 0:
        pytest.skip("a device is visible")
    a = mspmv.CsrMatrix.synth_banded(100, 500, 20)
    with pytest.raises(mspmv.MspmvError):
        mspmv.GpuCsr(a)  # fails loudly -- there is no CPU fallback


def test_product_does_not_link_oracle(mspmv):
    import subprocess
    out = subprocess.run(["ldd", mspmv.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out and "mspmv_ref" not in out
    syms = subprocess.run(["nm", "-D", mspmv.LIB_PATH], capture_output=True, text=True).stdout
    assert "orc_" not in syms and "ref_" not in syms


def test_synth_banded_exact(mspmv):
    a = mspmv.CsrMatrix.synth_banded(1000, 52345, 200, seed=5)
    assert a.row_offsets[-1] == 52345 == a.num_nonzeros
    lens = np.diff(a.row_offsets)
    assert lens.max() - lens.min() <= 1
    for i in (0, 1, 500, 999):
        c = a.column_indices[a.row_offsets[i]:a.row_offsets[i + 1]]
        assert np.all(np.diff(c) > 0) and c.min() >= max(0, i - 200) and c.max() <= min(999, i + 200)
    assert np.all((a.values >= 0.5) & (a.values < 1.5))
    b = mspmv.CsrMatrix.synth_banded(1000, 52345, 200, seed=5)
    assert a.values.tobytes() == b.values.tobytes() and np.array_equal(a.column_indices, b.column_indices)


@pytest.mark.parametrize("kind,m,dims", [(0, 1000, (37, 0, 0)), (1, 6 * 7 * 8, (6, 7, 8))])
def test_synth_stencil_spd(mspmv, kind, m, dims):
    a = mspmv.CsrMatrix.synth_stencil(kind, m, *dims)
    dense = np.zeros((m, m))
    for i in range(m):
        s, e = a.row_offsets[i], a.row_offsets[i + 1]
        assert np.all(np.diff(a.column_indices[s:e]) > 0)
        dense[i, a.column_indices[s:e]] = a.values[s:e]
    assert np.array_equal(dense, dense.T)
    assert np.linalg.eigvalsh(dense).min() > 0
    if kind == 1:
        assert np.diff(a.row_offsets).max() == 27


def test_synth_powerlaw_exact(mspmv):
    a = mspmv.CsrMatrix.synth_powerlaw(5000, 4000, 200000, exponent=1.5, seed=2)
    lens = np.diff(a.row_offsets)
    assert lens.sum() == 200000 and lens.max() <= 4000 and lens.max() > 20 * lens.mean()
    for i in np.flatnonzero(lens)[:50]:
        c = a.column_indices[a.row_offsets[i]:a.row_offsets[i + 1]]
        assert np.all(np.diff(c) > 0) and c.max() < 4000


def xcd_tile(b, T):
    """Host mirror of mspmv_device.h xcd_tile: block b -> tile (XCD k = b % 8 walks a contiguous range)."""
    q, r = T >> 3, T & 7
    k, i = b & 7, b >> 3
    return k * q + (k if k < r else r) + i


@pytest.mark.parametrize("T", [1, 2, 7, 8, 9, 15, 16, 17, 255, 256, 257, 1023, 9221, 12123])
def test_xcd_tile_bijective(T):
    """Every tile kernel maps blockIdx through xcd_tile: it must be a permutation of 0..T-1."""
    got = sorted(xcd_tile(b, T) for b in range(T))
    assert got == list(range(T))
