"""Product MatrixMarket reader and generators (libmspmv.so, host side) vs the reference's own
CSR arrays (golden fixtures from CooMatrix::InitMarket / Init* + CsrMatrix::Init) -- bit-exact."""
import os

import numpy as np
import pytest

import mspmv
from test_oracle_pinning import GOLD, csr, same_csr


@pytest.mark.parametrize("key", ["general", "symmetric", "skew", "pattern", "array", "noeol"])
def test_market_reader_matches_reference(key):
    same_csr(mspmv.CsrMatrix.from_market(os.path.join(GOLD, f"market_{key}.mtx")), csr("mtx_" + key))


@pytest.mark.parametrize("key,kind,p0,p1", [
    ("g2d5", "grid2d", 5, 0), ("g2d5s", "grid2d", 5, 1), ("g3d4", "grid3d", 4, 0), ("g3d4s", "grid3d", 4, 1),
    ("wheel7", "wheel", 7, 0), ("dense3x5", "dense", 3, 5)])
def test_generators_match_reference(key, kind, p0, p1):
    same_csr(mspmv.CsrMatrix.generate(kind, p0, p1), csr("gen_" + key))


def test_lattice_kat():
    a = mspmv.CsrMatrix.generate("grid2d", 3, 0)
    same_csr(a, csr("lat"))


def test_market_errors(tmp_path):
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix coordinate real general\nthis is not a size line\n")
    with pytest.raises(mspmv.MspmvError):
        mspmv.CsrMatrix.from_market(str(bad))
    with pytest.raises(mspmv.MspmvError):
        mspmv.CsrMatrix.from_market(str(tmp_path / "missing.mtx"))
    over = tmp_path / "over.mtx"
    over.write_text("%%MatrixMarket matrix coordinate real general\n2 2 1\n1 1 1\n2 2 2\n")
    with pytest.raises(mspmv.MspmvError):   # more entries than declared (sparse_matrix.h:303-307)
        mspmv.CsrMatrix.from_market(str(over))


def test_market_duplicates_and_order(tmp_path, orc):
    rng = np.random.default_rng(0)
    rows = rng.integers(1, 40, 500)
    cols = rng.integers(1, 30, 500)
    vals = rng.standard_normal(500)
    p = tmp_path / "dup.mtx"
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n% random with duplicates\n40 30 500\n")
        for r, c, v in zip(rows, cols, vals):
            f.write(f"{r} {c} {float(v)!r}\n")
    a = mspmv.CsrMatrix.from_market(str(p))
    rc, b = orc.read_market(str(p))
    assert rc == 0
    same_csr(a, b)
