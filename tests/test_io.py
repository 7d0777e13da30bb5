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


# --- the parallel parser (mspmv_io.cpp market_entries_parallel + the parallel stable COO->CSR) ---
def _mtx(path, banner, size, lines, eol="\n", last_eol=True):
    body = eol.join([banner, size] + lines)
    path.write_bytes((body + (eol if last_eol else "")).encode())
    return str(path)


def _entries(rng, n, m, ncol, fmt="{r} {c} {v!r}", diag=True):
    out = []
    for _ in range(n):
        r = int(rng.integers(1, m + 1))
        c = r if (diag and r <= ncol and rng.random() < 0.1) else int(rng.integers(1, ncol + 1))
        out.append(fmt.format(r=r, c=c, v=float(rng.standard_normal())))
    return out


def _cases(tmp_path):
    rng = np.random.default_rng(7)
    ent = _entries(rng, 4000, 300, 250)
    with_comments = list(ent)
    for k in range(0, 4000, 97):
        with_comments.insert(k, "% a comment line")
    sym = _entries(rng, 3000, 200, 200)
    sym = [ln for ln in sym if int(ln.split()[1]) <= int(ln.split()[0])]
    pat = [" ".join(ln.split()[:2]) for ln in ent]
    octal = ["0%o 0x%x %r" % (int(ln.split()[0]), int(ln.split()[1]), float(ln.split()[2])) for ln in ent[:2000]]
    long_mid = list(ent)
    long_mid[2500] = long_mid[2500] + " " + "9" * 1100          # > 1022 chars: the parse ends here
    banner_mid = list(sym)
    banner_mid.insert(1500, "%%MatrixMarket matrix coordinate real general")
    bad_mid = list(ent)
    bad_mid[3100] = "x y z"
    g = "%%MatrixMarket matrix coordinate real general"
    return {
        "general": (_mtx(tmp_path / "g.mtx", g, "300 250 4000", ent), 0),
        "comments": (_mtx(tmp_path / "c.mtx", g, "300 250 4000", with_comments), 0),
        "symmetric": (_mtx(tmp_path / "s.mtx", "%%MatrixMarket matrix coordinate real symmetric",
                           f"200 200 {len(sym)}", sym), 0),
        "skew": (_mtx(tmp_path / "k.mtx", "%%MatrixMarket matrix coordinate real skew-symmetric",
                      f"200 200 {len(sym)}", sym), 0),
        "pattern": (_mtx(tmp_path / "p.mtx", "%%MatrixMarket matrix coordinate pattern general",
                         "300 250 4000", pat), 0),
        "crlf": (_mtx(tmp_path / "r.mtx", g, "300 250 4000", ent, eol="\r\n"), 0),
        "noeol": (_mtx(tmp_path / "n.mtx", g, "300 250 4000", ent, last_eol=False), 0),
        "base0_ints": (_mtx(tmp_path / "o.mtx", g, "300 250 2000", octal), 0),
        "long_line_mid": (_mtx(tmp_path / "l.mtx", g, "300 250 4000", long_mid), 0),
        "banner_mid": (_mtx(tmp_path / "b.mtx", "%%MatrixMarket matrix coordinate real symmetric",
                            f"200 200 {len(banner_mid)}", banner_mid), 0),
        "too_many": (_mtx(tmp_path / "t.mtx", g, "300 250 3999", ent), 1),
        "bad_mid": (_mtx(tmp_path / "x.mtx", g, "300 250 4000", bad_mid), 1),
    }


@pytest.mark.parametrize("chunk", ["64", "4096", "1048576"])
def test_parallel_market_reader_bit_exact(tmp_path, orc, monkeypatch, chunk):
    """Forced into many chunks (MSPMV_IO_MIN_CHUNK), the parallel reader returns exactly what the
    oracle's InitMarket restatement (pinned to the reference above) returns, errors included."""
    monkeypatch.setenv("MSPMV_IO_MIN_CHUNK", chunk)
    for name, (path, want_err) in _cases(tmp_path).items():
        rc, b = orc.read_market(path)
        assert (rc != 0) == bool(want_err), name
        if want_err:
            with pytest.raises(mspmv.MspmvError):
                mspmv.CsrMatrix.from_market(path)
            continue
        same_csr(mspmv.CsrMatrix.from_market(path), b)


def test_parallel_coo_to_csr_large(tmp_path, orc, monkeypatch):
    """A file big enough for the multi-threaded COO->CSR (>= 65536 entries per thread) and the
    default chunking: stable (row, col) order with duplicates, bit-exact."""
    rng = np.random.default_rng(11)
    n = 600000
    rows = rng.integers(1, 5001, n)
    cols = rng.integers(1, 4001, n)
    vals = rng.standard_normal(n)
    p = tmp_path / "big.mtx"
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n5000 4000 %d\n" % n)
        f.write("".join(f"{r} {c} {float(v)!r}\n" for r, c, v in zip(rows, cols, vals)))
    monkeypatch.setenv("MSPMV_IO_MIN_CHUNK", "65536")
    rc, b = orc.read_market(str(p))
    assert rc == 0
    same_csr(mspmv.CsrMatrix.from_market(str(p)), b)
