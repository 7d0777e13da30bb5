"""Shared helpers for the GPU parity tests."""
import numpy as np

EPS = 2.0 ** -53


def groups_per_tile(L, lanes=256):
    """Merge walkers per tile: one per thread (L == 1; 256 threads, or 64 on a one-wave plan) or
    one per L/2 lanes of a 256-thread tile."""
    return lanes if L == 1 else 256 // (L // 2)


def unsplit_rows(a, plan, L):
    """Rows the kernel sums sequentially in CSR order from 0.0, i.e. bit-identically to
    SpmvGold (cpu_spmv.cpp:241-265).

    Mirrors the kernel's partition exactly: tile t spans plan bounds t..t+1.  A merge-walk tile
    (mode 0) gives its walkers ceil(items / groups) consecutive diagonals each, and a row is
    sequential when all its items fall in one walker.  A row-group tile (mode g > 0, groups of
    2^(g-1) lanes) is sequential for its whole rows only when g == 1 (one row per thread).
    """
    bounds = plan["bounds"]
    modes = plan.get("modes")
    ng = groups_per_tile(L, plan.get("lanes", 256))
    ro = a.row_offsets.astype(np.int64)
    mask = np.zeros(a.num_rows, bool)
    for t in range(plan["num_tiles"]):
        r0, n0 = (int(v) for v in bounds[t])
        r1, n1 = (int(v) for v in bounds[t + 1])
        nrows = r1 - r0
        if nrows <= 0:
            continue
        r = np.arange(nrows)
        rs = ro[r0 + r] - n0
        re = ro[r0 + r + 1] - n0
        mode = int(modes[t]) if modes is not None and len(modes) else 0
        if mode == 0:
            items = nrows + (n1 - n0)
            ipt = -(-items // ng)
            ok = (rs >= 0) & ((r + rs) // ipt == (r + re) // ipt)
        else:
            ok = (rs >= 0) & (mode == 1)
        mask[r0 + r] = ok
    return mask


def abs_bound(a, X):
    """Per-row (and column) |A| |X| and row lengths, for reordering-error bounds."""
    X = np.asarray(X, np.float64)
    if X.ndim == 1:
        X = X[:, None]
    ro = a.row_offsets.astype(np.int64)
    lens = np.diff(ro)
    acc = np.zeros((a.num_rows, X.shape[1]))
    if a.num_nonzeros:  # segment sums over the non-empty rows (fast at 10^8 nonzeros)
        prod = np.abs(a.values)[:, None] * np.abs(X[a.column_indices])
        ne = lens > 0
        acc[ne] = np.add.reduceat(prod, ro[:-1][ne], axis=0)
    return acc, lens


def check_parity(a, y_gpu, y_seq, X, plan, L):
    """Unsplit rows bit-identical to the sequential CSR-order sum; split rows within the
    summation-reordering bound 2 (len+1) eps (|A||x|)_i.  Returns (#bit-exact, #rows)."""
    y_gpu = np.asarray(y_gpu, np.float64).reshape(a.num_rows, -1)
    y_seq = np.asarray(y_seq, np.float64).reshape(a.num_rows, -1)
    mask = unsplit_rows(a, plan, L)
    g, s = y_gpu[mask], y_seq[mask]
    diff = np.flatnonzero(g.view(np.uint64) != s.view(np.uint64))
    assert diff.size == 0, f"{diff.size} unsplit entries not bit-identical, e.g. {g.ravel()[diff[:3]]} vs {s.ravel()[diff[:3]]}"
    bound, lens = abs_bound(a, X)
    tol = 2.0 * (lens[:, None] + 1) * EPS * bound + 1e-300
    err = np.abs(y_gpu - y_seq)
    bad = np.argwhere(err > tol)
    assert bad.size == 0, f"{len(bad)} entries exceed the reordering bound, e.g. row {bad[:3]}"
    assert np.all(np.isfinite(y_gpu) == np.isfinite(y_seq))
    return int(mask.sum()), a.num_rows


def chunk_widths(L):
    """Column chunks mspmv_dspmm runs for a width outside {1, 2, 4, 8, 16} (mspmv_api.hip
    spmm_chunks): odd L > 1 padded to L + 1, then 16, 8, 4, 2 greedily; [(offset, width)]."""
    Lp = L + 1 if L > 1 and L % 2 else L
    out, c0 = [], 0
    while c0 < Lp:
        w = 16
        while w > Lp - c0:
            w //= 2
        out.append((c0, w))
        c0 += w
    return out


def check_parity_chunked(a, g, Y, Yseq, X, L):
    """check_parity per column chunk, each against its own width's tile plan."""
    for c0, w in chunk_widths(L):
        c1 = min(c0 + w, L)
        check_parity(a, Y[:, c0:c1], Yseq[:, c0:c1], X[:, c0:c1], g.tile_plan(w), w)
