"""Generate the golden vectors under tests/golden/ from the REFERENCE'S OWN CODE.

Runs oracle/_ref/libmspmv_ref.so, i.e. the reference's header-only kernels
(sparse_matrix.h, work_2025/spmm/{merge_based,sample,row_splitting,nonzero_splitting}.hpp)
compiled in place from /root/reference by `make -C oracle ref` (see oracle/ref_harness.cpp).
Only data goes into the fixtures: inputs and the reference's outputs.

    make -C oracle ref && python tests/golden/make_golden.py

Known-answer tests that the reference documents independently of its code are added as
well: the 4x4 merge-path figure (merge_decomposition.png / merge_spmv.png) and the 9x9
lattice of cub/device/device_spmv.cuh:90-123.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]

from _oracle import RefLib  # noqa: E402
import mspmv  # noqa: E402

PS = (1, 2, 3, 4, 8, 64, 256)


def csr_dict(prefix, a):
    return {f"{prefix}_shape": np.array([a.num_rows, a.num_cols, a.num_nonzeros], np.int64),
            f"{prefix}_ro": a.row_offsets, f"{prefix}_ci": a.column_indices, f"{prefix}_va": a.values}


def random_csr(rng, m, n, lens):
    """CSR with the given row lengths (sorted unique columns), values U(-1, 1)."""
    ro = np.zeros(m + 1, np.int32)
    ro[1:] = np.cumsum(lens)
    cols = []
    for ell in lens:
        cols.append(np.sort(rng.choice(n, size=ell, replace=False)).astype(np.int32))
    ci = np.concatenate(cols) if cols else np.zeros(0, np.int32)
    va = rng.uniform(-1.0, 1.0, size=len(ci))
    return mspmv.CsrMatrix(m, n, int(ro[-1]), ro, ci, va)


def coords_ref(ref, a, P):
    total = a.num_rows + a.num_nonzeros
    ipt = (total + P - 1) // P
    out = np.empty((P + 1, 2), np.int32)
    row_end = np.ascontiguousarray(a.row_offsets[1:])
    for t in range(P + 1):
        out[t] = ref.merge_path_search(min(ipt * t, total), row_end, a.num_rows, a.num_nonzeros)
    return out


def main():
    ref = RefLib()
    rng = np.random.default_rng(20240918)
    out = {}

    # --- KATs ------------------------------------------------------------------------
    fig = mspmv.CsrMatrix(4, 4, 8, np.array([0, 2, 2, 4, 8], np.int32),
                          np.array([0, 2, 2, 3, 0, 1, 2, 3], np.int32), np.ones(8))
    out.update(csr_dict("fig", fig))
    out["fig_y"] = ref.merge_csrmm(fig, np.ones((4, 1)), 4)[:, 0]
    for P in (2, 3, 4, 12):
        out[f"fig_coords_P{P}"] = coords_ref(ref, fig, P)
    lat = ref.build("grid2d", 3, 0)
    out.update(csr_dict("lat", lat))
    out["lat_y"] = ref.spmv_gold(lat, np.ones(9))

    # --- generators (CooMatrix::Init* + CsrMatrix::Init) ----------------------------
    gens = {"g2d5": ("grid2d", 5, 0), "g2d5s": ("grid2d", 5, 1), "g3d4": ("grid3d", 4, 0),
            "g3d4s": ("grid3d", 4, 1), "wheel7": ("wheel", 7), "dense3x5": ("dense", 3, 5)}
    for key, (kind, *params) in gens.items():
        out.update(csr_dict("gen_" + key, ref.build(kind, *params)))

    # --- MatrixMarket files ----------------------------------------------------------
    mtx = {
        "general": "%%MatrixMarket matrix coordinate real general\n% comment\n4 5 6\n"
                   "1 1 1.5\n3 2 -2.0\n1 5 3e-1\n4 4 7\n2 3 0.25\n1 1 2.0\n",
        "symmetric": "%%MatrixMarket matrix coordinate real symmetric\n5 5 7\n"
                     "1 1 4\n2 1 -1\n2 2 4\n3 2 -1\n3 3 4\n5 1 0.5\n5 5 2\n",
        "skew": "%%MatrixMarket matrix coordinate real skew-symmetric\n3 3 2\n2 1 1.5\n3 1 -2\n",
        "pattern": "%%MatrixMarket matrix coordinate pattern general\n3 4 4\n1 2\n2 1\n3 4\n3 3\n",
        "array": "%%MatrixMarket matrix array real general\n2 3\n1\n2\n3\n4\n5\n6\n",
        "noeol": "%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1\n2 2 2\n1 2 3",
    }
    for key, text in mtx.items():
        path = os.path.join(HERE, f"market_{key}.mtx")
        with open(path, "w") as f:
            f.write(text)
        out.update(csr_dict("mtx_" + key, ref.build_market(path, 1.0)))

    # --- test matrices ---------------------------------------------------------------
    mats = {
        "grid2d20": ref.build("grid2d", 20, 1),
        "grid3d6": ref.build("grid3d", 6, 0),
        "wheel50": ref.build("wheel", 50),
        "dense16x8": ref.build("dense", 16, 8),
    }
    lens = rng.integers(0, 6, size=300)
    lens[[5, 77, 200]] = [120, 250, 90]        # a few long rows
    lens[100:140] = 0                          # a run of empty rows
    mats["skew300"] = random_csr(rng, 300, 280, lens)
    mats["empty_tail"] = random_csr(rng, 40, 40, np.r_[rng.integers(1, 5, 30), np.zeros(10, int)])
    for key, a in mats.items():
        out.update(csr_dict("m_" + key, a))
        for P in PS:
            out[f"m_{key}_coords_P{P}"] = coords_ref(ref, a, P)
        x = rng.uniform(-1.0, 1.0, a.num_cols)
        out[f"m_{key}_x"] = x
        out[f"m_{key}_gold"] = ref.spmv_gold(a, x)
        # the reference harness convention: x = 0.0019, y_in = 1.0, alpha 1, beta 0
        out[f"m_{key}_gold_const"] = ref.spmv_gold(a, np.full(a.num_cols, 0.0019), np.ones(a.num_rows))
        for P in (1, 3, 8, 64, 256):
            out[f"m_{key}_merge_P{P}"] = ref.merge_csrmm(a, x[:, None], P)[:, 0]
        for L in (8, 16):
            X = rng.uniform(-1.0, 1.0, (a.num_cols, L))
            out[f"m_{key}_X{L}"] = X
            out[f"m_{key}_mm{L}_P8"] = ref.merge_csrmm(a, X, 8)
            out[f"m_{key}_mm{L}_P37"] = ref.merge_csrmm(a, X, 37)
            out[f"m_{key}_rowsplit{L}"] = ref.csr_spmm_t(a, X)
            out[f"m_{key}_nzsplit{L}_P8"] = ref.nonzero_split_csrmm(a, X, 8)  # pre-zeroed Y

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    size = os.path.getsize(os.path.join(HERE, "golden.npz"))
    print(f"wrote {len(out)} arrays, {size / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
