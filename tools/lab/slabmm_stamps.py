#!/usr/bin/env python3
"""LAB: per-chunk phase stamps of the column-slab SpMM (MSPMV_SLAB_STAMPS build) on the cant L = 16 and
nlpkkt120 L = 8 shapes; writes <out>/<shape>.bin ([64 blocks][2 roles][64 chunks][4] s_memtime) and prints
median phase lengths in shader cycles: store (wait for the chunk's registers + LDS writes), issue+barrier A,
runs, barrier B."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
os.environ["MSPMV_SPMM_SLAB"] = "1"
import mspmv  # noqa: E402

shapes = {"cant": (lambda: mspmv.CsrMatrix.synth_banded(62451, 4007383, 2000, seed=1), 16),
          "nlpkkt": (lambda: mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2), 8)}
for name, (make, L) in shapes.items():
    a = make()
    with mspmv.GpuCsr(a) as g:
        X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, L))
        dX, dY = mspmv.DeviceBuffer.from_array(X), mspmv.DeviceBuffer(8 * a.num_rows * L)
        g.spmm_dev(dX, dY, L)
        f = os.path.join(out, name + ".bin")
        os.environ["MSPMV_SLAB_STAMPS"] = f
        for _ in range(3):
            g.spmm_dev(dX, dY, L)
        del os.environ["MSPMV_SLAB_STAMPS"]
        dX.free()
        dY.free()
    st = np.fromfile(f, np.uint64).astype(np.int64).reshape(64, 2, 64, 4)
    res = {}
    for role in (0, 1):
        ph = [[], [], [], []]
        tot = []
        for b in range(64):
            s = st[b, role]
            n = int(np.sum(s[:, 0] > 0))
            if n < 2:
                continue
            s = s[:n]
            ph[0] += list(s[:, 1] - s[:, 0])
            ph[1] += list(s[:, 2] - s[:, 1])
            ph[2] += list(s[:, 3] - s[:, 2])
            ph[3] += list(s[1:, 0] - s[:-1, 3])
            tot.append(s[-1, 3] - s[0, 0])
        res[role] = {"chunks_med": int(np.median([int(np.sum(st[b, role, :, 0] > 0)) for b in range(64)])),
                     "store": int(np.median(ph[0])), "issue_barA": int(np.median(ph[1])), "runs": int(np.median(ph[2])),
                     "barB": int(np.median(ph[3])), "block_total_med": int(np.median(tot)),
                     "store_p90": int(np.percentile(ph[0], 90)), "runs_p90": int(np.percentile(ph[2], 90)),
                     "barA_p90": int(np.percentile(ph[1], 90))}
    print(name, "stream:", res[0], flush=True)
    print(name, "panel: ", res[1], flush=True)
