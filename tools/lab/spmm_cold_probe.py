#!/usr/bin/env python3
"""SpMM kernel times on the bench's configs[2] shapes, hot (back-to-back) and cold (512 MiB read
flush before every timed launch, as bench.py run_spmm16), one JSON line; MSPMV_LIB selects the
library (A/B of tools/lab/libmspmv_*.so against the in-tree one, tools/lab/ab_libs.sh)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

shapes = {
    "pwtk": (lambda: mspmv.CsrMatrix.synth_fem_blocked(217918, 11524432, 6, 1700, seed=1), (16, 8, 4)),
    "cant": (lambda: mspmv.CsrMatrix.synth_banded(62451, 4007383, 2000, seed=1), (16,)),
}
out = {"lib": os.path.basename(os.environ.get("MSPMV_LIB", "libmspmv.so"))}
for name, (make, Ls) in shapes.items():
    a = make()
    with mspmv.GpuCsr(a) as g:
        for L in Ls:
            X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, L))
            dX = mspmv.DeviceBuffer.from_array(X)
            dY = mspmv.DeviceBuffer(8 * a.num_rows * L)
            g.time_spmm(dX, dY, L, 5)
            _, hot, _ = g.time_spmm(dX, dY, L, 50)
            _, cold, _ = g.time_spmm(dX, dY, L, 20, 512 << 20)
            out[f"{name}_L{L}"] = [round(hot * 1e3, 2), round(cold * 1e3, 2)]
print(json.dumps(out), flush=True)
