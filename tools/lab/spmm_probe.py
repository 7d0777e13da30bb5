#!/usr/bin/env python3
"""SpMM kernel times (HIP events, back-to-back launches) on the bench shapes, one JSON line;
MSPMV_LIB selects the library (A/B of tools/lab/libmspmv_base.so against the in-tree one)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

shapes = {
    "cant": lambda: mspmv.CsrMatrix.synth_banded(62451, 4007383, 2000, seed=1),
    "pwtk": lambda: mspmv.CsrMatrix.synth_fem_blocked(217918, 11524432, 6, 1700, seed=1),
    "nlpkkt": lambda: mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2),
}
runs = {"cant": (16,), "pwtk": (2, 4, 8, 16), "nlpkkt": (8,)}
out = {"lib": os.path.basename(os.environ.get("MSPMV_LIB", "libmspmv.so"))}
for name, make in [(k, v) for k, v in shapes.items() if not os.environ.get("PROBE_ONLY") or k in os.environ["PROBE_ONLY"].split()]:
    a = make()
    with mspmv.GpuCsr(a) as g:
        for L in runs[name]:
            X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, L))
            dX = mspmv.DeviceBuffer.from_array(X)
            dY = mspmv.DeviceBuffer(8 * a.num_rows * L)
            g.time_spmm(dX, dY, L, 5)
            _, kern_ms, _ = g.time_spmm(dX, dY, L, 50)
            out[f"{name}_L{L}_us"] = round(kern_ms * 1e3, 2)
print(json.dumps(out), flush=True)
