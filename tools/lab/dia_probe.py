#!/usr/bin/env python3
"""Offset windows vs tiles (run under MSPMV_DIA=0 / unset): kernel times by HIP events on the
structured-grid shapes -- the nlpkkt120-size 27-point matrix (L = 1 and 8, never cache-resident) and
the parabolic_fem shape (L = 1 and 8, cold after a 512 MiB flush) -- and the kernel each ran; PROBE_L
lists other widths.
One JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

FLUSH = 512 << 20
shapes = {
    "nlpkkt": (lambda: mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2), 0),
    "pfem": (lambda: mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4), FLUSH),
}
out = {"dia": os.environ.get("MSPMV_DIA", "auto")}
only = os.environ.get("PROBE_ONLY", "").split()
for name, (make, flush) in shapes.items():
    if only and name not in only:
        continue
    a = make()
    with mspmv.GpuCsr(a) as g:
        for L in [int(v) for v in os.environ.get("PROBE_L", "1 8").split()]:
            X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, L))
            dX = mspmv.DeviceBuffer.from_array(X)
            dY = mspmv.DeviceBuffer(8 * a.num_rows * L)
            g.time_spmm(dX, dY, L, 5, flush)
            _, kern_ms, _ = g.time_spmm(dX, dY, L, 40, flush)
            nb = 12 * a.num_nonzeros + 4 * (a.num_rows + 1) + 8 * L * (a.num_cols + a.num_rows)
            out[f"{name}_L{L}_us"] = round(kern_ms * 1e3, 2)
            out[f"{name}_L{L}_frac"] = round(nb / (kern_ms * 1e-3) / 8e12, 4)
            out[f"{name}_L{L}_kernel"] = g.spmm_kernel_name(L)
            dX.free()
            dY.free()
print(json.dumps(out), flush=True)
