#!/usr/bin/env python3
"""Lab: the nlpkkt120-size L = 8 window SpMM alone (hot, back to back), kernel us per launch; MSPMV_DIA_EXACT
selects the lab ablations of the build (r06j).  One JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402
from bench import NLPKKT120  # noqa: E402

nx, ny, nz = NLPKKT120["dims"]
a = mspmv.CsrMatrix.synth_stencil(1, nx * ny * nz, nx, ny, nz, diag_shift=NLPKKT120["shift"])
out = {"env": {k: v for k, v in os.environ.items() if k.startswith("MSPMV_")}}
L = int(os.environ.get("PROBE_L", "8"))
with mspmv.GpuCsr(a) as g:
    X = mspmv.DeviceBuffer.from_array(np.random.default_rng(1).uniform(0, 1, (a.num_cols, L)))
    Y = mspmv.DeviceBuffer(8 * a.num_rows * L)
    g.time_spmm(X, Y, L, 3)
    _, hot, _ = g.time_spmm(X, Y, L, 30)
    out.update(L=L, kernel=g.spmm_kernel_name(L), hot_us=round(hot * 1e3, 2))
print(json.dumps(out), flush=True)
