#!/usr/bin/env python3
"""Counter-pass workload: the nlpkkt120-size 27-point matrix, L = 8 SpMM and the SpMV, 10 launches each,
first on the offset windows (MSPMV_DIA_SPMM=1), then on the merge tiles (MSPMV_DIA=0)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

a = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2)
for env in ({"MSPMV_DIA_SPMM": "1"}, {"MSPMV_DIA": "0", "MSPMV_DIA_SPMM": "0"}):
    os.environ.update(env)
    with mspmv.GpuCsr(a) as g:
        for L in (8, 1):
            dX = mspmv.DeviceBuffer.from_array(np.random.default_rng(3).uniform(0, 1, (a.num_cols, L)))
            dY = mspmv.DeviceBuffer(8 * a.num_rows * L)
            _, ms, _ = g.time_spmm(dX, dY, L, 10)
            print(env, L, g.spmm_kernel_name(L), round(ms * 1e3, 1), "us", flush=True)
            dX.free()
            dY.free()
