#!/usr/bin/env python3
"""configs[3] CGSolveSingle on the parabolic_fem shape: us per iteration of the register-resident
kernel and its phase stamps (bench.py resident_phases), one JSON line.  The form comes from the
environment (MSPMV_CG_RESIDENT_FORM)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402
from bench import glibc_rhs, resident_phases  # noqa: E402

pf = mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)
n = pf.num_rows
b = glibc_rhs(42, n)
thr = float(np.sqrt(np.sum(b * b)) * 1e-5)
out = {"form": os.environ.get("MSPMV_CG_RESIDENT_FORM", "default")}
with mspmv.GpuCsr(pf) as g:
    db, dx = mspmv.DeviceBuffer.from_array(b), mspmv.DeviceBuffer(8 * n)
    g.cg_dev(db, dx, 1, 10000, thr)
    best = None
    for _ in range(5):
        t0 = time.perf_counter()
        it, _, st = g.cg_dev(db, dx, 1, 10000, thr)
        el = time.perf_counter() - t0
        best = el / it if best is None else min(best, el / it)
    out.update(kernel=g.cg_kernel_name(), iterations=it, status=st, us_per_iter=round(best * 1e6, 3))
    out["phases"] = resident_phases(g, db, dx, thr)
print(json.dumps(out), flush=True)
