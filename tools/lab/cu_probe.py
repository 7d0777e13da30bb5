"""Lab: does mspmv_set_cu_limit confine the kernels?  SpMV kernel time on the pwtk shape and CG
ms/iteration at L = 1, 2, 8 on the parabolic_fem shape at ONE CU count (argv[1]) per process:
switching one process between several masked streams hung a launch (r02o)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd"), ROOT]
import mspmv  # noqa: E402
import bench  # noqa: E402

a = mspmv.CsrMatrix.synth_fem_blocked(217918, 11524432, 6, 1700, seed=1)
x = np.random.default_rng(2).uniform(0, 1, a.num_cols)
with mspmv.GpuCsr(a) as g:
    dx, dy = mspmv.DeviceBuffer.from_array(x, 0), mspmv.DeviceBuffer(8 * a.num_rows, 0)
    for cu in (int(sys.argv[1]),):
        g.set_cu_limit(cu)
        g.time_spmm(dx, dy, 1, 5)
        _, k, _ = g.time_spmm(dx, dy, 1, 50)
        print(f"spmv pwtk CUs={cu}: {k * 1e3:.2f} us", flush=True)
pf = mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)
for L in (1, 2, 8):
    B = np.random.default_rng(1).uniform(0, 1, (pf.num_rows, L))
    with mspmv.GpuCsr(pf) as g:
        dB, dX = mspmv.DeviceBuffer.from_array(B, 0), mspmv.DeviceBuffer(8 * pf.num_rows * L, 0)
        for cu in (int(sys.argv[1]),):
            g.set_cu_limit(cu)
            g.cg_dev(dB, dX, L, 100000, 1e-5)
            t0 = time.perf_counter()
            it, _, _ = g.cg_dev(dB, dX, L, 100000, 1e-5)
            el = time.perf_counter() - t0
            print(f"cg L={L} CUs={cu}: {it} it, {el / it * 1e6:.1f} us/iter", flush=True)
