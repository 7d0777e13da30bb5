#!/usr/bin/env python3
"""Column-group slab SpMV (MSPMV_SPMV_SLAB=2) vs the default plan on the power-law variant (pwtk's m and
nnz, exponent 1.2, seed 3) and the scattered band: cold (after a 512 MiB flush) and hot kernel times by HIP
events, the kernel each ran, and the largest deviation between the two results in units of the
reordering bound's eps (|A||x|)_i.  PROBE_MODES lists the MSPMV_SPMV_SLAB values ('' = default; 'v:g' also
sets MSPMV_SLAB_GROUPS=g).
One JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

FLUSH = 512 << 20
M, NNZ = 217918, 11524432
shapes = {
    "powerlaw": lambda: mspmv.CsrMatrix.synth_powerlaw(M, M, NNZ, 1.2, 3),
    "band": lambda: mspmv.CsrMatrix.synth_banded(M, M * 53, 10000, seed=77),
    # the default-choice test's power-law matrix (tests/test_gpu_slab.py)
    "powerlaw4m": lambda: mspmv.CsrMatrix.synth_powerlaw(120000, 120000, 4000000, exponent=1.2, seed=9),
}
modes = os.environ.get("PROBE_MODES", " 2").split(" ")
only = os.environ.get("PROBE_ONLY", "").split()
out = {}
for name, make in shapes.items():
    if only and name not in only:
        continue
    a = make()
    x = np.random.default_rng(3).uniform(0, 1, a.num_cols)
    absA = np.abs(a.values)
    bound = np.add.reduceat(absA * x[a.column_indices], a.row_offsets[:-1]) if a.num_nonzeros else None
    nb = 12 * a.num_nonzeros + 4 * (a.num_rows + 1) + 8 * (a.num_cols + a.num_rows)
    ys = {}
    for md in modes:
        sw, _, grp = md.partition(":")  # "3:8" = MSPMV_SPMV_SLAB=3 with MSPMV_SLAB_GROUPS=8
        for k, v in (("MSPMV_SPMV_SLAB", sw), ("MSPMV_SLAB_GROUPS", grp)):
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
        with mspmv.GpuCsr(a) as g:
            ys[md] = g.spmv(x)
            dX = mspmv.DeviceBuffer.from_array(x)
            dY = mspmv.DeviceBuffer(8 * a.num_rows)
            g.time_spmm(dX, dY, 1, 5, FLUSH)
            _, cold, _ = g.time_spmm(dX, dY, 1, 40, FLUSH)
            _, hot, _ = g.time_spmm(dX, dY, 1, 40, 0)
            key = f"{name}_{md or 'default'}"
            out[key + "_cold_us"] = round(cold * 1e3, 2)
            out[key + "_hot_us"] = round(hot * 1e3, 2)
            out[key + "_frac"] = round(nb / (cold * 1e-3) / 8e12, 4)
            out[key + "_kernel"] = g.kernel_name()
            out[key + "_tiles"] = g.tile_plan(1)["num_tiles"]
            dX.free()
            dY.free()
    base = ys[modes[0]]
    eps = np.finfo(np.float64).eps
    lens = np.diff(a.row_offsets)
    for md in modes[1:]:
        dev = np.abs(ys[md] - base) / ((lens + 1) * eps * bound + 1e-300)
        out[f"{name}_{md}_max_dev_eps_units"] = round(float(dev.max()), 3)
    print(json.dumps(out), flush=True)
os.environ.pop("MSPMV_SPMV_SLAB", None)
print(json.dumps(out), flush=True)
