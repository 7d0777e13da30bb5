#!/usr/bin/env python3
"""Single-RHS SpMV per-launch kernel times on named shapes, one JSON line per shape.  Matrices
below the Infinity Cache are timed as a batch of 4 distinct seeds back to back (as bench.py's
headline: every launch streams HBM); larger ones alone.  Kernel time from the kernels' own start /
end events.  usage: spmv_probe.py [shape ...]  (MSPMV_LIB selects the library for A/B runs)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

PW = (217918, 11524432, 6, 1700)
SHAPES = {
    "pwtk": lambda s: mspmv.CsrMatrix.synth_fem_blocked(*PW, seed=s),
    "pwtk_odd": lambda s: mspmv.CsrMatrix.synth_fem_perturbed(*PW, 0.02, 0.0, seed=s),
    "pwtk_extra": lambda s: mspmv.CsrMatrix.synth_fem_perturbed(*PW, 0.0, 0.01, seed=s),
    "pwtk_perturbed": lambda s: mspmv.CsrMatrix.synth_fem_perturbed(*PW, 0.02, 0.01, seed=s),
    "nlpkkt": lambda s: mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, seed=s, diag_shift=1e-2),
    "powerlaw": lambda s: mspmv.CsrMatrix.synth_powerlaw(PW[0], PW[0], PW[1], 1.2, 3 + s),
    "scatter": lambda s: mspmv.CsrMatrix.synth_banded(PW[0], PW[1], 10000, seed=77 + s),
    "cant": lambda s: mspmv.CsrMatrix.synth_banded(62451, 4007383, 2000, seed=s),
}
HBM = 8000.0
for name in (sys.argv[1:] or os.environ.get("PROBE_SHAPES", "").split() or list(SHAPES)):
    n = 1 if name == "nlpkkt" else 4
    mats = [SHAPES[name](s + 1) for s in range(n)]
    gs = [mspmv.GpuCsr(a) for a in mats]
    xs = [mspmv.DeviceBuffer.from_array(np.random.default_rng(s).uniform(0, 1, a.num_cols)) for s, a in enumerate(mats)]
    ys = [mspmv.DeviceBuffer(8 * a.num_rows) for a in mats]
    mspmv.time_spmm_batch(gs, xs, ys, 1, 5)
    step, kern, kps = mspmv.time_spmm_batch(gs, xs, ys, 1, 30 if n > 1 else 20)
    a = mats[0]
    nb = 12 * a.num_nonzeros + 4 * (a.num_rows + 1) + 8 * (a.num_cols + a.num_rows)
    plan = gs[0].tile_plan(1)
    print(json.dumps({"shape": name, "lib": os.path.basename(os.environ.get("MSPMV_LIB", "libmspmv.so")),
                      "kernel": gs[0].kernel_name(), "nnz": a.num_nonzeros, "tiles": plan["num_tiles"],
                      "tiles_all": [g.tile_plan(1)["num_tiles"] for g in gs],
                      "block_tiles": gs[0].plan_block_tiles(1), "carries": plan["num_carries"],
                      "kernel_us": round(kern * 1e3, 2), "step_us": round(step * 1e3, 2), "kernels_per_step": kps,
                      "frac": round(nb / (kern * 1e-3) / 1e9 / HBM, 4)}), flush=True)
    for g in gs:
        g.close()
    for b in xs + ys:
        b.free()
