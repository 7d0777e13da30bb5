#!/usr/bin/env python3
"""Repeat test_gpu_dist.py::test_dist_cg_any_width[windows] (world 1, offset-window dot mode, L = 3 and 12
as column groups) REPS times in one process and print the iteration counts (the oracle's: 43 at L = 3,
from the test), to chase the intermittent 70-vs-43 failure seen in r05at.  No oracle here: lab scripts
only compare runs with each other.  One JSON line per rep, then a summary."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

a = mspmv.CsrMatrix.synth_stencil(1, 16 * 17 * 18, 16, 17, 18)
rb = mspmv.dist_partition(a, 1)
reps = int(os.environ.get("REPS", "8"))
widths = [int(v) for v in os.environ.get("WIDTHS", "3 12").split()]
out = {"graph": os.environ.get("MSPMV_DIST_GRAPH", "default"), "runs": []}
for r in range(reps):
    d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))
    its = {}
    for L in widths:
        B = np.random.default_rng(L).uniform(0, 1, (a.num_rows, L))
        dB = mspmv.DeviceBuffer.from_array(B)
        dX = mspmv.DeviceBuffer(8 * a.num_rows * L)
        it, hist, st = d.cg_dev(dB, dX, L, 3000, 1e-9, hist_cap=3000)
        its[L] = (it, st)
        dB.free()
        dX.free()
    d.close()
    out["runs"].append(its)
    print(json.dumps({"rep": r, "its": its}), flush=True)
print(json.dumps(out), flush=True)
