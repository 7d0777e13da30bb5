#!/usr/bin/env python3
"""Sharded CG (world 1) per-iteration wall time with the batch graph on / off (MSPMV_DIST_GRAPH,
read once per process: run one child per setting).  usage: dist_graph_probe.py SHAPE L"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import numpy as np  # noqa: E402
import mspmv  # noqa: E402

shape, L = sys.argv[1], int(sys.argv[2])
if shape == "parabolic":
    a = mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)
else:
    a = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2)
rb = mspmv.dist_partition(a, 1)
d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))
dB = mspmv.DeviceBuffer.from_array(np.random.default_rng(2).uniform(0, 1, (a.num_rows, L)))
dX = mspmv.DeviceBuffer(8 * a.num_rows * L)
d.cg_dev(dB, dX, L, 100, 0.0)
best = 1e9
for _ in range(3):
    t0 = time.perf_counter()
    it, _, st = d.cg_dev(dB, dX, L, 300, 0.0)
    best = min(best, (time.perf_counter() - t0) / max(it, 1))
d.close()
print(json.dumps({"shape": shape, "L": L, "graph": os.environ.get("MSPMV_DIST_GRAPH", "1"),
                  "split": os.environ.get("MSPMV_DIST_FORCE_SPLIT", "0"), "us_per_iter": round(best * 1e6, 2)}))
