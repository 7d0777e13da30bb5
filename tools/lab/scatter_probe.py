#!/usr/bin/env python3
"""Lab: bench.py's scattered-band stress case (a batch of 4 pwtk-size matrices, 53 columns per row over +-10,000)
on the plan the environment selects (MSPMV_SPMV_SLAB, MSPMV_SLAB_GROUPS): kernel, us per launch, frac, and the
first matrix's max |y - y_default| check against the tile plan (MSPMV_SPMV_SLAB=0 build of the same matrix).
One JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402
from bench import PWTK, spmv_bytes, HBM_PEAK_GBS  # noqa: E402

scs = [mspmv.CsrMatrix.synth_banded(PWTK["m"], PWTK["nnz"], 10000, seed=77 + i) for i in range(4)]
sgs = [mspmv.GpuCsr(a) for a in scs]
sbx = [mspmv.DeviceBuffer.from_array(np.random.default_rng(3 + i).uniform(0, 1, a.num_cols)) for i, a in enumerate(scs)]
sby = [mspmv.DeviceBuffer(8 * a.num_rows) for a in scs]
mspmv.time_spmm_batch(sgs, sbx, sby, 1, 5)
_, sk, _ = mspmv.time_spmm_batch(sgs, sbx, sby, 1, 50)
snb = sum(spmv_bytes(a.num_rows, a.num_cols, a.num_nonzeros) for a in scs) / len(scs)
x0 = np.random.default_rng(3).uniform(0, 1, scs[0].num_cols)
y = sgs[0].spmv(x0)
lens = np.diff(scs[0].row_offsets)
rows = np.repeat(np.arange(scs[0].num_rows), lens)
ref = np.zeros(scs[0].num_rows)
np.add.at(ref, rows, scs[0].values * x0[scs[0].column_indices])
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("MSPMV_")},
                  "kernel": sgs[0].kernel_name(), "kernel_us": round(sk * 1e3, 2),
                  "frac": round(snb / sk / 1e6 / HBM_PEAK_GBS, 4),
                  "max_rel_err": float(np.max(np.abs(y - ref)) / np.max(np.abs(ref)))}), flush=True)
