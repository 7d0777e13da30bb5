#!/usr/bin/env python3
"""Per-iteration cost of the preconditioned block CGs on the parabolic_fem shape (m = 525,825),
GPU vs the oracle restatement on the host cores (measurement tool, not product).

    python tools/pcg_probe.py [L] [iters]

Prints one JSON line: setup seconds (host SPAI / IC(0)), GPU ms per iteration of CG, SPAI-PCG
and IC(0)-PCG (fixed iteration count, tolerance 0), and the oracle's ms per iteration.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd"), os.path.join(ROOT, "tests")]

import mspmv  # noqa: E402
from _oracle import Oracle  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    its = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    a = mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)
    n = a.num_rows
    B = np.random.default_rng(1).uniform(0, 1, (n, L))
    out = {"m": n, "nnz": a.num_nonzeros, "L": L, "iters": its}
    t0 = time.perf_counter()
    mv = mspmv.spai_values(a)
    out["spai_setup_s"] = round(time.perf_counter() - t0, 3)
    t0 = time.perf_counter()
    l, shift = mspmv.ic0_factor(a)
    out["ic0_setup_s"] = round(time.perf_counter() - t0, 3)
    out["ic0_shift"] = shift
    m = mspmv.CsrMatrix.from_arrays(n, a.row_offsets, a.column_indices, mv)
    with mspmv.GpuCsr(a) as ga, mspmv.GpuCsr(m) as gm, mspmv.GpuIc0(l) as ic:
        dB = mspmv.DeviceBuffer.from_array(B)
        dX = mspmv.DeviceBuffer(8 * n * L)
        for name, fn in (("cg", lambda: ga.cg_dev(dB, dX, L, its, 0.0)),
                         ("spai_pcg", lambda: ga.pcg_spai_dev(gm, dB, dX, L, its, 0.0)),
                         ("ic0_pcg", lambda: mspmv.lib.mspmv_dpcg_ic0_multi_dev(ga.h, ic.h, dB.ptr, dX.ptr, L, its,
                                                                               0.0, mspmv.MERGE, None, None, 0))):
            fn()
            t0 = time.perf_counter()
            fn()
            out[f"gpu_{name}_ms_per_iter"] = round((time.perf_counter() - t0) / its * 1e3, 3)
    orc = Oracle()
    k = max(2, its // 10)
    t0 = time.perf_counter()
    orc.pcg_ic0_multi(a, l.row_offsets, l.column_indices, l.values, B, k, 0.0)
    out["oracle_ic0_pcg_ms_per_iter"] = round((time.perf_counter() - t0) / k * 1e3, 2)
    t0 = time.perf_counter()
    orc.pcg_spai_multi(a, mv, B, k, 0.0)
    out["oracle_spai_pcg_ms_per_iter"] = round((time.perf_counter() - t0) / k * 1e3, 2)
    out["oracle_threads"] = orc.lib.orc_max_threads()
    # iterations to 1e-8 on the GPU (convergence benefit of each preconditioner)
    with mspmv.GpuCsr(a) as ga, mspmv.GpuCsr(m) as gm, mspmv.GpuIc0(l) as ic:
        _, it_cg, _, _ = ga.cg_multi(B, 5000, 1e-8)
        _, it_spai, _, _ = ga.pcg_spai(gm, B, 5000, 1e-8)
        _, it_ic0, _, _ = mspmv.pcg_ic0(ga, ic, B, 5000, 1e-8)
    out["iters_to_1e-8"] = {"cg": it_cg, "spai_pcg": it_spai, "ic0_pcg": it_ic0}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
