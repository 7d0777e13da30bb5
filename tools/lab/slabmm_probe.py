#!/usr/bin/env python3
"""Column-slab SpMM A/B probe: configs[2]'s cant-shaped L = 16 SpMM (hot and cold), configs[4]'s
nlpkkt120-size L = 8 SpMM (hot) and its CGSolveMultiple ms per iteration, one JSON line.  The variant is
chosen by the environment (MSPMV_SPMM_SLAB, MSPMV_SPMM_SLAB_CFG)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

FLUSH = 512 << 20
what = sys.argv[1] if len(sys.argv) > 1 else "all"
out = {"env": {k: v for k, v in os.environ.items() if k.startswith("MSPMV_")}}
if what in ("all", "cant"):
    a = mspmv.CsrMatrix.synth_banded(62451, 4007383, 2000, seed=1)
    L = 16
    nb = 12 * a.num_nonzeros + 4 * (a.num_rows + 1) + 8 * L * (a.num_cols + a.num_rows)
    with mspmv.GpuCsr(a) as g:
        X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, L))
        dX, dY = mspmv.DeviceBuffer.from_array(X), mspmv.DeviceBuffer(8 * a.num_rows * L)
        t0 = time.perf_counter()
        g.time_spmm(dX, dY, L, 5)
        out["cant_setup_s"] = round(time.perf_counter() - t0, 3)
        _, hot, _ = g.time_spmm(dX, dY, L, 100)
        _, cold, _ = g.time_spmm(dX, dY, L, 80, FLUSH)
        out["cant_L16_kernel"] = g.spmm_kernel_name(L)
        out["cant_L16_hot_us"] = round(hot * 1e3, 2)
        out["cant_L16_cold_us"] = round(cold * 1e3, 2)
        out["cant_L16_frac"] = round(nb / cold / 1e6 / 8000.0, 4)
        for b in (dX, dY):
            b.free()
if what in ("all", "nlpkkt"):
    nk = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2)
    n, L = nk.num_rows, 8
    B = np.random.default_rng(42).uniform(0, 1, (n, L))
    thr = float(np.sqrt(np.sum(B.reshape(-1)[:n] ** 2)) * 1e-5)
    with mspmv.GpuCsr(nk) as g:
        dB, dX, dY = mspmv.DeviceBuffer.from_array(B), mspmv.DeviceBuffer(8 * n * L), mspmv.DeviceBuffer(8 * n * L)
        t0 = time.perf_counter()
        g.time_spmm(dB, dY, L, 3)
        out["nlpkkt_setup_s"] = round(time.perf_counter() - t0, 3)
        _, kms, _ = g.time_spmm(dB, dY, L, 20)
        out["nlpkkt_L8_us"] = round(kms * 1e3, 1)
        out["nlpkkt_L8_kernel"] = g.spmm_kernel_name(L)
        if os.environ.get("MSPMV_SLAB_LAB"):  # ablations break the product: no CG
            print(json.dumps(out), flush=True)
            sys.exit(0)
        g.cg_dev(dB, dX, L, 50000, thr)
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            it, _, st = g.cg_dev(dB, dX, L, 50000, thr)
            el = time.perf_counter() - t0
            best = el / it if best is None else min(best, el / it)
        out["cg_iters"] = it
        out["cg_status"] = st
        out["cg_ms_per_iter"] = round(best * 1e3, 4)
        bytes_it = 12 * nk.num_nonzeros + 4 * (n + 1) + 88 * n * L
        out["cg_frac"] = round(bytes_it / best / 1e9 / 8000.0, 4)
        for b in (dB, dX, dY):
            b.free()
print(json.dumps(out), flush=True)
