#!/usr/bin/env python3
"""Per-iteration cost of the CG paths on the bench's CG workloads, for A/B runs of tile
variants (each variant in its own process: the MSPMV_SPMV_* tuning is read once).

    python tools/cg_probe.py            # parent: PROBE_VARIANTS="ipt:rg,..." (default 8:48,4:48,2:48)
    python tools/cg_probe.py --child    # one line for the environment's variant

Reports the SpMV kernel time on the parabolic_fem-shaped matrix (time_spmm, events) and the
wall time per CG iteration at a fixed iteration count (tolerance 0, 300 iterations).
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]


def child():
    import numpy as np
    import mspmv
    which = os.environ.get("PROBE_SHAPE", "parabolic")
    if which == "parabolic":
        a = mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)
        L = 1
    else:
        a = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2)
        L = 8
    n = a.num_rows
    out = {"ipt": os.environ.get("MSPMV_SPMV_IPT"), "rg": os.environ.get("MSPMV_SPMV_RG_COST"),
           "iptg": os.environ.get("MSPMV_SPMM_IPTG"), "shape": which, "L": L}
    with mspmv.GpuCsr(a) as g:
        dx = mspmv.DeviceBuffer.from_array(np.random.default_rng(1).uniform(0, 1, n * L))
        dy = mspmv.DeviceBuffer(8 * n * L)
        g.time_spmm(dx, dy, L, 20)
        call_ms, kern_ms, _ = g.time_spmm(dx, dy, L, 200)
        out["spmv_call_us"] = round(call_ms * 1e3, 2)
        out["spmv_kernel_us"] = round(kern_ms * 1e3, 2)
        out["tiles"] = g.tile_plan(L)["num_tiles"]
        db = mspmv.DeviceBuffer.from_array(np.random.default_rng(2).uniform(0, 1, n * L))
        g.cg_dev(db, dy, L, 50, 0.0)
        t0 = time.perf_counter()
        it, _, st = g.cg_dev(db, dy, L, 300, 0.0)
        el = time.perf_counter() - t0
        out["cg_iters"] = it
        out["cg_us_per_iter"] = round(el / max(it, 1) * 1e6, 2)
    print(json.dumps(out), flush=True)


def parent():
    spec = os.environ.get("PROBE_VARIANTS", "8:48,4:48,2:48")   # ipt:rg[:spmm_iptg]
    for v in spec.split(","):
        f = v.split(":")
        env = dict(os.environ, MSPMV_SPMV_IPT=f[0], MSPMV_SPMV_RG_COST=f[1], MSPMV_SPMM_IPTG=f[2] if len(f) > 2 else "0")
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(f"variant {v} failed rc={r.returncode}: {r.stderr[-400:]}", flush=True)
            sys.exit(r.returncode)
        print(r.stdout.strip(), flush=True)


if __name__ == "__main__":
    child() if "--child" in sys.argv else parent()
