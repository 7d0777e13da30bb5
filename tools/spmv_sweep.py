#!/usr/bin/env python3
"""A/B sweep of SpMV tile variants on the bench workload (pwtk-shaped batch, cold per launch).

    python tools/spmv_sweep.py                 # parent: runs every variant in child processes
    python tools/spmv_sweep.py --child         # child: one timing line for the env's variant

Variants are selected with MSPMV_SPMV_IPT / _NT / _PERSIST / _BPC / _RG_COST (read once per process), so each
runs in its own process; rounds alternate variants to spread device drift.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]


def child():
    import numpy as np
    import mspmv
    B = int(os.environ.get("SWEEP_BATCH", "4"))
    L = int(os.environ.get("SWEEP_L", "1"))
    gs, dx, dy = [], [], []
    for i in range(B):
        shape = os.environ.get("SWEEP_SHAPE", "fem")
        if shape == "fem":
            a = mspmv.CsrMatrix.synth_fem_blocked(217918, 11524432, 6, 1700, seed=1 + i)
        elif shape == "nlpkkt":   # nlpkkt120-sized 27-point stencil (the cg_multi workload)
            a = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, seed=1 + i, diag_shift=1e-2)
        elif shape == "powerlaw":
            a = mspmv.CsrMatrix.synth_powerlaw(1 << 20, 1 << 20, 11524432, 1.8, seed=1 + i)
        else:
            a = mspmv.CsrMatrix.synth_banded(217918, 11524432, 10000, seed=1 + i)
        gs.append(mspmv.GpuCsr(a))
        dx.append(mspmv.DeviceBuffer.from_array(np.random.default_rng(i).uniform(0, 1, a.num_cols * L)))
        dy.append(mspmv.DeviceBuffer(8 * a.num_rows * L))
    mspmv.time_spmm_batch(gs, dx, dy, L, 5)
    step, kern, _ = mspmv.time_spmm_batch(gs, dx, dy, L, 50)
    hot_step, hot_kern, _ = mspmv.time_spmm_batch(gs[:1], dx[:1], dy[:1], L, 200)
    a0 = gs[0]
    nbytes = 12 * a0.num_nonzeros + 4 * (a0.num_rows + 1) + 8 * L * (a0.num_rows + a0.num_cols)
    modes = np.bincount(a0.tile_plan(L)["modes"], minlength=8).tolist()
    print(json.dumps({"ipt": os.environ.get("MSPMV_SPMV_IPT"), "nt": os.environ.get("MSPMV_SPMV_NT"),
                      "persist": os.environ.get("MSPMV_SPMV_PERSIST"), "bpc": os.environ.get("MSPMV_SPMV_BPC"),
                      "rg": os.environ.get("MSPMV_SPMV_RG_COST"), "iptg": os.environ.get("MSPMV_SPMM_IPTG"), "L": L, "shape": shape, "modes": modes,
                      "cold_kernel_us": round(kern * 1e3, 2), "cold_GBps": round(nbytes / kern / 1e6, 1),
                      "step_us": round(step * 1e3, 2), "hot_kernel_us": round(hot_kern * 1e3, 2),
                      "hot_GBps": round(nbytes / hot_kern / 1e6, 1)}), flush=True)


def parent():
    spec = os.environ.get("SWEEP_VARIANTS", "8:1:0:0:0,8:1:0:0:48")   # ipt:nt:persist:bpc[:rg_cost[:spmm_iptg]]
    variants = []
    for v in spec.split(","):
        f = [int(x) for x in v.split(":")]
        variants.append(tuple(f + [48, 0][len(f) - 4:]) if len(f) < 6 else tuple(f[:6]))
    rounds = int(os.environ.get("SWEEP_ROUNDS", "2"))
    for r in range(rounds):
        for ipt, nt, persist, bpc, rg, iptg in variants:
            env = dict(os.environ, MSPMV_SPMV_IPT=str(ipt), MSPMV_SPMV_NT=str(nt), MSPMV_SPMV_PERSIST=str(persist),
                       MSPMV_SPMV_BPC=str(bpc), MSPMV_SPMV_RG_COST=str(rg), MSPMV_SPMM_RG_COST=str(rg if rg <= 0 else -1),
                       MSPMV_SPMM_IPTG=str(iptg))
            out = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode != 0:
                print(f"variant ipt={ipt} nt={nt} persist={persist} failed rc={out.returncode}: {out.stderr[-500:]}", flush=True)
                sys.exit(out.returncode)
            print(f"round {r} " + out.stdout.strip(), flush=True)


if __name__ == "__main__":
    child() if "--child" in sys.argv else parent()
