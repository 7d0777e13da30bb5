"""Lab: single / multi CG history and timing against the batch size (MSPMV_CG_BATCH is read once per
process, so each K runs in its own child process).  usage: python tools/lab/cg_batch_probe.py [K...]"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import hashlib, json, sys, time
import numpy as np
sys.path[:0] = [sys.argv[1] + "/sparse-matrix-linear-equations_amd", sys.argv[1] + "/tests", sys.argv[1]]
import mspmv
import bench
out = {}
pf = mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)
b = bench.glibc_rhs(42, pf.num_rows)
thr = float(np.sqrt(np.sum(b * b)) * 1e-5)
with mspmv.GpuCsr(pf) as g:
    for rep in range(2):
        x, it, h, st = g.cg_single(b, 10000, thr, hist_cap=10000)
        out[f"single{rep}"] = [it, hashlib.md5(h.tobytes()).hexdigest()[:12], hashlib.md5(x.tobytes()).hexdigest()[:12]]
    db, dx = mspmv.DeviceBuffer.from_array(b, 0), mspmv.DeviceBuffer(8 * pf.num_rows, 0)
    g.cg_dev(db, dx, 1, 10000, thr)
    t0 = time.perf_counter(); it, _, _ = g.cg_dev(db, dx, 1, 10000, thr); el = time.perf_counter() - t0
    out["single_us_per_iter"] = round(el / it * 1e6, 2)
nk = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, diag_shift=1e-2)
B = np.random.default_rng(42).uniform(0, 1, (nk.num_rows, 8))
thr = float(np.sqrt(np.sum(B.reshape(-1)[:nk.num_rows] ** 2)) * 1e-5)
with mspmv.GpuCsr(nk) as g:
    dB, dX = mspmv.DeviceBuffer.from_array(B, 0), mspmv.DeviceBuffer(8 * nk.num_rows * 8, 0)
    g.cg_dev(dB, dX, 8, 50000, thr)
    t0 = time.perf_counter(); it, h, st = g.cg_dev(dB, dX, 8, 50000, thr, hist_cap=1000); el = time.perf_counter() - t0
    out["multi"] = [it, hashlib.md5(h.tobytes()).hexdigest()[:12], round(el / it * 1e3, 4)]
print(json.dumps(out))
'''


def main(ks):
    for k in ks:
        env = dict(os.environ, MSPMV_CG_BATCH=str(k))
        r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
        print(f"K={k}", r.stdout.strip() or r.stderr[-800:], flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main([int(v) for v in sys.argv[1:]] or [32, 18, 8, 4, 2])
