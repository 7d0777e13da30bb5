#!/usr/bin/env python3
"""Lab: phase stamps of the sliced-ELL SpMV on bench's power-law leg (and the scattered band), from the stamped lab
library (tools/lab/sell_stamps_build.sh; run with MSPMV_LIB=tools/lab/libmspmv_sellstamps.so).  Thread 0 of each
block records wall_clock64() (100 MHz) at entry, per segment after the x stage, after its wave's long pieces and after
its wave's slices, and at exit.  Prints one JSON line per matrix: the span, the per-block phase medians and the
slowest block's breakdown (us)."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

NS, NB = 20, 1024
fn = mspmv.lib.mspmv_lab_sell_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
fn.restype = ctypes.c_int


def stamps():
    buf = (ctypes.c_ulonglong * (NS * NB))()
    assert fn(buf, NS * NB) == NS * NB
    return np.frombuffer(buf, dtype=np.uint64).reshape(NB, NS).astype(np.int64)


def analyse(name, a):
    x = np.random.default_rng(3).uniform(-1, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        for _ in range(6):
            stamps()  # cleared: the last launch's stamps only
            g.spmv(x)
        S = stamps()
        kname = g.kernel_name()
    used = S[:, 0] > 0
    S = S[used]
    t0 = S[:, 0].min()
    us = lambda v: float(v) / 100.0  # noqa: E731
    end = S[:, 19] - t0
    rows = []
    for s in S:
        segs = [i for i in range(6) if s[1 + 3 * i] > 0]
        r = {"entry": us(s[0] - t0), "first_stage": us(s[1] - s[0]), "segments": len(segs),
             "long": us(sum(s[2 + 3 * i] - s[1 + 3 * i] for i in segs)),
             "slices": us(sum(s[3 + 3 * i] - s[2 + 3 * i] for i in segs)),
             "stage_waits": us(sum(s[1 + 3 * i] - s[3 + 3 * (i - 1)] for i in segs if i > 0)),
             "tail": us(s[19] - s[3 + 3 * segs[-1]]) if segs else 0.0, "end": us(s[19] - t0)}
        rows.append(r)
    keys = ["entry", "first_stage", "long", "slices", "stage_waits", "tail", "end"]
    med = {k: round(float(np.median([r[k] for r in rows])), 2) for k in keys}
    mean = {k: round(float(np.mean([r[k] for r in rows])), 2) for k in keys}
    slow = max(rows, key=lambda r: r["end"])
    print(json.dumps({"matrix": name, "kernel": kname, "blocks": len(rows), "span_us": us(end.max()),
                      "end_p10_p50_p90": [round(us(np.percentile(end, q)), 2) for q in (10, 50, 90)],
                      "median": med, "mean": mean,
                      "slowest": {k: (round(v, 2) if isinstance(v, float) else v) for k, v in slow.items()}}), flush=True)


analyse("powerlaw", mspmv.CsrMatrix.synth_powerlaw(217918, 217918, 11524432, 1.2, 3))
analyse("scatter_band", mspmv.CsrMatrix.synth_banded(217918, 11524432, 10000, seed=77))
