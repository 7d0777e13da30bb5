"""Lab: per-tile phase stamps of the SpMV tile kernel (MSPMV_LAB_ABLATE=9 build), one cold launch."""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv
shape = os.environ.get("STAMP_SHAPE", "fem")
gs, dx, dy = [], [], []
for i in range(4):
    if shape == "fem":
        a = mspmv.CsrMatrix.synth_fem_blocked(217918, 11524432, 6, 1700, seed=1 + i)
    else:
        a = mspmv.CsrMatrix.synth_stencil(1, 160 * 135 * 164, 160, 135, 164, seed=1 + i, diag_shift=1e-2)
    gs.append(mspmv.GpuCsr(a))
    dx.append(mspmv.DeviceBuffer.from_array(np.random.default_rng(i).uniform(0, 1, a.num_cols)))
    dy.append(mspmv.DeviceBuffer(8 * a.num_rows))
step, kern, _ = mspmv.time_spmm_batch(gs, dx, dy, 1, 3)
T = gs[-1].tile_plan(1)["num_tiles"]
T = min(T, 1 << 17)
buf = np.zeros(T * 6, np.uint64)
rc = mspmv.lib.mspmv_lab_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), T)
s = buf.reshape(T, 6).astype(np.int64)
t0 = s[:, 0].min()
tt = (s[:, :4] - t0) / 100.0  # 100 MHz -> us
d_stream = tt[:, 1] - tt[:, 0]
d_rend = tt[:, 2] - tt[:, 1]
d_red = tt[:, 3] - tt[:, 2]
tot = tt[:, 3] - tt[:, 0]
pct = lambda v: [round(float(np.percentile(v, q)), 2) for q in (10, 50, 90)]
out = {"rc": rc, "tiles": T, "kernel_ms_batch_avg": kern, "span_us": round(float(tt[:, 3].max()), 2),
       "stream_gather_us_p10_50_90": pct(d_stream), "rowend_us": pct(d_rend), "reduce_us": pct(d_red),
       "tile_total_us": pct(tot), "start_us": pct(tt[:, 0]), "end_us": pct(tt[:, 3]),
       "cus": int(len(np.unique(s[:, 4])))}
# concurrency profile: WGs resident per 1-us bin, and per phase
bins = np.arange(0, np.ceil(tt[:, 3].max()) + 1, 1.0)
act = [int(((tt[:, 0] <= b + 0.5) & (tt[:, 3] > b + 0.5)).sum()) for b in bins]
inst = [int(((tt[:, 0] <= b + 0.5) & (tt[:, 1] > b + 0.5)).sum()) for b in bins]
out["resident_per_us"] = act
out["in_stream_gather_per_us"] = inst
print(json.dumps(out))
