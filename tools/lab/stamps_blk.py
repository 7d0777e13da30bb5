"""Lab: per-chunk phase stamps of k_spmm_blk (MSPMV_LAB_ABLATE=10 build, MSPMV_LIB=...), pwtk shape,
L = 16, one hot and one cold launch: per chunk (a wave's run chunk) the time to its values (fetch),
through its passes (gathers + FMAs), through the reduce-scatter; concurrency per microsecond."""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]
import mspmv
L = int(os.environ.get("STAMP_L", "16"))
a = mspmv.CsrMatrix.synth_fem_blocked(217918, 11524432, 6, 1700, seed=1)
fn = mspmv.lib.mspmv_lab_blk_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
with mspmv.GpuCsr(a) as g:
    X = np.random.default_rng(3).uniform(0, 1, (a.num_cols, L))
    dX, dY = mspmv.DeviceBuffer.from_array(X), mspmv.DeviceBuffer(8 * a.num_rows * L)
    T = g.tile_plan(1)["num_tiles"]
    res = {"tiles": T}
    for mode, flush in (("hot", 0), ("cold", 512 << 20)):
        g.time_spmm(dX, dY, L, 3)
        _, ms, _ = g.time_spmm(dX, dY, L, 1, flush)
        S = min(T * 8, 1 << 16)
        buf = np.zeros(S * 8, np.uint64)
        rc = fn(buf.ctypes.data, S)
        s = buf.reshape(S, 8).astype(np.int64)
        ok = s[:, 0] > 0
        s = s[ok]
        t0 = s[:, 0].min()
        tt = (s[:, :4] - t0) / 100.0
        pct = lambda v: [round(float(np.percentile(v, q)), 2) for q in (10, 50, 90)]
        r = {"rc": rc, "kernel_ms": ms, "chunks": int(ok.sum()), "span_us": round(float(tt[:, 3].max()), 2),
             "fetch_us": pct(tt[:, 1] - tt[:, 0]), "passes_us": pct(tt[:, 2] - tt[:, 1]),
             "reduce_us": pct(tt[:, 3] - tt[:, 2]), "chunk_us": pct(tt[:, 3] - tt[:, 0]),
             "wc": pct(s[:, 5] & 255), "h": pct((s[:, 5] >> 8) & 255), "nd": pct((s[:, 5] >> 16) & 255)}
        bins = np.arange(0, np.ceil(tt[:, 3].max()) + 1, 1.0)
        r["chunks_active_per_us"] = [int(((tt[:, 0] <= b + 0.5) & (tt[:, 3] > b + 0.5)).sum()) for b in bins]
        r["in_fetch_per_us"] = [int(((tt[:, 0] <= b + 0.5) & (tt[:, 1] > b + 0.5)).sum()) for b in bins]
        # gap between a wave slot's first chunk end and its second chunk start (same tile, same slot)
        res[mode] = r
print(json.dumps(res))
