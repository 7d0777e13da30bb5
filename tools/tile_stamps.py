#!/usr/bin/env python3
"""Per-tile phase stamps of the merge-tile SpMV on the configs[0] / configs[1] small shapes (cant, rma10):
where a tile's life goes.

mspmv_spmv_tile_stamps runs one plain SpMV through the stamped instantiation of k_spmv_tile (thread 0
records wall_clock64(), 100 MHz, at: 0 entry, 1 stream and x gathers issued, 2 products in LDS, 3 row
ends in LDS, 4 rows stored; 5 = the CU's HW_ID).  For each shape, after a warm run and after a 512 MiB
flush (cold, as the bench prices the fraction), this prints one JSON object: tile count, the span from
the first tile's entry to the last tile's end, tile-lifetime quantiles, the median of each phase, the
resident-tile profile over the span (how many tiles are live at once, per 1 us), and the tail after the
last tile entered.
The stamped instantiation is held to the production kernel's 8 workgroups per CU (amdgpu_waves_per_eu(8):
64 VGPRs, no spills; round 6's first stamped build held 70 VGPRs and ran 7 per CU, so its cant profile had
196 tiles in a second generation the production kernel does not have).  Dictionary tiles stage in one pass
and record no stamp 1: their "issue" phase is 0 and "stream_and_gathers_land" covers entry -> products in LDS.
  usage: python tools/tile_stamps.py [--device D] [--reps N]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd"), ROOT]

import mspmv  # noqa: E402

SHAPES = {"cant": dict(m=62451, nnz=4007383, band=2000, seed=1),   # bench.py CANT
          "rma10": dict(m=46835, nnz=2374001, band=3000, seed=2)}  # bench.py RMA10
TICK_US = 0.01  # wall_clock64: 100 MHz


def analyse(st):
    t0 = st[:, 0].astype(np.int64)
    st = st.copy()
    no_issue = st[:, 1] == 0  # dictionary tiles stage in one pass (no stamp 1): entry -> products in LDS whole
    st[no_issue, 1] = st[no_issue, 0]
    ph = np.diff(st[:, :5].astype(np.int64), axis=1) * TICK_US  # [tiles][4] us
    life = (st[:, 4].astype(np.int64) - t0) * TICK_US
    start, end = int(t0.min()), int(st[:, 4].max())
    span = (end - start) * TICK_US
    grid = np.arange(start, end, 100)  # 1 us steps
    live = [int(np.sum((t0 <= g) & (st[:, 4].astype(np.int64) > g))) for g in grid]
    last_entry = (int(t0.max()) - start) * TICK_US
    cus = len(np.unique(st[:, 5] & 0xFFFF))
    return {"tiles": int(st.shape[0]), "tiles_without_issue_stamp": int(no_issue.sum()), "cus_seen": cus,
            "max_resident": int(max(live)) if live else 0, "span_us": round(span, 2),
            "tile_life_us": {q: round(float(np.percentile(life, p)), 2) for q, p in
                             (("p10", 10), ("median", 50), ("p90", 90), ("max", 100))},
            "phase_median_us": {"issue": round(float(np.median(ph[:, 0])), 2),
                                "stream_and_gathers_land": round(float(np.median(ph[:, 1])), 2),
                                "row_ends_and_barrier": round(float(np.median(ph[:, 2])), 2),
                                "reduce_and_store": round(float(np.median(ph[:, 3])), 2)},
            "last_tile_entry_us": round(last_entry, 2), "tail_after_last_entry_us": round(span - last_entry, 2),
            "resident_tiles_per_us": live}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = args.device
    for name, sh in SHAPES.items():
        a = mspmv.CsrMatrix.synth_banded(sh["m"], sh["nnz"], sh["band"], seed=sh["seed"])
        x = np.random.default_rng(2).uniform(0.0, 1.0, a.num_cols)
        with mspmv.GpuCsr(a, device=dev) as g:
            dx, dy = mspmv.DeviceBuffer.from_array(x, dev), mspmv.DeviceBuffer(8 * a.num_rows, dev)
            g.time_spmm(dx, dy, 1, 5)
            _, hot, _ = g.time_spmm(dx, dy, 1, 100)
            _, cold, _ = g.time_spmm(dx, dy, 1, 80, 512 << 20)
            out = {"shape": name, "kernel": g.kernel_name(), "hot_kernel_us": round(hot * 1e3, 2),
                   "cold_kernel_us": round(cold * 1e3, 2), "warm": [], "cold": []}
            for _ in range(args.reps):
                out["warm"].append(analyse(g.spmv_tile_stamps(dx, dy)))
                out["cold"].append(analyse(g.spmv_tile_stamps(dx, dy, 512 << 20)))
            dx.free()
            dy.free()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
