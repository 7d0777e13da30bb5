#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py gpurun_out/<tag> profiles/<round>_pmc_traffic.json        (bench headline)
    python tools/pmc_traffic.py --leg gpurun_out/<tag>/<leg> profiles/<round>_<leg>_pmc_traffic.json

FETCH_SIZE and WRITE_SIZE (KB, separate passes: they do not fit one TCC pass) are averaged per
dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE tallies 128-B
memory-side read requests at 64 B, so it reads exactly half of a streaming read -> doubled here;
WRITE_SIZE is taken as is.  "kernels" (keyed by full kernel name, every launch geometry together) is
what bench.py's pmc_traffic() matches for the headline; "by_grid" splits each kernel by grid size
(one row per matrix shape it ran on).
"""
import collections
import csv
import glob
import json
import os
import sys


def per_dispatch(path, counter, by_grid=False):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    grid = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        key = (r["Kernel_Name"], int(r["Grid_Size"])) if by_grid else r["Kernel_Name"]
        tot[key] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
        grid[key] = int(r["Grid_Size"])
    return {k: (tot[k] * 1024.0 / len(disp[k]), len(disp[k]), grid[k]) for k in tot}


def _csv(d):
    hits = sorted(glob.glob(os.path.join(d, "*counter_collection.csv")))
    if not hits:
        raise SystemExit(f"no counter_collection.csv under {d}")
    return hits[0]


def summarize(fetch_csv, write_csv):
    out = {"correction": "fetch_bytes = 2 x FETCH_SIZE (gfx950 half-count); write_bytes = WRITE_SIZE",
           "kernels": {}, "by_grid": []}
    for by_grid in (False, True):
        f = per_dispatch(fetch_csv, "FETCH_SIZE", by_grid)
        w = per_dispatch(write_csv, "WRITE_SIZE", by_grid)
        for k in sorted(f):
            fb = 2.0 * f[k][0]
            wb = w.get(k, (0.0, 0, 0))[0]
            row = {"dispatches": f[k][1], "grid": f[k][2], "fetch_bytes": round(fb), "write_bytes": round(wb),
                   "traffic_bytes": round(fb + wb)}
            if by_grid:
                out["by_grid"].append({"kernel": k[0], **row})
            else:
                out["kernels"][k] = row
    return out


def main(argv):
    if len(argv) >= 4 and argv[1] == "--leg":
        src, dst = argv[2], argv[3]
        out = {"source": src, **summarize(_csv(os.path.join(src, "pmc_fetch")), _csv(os.path.join(src, "pmc_write")))}
    elif len(argv) >= 3:
        src, dst = argv[1], argv[2]
        out = {"source": src, **summarize(os.path.join(src, "pmc_fetch", "bench_counter_collection.csv"),
                                          os.path.join(src, "pmc_write", "bench_counter_collection.csv"))}
        bench = json.loads(open(os.path.join(src, "pmc_fetch.json")).read().strip().splitlines()[-1])
        out["bench_bytes_per_launch"] = bench["roofline"]["bytes_per_launch"]
        out["bench_kernel"] = bench["roofline"]["kernel"]
    else:
        raise SystemExit(__doc__)
    json.dump(out, open(dst, "w"), indent=1)
    for r in out["by_grid"]:
        print(f"{r['kernel'].split('(')[0][:70]:70s} grid {r['grid']:>9d} x{r['dispatches']:<5d} "
              f"traffic {r['traffic_bytes'] / 1e6:10.3f} MB/launch")


if __name__ == "__main__":
    main(sys.argv)
