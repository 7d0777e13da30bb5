#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from the rocprofv3 PMC passes of tools/gpu_session.sh.

    python tools/pmc_traffic.py gpurun_out/<tag> profiles/<round>_pmc_traffic.json

FETCH_SIZE and WRITE_SIZE (KB, separate passes: they do not fit one TCC pass) are averaged
per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE
tallies 128-B memory-side read requests at 64 B, so it reads exactly half of a streaming read
-> doubled here; WRITE_SIZE is taken as is.  bench.py reports the result as roofline.traffic
for the kernel and bytes_per_launch it was collected on.
"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    grid = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        tot[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        grid[k] = int(r["Grid_Size"])
    return {k: (tot[k] * 1024.0 / len(disp[k]), len(disp[k]), grid[k]) for k in tot}


def main(src, dst):
    f = per_dispatch(os.path.join(src, "pmc_fetch", "bench_counter_collection.csv"), "FETCH_SIZE")
    w = per_dispatch(os.path.join(src, "pmc_write", "bench_counter_collection.csv"), "WRITE_SIZE")
    bench = json.loads(open(os.path.join(src, "pmc_fetch.json")).read().strip().splitlines()[-1])
    out = {"source": src, "correction": "fetch_bytes = 2 x FETCH_SIZE (gfx950 half-count); write_bytes = WRITE_SIZE",
           "bench_bytes_per_launch": bench["roofline"]["bytes_per_launch"],
           "bench_kernel": bench["roofline"]["kernel"], "kernels": {}}
    for k in sorted(f):
        fb = 2.0 * f[k][0]
        wb = w.get(k, (0.0, 0, 0))[0]
        out["kernels"][k] = {"dispatches": f[k][1], "grid": f[k][2], "fetch_bytes": round(fb),
                             "write_bytes": round(wb), "traffic_bytes": round(fb + wb)}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
