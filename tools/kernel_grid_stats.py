#!/usr/bin/env python3
"""Per-(kernel, grid) duration statistics from a rocprofv3 --kernel-trace CSV.

    python tools/kernel_grid_stats.py <run>_kernel_trace.csv OUT.csv [--json OUT.json]

rocprofv3's own --stats summary averages every launch of one kernel instantiation together, so a
kernel launched on matrices of different sizes (the headline pwtk shape, the nlpkkt120 shape, the
stress shape) shows one meaningless mean.  This splits the trace by (kernel, grid size): one row per
launch geometry, with calls, total/avg/median/min/max duration in microseconds, LDS bytes and VGPRs.
Rows are sorted by total time.  bench.py's per-launch kernel_ms for a leg is compared with the
matching row's avg (tools/recompute_frac.py).
"""
import collections
import csv
import json
import statistics
import sys


def short_name(name):
    n = name.replace("void ", "").replace("mspmv::", "").replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace(" ", "")


def grid_stats(trace_csv):
    """Rows per (kernel, grid, after_flush).  after_flush = 1 marks launches whose preceding
    dispatch was bench's 512 MiB MALL-flush kernel (k_flush): the cold launches of a hot/cold
    measurement, kept apart from the hot ones."""
    groups = collections.defaultdict(list)
    meta, first = {}, {}
    recs = [r for r in csv.DictReader(open(trace_csv)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    recs.sort(key=lambda r: int(r["Dispatch_Id"]))
    prev = ""
    for r in recs:
        k = short_name(r["Kernel_Name"])
        key = (k, int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]), int(prev in ("k_flush", "k_flush_read")))
        prev = k.split("<")[0]
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
        first.setdefault(key, int(r["Dispatch_Id"]))
        meta[key] = (int(r["Workgroup_Size_X"]), int(r["LDS_Block_Size"]), int(r["VGPR_Count"]),
                     int(r.get("Accum_VGPR_Count", 0) or 0))
    rows = []
    for (k, grid, cold), d in groups.items():
        wg, lds, vgpr, agpr = meta[(k, grid, cold)]
        rows.append({"kernel": k, "grid": grid, "after_flush": cold, "workgroups": grid // max(wg, 1),
                     "workgroup_size": wg,
                     "lds_bytes": lds, "vgpr": vgpr, "agpr": agpr, "calls": len(d),
                     "total_us": round(sum(d), 3), "avg_us": round(sum(d) / len(d), 3),
                     "median_us": round(statistics.median(d), 3), "min_us": round(min(d), 3),
                     "max_us": round(max(d), 3), "first_dispatch": first[(k, grid, cold)]})
    rows.sort(key=lambda r: -r["total_us"])
    return rows


def main(argv):
    if len(argv) < 3:
        raise SystemExit(__doc__)
    rows = grid_stats(argv[1])
    with open(argv[2], "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) if rows else ["kernel"])
        w.writeheader()
        w.writerows(rows)
    if "--json" in argv:
        json.dump(rows, open(argv[argv.index("--json") + 1], "w"), indent=1)
    for r in rows[:12]:
        print(f"{r['kernel'][:60]:60s} grid {r['grid']:>9d}{' cold' if r['after_flush'] else '     '} calls {r['calls']:>6d} "
              f"avg {r['avg_us']:>10.3f} us  median {r['median_us']:>10.3f} us")


if __name__ == "__main__":
    main(sys.argv)
