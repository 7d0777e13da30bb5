#!/usr/bin/env python3
"""Summarise tools/pmc_passes.sh output (one rocprofv3 --pmc run per pass) as a markdown table:
per kernel instantiation, every counter's per-dispatch average over the run's dispatches, and the
derived ratios used in DESIGN.md (wave wait fraction, instruction mix per wave, L2 read latency,
L2 hit rate, HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE per MI355X_MICROARCH.md's gfx950 note).

  python3 tools/counter_summary.py gpurun_out/TAG/counters_LEG [--kernel REGEX] [--title TEXT]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def load(outdir):
    """{kernel: {counter: [per-dispatch values]}} over every pass directory."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    meta = {}
    for path in sorted(glob.glob(os.path.join(outdir, "pass*", "*counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                per[k][row["Counter_Name"]][(path, row["Dispatch_Id"])] += float(row["Counter_Value"])
                meta[k] = (row.get("VGPR_Count"), row.get("Accum_VGPR_Count"), row.get("SGPR_Count"),
                           row.get("LDS_Block_Size"), row.get("Grid_Size"))
    out = {}
    for k, cs in per.items():
        out[k] = {c: sum(v.values()) / max(len(v), 1) for c, v in cs.items()}
        out[k]["_dispatches"] = max(len(v) for v in cs.values())
    return out, meta


def derived(c):
    d = {}
    g = c.get
    if g("SQ_WAVE_CYCLES"):
        if g("SQ_WAIT_ANY") is not None:
            d["SQ_WAIT_ANY / SQ_WAVE_CYCLES"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
        if g("SQ_ACTIVE_INST_ANY") is not None:
            d["SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES"] = g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES")
    if g("SQ_WAVES"):
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if g(n) is not None:
                d[f"{n} per wave"] = g(n) / g("SQ_WAVES")
    if g("TCP_TCC_READ_REQ"):
        d["L2 read latency (cycles) = TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ"] = \
            g("TCP_TCC_READ_REQ_LATENCY", 0) / g("TCP_TCC_READ_REQ")
    if g("TCC_HIT") is not None and g("TCC_MISS") is not None and g("TCC_HIT") + g("TCC_MISS") > 0:
        d["L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS)"] = g("TCC_HIT") / (g("TCC_HIT") + g("TCC_MISS"))
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        d["HBM bytes per dispatch = (2 FETCH_SIZE + WRITE_SIZE) x 1024"] = (2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--kernel", default=".")
    ap.add_argument("--title", default=None)
    args = ap.parse_args()
    data, meta = load(args.outdir)
    print(f"# {args.title or 'PMC counters: ' + args.outdir}\n")
    print("One rocprofv3 --pmc run per counter set (tools/pmc_passes.sh, --kernel-trace only); values are "
          "per-dispatch averages over the run's dispatches of each kernel.\n")
    for k in sorted(data):
        if not re.search(args.kernel, k):
            continue
        c = data[k]
        v, a, s, lds, grid = meta[k]
        print(f"## `{k}`\n")
        print(f"dispatches {c['_dispatches']}, grid {grid}, LDS {lds} B, VGPR_Count {v} (arch) + {a} (accum), "
              f"SGPR_Count {s}\n")
        print("| counter | per dispatch |\n|---|---|")
        for n in sorted(x for x in c if not x.startswith("_")):
            print(f"| {n} | {c[n]:.1f} |")
        print("\nDerived:\n")
        for n, val in derived(c).items():
            print(f"- {n}: {val:.3f}" if val < 100 else f"- {n}: {val:.0f}")
        print()


if __name__ == "__main__":
    main()
