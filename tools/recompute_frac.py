#!/usr/bin/env python3
"""Recompute every bench.py roofline fraction from rocprofv3 traces, and file the evidence.

    python tools/recompute_frac.py gpurun_out/<tag> profiles/<tag>

Reads what tools/gpu_session.sh (bench.json, prof/, pmc_fetch/, pmc_write/) and
tools/profile_legs.sh (<leg>/prof, <leg>/pmc_*, <leg>/leg.json) left under gpurun_out/<tag>, and
writes under profiles/:
  <tag>_bench.json                        the bench line
  <tag>_<part>_kernel_grid_stats.csv      per (kernel, grid, after-flush) durations (kernel_grid_stats.py)
  <tag>_<part>_pmc_traffic.json           per-launch HBM bytes, FETCH_SIZE x2 + WRITE_SIZE (pmc_traffic.py)
  <tag>_<leg>.json                        the leg's JSON line from its kernel-trace run
  <tag>_frac_check.md                     bench frac vs the frac recomputed from the trace
Algorithmic bytes: SpMV 12 nnz + 4 (m+1) + 8 n + 8 m; SpMM(L) 12 nnz + 4 (m+1) +
8 L (n+m); CG iteration 12 nnz + 4 (m+1) + 88 m L.  Peak 8 TB/s.
"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from kernel_grid_stats import grid_stats, short_name  # noqa: E402
import pmc_traffic  # noqa: E402

PEAK = 8000.0


def spmv_bytes(m, n, nnz, L=1):
    return 12 * nnz + 4 * (m + 1) + 8 * L * (n + m)


def cg_iter_bytes(m, nnz, L=1):
    return 12 * nnz + 4 * (m + 1) + 88 * m * L


def last_json(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def write_csv(rows, path):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)


def trace_file(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                return os.path.join(root, f)
    return None


def frac(nbytes, us):
    return nbytes / (us * 1e-6) / 1e9 / PEAK


def cg_loop_times(trace, iterations):
    """Kernel-busy time per iteration over both solves (warm + timed: same inputs, same iteration
    count), counting kernels launched at least once per iteration, and the timed solve's span (first
    start to last end of its loop kernels) per iteration."""
    recs = [r for r in csv.DictReader(open(trace)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    recs.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls = {}
    for r in recs:
        k = short_name(r["Kernel_Name"])
        calls[k] = calls.get(k, 0) + 1
    loop = {k for k, c in calls.items() if c >= iterations and not k.startswith("__amd")}  # not the runtime's copies
    if any(k.startswith("k_cg_resident") for k in calls):  # the resident CG's leg (its pipelined_large solves too)
        loop = set()
    if not loop:  # the register-resident CG: the whole solve is ONE cooperative launch (the last one is timed)
        # launches: the warm solve, the timed one, then (bench's resident_phases) a stamped one
        res = [r for r in recs if short_name(r["Kernel_Name"]).startswith("k_cg_resident")]
        if res:
            r = res[1] if len(res) >= 2 else res[-1]
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            return dur / iterations, dur / iterations, [short_name(r["Kernel_Name"])]
    lrecs = [r for r in recs if short_name(r["Kernel_Name"]) in loop]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in lrecs) / 1000.0
    half = lrecs[len(lrecs) // 2:]
    span = (int(half[-1]["End_Timestamp"]) - int(half[0]["Start_Timestamp"])) / 1000.0
    return busy / (2 * iterations), span / iterations, sorted(loop)


def main(src, dst):
    tag = os.path.basename(dst.rstrip("/"))
    pdir = os.path.dirname(dst) or "."
    out = lambda name: os.path.join(pdir, f"{tag}_{name}")  # noqa: E731
    lines = [f"# {tag}: bench roofline fractions recomputed from rocprofv3 traces", "",
             "| measurement | bench value | from trace | trace rows used |", "|---|---|---|---|"]

    bench = last_json(os.path.join(src, "bench.json")) if os.path.exists(os.path.join(src, "bench.json")) else None
    if bench:
        json.dump(bench, open(out("bench.json"), "w"), indent=1)
    tr = trace_file(os.path.join(src, "prof"))
    if tr:
        rows = grid_stats(tr)
        write_csv(rows, out("headline_kernel_grid_stats.csv"))
        prof_bench = last_json(os.path.join(src, "prof_bench.json"))
        rf = prof_bench["roofline"]
        norm = lambda k: k.replace(",256>", ">").replace(",6,false>", ",6>")  # noqa: E731  default template arguments
        kr = max((r for r in rows if norm(r["kernel"]) == norm(rf["kernel"])), key=lambda r: r["grid"])
        lines.append(f"| headline {rf['kernel']} | frac {bench['roofline']['frac'] if bench else '-'} "
                     f"(kernel_ms {bench['roofline']['kernel_ms'] if bench else '-'}) | frac "
                     f"{frac(rf['bytes_per_launch'], kr['avg_us']):.4f} (avg {kr['avg_us']} us, median "
                     f"{kr['median_us']} us) | {kr['kernel']} grid {kr['grid']} x{kr['calls']} |")
        if os.path.isdir(os.path.join(src, "pmc_fetch")):
            pmc_traffic.main(["", src, out("pmc_traffic.json")])

    if tr and os.path.exists(os.path.join(src, "prof", "bench_kernel_stats.csv")):  # rocprofv3's own --stats
        open(out("headline_kernel_stats.csv"), "w").write(open(os.path.join(src, "prof", "bench_kernel_stats.csv")).read())

    for leg in ("spmm16", "spmv_shapes", "cg_single", "cg_multi", "pwtk_perturbed"):
        ld = os.path.join(src, leg)
        if not os.path.isdir(ld):
            continue
        lj = last_json(os.path.join(ld, "leg.json"))
        lj0 = lj  # the leg's own (profiled) run, before the unprofiled bench numbers are merged in
        json.dump(lj, open(out(f"{leg}.json"), "w"), indent=1)
        # the bench column: the unprofiled bench run's numbers where it holds the leg (the leg's own
        # run is under rocprofv3, whose per-dispatch bookkeeping widens back-to-back launch gaps);
        # the trace's shape facts (m, nnz, iterations) come from the leg run either way
        bkey = {"pwtk_perturbed": "spmv_pwtk_perturbed"}.get(leg, leg)
        if bench and isinstance(bench.get(bkey), dict):
            src_leg = bench[bkey]
            lj = dict(lj, **{k: v for k, v in src_leg.items() if not isinstance(v, dict)},
                      **{k: dict(lj.get(k, {}), **v) for k, v in src_leg.items() if isinstance(v, dict)})
        tr = trace_file(os.path.join(ld, "prof"))
        rows = grid_stats(tr)
        write_csv(rows, out(f"{leg}_kernel_grid_stats.csv"))
        if os.path.isdir(os.path.join(ld, "pmc_fetch")) and os.path.isdir(os.path.join(ld, "pmc_write")):
            pmc_traffic.main(["", "--leg", ld, out(f"{leg}_pmc_traffic.json")])
        st = os.path.join(ld, "prof", "leg_kernel_stats.csv")
        if os.path.exists(st):
            open(out(f"{leg}_kernel_stats.csv"), "w").write(open(st).read())
        if leg == "pwtk_perturbed":
            norm = lambda k: k.replace(",6,false>", ",6>")  # noqa: E731
            kr = max((r for r in rows if norm(r["kernel"]) == norm(lj["kernel"])), key=lambda r: r["calls"])
            lines.append(f"| {leg} {lj['kernel']} | frac {lj['frac']} (kernel_ms {lj['kernel_ms']}) | frac "
                         f"{frac(lj['bytes_per_launch'], kr['avg_us']):.4f} (avg {kr['avg_us']} us, median "
                         f"{kr['median_us']} us) | {kr['kernel']} grid {kr['grid']} x{kr['calls']} |")
        elif leg in ("spmm16", "spmv_shapes"):
            L = 16 if leg == "spmm16" else 1
            shapes = [k for k in (("cant", "pwtk") if leg == "spmm16" else ("cant", "rma10", "powerlaw")) if k in lj]
            cold = sorted((r for r in rows if r["after_flush"] and r["kernel"].startswith(("k_spmm", "k_spmv"))),
                          key=lambda r: r["first_dispatch"])
            for name, r in zip(shapes, cold):
                s = lj[name]
                nb = spmv_bytes(s["m"], s["m"], s["nnz"], L)
                lines.append(f"| {leg} {name} cold | frac {s['frac']} (cold_kernel_ms {s['cold_kernel_ms']}) | frac "
                             f"{frac(nb, r['avg_us']):.4f} (avg {r['avg_us']} us) | {r['kernel']} grid {r['grid']} "
                             f"after flush x{r['calls']} |")
                hot = [h for h in rows if h["kernel"] == r["kernel"] and h["grid"] == r["grid"] and not h["after_flush"]]
                if hot:
                    h = hot[0]
                    lines.append(f"| {leg} {name} hot | hot_kernel_ms {s['hot_kernel_ms']} | {h['avg_us']} us avg "
                                 f"(incl. 5 warm-up launches) | {h['kernel']} grid {h['grid']} x{h['calls']} |")
        else:
            m = int(lj["workload"].split(" m=")[1].split()[0])
            nnz = int(lj["workload"].split(" nnz=")[1].split(",")[0].split()[0])
            L = 8 if leg == "cg_multi" else 1
            it = lj["iterations"]
            busy, span, loop = cg_loop_times(tr, it)
            nb = cg_iter_bytes(m, nnz, L)
            fk = "roofline_frac" if "roofline_frac" in lj else "speed_equiv_frac"
            lines.append(f"| {leg} | {fk} {lj[fk]} ({lj.get('us_per_iter') or lj.get('ms_per_iter')} "
                         f"{'us' if 'us_per_iter' in lj else 'ms'}/iter, wall) | span frac {frac(nb, span):.4f} "
                         f"({span:.2f} us/iter); kernel-busy frac {frac(nb, busy):.4f} ({busy:.2f} us/iter) | "
                         f"{', '.join(loop)} |")
            pl = lj.get("pipelined_large") if leg == "cg_single" else None
            if isinstance(pl, dict) and "workload" in pl:
                # the two-kernel pipelined CG on the pwtk-size stencil (bench cg_single.pipelined_large): the median
                # launch of each loop kernel (a solve also launches up to 2 graph batches past convergence, which
                # return at their stop test: the medians are the iterations' own launches)
                pm = int(pl["workload"].split(" m=")[1].split()[0])
                pnnz = int(pl["workload"].split(" nnz=")[1].split(",")[0].split()[0])
                med = {}
                for r in rows:
                    k = r["kernel"]
                    if k.startswith(("k_cg1_dia", "k_cg1_update")) or (k.startswith("k_spmv_tile<8,1,")):
                        if r["calls"] >= pl["iterations"] and (k not in med or r["calls"] > med[k][1]):
                            med[k] = (r["median_us"], r["calls"])
                if med:
                    per = sum(v[0] for v in med.values())
                    lines.append(f"| cg_single.pipelined_large | roofline_frac {pl['roofline_frac']} ({pl['us_per_iter']} "
                                 f"us/iter, wall) | kernel frac {frac(cg_iter_bytes(pm, pnnz), per):.4f} ({per:.2f} us/iter: "
                                 f"{' + '.join(f'{v[0]}' for v in med.values())} us, median launches) | "
                                 f"{', '.join(f'{k} x{v[1]}' for k, v in med.items())} |")
            if leg == "cg_multi" and bench and isinstance(bench.get("spmv_nlpkkt120_size"), dict):
                # SURVEY 8(d)'s named 70 % case: the nlpkkt120-size single-RHS SpMV timed in the same leg
                # (back-to-back launches) against its rows in this trace
                sl = bench["spmv_nlpkkt120_size"]
                own = lj0.get("spmv_nlpkkt120_size") if isinstance(lj0, dict) else None
                for label, ent, oent in (("", sl, own), (" merge_path", sl.get("merge_path"),
                                                          own.get("merge_path") if isinstance(own, dict) else None)):
                    if not isinstance(ent, dict) or "kernel" not in ent:
                        continue
                    pre = ent["kernel"].rstrip(">")  # the bench's name leaves out default template arguments
                    sp = [r for r in rows if r["kernel"].startswith(pre) and r["calls"] >= 40]
                    if not sp:
                        continue
                    r = max(sp, key=lambda q: q["calls"])
                    own_s = f"; this profiled run's own events: kernel_ms {oent['kernel_ms']}" if isinstance(oent, dict) else ""
                    lines.append(f"| spmv_nlpkkt120_size{label} | frac {ent['frac']} (kernel_ms {ent['kernel_ms']}{own_s}) | "
                                 f"frac {frac(sl['bytes_per_launch'], r['avg_us']):.4f} (avg {r['avg_us']} us, median "
                                 f"{r['median_us']} us) | {r['kernel']} grid {r['grid']} x{r['calls']} |")
    lines += ["", "hot rows include the untimed warm-up launches; cold rows are the launches right after bench's "
              "512 MiB flush kernel.  CG: span = the timed solve's first-to-last loop-kernel time / iterations "
              "(bench divides wall time, which adds the host call); kernel-busy = the loop kernels' summed "
              "durations per iteration.  spmm16 / spmv_shapes: since r04k one kernel per product (split rows "
              "closed inside the tile kernel); bench's cold time = (flush + launch region - flush-only region) / "
              "reps, its hot time = back-to-back region / reps.  Bench column: the unprofiled bench run (bench.json) where it "
              "holds the leg; the trace column: the leg's rocprofv3 run."]
    open(out("frac_check.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    if len(sys.argv) < 3:
        raise SystemExit(__doc__)
    main(sys.argv[1], sys.argv[2])
