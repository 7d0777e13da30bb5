#!/usr/bin/env python3
"""parallel_efficiency for the GPU: speedup and efficiency of the block CG over compute resources.

The reference's verification/efficiency/parallel_efficiency.cpp (:67-113 RunBenchmark, :177-229
CalculateEfficiency, :234-288 CSVs, :293-395 main) times TestCGMultipleRHS (num_vectors = 16,
NONZERO_SPLIT, max_iters 100000, raw tolerance 1e-5, min over timing_iters) on every .mtx of a
directory at thread counts 1, 2, 4, ..., 18, and writes

    <output_dir>/parallel_efficiency.csv           num_threads,avg_time_ms,avg_gflops,speedup,efficiency
    <output_dir>/parallel_efficiency_detailed.csv  matrix_name,num_threads,time_ms,gflops,iterations

which verification/efficiency/efficiency_plot.py reads.  The GPU has no thread count; its two
parallel resources are swept instead, into the same files and columns (num_threads = the unit):

  --units=cus   (default) compute units of one GPU: the handle's stream is CU-masked
                (mspmv_set_cu_limit) to 8, 16, 32, ..., 256 CUs.  speedup = T(first) / T(n),
                efficiency = speedup / (n / first) -- the reference's T(1)/T(n) and speedup/n with the
                first count as the unit.
  --units=gpus  GPUs of one node, the row-sharded block CG (mspmv_dist_cg_dev over RCCL) on 1, 2, 4,
                ... of the ranks of a torch.distributed.run launch:
                    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
                        --master-addr 127.0.0.1 --master-port 29511 tools/parallel_efficiency.py --units=gpus
                (gloo carries the ids and timings; ranks outside a point wait at its barrier).

Matrices: every .mtx under --mtx_dir (sorted; trivial ones skipped, as the reference does), or with
--synthetic the built-in SPD shapes (SuiteSparse files are not available offline).  RHS: srand(42);
rand()/RAND_MAX over n x num_vectors, interleaved (parallel_efficiency.cpp:91-93).  GFLOPS =
(2 nnz + 10 m) * num_vectors * iterations / time (:96-107).  Times exclude the upload (inputs
resident in HBM), each point the min over timing_iters solves.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]

import mspmv  # noqa: E402


def glibc_rhs(n):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(42))
    r = libc.rand
    r.restype = ctypes.c_int
    return np.fromiter((r() for _ in range(n)), dtype=np.float64, count=n) / 2147483647.0


def synthetic_set():
    """SPD shapes standing in for download/final_mtx (name, generator)."""
    return [
        ("fem2d_400x400", lambda: mspmv.CsrMatrix.synth_stencil(0, 160000, 400, diag_shift=1e-3)),
        ("parabolic_fem_shape", lambda: mspmv.CsrMatrix.synth_stencil(0, 525825, 725, diag_shift=1e-4)),
        ("stencil27_64", lambda: mspmv.CsrMatrix.synth_stencil(1, 64 ** 3, 64, 64, 64, diag_shift=1e-2)),
    ]


def matrix_set(args):
    if args.synthetic:
        return synthetic_set()
    if not os.path.isdir(args.mtx_dir):
        raise SystemExit(f"Error: No .mtx files found in {args.mtx_dir}")
    files = sorted(os.path.join(args.mtx_dir, f) for f in os.listdir(args.mtx_dir) if f.endswith(".mtx"))
    if not files:
        raise SystemExit(f"Error: No .mtx files found in {args.mtx_dir}")
    return [(os.path.splitext(os.path.basename(f))[0], (lambda f=f: mspmv.CsrMatrix.from_market(f))) for f in files]


def efficiency(rows, units):
    """CalculateEfficiency (parallel_efficiency.cpp:177-229): per unit count the mean over
    matrices, speedup from the first count's mean time."""
    out = []
    for u in units:
        pts = [r for r in rows if r[1] == u]
        if not pts:
            continue
        out.append([u, float(np.mean([p[2] for p in pts])), float(np.mean([p[3] for p in pts]))])
    if out:
        t0, u0 = out[0][1], out[0][0]
        for r in out:
            sp = t0 / r[1]
            r += [sp, sp / (r[0] / u0)]
    return out


def save(args, rows, eff, tag):
    os.makedirs(args.output_dir, exist_ok=True)
    p = os.path.join(args.output_dir, f"parallel_efficiency{tag}.csv")
    with open(p, "w") as f:
        f.write("num_threads,avg_time_ms,avg_gflops,speedup,efficiency\n")
        for u, t, g, sp, ef in eff:
            f.write(f"{u},{t:.3f},{g:.2f},{sp:.3f},{ef:.4f}\n")
    print(f"Results saved to: {p}")
    p = os.path.join(args.output_dir, f"parallel_efficiency{tag}_detailed.csv")
    with open(p, "w") as f:
        f.write("matrix_name,num_threads,time_ms,gflops,iterations\n")
        for name, u, t, g, it in rows:
            f.write(f"{name},{u},{t:.3f},{g:.2f},{it}\n")
    print(f"Detailed results saved to: {p}")


def summary(eff, n, what):
    print(f"\n=== Summary (Average across {n} matrices) ===")
    print(f"{what:>7s}  Time(ms)   GFLOPS   Speedup  Efficiency")
    print("-------  --------   ------   -------  ----------")
    for u, t, g, sp, ef in eff:
        print(f"{u:7d}  {t:8.3f}   {g:6.2f}   {sp:7.3f}  {ef:10.4f}")


def gflops(a, L, it, ms):
    return (2.0 * a.num_nonzeros + 10.0 * a.num_rows) * L * it / (ms / 1000.0) / 1e9


def cus_child(args):
    """One CU count, every matrix: prints one 'ROW <json>' line per matrix."""
    import json
    u = int(args.cus)
    for name, make in matrix_set(args):
        a = make()
        if a.num_rows == 1 or a.num_cols == 1 or a.num_nonzeros == 1:
            continue
        L = args.num_vectors
        B = glibc_rhs(a.num_rows * L).reshape(a.num_rows, L)
        with mspmv.GpuCsr(a, device=args.device) as g:
            g.set_cu_limit(u)
            dB = mspmv.DeviceBuffer.from_array(B, args.device)
            dX = mspmv.DeviceBuffer(8 * a.num_rows * L, args.device)
            g.cg_dev(dB, dX, L, args.max_iters, args.tolerance)   # warm: graph, workspace
            best, best_it = float("inf"), 0
            for _ in range(args.timing_iters):
                t0 = time.perf_counter()
                it, _, _ = g.cg_dev(dB, dX, L, args.max_iters, args.tolerance)
                ms = (time.perf_counter() - t0) * 1e3
                if ms < best:
                    best, best_it = ms, it
        print("ROW " + json.dumps([name, a.num_rows, a.num_nonzeros, u, best, gflops(a, L, best_it, best), best_it]),
              flush=True)


def sweep_cus(args):
    """Each CU count in its own child process: a CU-masked stream takes a hardware queue of its own,
    and a process holds only a few (GPU_MAX_HW_QUEUES), so one process per count keeps every
    point on a fresh queue set."""
    import json
    import subprocess
    units = [int(v) for v in args.cus.split(",")]
    rows = []
    for u in units:
        cmd = [sys.executable, os.path.abspath(__file__), "--units=cus", f"--cus={u}", "--_child",
               f"--num_vectors={args.num_vectors}", f"--timing_iters={args.timing_iters}",
               f"--max_iters={args.max_iters}", f"--tolerance={args.tolerance}", f"--device={args.device}",
               f"--mtx_dir={args.mtx_dir}"] + (["--synthetic"] if args.synthetic else [])
        # one algorithm at every point: the register-resident single-RHS CG needs the whole device
        # (one workgroup per CU), so a CU-limited child would fall back to the pipelined CG and the
        # full-device point alone would compare a different algorithm -- L = 1 sweeps run pipelined
        env = dict(os.environ)
        if args.num_vectors == 1:
            env["MSPMV_CG_RESIDENT"] = "0"
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.child_timeout, env=env)
        if r.returncode != 0:
            raise SystemExit(f"CUs={u}: child failed ({r.returncode}): {r.stderr[-1500:]}")
        for ln in r.stdout.splitlines():
            if ln.startswith("ROW "):
                rows.append(json.loads(ln[4:]))
        print(f"  CUs={u:3d}: done", flush=True)
    names = []
    for r in rows:
        if r[0] not in names:
            names.append(r[0])
    rows.sort(key=lambda r: (names.index(r[0]), units.index(r[3])))
    out = []
    for name in names:
        rs = [r for r in rows if r[0] == name]
        print(f"Processing: {name} (rows={rs[0][1]}, nnz={rs[0][2]})")
        for r in rs:
            print(f"  CUs={r[3]:3d}: {r[4]:.3f} ms, {r[5]:.2f} GFLOPS")
            out.append([name, r[3], r[4], r[5], r[6]])
        print()
    eff = efficiency(out, units)
    summary(eff, len(names), "CUs")
    save(args, out, eff, "")


def sweep_gpus(args):
    import torch.distributed as td
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        td.init_process_group("gloo")
    units = [int(v) for v in args.gpus.split(",")] if args.gpus else [g for g in (1, 2, 4, 8, 16) if g <= world]
    if any(u > world for u in units):
        raise SystemExit(f"--gpus asks for more than WORLD_SIZE={world} ranks")
    rows, nmat = [], 0

    def bcast(obj):
        if world == 1:
            return obj
        o = [obj]
        td.broadcast_object_list(o, src=0)
        return o[0]

    def tmax(v):
        if world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        return float(t.item())

    for name, make in matrix_set(args):
        a = make()  # every rank builds / reads the same matrix (deterministic)
        if a.num_rows == 1 or a.num_cols == 1 or a.num_nonzeros == 1:
            if rank == 0:
                print(f"Skipping trivial matrix: {name}")
            continue
        nmat += 1
        if rank == 0:
            print(f"Processing: {name} (rows={a.num_rows}, nnz={a.num_nonzeros})")
        L = args.num_vectors
        B = glibc_rhs(a.num_rows * L).reshape(a.num_rows, L)
        for u in units:
            uid = bcast(mspmv.comm_unique_id() if rank == 0 else None)
            best, best_it = float("inf"), 0
            if rank < u:
                rb = mspmv.dist_partition(a, u)
                dc = mspmv.DistCsr(uid, u, rank, local, rb, mspmv.local_rows(a, rb, rank))
                lo, hi = int(rb[rank]), int(rb[rank + 1])
                dB = mspmv.DeviceBuffer.from_array(np.ascontiguousarray(B[lo:hi]), local)
                dX = mspmv.DeviceBuffer(8 * max(hi - lo, 1) * L, local)
                dc.cg_dev(dB, dX, L, args.max_iters, args.tolerance)
            for _ in range(args.timing_iters):
                if world > 1:
                    td.barrier()
                ms, it = 0.0, 0
                if rank < u:
                    t0 = time.perf_counter()
                    it, _, _ = dc.cg_dev(dB, dX, L, args.max_iters, args.tolerance)
                    ms = (time.perf_counter() - t0) * 1e3
                ms = tmax(ms)
                it = int(tmax(float(it)))
                if ms < best:
                    best, best_it = ms, it
            if rank < u:
                dc.close()
            gf = gflops(a, L, best_it, best)
            rows.append([name, u, best, gf, best_it])
            if rank == 0:
                print(f"  GPUs={u:3d}: {best:.3f} ms, {gf:.2f} GFLOPS", flush=True)
        if rank == 0:
            print()
    if rank == 0:
        eff = efficiency(rows, units)
        summary(eff, nmat, "GPUs")
        save(args, rows, eff, "_gpus")
    if world > 1:
        td.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--mtx_dir", default=os.path.join(ROOT, "download", "final_mtx"))
    ap.add_argument("--output_dir", default=os.path.join(ROOT, "data", "parallel"))
    ap.add_argument("--num_vectors", type=int, default=16)
    ap.add_argument("--timing_iters", type=int, default=3)
    ap.add_argument("--max_iters", type=int, default=100000)
    ap.add_argument("--tolerance", type=float, default=1.0e-5)
    ap.add_argument("--units", choices=["cus", "gpus"], default="cus")
    ap.add_argument("--cus", default="8,16,32,64,128,256")
    ap.add_argument("--gpus", default="", help="GPU counts (default 1, 2, 4, ... up to WORLD_SIZE)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--synthetic", action="store_true", help="built-in SPD shapes instead of --mtx_dir")
    ap.add_argument("--child_timeout", type=float, default=600.0, help="seconds allowed per CU-count child")
    ap.add_argument("--_child", action="store_true", help=argparse.SUPPRESS)
    # the reference spells its options --key=value; argparse accepts both forms
    args = ap.parse_args(argv)
    if args._child:
        return cus_child(args)
    print("=== Parallel Efficiency Benchmark ===")
    print(f"Matrix directory: {'(synthetic)' if args.synthetic else args.mtx_dir}")
    print(f"num_vectors: {args.num_vectors}")
    if args.units == "cus":
        print(f"CU counts: {args.cus.replace(',', ' ')}\n")
        sweep_cus(args)
    else:
        sweep_gpus(args)
    print("\nAll benchmarks completed.")


if __name__ == "__main__":
    main()
