#!/usr/bin/env python3
"""bench.py -- MI355X merge-path fp64 SpMV (+ CG) benchmark; prints ONE JSON line on rank 0.

Headline workload (BASELINE.json configs[1], "merge-based CSR SpMV fp64, 1 RHS, pwtk/rma10 on
1xMI355X"): a STEP is one SpMV over each matrix of a batch of 4 distinct synthetic
pwtk-shaped matrices -- m = 217,918, nnz = 11,524,432 (52.9 per row), 6 unknowns per mesh node
with every row of a node coupling to the same neighbour nodes within +-1,700 nodes (pwtk is a
6-DOF structural FEM matrix; SuiteSparse files are not available offline).  The batch (571 MB)
exceeds the 256 MiB Infinity Cache, so every launch streams its matrix from HBM.  All inputs
are resident in HBM before the timed region.

  value        = 2 * nnz * batch * steps * n_gpus / max-over-ranks(time)  [GFLOP/s, whole job]
  roofline     = algorithmic bytes per SpMV launch, 12 nnz + 4 (m+1) + 8 n + 8 m,
                 / the merge-tile kernel's average duration: HIP events on its stream around
                 the timed region / launches in it (every launch of a pwtk-shaped step is a
                 tile kernel; the ~1.5 us launch boundary is included); peak 8 TB/s HBM3E
  cpu_baseline = the reference's own merge CsrMV (work_2025 OmpMergeCsrmm with num_vectors = 1,
                 == cpu_spmv.cpp OmpMergeCsrmv) compiled from /root/reference into oracle/_ref,
                 else the oracle port; host cores, ~10 s on matrix #0 (rank 0, N = 1 only)

Extra fields: the scattered-band stress shape, CG iterations/s for configs[3] (single CG,
parabolic_fem shape) and configs[4] (8-RHS block CG, nlpkkt120 size; at N > 1 row-sharded over
all ranks with RCCL halo exchange + dot all-reduces).

Launch: `python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts its own N
ranks -- before it imports mspmv or touches a GPU, the parent runs `python -m torch.distributed.run
--nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port <free> bench.py <same args>` as a
child process (never an exec), relays rank 0's JSON line and exits with the launcher's status (non-zero
when any rank fails).  Under torch.distributed.run (WORLD_SIZE set) it runs as one rank.  --dry-run: every
rank joins the gloo group, reports its WORLD_SIZE / RANK, and rank 0 prints them without touching a GPU
(tests/test_bench_launch.py checks the launch on CPU).

Multi-GPU (--gpus N via torch.distributed.run; run_sharded_headline): weak scaling with a real
exchange step -- each matrix of the batch is ONE FEM-blocked matrix of N x 217,918 rows, sharded by
merge-path row blocks; every rank generates only its pwtk-sized block, and each SpMV exchanges the
halo rows of x over RCCL (send/recv, xGMI) while the block interior is multiplied.  value = all
ranks' flops / max-over-ranks time; roofline = the per-rank local SpMV (no exchange).  gloo
carries the barrier, the max-over-ranks reductions and the RCCL ids.  A watchdog turns a hang of
the collective part into exit 3 with the line printed.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "sparse-matrix-linear-equations_amd")]


def launch_ranks():
    """`--gpus N` (N > 1) outside a torch.distributed launch: start the N ranks as a child launcher
    process and relay rank 0's JSON line; returns the exit status (None: run here as one process).
    Runs before mspmv is imported, so this parent never initialises a GPU."""
    if "WORLD_SIZE" in os.environ:
        return None
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    known, _ = pre.parse_known_args()
    if known.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={known.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    proc = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    for ln in proc.stdout.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)  # anything else the ranks printed: kept, off the JSON channel
    if lines:
        print(lines[-1], flush=True)
    if proc.returncode != 0:
        print(f"bench.py: the {known.gpus}-rank launch exited with status {proc.returncode}", file=sys.stderr)
        return proc.returncode or 1
    return 0 if lines else 1


if __name__ == "__main__":
    _rc = launch_ranks()
    if _rc is not None:
        sys.exit(_rc)

import mspmv  # noqa: E402

METRIC = "fp64 SpMV GFLOP/s + achieved HBM GB/s vs roofline; CG iters/sec"
HBM_PEAK_GBS = 8000.0


def pmc_traffic(kernel, bytes_launch):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from separate rocprofv3
    --pmc FETCH_SIZE / WRITE_SIZE passes of this same bench command), or None when no summary
    matches this kernel instantiation and workload size."""
    import glob
    import re

    def tag_order(path):  # r01 < r01z < r02 < r02t < r02aa < r02ai: round, then session letters
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), key=tag_order, reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("bench_bytes_per_launch") != bytes_launch:
            continue
        for name, v in d.get("kernels", {}).items():
            short = name.replace("void mspmv::", "").split("(")[0].replace(" ", "")
            norm = lambda k: k.replace(",256>", ">").replace(",6,false>", ",6>")  # noqa: E731  default arguments
            if norm(short) == norm(kernel):
                return v["traffic_bytes"], os.path.basename(path)
    return None, None
PWTK = dict(m=217918, nnz=11524432, block=6, half_band_nodes=1700)
PARABOLIC_FEM = dict(m=525825, width=725, shift=1e-4)
NLPKKT120 = dict(dims=(160, 135, 164), shift=1e-2, L=8)
KKT120 = dict(dims=(120, 120, 123), eps=1e-2)  # 2 x 120 x 120 x 123 = nlpkkt120's 3,542,400 rows


def spmv_bytes(m, n, nnz):
    return 12 * nnz + 4 * (m + 1) + 8 * n + 8 * m


def cg_iter_bytes(m, nnz, L=1):
    return 12 * nnz + 4 * (m + 1) + 88 * m * L  # compulsory bytes per CG iteration


def glibc_rhs(seed, n):
    """srand(seed); b[i] = rand()/RAND_MAX -- the reference's RHS (cpu_singlecg.cpp:87-90)."""
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(seed))
    r = libc.rand
    r.restype = ctypes.c_int
    return np.fromiter((r() for _ in range(n)), dtype=np.float64, count=n) / 2147483647.0


class Dist:
    def __init__(self, want):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.td = None
        if self.world > 1:
            import torch.distributed as td
            td.init_process_group("gloo")
            self.td = td
        if want != self.world and self.rank == 0:
            print(f"warning: --gpus {want} but WORLD_SIZE {self.world}", file=sys.stderr)

    def barrier(self):
        if self.td:
            self.td.barrier()

    def max(self, v):
        if not self.td:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.td.all_reduce(t, op=self.td.ReduceOp.MAX)
        return float(t.item())

    def comm(self, dev):
        """This rank's one RCCL communicator (mspmv.Comm, created on first use, collective), shared
        by every sharded matrix of the run: no two communicators ever have collectives in flight."""
        if getattr(self, "_comm", None) is None:
            uid = self.bcast_bytes(mspmv.comm_unique_id() if self.rank == 0 else None)
            self._comm = mspmv.Comm(uid, self.world, self.rank, dev)
        return self._comm

    def close_comm(self):
        if getattr(self, "_comm", None) is not None:
            try:
                self._comm.close()
            except RuntimeError as e:  # a sharded matrix left open by a failed leg: the process exit frees it
                print(f"rank {self.rank}: {e}", file=sys.stderr)
            self._comm = None

    def bcast_bytes(self, b):
        if not self.td:
            return b
        obj = [b]
        self.td.broadcast_object_list(obj, src=0)
        return obj[0]


def host_cores():
    """Host cores this process may run on: its CPU affinity (os.sched_getaffinity -- what the
    reference's omp_get_num_procs() default counts), capped by the cgroup's CPU quota
    when one is set (a GPU box's share of a larger machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 256))  # cpu_spmv.cpp:370-371 sizes its carry arrays for <= 256 threads


def cpu_baseline(a, x, seconds):
    """The reference's merge CsrMV on the host cores (bounded sample)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import REF_SO, Oracle, RefLib
    threads = host_cores()
    if os.path.exists(REF_SO):
        ref = RefLib()
        kind = "reference"
        X = np.ascontiguousarray(x[:, None])
        fn = lambda: ref.merge_csrmm(a, X, threads)[:, 0]  # noqa: E731
        what = "work_2025 OmpMergeCsrmm(num_vectors=1) == cpu_spmv.cpp OmpMergeCsrmv"
    else:
        orc = Oracle()
        kind = "port"
        fn = lambda: orc.merge_csrmv(a, x, threads)  # noqa: E731
        what = "oracle port of cpu_spmv.cpp OmpMergeCsrmv"
    y = fn()
    calls, t0 = 0, time.perf_counter()
    while True:
        fn()
        calls += 1
        el = time.perf_counter() - t0
        if el >= seconds and calls >= 3:
            break
    gflops = 2.0 * a.num_nonzeros * calls / el / 1e9
    return y, {"value": round(gflops, 3), "unit": "GFLOP/s", "cores": threads, "kind": kind,
               "sample": f"{what}, P={threads} threads, pwtk-shaped matrix #0 (nnz={a.num_nonzeros}), "
                         f"{calls} calls in {el:.1f} s"}


FLUSH_BYTES = 512 << 20   # >= 512 MB MALL flush between cold calls (a read sweep: clean lines,
                          # so the timed launch does not pay the flush's own write-back)
CANT = dict(m=62451, nnz=4007383, band=2000, seed=1)
RMA10 = dict(m=46835, nnz=2374001, band=3000, seed=2)


def gpu_spmv_hot_cold(a, dev, seed=2):
    """One matrix's SpMV tile kernel: hot (back-to-back launches; a matrix below 256 MiB stays
    Infinity-Cache resident) and cold (a 512 MiB flush read sweep before every timed launch, SURVEY
    8(d)); HIP events around each launch.  frac is priced on the cold time."""
    x = np.random.default_rng(seed).uniform(0.0, 1.0, a.num_cols)
    with mspmv.GpuCsr(a, device=dev) as g:
        dx, dy = mspmv.DeviceBuffer.from_array(x, dev), mspmv.DeviceBuffer(8 * a.num_rows, dev)
        g.time_spmm(dx, dy, 1, 5)
        _, hot, _ = g.time_spmm(dx, dy, 1, 200)
        _, cold, _ = g.time_spmm(dx, dy, 1, 160, FLUSH_BYTES)  # 8 blocks beside flush-only controls
        kname = g.kernel_name()
    nb = spmv_bytes(a.num_rows, a.num_cols, a.num_nonzeros)
    return x, {"m": a.num_rows, "nnz": a.num_nonzeros, "kernel": kname, "bytes_per_launch": nb,
               "hot_kernel_ms": round(hot, 5), "hot_GBps": round(nb / hot / 1e6, 1),
               "cold_kernel_ms": round(cold, 5), "cold_GBps": round(nb / cold / 1e6, 1),
               "gflops_cold": round(2.0 * a.num_nonzeros / cold / 1e6, 1),
               "frac": round(nb / cold / 1e6 / HBM_PEAK_GBS, 4)}


def _threads():
    return host_cores()


def _time_calls(fn, seconds):
    fn()
    calls, t0 = 0, time.perf_counter()
    while True:
        fn()
        calls += 1
        el = time.perf_counter() - t0
        if el >= seconds and calls >= 3:
            return calls, el


def cpu_spmv_baselines(a, x, seconds):
    """cpu_spmv.cpp's three CsrMV strategies on the host cores, ~`seconds` each: the merge-path
    CsrMV, the row-split OmpCsrSpmv (:271-294) and the nonzero-split OmpNonzeroSplitCsrmm
    (:506-570).  cpu_spmv.cpp itself needs <mkl.h>; its kernels are timed through the reference's
    compiled work_2025 twins (oracle/_ref: OmpMergeCsrmm / OmpCsrSpmmT / OmpNonzeroSplitCsrmm at
    num_vectors = 1, the same operation order) where that build exists, else the oracle ports."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import REF_SO, Oracle, RefLib
    P = _threads()
    X = np.ascontiguousarray(x[:, None])
    orc = Oracle()
    legs = {}
    if os.path.exists(REF_SO):
        ref = RefLib()
        fns = {"merge_OmpMergeCsrmv": (lambda: ref.merge_csrmm(a, X, P), "reference"),
               "row_split_OmpCsrSpmv": (lambda: ref.csr_spmm_t(a, X, P), "reference"),
               "nonzero_split_OmpNonzeroSplitCsrmm": (lambda: ref.nonzero_split_csrmm(a, X, P), "reference")}
    else:
        y0 = np.zeros(a.num_rows)
        fns = {"merge_OmpMergeCsrmv": (lambda: orc.merge_csrmv(a, x, P), "port"),
               "row_split_OmpCsrSpmv": (lambda: orc.csr_spmv(a, x), "port"),
               "nonzero_split_OmpNonzeroSplitCsrmm": (lambda: orc.nonzero_split_csrmv_v1(a, x, min(P, 256), y0),
                                                      "port")}
    for name, (fn, kind) in fns.items():
        calls, el = _time_calls(fn, seconds)
        legs[name] = {"gflops": round(2.0 * a.num_nonzeros * calls / el / 1e9, 3),
                      "ms_per_call": round(el / calls * 1e3, 4), "cores": P, "kind": kind,
                      "sample": f"{calls} calls in {el:.1f} s"}
    return legs


def run_spmv_shapes(dev, cpu_seconds, do_cpu):
    """configs[0] (the reference's CPU merge SpMV on cant, core count stated) beside the GPU on
    the same cant-shaped matrix, and configs[1]'s second matrix (rma10 shape) on the GPU; both
    fit the Infinity Cache, so hot and cold (flushed) kernel times are reported."""
    out = {}
    shapes = {"cant": (CANT, "configs[0]: cant-shaped banded, 64.2 nnz/row, band +-2,000"),
              "rma10": (RMA10, "configs[1] second matrix: rma10-shaped banded, 50.7 nnz/row, band +-3,000"),
              # SURVEY 8(d) skewed variant: pwtk's m and nnz with power-law row lengths (merge-path balance)
              "powerlaw": (None, "skewed variant: pwtk's m and nnz, power-law row lengths (exponent 1.2, seed 3)")}
    for name, (sh, what) in shapes.items():
        if sh is None:
            a = mspmv.CsrMatrix.synth_powerlaw(PWTK["m"], PWTK["m"], PWTK["nnz"], 1.2, 3)
        else:
            a = mspmv.CsrMatrix.synth_banded(sh["m"], sh["nnz"], sh["band"], seed=sh["seed"])
        x, r = gpu_spmv_hot_cold(a, dev)
        r["workload"] = what
        if name == "powerlaw":
            lens = np.diff(a.row_offsets)
            r["row_length_max"], r["row_length_mean"] = int(lens.max()), round(float(lens.mean()), 1)
        if name in ("cant", "powerlaw") and do_cpu:
            r["cpu_baselines"] = cpu_spmv_baselines(a, x, cpu_seconds)
            best = max(v["gflops"] for v in r["cpu_baselines"].values())
            r["gpu_cold_vs_best_cpu"] = round(r["gflops_cold"] / best, 1)
        out[name] = r
    return out


class env_set:
    """Environment switches for the handles created inside the block (the plan decisions read them per
    handle: MSPMV_DIA, MSPMV_SPMV_RUNS)."""

    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def time_batch_on(mats, dxs, dys, dev, steps, **env):
    """Per-launch kernel ms of a batch of plain SpMVs on handles created under `env`, and the kernel name."""
    with env_set(**env):
        gs = [mspmv.GpuCsr(a, device=dev) for a in mats]
    try:
        mspmv.time_spmm_batch(gs, dxs, dys, 1, 5)
        _, kern_ms, _ = mspmv.time_spmm_batch(gs, dxs, dys, 1, steps)
        return kern_ms, gs[0].kernel_name()
    finally:
        for g in gs:
            g.close()


def merge_path_entry(kern_ms, kname, nb, nnz, what):
    return {"plan": what, "kernel": kname, "kernel_ms": round(kern_ms, 5),
            "gflops": round(2.0 * nnz / kern_ms / 1e6, 1), "bytes_per_launch": nb,
            "frac": round(nb / kern_ms / 1e6 / HBM_PEAK_GBS, 4)}


def run_merge_path_generic(dev, batch=4, steps=50):
    """The headline batch on the plain merge-path tiles with no node blocks (k_spmv_tile; run by bench.py
    as a child process under MSPMV_SPMV_BLOCKS=0, a per-process switch)."""
    mats = [mspmv.CsrMatrix.synth_fem_blocked(PWTK["m"], PWTK["nnz"], PWTK["block"], PWTK["half_band_nodes"],
                                              seed=1 + i) for i in range(batch)]
    dxs = [mspmv.DeviceBuffer.from_array(np.random.default_rng(2 + i).uniform(0.0, 1.0, a.num_cols), dev)
           for i, a in enumerate(mats)]
    dys = [mspmv.DeviceBuffer(8 * a.num_rows, dev) for a in mats]
    k, name = time_batch_on(mats, dxs, dys, dev, steps, MSPMV_SPMV_RUNS="0")
    a0 = mats[0]
    return merge_path_entry(k, name, spmv_bytes(a0.num_rows, a0.num_cols, a0.num_nonzeros), a0.num_nonzeros,
                            "merge-path tiles of 2,048 merge items, striped staging, no node blocks (MSPMV_SPMV_BLOCKS=0)")


def merge_path_generic_child(dev):
    """run_merge_path_generic in a child process (MSPMV_SPMV_BLOCKS is read once per process)."""
    import subprocess
    env = dict(os.environ, MSPMV_SPMV_BLOCKS="0")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--only", "merge_path_generic", "--device", str(dev)],
                       env=env, capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": (r.stderr or "no output")[-300:]}
    d = json.loads(lines[-1])
    d.pop("leg", None)
    return d


def run_window_shapes(dev, steps=40):
    """Shapes the offset windows were not designed on, at the nlpkkt120 size, SpMV cold-free
    back to back (1 GB+ per launch: never Infinity-Cache resident): the 27-point stencil with 1 % of the
    rows holding an off-pattern column and 0.1 % holding eight (rows of 35), and a KKT saddle point
    [[H, B^T], [B, -eps I]] (nlpkkt120's block structure: 27-point H, 7-point B; 34 offsets in the upper
    rows).  The default plan (windows plus a remainder) beside the merge-path tiles (MSPMV_DIA=0)."""
    out = {}
    shapes = {
        "stencil27_perturbed": (lambda: mspmv.CsrMatrix.synth_stencil_perturbed(
            NLPKKT120["dims"], seed=5, diag_shift=NLPKKT120["shift"], extra_frac=0.01, long_frac=0.001),
            "nlpkkt120-size 27-point stencil, 1 % of rows one off-pattern column, 0.1 % eight"),
        "kkt": (lambda: mspmv.CsrMatrix.synth_kkt(KKT120["dims"], seed=6, eps=KKT120["eps"]),
                "KKT saddle point [[H, B^T], [B, -eps I]], 27-point H, 7-point B, 2 x 120 x 120 x 123 rows"),
    }
    for name, (make, what) in shapes.items():
        a = make()
        n, nnz = a.num_rows, a.num_nonzeros
        nb = spmv_bytes(n, a.num_cols, nnz)
        w = mspmv.offset_windows(a)
        dx = mspmv.DeviceBuffer.from_array(np.random.default_rng(7).uniform(0, 1, a.num_cols), dev)
        dy = mspmv.DeviceBuffer(8 * n, dev)
        r = {"workload": what, "m": n, "nnz": nnz, "bytes_per_launch": nb,
             "window_remainder_entries": w["remainder"] if w else None,
             "window_sum_offsets": w["sum_offsets"] if w else None}
        for plan, env in (("default", {}), ("merge_path", {"MSPMV_DIA": "0"})):
            with env_set(**env):
                g = mspmv.GpuCsr(a, device=dev)
            with g:
                g.time_spmm(dx, dy, 1, 5)
                _, k, _ = g.time_spmm(dx, dy, 1, steps)
                r[plan] = {"kernel": g.kernel_name(), "kernel_ms": round(k, 5), "gflops": round(2.0 * nnz / k / 1e6, 1),
                           "frac": round(nb / k / 1e6 / HBM_PEAK_GBS, 4), "setup_ms": round(g.setup_ms, 2)}
        r["frac"] = r["default"]["frac"]
        dx.free()
        dy.free()
        out[name] = r
    return out


def run_pwtk_perturbed(dev, batch=4, steps=50):
    """The headline's FEM shape made imperfect (the node-block plan must not be all-or-
    nothing): pwtk's m and nnz, ~2 % of the nodes with 5 or 7 unknowns instead of 6 and ~1 % of the
    rows with one column outside their node's pattern (mspmv_synth_fem_perturbed).  Timed as the
    headline is: a batch of `batch` such matrices (> the Infinity Cache) back to back, per-launch
    kernel time from the kernels' own events."""
    mats, gs, dxs, dys = [], [], [], []
    for i in range(batch):
        a = mspmv.CsrMatrix.synth_fem_perturbed(PWTK["m"], PWTK["nnz"], PWTK["block"], PWTK["half_band_nodes"],
                                                0.02, 0.01, seed=11 + i)
        mats.append(a)
        gs.append(mspmv.GpuCsr(a, device=dev))
        dxs.append(mspmv.DeviceBuffer.from_array(np.random.default_rng(12 + i).uniform(0, 1, a.num_cols), dev))
        dys.append(mspmv.DeviceBuffer(8 * a.num_rows, dev))
    mspmv.time_spmm_batch(gs, dxs, dys, 1, 5)
    step_ms, kern_ms, kps = mspmv.time_spmm_batch(gs, dxs, dys, 1, steps)
    a0 = mats[0]
    nb = sum(spmv_bytes(a.num_rows, a.num_cols, a.num_nonzeros) for a in mats) / batch
    plan = gs[0].tile_plan(1)
    nt = plan["num_tiles"]
    reg = int(np.sum(plan["modes"] == 255))
    out = {"workload": "pwtk-shaped FEM, imperfect: 2 % of nodes 5 or 7 unknowns, 1 % of rows one off-pattern "
                       f"column; batch of {batch}, back to back",
           "m": a0.num_rows, "nnz": a0.num_nonzeros, "kernel": gs[0].kernel_name(),
           "tiles": nt, "block_tiles": gs[0].plan_block_tiles(1), "register_tiles_reported": reg,
           "bytes_per_launch": round(nb), "kernel_ms": round(kern_ms, 5), "step_ms": round(step_ms, 5),
           "kernels_per_step": kps, "GBps": round(nb / kern_ms / 1e6, 1),
           "gflops": round(2.0 * a0.num_nonzeros / kern_ms / 1e6, 1),
           "frac": round(nb / kern_ms / 1e6 / HBM_PEAK_GBS, 4)}
    for g in gs:
        g.close()
    for b in dxs + dys:
        b.free()
    return out


def run_spmm16(dev, cpu_seconds, do_cpu):
    """configs[2]: CSR SpMM fp64 with a 16-column row-major panel (OmpMergeCsrmm's layout,
    merge_based.hpp:46-153) on the cant and pwtk shapes; kernel time by HIP events over
    back-to-back launches, bytes = 12 nnz + 4 (m+1) + 8 L (n+m).  Beside it, the
    reference's own OmpMergeCsrmm(num_vectors = 16) on the host cores (cant shape, bounded)."""
    L, out = 16, {}
    shapes = {"cant": lambda: mspmv.CsrMatrix.synth_banded(62451, 4007383, 2000, seed=1),
              "pwtk": lambda: mspmv.CsrMatrix.synth_fem_blocked(PWTK["m"], PWTK["nnz"], PWTK["block"],
                                                                PWTK["half_band_nodes"], seed=1)}
    for name, make in shapes.items():
        a = make()
        X = np.random.default_rng(3).uniform(0.0, 1.0, (a.num_cols, L))
        with mspmv.GpuCsr(a, device=dev) as g:
            dX = mspmv.DeviceBuffer.from_array(X, dev)
            dY = mspmv.DeviceBuffer(8 * a.num_rows * L, dev)
            g.time_spmm(dX, dY, L, 5)
            _, kern_ms, _ = g.time_spmm(dX, dY, L, 100)
            _, cold_ms, _ = g.time_spmm(dX, dY, L, 80, FLUSH_BYTES)  # 8 blocks beside flush-only controls
            kname = g.spmm_kernel_name(L)
        nb = 12 * a.num_nonzeros + 4 * (a.num_rows + 1) + 8 * L * (a.num_cols + a.num_rows)
        out[name] = {"m": a.num_rows, "nnz": a.num_nonzeros, "kernel": kname, "bytes_per_launch": nb,
                     "hot_kernel_ms": round(kern_ms, 5), "hot_GBps": round(nb / kern_ms / 1e6, 1),
                     "hot_frac": round(nb / kern_ms / 1e6 / HBM_PEAK_GBS, 4),
                     "cold_kernel_ms": round(cold_ms, 5), "gflops_cold": round(2.0 * L * a.num_nonzeros / cold_ms / 1e6, 1),
                     "achieved_GBps": round(nb / cold_ms / 1e6, 1), "frac": round(nb / cold_ms / 1e6 / HBM_PEAK_GBS, 4),
                     "note": "hot: back-to-back launches (matrix + panel Infinity-Cache resident); cold: a 512 MiB "
                             "flush read sweep before every timed launch; frac on the cold time (SURVEY 8(d))"}
        if name == "cant" and do_cpu:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            from _oracle import REF_SO, RefLib
            if os.path.exists(REF_SO):
                threads = host_cores()
                ref = RefLib()
                ref.merge_csrmm(a, X, threads)
                calls, t0 = 0, time.perf_counter()
                while True:
                    ref.merge_csrmm(a, X, threads)
                    calls += 1
                    el = time.perf_counter() - t0
                    if el >= cpu_seconds and calls >= 3:
                        break
                out[name]["cpu_baseline"] = {
                    "gflops": round(2.0 * L * a.num_nonzeros * calls / el / 1e9, 2), "cores": threads,
                    "kind": "reference", "sample": f"work_2025 OmpMergeCsrmm(num_vectors=16), P={threads}, "
                                                   f"{calls} calls in {el:.1f} s"}
    out["workload"] = "CSR SpMM fp64, 16-column row-major panel (configs[2]), X ~ U(0,1) seed 3"
    return out


def resident_phases(g, db, dx, thr, stamp_iters=256):
    """Where an iteration of the register-resident CG goes (configs[3]'s kernel keeps the matrix in
    VGPRs/LDS, so its 'bytes per iteration' are a speed figure, not HBM traffic): one extra solve with
    wall_clock64() stamps (100 MHz) at the phase boundaries of every workgroup (mspmv_cg_resident_stamps),
    medians over workgroups and iterations 1..stamp_iters-1:
      spmv    iteration start -> the workgroup's rows of Ap done (p gathers + row sums)
      handoff1 the LAST workgroup's Ap done -> this workgroup has the p.Ap total (the reduction hand-off
               itself; time waiting for slower workgroups is 'skew1')
      update  p.Ap total -> the workgroup's r update done
      handoff2 the last workgroup's r done -> this workgroup has the r.r total ('skew2' likewise)
    The stamped solve runs beside no other work; its stamps add a barrier per phase, so its
    iteration time is quoted next to the unstamped one."""
    its, st = g.cg_resident_stamps(db, dx, 10000, thr, stamp_iters)
    k = min(its, stamp_iters)
    if k < 3:
        return None
    t = st[1:k].astype(np.int64)          # [iters][G][5], skip iteration 0 (cold)
    us = 0.01                             # one tick of the 100 MHz clock in microseconds
    last1 = t[:, :, 1].max(axis=1, keepdims=True)
    last3 = t[:, :, 3].max(axis=1, keepdims=True)
    med = lambda a: round(float(np.median(a)) * us, 3)
    if "single_reduction" in g.cg_kernel_name():
        # one hand-off per iteration: stamps 1 = 2 = 3 after the SpMV (A w) and the vector updates
        out = {"form": "single_reduction", "stamped_iterations": int(k - 1), "workgroups": int(t.shape[1]),
               "spmv_update_us": med(t[:, :, 1] - t[:, :, 0]),
               "skew_us": med(last3[:, 0:1] - t[:, :, 3]),
               "handoff_us": med(t[:, :, 4] - last3),
               "spmv_update_max_us": round(float(np.median((t[:, :, 1] - t[:, :, 0]).max(axis=1))) * us, 3)}
    else:
        out = {"form": "classic", "stamped_iterations": int(k - 1), "workgroups": int(t.shape[1]),
               "spmv_us": med(t[:, :, 1] - t[:, :, 0]),
               "skew1_us": med(last1[:, 0:1] - t[:, :, 1]),
               "handoff1_us": med(t[:, :, 2] - last1),
               "update_us": med(t[:, :, 3] - t[:, :, 2]),
               "skew2_us": med(last3[:, 0:1] - t[:, :, 3]),
               "handoff2_us": med(t[:, :, 4] - last3),
               "spmv_max_us": round(float(np.median((t[:, :, 1] - t[:, :, 0]).max(axis=1))) * us, 3)}
    out["iteration_us"] = med(t[1:, :, 0] - t[:-1, :, 0])
    out["note"] = ("medians over workgroups x iterations of wall_clock64 phase stamps; handoff = last "
                   "publisher -> total received; skew = own publish -> last publisher")
    return out


def run_cg_single(dev, cpu_seconds, do_cpu):
    """configs[3]: CGSolveSingle on a parabolic_fem-shaped SPD matrix."""
    pf = mspmv.CsrMatrix.synth_stencil(0, PARABOLIC_FEM["m"], PARABOLIC_FEM["width"],
                                       diag_shift=PARABOLIC_FEM["shift"])
    n = pf.num_rows
    b = glibc_rhs(42, n)
    thr = float(np.sqrt(np.sum(b * b)) * 1e-5)  # calculate_threshold quirk, cpu_singlecg.cpp:92
    with mspmv.GpuCsr(pf, device=dev) as g:
        db, dx = mspmv.DeviceBuffer.from_array(b, dev), mspmv.DeviceBuffer(8 * n, dev)
        g.cg_dev(db, dx, 1, 10000, thr)  # warm (graph, workspace)
        t0 = time.perf_counter()
        it, _, st = g.cg_dev(db, dx, 1, 10000, thr)
        el = time.perf_counter() - t0
        kernel = g.cg_kernel_name()
        phases = resident_phases(g, db, dx, thr) if kernel.startswith("k_cg_resident") else None
        db.free()
        dx.free()
    ips = it / el
    out = {"workload": f"CGSolveSingle, parabolic_fem-shaped SPD (7-pt FEM, diag shift {PARABOLIC_FEM['shift']}) "
                       f"m={n} nnz={pf.num_nonzeros}, srand(42) RHS, tol = 1e-5*||b|| (cpu_singlecg quirk)",
           "iterations": it, "seconds": round(el, 5), "iters_per_s": round(ips, 1),
           "us_per_iter": round(el / max(it, 1) * 1e6, 2),
           # SURVEY 8(d)'s bytes per iteration x iterations/s: a SPEED figure here, not HBM traffic --
           # the register-resident kernel keeps the matrix in VGPRs/LDS and moves only the gathered
           # vector and the hand-offs per iteration, so this can exceed the 8 TB/s HBM peak
           "equiv_GBps": round(cg_iter_bytes(n, pf.num_nonzeros) * ips / 1e9, 1),
           "speed_equiv_frac": round(cg_iter_bytes(n, pf.num_nonzeros) * ips / 1e9 / HBM_PEAK_GBS, 4),
           "speed_equiv_note": "SURVEY 8(d) bytes/iteration x iterations/s over 8 TB/s; the resident kernel does not "
                               "stream these bytes (matrix on chip), so this is a speed figure, not an HBM fraction",
           "status": st, "kernel": kernel}
    if phases:
        out["resident_phases"] = phases
    out["pipelined_large"] = run_cg_single_pipelined(dev)
    if do_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from _oracle import Oracle
        orc = Oracle()
        k, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < cpu_seconds:
            _, its, _ = orc.cg_single(pf, b, 200, thr)
            k += its
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"iters_per_s": round(k / el, 1), "cores": orc.lib.orc_max_threads(), "kind": "port",
                               "sample": f"oracle CGSolveSingle restatement (the reference's CG headers need "
                                         f"<mkl.h>), {k} iterations in {el:.1f} s"}
    return out


CG_LARGE = dict(dims=(75, 76, 75), shift=1e-2)  # 427,500 rows, 11.2 M nonzeros: pwtk's size, SPD


def run_cg_single_pipelined(dev):
    """CGSolveSingle on a pwtk-size SPD matrix (27-point stencil, 11.2 M nonzeros) through the two-kernel
    pipelined form -- the path a single-RHS matrix takes when it does not fit the register-resident
    kernel (MSPMV_CG_RESIDENT=0 makes sure of it here).  Every iteration streams the matrix from HBM /
    the Infinity Cache, so the SURVEY 8(d) bytes per iteration give a real fraction of the roofline."""
    nx, ny, nz = CG_LARGE["dims"]
    a = mspmv.CsrMatrix.synth_stencil(1, nx * ny * nz, nx, ny, nz, seed=9, diag_shift=CG_LARGE["shift"])
    n = a.num_rows
    b = glibc_rhs(42, n)
    thr = float(np.sqrt(np.sum(b * b)) * 1e-5)
    with env_set(MSPMV_CG_RESIDENT="0"), mspmv.GpuCsr(a, device=dev) as g:
        db, dx = mspmv.DeviceBuffer.from_array(b, dev), mspmv.DeviceBuffer(8 * n, dev)
        g.cg_dev(db, dx, 1, 10000, thr)
        els = []
        for _ in range(5):  # whole solves (host loop, graph replays, final sync): the median
            t0 = time.perf_counter()
            it, _, st = g.cg_dev(db, dx, 1, 10000, thr)
            els.append(time.perf_counter() - t0)
        el = float(np.median(els))
        kernel = g.cg_kernel_name()
        db.free()
        dx.free()
    ips = it / el
    return {"workload": f"CGSolveSingle, pwtk-size SPD 27-point stencil (diag shift {CG_LARGE['shift']}) m={n} "
                        f"nnz={a.num_nonzeros}, srand(42) RHS, tol = 1e-5*||b||; the two-kernel pipelined form "
                        f"(MSPMV_CG_RESIDENT=0), median of 5 solves",
            "iterations": it, "seconds": round(el, 5), "iters_per_s": round(ips, 1),
            "us_per_iter": round(el / max(it, 1) * 1e6, 2),
            "achieved_GBps": round(cg_iter_bytes(n, a.num_nonzeros) * ips / 1e9, 1),
            "roofline_frac": round(cg_iter_bytes(n, a.num_nonzeros) * ips / 1e9 / HBM_PEAK_GBS, 4),
            "status": st, "kernel": kernel}


def run_cg_multi(d, dev):
    """configs[4]: CGSolveMultiple, 8 RHS, nlpkkt120-sized 27-point SPD; row-sharded at N > 1."""
    nx, ny, nz = NLPKKT120["dims"]
    L = NLPKKT120["L"]
    nk = mspmv.CsrMatrix.synth_stencil(1, nx * ny * nz, nx, ny, nz, diag_shift=NLPKKT120["shift"])
    n = nk.num_rows
    B = np.random.default_rng(42).uniform(0, 1, (n, L))
    thr = float(np.sqrt(np.sum(B.reshape(-1)[:n] ** 2)) * 1e-5)  # calculate_threshold on the flat buffer
    spmv_large = None
    if d.world == 1:
        with mspmv.GpuCsr(nk, device=dev) as g:
            dB, dX = mspmv.DeviceBuffer.from_array(B, dev), mspmv.DeviceBuffer(8 * n * L, dev)
            g.cg_dev(dB, dX, L, 50000, thr)
            t0 = time.perf_counter()
            it, _, st = g.cg_dev(dB, dX, L, 50000, thr)
            el = time.perf_counter() - t0
            # the north-star SpMV target is also judged on this nlpkkt120-sized,
            # never-cache-resident matrix (1.2 GB per SpMV); single RHS, back-to-back launches
            dx1 = mspmv.DeviceBuffer.from_array(np.random.default_rng(5).uniform(0, 1, n), dev)
            dy1 = mspmv.DeviceBuffer(8 * n, dev)
            g.time_spmm(dx1, dy1, 1, 5)
            call_ms, kern_ms, _ = g.time_spmm(dx1, dy1, 1, 40)
            nb = spmv_bytes(n, n, nk.num_nonzeros)
            spmv_large = {"workload": f"SpMV fp64 1 RHS, nlpkkt120-sized 27-pt matrix m={n} nnz={nk.num_nonzeros}",
                          "kernel": g.kernel_name(), "kernel_ms": round(kern_ms, 5), "gflops": round(2.0 * nk.num_nonzeros / kern_ms / 1e6, 1),
                          "bytes_per_launch": nb, "achieved_GBps": round(nb / kern_ms / 1e6, 1),
                          "frac": round(nb / kern_ms / 1e6 / HBM_PEAK_GBS, 4)}
            with env_set(MSPMV_DIA="0"):  # north_star's merge-based figure: the same matrix on the merge-path tiles
                gm = mspmv.GpuCsr(nk, device=dev)
            with gm:
                gm.time_spmm(dx1, dy1, 1, 5)
                _, mk, _ = gm.time_spmm(dx1, dy1, 1, 40)
                spmv_large["merge_path"] = merge_path_entry(mk, gm.kernel_name(), nb, nk.num_nonzeros,
                                                            "merge-path tiles (MSPMV_DIA=0)")
        mode = "1 GPU"
    else:
        rb = mspmv.dist_partition(nk, d.world)
        loc = mspmv.local_rows(nk, rb, d.rank)
        dc = mspmv.DistCsr(d.comm(dev), rb, loc)  # the rank's one communicator (Dist.comm)
        lo, hi = int(rb[d.rank]), int(rb[d.rank + 1])
        dB = mspmv.DeviceBuffer.from_array(np.ascontiguousarray(B[lo:hi]), dev)
        dX = mspmv.DeviceBuffer(8 * max(hi - lo, 1) * L, dev)
        dc.cg_dev(dB, dX, L, 50000, thr)
        d.barrier()
        t0 = time.perf_counter()
        it, _, st = dc.cg_dev(dB, dX, L, 50000, thr)
        el = time.perf_counter() - t0
        d.barrier()
        el = d.max(el)
        dc.close()
        mode = f"row-sharded over {d.world} GPUs (RCCL halo exchange + 2 all-reduces per iteration)"
    ips = it / el
    out = {"workload": f"CGSolveMultiple L={L}, nlpkkt120-sized 27-pt SPD (diag shift {NLPKKT120['shift']}) "
                       f"m={n} nnz={nk.num_nonzeros}, {mode}",
           "iterations": it, "seconds": round(el, 4), "iters_per_s": round(ips, 1),
           "ms_per_iter": round(el / max(it, 1) * 1e3, 3),
           "achieved_GBps": round(cg_iter_bytes(n, nk.num_nonzeros, L) * ips / 1e9, 1),
           "roofline_frac": round(cg_iter_bytes(n, nk.num_nonzeros, L) * ips / 1e9 / HBM_PEAK_GBS, 4), "status": st}
    return out, spmv_large


class Watchdog:
    """N > 1: the collective part of the run (sharded SpMV headline, sharded CG) must finish within
    `seconds`.  If it does not -- an RCCL hang, or a rank that failed while the others wait in a
    collective -- rank 0 prints what it has (the headline, if measured, with an error field) and
    every rank exits 3: a hang is reported as a failure, never as a success.  The lock is held
    through the print and exit, and finish() takes it too, so exactly one thread prints."""

    def __init__(self, d, seconds):
        self.d, self.seconds, self.result = d, seconds, None
        self.lock, self.done = threading.Lock(), False
        self.timer = threading.Timer(seconds, self._fire)
        self.timer.daemon = True
        self.timer.start()

    def _fire(self):
        with self.lock:
            if self.done:
                return
            self.done = True
            if self.d.rank == 0:
                out = dict(self.result or {"metric": METRIC, "value": None, "n_gpus": self.d.world})
                out["error"] = f"multi-GPU run did not finish within {self.seconds:.0f} s (RCCL hang?)"
                print(json.dumps(out), flush=True)
            print(f"rank {self.d.rank}: multi-GPU run hung (> {self.seconds:.0f} s), exiting 3", file=sys.stderr)
            sys.stderr.flush()
            os._exit(3)

    def finish(self):
        """Mark the run finished; False if the watchdog already fired (and is exiting)."""
        with self.lock:
            if self.done:
                return False
            self.done = True
        self.timer.cancel()
        return True


def run_sharded_headline(d, dev, args):
    """N > 1 headline (weak scaling): each of the batch's matrices is ONE node-blocked FEM matrix of
    N x 217,918 rows (N x 11,524,432 nonzeros, the pwtk shape's rows, band and seeds), sharded by
    merge-path row blocks (mspmv_dist_partition): every rank holds a pwtk-sized row block and x's
    slice, and each SpMV exchanges the halo rows of x with RCCL send/recv over xGMI (the row blocks
    couple through the band) while the block interior is multiplied; the rows next to the block
    ends follow the exchange.  At N = 1 this is exactly the single-GPU headline (no halo)."""
    world, rank = d.world, d.rank
    M, NNZ = PWTK["m"] * world, PWTK["nnz"] * world
    ro = (np.arange(M + 1, dtype=np.int64) * NNZ // M).astype(np.int32)  # the generator's row offsets
    rb = mspmv.dist_partition_offsets(ro, M, NNZ, world)
    lo, hi = int(rb[rank]), int(rb[rank + 1])
    dcs, dys, xps, infos, nnz_loc = [], [], [], [], 0
    comm = d.comm(dev)  # ONE communicator (and stream) for every matrix of the batch: the exchanges are
    for i in range(args.batch):  # one stream-ordered sequence, issued in the same order on every rank
        loc = mspmv.CsrMatrix.synth_fem_blocked_rows(M, NNZ, PWTK["block"], PWTK["half_band_nodes"], 1 + i, lo, hi)
        dc = mspmv.DistCsr(comm, rb, loc)
        xp = dc.x_ext(1)
        mspmv.memcpy_h2d_ptr(xp, np.random.default_rng(2 + i).uniform(0.0, 1.0, M)[lo:hi])
        dcs.append(dc)
        xps.append(xp)
        dys.append(mspmv.DeviceBuffer(8 * max(hi - lo, 1), dev))
        infos.append(dc.info())
        nnz_loc = loc.num_nonzeros
    for _ in range(max(args.warmup, 1)):
        for dc, xp, dy in zip(dcs, xps, dys):
            dc.spmm_dev(xp, dy, 1, sync=False)
    for dc in dcs:
        dc.sync()
    # per-rank SpMV alone (no exchange): the head / interior / tail launches back to back
    loc_ms = float(np.mean([dc.time_local(dy, 1, 100) for dc, dy in zip(dcs, dys)]))
    loc_ms = d.max(loc_ms)
    d.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for dc, xp, dy in zip(dcs, xps, dys):
            dc.spmm_dev(xp, dy, 1, sync=False)
    for dc in dcs:
        dc.sync()
    el = time.perf_counter() - t0
    d.barrier()
    el = d.max(el)
    inf = infos[0]
    m_loc, n_ext = inf["n_own"], inf["n_own"] + inf["n_halo"]
    bytes_local = 12 * nnz_loc + 4 * (m_loc + 1) + 8 * n_ext + 8 * m_loc
    achieved = bytes_local / (loc_ms * 1e-3) / 1e9
    value = 2.0 * NNZ * args.batch * args.steps / el / 1e9
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "GFLOP/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (pwtk-shaped 6-DOF FEM-blocked CSR scaled to N x the rows, splitmix64 values; "
                "SuiteSparse unavailable offline)",
        "config": {"workload": f"merge-path CSR SpMV fp64, 1 RHS, batch of {args.batch} FEM-blocked matrices of "
                               f"{world} x 217,918 rows per step, row-block sharded (configs[1] per GPU)",
                   "m": M, "nnz": NNZ, "m_per_gpu": m_loc, "nnz_per_gpu": nnz_loc, "batch": args.batch,
                   "parallelism": f"row-block sharding over {world} GPUs: RCCL halo exchange of x (send/recv over "
                                  f"xGMI) overlapped with the block interior"},
        "halo": {"rows": inf["n_halo"], "rows_sent": inf["n_send"], "bytes_per_exchange": 8 * inf["n_halo"]},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "local SpMV (head + interior + tail launches)", "bytes_per_launch": bytes_local,
                     "kernel_ms": round(loc_ms, 5),
                     "note": "per-rank local SpMV without the exchange, HIP events, max over ranks; algorithmic "
                             "bytes 12 nnz + 4 (m+1) + 8 (n_own + n_halo) + 8 m of the rank's block"},
    }
    for dc in dcs:
        dc.close()
    return result


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-cg", action="store_true")
    ap.add_argument("--cg-timeout", type=float, default=400.0,
                    help="N > 1: seconds allowed for the collective part (sharded SpMV headline + sharded CG); "
                         "past it rank 0 prints what it has and every rank exits 3")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the hot-matrix and scatter-band side measurements (profiling runs: the "
                         "headline kernel's rocprofv3 average then covers exactly the timed launches)")
    ap.add_argument("--device", type=int, default=None, help="--only legs: the HIP device (default LOCAL_RANK)")
    ap.add_argument("--only", choices=["spmm16", "spmv_shapes", "cg_single", "cg_multi", "pwtk_perturbed",
                                       "merge_path_generic", "window_shapes"],
                    help="run one side measurement alone and print its JSON (profiling: rocprofv3 then sees only "
                         "that leg's launches; tools/profile_legs.sh)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch check only: every rank joins the gloo group and reports WORLD_SIZE / RANK; "
                         "no GPU is touched")
    args = ap.parse_args()

    d = Dist(args.gpus)
    if args.dry_run:
        ranks = [(d.rank, d.world)]
        if d.td:
            ranks = [None] * d.world
            d.td.all_gather_object(ranks, (d.rank, d.world))
        if d.rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": args.gpus, "world_size": d.world,
                              "ranks": [{"rank": r, "world_size": w} for r, w in ranks]}), flush=True)
        if d.td:
            d.td.destroy_process_group()
        return
    if args.only:
        dev = d.local if args.device is None else args.device
        do_cpu = not args.no_cpu
        if args.only == "merge_path_generic":
            r = run_merge_path_generic(dev)
        elif args.only == "window_shapes":
            r = run_window_shapes(dev)
        elif args.only == "spmm16":
            r = run_spmm16(dev, min(args.cpu_seconds, 5.0), do_cpu)
        elif args.only == "spmv_shapes":
            r = run_spmv_shapes(dev, min(args.cpu_seconds, 3.0), do_cpu)
        elif args.only == "cg_single":
            r = run_cg_single(dev, min(args.cpu_seconds, 10.0), do_cpu)
        elif args.only == "pwtk_perturbed":
            r = run_pwtk_perturbed(dev)
        else:
            r, large = run_cg_multi(d, dev)
            if large:
                r["spmv_nlpkkt120_size"] = large
        if d.rank == 0:
            print(json.dumps({"leg": args.only, **r}), flush=True)
        return
    dev = d.local
    if os.environ.get("MSPMV_BENCH_SHARE_DEVICE") == "1":  # rehearsal of N > 1 on a one-GPU box
        dev = d.local % max(mspmv.device_count(), 1)
    if mspmv.device_count() <= dev:
        raise SystemExit(f"rank {d.rank}: no HIP device {dev}")

    # The headline runs under a watchdog at N > 1: an RCCL hang must end the job (exit 3) with
    # the line printed so far, never hang it or pass as success.
    guard = Watchdog(d, args.cg_timeout) if d.world > 1 else None
    if d.world > 1 or os.environ.get("MSPMV_BENCH_SHARDED") == "1":  # the latter: the N > 1 path at N = 1 (tests)
        result = run_sharded_headline(d, dev, args)
        if guard:
            guard.result = result
    else:
        mats, gs, dxs, dys, xs = [], [], [], [], []
        for i in range(args.batch):
            a = mspmv.CsrMatrix.synth_fem_blocked(PWTK["m"], PWTK["nnz"], PWTK["block"], PWTK["half_band_nodes"],
                                                  seed=1 + i + 1000 * d.rank)
            x = np.random.default_rng(2 + i + 1000 * d.rank).uniform(0.0, 1.0, a.num_cols)
            mats.append(a)
            gs.append(mspmv.GpuCsr(a, device=dev))
            xs.append(x)
            dxs.append(mspmv.DeviceBuffer.from_array(x, dev))
            dys.append(mspmv.DeviceBuffer(8 * a.num_rows, dev))
        a0 = mats[0]

        mspmv.time_spmm_batch(gs, dxs, dys, 1, max(args.warmup, 1))   # warmup (untimed)
        for g in gs:
            g.sync()
        d.barrier()
        t0 = time.perf_counter()
        step_ms_ev, kern_ms, kps = mspmv.time_spmm_batch(gs, dxs, dys, 1, args.steps)
        for g in gs:
            g.sync()
        el = time.perf_counter() - t0
        d.barrier()
        el = d.max(el)
        kern_ms = d.max(kern_ms)

        flops = 2.0 * a0.num_nonzeros * args.batch * args.steps * d.world
        value = flops / el / 1e9
        bytes_launch = spmv_bytes(a0.num_rows, a0.num_cols, a0.num_nonzeros)
        achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
        hot_ms = hot_kern = None
        if not args.no_extras:
            hot_ms, hot_kern, _ = mspmv.time_spmm_batch(gs[:1], dxs[:1], dys[:1], 1, 200)
        kname = gs[0].kernel_name()
        traffic, traffic_src = pmc_traffic(kname, bytes_launch)
        ref_eff = (a0.num_nonzeros * 20 + a0.num_rows * 12) / (kern_ms * 1e-3) / 1e9  # cpu_spmv.cpp:722-726

        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "GFLOP/s", "n_gpus": d.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (pwtk-shaped 6-DOF FEM-blocked CSR, splitmix64 values; SuiteSparse unavailable offline)",
            "config": {"workload": f"merge-path CSR SpMV fp64, 1 RHS, batch of {args.batch} pwtk-shaped matrices "
                                   f"per step per GPU (configs[1])",
                       "m": a0.num_rows, "nnz": a0.num_nonzeros, "batch": args.batch,
                       "parallelism": f"independent SpMV batches, {d.world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kname, "bytes_per_launch": bytes_launch,
                         "kernel_ms": round(kern_ms, 5), "kernels_per_step": kps,
                         "note": "achieved = algorithmic bytes (12 B/nnz: int32 columns + f64 values, SURVEY 8(d)) / "
                                 "kernel time; the kernel streams per-tile 16-bit column offsets (10 B/nnz), so "
                                 "traffic (PMC bytes actually moved per launch) is below bytes_per_launch"},
            "spmv_gflops_per_launch": round(2.0 * a0.num_nonzeros / (kern_ms * 1e-3) / 1e9, 2),
            "reference_effective_GBps": round(ref_eff, 1),
            "setup_ms": round(gs[0].setup_ms, 2),
        }
        if not args.no_extras:  # the practical ceiling beside the spec peak
            rd = mspmv.time_stream_read(dev, 1 << 30, 20)
            result["roofline"]["measured_read_GBps"] = round(rd, 1)
            result["roofline"]["frac_of_measured_read"] = round(achieved / rd, 4) if rd > 0 else None
            result["roofline"]["measured_read_note"] = ("nontemporal read of 1 GiB (> the 256 MiB Infinity Cache), "
                                                        "one contiguous slice per workgroup, 4 workgroups per CU, "
                                                        "20 passes, HIP events (the best of the read shapes in "
                                                        "tools/read_ceiling.hip)")
        if not args.no_extras:
            # north_star's figure is merge-based CsrMV: the same batch on the merge-path tile plan (node blocks
            # in registers, tiles cut at 2,048 merge items) beside the default run-balanced plan, and on the
            # generic merge-path tiles (no node blocks) in a child process
            mk, mname = time_batch_on(mats, dxs, dys, dev, 50, MSPMV_SPMV_RUNS="0")
            result["merge_path"] = {
                "note": "the headline batch on merge-path plans (the default plan above is run-balanced: tiles cut at "
                        "FEM node-run starts, DESIGN 4.2)",
                "node_blocks": merge_path_entry(mk, mname, bytes_launch, a0.num_nonzeros,
                                                "merge-path tiles of 2,048 merge items, node blocks in registers "
                                                "(MSPMV_SPMV_RUNS=0)"),
                "generic": merge_path_generic_child(dev) if d.world == 1 else None}
        if hot_ms is not None:
            result["hot_single_matrix"] = {"ms_per_call": round(hot_ms, 5), "kernel_ms": round(hot_kern, 5),
                                           "GBps_vs_algorithmic": round(bytes_launch / (hot_kern * 1e-3) / 1e9, 1),
                                           "note": "one 143 MB matrix back to back: Infinity-Cache resident"}
        for g in gs:
            g.close()

        if d.rank == 0 and not args.no_extras:  # stress shape: columns scattered one per band slice (x gathers hit a new line each)
            # a batch of 4 (> the Infinity Cache, as the headline); the plain SpMV takes the column-slab
            # plan here by default (line-bound gathers: mspmv_slab.hip)
            scs = [mspmv.CsrMatrix.synth_banded(PWTK["m"], PWTK["nnz"], 10000, seed=77 + i) for i in range(4)]
            sgs = [mspmv.GpuCsr(a, device=dev) for a in scs]
            sbx = [mspmv.DeviceBuffer.from_array(np.random.default_rng(3 + i).uniform(0, 1, a.num_cols), dev)
                   for i, a in enumerate(scs)]
            sby = [mspmv.DeviceBuffer(8 * a.num_rows, dev) for a in scs]
            mspmv.time_spmm_batch(sgs, sbx, sby, 1, 5)
            _, sk, _ = mspmv.time_spmm_batch(sgs, sbx, sby, 1, 50)
            snb = sum(spmv_bytes(a.num_rows, a.num_cols, a.num_nonzeros) for a in scs) / len(scs)
            result["scatter_band_stress"] = {"kernel": sgs[0].kernel_name(), "kernel_ms": round(sk, 5),
                                             "bytes_per_launch": round(snb),
                                             "GBps_vs_algorithmic": round(snb / (sk * 1e-3) / 1e9, 1),
                                             "frac": round(snb / sk / 1e6 / HBM_PEAK_GBS, 4),
                                             "note": "pwtk size, 53 columns per row scattered over +-10,000; batch of 4 "
                                                     "distinct matrices back to back"}
            for g in sgs:
                g.close()
            for b_ in sbx + sby:
                b_.free()

        if d.rank == 0 and not args.no_extras:
            result["spmv_pwtk_perturbed"] = run_pwtk_perturbed(dev)
            result["spmm16"] = run_spmm16(dev, min(args.cpu_seconds, 5.0), d.world == 1 and not args.no_cpu)
            result["spmv_shapes"] = run_spmv_shapes(dev, min(args.cpu_seconds, 3.0), d.world == 1 and not args.no_cpu)
            result["window_shapes"] = run_window_shapes(dev)

        if d.rank == 0 and d.world == 1 and not args.no_cpu:
            y_cpu, cb = cpu_baseline(a0, xs[0], args.cpu_seconds)
            result["cpu_baseline"] = cb
            with mspmv.GpuCsr(a0, device=dev) as g:
                y_gpu = g.spmv(xs[0])
            rel = float(np.max(np.abs(y_gpu - y_cpu) / np.maximum(np.abs(y_cpu), 1e-300)))
            result["cpu_baseline"]["gpu_vs_cpu_max_rel_diff"] = rel
            result["speedup_vs_cpu"] = round(value / cb["value"], 1)
    if not args.no_cg:
        try:
            if d.world == 1:
                result["cg_single"] = run_cg_single(dev, min(args.cpu_seconds, 10.0), not args.no_cpu)
            result["cg_multi"], large = run_cg_multi(d, dev)
            if large:
                result["spmv_nlpkkt120_size"] = large
        except Exception as e:  # the headline line must still print
            result["cg_error"] = repr(e)[:300]

    d.close_comm()
    if guard:
        if not guard.finish():  # the watchdog fired meanwhile and owns the exit
            return
    if d.world > 1 and not args.no_cpu:
        # north_star: the reference CPU path timed on the host cores "in the same run" at every N;
        # rank 0, after the GPU legs (the other ranks wait at the barrier below)
        if d.rank == 0:
            a0 = mspmv.CsrMatrix.synth_fem_blocked(PWTK["m"], PWTK["nnz"], PWTK["block"], PWTK["half_band_nodes"],
                                                   seed=1)
            x0 = np.random.default_rng(2).uniform(0.0, 1.0, a0.num_cols)
            _, cb = cpu_baseline(a0, x0, args.cpu_seconds)
            cb["sample"] += "; one GPU's share of the sharded workload (a pwtk-shaped matrix), rank 0's host"
            result["cpu_baseline"] = cb
            result["speedup_vs_cpu"] = round(result["value"] / cb["value"], 1)
        d.barrier()
    if d.rank == 0:
        print(json.dumps(result), flush=True)
    if d.td:
        d.td.destroy_process_group()


if __name__ == "__main__":
    main()
