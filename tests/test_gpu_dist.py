"""GPU: the row-sharded SpMM / CG through RCCL (mspmv_dist.hip), against the oracle.

World size 1 runs the whole RCCL code path (communicator, request exchange, pack, all-reduces)
on the one GPU of a test box.  A 2-rank run on one device is attempted as well; RCCL may
refuse two ranks on one GPU, in which case that case is skipped (the 8-GPU path runs in the
driver's multi-GPU bench).
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    return gpu_available


def _matrix():
    import mspmv
    return mspmv.CsrMatrix.synth_stencil(1, 16 * 17 * 18, 16, 17, 18)


def _run_rank(rank, world, uid, L, out_dir):
    for p in (ROOT, os.path.join(ROOT, "sparse-matrix-linear-equations_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import mspmv
    a = _matrix()
    rb = mspmv.dist_partition(a, world)
    loc = mspmv.local_rows(a, rb, rank)
    d = mspmv.DistCsr(uid, world, rank, 0, rb, loc)
    lo, hi = int(rb[rank]), int(rb[rank + 1])
    rng = np.random.default_rng(5)
    X = rng.uniform(-1, 1, (a.num_rows, L))
    dX = mspmv.DeviceBuffer.from_array(np.ascontiguousarray(X[lo:hi]))
    dY = mspmv.DeviceBuffer(8 * (hi - lo) * L)
    d.spmm_dev(dX, dY, L)
    Y = dY.download((hi - lo, L))
    B = rng.uniform(0, 1, (a.num_rows, L))
    dB = mspmv.DeviceBuffer.from_array(np.ascontiguousarray(B[lo:hi]))
    dXs = mspmv.DeviceBuffer(8 * (hi - lo) * L)
    it, hist, st = d.cg_dev(dB, dXs, L, 3000, 1e-9, hist_cap=3000)
    Xs = dXs.download((hi - lo, L))
    d.close()
    np.save(os.path.join(out_dir, f"Y_{rank}.npy"), Y)
    np.save(os.path.join(out_dir, f"X_{rank}.npy"), Xs)
    np.save(os.path.join(out_dir, f"h_{rank}.npy"), hist)
    np.save(os.path.join(out_dir, f"m_{rank}.npy"), np.array([it, st]))


def _check(tmp_path, orc, world, L):
    a = _matrix()
    rng = np.random.default_rng(5)
    X = rng.uniform(-1, 1, (a.num_rows, L))
    B = rng.uniform(0, 1, (a.num_rows, L))
    Y = np.concatenate([np.load(tmp_path / f"Y_{g}.npy") for g in range(world)])
    np.testing.assert_allclose(Y, orc.csr_spmm_t(a, X), rtol=1e-13, atol=1e-13)
    Xo, it_o, ho = orc.cg_multi(a, B, 3000, 1e-9, kernel=1, P=8, hist_cap=3000)
    it, st = np.load(tmp_path / "m_0.npy")
    assert st == 0 and abs(int(it) - it_o) <= 1
    h = np.load(tmp_path / "h_0.npy")
    k = min(len(h), len(ho))
    np.testing.assert_allclose(h[:k], ho[:k], rtol=0, atol=1e-10)
    Xg = np.concatenate([np.load(tmp_path / f"X_{g}.npy") for g in range(world)])
    assert np.linalg.norm(Xg - Xo) <= 1e-8 * np.linalg.norm(Xo)


@pytest.mark.parametrize("L", [1, 8])
def test_dist_world1(tmp_path, orc, L):
    import mspmv
    _run_rank(0, 1, mspmv.comm_unique_id(), L, str(tmp_path))
    _check(tmp_path, orc, 1, L)


def _spawn_rank(rank, world, uid, L, out_dir):
    try:
        _run_rank(rank, world, uid, L, out_dir)
    except Exception as e:  # report, the parent decides
        with open(os.path.join(out_dir, f"err_{rank}.txt"), "w") as f:
            f.write(repr(e))


def test_dist_world2_one_device(tmp_path, orc):
    import multiprocessing as mp
    import mspmv
    uid = mspmv.comm_unique_id()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_spawn_rank, args=(r, 2, uid, 4, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        if p.is_alive():
            p.kill()
            pytest.fail("2-rank RCCL run did not finish")
    errs = [open(tmp_path / f).read() for f in os.listdir(tmp_path) if f.startswith("err_")]
    if errs:
        if any("RCCL" in e or "ncclCommInitRank" in e for e in errs):
            pytest.skip(f"RCCL refuses two ranks on one device: {errs[0][:200]}")
        pytest.fail("; ".join(errs))
    _check(tmp_path, orc, 2, 4)


_SPLIT_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import mspmv
from _oracle import Oracle
orc = Oracle()
a = mspmv.CsrMatrix.synth_fem_blocked(36000, 36000 * 53, 6, 340, seed=3)
rb = mspmv.dist_partition(a, 1)
d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))
rng = np.random.default_rng(4)
for L in (1, 3, 8):
    X = rng.uniform(-1, 1, (a.num_rows, L))
    dX = mspmv.DeviceBuffer.from_array(X)
    dY = mspmv.DeviceBuffer(8 * a.num_rows * L)
    d.spmm_dev(dX, dY, L)
    Y = dY.download((a.num_rows, L))
    ref = orc.csr_spmm_t(a, X)
    bound = np.zeros_like(ref)   # reordering bound: 2 (len + 1) eps (|A| |X|)
    np.add.at(bound, np.repeat(np.arange(a.num_rows), np.diff(a.row_offsets)),
              np.abs(a.values)[:, None] * np.abs(X[a.column_indices]))
    assert np.all(np.abs(Y - ref) <= 2 * 54 * 2.0 ** -53 * bound + 1e-300), L
    xp = d.x_ext(L)                       # the copy-free form the bench uses
    mspmv.memcpy_h2d_ptr(xp, X)
    d.spmm_dev(xp, dY, L)
    assert np.array_equal(dY.download((a.num_rows, L)), Y), L
assert d.time_local(dY, 1, 5) > 0
d.close()
print("SPLIT OK")
"""


def test_dist_three_stream_split_one_gpu(tmp_path):
    """MSPMV_DIST_FORCE_SPLIT=1: the local rows split at their thirds (head | interior | tail), the
    interior on its own stream beside the (here empty) exchange, the ends after it, every part
    joined into the local stream -- the overlapped SpMM of N > 1 ranks, run on one GPU (RCCL
    refuses two ranks on one device), for L = 1, 3 (chunked) and 8, and through x_ext."""
    import subprocess
    env = dict(os.environ, MSPMV_DIST_FORCE_SPLIT="1")
    r = subprocess.run([sys.executable, "-c", _SPLIT_CHILD, os.path.join(ROOT, "sparse-matrix-linear-equations_amd"),
                        os.path.join(ROOT, "tests")], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "SPLIT OK" in r.stdout, r.stdout + r.stderr[-3000:]


_SPLIT_CG_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import mspmv
a = mspmv.CsrMatrix.synth_stencil(1, 16 * 17 * 18, 16, 17, 18)
rb = mspmv.dist_partition(a, 1)
d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))
for L in (1, 3, 8):
    B = np.random.default_rng(L).uniform(0, 1, (a.num_rows, L))
    dB = mspmv.DeviceBuffer.from_array(B)
    dX = mspmv.DeviceBuffer(8 * a.num_rows * L)
    it, hist, st = d.cg_dev(dB, dX, L, 3000, 1e-9, hist_cap=3000)
    np.save(sys.argv[3] + f"/X_{L}.npy", dX.download((a.num_rows, L)))
    np.save(sys.argv[3] + f"/h_{L}.npy", hist)
    np.save(sys.argv[3] + f"/m_{L}.npy", np.array([it, st]))
d.close()
print("SPLIT CG OK")
"""


@pytest.mark.parametrize("plan", ["tiles", "windows"])
def test_dist_cg_three_stream_split_one_gpu(tmp_path, orc, plan):
    """The sharded CG's overlapped iteration (MSPMV_DIST_FORCE_SPLIT=1: head | interior | tail, the
    interior's dot-mode SpMM on its own stream beside the exchange, each part's p.Ap partials at its
    offset, one fold over the three in tile order) at L = 1, 3, 8: iterations, history within 1e-10
    and X as the oracle's CGSolveMultiple.  `windows`: every part (a stencil's rows, no halo at world 1)
    on the offset windows' dot mode (csrc/mspmv_dia.hip), one partial per window."""
    import subprocess
    import mspmv
    env = dict(os.environ, MSPMV_DIST_FORCE_SPLIT="1", MSPMV_DIA="0" if plan == "tiles" else "")
    r = subprocess.run([sys.executable, "-c", _SPLIT_CG_CHILD, os.path.join(ROOT, "sparse-matrix-linear-equations_amd"),
                        os.path.join(ROOT, "tests"), str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "SPLIT CG OK" in r.stdout, r.stdout + r.stderr[-3000:]
    a = _matrix()
    for L in (1, 3, 8):
        B = np.random.default_rng(L).uniform(0, 1, (a.num_rows, L))
        Xo, it_o, ho = orc.cg_multi(a, B, 3000, 1e-9, kernel=1, P=8, hist_cap=3000)
        it, st = np.load(tmp_path / f"m_{L}.npy")
        assert st == 0 and abs(int(it) - it_o) <= 1, (L, it, it_o)
        h = np.load(tmp_path / f"h_{L}.npy")
        k = min(len(h), len(ho))
        np.testing.assert_allclose(h[:k], ho[:k], rtol=0, atol=1e-10)
        Xg = np.load(tmp_path / f"X_{L}.npy")
        assert np.linalg.norm(Xg - Xo) <= 1e-8 * np.linalg.norm(Xo), L


@pytest.mark.parametrize("plan", ["tiles", "windows"])
def test_dist_cg_any_width(orc, monkeypatch, plan):
    """mspmv_dist_cg_dev at L = 3 and 12: column groups of native widths, every rank (here one) the
    same groups; iterations, history and X as the oracle's single L-wide CGSolveMultiple.  `windows`:
    the unsplit local rows on the offset windows' dot mode."""
    import mspmv
    if plan == "windows":
        monkeypatch.delenv("MSPMV_DIA", raising=False)
    a = _matrix()
    rb = mspmv.dist_partition(a, 1)
    d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))
    for L in (3, 12):
        B = np.random.default_rng(L).uniform(0, 1, (a.num_rows, L))
        dB = mspmv.DeviceBuffer.from_array(B)
        dX = mspmv.DeviceBuffer(8 * a.num_rows * L)
        it, hist, st = d.cg_dev(dB, dX, L, 3000, 1e-9, hist_cap=3000)
        Xg = dX.download((a.num_rows, L))
        Xo, it_o, ho = orc.cg_multi(a, B, 3000, 1e-9, kernel=1, P=8, hist_cap=3000)
        assert st == 0 and abs(it - it_o) <= 1
        k = min(len(hist), len(ho))
        np.testing.assert_allclose(hist[:k], ho[:k], rtol=0, atol=1e-10)
        assert np.linalg.norm(Xg - Xo) <= 1e-8 * np.linalg.norm(Xo)
    d.close()


def test_bench_sharded_headline_world1(tmp_path):
    """bench.py's N > 1 headline (run_sharded_headline: per-rank row blocks generated alone,
    x_ext, overlapped SpMM, local timing) run at world 1 (MSPMV_BENCH_SHARDED=1): one JSON line with
    the contract's fields and a plausible roofline."""
    import json
    import subprocess
    env = dict(os.environ, MSPMV_BENCH_SHARDED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", "--no-cg",
                        "--no-cpu"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["scaling"] == "weak" and line["value"] > 100
    assert 0.2 < line["roofline"]["frac"] < 1.0


_GRAPH_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import mspmv
a = mspmv.CsrMatrix.synth_stencil(1, 16 * 17 * 18, 16, 17, 18)
rb = mspmv.dist_partition(a, 1)
d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, mspmv.local_rows(a, rb, 0))
out = []
for L in (1, 8):
    B = np.random.default_rng(L).uniform(0, 1, (a.num_rows, L))
    dB = mspmv.DeviceBuffer.from_array(B)
    for rep in range(2):  # the second solve replays the graph from its first batch
        dX = mspmv.DeviceBuffer(8 * a.num_rows * L)
        it, hist, st = d.cg_dev(dB, dX, L, 3000, 1e-9, hist_cap=3000)
        np.save(sys.argv[3] + f"/X_{L}_{rep}.npy", dX.download((a.num_rows, L)))
        np.save(sys.argv[3] + f"/h_{L}_{rep}.npy", hist)
        np.save(sys.argv[3] + f"/m_{L}_{rep}.npy", np.array([it, st]))
d.close()
print("GRAPH CG OK")
"""


@pytest.mark.parametrize("split", ["0", "1"])
def test_dist_cg_graph_matches_eager(tmp_path, split):
    """The sharded CG's batches replayed from a captured hipGraph (kernels, the interior's second
    stream, the RCCL exchange and all-reduces; MSPMV_DIST_GRAPH, default on) give bit for bit the
    eager enqueue's iterations, history and X, for the whole-local and the split (head | interior
    | tail) iteration, on the first solve (eager batches, then graph) and a repeated one (graph
    from the first batch)."""
    import subprocess
    res = {}
    for g in ("0", "1"):
        od = tmp_path / g
        od.mkdir()
        env = dict(os.environ, MSPMV_DIST_GRAPH=g, MSPMV_DIST_FORCE_SPLIT=split, MSPMV_CG_BATCH="8",
                   MSPMV_DEBUG_GRAPH="1")
        r = subprocess.run([sys.executable, "-c", _GRAPH_CHILD, os.path.join(ROOT, "sparse-matrix-linear-equations_amd"),
                            os.path.join(ROOT, "tests"), str(od)], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0 and "GRAPH CG OK" in r.stdout, r.stdout + r.stderr[-3000:]
        assert "capture failed" not in r.stderr, r.stderr[-2000:]
        assert ("batch of 8 iterations captured" in r.stderr) == (g == "1"), r.stderr[-2000:]
        res[g] = od
    for L in (1, 8):
        for rep in range(2):
            for f in ("X", "h", "m"):
                e = np.load(res["0"] / f"{f}_{L}_{rep}.npy")
                gr = np.load(res["1"] / f"{f}_{L}_{rep}.npy")
                assert np.array_equal(e.view(np.uint8), gr.view(np.uint8)), (f, L, rep)
        it, st = np.load(res["1"] / f"m_{L}_0.npy")
        assert st == 0 and it > 24, (L, it)  # 8-iteration batches: the graph replayed several times


def test_dist_shared_comm(orc):
    """Several sharded matrices on ONE communicator (mspmv.Comm, the bench's N > 1 form): every
    object's kernels and collectives run on the communicator's one stream, interleaved calls on two
    matrices give each its own oracle result, the CG on each matches the oracle, and the
    communicator refuses to close while a matrix still uses it."""
    import mspmv
    a1 = _matrix()
    a2 = mspmv.CsrMatrix.synth_fem_blocked(36000, 36000 * 53, 6, 340, seed=3)
    comm = mspmv.Comm(mspmv.comm_unique_id(), 1, 0, 0)
    ds, Xs, dYs = [], [], []
    for a in (a1, a2):
        rb = mspmv.dist_partition(a, 1)
        ds.append(mspmv.DistCsr(comm, rb, mspmv.local_rows(a, rb, 0)))
        Xs.append(np.random.default_rng(a.num_rows).uniform(-1, 1, (a.num_rows, 4)))
        dYs.append(mspmv.DeviceBuffer(8 * a.num_rows * 4))
    with pytest.raises(mspmv.MspmvError):
        comm.close()
    dXs = [mspmv.DeviceBuffer.from_array(X) for X in Xs]
    for _ in range(3):  # interleaved, no sync in between (the stream orders them)
        for d, dX, dY in zip(ds, dXs, dYs):
            d.spmm_dev(dX, dY, 4, sync=False)
    ds[0].sync()
    for a, X, dY in zip((a1, a2), Xs, dYs):
        np.testing.assert_allclose(dY.download((a.num_rows, 4)), orc.csr_spmm_t(a, X), rtol=1e-13, atol=1e-13)
    B = np.random.default_rng(9).uniform(0, 1, (a1.num_rows, 8))
    dB, dX = mspmv.DeviceBuffer.from_array(B), mspmv.DeviceBuffer(8 * a1.num_rows * 8)
    it, hist, st = ds[0].cg_dev(dB, dX, 8, 3000, 1e-9, hist_cap=3000)
    Xo, it_o, ho = orc.cg_multi(a1, B, 3000, 1e-9, kernel=1, P=8, hist_cap=3000)
    assert st == 0 and abs(it - it_o) <= 1
    k = min(len(hist), len(ho))
    np.testing.assert_allclose(hist[:k], ho[:k], rtol=0, atol=1e-10)
    for d in ds:
        d.close()
    comm.close()


_L2_CHILD = r"""
import sys
sys.path[:0] = [sys.argv[1]]
import mspmv
a = mspmv.CsrMatrix.synth_fem_blocked(21792, 1152443, 6, 170, seed=3)
with mspmv.GpuCsr(a) as g:
    print("NAMES", g.kernel_name(), g.spmm_kernel_name(2), g.spmm_kernel_name(16))
"""


@pytest.mark.parametrize("knob", ["1", "0"])
def test_spmm_blk_knob_names_kernel(knob):
    """MSPMV_SPMM_BLK=0 takes every L > 1 off the node-block SpMM -- L = 2 too, whose merge tiles
    have the single-RHS tile size and so share that plan -- and mspmv_spmm_kernel_name reports the
    kernel each width launches (the single-RHS SpMV keeps its node-block kernel either way)."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", _L2_CHILD, os.path.join(ROOT, "sparse-matrix-linear-equations_amd")],
                       env=dict(os.environ, MSPMV_SPMM_BLK=knob), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    spmv, l2, l16 = r.stdout.split("NAMES", 1)[1].split()
    assert spmv.startswith("k_spmv_blk")
    want = "k_spmm_blk<" if knob == "1" else "k_spmm_tile<"
    assert l2.startswith(want + "2,") and l16.startswith(want + "16,"), (l2, l16)
