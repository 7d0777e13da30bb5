"""tools/parallel_efficiency.py: the reference's parallel_efficiency CSVs
(verification/efficiency/parallel_efficiency.cpp:177-288) over GPU compute units / GPUs."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import parallel_efficiency as pe  # noqa: E402


def test_efficiency_math_and_csv(tmp_path):
    # two matrices, three unit counts: means per count, speedup from the first count's mean
    rows = [["a", 8, 40.0, 1.0, 10], ["b", 8, 80.0, 2.0, 12], ["a", 16, 20.0, 2.0, 10], ["b", 16, 40.0, 4.0, 12],
            ["a", 32, 12.5, 3.2, 10], ["b", 32, 25.0, 6.4, 12]]
    eff = pe.efficiency(rows, [8, 16, 32])
    np.testing.assert_allclose([e[1] for e in eff], [60.0, 30.0, 18.75])
    np.testing.assert_allclose([e[3] for e in eff], [1.0, 2.0, 3.2])
    np.testing.assert_allclose([e[4] for e in eff], [1.0, 1.0, 0.8])
    args = type("A", (), {"output_dir": str(tmp_path)})()
    pe.save(args, rows, eff, "")
    lines = (tmp_path / "parallel_efficiency.csv").read_text().splitlines()
    assert lines[0] == "num_threads,avg_time_ms,avg_gflops,speedup,efficiency"   # :245
    assert lines[1] == "8,60.000,1.50,1.000,1.0000"                              # :249-252 precisions
    det = (tmp_path / "parallel_efficiency_detailed.csv").read_text().splitlines()
    assert det[0] == "matrix_name,num_threads,time_ms,gflops,iterations"           # :273
    assert det[1] == "a,8,40.000,1.00,10"


def test_missing_dir_fails_like_the_reference(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "parallel_efficiency.py"),
                        f"--mtx_dir={tmp_path}"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "No .mtx files found" in (r.stdout + r.stderr)


@pytest.mark.gpu
def test_cu_sweep_on_gpu(tmp_path, gpu_available):
    if not gpu_available:
        pytest.skip("no GPU")
    out = tmp_path / "par"
    pe.main(["--synthetic", "--cus", "16,64,256", "--timing_iters", "1", "--num_vectors", "2",
             f"--output_dir={out}"])
    lines = (out / "parallel_efficiency.csv").read_text().splitlines()
    vals = [list(map(float, ln.split(","))) for ln in lines[1:]]
    assert [int(v[0]) for v in vals] == [16, 64, 256]
    assert vals[0][3] == 1.0 and vals[2][3] > 1.0       # more CUs, faster
    det = (out / "parallel_efficiency_detailed.csv").read_text().splitlines()
    its = {}
    for ln in det[1:]:
        name, u, t, g, it = ln.split(",")
        its.setdefault(name, set()).add(int(it))
    assert all(len(v) == 1 for v in its.values())      # the CU mask changes speed, never the solve


@pytest.mark.gpu
def test_gpu_count_sweep_single_rank(tmp_path, gpu_available):
    if not gpu_available:
        pytest.skip("no GPU")
    out = tmp_path / "par"
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "parallel_efficiency.py"), "--units=gpus",
                        "--synthetic", "--timing_iters=1", "--num_vectors=2", f"--output_dir={out}"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = (out / "parallel_efficiency_gpus.csv").read_text().splitlines()
    assert lines[1].startswith("1,") and lines[1].endswith(",1.000,1.0000")
