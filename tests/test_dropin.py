"""The drop-in boundary against the reference's REAL CsrMatrix (the facade had only
been compiled against a stand-in struct).

Container side (needs /root/reference; skipped elsewhere): oracle/dropin_check.cpp -- the
reference's sparse_matrix.h / utils.h / hyper_parameters.hpp by path, include/mspmv_dropin.hpp,
then the reference's work_2025/main/*.hpp exactly as cpu_multicg.cpp:43-48 includes them -- must
compile and link against libmspmv.so, and every reference entry point it calls must resolve to
the facade (a CPU-only run fails loudly with "no HIP device": no fallback).  Including a replaced
header before the drop-in must be a compile error, never a silent CPU path.
GPU side (tests/test_gpu_tools.py::test_dropin_check_on_gpu): the same binary, shipped in
oracle/_ref, runs every call on the MI355X and checks it against the reference's own SpmvGold /
OmpCsrSpmmT."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
INC = os.path.join(ROOT, "include")
BIN = os.path.join(ROOT, "oracle", "_ref", "dropin_check")

needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout absent (GPU box)")


@needs_ref
def test_dropin_builds_against_reference_headers(mspmv):
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "dropin", "REF=" + REF],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert os.path.exists(BIN)
    nm = subprocess.run(["nm", "-C", BIN], capture_output=True, text=True).stdout
    # the reference names resolve to the facade, which calls the C-ABI (undefined, from libmspmv)
    for sym in ("mspmv_dcg_multi_dev", "mspmv_dpcg_ic0_multi_dev", "mspmv_dpcg_spai_multi_dev",
                "mspmv_dcg_single_dev", "mspmv_dspmm", "mspmv_time_spmm_dev", "mspmv_csr_transpose"):
        assert f"U {sym}" in nm, sym
    # and no CPU CG of the reference was compiled in (its headers were guarded away)
    assert "dot_multiple" not in nm and "ForwardSolveMultiple" not in nm


@needs_ref
def test_dropin_without_gpu_fails_loudly(mspmv):
    if mspmv.device_count() > 0:
        pytest.skip("a device is visible: tests/test_gpu_tools.py runs it")
    if not os.path.exists(BIN):
        pytest.skip("dropin_check not built")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3 and "no HIP device" in r.stdout, r.stdout + r.stderr


@needs_ref
def test_replaced_header_first_is_a_compile_error(tmp_path):
    src = tmp_path / "bad.cpp"
    src.write_text('#include "sparse_matrix.h"\n#include "utils.h"\n#include "work_2025/hyper_parameters.hpp"\n'
                   '#include "work_2025/spmm/merge_based.hpp"\n#include "mspmv_dropin.hpp"\nint main() {}\n')
    r = subprocess.run(["g++", "-std=c++17", "-fopenmp", "-fsyntax-only", f"-I{REF}", f"-I{INC}", str(src)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "include it before them" in r.stderr, r.stderr[-1500:]


@needs_ref
def test_namespace_mode_beside_reference_headers(tmp_path):
    """Namespace mode declares nothing global: it compiles next to the reference's own
    merge_based.hpp (cpu_spmv.cpp-style callers qualify mspmv_ref::)."""
    src = tmp_path / "ns.cpp"
    src.write_text('#include "sparse_matrix.h"\n#include "work_2025/spmm/merge_based.hpp"\n#include "mspmv.hpp"\n'
                   'int main() { CsrMatrix<double,int> a; double x[1], y[1];\n'
                   '  if (a.num_rows) mspmv_ref::OmpMergeCsrmv(1, a, a.row_offsets + 1, a.column_indices, a.values, x, y);\n'
                   '  return 0; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fopenmp", "-fsyntax-only", f"-I{REF}", f"-I{INC}", str(src)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-1500:]
