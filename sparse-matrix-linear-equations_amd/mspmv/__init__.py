"""mspmv -- Python host mirror of the reference's hot-path interface, over libmspmv.so.

The product is the C-ABI library next to this file (HIP kernels for gfx950 + C++ host code,
include/mspmv.h).  This module is a thin ctypes layer so tests and bench.py can drive it:

* ``CsrMatrix`` mirrors ``CsrMatrix<double,int>`` (sparse_matrix.h:633-653);
* ``GpuCsr`` owns one uploaded matrix (``mspmv_csr_create``) and exposes SpMV/SpMM/CG;
* ``OmpMergeCsrmv`` / ``OmpMergeCsrmm`` / ``CGSolveSingle`` / ``CGSolveMultiple`` keep the
  reference's names, argument order and meaning (cpu_spmv.cpp:357-367,
  work_2025/spmm/merge_based.hpp:46-57, work_2025/main/single_strategy.hpp:102-110,
  work_2025/main/no_pretreatment.hpp:32-43); ``num_threads`` is accepted and ignored.

There is no CPU fallback: importing this module fails loudly if libmspmv.so is missing,
and every compute call goes through the HIP library.
"""
from __future__ import annotations

import atexit
import ctypes
import itertools
import os
import weakref
from dataclasses import dataclass
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MSPMV_LIB") or os.path.join(_HERE, "libmspmv.so")  # MSPMV_LIB: A/B builds

SIMPLE, MERGE, NONZERO_SPLIT = 0, 1, 2  # SpmmKernel, work_2025/types.hpp:11-16

STATUS = {
    0: "OK", 1: "INVALID", 2: "HIP", 3: "OOM", 4: "BREAKDOWN", 5: "RCCL", 6: "UNSUPPORTED", 7: "IO",
    8: "STALL", 9: "FAULT",
}
FAULT = 9  # a fold ticket drew past its group (mspmv_check_faults): results invalid, always raised
# unless a caller asks for it (the poisoned-ticket tests)
POISON_FILL, POISON_LATE_ZERO, POISON_NO_STOP = 1, 2, 4  # mspmv_test_poison_tickets flags
# CG calls return their status beside X: BREAKDOWN (4) is a per-column numerical event (the
# frozen columns are reported, the others solved), so it is returned, not raised; everything
# else -- STALL (8, an IC(0) triangular solve that never progressed) included -- raises.
SUPPORTED_L = (1, 2, 4, 8, 16)  # native tile-kernel widths; SpMM and the CGs take any L >= 1
# (column chunks / groups of these widths; the sharded CG and the timing helpers native only)


class MspmvError(RuntimeError):
    def __init__(self, status: int, where: str, msg: str):
        super().__init__(f"{where}: {STATUS.get(status, status)}: {msg}")
        self.status = status


class Coord(ctypes.Structure):
    _fields_ = [("x", ctypes.c_int), ("y", ctypes.c_int)]


class _CsrD(ctypes.Structure):
    _fields_ = [
        ("num_rows", ctypes.c_int),
        ("num_cols", ctypes.c_int),
        ("num_nonzeros", ctypes.c_int),
        ("row_offsets", ctypes.c_void_p),
        ("column_indices", ctypes.c_void_p),
        ("values", ctypes.c_void_p),
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double
_PI = ctypes.POINTER(ctypes.c_int)
_PD = ctypes.POINTER(ctypes.c_double)
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); the single source of truth for the ctypes declarations
_SIGS = {
    "mspmv_last_error": (ctypes.c_char_p, []),
    "mspmv_version": (ctypes.c_char_p, []),
    "mspmv_device_count": (_I, []),
    "mspmv_csr_create": (_I, [ctypes.POINTER(_CsrD), _I, ctypes.POINTER(_P)]),
    "mspmv_csr_create_dev": (_I, [ctypes.POINTER(_CsrD), _I, ctypes.POINTER(_P)]),
    "mspmv_destroy": (_I, [_P]),
    "mspmv_shape": (_I, [_P, _PI, _PI, _PI]),
    "mspmv_setup_ms": (_D, [_P]),
    "mspmv_sync": (_I, [_P]),
    "mspmv_check_faults": (_I, [_P]),
    "mspmv_spmv_tile_stamps": (_I, [_P, _P, _P, ctypes.c_size_t, _P, _PI]),
    "mspmv_test_poison_tickets": (_I, [_P, ctypes.c_uint, _I]),
    "mspmv_dist_test_poison_tickets": (_I, [_P, ctypes.c_uint, _I]),
    "mspmv_set_cu_limit": (_I, [_P, _I]),
    "mspmv_merge_coords": (_I, [_P, _I, ctypes.POINTER(Coord)]),
    "mspmv_dspmv": (_I, [_P, _P, _P]),
    "mspmv_dspmv_dev": (_I, [_P, _P, _P]),
    "mspmv_dspmm": (_I, [_P, _P, _P, _I]),
    "mspmv_dspmm_dev": (_I, [_P, _P, _P, _I]),
    "mspmv_dcg_single": (_I, [_P, _P, _P, _I, _D, _PI, _P, _I]),
    "mspmv_dcg_single_dev": (_I, [_P, _P, _P, _I, _D, _PI, _P, _I]),
    "mspmv_cg_resident_stamps": (_I, [_P, _P, _P, _I, _D, _PI, _P, _I, _PI]),
    "mspmv_dcg_multi": (_I, [_P, _P, _P, _I, _I, _D, _I, _PI, _P, _I]),
    "mspmv_dcg_multi_dev": (_I, [_P, _P, _P, _I, _I, _D, _I, _PI, _P, _I]),
    "mspmv_spai_values": (_I, [ctypes.POINTER(_CsrD), _P]),
    "mspmv_ic0_nnz": (_I, [ctypes.POINTER(_CsrD), _PI]),
    "mspmv_ic0_factor": (_I, [ctypes.POINTER(_CsrD), _P, _P, _P, _PD]),
    "mspmv_ic0_create": (_I, [ctypes.POINTER(_CsrD), _I, ctypes.POINTER(_P)]),
    "mspmv_csr_transpose": (_I, [ctypes.POINTER(_CsrD), _P, _P, _P]),
    "mspmv_ic0_destroy": (_I, [_P]),
    "mspmv_dpcg_ic0_multi": (_I, [_P, _P, _P, _P, _I, _I, _D, _I, _PI, _P, _I]),
    "mspmv_dpcg_ic0_multi_dev": (_I, [_P, _P, _P, _P, _I, _I, _D, _I, _PI, _P, _I]),
    "mspmv_dpcg_spai_multi": (_I, [_P, _P, _P, _P, _I, _I, _D, _I, _PI, _P, _I]),
    "mspmv_dpcg_spai_multi_dev": (_I, [_P, _P, _P, _P, _I, _I, _D, _I, _PI, _P, _I]),
    "mspmv_time_spmm_dev": (_I, [_P, _P, _P, _I, _I, _SZ, _PD]),
    "mspmv_time_stream_read": (_I, [_I, _SZ, _I, _PD]),
    "mspmv_last_kernel_ms": (_I, [_P, _PD, _PI]),
    "mspmv_time_spmm_batch_dev": (_I, [_I, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _I,
                                       _PD, _PD, _PI]),
    "mspmv_tile_plan": (_I, [_P, _I, _PI, _PI, _PI, ctypes.POINTER(Coord)]),
    "mspmv_tile_streams": (_I, [_P, _PI, _PI]),
    "mspmv_plan_dict_tiles": (_I, [_P, _I, _PI]),
    "mspmv_plan_block_tiles": (_I, [_P, _I, _PI]),
    "mspmv_tile_modes": (_I, [_P, _I, _P]),
    "mspmv_tile_lanes": (_I, [_P, _I, _PI]),
    "mspmv_offset_windows": (_I, [ctypes.POINTER(_CsrD), _D, _D, _PI, _PI, ctypes.POINTER(ctypes.c_longlong), _PI, _P,
                                  ctypes.POINTER(ctypes.c_longlong)]),
    "mspmv_spmv_kernel_name": (ctypes.c_char_p, [_P]),
    "mspmv_spmm_kernel_name": (ctypes.c_char_p, [_P, _I]),
    "mspmv_cg_kernel_name": (ctypes.c_char_p, [_P]),
    "mspmv_device_malloc": (_I, [_I, _SZ, ctypes.POINTER(_P)]),
    "mspmv_device_free": (_I, [_P]),
    "mspmv_memcpy_h2d": (_I, [_P, _P, _SZ]),
    "mspmv_memcpy_d2h": (_I, [_P, _P, _SZ]),
    "mspmv_memcpy_d2d": (_I, [_P, _P, _SZ]),
    "mspmv_memset_dev": (_I, [_P, _I, _SZ]),
    "mspmv_synth_banded": (_I, [_I, ctypes.c_longlong, _I, ctypes.c_ulonglong, _P, _P, _P]),
    "mspmv_market_read": (_I, [ctypes.c_char_p, _D, _PI, _PI, _PI, ctypes.POINTER(_P), ctypes.POINTER(_P),
                               ctypes.POINTER(_P)]),
    "mspmv_generate": (_I, [_I, _I, _I, _D, _PI, _PI, _PI, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "mspmv_host_free": (None, [_P]),
    "mspmv_dist_partition": (_I, [_P, _I, _I, _I, _P]),
    "mspmv_dist_localize": (_I, [_P, _I, _I, _P, _P, _P, _PI, _P, _I, _P]),
    "mspmv_comm_unique_id": (_I, [_P]),
    "mspmv_dist_create": (_I, [_P, _I, _I, _I, _P, ctypes.POINTER(_CsrD), ctypes.POINTER(_P)]),
    "mspmv_comm_create": (_I, [_P, _I, _I, _I, ctypes.POINTER(_P)]),
    "mspmv_comm_destroy": (_I, [_P]),
    "mspmv_dist_create_on": (_I, [_P, _P, ctypes.POINTER(_CsrD), ctypes.POINTER(_P)]),
    "mspmv_dist_destroy": (_I, [_P]),
    "mspmv_dist_info": (_I, [_P, _PI, _PI, _PI]),
    "mspmv_dist_spmm_dev": (_I, [_P, _P, _P, _I]),
    "mspmv_dist_x_ext": (_I, [_P, _I, ctypes.POINTER(_P)]),
    "mspmv_dist_sync": (_I, [_P]),
    "mspmv_dist_time_local_dev": (_I, [_P, _P, _I, _I, _PD]),
    "mspmv_dist_cg_dev": (_I, [_P, _P, _P, _I, _I, _D, _PI, _P, _I]),
    "mspmv_synth_fem_blocked": (_I, [_I, ctypes.c_longlong, _I, _I, ctypes.c_ulonglong, _P, _P, _P]),
    "mspmv_synth_fem_blocked_rows": (_I, [_I, ctypes.c_longlong, _I, _I, ctypes.c_ulonglong, _I, _I, _P, _P, _P]),
    "mspmv_synth_fem_perturbed": (_I, [_I, ctypes.c_longlong, _I, _I, _D, _D, ctypes.c_ulonglong, _P, _P, _P,
                                       ctypes.POINTER(ctypes.c_longlong)]),
    "mspmv_synth_powerlaw": (_I, [_I, _I, ctypes.c_longlong, _D, ctypes.c_ulonglong, _P, _P, _P]),
    "mspmv_synth_stencil": (_I, [_I, _I, _I, _I, _I, ctypes.c_ulonglong, _D, _P, _P, _P,
                                 ctypes.POINTER(ctypes.c_longlong)]),
    "mspmv_synth_stencil_perturbed": (_I, [_I, _I, _I, ctypes.c_ulonglong, _D, _D, _D, _P, _P, _P,
                                           ctypes.POINTER(ctypes.c_longlong)]),
    "mspmv_synth_kkt": (_I, [_I, _I, _I, ctypes.c_ulonglong, _D, _D, _P, _P, _P, ctypes.POINTER(ctypes.c_longlong)]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C sparse-matrix-linear-equations_amd/csrc`")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        if not hasattr(lib, name) and "MSPMV_LIB" in os.environ:
            continue  # an older build under A/B (tools/lab): entry points it lacks stay unbound
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()

# Live device objects, released in reverse creation order at interpreter exit (atexit runs before
# the C runtime's exit handlers, so the HIP runtime -- and a profiler's hooks into it -- are still
# up when the handles and buffers go).  A plain __del__ at shutdown may run after them or never.
_LIVE = weakref.WeakValueDictionary()
_SEQ = itertools.count()


def _track(obj):
    _LIVE[next(_SEQ)] = obj


@atexit.register
def _release_all():
    for k in sorted(list(_LIVE.keys()), reverse=True):
        obj = _LIVE.get(k)
        if obj is None:
            continue
        try:
            (obj.free if isinstance(obj, DeviceBuffer) else obj.close)()
        except Exception:
            pass


def _check(status: int, where: str, allow=()):
    if status != 0 and status not in allow:
        raise MspmvError(status, where, lib.mspmv_last_error().decode(errors="replace"))
    return status


def device_count() -> int:
    return int(lib.mspmv_device_count())


def time_stream_read(device: int = 0, nbytes: int = 1 << 30, reps: int = 20) -> float:
    """GB/s of a STREAM-like nontemporal HBM read (the practical roofline ceiling)."""
    g = ctypes.c_double(0.0)
    _check(lib.mspmv_time_stream_read(device, nbytes, reps, ctypes.byref(g)), "time_stream_read")
    return g.value


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ----------------------------------------------------------------------------------------
# CsrMatrix mirror
# ----------------------------------------------------------------------------------------
@dataclass
class CsrMatrix:
    """Host CSR with the fields of CsrMatrix<double,int> (sparse_matrix.h:648-653)."""

    num_rows: int
    num_cols: int
    num_nonzeros: int
    row_offsets: np.ndarray      # int32[num_rows+1]
    column_indices: np.ndarray   # int32[num_nonzeros]
    values: np.ndarray           # float64[num_nonzeros]

    @classmethod
    def from_arrays(cls, num_cols: int, row_offsets, column_indices, values) -> "CsrMatrix":
        ro = np.ascontiguousarray(row_offsets, dtype=np.int32)
        ci = np.ascontiguousarray(column_indices, dtype=np.int32)
        va = np.ascontiguousarray(values, dtype=np.float64)
        return cls(len(ro) - 1, int(num_cols), int(ro[-1]) if len(ro) else 0, ro, ci, va)

    def _c(self) -> _CsrD:
        return _CsrD(self.num_rows, self.num_cols, self.num_nonzeros, _ptr(self.row_offsets),
                     _ptr(self.column_indices), _ptr(self.values))

    # --- the reference's constructors (sparse_matrix.h), natively in libmspmv.so --------
    @classmethod
    def _from_c(cls, m, n, nnz, ro, ci, va) -> "CsrMatrix":
        try:
            r = np.ctypeslib.as_array(ctypes.cast(ro, ctypes.POINTER(ctypes.c_int)), (m.value + 1,)).copy()
            k = nnz.value
            c = np.ctypeslib.as_array(ctypes.cast(ci, ctypes.POINTER(ctypes.c_int)), (max(k, 1),))[:k].copy()
            v = np.ctypeslib.as_array(ctypes.cast(va, ctypes.POINTER(ctypes.c_double)), (max(k, 1),))[:k].copy()
        finally:
            for p in (ro, ci, va):
                lib.mspmv_host_free(p)
        return cls(m.value, n.value, k, r, c, v)

    @classmethod
    def from_market(cls, path: str, default_value: float = 1.0) -> "CsrMatrix":
        """CooMatrix::InitMarket + CsrMatrix::Init (sparse_matrix.h:211-380, 668-733)."""
        m, n, nnz = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        ro, ci, va = _P(), _P(), _P()
        _check(lib.mspmv_market_read(path.encode(), default_value, ctypes.byref(m), ctypes.byref(n),
                                     ctypes.byref(nnz), ctypes.byref(ro), ctypes.byref(ci), ctypes.byref(va)),
               f"market_read({path})")
        return cls._from_c(m, n, nnz, ro, ci, va)

    @classmethod
    def generate(cls, kind: str, p0: int, p1: int = 0) -> "CsrMatrix":
        """The reference's grid2d / grid3d / wheel / dense generators (sparse_matrix.h:385-623)."""
        k = {"grid2d": 0, "grid3d": 1, "wheel": 2, "dense": 3}[kind]
        m, n, nnz = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        ro, ci, va = _P(), _P(), _P()
        _check(lib.mspmv_generate(k, p0, p1, 1.0, ctypes.byref(m), ctypes.byref(n), ctypes.byref(nnz),
                                  ctypes.byref(ro), ctypes.byref(ci), ctypes.byref(va)), f"generate({kind})")
        return cls._from_c(m, n, nnz, ro, ci, va)

    # --- synthetic shapes; generated natively in libmspmv.so -------------
    @classmethod
    def synth_banded(cls, m: int, nnz: int, half_band: int, seed: int = 1) -> "CsrMatrix":
        ro = np.empty(m + 1, np.int32)
        ci = np.empty(max(nnz, 1), np.int32)
        va = np.empty(max(nnz, 1), np.float64)
        _check(lib.mspmv_synth_banded(m, nnz, half_band, seed, _ptr(ro), _ptr(ci), _ptr(va)), "synth_banded")
        return cls(m, m, nnz, ro, ci[:nnz], va[:nnz])

    @classmethod
    def synth_fem_blocked(cls, m: int, nnz: int, block: int, half_band_nodes: int, seed: int = 1) -> "CsrMatrix":
        """FEM-like pattern: nodes of `block` unknowns, runs of `block` consecutive columns."""
        ro = np.empty(m + 1, np.int32)
        ci = np.empty(max(nnz, 1), np.int32)
        va = np.empty(max(nnz, 1), np.float64)
        _check(lib.mspmv_synth_fem_blocked(m, nnz, block, half_band_nodes, seed, _ptr(ro), _ptr(ci), _ptr(va)),
               "synth_fem_blocked")
        return cls(m, m, nnz, ro, ci[:nnz], va[:nnz])

    @classmethod
    def synth_fem_blocked_rows(cls, m: int, nnz: int, block: int, half_band_nodes: int, seed: int,
                               row_lo: int, row_hi: int) -> "CsrMatrix":
        """Rows [row_lo, row_hi) of synth_fem_blocked(m, nnz, ...) with GLOBAL column ids (num_cols
        = m): one rank's row block, generated without the rest of the matrix."""
        ro = np.empty(row_hi - row_lo + 1, np.int32)
        _check(lib.mspmv_synth_fem_blocked_rows(m, nnz, block, half_band_nodes, seed, row_lo, row_hi, _ptr(ro),
                                                None, None), "synth_fem_blocked_rows")
        k = int(ro[-1])
        ci = np.empty(max(k, 1), np.int32)
        va = np.empty(max(k, 1), np.float64)
        _check(lib.mspmv_synth_fem_blocked_rows(m, nnz, block, half_band_nodes, seed, row_lo, row_hi, _ptr(ro),
                                                _ptr(ci), _ptr(va)), "synth_fem_blocked_rows")
        return cls(row_hi - row_lo, m, k, ro, ci[:k], va[:k])

    @classmethod
    def synth_fem_perturbed(cls, m: int, nnz: int, block: int, half_band_nodes: int, odd_node_frac: float = 0.02,
                            extra_row_frac: float = 0.01, seed: int = 1) -> "CsrMatrix":
        """Imperfect FEM pattern: ~odd_node_frac of the nodes with block -+ 1 unknowns, ~extra_row_frac
        of the rows with one column outside their node's pattern (mspmv_synth_fem_perturbed)."""
        ro = np.empty(m + 1, np.int32)
        nz = ctypes.c_longlong(0)
        _check(lib.mspmv_synth_fem_perturbed(m, nnz, block, half_band_nodes, odd_node_frac, extra_row_frac, seed,
                                             _ptr(ro), None, None, ctypes.byref(nz)), "synth_fem_perturbed(size)")
        ci = np.empty(max(nz.value, 1), np.int32)
        va = np.empty(max(nz.value, 1), np.float64)
        _check(lib.mspmv_synth_fem_perturbed(m, nnz, block, half_band_nodes, odd_node_frac, extra_row_frac, seed,
                                             _ptr(ro), _ptr(ci), _ptr(va), ctypes.byref(nz)), "synth_fem_perturbed")
        return cls(m, m, int(nz.value), ro, ci[: nz.value], va[: nz.value])

    @classmethod
    def synth_powerlaw(cls, m: int, n: int, nnz: int, exponent: float = 1.2, seed: int = 3) -> "CsrMatrix":
        ro = np.empty(m + 1, np.int32)
        ci = np.empty(max(nnz, 1), np.int32)
        va = np.empty(max(nnz, 1), np.float64)
        _check(lib.mspmv_synth_powerlaw(m, n, nnz, exponent, seed, _ptr(ro), _ptr(ci), _ptr(va)), "synth_powerlaw")
        return cls(m, n, nnz, ro, ci[:nnz], va[:nnz])

    @classmethod
    def synth_stencil(cls, kind: int, m: int, dim0: int, dim1: int = 0, dim2: int = 0, seed: int = 7,
                      diag_shift: float = 1.0) -> "CsrMatrix":
        """kind 0: 2-D 7-point triangular FEM stencil (parabolic_fem shape), kind 1: 3-D
        27-point (nlpkkt120 size).  Symmetric, diagonal = sum|off| + diag_shift -> SPD."""
        ro = np.empty(m + 1, np.int32)
        nnz = ctypes.c_longlong(0)
        _check(lib.mspmv_synth_stencil(kind, m, dim0, dim1, dim2, seed, diag_shift, _ptr(ro), None, None,
                                       ctypes.byref(nnz)), "synth_stencil(size)")
        ci = np.empty(max(nnz.value, 1), np.int32)
        va = np.empty(max(nnz.value, 1), np.float64)
        _check(lib.mspmv_synth_stencil(kind, m, dim0, dim1, dim2, seed, diag_shift, _ptr(ro), _ptr(ci), _ptr(va),
                                       ctypes.byref(nnz)), "synth_stencil")
        return cls(m, m, int(nnz.value), ro, ci[: nnz.value], va[: nnz.value])

    @classmethod
    def synth_stencil_perturbed(cls, dims, seed: int = 7, diag_shift: float = 1.0, extra_frac: float = 0.01,
                                long_frac: float = 0.001) -> "CsrMatrix":
        """The 27-point stencil with off-pattern columns (mspmv_synth_stencil_perturbed)."""
        nx, ny, nz = dims
        m = nx * ny * nz
        ro = np.empty(m + 1, np.int32)
        nnz = ctypes.c_longlong(0)
        args = (nx, ny, nz, seed, diag_shift, extra_frac, long_frac)
        _check(lib.mspmv_synth_stencil_perturbed(*args, _ptr(ro), None, None, ctypes.byref(nnz)), "synth_perturbed")
        ci = np.empty(max(nnz.value, 1), np.int32)
        va = np.empty(max(nnz.value, 1), np.float64)
        _check(lib.mspmv_synth_stencil_perturbed(*args, _ptr(ro), _ptr(ci), _ptr(va), ctypes.byref(nnz)),
               "synth_perturbed")
        return cls(m, m, int(nnz.value), ro, ci[: nnz.value], va[: nnz.value])

    @classmethod
    def synth_kkt(cls, dims, seed: int = 7, diag_shift: float = 1.0, eps: float = 1e-2) -> "CsrMatrix":
        """KKT-shaped [[H, B^T], [B, -eps I]] with grid blocks (mspmv_synth_kkt)."""
        nx, ny, nz = dims
        m = 2 * nx * ny * nz
        ro = np.empty(m + 1, np.int32)
        nnz = ctypes.c_longlong(0)
        _check(lib.mspmv_synth_kkt(nx, ny, nz, seed, diag_shift, eps, _ptr(ro), None, None, ctypes.byref(nnz)),
               "synth_kkt")
        ci = np.empty(max(nnz.value, 1), np.int32)
        va = np.empty(max(nnz.value, 1), np.float64)
        _check(lib.mspmv_synth_kkt(nx, ny, nz, seed, diag_shift, eps, _ptr(ro), _ptr(ci), _ptr(va), ctypes.byref(nnz)),
               "synth_kkt")
        return cls(m, m, int(nnz.value), ro, ci[: nnz.value], va[: nnz.value])


# ----------------------------------------------------------------------------------------
# device memory
# ----------------------------------------------------------------------------------------
class DeviceBuffer:
    """A raw HBM allocation (mspmv_device_malloc)."""

    def __init__(self, nbytes: int, device: int = 0):
        p = ctypes.c_void_p()
        _check(lib.mspmv_device_malloc(device, nbytes, ctypes.byref(p)), "device_malloc")
        self.ptr = p.value
        self.nbytes = nbytes
        _track(self)

    @classmethod
    def from_array(cls, a: np.ndarray, device: int = 0) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, device)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        _check(lib.mspmv_memcpy_h2d(self.ptr, _ptr(a), a.nbytes), "memcpy_h2d")

    def download(self, shape, dtype=np.float64) -> np.ndarray:
        out = np.empty(shape, dtype)
        assert out.nbytes <= self.nbytes
        _check(lib.mspmv_memcpy_d2h(_ptr(out), self.ptr, out.nbytes), "memcpy_d2h")
        return out

    def fill_bytes(self, value: int = 0):
        _check(lib.mspmv_memset_dev(self.ptr, value, self.nbytes), "memset")

    def free(self):
        if self.ptr:
            lib.mspmv_device_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ----------------------------------------------------------------------------------------
# the uploaded matrix
# ----------------------------------------------------------------------------------------
class GpuCsr:
    """One CSR matrix resident in HBM with its merge-path tile plans (mspmv_csr_create)."""

    def __init__(self, a: CsrMatrix, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib.mspmv_csr_create(ctypes.byref(a._c()), device, ctypes.byref(h)), "csr_create")
        self.h = h.value
        self.num_rows, self.num_cols, self.num_nonzeros = a.num_rows, a.num_cols, a.num_nonzeros
        self.device = device
        _track(self)

    def close(self):
        if getattr(self, "h", None):
            lib.mspmv_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def setup_ms(self) -> float:
        return float(lib.mspmv_setup_ms(self.h))

    def sync(self):
        _check(lib.mspmv_sync(self.h), "sync")

    def spmv_tile_stamps(self, dX: "DeviceBuffer", dY: "DeviceBuffer", flush_bytes: int = 0) -> np.ndarray:
        """mspmv_spmv_tile_stamps: per-tile wall_clock64() phase stamps of one plain SpMV, [tiles][6]
        (flush_bytes > 0: after the cold protocol's read sweep)."""
        nt = ctypes.c_int()
        _check(lib.mspmv_spmv_tile_stamps(self.h, None, None, 0, None, ctypes.byref(nt)), "spmv_tile_stamps")
        st = np.zeros((max(nt.value, 1), 6), np.uint64)
        _check(lib.mspmv_spmv_tile_stamps(self.h, dX.ptr, dY.ptr, flush_bytes, _ptr(st), ctypes.byref(nt)),
               "spmv_tile_stamps")
        return st[: nt.value]

    def check_faults(self):
        """mspmv_check_faults: raises MspmvError(FAULT) if a product since the last check drew a ticket
        past its group."""
        _check(lib.mspmv_check_faults(self.h), "check_faults")

    def test_poison_tickets(self, value: int, flags: int = POISON_FILL):
        """Test hook: the next CG solve's fold tickets start at `value` (mspmv_test_poison_tickets)."""
        _check(lib.mspmv_test_poison_tickets(self.h, value, flags), "test_poison_tickets")

    def set_cu_limit(self, num_cus: int):
        """Run this handle's work on num_cus compute units (<= 0: all) -- mspmv_set_cu_limit."""
        _check(lib.mspmv_set_cu_limit(self.h, int(num_cus)), "set_cu_limit")

    def merge_coords(self, num_parts: int) -> np.ndarray:
        out = (Coord * (num_parts + 1))()
        _check(lib.mspmv_merge_coords(self.h, num_parts, out), "merge_coords")
        return np.ctypeslib.as_array(out).view(np.int32).reshape(num_parts + 1, 2).copy()

    def tile_plan(self, L: int = 1):
        nt, ti, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib.mspmv_tile_plan(self.h, L, ctypes.byref(nt), ctypes.byref(ti), ctypes.byref(nc), None), "tile_plan")
        b = (Coord * (nt.value + 1))()
        _check(lib.mspmv_tile_plan(self.h, L, None, None, None, b), "tile_plan")
        bounds = np.ctypeslib.as_array(b).view(np.int32).reshape(nt.value + 1, 2).copy()
        modes = np.zeros(max(nt.value, 1), np.uint8)
        _check(lib.mspmv_tile_modes(self.h, L, _ptr(modes)), "tile_modes")
        lanes = ctypes.c_int()
        _check(lib.mspmv_tile_lanes(self.h, L, ctypes.byref(lanes)), "tile_lanes")
        return {"num_tiles": nt.value, "tile_items": ti.value, "num_carries": nc.value, "bounds": bounds,
                "modes": modes[: nt.value], "lanes": lanes.value}

    def tile_streams(self):
        """(tiles on 16-bit column offsets, tiles gathering through column dictionaries)."""
        c16, dic = ctypes.c_int(), ctypes.c_int()
        _check(lib.mspmv_tile_streams(self.h, ctypes.byref(c16), ctypes.byref(dic)), "tile_streams")
        return c16.value, dic.value

    def dict_tiles(self, L: int = 1) -> int:
        """Tiles of the L-column plan that gather through a column dictionary."""
        n = ctypes.c_int()
        _check(lib.mspmv_plan_dict_tiles(self.h, L, ctypes.byref(n)), "plan_dict_tiles")
        return n.value
    def kernel_name(self) -> str:
        """The single-RHS SpMV kernel instantiation used for this matrix (rocprofv3's name)."""
        return lib.mspmv_spmv_kernel_name(self.h).decode()

    def cg_kernel_name(self) -> str:
        """The CG path the last solve on this matrix ran (mspmv_cg_kernel_name)."""
        return lib.mspmv_cg_kernel_name(self.h).decode()

    def cg_resident_stamps(self, db: "DeviceBuffer", dx: "DeviceBuffer", max_iters: int, tolerance: float,
                           stamp_iters: int):
        """One register-resident single-RHS solve with wall_clock64() phase stamps
        (mspmv_cg_resident_stamps): (iterations, stamps[stamp_iters][G][5] as uint64)."""
        it, G = ctypes.c_int(), ctypes.c_int()
        # one workgroup per CU: the buffer is sized for up to 1024 CUs (MI355X: 256)
        st = np.zeros(stamp_iters * 1024 * 5, np.uint64)
        _check(lib.mspmv_cg_resident_stamps(self.h, db.ptr, dx.ptr, max_iters, tolerance, ctypes.byref(it),
                                            _ptr(st), stamp_iters, ctypes.byref(G)), "cg_resident_stamps")
        return it.value, st[: stamp_iters * G.value * 5].reshape(stamp_iters, G.value, 5)

    def spmm_kernel_name(self, L: int) -> str:
        """The SpMM kernel instantiation launched for L right-hand sides (rocprofv3's spelling)."""
        return lib.mspmv_spmm_kernel_name(self.h, L).decode()

    def plan_block_tiles(self, L: int = 1) -> int:
        """Tiles of the L-column plan staged by node blocks (mspmv_plan_block_tiles)."""
        n = ctypes.c_int()
        _check(lib.mspmv_plan_block_tiles(self.h, L, ctypes.byref(n)), "plan_block_tiles")
        return n.value

    def spmv(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float64)
        assert x.shape == (self.num_cols,)
        y = np.empty(self.num_rows, np.float64)
        _check(lib.mspmv_dspmv(self.h, _ptr(x), _ptr(y)), "dspmv")
        return y

    def spmm(self, X: np.ndarray) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float64)
        L = X.shape[1]
        assert X.shape == (self.num_cols, L)
        Y = np.empty((self.num_rows, L), np.float64)
        _check(lib.mspmv_dspmm(self.h, _ptr(X), _ptr(Y), L), "dspmm")
        return Y

    def spmm_dev(self, dX: DeviceBuffer, dY: DeviceBuffer, L: int = 1, sync: bool = True):
        """Y = A X on device buffers: mspmv_dspmm_dev runs on the handle's (non-blocking) stream, so the
        result is complete only after a sync -- done here unless sync=False."""
        _check(lib.mspmv_dspmm_dev(self.h, dX.ptr, dY.ptr, L), "dspmm_dev")
        if sync:
            self.sync()

    def time_spmm(self, dX: DeviceBuffer, dY: DeviceBuffer, L: int, reps: int, flush_bytes: int = 0):
        """(avg ms per call, avg ms of the tile kernel, kernels per call), HIP events."""
        ms = ctypes.c_double()
        _check(lib.mspmv_time_spmm_dev(self.h, dX.ptr, dY.ptr, L, reps, flush_bytes, ctypes.byref(ms)), "time")
        kms, kpc = ctypes.c_double(), ctypes.c_int()
        _check(lib.mspmv_last_kernel_ms(self.h, ctypes.byref(kms), ctypes.byref(kpc)), "last_kernel_ms")
        return ms.value, kms.value, kpc.value

    def cg_single(self, b: np.ndarray, max_iters: int, tolerance: float, hist_cap: int = 0):
        b = np.ascontiguousarray(b, np.float64)
        x = np.empty_like(b)
        it = ctypes.c_int()
        hist = np.zeros(max(hist_cap, 1), np.float64)
        st = lib.mspmv_dcg_single(self.h, _ptr(b), _ptr(x), max_iters, tolerance, ctypes.byref(it),
                                  _ptr(hist) if hist_cap else None, hist_cap)
        _check(st, "dcg_single", allow=(4,))
        return x, it.value, hist[: min(it.value, hist_cap)], st

    def cg_multi(self, B: np.ndarray, max_iters: int, tolerance: float, kernel: int = MERGE, hist_cap: int = 0,
                 allow_fault: bool = False):
        B = np.ascontiguousarray(B, np.float64)
        L = B.shape[1]
        X = np.empty_like(B)
        it = ctypes.c_int()
        hist = np.zeros(max(hist_cap, 1), np.float64)
        st = lib.mspmv_dcg_multi(self.h, _ptr(B), _ptr(X), L, max_iters, tolerance, kernel, ctypes.byref(it),
                                 _ptr(hist) if hist_cap else None, hist_cap)
        _check(st, "dcg_multi", allow=(4, FAULT) if allow_fault else (4,))
        return X, it.value, hist[: min(it.value, hist_cap)], st

    def cg_dev(self, dB: DeviceBuffer, dX: DeviceBuffer, L: int, max_iters: int, tolerance: float,
               hist_cap: int = 0):
        it = ctypes.c_int()
        hist = np.zeros(max(hist_cap, 1), np.float64)
        st = lib.mspmv_dcg_multi_dev(self.h, dB.ptr, dX.ptr, L, max_iters, tolerance, MERGE, ctypes.byref(it),
                                     _ptr(hist) if hist_cap else None, hist_cap)
        _check(st, "dcg_multi_dev", allow=(4,))
        return it.value, hist[: min(it.value, hist_cap)], st

    def pcg_spai(self, m: "GpuCsr", B: np.ndarray, max_iters: int, tolerance: float, hist_cap: int = 0):
        """SPAISolveMultiple with the preconditioner M's handle `m` (mspmv_dpcg_spai_multi)."""
        B = np.ascontiguousarray(B, np.float64)
        if B.ndim == 1:
            B = B[:, None]
        L = B.shape[1]
        X = np.empty_like(B)
        it = ctypes.c_int()
        hist = np.zeros(max(hist_cap, 1), np.float64)
        st = lib.mspmv_dpcg_spai_multi(self.h, m.h, _ptr(B), _ptr(X), L, max_iters, tolerance, MERGE,
                                       ctypes.byref(it), _ptr(hist) if hist_cap else None, hist_cap)
        _check(st, "dpcg_spai_multi", allow=(4,))
        return X, it.value, hist[: min(it.value, hist_cap)], st

    def pcg_spai_dev(self, m: "GpuCsr", dB: DeviceBuffer, dX: DeviceBuffer, L: int, max_iters: int,
                     tolerance: float, hist_cap: int = 0):
        it = ctypes.c_int()
        hist = np.zeros(max(hist_cap, 1), np.float64)
        st = lib.mspmv_dpcg_spai_multi_dev(self.h, m.h, dB.ptr, dX.ptr, L, max_iters, tolerance, MERGE,
                                           ctypes.byref(it), _ptr(hist) if hist_cap else None, hist_cap)
        _check(st, "dpcg_spai_multi_dev", allow=(4,))
        return it.value, hist[: min(it.value, hist_cap)], st


def ic0_factor(a: CsrMatrix):
    """IncompleteCholesky (incomplete_cholesky_decomp.hpp:84-201) on the host: (L, shift used)."""
    nz = ctypes.c_int()
    _check(lib.mspmv_ic0_nnz(ctypes.byref(a._c()), ctypes.byref(nz)), "ic0_nnz")
    ro = np.zeros(a.num_rows + 1, np.int32)
    ci = np.zeros(max(nz.value, 1), np.int32)
    va = np.zeros(max(nz.value, 1), np.float64)
    sh = ctypes.c_double()
    _check(lib.mspmv_ic0_factor(ctypes.byref(a._c()), _ptr(ro), _ptr(ci), _ptr(va), ctypes.byref(sh)), "ic0_factor")
    return CsrMatrix.from_arrays(a.num_cols, ro, ci[: nz.value], va[: nz.value]), sh.value


class GpuIc0:
    """An IC(0) factor L (and L^T) resident on a device for the GPU triangular solves."""

    def __init__(self, l: CsrMatrix, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib.mspmv_ic0_create(ctypes.byref(l._c()), device, ctypes.byref(h)), "ic0_create")
        self.h = h.value
        _track(self)

    def close(self):
        if getattr(self, "h", None):
            lib.mspmv_ic0_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def pcg_ic0(g: "GpuCsr", ic: GpuIc0, B: np.ndarray, max_iters: int, tolerance: float, hist_cap: int = 0):
    """PCGSolveMultiple (mspmv_dpcg_ic0_multi): (X, iterations, history, status)."""
    B = np.ascontiguousarray(B, np.float64)
    if B.ndim == 1:
        B = B[:, None]
    L = B.shape[1]
    X = np.empty_like(B)
    it = ctypes.c_int()
    hist = np.zeros(max(hist_cap, 1), np.float64)
    st = lib.mspmv_dpcg_ic0_multi(g.h, ic.h, _ptr(B), _ptr(X), L, max_iters, tolerance, MERGE, ctypes.byref(it),
                                  _ptr(hist) if hist_cap else None, hist_cap)
    _check(st, "dpcg_ic0_multi", allow=(4,))
    return X, it.value, hist[: min(it.value, hist_cap)], st


def offset_windows(a: CsrMatrix, min_fill: float = 0.85, min_window_fill: float = 0.3):
    """Host-side offset-window planning (mspmv_offset_windows; no device): None when the matrix does
    not fit the plan, else {"windows", "sum_offsets", "masked_windows", "k", "remainder"} (k: offsets
    per 64-row window; remainder: entries left off the windows' offset lists).  The library's automatic
    choice uses the default thresholds."""
    ok, nw, mw = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    sk, rem = ctypes.c_longlong(), ctypes.c_longlong()
    k = np.zeros(max((a.num_rows + 63) // 64, 1), np.int32)
    _check(lib.mspmv_offset_windows(ctypes.byref(a._c()), min_fill, min_window_fill, ctypes.byref(ok), ctypes.byref(nw),
                                    ctypes.byref(sk), ctypes.byref(mw), _ptr(k), ctypes.byref(rem)), "offset_windows")
    if not ok.value:
        return None
    return {"windows": nw.value, "sum_offsets": sk.value, "masked_windows": mw.value, "k": k[: nw.value],
            "remainder": rem.value}


def spai_values(a: CsrMatrix) -> np.ndarray:
    """M's values on A's pattern (mspmv_spai_values; SparseApproximateInversion,
    work_2025/cg/sparse_approximate_inversion.hpp:40-321).  Host setup, as in the reference."""
    out = np.zeros(max(a.num_nonzeros, 1), np.float64)
    _check(lib.mspmv_spai_values(ctypes.byref(a._c()), _ptr(out)), "spai_values")
    return out[: a.num_nonzeros]


def time_spmm_batch(gs, dXs, dYs, L: int, reps: int):
    """Time `reps` steps of one SpMM launch per matrix, all on gs[0]'s stream.
    Returns (ms per step, ms per merge-tile kernel launch, kernels per step)."""
    n = len(gs)
    H = (_P * n)(*[g.h for g in gs])
    X = (_P * n)(*[b.ptr for b in dXs])
    Y = (_P * n)(*[b.ptr for b in dYs])
    step, kern, kps = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    _check(lib.mspmv_time_spmm_batch_dev(n, H, X, Y, L, reps, ctypes.byref(step), ctypes.byref(kern),
                                         ctypes.byref(kps)), "time_spmm_batch")
    return step.value, kern.value, kps.value


# ----------------------------------------------------------------------------------------
# the reference's operator names (drop-in facade)
# ----------------------------------------------------------------------------------------
def _note_breakdown(st: int, where: str) -> None:
    """The reference-named solvers return an iteration count only, as the reference's do; a CG
    breakdown (non-finite alpha in some column: that column frozen, the others solved) is
    surfaced as a RuntimeWarning instead of passing silently."""
    if st == 4:
        import warnings
        warnings.warn(f"{where}: {lib.mspmv_last_error().decode(errors='replace')}", RuntimeWarning, stacklevel=3)


def _gpu(a: CsrMatrix) -> GpuCsr:
    g = getattr(a, "_gpu", None)
    if g is None or g.h is None:
        g = GpuCsr(a)
        object.__setattr__(a, "_gpu", g)
    return g


def OmpMergeCsrmv(num_threads, a: CsrMatrix, row_end_offsets, column_indices, values, vector_x, vector_y_out):
    """cpu_spmv.cpp:357-421: vector_y_out[:] = A @ vector_x (num_threads ignored on the GPU)."""
    vector_y_out[:] = _gpu(a).spmv(vector_x)


def OmpMergeCsrmm(num_threads, a: CsrMatrix, row_end_offsets, column_indices, values, vector_x, vector_y_out,
                  num_vectors):
    """work_2025/spmm/merge_based.hpp:46-153 on flat row-major n x num_vectors panels."""
    X = np.asarray(vector_x, np.float64).reshape(a.num_cols, num_vectors)
    vector_y_out[:] = _gpu(a).spmm(X).reshape(-1)


def CGSolveSingle(a: CsrMatrix, b, x, max_iters: int, tolerance: float) -> int:
    """work_2025/main/single_strategy.hpp:102-170; returns the iteration count."""
    xs, it, _, st = _gpu(a).cg_single(b, max_iters, tolerance)
    _note_breakdown(st, "CGSolveSingle")
    x[:] = xs
    return it


def CGSolveMultiple(a: CsrMatrix, B, X, num_vectors: int, max_iters: int, tolerance: float,
                    kernel_type: int = MERGE, max_errors: Optional[list] = None) -> int:
    """work_2025/main/no_pretreatment.hpp:32-197 on flat interleaved n x num_vectors panels."""
    Bm = np.asarray(B, np.float64).reshape(a.num_rows, num_vectors)
    cap = max_iters if max_errors is not None else 0
    Xs, it, hist, st = _gpu(a).cg_multi(Bm, max_iters, tolerance, kernel_type, hist_cap=cap)
    _note_breakdown(st, "CGSolveMultiple")
    X[:] = Xs.reshape(-1)
    if max_errors is not None:
        max_errors.clear()
        max_errors.extend(hist.tolist())
    return it


def SparseApproximateInversion(a: CsrMatrix) -> CsrMatrix:
    """work_2025/cg/sparse_approximate_inversion.hpp:40-321: returns M (A's pattern, SPAI values).
    The reference fills an output CsrMatrix argument and returns true; here M is returned."""
    return CsrMatrix.from_arrays(a.num_cols, a.row_offsets, a.column_indices, spai_values(a))


def SPAISolveMultiple(a: CsrMatrix, m: CsrMatrix, B, X, num_vectors: int, max_iters: int, tolerance: float,
                      kernel_type: int = MERGE, max_errors: Optional[list] = None) -> int:
    """work_2025/main/sparse_approximate_inverse.hpp:30-230 on flat interleaved n x num_vectors panels."""
    Bm = np.asarray(B, np.float64).reshape(a.num_rows, num_vectors)
    cap = max_iters if max_errors is not None else 0
    Xs, it, hist, st = _gpu(a).pcg_spai(_gpu(m), Bm, max_iters, tolerance, hist_cap=cap)
    _note_breakdown(st, "SPAISolveMultiple")
    X[:] = Xs.reshape(-1)
    if max_errors is not None:
        max_errors.clear()
        max_errors.extend(hist.tolist())
    return it


def IncompleteCholesky(a: CsrMatrix) -> CsrMatrix:
    """work_2025/cg/incomplete_cholesky_decomp.hpp:84-201: returns L (raises if it fails)."""
    return ic0_factor(a)[0]


def PCGSolveMultiple(a: CsrMatrix, l: CsrMatrix, l_transpose, B, X, num_vectors: int, max_iters: int,
                     tolerance: float, kernel_type: int = MERGE, max_errors: Optional[list] = None) -> int:
    """work_2025/main/incomplete_cholesky.hpp:33-199.  l_transpose is accepted for signature
    compatibility; the device factor forms its own transpose."""
    Bm = np.asarray(B, np.float64).reshape(a.num_rows, num_vectors)
    cap = max_iters if max_errors is not None else 0
    ic = getattr(l, "_gpu_ic0", None)
    if ic is None or ic.h is None:
        ic = GpuIc0(l)
        object.__setattr__(l, "_gpu_ic0", ic)
    Xs, it, hist, st = pcg_ic0(_gpu(a), ic, Bm, max_iters, tolerance, hist_cap=cap)
    _note_breakdown(st, "PCGSolveMultiple")
    X[:] = Xs.reshape(-1)
    if max_errors is not None:
        max_errors.clear()
        max_errors.extend(hist.tolist())
    return it


# ----------------------------------------------------------------------------------------
# row-block sharding over several GPUs (include/mspmv_dist.h)
# ----------------------------------------------------------------------------------------
def dist_partition(a: CsrMatrix, nranks: int) -> np.ndarray:
    """Row blocks balanced by merge path (equal rows + nonzeros per rank)."""
    rb = np.empty(nranks + 1, np.int32)
    _check(lib.mspmv_dist_partition(_ptr(a.row_offsets), a.num_rows, a.num_nonzeros, nranks, _ptr(rb)),
           "dist_partition")
    return rb


def dist_partition_offsets(row_offsets: np.ndarray, num_rows: int, num_nonzeros: int, nranks: int) -> np.ndarray:
    """dist_partition from a global row_offsets array alone (ranks that never build the matrix)."""
    ro = np.ascontiguousarray(row_offsets, np.int32)
    rb = np.empty(nranks + 1, np.int32)
    _check(lib.mspmv_dist_partition(_ptr(ro), num_rows, num_nonzeros, nranks, _ptr(rb)), "dist_partition")
    return rb


def memcpy_h2d_ptr(d_ptr: int, a: np.ndarray) -> None:
    """Copy a host array to a raw device pointer (e.g. DistCsr.x_ext)."""
    a = np.ascontiguousarray(a)
    _check(lib.mspmv_memcpy_h2d(d_ptr, _ptr(a), a.nbytes), "memcpy_h2d")


def local_rows(a: CsrMatrix, row_begin: np.ndarray, rank: int) -> CsrMatrix:
    """This rank's rows with GLOBAL column ids (num_cols = global n)."""
    lo, hi = int(row_begin[rank]), int(row_begin[rank + 1])
    s, e = int(a.row_offsets[lo]), int(a.row_offsets[hi])
    ro = np.ascontiguousarray(a.row_offsets[lo:hi + 1] - s, np.int32)
    return CsrMatrix(hi - lo, a.num_cols, e - s, ro, np.ascontiguousarray(a.column_indices[s:e]),
                     np.ascontiguousarray(a.values[s:e]))


def dist_localize(row_begin: np.ndarray, rank: int, loc: CsrMatrix):
    """(local column ids, sorted halo global ids, halo counts per owner rank)."""
    nranks = len(row_begin) - 1
    rb = np.ascontiguousarray(row_begin, np.int32)
    nh = ctypes.c_int()
    _check(lib.mspmv_dist_localize(_ptr(rb), nranks, rank, _ptr(loc.row_offsets), _ptr(loc.column_indices), None,
                                   ctypes.byref(nh), None, 0, None), "dist_localize(size)")
    lcols = np.empty(max(loc.num_nonzeros, 1), np.int32)
    halo = np.empty(max(nh.value, 1), np.int32)
    counts = np.empty(nranks, np.int32)
    _check(lib.mspmv_dist_localize(_ptr(rb), nranks, rank, _ptr(loc.row_offsets), _ptr(loc.column_indices),
                                   _ptr(lcols), ctypes.byref(nh), _ptr(halo), nh.value, _ptr(counts)),
           "dist_localize")
    return lcols[:loc.num_nonzeros], halo[:nh.value], counts


def comm_unique_id() -> bytes:
    buf = (ctypes.c_ubyte * 128)()
    _check(lib.mspmv_comm_unique_id(buf), "comm_unique_id")
    return bytes(buf)


class Comm:
    """This rank's RCCL communicator and its one stream (mspmv_comm_create, collective): every
    DistCsr created on it runs its kernels and collectives on that stream, so a rank's collectives
    are one sequence in program order.  Close it after every DistCsr on it."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int):
        idb = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        _check(lib.mspmv_comm_create(idb, nranks, rank, device, ctypes.byref(h)), "comm_create")
        self.h, self.nranks, self.rank, self.device = h.value, nranks, rank, device
        _track(self)

    def close(self):
        if getattr(self, "h", None):
            _check(lib.mspmv_comm_destroy(self.h), "comm_destroy")
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class DistCsr:
    """This rank's row block of a matrix sharded over `nranks` GPUs (collective create).  Either
    on a shared Comm -- DistCsr(comm, row_begin, loc), the form for several matrices per rank -- or
    on a private communicator: DistCsr(uid, nranks, rank, device, row_begin, loc)."""

    def __init__(self, *args):
        if len(args) == 3:
            comm, row_begin, loc = args
            self.row_begin = np.ascontiguousarray(row_begin, np.int32)
            h = ctypes.c_void_p()
            _check(lib.mspmv_dist_create_on(comm.h, _ptr(self.row_begin), ctypes.byref(loc._c()), ctypes.byref(h)),
                   "dist_create_on")
        else:
            uid, nranks, rank, device, row_begin, loc = args
            self.row_begin = np.ascontiguousarray(row_begin, np.int32)
            idb = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
            h = ctypes.c_void_p()
            _check(lib.mspmv_dist_create(idb, nranks, rank, device, _ptr(self.row_begin), ctypes.byref(loc._c()),
                                         ctypes.byref(h)), "dist_create")
        self.h = h.value
        self.n_own = loc.num_rows
        _track(self)

    def info(self):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib.mspmv_dist_info(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "dist_info")
        return {"n_own": a.value, "n_halo": b.value, "n_send": c.value}

    def spmm_dev(self, dX, dY: DeviceBuffer, L: int, sync: bool = True):
        """Y_own = (A X)_own with the halo exchange.  dX: a DeviceBuffer of X_own, or the
        extended buffer's pointer (x_ext) whose first n_own rows the caller filled."""
        xp = dX.ptr if isinstance(dX, DeviceBuffer) else dX
        _check(lib.mspmv_dist_spmm_dev(self.h, xp, dY.ptr, L), "dist_spmm_dev")
        if sync:
            self.sync()

    def x_ext(self, L: int) -> int:
        """Device pointer of the (n_own + n_halo) x L extended panel (rows [0, n_own) = X_own)."""
        p = ctypes.c_void_p()
        _check(lib.mspmv_dist_x_ext(self.h, L, ctypes.byref(p)), "dist_x_ext")
        return p.value

    def sync(self):
        _check(lib.mspmv_dist_sync(self.h), "dist_sync")

    def time_local(self, dY: DeviceBuffer, L: int, reps: int) -> float:
        """Average ms of the local SpMM alone (no exchange), HIP events on the local stream."""
        ms = ctypes.c_double()
        _check(lib.mspmv_dist_time_local_dev(self.h, dY.ptr, L, reps, ctypes.byref(ms)), "dist_time_local")
        return ms.value

    def cg_dev(self, dB: DeviceBuffer, dX: DeviceBuffer, L: int, max_iters: int, tolerance: float,
               hist_cap: int = 0, allow_fault: bool = False):
        it = ctypes.c_int()
        hist = np.zeros(max(hist_cap, 1))
        st = lib.mspmv_dist_cg_dev(self.h, dB.ptr, dX.ptr, L, max_iters, tolerance, ctypes.byref(it),
                                   _ptr(hist) if hist_cap else None, hist_cap)
        _check(st, "dist_cg_dev", allow=(4, FAULT) if allow_fault else (4,))
        return it.value, hist[: min(it.value, hist_cap)], st

    def test_poison_tickets(self, value: int, flags: int = POISON_FILL):
        """Test hook: the next sharded CG solve's fold tickets start at `value`."""
        _check(lib.mspmv_dist_test_poison_tickets(self.h, value, flags), "dist_test_poison_tickets")

    def close(self):
        if getattr(self, "h", None):
            lib.mspmv_dist_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
