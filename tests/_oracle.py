"""ctypes wrapper over oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY (the checker).

Also wraps oracle/_ref/libmspmv_ref.so (the reference's own kernels compiled from
/root/reference) when it exists; it exists only where the reference checkout does.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libmspmv_ref.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double
_PI = ctypes.POINTER(ctypes.c_int)


def _p(a):
    return None if a is None else a.ctypes.data


class Oracle:
    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        sig = {
            "orc_merge_path_search": (None, [_I, _P, _I, _I, _PI, _PI]),
            "orc_merge_coords": (None, [_P, _I, _I, _I, _P]),
            "orc_spmv_gold": (None, [_I, _P, _P, _P, _P, _P, _P, _D, _D]),
            "orc_csr_spmv": (None, [_I, _P, _P, _P, _P, _P]),
            "orc_merge_csrmv": (None, [_I, _I, _I, _P, _P, _P, _P, _P]),
            "orc_merge_csrmm": (None, [_I, _I, _I, _P, _P, _P, _P, _P, _I]),
            "orc_csr_spmm_t": (None, [_I, _P, _P, _P, _P, _P, _I]),
            "orc_nonzero_split_csrmm": (None, [_I, _I, _I, _P, _P, _P, _P, _P, _I]),
            "orc_cg_single": (_I, [_I, _P, _P, _P, _P, _P, _I, _D, _P, _I]),
            "orc_cg_multi": (_I, [_I, _I, _P, _P, _P, _P, _P, _I, _I, _D, _I, _I, _P, _I]),
            "orc_pcg_spai_multi": (_I, [_I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _D, _I, _I, _P, _I]),
            "orc_ic0_factor": (_I, [_I, _P, _P, _P, _P, _P, _P, _P]),
            "orc_pcg_ic0_multi": (_I, [_I, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _D, _I, _I, _P, _I]),
            "orc_nonzero_split_csrmv_v1": (_I, [_I, _I, _I, _P, _P, _P, _P, _P]),
            "orc_calculate_threshold": (_D, [_P, _I, _D]),
            "orc_glibc_rand_fill": (None, [ctypes.c_uint, ctypes.c_longlong, _P]),
            "orc_coo_to_csr": (None, [_I, _I, _P, _P, _P, _P, _P, _P]),
            "orc_grid2d_coo": (_I, [_I, _I, _D, _P, _P, _P]),
            "orc_grid3d_coo": (_I, [_I, _I, _D, _P, _P, _P]),
            "orc_wheel_coo": (_I, [_I, _D, _P, _P, _P]),
            "orc_dense_coo": (_I, [_I, _I, _D, _P, _P, _P]),
            "orc_read_market": (_I, [ctypes.c_char_p, _D, _PI, _PI, _PI, _I, _P, _P, _P]),
            "orc_num_procs": (_I, []),
            "orc_set_threads": (None, [_I]),
            "orc_max_threads": (_I, []),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        self.lib = L

    # -- partition ---------------------------------------------------------------------
    def merge_path_search(self, diagonal, row_end_offsets, a_len, b_len):
        x, y = ctypes.c_int(), ctypes.c_int()
        self.lib.orc_merge_path_search(diagonal, _p(row_end_offsets), a_len, b_len, ctypes.byref(x), ctypes.byref(y))
        return x.value, y.value

    def merge_coords(self, a, P):
        out = np.empty((P + 1, 2), np.int32)
        self.lib.orc_merge_coords(_p(a.row_offsets), a.num_rows, a.num_nonzeros, P, _p(out))
        return out

    # -- kernels -----------------------------------------------------------------------
    def spmv_gold(self, a, x, y_in=None, alpha=1.0, beta=0.0):
        x = np.ascontiguousarray(x, np.float64)
        y_in = np.ones(a.num_rows) if y_in is None else np.ascontiguousarray(y_in, np.float64)
        y = np.empty(a.num_rows)
        self.lib.orc_spmv_gold(a.num_rows, _p(a.row_offsets), _p(a.column_indices), _p(a.values), _p(x), _p(y_in),
                               _p(y), alpha, beta)
        return y

    def csr_spmv(self, a, x):
        x = np.ascontiguousarray(x, np.float64)
        y = np.empty(a.num_rows)
        self.lib.orc_csr_spmv(a.num_rows, _p(a.row_offsets), _p(a.column_indices), _p(a.values), _p(x), _p(y))
        return y

    def merge_csrmv(self, a, x, P):
        x = np.ascontiguousarray(x, np.float64)
        y = np.empty(a.num_rows)
        self.lib.orc_merge_csrmv(P, a.num_rows, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices),
                                 _p(a.values), _p(x), _p(y))
        return y

    def merge_csrmm(self, a, X, P):
        X = np.ascontiguousarray(X, np.float64)
        L = X.shape[1]
        Y = np.empty((a.num_rows, L))
        self.lib.orc_merge_csrmm(P, a.num_rows, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices),
                                 _p(a.values), _p(X), _p(Y), L)
        return Y

    def csr_spmm_t(self, a, X):
        X = np.ascontiguousarray(X, np.float64)
        L = X.shape[1]
        Y = np.empty((a.num_rows, L))
        self.lib.orc_csr_spmm_t(a.num_rows, _p(a.row_offsets), _p(a.column_indices), _p(a.values), _p(X), _p(Y), L)
        return Y

    def nonzero_split_csrmm(self, a, X, P, Y0=None):
        X = np.ascontiguousarray(X, np.float64)
        L = X.shape[1]
        Y = np.zeros((a.num_rows, L)) if Y0 is None else np.array(Y0, np.float64, copy=True)
        self.lib.orc_nonzero_split_csrmm(P, a.num_rows, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices),
                                         _p(a.values), _p(X), _p(Y), L)
        return Y

    def nonzero_split_csrmv_v1(self, a, x, P, y0):
        """cpu_spmv.cpp's OmpNonzeroSplitCsrmm (:506-570): y is in/out (its last-row bug)."""
        x = np.ascontiguousarray(x, np.float64)
        y = np.array(y0, np.float64, copy=True)
        rc = self.lib.orc_nonzero_split_csrmv_v1(P, a.num_rows, a.num_nonzeros, _p(a.row_offsets),
                                                 _p(a.column_indices), _p(a.values), _p(x), _p(y))
        if rc:
            raise ValueError("P must be in [1, 256] (row_carry_out[256], cpu_spmv.cpp:513)")
        return y

    def cg_single(self, a, b, max_iters, tol, hist_cap=0):
        b = np.ascontiguousarray(b, np.float64)
        x = np.empty_like(b)
        hist = np.zeros(max(hist_cap, 1))
        it = self.lib.orc_cg_single(a.num_rows, _p(a.row_offsets), _p(a.column_indices), _p(a.values), _p(b), _p(x),
                                    max_iters, tol, _p(hist) if hist_cap else None, hist_cap)
        return x, it, hist[: min(it, hist_cap)]

    def cg_multi(self, a, B, max_iters, tol, kernel=1, P=8, hist_cap=0):
        B = np.ascontiguousarray(B, np.float64)
        L = B.shape[1]
        X = np.empty_like(B)
        hist = np.zeros(max(hist_cap, 1))
        it = self.lib.orc_cg_multi(a.num_rows, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices), _p(a.values),
                                   _p(B), _p(X), L, max_iters, tol, kernel, P, _p(hist) if hist_cap else None,
                                   hist_cap)
        return X, it, hist[: min(it, hist_cap)]

    def pcg_spai_multi(self, a, m_vals, B, max_iters, tol, kernel=1, P=8, hist_cap=0):
        """SPAISolveMultiple (sparse_approximate_inverse.hpp:30-230); M = (A's pattern, m_vals)."""
        B = np.ascontiguousarray(B, np.float64)
        m_vals = np.ascontiguousarray(m_vals, np.float64)
        L = B.shape[1]
        X = np.empty_like(B)
        hist = np.zeros(max(hist_cap, 1))
        it = self.lib.orc_pcg_spai_multi(a.num_rows, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices),
                                         _p(a.values), _p(m_vals), _p(B), _p(X), L, max_iters, tol, kernel, P,
                                         _p(hist) if hist_cap else None, hist_cap)
        return X, it, hist[: min(it, hist_cap)]

    def ic0_factor(self, a):
        """IncompleteCholesky (incomplete_cholesky_decomp.hpp:84-201) -> (l_ro, l_ci, l_va, shift)."""
        n = a.num_rows
        lro = np.zeros(n + 1, np.int32)
        lci = np.zeros(max(a.num_nonzeros, 1), np.int32)
        lva = np.zeros(max(a.num_nonzeros, 1))
        sh = ctypes.c_double()
        ok = self.lib.orc_ic0_factor(n, _p(a.row_offsets), _p(a.column_indices), _p(a.values), _p(lro), _p(lci),
                                     _p(lva), ctypes.byref(sh))
        if not ok:
            raise RuntimeError("oracle IC(0) failed")
        nz = int(lro[-1])
        return lro, lci[:nz].copy(), lva[:nz].copy(), sh.value

    def pcg_ic0_multi(self, a, l_ro, l_ci, l_va, B, max_iters, tol, kernel=1, P=8, hist_cap=0):
        """PCGSolveMultiple (incomplete_cholesky.hpp:33-199) with the factor L."""
        B = np.ascontiguousarray(B, np.float64)
        L = B.shape[1]
        X = np.empty_like(B)
        hist = np.zeros(max(hist_cap, 1))
        l_ro, l_ci, l_va = (np.ascontiguousarray(l_ro, np.int32), np.ascontiguousarray(l_ci, np.int32),
                            np.ascontiguousarray(l_va, np.float64))
        it = self.lib.orc_pcg_ic0_multi(a.num_rows, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices),
                                        _p(a.values), int(l_ro[-1]), _p(l_ro), _p(l_ci), _p(l_va), _p(B), _p(X), L,
                                        max_iters, tol, kernel, P, _p(hist) if hist_cap else None, hist_cap)
        return X, it, hist[: min(it, hist_cap)]

    def calculate_threshold(self, b, n, tol):
        return self.lib.orc_calculate_threshold(_p(np.ascontiguousarray(b, np.float64)), n, tol)

    def glibc_rand(self, seed, n):
        out = np.empty(n)
        self.lib.orc_glibc_rand_fill(seed, n, _p(out))
        return out

    # -- matrices ----------------------------------------------------------------------
    def coo_to_csr(self, m, n, rows, cols, vals):
        import mspmv
        nnz = len(rows)
        rows = np.ascontiguousarray(rows, np.int32)
        cols = np.ascontiguousarray(cols, np.int32)
        vals = np.ascontiguousarray(vals, np.float64)
        ro = np.empty(m + 1, np.int32)
        ci = np.empty(max(nnz, 1), np.int32)
        va = np.empty(max(nnz, 1), np.float64)
        self.lib.orc_coo_to_csr(m, nnz, _p(rows), _p(cols), _p(vals), _p(ro), _p(ci), _p(va))
        return mspmv.CsrMatrix(m, n, nnz, ro, ci[:nnz], va[:nnz])

    def generator(self, kind, *params):
        """kind in grid2d(width, self_loop) / grid3d(width, self_loop) / wheel(spokes) / dense(rows, cols)."""
        if kind == "grid2d":
            w, sl = params
            cap, m = w * w * 5, w * w
        elif kind == "grid3d":
            w, sl = params
            cap, m = w ** 3 * 7, w ** 3
        elif kind == "wheel":
            (s,) = params
            cap, m = 2 * s, s + 1
        else:
            r, c = params
            cap, m = r * c, r
        rows = np.empty(cap, np.int32)
        cols = np.empty(cap, np.int32)
        vals = np.empty(cap, np.float64)
        if kind == "grid2d":
            nz = self.lib.orc_grid2d_coo(w, sl, 1.0, _p(rows), _p(cols), _p(vals))
        elif kind == "grid3d":
            nz = self.lib.orc_grid3d_coo(w, sl, 1.0, _p(rows), _p(cols), _p(vals))
        elif kind == "wheel":
            nz = self.lib.orc_wheel_coo(s, 1.0, _p(rows), _p(cols), _p(vals))
        else:
            nz = self.lib.orc_dense_coo(r, c, 1.0, _p(rows), _p(cols), _p(vals))
        n = c if kind == "dense" else m
        return self.coo_to_csr(m, n, rows[:nz], cols[:nz], vals[:nz])

    def read_market(self, path, default_value=1.0):
        m, n, nnz = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = self.lib.orc_read_market(path.encode(), default_value, ctypes.byref(m), ctypes.byref(n),
                                      ctypes.byref(nnz), 0, None, None, None)
        if rc:
            return rc, None
        cap = max(nnz.value, 1)
        rows = np.empty(cap, np.int32)
        cols = np.empty(cap, np.int32)
        vals = np.empty(cap, np.float64)
        rc = self.lib.orc_read_market(path.encode(), default_value, ctypes.byref(m), ctypes.byref(n),
                                      ctypes.byref(nnz), cap, _p(rows), _p(cols), _p(vals))
        if rc:
            return rc, None
        k = nnz.value
        return 0, self.coo_to_csr(m.value, n.value, rows[:k], cols[:k], vals[:k])


class RefLib:
    """The reference's own kernels (oracle/_ref), only where /root/reference was built."""

    def __init__(self, path=REF_SO):
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing (build with `make -C oracle ref` where /root/reference exists)")
        L = ctypes.CDLL(path)
        sig = {
            "ref_merge_path_search": (None, [_I, _P, _I, _I, _PI, _PI]),
            "ref_spmv_gold": (None, [_I, _I, _I, _P, _P, _P, _P, _P, _P, _D, _D]),
            "ref_merge_csrmm": (None, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _I]),
            "ref_csr_spmm_t": (None, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _I]),
            "ref_nonzero_split_csrmm": (None, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _I]),
            "ref_build_market": (_I, [ctypes.c_char_p, _D]),
            "ref_build_grid2d": (_I, [_I, _I]),
            "ref_build_grid3d": (_I, [_I, _I]),
            "ref_build_wheel": (_I, [_I]),
            "ref_build_dense": (_I, [_I, _I]),
            "ref_last_shape": (None, [_PI, _PI, _PI]),
            "ref_last_copy": (None, [_P, _P, _P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        self.lib = L

    def _fetch(self):
        import mspmv
        m, n, nnz = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.lib.ref_last_shape(ctypes.byref(m), ctypes.byref(n), ctypes.byref(nnz))
        ro = np.empty(m.value + 1, np.int32)
        ci = np.empty(max(nnz.value, 1), np.int32)
        va = np.empty(max(nnz.value, 1), np.float64)
        self.lib.ref_last_copy(_p(ro), _p(ci), _p(va))
        k = nnz.value
        return mspmv.CsrMatrix(m.value, n.value, k, ro, ci[:k], va[:k])

    def build(self, kind, *params):
        getattr(self.lib, "ref_build_" + kind)(*params)
        return self._fetch()

    def build_market(self, path, default_value=1.0):
        self.lib.ref_build_market(path.encode(), default_value)
        return self._fetch()

    def merge_path_search(self, diagonal, row_end_offsets, a_len, b_len):
        x, y = ctypes.c_int(), ctypes.c_int()
        self.lib.ref_merge_path_search(diagonal, _p(row_end_offsets), a_len, b_len, ctypes.byref(x), ctypes.byref(y))
        return x.value, y.value

    def spmv_gold(self, a, x, y_in=None, alpha=1.0, beta=0.0):
        y_in = np.ones(a.num_rows) if y_in is None else np.ascontiguousarray(y_in, np.float64)
        y = np.empty(a.num_rows)
        self.lib.ref_spmv_gold(a.num_rows, a.num_cols, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices),
                               _p(a.values), _p(np.ascontiguousarray(x, np.float64)), _p(y_in), _p(y), alpha, beta)
        return y

    def _mm(self, fn, a, X, P, Y0=None):
        X = np.ascontiguousarray(X, np.float64)
        L = X.shape[1]
        Y = np.zeros((a.num_rows, L)) if Y0 is None else np.array(Y0, np.float64, copy=True)
        fn(P, a.num_rows, a.num_cols, a.num_nonzeros, _p(a.row_offsets), _p(a.column_indices), _p(a.values), _p(X),
           _p(Y), L)
        return Y

    def merge_csrmm(self, a, X, P):
        return self._mm(self.lib.ref_merge_csrmm, a, X, P)

    def csr_spmm_t(self, a, X, P=8):
        return self._mm(self.lib.ref_csr_spmm_t, a, X, P)

    def nonzero_split_csrmm(self, a, X, P, Y0=None):
        return self._mm(self.lib.ref_nonzero_split_csrmm, a, X, P, Y0)
