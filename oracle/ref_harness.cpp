// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" driver around the reference's OWN header-only kernels, compiled
// from the sources where they lie under /root/reference (oracle/Makefile, output
// oracle/_ref/libmspmv_ref.so, never committed).  No reference source is copied
// here; only its headers are #included by path.  Used to:
//   * pin oracle/mspmv_oracle.c (tests/test_oracle_pinning.py), and
//   * generate the committed golden vectors (tests/golden/make_golden.py).
//
// Buildable subset (no <mkl.h> on this image; every header below is MKL-free
// when CUB_MKL is undefined):
//   sparse_matrix.h                    CooMatrix::InitMarket/InitGrid2d/InitGrid3d/
//                                      InitWheel/InitDense, CsrMatrix::Init
//   work_2025/spmm/merge_based.hpp     MergePathSearch, OmpMergeCsrmm
//   work_2025/spmm/sample.hpp          SpmvGold
//   work_2025/spmm/row_splitting.hpp   OmpCsrSpmmT
//   work_2025/spmm/nonzero_splitting.hpp OmpNonzeroSplitCsrmm
// NOT buildable here: cpu_spmv.cpp (#include <mkl.h> at :59), work_2025/main/*.hpp and
// work_2025/cg/utils_multiple.hpp (#include <mkl.h>).  cpu_spmv.cpp's OmpMergeCsrmv
// (:357-421) is pinned through OmpMergeCsrmm with num_vectors = 1, which performs the
// identical operation sequence (same partition, same running_total order, same fix-up;
// its extra fix-up of the last thread is a no-op because that carry's row is m).

#include <cstdlib>
#include <cstring>
#include <string>

#include "sparse_matrix.h"
#include "work_2025/hyper_parameters.hpp"
#include "work_2025/types.hpp"
#include "work_2025/spmm/merge_based.hpp"
#include "work_2025/spmm/sample.hpp"
#include "work_2025/spmm/row_splitting.hpp"
#include "work_2025/spmm/nonzero_splitting.hpp"

#define REF_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

// Borrowing view: CsrMatrix frees its arrays in ~CsrMatrix (sparse_matrix.h:738-792),
// so the borrowed pointers are detached before destruction.
struct CsrView {
    CsrMatrix<double, int> a;
    CsrView(int m, int n, int nnz, const int *ro, const int *ci, const double *v)
    {
        a.num_rows = m;
        a.num_cols = n;
        a.num_nonzeros = nnz;
        a.row_offsets = const_cast<int *>(ro);
        a.column_indices = const_cast<int *>(ci);
        a.values = const_cast<double *>(v);
    }
    ~CsrView()
    {
        a.row_offsets = nullptr;
        a.column_indices = nullptr;
        a.values = nullptr;
    }
};

CsrMatrix<double, int> *g_last = nullptr;  // last matrix built by a ref_build_* call

void keep(CooMatrix<double, int> &coo)
{
    if (g_last)
        delete g_last;
    g_last = new CsrMatrix<double, int>(coo);  // CsrMatrix::Init: stable_sort + CSR fill
    coo.Clear();
}

}  // namespace

REF_EXPORT void ref_merge_path_search(int diagonal, const int *row_end_offsets, int a_len, int b_len, int *x, int *y)
{
    CountingInputIterator<int> nonzero_indices(0);
    int2 c;
    MergePathSearch(diagonal, row_end_offsets, nonzero_indices, a_len, b_len, c);
    *x = c.x;
    *y = c.y;
}

REF_EXPORT void ref_spmv_gold(int m, int n, int nnz, const int *ro, const int *ci, const double *v, const double *x,
                              const double *y_in, double *y_out, double alpha, double beta)
{
    CsrView w(m, n, nnz, ro, ci, v);
    SpmvGold(w.a, const_cast<double *>(x), const_cast<double *>(y_in), y_out, alpha, beta);
}

REF_EXPORT void ref_merge_csrmm(int num_threads, int m, int n, int nnz, const int *ro, const int *ci, const double *v,
                                const double *X, double *Y, int L)
{
    CsrView w(m, n, nnz, ro, ci, v);
    OmpMergeCsrmm(num_threads, w.a, const_cast<int *>(ro) + 1, const_cast<int *>(ci), const_cast<double *>(v),
                  const_cast<double *>(X), Y, L);
}

REF_EXPORT void ref_csr_spmm_t(int num_threads, int m, int n, int nnz, const int *ro, const int *ci, const double *v,
                               const double *X, double *Y, int L)
{
    CsrView w(m, n, nnz, ro, ci, v);
    OmpCsrSpmmT(num_threads, w.a, const_cast<double *>(X), Y, L);
}

REF_EXPORT void ref_nonzero_split_csrmm(int num_threads, int m, int n, int nnz, const int *ro, const int *ci,
                                        const double *v, const double *X, double *Y, int L)
{
    CsrView w(m, n, nnz, ro, ci, v);
    OmpNonzeroSplitCsrmm(num_threads, w.a, const_cast<int *>(ro) + 1, const_cast<int *>(ci), const_cast<double *>(v),
                         const_cast<double *>(X), Y, L);
}

// --- matrix builders: build, then query sizes, then copy out ------------------
REF_EXPORT int ref_build_market(const char *path, double default_value)
{
    CooMatrix<double, int> coo;
    coo.InitMarket(std::string(path), default_value, false);
    keep(coo);
    return 0;
}

REF_EXPORT int ref_build_grid2d(int width, int self_loop)
{
    CooMatrix<double, int> coo;
    coo.InitGrid2d(width, self_loop != 0);
    keep(coo);
    return 0;
}

REF_EXPORT int ref_build_grid3d(int width, int self_loop)
{
    CooMatrix<double, int> coo;
    coo.InitGrid3d(width, self_loop != 0);
    keep(coo);
    return 0;
}

REF_EXPORT int ref_build_wheel(int spokes)
{
    CooMatrix<double, int> coo;
    coo.InitWheel(spokes);
    keep(coo);
    return 0;
}

REF_EXPORT int ref_build_dense(int rows, int cols)
{
    CooMatrix<double, int> coo;
    coo.InitDense(rows, cols);
    keep(coo);
    return 0;
}

REF_EXPORT void ref_last_shape(int *m, int *n, int *nnz)
{
    *m = g_last ? g_last->num_rows : 0;
    *n = g_last ? g_last->num_cols : 0;
    *nnz = g_last ? g_last->num_nonzeros : 0;
}

REF_EXPORT void ref_last_copy(int *ro, int *ci, double *v)
{
    std::memcpy(ro, g_last->row_offsets, sizeof(int) * (g_last->num_rows + 1));
    std::memcpy(ci, g_last->column_indices, sizeof(int) * g_last->num_nonzeros);
    std::memcpy(v, g_last->values, sizeof(double) * g_last->num_nonzeros);
}
