// mspmv.hpp -- header-only C++ facade with the reference's own names and signatures, over the
// C-ABI in mspmv.h.  A reference caller replaces
//     #include "work_2025/spmm/merge_based.hpp" / single_strategy.hpp / no_pretreatment.hpp
// by this header and links libmspmv.so; call sites stay as they are:
//     OmpMergeCsrmv(g_omp_threads, a, a.row_offsets + 1, a.column_indices, a.values, x, y);   // cpu_spmv.cpp:448
//     OmpMergeCsrmm(g_omp_threads, a, a.row_offsets + 1, a.column_indices, a.values, X, Y, L); // merge_based.hpp:46
//     int it = CGSolveSingle(a, b, x, max_iters, threshold);                                   // single_strategy.hpp:102
//     int it = CGSolveMultiple(a, B, X, L, max_iters, threshold, NONZERO_SPLIT, &errs);        // no_pretreatment.hpp:32
// `Csr` is any type with the CsrMatrix<double,int> fields (sparse_matrix.h:648-653).  The matrix is
// uploaded to HBM on first use and cached per (values pointer, nnz); call mspmv_facade_release(a)
// before freeing or mutating a matrix.  num_threads is accepted and ignored (the GPU decides).
// Errors throw std::runtime_error with mspmv_last_error() (the reference exit()s instead).
#pragma once

#include <algorithm>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "mspmv.h"

namespace mspmv_facade {

inline void check(mspmv_status s, const char *where)
{
    if (s != MSPMV_OK && s != MSPMV_ERR_BREAKDOWN)
        throw std::runtime_error(std::string(where) + ": " + mspmv_last_error());
}

inline std::map<std::pair<const void *, int>, mspmv_handle> &cache()
{
    static std::map<std::pair<const void *, int>, mspmv_handle> c;
    return c;
}

template <typename Csr>
mspmv_handle handle_for(const Csr &a, int device = 0)
{
    auto key = std::make_pair((const void *)a.values, (int)a.num_nonzeros);
    auto it = cache().find(key);
    if (it != cache().end())
        return it->second;
    mspmv_csr_d d{a.num_rows, a.num_cols, a.num_nonzeros, a.row_offsets, a.column_indices, a.values};
    mspmv_handle h = nullptr;
    check(mspmv_csr_create(&d, device, &h), "mspmv_csr_create");
    cache().emplace(key, h);
    return h;
}

}  // namespace mspmv_facade

template <typename Csr>
void mspmv_facade_release(const Csr &a)
{
    auto key = std::make_pair((const void *)a.values, (int)a.num_nonzeros);
    auto it = mspmv_facade::cache().find(key);
    if (it != mspmv_facade::cache().end()) {
        mspmv_destroy(it->second);
        mspmv_facade::cache().erase(it);
    }
}

// cpu_spmv.cpp:357-421
template <typename Csr, typename OffsetT, typename ValueT>
void OmpMergeCsrmv(int /*num_threads*/, Csr &a, OffsetT * /*row_end_offsets*/, OffsetT * /*column_indices*/,
                   ValueT * /*values*/, ValueT *vector_x, ValueT *vector_y_out)
{
    static_assert(sizeof(ValueT) == 8 && sizeof(OffsetT) == 4, "mspmv: CsrMatrix<double,int> only");
    mspmv_facade::check(mspmv_dspmv(mspmv_facade::handle_for(a), vector_x, vector_y_out), "mspmv_dspmv");
}

// work_2025/spmm/merge_based.hpp:46-153 (row-major n x num_vectors panels)
template <typename Csr, typename OffsetT, typename ValueT>
void OmpMergeCsrmm(int /*num_threads*/, Csr &a, OffsetT * /*row_end_offsets*/, OffsetT * /*column_indices*/,
                   ValueT * /*values*/, ValueT *vector_x, ValueT *vector_y_out, int num_vectors)
{
    static_assert(sizeof(ValueT) == 8 && sizeof(OffsetT) == 4, "mspmv: CsrMatrix<double,int> only");
    mspmv_facade::check(mspmv_dspmm(mspmv_facade::handle_for(a), vector_x, vector_y_out, num_vectors),
                        "mspmv_dspmm");
}

// work_2025/main/single_strategy.hpp:102-170
template <typename Csr, typename ValueT>
int CGSolveSingle(Csr &a, const ValueT *b, ValueT *x, int max_iters, ValueT tolerance)
{
    int iters = 0;
    mspmv_facade::check(
        mspmv_dcg_single(mspmv_facade::handle_for(a), b, x, max_iters, tolerance, &iters, nullptr, 0),
        "mspmv_dcg_single");
    return iters;
}

// work_2025/main/no_pretreatment.hpp:32-197.  kernel_type is any value convertible to int
// (the reference's SpmmKernel enum, work_2025/types.hpp:11-16).
template <typename Csr, typename ValueT, typename KernelT>
int CGSolveMultiple(Csr &a, const ValueT *B, ValueT *X, int num_vectors, int max_iters, ValueT tolerance,
                    KernelT kernel_type, std::vector<double> *max_errors = nullptr)
{
    int iters = 0;
    std::vector<double> hist(max_errors ? (size_t)max_iters : 0);
    mspmv_facade::check(mspmv_dcg_multi(mspmv_facade::handle_for(a), B, X, num_vectors, max_iters, tolerance,
                                        (mspmv_spmm_kernel)(int)kernel_type, &iters,
                                        max_errors ? hist.data() : nullptr, max_errors ? max_iters : 0),
                        "mspmv_dcg_multi");
    if (max_errors)
        max_errors->assign(hist.begin(), hist.begin() + std::min<size_t>(hist.size(), (size_t)iters));
    return iters;
}

// work_2025/cg/sparse_approximate_inversion.hpp:40-321: l receives A's pattern and the SPAI
// values (arrays allocated with new[], the reference's own non-MKL branch, :68-72).
template <typename Csr>
bool SparseApproximateInversion(const Csr &a, Csr &l)
{
    l.num_rows = a.num_rows;
    l.num_cols = a.num_cols;
    l.num_nonzeros = a.num_nonzeros;
    l.row_offsets = new int[(size_t)a.num_rows + 1];
    l.column_indices = new int[(size_t)a.num_nonzeros];
    l.values = new double[(size_t)a.num_nonzeros];
    std::copy(a.row_offsets, a.row_offsets + a.num_rows + 1, l.row_offsets);
    std::copy(a.column_indices, a.column_indices + a.num_nonzeros, l.column_indices);
    mspmv_csr_d d{a.num_rows, a.num_cols, a.num_nonzeros, a.row_offsets, a.column_indices, a.values};
    mspmv_facade::check(mspmv_spai_values(&d, l.values), "mspmv_spai_values");
    return true;
}

// work_2025/cg/incomplete_cholesky_decomp.hpp:84-201: l receives L (new[] arrays, the
// reference's non-MKL branch); false when the factorization fails after its 20 shifted attempts.
template <typename Csr>
bool IncompleteCholesky(const Csr &a, Csr &l)
{
    mspmv_csr_d d{a.num_rows, a.num_cols, a.num_nonzeros, a.row_offsets, a.column_indices, a.values};
    int nz = 0;
    mspmv_facade::check(mspmv_ic0_nnz(&d, &nz), "mspmv_ic0_nnz");
    l.num_rows = a.num_rows;
    l.num_cols = a.num_cols;
    l.num_nonzeros = nz;
    l.row_offsets = new int[(size_t)a.num_rows + 1];
    l.column_indices = new int[(size_t)std::max(nz, 1)];
    l.values = new double[(size_t)std::max(nz, 1)];
    return mspmv_ic0_factor(&d, l.row_offsets, l.column_indices, l.values, nullptr) == MSPMV_OK;
}

// work_2025/main/incomplete_cholesky.hpp:33-199 (l_transpose accepted for the signature; the
// device factor forms its own transpose).  The factor is uploaded once per L and cached.
template <typename Csr, typename ValueT, typename KernelT>
int PCGSolveMultiple(Csr &a, const Csr &l, const Csr & /*l_transpose*/, const ValueT *B, ValueT *X, int num_vectors,
                     int max_iters, ValueT tolerance, KernelT kernel_type, std::vector<double> *max_errors = nullptr)
{
    static std::map<const void *, mspmv_ic0> factors;
    mspmv_ic0 &ic = factors[(const void *)l.values];
    if (!ic) {
        mspmv_csr_d d{l.num_rows, l.num_cols, l.num_nonzeros, l.row_offsets, l.column_indices, l.values};
        mspmv_facade::check(mspmv_ic0_create(&d, 0, &ic), "mspmv_ic0_create");
    }
    int iters = 0;
    std::vector<double> hist(max_errors ? (size_t)max_iters : 0);
    mspmv_facade::check(mspmv_dpcg_ic0_multi(mspmv_facade::handle_for(a), ic, B, X, num_vectors, max_iters,
                                             tolerance, (mspmv_spmm_kernel)(int)kernel_type, &iters,
                                             max_errors ? hist.data() : nullptr, max_errors ? max_iters : 0),
                        "mspmv_dpcg_ic0_multi");
    if (max_errors)
        max_errors->assign(hist.begin(), hist.begin() + std::min<size_t>(hist.size(), (size_t)iters));
    return iters;
}

// work_2025/main/sparse_approximate_inverse.hpp:30-230
template <typename Csr, typename ValueT, typename KernelT>
int SPAISolveMultiple(Csr &a, Csr &m, const ValueT *B, ValueT *X, int num_vectors, int max_iters,
                      ValueT tolerance, KernelT kernel_type, std::vector<double> *max_errors = nullptr)
{
    int iters = 0;
    std::vector<double> hist(max_errors ? (size_t)max_iters : 0);
    mspmv_facade::check(mspmv_dpcg_spai_multi(mspmv_facade::handle_for(a), mspmv_facade::handle_for(m), B, X,
                                              num_vectors, max_iters, tolerance,
                                              (mspmv_spmm_kernel)(int)kernel_type, &iters,
                                              max_errors ? hist.data() : nullptr, max_errors ? max_iters : 0),
                        "mspmv_dpcg_spai_multi");
    if (max_errors)
        max_errors->assign(hist.begin(), hist.begin() + std::min<size_t>(hist.size(), (size_t)iters));
    return iters;
}
