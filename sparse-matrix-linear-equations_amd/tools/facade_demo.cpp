// facade_demo -- a reference-style C++ caller using include/mspmv.hpp in namespace mode
// (`using namespace mspmv_ref`; the drop-in mode against the reference's real CsrMatrix is
// oracle/dropin_check.cpp) with unchanged call sites:
// the CsrMatrix<double,int> field layout (sparse_matrix.h:648-653), OmpMergeCsrmv /
// OmpMergeCsrmm / CGSolveSingle / CGSolveMultiple (and, at num_vectors = 32 as cpu_spmm_v2 and
// preconditioner_benchmark default, OmpMergeCsrmm, IncompleteCholesky + PCGSolveMultiple,
// SparseApproximateInversion + SPAISolveMultiple) with the reference's argument lists.
// Prints one line per call; exit code 0 when every result checks out against a host loop.
#include <cmath>
#include <cstdio>
#include <vector>

#include "mspmv.hpp"
#include "mspmv_synth.h"

template <typename ValueT, typename OffsetT>
struct CsrMatrix {  // the reference's field names and order
    OffsetT num_rows, num_cols, num_nonzeros;
    OffsetT *row_offsets, *column_indices;
    ValueT *values;
};
enum SpmmKernel { SIMPLE, MERGE, NONZERO_SPLIT };  // work_2025/types.hpp:11-16
using namespace mspmv_ref;

int main()
{
    const int m = 4000;
    std::vector<int> ro(m + 1);
    long long nnz = 0;
    if (mspmv_synth_stencil(0, m, 64, 0, 0, 7, 1e-2, ro.data(), nullptr, nullptr, &nnz) != MSPMV_OK)
        return 1;
    std::vector<int> ci(nnz);
    std::vector<double> va(nnz);
    mspmv_synth_stencil(0, m, 64, 0, 0, 7, 1e-2, ro.data(), ci.data(), va.data(), &nnz);
    CsrMatrix<double, int> a{m, m, (int)nnz, ro.data(), ci.data(), va.data()};
    std::vector<double> x(m), y(m), b(m), sol(m);
    for (int i = 0; i < m; ++i)
        x[i] = b[i] = 1.0 + (i % 7) * 0.125;
    try {
        OmpMergeCsrmv(8, a, a.row_offsets + 1, a.column_indices, a.values, x.data(), y.data());
        double err = 0;
        for (int r = 0; r < m; ++r) {
            double s = 0, ab = 0;  // error measured against sum |a_k x_k| (reordered-sum bound)
            for (int k = ro[r]; k < ro[r + 1]; ++k) {
                s += va[k] * x[ci[k]];
                ab += std::fabs(va[k] * x[ci[k]]);
            }
            err = std::max(err, std::fabs(s - y[r]) / std::max(ab, 1e-300));
        }
        printf("OmpMergeCsrmv max err relative to |A||x| %.3g\n", err);
        const int L = 4;
        std::vector<double> X((size_t)m * L, 1.0), Y((size_t)m * L), B((size_t)m * L), XS((size_t)m * L);
        OmpMergeCsrmm(8, a, a.row_offsets + 1, a.column_indices, a.values, X.data(), Y.data(), L);
        printf("OmpMergeCsrmm Y[0] %.6f\n", Y[0]);
        const int it1 = CGSolveSingle(a, b.data(), sol.data(), 5000, 1e-10);
        for (size_t i = 0; i < B.size(); ++i)
            B[i] = b[i / L] * (1 + (int)(i % L));
        std::vector<double> errs;
        const int itm = CGSolveMultiple(a, B.data(), XS.data(), L, 5000, 1e-10, NONZERO_SPLIT, &errs);
        printf("CGSolveSingle %d iters, CGSolveMultiple %d iters (last max err %.3g)\n", it1, itm,
               errs.empty() ? -1.0 : errs.back());
        // num_vectors = 32: column chunks of the native widths over the same row-major panels
        const int L32 = 32;
        std::vector<double> X32((size_t)m * L32), Y32((size_t)m * L32), B32((size_t)m * L32), S32((size_t)m * L32);
        for (size_t i = 0; i < X32.size(); ++i)
            X32[i] = B32[i] = 0.5 + (double)((i * 2654435761u) % 1000) / 1000.0;
        OmpMergeCsrmm(8, a, a.row_offsets + 1, a.column_indices, a.values, X32.data(), Y32.data(), L32);
        double err32 = 0;
        for (int r = 0; r < m; ++r)
            for (int j = 0; j < L32; ++j) {
                double s = 0, ab = 0;
                for (int k = ro[r]; k < ro[r + 1]; ++k) {
                    s += va[k] * X32[(size_t)ci[k] * L32 + j];
                    ab += std::fabs(va[k] * X32[(size_t)ci[k] * L32 + j]);
                }
                err32 = std::max(err32, std::fabs(s - Y32[(size_t)r * L32 + j]) / std::max(ab, 1e-300));
            }
        printf("OmpMergeCsrmm num_vectors=32 max err relative to |A||X| %.3g\n", err32);
        CsrMatrix<double, int> l{}, mi{};
        const bool icok = IncompleteCholesky(a, l);
        std::vector<double> e_ic, e_spai;
        const int itic = icok ? PCGSolveMultiple(a, l, l, B32.data(), S32.data(), L32, 5000, 1e-10, MERGE, &e_ic) : -1;
        const bool spok = SparseApproximateInversion(a, mi);
        const int itsp = spok ? SPAISolveMultiple(a, mi, B32.data(), S32.data(), L32, 5000, 1e-10, MERGE, &e_spai) : -1;
        printf("IncompleteCholesky %d, PCGSolveMultiple(32) %d iters; SparseApproximateInversion %d, "
               "SPAISolveMultiple(32) %d iters\n", (int)icok, itic, (int)spok, itsp);
        for (auto *c : {&l, &mi}) {
            delete[] c->row_offsets;
            delete[] c->column_indices;
            delete[] c->values;
        }
        release(mi);
        release(a);
        const bool ok32 = err32 < 1e-12 && itic > 0 && itsp > 0 && !e_ic.empty() && e_ic.back() < 1e-10 &&
                          !e_spai.empty() && e_spai.back() < 1e-10;
        return (err < 1e-12 && it1 > 0 && itm > 0 && !errs.empty() && errs.back() < 1e-10 && ok32) ? 0 : 2;
    } catch (const std::exception &e) {
        printf("error: %s\n", e.what());
        return 3;
    }
}
