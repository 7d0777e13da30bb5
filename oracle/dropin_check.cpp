// dropin_check.cpp -- TEST INFRASTRUCTURE ONLY (built by `make -C oracle dropin` where
// /root/reference exists; output oracle/_ref/dropin_check, never committed).
//
// Proves the drop-in boundary against the REAL reference container: this translation unit
// includes the reference's own sparse_matrix.h, utils.h and work_2025/hyper_parameters.hpp by
// path, then include/mspmv_dropin.hpp, then -- exactly as cpu_multicg.cpp does (:43-48) -- the
// reference's work_2025/main/*.hpp, which the drop-in has pre-guarded to nothing.  Every
// reference entry point a driver calls is then called by its reference name with a real
// CsrMatrix<double,int> built by the reference's own CooMatrix::InitGrid2d + CsrMatrix(coo)
// (sparse_matrix.h:458-531, :633-733), and checked against the reference's own CPU kernels
// SpmvGold (work_2025/spmm/sample.hpp) and OmpCsrSpmmT (work_2025/spmm/row_splitting.hpp),
// which stay un-replaced.  Exit code 0 = every check passed; 2 = a check failed; 3 = the
// library threw (e.g. no GPU: the facade has no CPU fallback).
#include "sparse_matrix.h"
#include "utils.h"
#include "work_2025/hyper_parameters.hpp"

#include "mspmv_dropin.hpp"

#include "work_2025/main/no_pretreatment.hpp"            // replaced: expands to nothing
#include "work_2025/main/single_strategy.hpp"            // replaced
#include "work_2025/main/incomplete_cholesky.hpp"        // replaced
#include "work_2025/main/sparse_approximate_inverse.hpp" // replaced
#include "work_2025/spmm/sample.hpp"                     // the reference's SpmvGold (CPU, checker)
#include "work_2025/spmm/row_splitting.hpp"              // the reference's OmpCsrSpmmT (CPU, checker)

#include <cmath>
#include <cstdio>
#include <vector>

static int g_fail = 0;

static void expect(bool ok, const char *what, double v)
{
    printf("%-34s %s (%.3g)\n", what, ok ? "ok" : "FAILED", v);
    if (!ok)
        g_fail = 1;
}

// max_j ||B_j - A X_j|| / ||B_j|| with the reference's own OmpCsrSpmmT
static double true_residual(CsrMatrix<double, int> &a, std::vector<double> &X, const std::vector<double> &B, int L)
{
    std::vector<double> AX(B.size());
    OmpCsrSpmmT(1, a, X.data(), AX.data(), L);
    double worst = 0.0;
    for (int j = 0; j < L; ++j) {
        double r = 0.0, b = 0.0;
        for (int i = 0; i < a.num_rows; ++i) {
            const double d = B[(size_t)i * L + j] - AX[(size_t)i * L + j];
            r += d * d;
            b += B[(size_t)i * L + j] * B[(size_t)i * L + j];
        }
        worst = std::max(worst, std::sqrt(r / b));
    }
    return worst;
}

int main(int argc, char **argv)
{
    g_quiet = argc < 2;  // any argument: the harnesses print the reference's progress lines
    const int width = 120;
    CooMatrix<double, int> coo;
    coo.InitGrid2d(width, true);  // 5-point grid with self loops, the reference's generator
    CsrMatrix<double, int> a(coo);
    coo.Clear();
    for (int r = 0; r < a.num_rows; ++r)  // values -> an SPD M-matrix (diagonal 4.5, neighbours -1)
        for (int k = a.row_offsets[r]; k < a.row_offsets[r + 1]; ++k)
            a.values[k] = a.column_indices[k] == r ? 4.5 : -1.0;
    const int n = a.num_rows;
    try {
        // cpu_spmv.cpp:426-475 beside the reference's SpmvGold
        std::vector<double> x(n), y0(n), yg(n), yin(n, 1.0);
        for (int i = 0; i < n; ++i)
            x[i] = 0.5 + 0.001 * (i % 97);
        SpmvGold(a, x.data(), yin.data(), y0.data(), 1.0, 0.0);
        float setup_ms = 0.f;
        const float ms = TestOmpMergeCsrmv(a, x.data(), y0.data(), yg.data(), 20, setup_ms);
        double e = 0.0;
        for (int i = 0; i < n; ++i)
            e = std::max(e, std::fabs(yg[i] - y0[i]) / (std::fabs(y0[i]) + 1e-300));
        expect(e < 1e-14 && ms > 0.f, "TestOmpMergeCsrmv vs SpmvGold", e);

        // work_2025/spmm/merge_based.hpp OmpMergeCsrmm beside the reference's OmpCsrSpmmT
        const int L = 8;
        std::vector<double> X((size_t)n * L), Y0((size_t)n * L), Yg((size_t)n * L);
        for (size_t i = 0; i < X.size(); ++i)
            X[i] = 0.25 + 0.01 * (double)(i % 101);
        OmpCsrSpmmT(g_omp_threads, a, X.data(), Y0.data(), L);
        OmpMergeCsrmm(g_omp_threads, a, a.row_offsets + 1, a.column_indices, a.values, X.data(), Yg.data(), L);
        e = 0.0;
        for (size_t i = 0; i < Y0.size(); ++i)
            e = std::max(e, std::fabs(Yg[i] - Y0[i]) / (std::fabs(Y0[i]) + 1e-300));
        expect(e < 1e-14, "OmpMergeCsrmm vs OmpCsrSpmmT", e);

        // RHS as the drivers make them (cpu_singlecg.cpp:87-92): srand(42), rand()/RAND_MAX
        srand(42);
        std::vector<double> B((size_t)n * L), XS((size_t)n * L);
        for (auto &b : B)
            b = (double)rand() / (double)RAND_MAX;
        const double tol = 1e-9;

        // single_strategy.hpp:102-240
        const int it1 = CGSolveSingle(a, B.data(), XS.data(), 5000, tol);
        double min_ms = 0, iters = 0;
        TestCGSolveSingle(a, B.data(), XS.data(), 5000, tol, 2, 2, min_ms, iters);
        expect(it1 > 0 && iters > it1 && min_ms > 0, "CGSolveSingle / TestCGSolveSingle", iters);

        // no_pretreatment.hpp:32-256, the kernel cpu_multicg.cpp:202 passes
        std::vector<double> errs;
        const int itm = CGSolveMultiple(a, B.data(), XS.data(), L, 5000, tol, SpmmKernel::NONZERO_SPLIT, &errs);
        expect(itm > 0 && (int)errs.size() == itm && errs.back() < tol && true_residual(a, XS, B, L) < 10 * tol,
               "CGSolveMultiple(NONZERO_SPLIT)", true_residual(a, XS, B, L));
        errs.clear();
        TestCGMultipleRHS(a, B.data(), XS.data(), 5000, tol, L, 2, SpmmKernel::NONZERO_SPLIT, min_ms, iters, &errs);
        expect((int)iters == itm && (int)errs.size() == itm, "TestCGMultipleRHS", iters);

        // incomplete_cholesky_decomp.hpp + incomplete_cholesky.hpp (cpu_multicg.cpp:222-250)
        CsrMatrix<double, int> Lm, Lt;
        const bool icok = IncompleteCholesky(a, Lm);
        TransposeCsr(Lm, Lt);
        bool tr_ok = Lt.num_rows == Lm.num_cols && Lt.num_nonzeros == Lm.num_nonzeros;
        for (int r = 0; tr_ok && r < Lt.num_rows; ++r)  // L^T is upper triangular with the diagonal first
            tr_ok = Lt.row_offsets[r + 1] > Lt.row_offsets[r] && Lt.column_indices[Lt.row_offsets[r]] == r;
        expect(icok && tr_ok, "IncompleteCholesky / TransposeCsr", Lm.num_nonzeros);
        errs.clear();
        const int itp = PCGSolveMultiple(a, Lm, Lt, B.data(), XS.data(), L, 5000, tol, SpmmKernel::NONZERO_SPLIT, &errs);
        expect(itp > 0 && itp < itm && true_residual(a, XS, B, L) < 10 * tol, "PCGSolveMultiple", itp);
        TestPCGMultipleRHS(a, Lm, Lt, B.data(), XS.data(), 5000, tol, L, 2, SpmmKernel::NONZERO_SPLIT, min_ms, iters,
                           &errs);
        expect((int)iters == itp, "TestPCGMultipleRHS", iters);

        // sparse_approximate_inversion.hpp + sparse_approximate_inverse.hpp (cpu_multicg.cpp:264-290)
        CsrMatrix<double, int> M;
        const bool spok = SparseApproximateInversion(a, M);
        errs.clear();
        const int its = SPAISolveMultiple(a, M, B.data(), XS.data(), L, 5000, tol, SpmmKernel::SIMPLE, &errs);
        expect(spok && its > 0 && true_residual(a, XS, B, L) < 10 * tol, "SPAISolveMultiple", its);
        TestCGMultipleSPAI(a, M, B.data(), XS.data(), 5000, tol, L, 2, SpmmKernel::SIMPLE, min_ms, iters, &errs);
        expect((int)iters == its, "TestCGMultipleSPAI", iters);
        mspmv_ref::release_all();
    } catch (const std::exception &ex) {
        printf("error: %s\n", ex.what());
        return 3;
    }
    printf("%s\n", g_fail ? "DROP-IN CHECK FAILED" : "DROP-IN CHECK PASSED");
    return g_fail ? 2 : 0;
}
