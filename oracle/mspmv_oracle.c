/*
 * mspmv_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C (C11 + OpenMP) restatement of the reference's hot path:
 *   merge-path CSR SpMV / SpMM (fp64, int32 indices) and the CG solvers built on them.
 * Every function cites the reference file:line it follows (paths relative to the
 * reference checkout, YuyaW-0118/Sparse-Matrix-Linear-Equations).
 *
 * Who may load this library: tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg -- and there only as the checker / the timed CPU baseline.
 * The product library (libmspmv.so) neither links nor calls anything here.
 *
 * Pinning: tests/test_oracle_pinning.py checks these functions against golden
 * vectors produced by the reference's own code (oracle/ref_harness.cpp compiled
 * from /root/reference by oracle/Makefile, outputs in tests/golden/).  The CG
 * loops live in headers that include <mkl.h> (single_strategy.hpp:13,
 * no_pretreatment.hpp:17, utils_multiple.hpp:5), which this image lacks, so they
 * cannot be built here; their SpMV/SpMM building blocks are pinned and the loop is
 * a line-by-line restatement ("Parity").
 *
 * Floating point: compiled with -ffp-contract=off, so every a*b+c is two roundings
 * exactly as in the reference built without FMA (x86-64 baseline ISA).
 */
#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EXPORT __attribute__((visibility("default")))

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

/* ------------------------------------------------------------------------- */
/* Merge-path search.  cpu_spmv.cpp:208-235 (byte-identical twin:            */
/* work_2025/spmm/merge_based.hpp:17-44).  List A = row end offsets          */
/* (row_offsets + 1), list B = the counting sequence 0..nnz-1                */
/* (CountingInputIterator, cpu_spmv.cpp:87-199), so b[k] == k.               */
/* ------------------------------------------------------------------------- */
ORC_EXPORT void orc_merge_path_search(int diagonal, const int *row_end_offsets, int a_len, int b_len,
                                      int *out_x, int *out_y)
{
    int x_min = imax(diagonal - b_len, 0);
    int x_max = imin(diagonal, a_len);
    while (x_min < x_max) {
        int x_pivot = (x_min + x_max) >> 1;
        if (row_end_offsets[x_pivot] <= diagonal - x_pivot - 1)
            x_min = x_pivot + 1;
        else
            x_max = x_pivot;
    }
    *out_x = imin(x_min, a_len);
    *out_y = diagonal - x_min;
}

/* Coordinates of the P+1 partition boundaries used by OmpMergeCsrmv:
 * items_per_thread = ceil((m+nnz)/P), start_diagonal = min(ipt*t, m+nnz)
 * (cpu_spmv.cpp:379-386; merge_based.hpp:72-80).  coords[2t]=row, coords[2t+1]=nnz. */
ORC_EXPORT void orc_merge_coords(const int *row_offsets, int num_rows, int num_nonzeros, int num_parts,
                                 int *coords)
{
    int total = num_rows + num_nonzeros;
    int ipt = (total + num_parts - 1) / num_parts;
    for (int t = 0; t <= num_parts; ++t) {
        long long d = (long long)ipt * t;
        int diag = (int)(d < total ? d : total);
        orc_merge_path_search(diag, row_offsets + 1, num_rows, num_nonzeros, &coords[2 * t], &coords[2 * t + 1]);
    }
}

/* ------------------------------------------------------------------------- */
/* SpmvGold: cpu_spmv.cpp:241-265 (twin work_2025/spmm/sample.hpp:11-34).    */
/* ------------------------------------------------------------------------- */
ORC_EXPORT void orc_spmv_gold(int num_rows, const int *row_offsets, const int *cols, const double *vals,
                              const double *x, const double *y_in, double *y_out, double alpha, double beta)
{
    for (int row = 0; row < num_rows; ++row) {
        double partial = beta * y_in[row];
        for (int off = row_offsets[row]; off < row_offsets[row + 1]; ++off)
            partial += alpha * vals[off] * x[cols[off]];
        y_out[row] = partial;
    }
}

/* Row-split CsrMV: cpu_spmv.cpp:271-294 (also the CG's OmpCsrSpmv,
 * work_2025/main/single_strategy.hpp:28-55, whose `omp simd reduction` may reorder
 * a row's sum; this restatement sums each row in CSR order). */
ORC_EXPORT void orc_csr_spmv(int num_rows, const int *row_offsets, const int *cols, const double *vals,
                             const double *x, double *y)
{
#pragma omp parallel for schedule(static)
    for (int row = 0; row < num_rows; ++row) {
        double partial = 0.0;
        for (int off = row_offsets[row]; off < row_offsets[row + 1]; ++off)
            partial += vals[off] * x[cols[off]];
        y[row] = partial;
    }
}

/* ------------------------------------------------------------------------- */
/* OmpMergeCsrmv: cpu_spmv.cpp:357-421.                                      */
/* ------------------------------------------------------------------------- */
ORC_EXPORT void orc_merge_csrmv(int num_threads, int num_rows, int num_nonzeros, const int *row_offsets,
                                const int *cols, const double *vals, const double *x, double *y)
{
    const int *row_end = row_offsets + 1;
    int *row_carry_out = (int *)malloc(sizeof(int) * num_threads);
    double *value_carry_out = (double *)malloc(sizeof(double) * num_threads);

#pragma omp parallel for schedule(static) num_threads(num_threads)
    for (int tid = 0; tid < num_threads; tid++) {
        int num_merge_items = num_rows + num_nonzeros;
        int items_per_thread = (num_merge_items + num_threads - 1) / num_threads;
        int start_diagonal = imin(items_per_thread * tid, num_merge_items);
        int end_diagonal = imin(start_diagonal + items_per_thread, num_merge_items);
        int cx, cy, ex, ey;
        orc_merge_path_search(start_diagonal, row_end, num_rows, num_nonzeros, &cx, &cy);
        orc_merge_path_search(end_diagonal, row_end, num_rows, num_nonzeros, &ex, &ey);

        for (; cx < ex; ++cx) { /* whole rows, :392-401 */
            double running_total = 0.0;
            for (; cy < row_end[cx]; ++cy)
                running_total += vals[cy] * x[cols[cy]];
            y[cx] = running_total;
        }
        double running_total = 0.0; /* partial last row, :404-408 */
        for (; cy < ey; ++cy)
            running_total += vals[cy] * x[cols[cy]];
        row_carry_out[tid] = ex; /* :411-412 */
        value_carry_out[tid] = running_total;
    }
    for (int tid = 0; tid < num_threads - 1; ++tid) /* serial fix-up, :416-420 */
        if (row_carry_out[tid] < num_rows)
            y[row_carry_out[tid]] += value_carry_out[tid];
    free(row_carry_out);
    free(value_carry_out);
}

/* ------------------------------------------------------------------------- */
/* OmpMergeCsrmm (the correct SpMM used by the CG): merge_based.hpp:46-153.  */
/* X is n x L row-major (X[c*L+j]), Y is m x L row-major.                    */
/* ------------------------------------------------------------------------- */
ORC_EXPORT void orc_merge_csrmm(int num_threads, int num_rows, int num_nonzeros, const int *row_offsets,
                                const int *cols, const double *vals, const double *X, double *Y, int L)
{
    const int *row_end = row_offsets + 1;
    int *row_carry_out = (int *)malloc(sizeof(int) * num_threads);
    double *value_carry_out = (double *)malloc(sizeof(double) * (size_t)num_threads * L);

#pragma omp parallel for schedule(static) num_threads(num_threads)
    for (int tid = 0; tid < num_threads; tid++) {
        int num_merge_items = num_rows + num_nonzeros;
        int items_per_thread = (num_merge_items + num_threads - 1) / num_threads;
        int start_diagonal = imin(items_per_thread * tid, num_merge_items);
        int end_diagonal = imin(start_diagonal + items_per_thread, num_merge_items);
        int cx, cy, ex, ey;
        orc_merge_path_search(start_diagonal, row_end, num_rows, num_nonzeros, &cx, &cy);
        orc_merge_path_search(end_diagonal, row_end, num_rows, num_nonzeros, &ex, &ey);

        double *running_total = (double *)malloc(sizeof(double) * L);
        for (int i = 0; i < L; i++)
            running_total[i] = 0.0;
        for (; cx < ex; ++cx) { /* :92-117 */
            for (; cy < row_end[cx]; ++cy) {
                double val = vals[cy];
                const double *tmp = X + (size_t)cols[cy] * L;
                for (int i = 0; i < L; i++)
                    running_total[i] += val * tmp[i];
            }
            double *out = Y + (size_t)cx * L;
            for (int i = 0; i < L; i++) {
                out[i] = running_total[i];
                running_total[i] = 0.0;
            }
        }
        for (; cy < ey; ++cy) { /* :120-129 */
            double val = vals[cy];
            const double *tmp = X + (size_t)cols[cy] * L;
            for (int i = 0; i < L; i++)
                running_total[i] += val * tmp[i];
        }
        row_carry_out[tid] = ex; /* :132-135 */
        for (int i = 0; i < L; i++)
            value_carry_out[(size_t)tid * L + i] = running_total[i];
        free(running_total);
    }
    for (int tid = 0; tid < num_threads; ++tid) { /* fix-up over all t, :138-149 */
        int row_idx = row_carry_out[tid];
        if (row_idx < num_rows)
            for (int i = 0; i < L; i++)
                Y[(size_t)row_idx * L + i] += value_carry_out[(size_t)tid * L + i];
    }
    free(row_carry_out);
    free(value_carry_out);
}

/* Row-split SpMM: work_2025/spmm/row_splitting.hpp:15-54. */
ORC_EXPORT void orc_csr_spmm_t(int num_rows, const int *row_offsets, const int *cols, const double *vals,
                               const double *X, double *Y, int L)
{
#pragma omp parallel for schedule(static)
    for (int row = 0; row < num_rows; ++row) {
        double *row_sum = Y + (size_t)row * L;
        double acc[64];
        double *s = L <= 64 ? acc : (double *)malloc(sizeof(double) * L);
        for (int i = 0; i < L; i++)
            s[i] = 0.0;
        for (int off = row_offsets[row]; off < row_offsets[row + 1]; ++off) {
            double val = vals[off];
            const double *xr = X + (size_t)cols[off] * L;
            for (int i = 0; i < L; i++)
                s[i] += val * xr[i];
        }
        for (int i = 0; i < L; i++)
            row_sum[i] = s[i];
        if (s != acc)
            free(s);
    }
}

/* RowPathSearch: work_2025/spmm/nonzero_splitting.hpp:14-44. */
static void orc_row_path_search(const int *row_end, int a_len, int y, int *out_x)
{
    if (y == 0) {
        *out_x = 0;
        return;
    }
    int x_min = 0, x_max = a_len;
    while (x_min < x_max) {
        int x_pivot = (x_min + x_max) >> 1;
        if (row_end[x_pivot] <= y - 1)
            x_min = x_pivot + 1;
        else
            x_max = x_pivot;
    }
    *out_x = imin(x_min, a_len);
}

/* OmpNonzeroSplitCsrmm: work_2025/spmm/nonzero_splitting.hpp:49-150.  Restated
 * faithfully, including its precondition that Y is pre-zeroed (the last nonempty
 * row and trailing empty rows only receive the `+=` of the carry fix-up;
 * CGSolveMultiple masks this with memset(AP, 0), no_pretreatment.hpp:93). */
static void nonzero_split(int num_threads, int num_rows, int num_nonzeros, const int *row_offsets, const int *cols,
                          const double *vals, const double *X, double *Y, int L, int fixup_threads)
{
    const int *row_end = row_offsets + 1;
    int *row_carry_out = (int *)malloc(sizeof(int) * num_threads);
    double *value_carry_out = (double *)malloc(sizeof(double) * (size_t)num_threads * L);

#pragma omp parallel for schedule(static) num_threads(num_threads)
    for (int tid = 0; tid < num_threads; tid++) {
        int items_per_thread = (num_nonzeros + num_threads - 1) / num_threads;
        int cy = imin(items_per_thread * tid, num_nonzeros);
        int ey = imin(cy + items_per_thread, num_nonzeros);
        int cx, ex;
        orc_row_path_search(row_end, num_rows, cy, &cx);
        orc_row_path_search(row_end, num_rows, ey, &ex);

        double *running_total = (double *)calloc((size_t)L, sizeof(double));
        for (; cx < ex; ++cx) {
            for (; cy < row_end[cx]; ++cy) {
                double val = vals[cy];
                const double *tmp = X + (size_t)cols[cy] * L;
                for (int i = 0; i < L; i++)
                    running_total[i] += val * tmp[i];
            }
            double *out = Y + (size_t)cx * L;
            for (int i = 0; i < L; i++) {
                out[i] = running_total[i];
                running_total[i] = 0.0;
            }
        }
        for (; cy < ey; ++cy) {
            double val = vals[cy];
            const double *tmp = X + (size_t)cols[cy] * L;
            for (int i = 0; i < L; i++)
                running_total[i] += val * tmp[i];
        }
        row_carry_out[tid] = ex;
        for (int i = 0; i < L; i++)
            value_carry_out[(size_t)tid * L + i] = running_total[i];
        free(running_total);
    }
    for (int tid = 0; tid < fixup_threads; ++tid) {
        int row_idx = row_carry_out[tid];
        if (row_idx < num_rows)
            for (int i = 0; i < L; i++)
                Y[(size_t)row_idx * L + i] += value_carry_out[(size_t)tid * L + i];
    }
    free(row_carry_out);
    free(value_carry_out);
}

ORC_EXPORT void orc_nonzero_split_csrmm(int num_threads, int num_rows, int num_nonzeros, const int *row_offsets,
                                        const int *cols, const double *vals, const double *X, double *Y, int L)
{
    nonzero_split(num_threads, num_rows, num_nonzeros, row_offsets, cols, vals, X, Y, L, num_threads);
}

/* The older single-vector twin, cpu_spmv.cpp:476-570 (RowPathSearch :476-500, OmpNonzeroSplitCsrmm
 * :506-570): the same partition and loops at L = 1, but its fix-up stops before the last thread
 * (`tid < num_threads - 1`, :564), so the last thread's carry is dropped.  Rows before the last
 * nonempty row r* come out as in the work_2025 twin; y[r*] = (its prior content) + the carries of
 * the earlier threads that ended inside r*; rows after r* keep their prior content.  y is in/out.
 * The fixed carry arrays (`row_carry_out[256]`, :513-514) limit it to 256 threads.
 * cpu_spmv.cpp includes <mkl.h> (:59), so it is not compiled here: this restatement is checked
 * against the compiled work_2025 twin (tests/test_oracle_pinning.py), whose only textual
 * difference is that fix-up bound. */
ORC_EXPORT int orc_nonzero_split_csrmv_v1(int num_threads, int num_rows, int num_nonzeros, const int *row_offsets,
                                          const int *cols, const double *vals, const double *x, double *y)
{
    if (num_threads < 1 || num_threads > 256)
        return -1;
    nonzero_split(num_threads, num_rows, num_nonzeros, row_offsets, cols, vals, x, y, 1, num_threads - 1);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* BLAS-1 used by the single-RHS CG: single_strategy.hpp:60-97.              */
/* ------------------------------------------------------------------------- */
static double dot_single(int n, const double *x, const double *y)
{
    double result = 0.0;
#pragma omp parallel for reduction(+ : result)
    for (int i = 0; i < n; ++i)
        result += x[i] * y[i];
    return result;
}

static void axpy_single(int n, double a, const double *x, double *y)
{
#pragma omp parallel for simd
    for (int i = 0; i < n; ++i)
        y[i] += a * x[i];
}

static void update_p_single(int n, const double *r, double beta, double *p)
{
#pragma omp parallel for simd
    for (int i = 0; i < n; ++i)
        p[i] = r[i] + beta * p[i];
}

/* CGSolveSingle: single_strategy.hpp:102-170.  `resid_hist[k]` (optional,
 * capacity hist_cap) receives sqrt(rs_new)/b_norm of iteration k -- the quantity
 * the stop rule tests at :152; recording it does not change the recurrence. */
ORC_EXPORT int orc_cg_single(int num_rows, const int *row_offsets, const int *cols, const double *vals,
                             const double *b, double *x, int max_iters, double tolerance, double *resid_hist,
                             int hist_cap)
{
    int n = num_rows;
    double *r = (double *)malloc(sizeof(double) * n);
    double *p = (double *)malloc(sizeof(double) * n);
    double *Ap = (double *)malloc(sizeof(double) * n);
#pragma omp parallel for simd
    for (int i = 0; i < n; ++i) { /* :120-126 */
        x[i] = 0.0;
        r[i] = b[i];
        p[i] = b[i];
    }
    double rs_old = dot_single(n, r, r);         /* :128 */
    double b_norm = sqrt(dot_single(n, b, b));   /* :129 */
    if (b_norm == 0.0)
        b_norm = 1.0;
    int iter = 0;
    for (; iter < max_iters; ++iter) {
        orc_csr_spmv(n, row_offsets, cols, vals, p, Ap);   /* :137 */
        double pAp = dot_single(n, p, Ap);                 /* :140 */
        double alpha = rs_old / pAp;
        axpy_single(n, alpha, p, x);                       /* :144 */
        axpy_single(n, -alpha, Ap, r);                     /* :147 */
        double rs_new = dot_single(n, r, r);               /* :149 */
        double rel = sqrt(rs_new) / b_norm;
        if (resid_hist && iter < hist_cap)
            resid_hist[iter] = rel;
        if (rel < tolerance) { /* :152-156 */
            iter++;
            break;
        }
        double beta = rs_new / rs_old;                     /* :159-160 */
        update_p_single(n, r, beta, p);
        rs_old = rs_new;
    }
    free(r);
    free(p);
    free(Ap);
    return iter;
}

/* ------------------------------------------------------------------------- */
/* Multi-RHS BLAS-1: work_2025/cg/utils_multiple.hpp:8-59 (interleaved n x L) */
/* ------------------------------------------------------------------------- */
static void dot_multiple(int n, int L, const double *x, const double *y, double *result)
{
    for (int i = 0; i < L; i++)
        result[i] = 0.0;
#pragma omp parallel for reduction(+ : result[0 : L])
    for (int j = 0; j < n; ++j) {
        const double *xr = x + (size_t)j * L;
        const double *yr = y + (size_t)j * L;
        for (int i = 0; i < L; ++i)
            result[i] += xr[i] * yr[i];
    }
}

static void axpy_multiple(int n, int L, const double *a, const double *x, double *y)
{
#pragma omp parallel for
    for (int j = 0; j < n; ++j) {
        double *yr = y + (size_t)j * L;
        const double *xr = x + (size_t)j * L;
        for (int i = 0; i < L; ++i)
            yr[i] += a[i] * xr[i];
    }
}

static void update_p_multiple(int n, int L, const double *r, const double *beta, double *p)
{
#pragma omp parallel for
    for (int j = 0; j < n; ++j) {
        const double *rr = r + (size_t)j * L;
        double *pr = p + (size_t)j * L;
        for (int i = 0; i < L; ++i)
            pr[i] = rr[i] + beta[i] * pr[i];
    }
}

/* SpmmKernel: work_2025/types.hpp:11-16. */
enum { ORC_SIMPLE = 0, ORC_MERGE = 1, ORC_NONZERO_SPLIT = 2 };

/* CGSolveMultiple: work_2025/main/no_pretreatment.hpp:32-197.  `num_threads`
 * plays g_omp_threads (hyper_parameters.hpp:11; the merge/nonzero partition count).
 * max_err_hist[k] = max over ALL columns of sqrt(rs_new)/b_norm (:132-155). */
ORC_EXPORT int orc_cg_multi(int num_rows, int num_nonzeros, const int *row_offsets, const int *cols,
                            const double *vals, const double *B, double *X, int L, int max_iters, double tolerance,
                            int kernel_type, int num_threads, double *max_err_hist, int hist_cap)
{
    int n = num_rows;
    size_t nl = (size_t)n * L;
    double *R = (double *)malloc(sizeof(double) * nl);
    double *P = (double *)malloc(sizeof(double) * nl);
    double *AP = (double *)malloc(sizeof(double) * nl);
    double *alpha = (double *)malloc(sizeof(double) * L);
    double *beta = (double *)malloc(sizeof(double) * L);
    double *rs_old = (double *)malloc(sizeof(double) * L);
    double *rs_new = (double *)malloc(sizeof(double) * L);
    double *pAp = (double *)malloc(sizeof(double) * L);
    double *b_norms = (double *)malloc(sizeof(double) * L);
    char *converged = (char *)malloc(L);

#pragma omp parallel for
    for (long long i = 0; i < (long long)nl; ++i) { /* :61-67 */
        X[i] = 0.0;
        R[i] = B[i];
        P[i] = B[i];
    }
    dot_multiple(n, L, B, B, b_norms); /* :69-77 */
    for (int i = 0; i < L; ++i) {
        b_norms[i] = sqrt(b_norms[i]);
        if (b_norms[i] == 0.0)
            b_norms[i] = 1.0;
        converged[i] = 0;
    }
    dot_multiple(n, L, R, R, rs_old); /* :79 */

    int iter;
    for (iter = 0; iter < max_iters; ++iter) {
        memset(AP, 0, sizeof(double) * nl); /* :93 */
        switch (kernel_type) {              /* :94-105 */
        case ORC_SIMPLE:
            orc_csr_spmm_t(n, row_offsets, cols, vals, P, AP, L);
            break;
        case ORC_MERGE:
            orc_merge_csrmm(num_threads, n, num_nonzeros, row_offsets, cols, vals, P, AP, L);
            break;
        default:
            orc_nonzero_split_csrmm(num_threads, n, num_nonzeros, row_offsets, cols, vals, P, AP, L);
            break;
        }
        dot_multiple(n, L, P, AP, pAp); /* :107 */
        for (int i = 0; i < L; ++i)     /* :109-120 */
            alpha[i] = converged[i] ? 0.0 : rs_old[i] / pAp[i];
        axpy_multiple(n, L, alpha, P, X); /* :123 */
        for (int i = 0; i < L; ++i)
            alpha[i] = -alpha[i];
        axpy_multiple(n, L, alpha, AP, R); /* :128 */
        dot_multiple(n, L, R, R, rs_new);  /* :130 */

        int num_converged = 0;             /* :132-155 */
        double max_relative_error = 0.0;
        for (int i = 0; i < L; ++i) {
            double rel_error = sqrt(rs_new[i]) / b_norms[i];
            /* std::max(max, rel) = (max < rel) ? rel : max: a NaN rel is skipped */
            max_relative_error = max_relative_error < rel_error ? rel_error : max_relative_error;
            if (!converged[i] && rel_error < tolerance)
                converged[i] = 1;
            if (converged[i])
                num_converged++;
        }
        if (max_err_hist && iter < hist_cap)
            max_err_hist[iter] = max_relative_error;
        if (num_converged == L) { /* :157-161 */
            iter++;
            break;
        }
        for (int i = 0; i < L; ++i) /* :163-176 */
            beta[i] = converged[i] ? 0.0 : rs_new[i] / rs_old[i];
        update_p_multiple(n, L, R, beta, P); /* :177 */
        for (int i = 0; i < L; ++i)
            rs_old[i] = rs_new[i];
    }
    free(R); free(P); free(AP); free(alpha); free(beta);
    free(rs_old); free(rs_new); free(pAp); free(b_norms); free(converged);
    return iter;
}

/* SPAISolveMultiple: work_2025/main/sparse_approximate_inverse.hpp:30-230.  M shares A's
 * pattern (SparseApproximateInversion's static pattern), so only its values m_vals are passed.
 * Z = M R and A P run through the same SpmmKernel dispatch as the reference (:81-92, :114-125,
 * :184-195). */
static void spmm_dispatch(int kernel_type, int num_threads, int n, int nnz, const int *row_offsets, const int *cols,
                          const double *vals, const double *X, double *Y, int L)
{
    switch (kernel_type) {
    case ORC_SIMPLE:
        orc_csr_spmm_t(n, row_offsets, cols, vals, X, Y, L);
        break;
    case ORC_MERGE:
        orc_merge_csrmm(num_threads, n, nnz, row_offsets, cols, vals, X, Y, L);
        break;
    default:
        orc_nonzero_split_csrmm(num_threads, n, nnz, row_offsets, cols, vals, X, Y, L);
        break;
    }
}

ORC_EXPORT int orc_pcg_spai_multi(int num_rows, int num_nonzeros, const int *row_offsets, const int *cols,
                                  const double *vals, const double *m_vals, const double *B, double *X, int L,
                                  int max_iters, double tolerance, int kernel_type, int num_threads,
                                  double *max_err_hist, int hist_cap)
{
    int n = num_rows;
    size_t nl = (size_t)n * L;
    double *R = (double *)malloc(sizeof(double) * nl);
    double *P = (double *)malloc(sizeof(double) * nl);
    double *AP = (double *)malloc(sizeof(double) * nl);
    double *Z = (double *)malloc(sizeof(double) * nl);
    double *alpha = (double *)malloc(sizeof(double) * L);
    double *beta = (double *)malloc(sizeof(double) * L);
    double *rs_old = (double *)malloc(sizeof(double) * L);
    double *rs_new = (double *)malloc(sizeof(double) * L);
    double *pAp = (double *)malloc(sizeof(double) * L);
    double *b_norms = (double *)malloc(sizeof(double) * L);
    char *converged = (char *)malloc(L);

    for (size_t i = 0; i < nl; ++i) { /* :59-67 */
        X[i] = 0.0;
        R[i] = B[i];
        P[i] = 0.0;
        Z[i] = 0.0;
    }
    dot_multiple(n, L, B, B, b_norms); /* :69-78 */
    for (int i = 0; i < L; ++i) {
        b_norms[i] = sqrt(b_norms[i]);
        if (b_norms[i] == 0.0)
            b_norms[i] = 1.0;
        converged[i] = 0;
    }
    memset(Z, 0, sizeof(double) * nl);
    spmm_dispatch(kernel_type, num_threads, n, num_nonzeros, row_offsets, cols, m_vals, R, Z, L); /* :80-92 */
    for (size_t i = 0; i < nl; ++i)                                                              /* :94-97 */
        P[i] = Z[i];
    dot_multiple(n, L, R, Z, rs_old); /* :99-100 */

    int iter;
    for (iter = 0; iter < max_iters; ++iter) {
        memset(AP, 0, sizeof(double) * nl);
        spmm_dispatch(kernel_type, num_threads, n, num_nonzeros, row_offsets, cols, vals, P, AP, L); /* :111-125 */
        dot_multiple(n, L, P, AP, pAp);                                                           /* :127-128 */
        for (int i = 0; i < L; ++i)                                                               /* :130-138 */
            alpha[i] = (!converged[i] && pAp[i] != 0.0) ? rs_old[i] / pAp[i] : 0.0;
        axpy_multiple(n, L, alpha, P, X); /* :140-141 */
        for (int i = 0; i < L; ++i)
            alpha[i] = -alpha[i];
        axpy_multiple(n, L, alpha, AP, R); /* :143-149 */
        dot_multiple(n, L, R, R, pAp);     /* :151-153 */
        int num_converged = 0;             /* :155-169 */
        double max_relative_error = 0.0;
        for (int i = 0; i < L; ++i) {
            double rel_error = sqrt(pAp[i]) / b_norms[i];
            /* std::max(max, rel) = (max < rel) ? rel : max: a NaN rel is skipped */
            max_relative_error = max_relative_error < rel_error ? rel_error : max_relative_error;
            if (!converged[i] && rel_error < tolerance)
                converged[i] = 1;
            if (converged[i])
                num_converged++;
        }
        if (max_err_hist && iter < hist_cap) /* :171-175 */
            max_err_hist[iter] = max_relative_error;
        if (num_converged == L) { /* :177-181 */
            iter++;
            break;
        }
        memset(Z, 0, sizeof(double) * nl);
        spmm_dispatch(kernel_type, num_threads, n, num_nonzeros, row_offsets, cols, m_vals, R, Z, L); /* :183-195 */
        dot_multiple(n, L, R, Z, rs_new);                                                            /* :197-198 */
        for (int i = 0; i < L; ++i) {                                                                /* :200-210 */
            beta[i] = (!converged[i] && rs_old[i] != 0.0) ? rs_new[i] / rs_old[i] : 0.0;
            rs_old[i] = rs_new[i];
        }
        update_p_multiple(n, L, Z, beta, P); /* :212-214 */
    }
    free(R); free(P); free(AP); free(Z); free(alpha); free(beta);
    free(rs_old); free(rs_new); free(pAp); free(b_norms); free(converged);
    return iter;
}

/* ------------------------------------------------------------------------- */
/* IC(0): work_2025/cg/incomplete_cholesky_decomp.hpp (the file includes      */
/* <mkl.h>, so it is restated, not built) and PCGSolveMultiple,               */
/* work_2025/main/incomplete_cholesky.hpp:33-199.                             */
/* ------------------------------------------------------------------------- */
/* IncompleteCholesky :84-201.  l_* receive L (A's lower triangle, A's order); returns 1 on
 * success (after at most 20 shifted attempts), 0 on failure; *shift_out the shift used. */
ORC_EXPORT int orc_ic0_factor(int n, const int *ro, const int *ci, const double *va, int *l_ro, int *l_ci,
                              double *l_va, double *shift_out)
{
    int nz = 0;
    l_ro[0] = 0;
    for (int i = 0; i < n; ++i) { /* :91-148 */
        for (int k = ro[i]; k < ro[i + 1]; ++k)
            if (ci[k] <= i) {
                l_ci[nz] = ci[k];
                l_va[nz] = va[k];
                ++nz;
            }
        l_ro[i + 1] = nz;
    }
    double *backup = (double *)malloc(sizeof(double) * (nz > 0 ? nz : 1));
    memcpy(backup, l_va, sizeof(double) * nz);
    double shift = 0.0;
    for (int retry = 0; retry < 20; ++retry) { /* :150-225 */
        int failed = 0;
        if (retry > 0)
            for (int idx = 0; idx < n; ++idx)
                for (int off = l_ro[idx]; off < l_ro[idx + 1]; ++off) {
                    l_va[off] = backup[off];
                    if (l_ci[off] == idx)
                        l_va[off] += shift;
                }
        for (int i = 0; i < n && !failed; ++i) {
            for (int ko = l_ro[i]; ko < l_ro[i + 1]; ++ko) {
                int k = l_ci[ko];
                double sum = 0.0;
                int jl = l_ro[i], jk = l_ro[k];
                while (jl < ko && jk < l_ro[k + 1]) {
                    if (l_ci[jl] == l_ci[jk]) {
                        sum += l_va[jl] * l_va[jk];
                        jl++;
                        jk++;
                    } else if (l_ci[jl] < l_ci[jk]) {
                        jl++;
                    } else {
                        jk++;
                    }
                }
                l_va[ko] -= sum;
                if (k == i) {
                    if (l_va[ko] <= 0) {
                        failed = 1;
                        break;
                    }
                    l_va[ko] = sqrt(l_va[ko]);
                } else {
                    l_va[ko] /= l_va[l_ro[k + 1] - 1];
                }
            }
        }
        if (!failed) {
            free(backup);
            if (shift_out)
                *shift_out = shift;
            return 1;
        }
        shift = shift == 0.0 ? 1e-3 : shift * 10.0;
    }
    free(backup);
    return 0;
}

/* TransposeCsr :11-78 (counting sort by column; rows in order within each output row). */
static void transpose_csr(int n, int nnz, const int *ro, const int *ci, const double *va, int *t_ro, int *t_ci,
                          double *t_va)
{
    int *cnt = (int *)calloc((size_t)n + 1, sizeof(int));
    for (int k = 0; k < nnz; ++k)
        cnt[ci[k] + 1]++;
    for (int c = 0; c < n; ++c)
        cnt[c + 1] += cnt[c];
    memcpy(t_ro, cnt, sizeof(int) * ((size_t)n + 1));
    for (int r = 0; r < n; ++r)
        for (int k = ro[r]; k < ro[r + 1]; ++k) {
            int d = cnt[ci[k]]++;
            t_ci[d] = r;
            t_va[d] = va[k];
        }
    free(cnt);
}

/* ForwardSolveMultiple :231-271 and BackwardSolveMultiple :277-346 (sequential, CSR order). */
static void forward_solve_multiple(int n, const int *ro, const int *ci, const double *va, const double *b, double *x,
                                   int L, double *sum)
{
    for (int i = 0; i < n; ++i) {
        for (int v = 0; v < L; ++v)
            sum[v] = 0.0;
        int diag_offset = 0;
        for (int k = ro[i]; k < ro[i + 1]; ++k) {
            int j = ci[k];
            if (i == j) {
                diag_offset = k;
                continue;
            }
            for (int v = 0; v < L; ++v)
                sum[v] += va[k] * x[(size_t)j * L + v];
        }
        double d = va[diag_offset];
        for (int v = 0; v < L; ++v)
            x[(size_t)i * L + v] = (b[(size_t)i * L + v] - sum[v]) / d;
    }
}

static void backward_solve_multiple(int n, const int *ro, const int *ci, const double *va, const double *b, double *x,
                                    int L, double *sum)
{
    for (int i = n - 1; i >= 0; --i) {
        for (int v = 0; v < L; ++v)
            sum[v] = 0.0;
        double d = 0.0;
        for (int k = ro[i]; k < ro[i + 1]; ++k) {
            int j = ci[k];
            if (i == j) {
                d = va[k];
                continue;
            }
            for (int v = 0; v < L; ++v)
                sum[v] += va[k] * x[(size_t)j * L + v];
        }
        for (int v = 0; v < L; ++v)
            x[(size_t)i * L + v] = d == 0.0 ? 0.0 : (b[(size_t)i * L + v] - sum[v]) / d;
    }
}

/* PCGSolveMultiple :33-199 with the factor L (l_*); L^T is formed here as the driver does. */
ORC_EXPORT int orc_pcg_ic0_multi(int num_rows, int num_nonzeros, const int *row_offsets, const int *cols,
                                 const double *vals, int l_nnz, const int *l_ro, const int *l_ci, const double *l_va,
                                 const double *B, double *X, int L, int max_iters, double tolerance, int kernel_type,
                                 int num_threads, double *max_err_hist, int hist_cap)
{
    int n = num_rows;
    size_t nl = (size_t)n * L;
    int *t_ro = (int *)malloc(sizeof(int) * ((size_t)n + 1));
    int *t_ci = (int *)malloc(sizeof(int) * (l_nnz > 0 ? l_nnz : 1));
    double *t_va = (double *)malloc(sizeof(double) * (l_nnz > 0 ? l_nnz : 1));
    transpose_csr(n, l_nnz, l_ro, l_ci, l_va, t_ro, t_ci, t_va);
    double *R = (double *)malloc(sizeof(double) * nl);
    double *P = (double *)malloc(sizeof(double) * nl);
    double *AP = (double *)malloc(sizeof(double) * nl);
    double *Z = (double *)malloc(sizeof(double) * nl);
    double *Y = (double *)malloc(sizeof(double) * nl);
    double *alpha = (double *)malloc(sizeof(double) * L);
    double *beta = (double *)malloc(sizeof(double) * L);
    double *rho_old = (double *)malloc(sizeof(double) * L);
    double *rho_new = (double *)malloc(sizeof(double) * L);
    double *pAp = (double *)malloc(sizeof(double) * L);
    double *rn = (double *)malloc(sizeof(double) * L);
    double *b_norms = (double *)malloc(sizeof(double) * L);
    double *sum = (double *)malloc(sizeof(double) * L);
    char *converged = (char *)malloc(L);

    for (size_t i = 0; i < nl; ++i) /* :64-70 */
        X[i] = 0.0;
    memcpy(R, B, sizeof(double) * nl);
    dot_multiple(n, L, B, B, b_norms); /* :72-81 */
    for (int i = 0; i < L; ++i) {
        b_norms[i] = sqrt(b_norms[i]);
        if (b_norms[i] == 0.0)
            b_norms[i] = 1.0;
        converged[i] = 0;
    }
    forward_solve_multiple(n, l_ro, l_ci, l_va, R, Y, L, sum); /* :83-86 */
    backward_solve_multiple(n, t_ro, t_ci, t_va, Y, Z, L, sum);
    memcpy(P, Z, sizeof(double) * nl);  /* :88-89 */
    dot_multiple(n, L, R, Z, rho_old); /* :91 */

    int iter;
    for (iter = 0; iter < max_iters; ++iter) {
        memset(AP, 0, sizeof(double) * nl); /* :101-114 */
        spmm_dispatch(kernel_type, num_threads, n, num_nonzeros, row_offsets, cols, vals, P, AP, L);
        dot_multiple(n, L, P, AP, pAp); /* :116 */
        for (int i = 0; i < L; ++i)     /* :118-125 */
            alpha[i] = converged[i] ? 0.0 : rho_old[i] / pAp[i];
        axpy_multiple(n, L, alpha, P, X); /* :127 */
        for (int i = 0; i < L; ++i)
            alpha[i] = -alpha[i];
        axpy_multiple(n, L, alpha, AP, R); /* :129-132 */
        dot_multiple(n, L, R, R, rn);      /* :134-135 */
        int num_converged = 0;             /* :137-150 */
        double max_relative_error = 0.0;
        for (int i = 0; i < L; ++i) {
            double rel_error = sqrt(rn[i]) / b_norms[i];
            /* std::max(max, rel) = (max < rel) ? rel : max: a NaN rel is skipped */
            max_relative_error = max_relative_error < rel_error ? rel_error : max_relative_error;
            if (!converged[i] && rel_error < tolerance)
                converged[i] = 1;
            if (converged[i])
                num_converged++;
        }
        if (max_err_hist && iter < hist_cap) /* :153-157 */
            max_err_hist[iter] = max_relative_error;
        if (num_converged == L) { /* :159-163 */
            iter++;
            break;
        }
        forward_solve_multiple(n, l_ro, l_ci, l_va, R, Y, L, sum); /* :165-166 */
        backward_solve_multiple(n, t_ro, t_ci, t_va, Y, Z, L, sum);
        dot_multiple(n, L, R, Z, rho_new); /* :168 */
        for (int i = 0; i < L; ++i)        /* :170-177 */
            beta[i] = converged[i] ? 0.0 : rho_new[i] / rho_old[i];
        update_p_multiple(n, L, Z, beta, P); /* :179 */
        memcpy(rho_old, rho_new, sizeof(double) * L);
    }
    free(t_ro); free(t_ci); free(t_va); free(R); free(P); free(AP); free(Z); free(Y);
    free(alpha); free(beta); free(rho_old); free(rho_new); free(pAp); free(rn); free(b_norms); free(sum);
    free(converged);
    return iter;
}

/* calculate_threshold: cpu_singlecg.cpp:22-34 (dup cpu_multicg.cpp:49-61). */
ORC_EXPORT double orc_calculate_threshold(const double *b, int num_rows, double tolerance)
{
    double norm_sq = 0.0;
#pragma omp parallel for reduction(+ : norm_sq)
    for (int i = 0; i < num_rows; ++i)
        norm_sq += b[i] * b[i];
    return sqrt(norm_sq) * tolerance;
}

/* RHS fill: srand(seed); B[i] = rand()/RAND_MAX  (cpu_singlecg.cpp:87-90). */
ORC_EXPORT void orc_glibc_rand_fill(unsigned seed, long long n, double *out)
{
    srand(seed);
    for (long long i = 0; i < n; ++i)
        out[i] = (double)rand() / (double)RAND_MAX;
}

/* ------------------------------------------------------------------------- */
/* COO -> CSR: CsrMatrix::Init, sparse_matrix.h:668-733 (std::stable_sort by */
/* (row, col), duplicates kept, trailing empty rows filled).                 */
/* ------------------------------------------------------------------------- */
typedef struct {
    int row, col;
    double val;
    long long idx;
} orc_tuple;

static int tuple_cmp(const void *pa, const void *pb)
{
    const orc_tuple *a = (const orc_tuple *)pa, *b = (const orc_tuple *)pb;
    if (a->row != b->row)
        return a->row < b->row ? -1 : 1;
    if (a->col != b->col)
        return a->col < b->col ? -1 : 1;
    return a->idx < b->idx ? -1 : (a->idx > b->idx); /* stability */
}

ORC_EXPORT void orc_coo_to_csr(int num_rows, int num_nonzeros, const int *coo_rows, const int *coo_cols,
                               const double *coo_vals, int *row_offsets, int *cols, double *vals)
{
    orc_tuple *t = (orc_tuple *)malloc(sizeof(orc_tuple) * (size_t)(num_nonzeros > 0 ? num_nonzeros : 1));
    for (int i = 0; i < num_nonzeros; ++i) {
        t[i].row = coo_rows[i];
        t[i].col = coo_cols[i];
        t[i].val = coo_vals[i];
        t[i].idx = i;
    }
    qsort(t, (size_t)num_nonzeros, sizeof(orc_tuple), tuple_cmp);
    int prev_row = -1;
    for (int nz = 0; nz < num_nonzeros; nz++) {
        int cur = t[nz].row;
        for (int row = prev_row + 1; row <= cur; row++)
            row_offsets[row] = nz;
        prev_row = cur;
        cols[nz] = t[nz].col;
        vals[nz] = t[nz].val;
    }
    for (int row = prev_row + 1; row <= num_rows; row++)
        row_offsets[row] = num_nonzeros;
    free(t);
}

/* ------------------------------------------------------------------------- */
/* Generators (COO, in the reference's emission order).                      */
/* ------------------------------------------------------------------------- */
/* CooMatrix::InitGrid2d, sparse_matrix.h:458-528.  Returns nnz written. */
ORC_EXPORT int orc_grid2d_coo(int width, int self_loop, double default_value, int *rows, int *cols, double *vals)
{
    int nz = 0;
    for (int j = 0; j < width; j++)
        for (int k = 0; k < width; k++) {
            int me = j * width + k;
            if (k - 1 >= 0) { rows[nz] = me; cols[nz] = j * width + (k - 1); vals[nz++] = default_value; }
            if (k + 1 < width) { rows[nz] = me; cols[nz] = j * width + (k + 1); vals[nz++] = default_value; }
            if (j - 1 >= 0) { rows[nz] = me; cols[nz] = (j - 1) * width + k; vals[nz++] = default_value; }
            if (j + 1 < width) { rows[nz] = me; cols[nz] = (j + 1) * width + k; vals[nz++] = default_value; }
            if (self_loop) { rows[nz] = me; cols[nz] = me; vals[nz++] = default_value; }
        }
    return nz;
}

/* CooMatrix::InitGrid3d, sparse_matrix.h:533-623. */
ORC_EXPORT int orc_grid3d_coo(int width, int self_loop, double default_value, int *rows, int *cols, double *vals)
{
    int nz = 0, w2 = width * width;
    for (int i = 0; i < width; i++)
        for (int j = 0; j < width; j++)
            for (int k = 0; k < width; k++) {
                int me = i * w2 + j * width + k;
                if (k - 1 >= 0) { rows[nz] = me; cols[nz] = i * w2 + j * width + (k - 1); vals[nz++] = default_value; }
                if (k + 1 < width) { rows[nz] = me; cols[nz] = i * w2 + j * width + (k + 1); vals[nz++] = default_value; }
                if (j - 1 >= 0) { rows[nz] = me; cols[nz] = i * w2 + (j - 1) * width + k; vals[nz++] = default_value; }
                if (j + 1 < width) { rows[nz] = me; cols[nz] = i * w2 + (j + 1) * width + k; vals[nz++] = default_value; }
                if (i - 1 >= 0) { rows[nz] = me; cols[nz] = (i - 1) * w2 + j * width + k; vals[nz++] = default_value; }
                if (i + 1 < width) { rows[nz] = me; cols[nz] = (i + 1) * w2 + j * width + k; vals[nz++] = default_value; }
                if (self_loop) { rows[nz] = me; cols[nz] = me; vals[nz++] = default_value; }
            }
    return nz;
}

/* CooMatrix::InitWheel, sparse_matrix.h:417-451. */
ORC_EXPORT int orc_wheel_coo(int spokes, double default_value, int *rows, int *cols, double *vals)
{
    int nz = 0;
    for (int i = 0; i < spokes; i++) { rows[nz] = 0; cols[nz] = i + 1; vals[nz++] = default_value; }
    for (int i = 0; i < spokes; i++) {
        int dest = (i + 1) % spokes;
        rows[nz] = i + 1; cols[nz] = dest + 1; vals[nz++] = default_value;
    }
    return nz;
}

/* CooMatrix::InitDense, sparse_matrix.h:385-412. */
ORC_EXPORT int orc_dense_coo(int num_rows, int num_cols, double default_value, int *rows, int *cols, double *vals)
{
    for (int r = 0; r < num_rows; ++r)
        for (int c = 0; c < num_cols; ++c) {
            rows[r * num_cols + c] = r;
            cols[r * num_cols + c] = c;
            vals[r * num_cols + c] = default_value;
        }
    return num_rows * num_cols;
}

/* ------------------------------------------------------------------------- */
/* MatrixMarket reader: CooMatrix::InitMarket, sparse_matrix.h:211-380.      */
/* Two calls: first with rows/cols/vals NULL to get the header counts, then  */
/* with buffers of capacity *cap.  Returns 0 on success, nonzero where the    */
/* reference calls exit(1) (:232,297,305,312,327,338,348).                   */
/* Line handling mirrors std::istream::getline(line, 1024) + good(): a line  */
/* of >= 1023 chars, or a final line without '\n', ends the parse (:247-252). */
/* ------------------------------------------------------------------------- */
ORC_EXPORT int orc_read_market(const char *path, double default_value, int *num_rows, int *num_cols,
                               int *num_nonzeros, int cap, int *rows, int *cols, double *vals)
{
    FILE *f = fopen(path, "r");
    if (!f)
        return 1;
    int array = 0, symmetric = 0, skew = 0;
    int current_nz = -1;
    int nrows = 0, ncols = 0, nnz = 0;
    char line[1024];
    int rc = 0;
    for (;;) {
        if (!fgets(line, sizeof(line), f))
            break;
        size_t len = strlen(line);
        if (len == 0 || line[len - 1] != '\n')
            break; /* over-long line or EOF without newline: getline leaves !good() */
        line[len - 1] = '\0';
        if (line[0] == '%') {
            if (line[1] == '%') {
                symmetric = strstr(line, "symmetric") != NULL;
                skew = strstr(line, "skew") != NULL;
                array = strstr(line, "array") != NULL;
            }
        } else if (current_nz == -1) {
            int nparsed = sscanf(line, "%d %d %d", &nrows, &ncols, &nnz);
            if (!array && nparsed == 3) {
                if (symmetric)
                    nnz *= 2;
                current_nz = 0;
            } else if (array && nparsed == 2) {
                nnz = nrows * ncols;
                current_nz = 0;
            } else {
                rc = 2;
                break;
            }
            *num_rows = nrows;
            *num_cols = ncols;
            *num_nonzeros = nnz;
            if (!rows) { /* header probe */
                fclose(f);
                return 0;
            }
            if (cap < nnz) {
                rc = 3;
                break;
            }
        } else {
            if (current_nz >= nnz) {
                rc = 4;
                break;
            }
            int row, col;
            double val;
            if (array) {
                if (sscanf(line, "%lf", &val) != 1) {
                    rc = 5;
                    break;
                }
                col = current_nz / nrows;
                row = current_nz - nrows * col;
                rows[current_nz] = row;
                cols[current_nz] = col;
                vals[current_nz] = val;
            } else {
                char *l = line, *t = NULL;
                row = (int)strtol(l, &t, 0);
                if (t == l) { rc = 6; break; }
                l = t;
                col = (int)strtol(l, &t, 0);
                if (t == l) { rc = 7; break; }
                l = t;
                val = strtod(l, &t);
                if (t == l)
                    val = default_value;
                rows[current_nz] = row - 1;
                cols[current_nz] = col - 1;
                vals[current_nz] = val;
            }
            current_nz++;
            if (symmetric && row != col) {
                rows[current_nz] = cols[current_nz - 1];
                cols[current_nz] = rows[current_nz - 1];
                vals[current_nz] = vals[current_nz - 1] * (skew ? -1 : 1);
                current_nz++;
            }
        }
    }
    fclose(f);
    if (rc)
        return rc;
    if (current_nz < 0)
        return 8; /* no size line: the reference would leave an empty matrix */
    *num_nonzeros = current_nz; /* :371-372 */
    return 0;
}

ORC_EXPORT int orc_num_procs(void) { return omp_get_num_procs(); }
ORC_EXPORT void orc_set_threads(int n) { omp_set_num_threads(n); }
ORC_EXPORT int orc_max_threads(void) { return omp_get_max_threads(); }
