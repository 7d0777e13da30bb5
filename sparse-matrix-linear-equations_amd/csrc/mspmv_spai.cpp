// mspmv_spai.cpp -- SPAI preconditioner setup on the host: SparseApproximateInversion
// (work_2025/cg/sparse_approximate_inversion.hpp:40-321).
//
//   * static pattern S_M = S_A (:45-82);
//   * column k of M minimises ||A(I, J) m - e_k(I)||_2, J = the rows of A's column k, I = every
//     row a column in J touches (:137-208); the reference solves each small dense problem with
//     LAPACKE_dgels (a Householder QR, :210-222) -- LAPACK is not in this image, so the same
//     QR least squares is written out here; an exactly-zero diagonal of R (dgels' info > 0)
//     gives a zero column, as the reference's fallback does (:240-248);
//   * then M = (M + M^T) / 2 over the pattern (:258-318).
//
// This is setup, not the hot path: the reference runs it once per matrix on the CPU, and so does
// this library (OpenMP over columns); the PCG that applies M every iteration runs on the GPU
// (mspmv_dpcg_spai_multi, two merge-path SpMMs per iteration).
#include "mspmv.h"

#include <omp.h>

#include <cmath>
#include <string>
#include <utility>
#include <vector>

namespace mspmv {
void set_error(const std::string &msg);
}

namespace {

// min ||A x - b||_2 for a row-major m x n A with m >= n, by Householder QR in place; on success
// b[0..n) holds x.  false: m < n, or R has an exactly-zero diagonal entry (rank deficient).
bool householder_lstsq(int m, int n, double *A, double *b)
{
    if (m < n)
        return false;
    for (int j = 0; j < n; ++j) {
        double norm2 = 0.0;
        for (int i = j; i < m; ++i)
            norm2 += A[(size_t)i * n + j] * A[(size_t)i * n + j];
        if (norm2 == 0.0)
            return false;
        const double ajj = A[(size_t)j * n + j];
        const double alpha = ajj > 0.0 ? -std::sqrt(norm2) : std::sqrt(norm2);
        const double v0 = ajj - alpha;             // v = x - alpha e_1, v[i > 0] = A[i][j]
        const double vtv = v0 * v0 + (norm2 - ajj * ajj);
        if (vtv > 0.0) {
            for (int c = j + 1; c < n; ++c) {
                double s = v0 * A[(size_t)j * n + c];
                for (int i = j + 1; i < m; ++i)
                    s += A[(size_t)i * n + j] * A[(size_t)i * n + c];
                const double f = 2.0 * s / vtv;
                A[(size_t)j * n + c] -= f * v0;
                for (int i = j + 1; i < m; ++i)
                    A[(size_t)i * n + c] -= f * A[(size_t)i * n + j];
            }
            double s = v0 * b[j];
            for (int i = j + 1; i < m; ++i)
                s += A[(size_t)i * n + j] * b[i];
            const double f = 2.0 * s / vtv;
            b[j] -= f * v0;
            for (int i = j + 1; i < m; ++i)
                b[i] -= f * A[(size_t)i * n + j];
        }
        A[(size_t)j * n + j] = alpha;  // R_jj
    }
    for (int j = n - 1; j >= 0; --j) {
        double s = b[j];
        for (int c = j + 1; c < n; ++c)
            s -= A[(size_t)j * n + c] * b[c];
        b[j] = s / A[(size_t)j * n + j];
    }
    return true;
}

}  // namespace

extern "C" MSPMV_API mspmv_status mspmv_spai_values(const mspmv_csr_d *a, double *m_values)
{
    if (!a || !m_values || a->num_rows < 0 || a->num_cols < 0 || a->num_nonzeros < 0 ||
        (a->num_nonzeros > 0 && (!a->row_offsets || !a->column_indices || !a->values))) {
        mspmv::set_error("spai: bad arguments");
        return MSPMV_ERR_INVALID;
    }
    if (a->num_rows != a->num_cols) {
        mspmv::set_error("spai: the static-pattern SPAI needs a square matrix");
        return MSPMV_ERR_INVALID;
    }
    const int n = a->num_rows, nnz = a->num_nonzeros;
    const int *ro = a->row_offsets, *ci = a->column_indices;
    const double *va = a->values;
    for (int r = 0; r < n; ++r)
        if (ro[r + 1] < ro[r]) {
            mspmv::set_error("spai: row_offsets not monotone");
            return MSPMV_ERR_INVALID;
        }
    if (ro[0] != 0 || ro[n] != nnz) {
        mspmv::set_error("spai: row_offsets inconsistent with num_nonzeros");
        return MSPMV_ERR_INVALID;
    }
    for (int i = 0; i < nnz; ++i)
        if (ci[i] < 0 || ci[i] >= n) {
            mspmv::set_error("spai: column index out of range");
            return MSPMV_ERR_INVALID;
        }
    // CSC of A plus the CSC -> CSR position map (:84-119)
    std::vector<int> cptr((size_t)n + 1, 0), crow(nnz), cmap(nnz);
    std::vector<double> cval(nnz);
    for (int i = 0; i < nnz; ++i)
        ++cptr[(size_t)ci[i] + 1];
    for (int c = 0; c < n; ++c)
        cptr[(size_t)c + 1] += cptr[c];
    {
        std::vector<int> pos(cptr.begin(), cptr.end() - 1);
        for (int r = 0; r < n; ++r)
            for (int i = ro[r]; i < ro[r + 1]; ++i) {
                const int d = pos[ci[i]]++;
                crow[d] = r;
                cval[d] = va[i];
                cmap[d] = i;
            }
    }
    // per-column least squares (:121-256)
#pragma omp parallel
    {
        std::vector<double> dense, rhs;
        std::vector<int> rows;
        std::vector<int> g2l((size_t)n, -1);
#pragma omp for schedule(dynamic, 64)
        for (int k = 0; k < n; ++k) {
            const int j0 = cptr[k], j1 = cptr[(size_t)k + 1];
            const int nv = j1 - j0;
            if (nv == 0)
                continue;
            rows.clear();
            for (int idx = j0; idx < j1; ++idx) {
                const int c = crow[idx];
                for (int t = cptr[c]; t < cptr[(size_t)c + 1]; ++t) {
                    const int r = crow[t];
                    if (g2l[r] == -1) {
                        g2l[r] = (int)rows.size();
                        rows.push_back(r);
                    }
                }
            }
            const int ne = (int)rows.size();
            dense.assign((size_t)ne * nv, 0.0);
            rhs.assign(ne > nv ? ne : nv, 0.0);
            if (g2l[k] != -1)
                rhs[g2l[k]] = 1.0;
            for (int jl = 0; jl < nv; ++jl) {
                const int c = crow[j0 + jl];
                for (int t = cptr[c]; t < cptr[(size_t)c + 1]; ++t)
                    dense[(size_t)g2l[crow[t]] * nv + jl] = cval[t];
            }
            const bool ok = householder_lstsq(ne, nv, dense.data(), rhs.data());
            for (int jl = 0; jl < nv; ++jl)
                m_values[cmap[j0 + jl]] = ok ? rhs[jl] : 0.0;
            for (int r : rows)
                g2l[r] = -1;
        }
    }
    // M = (M + M^T) / 2 over the pattern: each upper entry with the first matching lower one
    // (:265-318)
#pragma omp parallel for schedule(dynamic, 256)
    for (int r = 0; r < n; ++r)
        for (int i = ro[r]; i < ro[r + 1]; ++i) {
            const int c = ci[i];
            if (c <= r)
                continue;
            for (int t = ro[c]; t < ro[(size_t)c + 1]; ++t)
                if (ci[t] == r) {
                    const double avg = (m_values[i] + m_values[t]) * 0.5;
                    m_values[i] = avg;
                    m_values[t] = avg;
                    break;
                }
        }
    return MSPMV_OK;
}
