// mspmv_ic0.cpp -- IC(0) preconditioner setup on the host: IncompleteCholesky and TransposeCsr
// (work_2025/cg/incomplete_cholesky_decomp.hpp:11-201).
//
//   * L's pattern is A's lower triangle (diagonal included), in A's CSR order (:91-148);
//   * row by row, entry (i, k): sum over the common columns of rows i (before k) and k of
//     L(i,c) L(k,c), merged in CSR order; L(i,k) -= sum; the diagonal takes sqrt and fails when
//     <= 0; an off-diagonal divides by L(k,k), taken as the LAST entry of row k (:175-212);
//   * on failure the factorization restarts from A's values with the diagonal shifted by
//     1e-3, then x10 per attempt, 20 attempts (:150-173, :213-225).
// The reference factorizes sequentially on the CPU; this is setup, run once, and stays on the
// host the same way.  The two triangular solves it feeds run on the GPU every iteration
// (k_trsv, sync-free, mspmv_kernels.hip).
#include "mspmv.h"

#include <cmath>
#include <string>
#include <vector>

namespace mspmv {
void set_error(const std::string &msg);
}

namespace {

mspmv_status check_square(const mspmv_csr_d *a)
{
    if (!a || a->num_rows < 0 || a->num_nonzeros < 0 || !a->row_offsets ||
        (a->num_nonzeros > 0 && (!a->column_indices || !a->values))) {
        mspmv::set_error("ic0: bad arguments");
        return MSPMV_ERR_INVALID;
    }
    if (a->num_rows != a->num_cols) {
        mspmv::set_error("ic0: IC(0) needs a square (symmetric) matrix");
        return MSPMV_ERR_INVALID;
    }
    const int n = a->num_rows;
    if (a->row_offsets[0] != 0 || a->row_offsets[n] != a->num_nonzeros) {
        mspmv::set_error("ic0: row_offsets inconsistent with num_nonzeros");
        return MSPMV_ERR_INVALID;
    }
    for (int r = 0; r < n; ++r)
        if (a->row_offsets[r + 1] < a->row_offsets[r]) {
            mspmv::set_error("ic0: row_offsets not monotone");
            return MSPMV_ERR_INVALID;
        }
    for (int i = 0; i < a->num_nonzeros; ++i)
        if (a->column_indices[i] < 0 || a->column_indices[i] >= n) {
            mspmv::set_error("ic0: column index out of range");
            return MSPMV_ERR_INVALID;
        }
    return MSPMV_OK;
}

}  // namespace

extern "C" MSPMV_API mspmv_status mspmv_ic0_nnz(const mspmv_csr_d *a, int *nnz_l)
{
    mspmv_status st = check_square(a);
    if (st != MSPMV_OK)
        return st;
    if (!nnz_l) {
        mspmv::set_error("ic0: null output");
        return MSPMV_ERR_INVALID;
    }
    int c = 0;
    for (int i = 0; i < a->num_rows; ++i)
        for (int k = a->row_offsets[i]; k < a->row_offsets[i + 1]; ++k)
            c += a->column_indices[k] <= i;
    *nnz_l = c;
    return MSPMV_OK;
}

extern "C" MSPMV_API mspmv_status mspmv_ic0_factor(const mspmv_csr_d *a, int *l_row_offsets, int *l_cols,
                                                   double *l_vals, double *shift_out)
{
    mspmv_status st = check_square(a);
    if (st != MSPMV_OK)
        return st;
    if (!l_row_offsets || (a->num_nonzeros > 0 && (!l_cols || !l_vals))) {
        mspmv::set_error("ic0: null output");
        return MSPMV_ERR_INVALID;
    }
    const int n = a->num_rows;
    const int *ro = a->row_offsets, *ci = a->column_indices;
    l_row_offsets[0] = 0;
    int nz = 0;
    for (int i = 0; i < n; ++i) {  // :91-148
        for (int k = ro[i]; k < ro[i + 1]; ++k)
            if (ci[k] <= i) {
                l_cols[nz] = ci[k];
                l_vals[nz] = a->values[k];
                ++nz;
            }
        l_row_offsets[i + 1] = nz;
    }
    const std::vector<double> backup(l_vals, l_vals + nz);
    const int *lro = l_row_offsets, *lci = l_cols;
    double *lv = l_vals;
    double shift = 0.0;
    for (int retry = 0; retry < 20; ++retry) {
        bool failed = false;
        if (retry > 0)  // :159-173
            for (int idx = 0; idx < n; ++idx)
                for (int off = lro[idx]; off < lro[idx + 1]; ++off) {
                    lv[off] = backup[off];
                    if (lci[off] == idx)
                        lv[off] += shift;
                }
        for (int i = 0; i < n && !failed; ++i) {  // :175-212
            for (int ko = lro[i]; ko < lro[i + 1]; ++ko) {
                const int k = lci[ko];
                double sum = 0.0;
                int jl = lro[i], jk = lro[k];
                while (jl < ko && jk < lro[k + 1]) {
                    if (lci[jl] == lci[jk]) {
                        sum += lv[jl] * lv[jk];
                        ++jl;
                        ++jk;
                    } else if (lci[jl] < lci[jk]) {
                        ++jl;
                    } else {
                        ++jk;
                    }
                }
                lv[ko] -= sum;
                if (k == i) {
                    if (lv[ko] <= 0) {
                        failed = true;
                        break;
                    }
                    lv[ko] = std::sqrt(lv[ko]);
                } else {
                    lv[ko] /= lv[lro[k + 1] - 1];  // the reference takes row k's last entry as its diagonal
                }
            }
        }
        if (!failed) {
            if (shift_out)
                *shift_out = shift;
            return MSPMV_OK;
        }
        shift = shift == 0.0 ? 1e-3 : shift * 10.0;  // :218-224
    }
    mspmv::set_error("ic0: Incomplete Cholesky factorization failed after 20 attempts");
    return MSPMV_ERR_BREAKDOWN;
}

// TransposeCsr (work_2025/cg/incomplete_cholesky_decomp.hpp:11-78): counting sort by column with
// rows visited in order, so each output row lists its entries by ascending input row, as the
// reference's.  Host code (setup of the IC(0) preconditioner, as in the reference).
extern "C" MSPMV_API mspmv_status mspmv_csr_transpose(const mspmv_csr_d *in, int *out_row_offsets, int *out_cols,
                                                      double *out_vals)
{
    if (!in || in->num_rows < 0 || in->num_cols < 0 || in->num_nonzeros < 0 || !in->row_offsets ||
        !out_row_offsets || (in->num_nonzeros > 0 && (!in->column_indices || !in->values || !out_cols || !out_vals))) {
        mspmv::set_error("csr_transpose: bad arguments");
        return MSPMV_ERR_INVALID;
    }
    const int m = in->num_rows, n = in->num_cols, nnz = in->num_nonzeros;
    if (in->row_offsets[0] != 0 || in->row_offsets[m] != nnz) {
        mspmv::set_error("csr_transpose: row_offsets inconsistent with num_nonzeros");
        return MSPMV_ERR_INVALID;
    }
    for (int k = 0; k < nnz; ++k)
        if (in->column_indices[k] < 0 || in->column_indices[k] >= n) {
            mspmv::set_error("csr_transpose: column index out of range");
            return MSPMV_ERR_INVALID;
        }
    std::vector<int> pos((size_t)n + 1, 0);
    for (int k = 0; k < nnz; ++k)
        ++pos[(size_t)in->column_indices[k] + 1];
    for (int c = 0; c < n; ++c)
        pos[(size_t)c + 1] += pos[c];
    for (int c = 0; c <= n; ++c)
        out_row_offsets[c] = pos[c];
    for (int r = 0; r < m; ++r)
        for (int k = in->row_offsets[r]; k < in->row_offsets[r + 1]; ++k) {
            const int d = pos[in->column_indices[k]]++;
            out_cols[d] = r;
            out_vals[d] = in->values[k];
        }
    return MSPMV_OK;
}
