// mspmv_io.cpp -- host-side matrix construction with the reference's exact semantics
// (include/mspmv_io.h): MatrixMarket reader (CooMatrix::InitMarket, sparse_matrix.h:211-380),
// the lattice/wheel/dense generators (:385-623) and COO -> CSR (CsrMatrix::Init, :668-733:
// stable order by (row, col), duplicates kept, trailing empty rows).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "mspmv_io.h"

namespace {

struct Coo {
    int rows = 0, cols = 0;
    std::vector<int> r, c;
    std::vector<double> v;
};

// Stable (row, col) order: counting sort by row (stable), then a stable sort of each row by
// column -- the same permutation std::stable_sort with CooComparator produces.
mspmv_status coo_to_csr(const Coo &coo, int **ro_out, int **ci_out, double **va_out)
{
    const int m = coo.rows;
    const size_t nnz = coo.r.size();
    int *ro = (int *)malloc(sizeof(int) * ((size_t)m + 1));
    int *ci = (int *)malloc(sizeof(int) * std::max<size_t>(nnz, 1));
    double *va = (double *)malloc(sizeof(double) * std::max<size_t>(nnz, 1));
    if (!ro || !ci || !va) {
        free(ro);
        free(ci);
        free(va);
        return MSPMV_ERR_OOM;
    }
    std::vector<size_t> cnt((size_t)m + 1, 0);
    for (size_t k = 0; k < nnz; ++k) {
        if (coo.r[k] < 0 || coo.r[k] >= m || coo.c[k] < 0 || coo.c[k] >= coo.cols) {
            free(ro);
            free(ci);
            free(va);
            return MSPMV_ERR_IO;
        }
        ++cnt[(size_t)coo.r[k] + 1];
    }
    for (int i = 0; i < m; ++i)
        cnt[i + 1] += cnt[i];
    std::vector<size_t> pos(cnt.begin(), cnt.end() - 1), order(nnz);
    for (size_t k = 0; k < nnz; ++k)
        order[pos[coo.r[k]]++] = k;
    for (int i = 0; i < m; ++i) {
        auto b = order.begin() + (long)cnt[i], e = order.begin() + (long)cnt[i + 1];
        std::stable_sort(b, e, [&](size_t x, size_t y) { return coo.c[x] < coo.c[y]; });
        ro[i] = (int)cnt[i];
    }
    ro[m] = (int)nnz;
    for (size_t k = 0; k < nnz; ++k) {
        ci[k] = coo.c[order[k]];
        va[k] = coo.v[order[k]];
    }
    *ro_out = ro;
    *ci_out = ci;
    *va_out = va;
    return MSPMV_OK;
}

}  // namespace

extern "C" {

void mspmv_host_free(void *p) { free(p); }

mspmv_status mspmv_market_read(const char *path, double default_value, int *num_rows, int *num_cols,
                               int *num_nonzeros, int **row_offsets, int **column_indices, double **values)
{
    if (!path || !num_rows || !num_cols || !num_nonzeros || !row_offsets || !column_indices || !values)
        return MSPMV_ERR_INVALID;
    FILE *f = fopen(path, "rb");
    if (!f)
        return MSPMV_ERR_IO;
    // getline(line, 1024) + good(): a line of >= 1023 characters, or a last line without a
    // newline, ends the parse (sparse_matrix.h:247-252).
    bool array = false, symmetric = false, skew = false;
    long long cur = -1, declared = 0;
    Coo coo;
    char line[1024];
    mspmv_status st = MSPMV_OK;
    for (;;) {
        if (!fgets(line, sizeof(line), f))
            break;
        size_t len = strlen(line);
        if (len == 0 || line[len - 1] != '\n')
            break;
        line[len - 1] = '\0';
        if (line[0] == '%') {
            if (line[1] == '%') {
                symmetric = strstr(line, "symmetric") != nullptr;
                skew = strstr(line, "skew") != nullptr;
                array = strstr(line, "array") != nullptr;
            }
            continue;
        }
        if (cur == -1) {
            int nr = 0, nc = 0, nz = 0;
            const int nparsed = sscanf(line, "%d %d %d", &nr, &nc, &nz);
            if (!array && nparsed == 3) {
                declared = symmetric ? 2LL * nz : nz;
            } else if (array && nparsed == 2) {
                declared = (long long)nr * nc;
            } else {
                st = MSPMV_ERR_IO;  // "invalid problem description" (:296-298)
                break;
            }
            coo.rows = nr;
            coo.cols = nc;
            coo.r.reserve((size_t)declared);
            coo.c.reserve((size_t)declared);
            coo.v.reserve((size_t)declared);
            cur = 0;
            continue;
        }
        if (cur >= declared) {
            st = MSPMV_ERR_IO;  // more entries than declared (:303-307)
            break;
        }
        int row, col;
        double val;
        if (array) {
            if (sscanf(line, "%lf", &val) != 1) {
                st = MSPMV_ERR_IO;
                break;
            }
            col = (int)(cur / coo.rows);
            row = (int)(cur - (long long)coo.rows * col);
            coo.r.push_back(row);
            coo.c.push_back(col);
        } else {
            char *l = line, *t = nullptr;
            row = (int)strtol(l, &t, 0);  // base 0 exactly as the reference parses
            if (t == l) {
                st = MSPMV_ERR_IO;
                break;
            }
            l = t;
            col = (int)strtol(l, &t, 0);
            if (t == l) {
                st = MSPMV_ERR_IO;
                break;
            }
            l = t;
            val = strtod(l, &t);
            if (t == l)
                val = default_value;  // pattern matrices
            coo.r.push_back(row - 1);
            coo.c.push_back(col - 1);
        }
        coo.v.push_back(val);
        ++cur;
        if (symmetric && row != col) {
            const size_t k = coo.r.size() - 1;
            coo.r.push_back(coo.c[k]);
            coo.c.push_back(coo.r[k]);
            coo.v.push_back(coo.v[k] * (skew ? -1 : 1));
            ++cur;
        }
    }
    fclose(f);
    if (st != MSPMV_OK)
        return st;
    if (cur < 0)
        return MSPMV_ERR_IO;
    *num_rows = coo.rows;
    *num_cols = coo.cols;
    *num_nonzeros = (int)coo.r.size();
    return coo_to_csr(coo, row_offsets, column_indices, values);
}

mspmv_status mspmv_generate(int kind, int p0, int p1, double default_value, int *num_rows, int *num_cols,
                            int *num_nonzeros, int **row_offsets, int **column_indices, double **values)
{
    if (!num_rows || !num_cols || !num_nonzeros || !row_offsets || !column_indices || !values)
        return MSPMV_ERR_INVALID;
    Coo coo;
    auto add = [&](int r, int c) {
        coo.r.push_back(r);
        coo.c.push_back(c);
        coo.v.push_back(default_value);
    };
    switch (kind) {
    case MSPMV_GEN_GRID2D: {  // InitGrid2d(width = p0, self_loop = p1), sparse_matrix.h:458-528
        const int w = p0;
        if (w < 1)
            return MSPMV_ERR_INVALID;
        coo.rows = coo.cols = w * w;
        for (int j = 0; j < w; j++)
            for (int k = 0; k < w; k++) {
                const int me = j * w + k;
                if (k - 1 >= 0) add(me, j * w + k - 1);
                if (k + 1 < w) add(me, j * w + k + 1);
                if (j - 1 >= 0) add(me, (j - 1) * w + k);
                if (j + 1 < w) add(me, (j + 1) * w + k);
                if (p1) add(me, me);
            }
        break;
    }
    case MSPMV_GEN_GRID3D: {  // InitGrid3d(width = p0, self_loop = p1), :533-623
        const int w = p0, w2 = p0 * p0;
        if (w < 1)
            return MSPMV_ERR_INVALID;
        coo.rows = coo.cols = w * w2;
        for (int i = 0; i < w; i++)
            for (int j = 0; j < w; j++)
                for (int k = 0; k < w; k++) {
                    const int me = i * w2 + j * w + k;
                    if (k - 1 >= 0) add(me, i * w2 + j * w + k - 1);
                    if (k + 1 < w) add(me, i * w2 + j * w + k + 1);
                    if (j - 1 >= 0) add(me, i * w2 + (j - 1) * w + k);
                    if (j + 1 < w) add(me, i * w2 + (j + 1) * w + k);
                    if (i - 1 >= 0) add(me, (i - 1) * w2 + j * w + k);
                    if (i + 1 < w) add(me, (i + 1) * w2 + j * w + k);
                    if (p1) add(me, me);
                }
        break;
    }
    case MSPMV_GEN_WHEEL: {  // InitWheel(spokes = p0), :417-451
        const int s = p0;
        if (s < 1)
            return MSPMV_ERR_INVALID;
        coo.rows = coo.cols = s + 1;
        for (int i = 0; i < s; i++) add(0, i + 1);
        for (int i = 0; i < s; i++) add(i + 1, (i + 1) % s + 1);
        break;
    }
    case MSPMV_GEN_DENSE: {  // InitDense(rows = p0, cols = p1), :385-412
        if (p0 < 1 || p1 < 1)
            return MSPMV_ERR_INVALID;
        coo.rows = p0;
        coo.cols = p1;
        for (int r = 0; r < p0; ++r)
            for (int c = 0; c < p1; ++c) add(r, c);
        break;
    }
    default:
        return MSPMV_ERR_INVALID;
    }
    *num_rows = coo.rows;
    *num_cols = coo.cols;
    *num_nonzeros = (int)coo.r.size();
    return coo_to_csr(coo, row_offsets, column_indices, values);
}

}  // extern "C"
