// mspmv_synth.cpp -- deterministic synthetic CSR of the benchmark shapes (include/mspmv_synth.h).
// Host C++17 + OpenMP; every value is a pure function of (seed, index).
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "mspmv_synth.h"

namespace {

inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

inline double u01(uint64_t seed, uint64_t idx)  // [0,1) with 53 random bits
{
    return (double)(splitmix64(seed * 0x2545F4914F6CDD1Dull + idx) >> 11) * (1.0 / 9007199254740992.0);
}

// ell unique sorted columns in [lo, hi] (hi-lo+1 >= ell): one uniform pick per equal bucket.
inline void bucket_cols(int lo, int hi, int ell, uint64_t seed, uint64_t key, int *out)
{
    const long long span = (long long)hi - lo + 1;
    for (int k = 0; k < ell; ++k) {
        const long long b0 = lo + span * k / ell;
        const long long b1 = lo + span * (k + 1) / ell;  // exclusive
        const long long w = b1 - b0;
        const long long pick = (long long)(u01(seed, key * 131 + k) * (double)w);
        out[k] = (int)(b0 + (pick < w ? pick : w - 1));
    }
}

void prefix_from_lengths(const std::vector<int> &len, int *row_offsets)
{
    long long acc = 0;
    row_offsets[0] = 0;
    for (size_t i = 0; i < len.size(); ++i) {
        acc += len[i];
        row_offsets[i + 1] = (int)acc;
    }
}

}  // namespace

extern "C" {

mspmv_status mspmv_synth_banded(int m, long long nnz, int half_band, unsigned long long seed, int *row_offsets,
                                int *cols, double *vals)
{
    if (m <= 0 || nnz < 0 || nnz > 0x7fffffffLL || !row_offsets || (nnz && (!cols || !vals)))
        return MSPMV_ERR_INVALID;
    const long long maxlen = (nnz + m - 1) / m;
    if (half_band < maxlen || half_band < 1)
        return MSPMV_ERR_INVALID;
#pragma omp parallel for schedule(static)
    for (int i = 0; i <= m; ++i)
        row_offsets[i] = (int)((long long)i * nnz / m);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int i = 0; i < m; ++i) {
        const int s = row_offsets[i], ell = row_offsets[i + 1] - s;
        const int lo = std::max(0, i - half_band), hi = std::min(m - 1, i + half_band);
        bucket_cols(lo, hi, ell, seed, (uint64_t)i, cols + s);
        for (int k = 0; k < ell; ++k)
            vals[s + k] = 0.5 + u01(seed ^ 0x5bd1e995ull, (uint64_t)(s + k));
    }
    return MSPMV_OK;
}

// Rows [row_lo, row_hi) of the node-blocked FEM matrix (global column ids, row offsets rebased to
// row_lo's); every value is the one the whole-matrix generator gives the same (row, position).
static mspmv_status fem_blocked_rows(int m, long long nnz, int block, int half_band_nodes, unsigned long long seed,
                                     int row_lo, int row_hi, int *row_offsets, int *cols, double *vals)
{
    if (m <= 0 || block <= 0 || nnz < 0 || nnz > 0x7fffffffLL || !row_offsets || row_lo < 0 || row_hi > m ||
        row_lo > row_hi)
        return MSPMV_ERR_INVALID;
    const int nodes = (m + block - 1) / block;
    const long long maxlen = (nnz + m - 1) / m;
    const int maxblk = (int)((maxlen + block - 1) / block);
    if (half_band_nodes < 0 || 2LL * half_band_nodes + 1 < maxblk || maxblk > nodes)
        return MSPMV_ERR_INVALID;
    auto ro = [&](long long i) { return (long long)(i * nnz / m); };  // global row offsets
    const long long base = ro(row_lo);
#pragma omp parallel for schedule(static)
    for (int i = row_lo; i <= row_hi; ++i)
        row_offsets[i - row_lo] = (int)(ro(i) - base);
    if (!cols || !vals)  // sizing call
        return MSPMV_OK;
    const int node_lo = row_lo / block, node_hi = row_hi == row_lo ? node_lo : (row_hi - 1) / block + 1;
#pragma omp parallel for schedule(dynamic, 64)
    for (int I = node_lo; I < node_hi; ++I) {
        // neighbour nodes of node I: maxblk picks, one per slice of the node band, own node forced
        int nb[1024];
        const int nblk = std::min(maxblk, 1024);
        const int lo = std::max(0, I - half_band_nodes), hi = std::min(nodes - 1, I + half_band_nodes);
        const int span = hi - lo + 1;
        const int take = std::min(nblk, span);
        bucket_cols(lo, hi, take, seed, (uint64_t)I, nb);
        bool has_self = false;
        for (int k = 0; k < take; ++k)
            has_self |= nb[k] == I;
        if (!has_self) {  // replace the pick in I's slice by I itself (keeps the list sorted)
            int k = 0;
            while (k + 1 < take && nb[k + 1] <= I)
                ++k;
            if (nb[k] > I)
                k = 0;
            nb[k] = I;
            std::sort(nb, nb + take);
            for (int q = 1; q < take; ++q)  // resolve a possible duplicate with a neighbour slot
                if (nb[q] <= nb[q - 1])
                    nb[q] = nb[q - 1] + 1;
        }
        const int r_beg = std::max(row_lo, I * block), r_end = std::min(row_hi, std::min(m, (I + 1) * block));
        for (int i = r_beg; i < r_end; ++i) {
            const long long sg = ro(i);                       // global position (values)
            const int s = (int)(sg - base), ell = (int)(ro(i + 1) - sg);
            int k = 0;
            for (int q = 0; q < take && k < ell; ++q)
                for (int d = 0; d < block && k < ell; ++d) {
                    const long long c = (long long)nb[q] * block + d;
                    if (c >= m)
                        break;
                    cols[s + k++] = (int)c;
                }
            for (int extra = 0; k < ell; ++extra)  // only when the matrix edge cut a block short
                cols[s + k++] = std::min(m - 1, (int)(((long long)nb[take - 1] + 1) * block + extra));
            for (int q = 0; q < ell; ++q)
                vals[s + q] = 0.5 + u01(seed ^ 0x5bd1e995ull, (uint64_t)(sg + q));
        }
    }
    return MSPMV_OK;
}

mspmv_status mspmv_synth_fem_blocked(int m, long long nnz, int block, int half_band_nodes,
                                     unsigned long long seed, int *row_offsets, int *cols, double *vals)
{
    if (nnz && (!cols || !vals))
        return MSPMV_ERR_INVALID;
    return fem_blocked_rows(m, nnz, block, half_band_nodes, seed, 0, m, row_offsets, cols, vals);
}

mspmv_status mspmv_synth_fem_blocked_rows(int m, long long nnz, int block, int half_band_nodes,
                                          unsigned long long seed, int row_lo, int row_hi, int *row_offsets,
                                          int *cols, double *vals)
{
    return fem_blocked_rows(m, nnz, block, half_band_nodes, seed, row_lo, row_hi, row_offsets, cols, vals);
}

// Imperfect node-blocked FEM pattern (include/mspmv_synth.h): nodes of `block` unknowns, a fraction
// of them with block - 1 or block + 1; row targets as mspmv_synth_fem_blocked's; a fraction of rows
// with one column outside its node's pattern.  Pass 1 sizes (row_offsets), pass 2 fills.
mspmv_status mspmv_synth_fem_perturbed(int m, long long nnz, int block, int half_band_nodes, double odd_node_frac,
                                       double extra_row_frac, unsigned long long seed, int *row_offsets, int *cols,
                                       double *vals, long long *nnz_out)
{
    if (m <= 0 || block < 2 || nnz < 0 || nnz > 0x7fffffffLL || !row_offsets || half_band_nodes < 0 ||
        odd_node_frac < 0.0 || odd_node_frac > 1.0 || extra_row_frac < 0.0 || extra_row_frac > 1.0)
        return MSPMV_ERR_INVALID;
    // nodes: sizes block, or block -+ 1 with probability odd_node_frac / 2 each
    std::vector<int> nstart;
    nstart.reserve((size_t)m / (block - 1) + 2);
    for (int r = 0, I = 0; r < m; ++I) {
        nstart.push_back(r);
        const double u = u01(seed ^ 0x0dd5eedull, (uint64_t)I);
        const int dof = u < 0.5 * odd_node_frac ? block - 1 : u < odd_node_frac ? block + 1 : block;
        r = std::min(m, r + dof);
    }
    const int nodes = (int)nstart.size();
    nstart.push_back(m);
    std::vector<int> node_of((size_t)m);
#pragma omp parallel for schedule(static)
    for (int I = 0; I < nodes; ++I)
        for (int r = nstart[(size_t)I]; r < nstart[(size_t)I + 1]; ++r)
            node_of[(size_t)r] = I;
    const long long maxlen = (nnz + m - 1) / m;
    const int maxblk = std::min<int>((int)((maxlen + block - 1) / block), 1024);
    if (2LL * half_band_nodes + 1 < maxblk || maxblk > nodes)
        return MSPMV_ERR_INVALID;
    // the node's pattern: all unknowns of maxblk neighbour nodes (one per slice of the node band,
    // own node forced), ascending
    auto pattern = [&](int I, std::vector<int> &pat) {
        int nb[1024];
        const int lo = std::max(0, I - half_band_nodes), hi = std::min(nodes - 1, I + half_band_nodes);
        const int take = std::min(maxblk, hi - lo + 1);
        bucket_cols(lo, hi, take, seed, (uint64_t)I, nb);
        bool has_self = false;
        for (int k = 0; k < take; ++k)
            has_self |= nb[k] == I;
        if (!has_self) {
            int k = 0;
            while (k + 1 < take && nb[k + 1] <= I)
                ++k;
            if (nb[k] > I)
                k = 0;
            nb[k] = I;
            std::sort(nb, nb + take);
            for (int q = 1; q < take; ++q)
                if (nb[q] <= nb[q - 1])
                    nb[q] = nb[q - 1] + 1;
        }
        pat.clear();
        for (int q = 0; q < take; ++q)
            for (int c = nstart[(size_t)nb[q]]; c < nstart[(size_t)nb[q] + 1]; ++c)
                pat.push_back(c);
    };
    // row i: the first min(target, |pattern|) pattern columns, plus (perturbed rows) one column of the
    // node band that the pattern lacks, inserted in order
    auto extra_col = [&](int i, const std::vector<int> &pat, int ell) {
        if (u01(seed ^ 0xe7a2ull, (uint64_t)i) >= extra_row_frac)
            return -1;
        const int I = node_of[(size_t)i];
        const int lo = nstart[(size_t)std::max(0, I - half_band_nodes)];
        const int hi = nstart[(size_t)std::min(nodes - 1, I + half_band_nodes) + 1] - 1;
        for (int tries = 0; tries < 16; ++tries) {
            const int c = lo + (int)(u01(seed ^ 0xc01ull, (uint64_t)i * 16 + tries) * (double)(hi - lo + 1));
            if (c < lo || c > hi)
                continue;
            if (!std::binary_search(pat.begin(), pat.begin() + ell, c))
                return c;
        }
        return -1;
    };
    auto target = [&](long long i) { return (int)((i + 1) * nnz / m - i * nnz / m); };
    std::vector<int> len((size_t)m);
#pragma omp parallel
    {
        std::vector<int> pat;
#pragma omp for schedule(dynamic, 64)
        for (int I = 0; I < nodes; ++I) {
            pattern(I, pat);
            for (int i = nstart[(size_t)I]; i < nstart[(size_t)I + 1]; ++i) {
                const int ell = std::min(target(i), (int)pat.size());
                len[(size_t)i] = ell + (extra_col(i, pat, ell) >= 0 ? 1 : 0);
            }
        }
    }
    long long acc = 0;
    row_offsets[0] = 0;
    for (int i = 0; i < m; ++i) {
        acc += len[(size_t)i];
        if (acc > 0x7fffffffLL)
            return MSPMV_ERR_INVALID;
        row_offsets[i + 1] = (int)acc;
    }
    if (nnz_out)
        *nnz_out = acc;
    if (!cols || !vals)  // sizing call
        return MSPMV_OK;
#pragma omp parallel
    {
        std::vector<int> pat;
#pragma omp for schedule(dynamic, 64)
        for (int I = 0; I < nodes; ++I) {
            pattern(I, pat);
            for (int i = nstart[(size_t)I]; i < nstart[(size_t)I + 1]; ++i) {
                const int s = row_offsets[i];
                const int ell = std::min(target(i), (int)pat.size());
                const int x = extra_col(i, pat, ell);
                int k = 0;
                bool placed = x < 0;
                for (int q = 0; q < ell; ++q) {
                    if (!placed && x < pat[(size_t)q]) {
                        cols[s + k++] = x;
                        placed = true;
                    }
                    cols[s + k++] = pat[(size_t)q];
                }
                if (!placed)
                    cols[s + k++] = x;
                for (int q = 0; q < k; ++q)
                    vals[s + q] = 0.5 + u01(seed ^ 0x5bd1e995ull, (uint64_t)(s + q));
            }
        }
    }
    return MSPMV_OK;
}

mspmv_status mspmv_synth_powerlaw(int m, int n, long long nnz, double exponent, unsigned long long seed,
                                  int *row_offsets, int *cols, double *vals)
{
    if (m <= 0 || n <= 0 || nnz < 0 || nnz > (long long)m * n || nnz > 0x7fffffffLL || !row_offsets ||
        (nnz && (!cols || !vals)))
        return MSPMV_ERR_INVALID;
    std::vector<double> w(m);
    for (int i = 0; i < m; ++i)
        w[i] = std::pow(1.0 - u01(seed, (uint64_t)i), -exponent);  // Pareto-tailed weights
    double W = 0.0;
    for (double v : w)
        W += v;
    std::vector<int> len(m);
    long long assigned = 0;
    double cum = 0.0;
    long long prev = 0;
    for (int i = 0; i < m; ++i) {
        cum += w[i];
        long long upto = (long long)std::floor((double)nnz * (cum / W));
        if (i == m - 1)
            upto = nnz;
        long long ell = std::max(0LL, upto - prev);
        prev = std::max(prev, upto);
        ell = std::min<long long>(ell, n);
        len[i] = (int)ell;
        assigned += ell;
    }
    for (int i = 0; assigned < nnz; i = (i + 1) % m)  // redistribute what the n-cap removed
        if (len[i] < n) {
            ++len[i];
            ++assigned;
        }
    prefix_from_lengths(len, row_offsets);
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < m; ++i) {
        const int s = row_offsets[i], ell = len[i];
        if (ell > 0)
            bucket_cols(0, n - 1, ell, seed ^ 0x9e37ull, (uint64_t)i, cols + s);
        for (int k = 0; k < ell; ++k)
            vals[s + k] = 0.5 + u01(seed ^ 0x5bd1e995ull, (uint64_t)(s + k));
    }
    return MSPMV_OK;
}

mspmv_status mspmv_synth_stencil(int kind, int m, int dim0, int dim1, int dim2, unsigned long long seed,
                                 double diag_shift, int *row_offsets, int *cols, double *vals, long long *nnz_out)
{
    if (!row_offsets || (kind != 0 && kind != 1) || dim0 <= 0 || !(diag_shift > 0.0))
        return MSPMV_ERR_INVALID;
    if (kind == 1) {
        if (dim1 <= 0 || dim2 <= 0)
            return MSPMV_ERR_INVALID;
        const long long mm = (long long)dim0 * dim1 * dim2;
        if (mm != m)
            return MSPMV_ERR_INVALID;
    }
    if (m <= 0)
        return MSPMV_ERR_INVALID;
    const int W = dim0;
    // neighbour list of point p in increasing column order (self included)
    auto neigh = [&](int p, int *out) -> int {
        int k = 0;
        if (kind == 0) {
            const int r = p / W, c = p % W;
            const int cand_r[7] = {r - 1, r - 1, r, r, r, r + 1, r + 1};
            const int cand_c[7] = {c, c + 1, c - 1, c, c + 1, c - 1, c};
            for (int t = 0; t < 7; ++t) {
                const int rr = cand_r[t], cc = cand_c[t];
                if (rr < 0 || cc < 0 || cc >= W)
                    continue;
                const long long q = (long long)rr * W + cc;
                if (q >= m)
                    continue;
                out[k++] = (int)q;
            }
        } else {
            const int nx = dim0, ny = dim1, nz = dim2;
            const int kx = p % nx, jy = (p / nx) % ny, iz = p / (nx * ny);
            for (int di = -1; di <= 1; ++di)
                for (int dj = -1; dj <= 1; ++dj)
                    for (int dk = -1; dk <= 1; ++dk) {
                        const int i2 = iz + di, j2 = jy + dj, k2 = kx + dk;
                        if (i2 < 0 || i2 >= nz || j2 < 0 || j2 >= ny || k2 < 0 || k2 >= nx)
                            continue;
                        out[k++] = (i2 * ny + j2) * nx + k2;
                    }
        }
        return k;
    };
    std::vector<int> len(m);
#pragma omp parallel for schedule(static)
    for (int p = 0; p < m; ++p) {
        int tmp[27];
        len[p] = neigh(p, tmp);
    }
    long long total = 0;
    for (int v : len)
        total += v;
    if (total > 0x7fffffffLL)
        return MSPMV_ERR_INVALID;
    prefix_from_lengths(len, row_offsets);
    if (nnz_out)
        *nnz_out = total;
    if (!cols || !vals)
        return MSPMV_OK;
#pragma omp parallel for schedule(static)
    for (int p = 0; p < m; ++p) {
        int nb[27];
        const int k = neigh(p, nb);
        const int s = row_offsets[p];
        double diag = diag_shift;
        int self = -1;
        for (int t = 0; t < k; ++t) {
            const int q = nb[t];
            cols[s + t] = q;
            if (q == p) {
                self = t;
                continue;
            }
            const uint64_t a = (uint64_t)std::min(p, q), b = (uint64_t)std::max(p, q);
            const double off = -u01(seed, a * 0x100000001B3ull + b);  // symmetric in (p, q)
            vals[s + t] = off;
            diag += -off;
        }
        vals[s + self] = diag;
    }
    return MSPMV_OK;
}

// The 27-point grid neighbours of point p (self included), in increasing column order.
static int neigh27(int p, int nx, int ny, int nz, int *out)
{
    const int kx = p % nx, jy = (p / nx) % ny, iz = p / (nx * ny);
    int k = 0;
    for (int di = -1; di <= 1; ++di)
        for (int dj = -1; dj <= 1; ++dj)
            for (int dk = -1; dk <= 1; ++dk) {
                const int i2 = iz + di, j2 = jy + dj, k2 = kx + dk;
                if (i2 < 0 || i2 >= nz || j2 < 0 || j2 >= ny || k2 < 0 || k2 >= nx)
                    continue;
                out[k++] = (i2 * ny + j2) * nx + k2;
            }
    return k;
}

// The 7-point grid neighbours (self included), increasing.
static int neigh7(int p, int nx, int ny, int nz, int *out)
{
    const int kx = p % nx, jy = (p / nx) % ny, iz = p / (nx * ny);
    int k = 0;
    const int plane = nx * ny;
    if (iz > 0)
        out[k++] = p - plane;
    if (jy > 0)
        out[k++] = p - nx;
    if (kx > 0)
        out[k++] = p - 1;
    out[k++] = p;
    if (kx < nx - 1)
        out[k++] = p + 1;
    if (jy < ny - 1)
        out[k++] = p + nx;
    if (iz < nz - 1)
        out[k++] = p + plane;
    return k;
}

// The SPD 27-point value of entry (p, q) as mspmv_synth_stencil kind 1 gives it (diagonal: sum|off| + shift).
static void stencil27_row(int p, const int *nb, int k, uint64_t seed, double diag_shift, double *v)
{
    double diag = diag_shift;
    int self = -1;
    for (int t = 0; t < k; ++t) {
        const int q = nb[t];
        if (q == p) {
            self = t;
            continue;
        }
        const uint64_t a = (uint64_t)std::min(p, q), b = (uint64_t)std::max(p, q);
        const double off = -u01(seed, a * 0x100000001B3ull + b);
        v[t] = off;
        diag += -off;
    }
    v[self] = diag;
}

mspmv_status mspmv_synth_stencil_perturbed(int dim0, int dim1, int dim2, unsigned long long seed, double diag_shift,
                                           double extra_frac, double long_frac, int *row_offsets, int *cols,
                                           double *vals, long long *nnz_out)
{
    if (!row_offsets || dim0 <= 0 || dim1 <= 0 || dim2 <= 0 || !(diag_shift > 0.0) || extra_frac < 0.0 ||
        long_frac < 0.0)
        return MSPMV_ERR_INVALID;
    const long long mm = (long long)dim0 * dim1 * dim2;
    if (mm > 0x7fffffffLL)
        return MSPMV_ERR_INVALID;
    const int m = (int)mm, nx = dim0, ny = dim1, nz = dim2;
    const uint64_t s2 = seed * 0x9E3779B97F4A7C15ull + 17;
    auto extras = [&](int p) {
        return (u01(s2, 2 * (uint64_t)p) < extra_frac ? 1 : 0) + (u01(s2, 2 * (uint64_t)p + 1) < long_frac ? 8 : 0);
    };
    std::vector<int> len(m);
#pragma omp parallel for schedule(static)
    for (int p = 0; p < m; ++p) {
        int tmp[27];
        len[p] = neigh27(p, nx, ny, nz, tmp) + extras(p);
    }
    long long total = 0;
    for (int v : len)
        total += v;
    if (total > 0x7fffffffLL)
        return MSPMV_ERR_INVALID;
    prefix_from_lengths(len, row_offsets);
    if (nnz_out)
        *nnz_out = total;
    if (!cols || !vals)
        return MSPMV_OK;
    const long long R = 2LL * nx * ny;  // extra columns within +-R of the row
#pragma omp parallel for schedule(static)
    for (int p = 0; p < m; ++p) {
        int nb[27 + 9];
        double v[27 + 9];
        const int k = neigh27(p, nx, ny, nz, nb);
        stencil27_row(p, nb, k, seed, diag_shift, v);
        const int e = extras(p);
        std::vector<std::pair<int, double>> row;
        row.reserve((size_t)(k + e));
        for (int t = 0; t < k; ++t)
            row.emplace_back(nb[t], v[t]);
        for (int t = 0; t < e; ++t) {  // a column not in the row yet (walk right from the pick)
            long long c = p - R + (long long)(u01(s2, (uint64_t)p * 16 + 1000 + t) * (double)(2 * R + 1));
            c = std::min<long long>(std::max<long long>(c, 0), m - 1);
            for (;;) {
                bool taken = false;
                for (const auto &q : row)
                    taken = taken || q.first == c;
                if (!taken)
                    break;
                c = c + 1 < m ? c + 1 : 0;
            }
            row.emplace_back((int)c, -u01(s2, (uint64_t)p * 16 + 2000 + t));
        }
        std::sort(row.begin(), row.end());
        const int s0 = row_offsets[p];
        for (size_t t = 0; t < row.size(); ++t) {
            cols[s0 + t] = row[t].first;
            vals[s0 + t] = row[t].second;
        }
    }
    return MSPMV_OK;
}

mspmv_status mspmv_synth_kkt(int dim0, int dim1, int dim2, unsigned long long seed, double diag_shift, double eps,
                             int *row_offsets, int *cols, double *vals, long long *nnz_out)
{
    if (!row_offsets || dim0 <= 0 || dim1 <= 0 || dim2 <= 0 || !(diag_shift > 0.0) || !(eps > 0.0))
        return MSPMV_ERR_INVALID;
    const long long NN = (long long)dim0 * dim1 * dim2;
    if (2 * NN > 0x7fffffffLL)
        return MSPMV_ERR_INVALID;
    const int N = (int)NN, m = 2 * N, nx = dim0, ny = dim1, nz = dim2;
    const uint64_t sb = seed * 0xD1B54A32D192ED03ull + 5;
    auto bval = [&](int j, int i) {  // B[j][i] (i a 7-point neighbour of j)
        return i == j ? 1.0 + u01(sb, (uint64_t)j) : -u01(sb, (uint64_t)j * 0x100000001B3ull + (uint64_t)i + 1) / 6.0;
    };
    std::vector<int> len(m);
#pragma omp parallel for schedule(static)
    for (int p = 0; p < N; ++p) {
        int t27[27], t7[7];
        len[p] = neigh27(p, nx, ny, nz, t27) + neigh7(p, nx, ny, nz, t7);
        len[N + p] = neigh7(p, nx, ny, nz, t7) + 1;
    }
    long long total = 0;
    for (int v : len)
        total += v;
    if (total > 0x7fffffffLL)
        return MSPMV_ERR_INVALID;
    prefix_from_lengths(len, row_offsets);
    if (nnz_out)
        *nnz_out = total;
    if (!cols || !vals)
        return MSPMV_OK;
#pragma omp parallel for schedule(static)
    for (int p = 0; p < N; ++p) {
        int nb[27], n7[7];
        double v[27];
        const int k = neigh27(p, nx, ny, nz, nb);
        stencil27_row(p, nb, k, seed, diag_shift, v);
        const int k7 = neigh7(p, nx, ny, nz, n7);
        int s0 = row_offsets[p];
        for (int t = 0; t < k; ++t) {  // [H | B^T]: H's row, then B^T's (B's column p: rows j with p in nb7(j))
            cols[s0 + t] = nb[t];
            vals[s0 + t] = v[t];
        }
        s0 += k;
        for (int t = 0; t < k7; ++t) {
            cols[s0 + t] = N + n7[t];
            vals[s0 + t] = bval(n7[t], p);
        }
        s0 = row_offsets[N + p];  // [B | -eps I]
        for (int t = 0; t < k7; ++t) {
            cols[s0 + t] = n7[t];
            vals[s0 + t] = bval(p, n7[t]);
        }
        cols[s0 + k7] = N + p;
        vals[s0 + k7] = -eps;
    }
    return MSPMV_OK;
}

}  // extern "C"
