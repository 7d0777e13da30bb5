// mspmv_io.cpp -- host-side matrix construction with the reference's exact semantics
// (include/mspmv_io.h): MatrixMarket reader (CooMatrix::InitMarket, sparse_matrix.h:211-380),
// the lattice/wheel/dense generators (:385-623) and COO -> CSR (CsrMatrix::Init, :668-733:
// stable order by (row, col), duplicates kept, trailing empty rows).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include <omp.h>

#include "mspmv_io.h"

namespace {

struct Coo {
    int rows = 0, cols = 0;
    std::vector<int> r, c;
    std::vector<double> v;
};

// Stable (row, col) order: counting sort by row (stable), then a stable sort of each row by
// column -- the same permutation std::stable_sort with CooComparator produces
// (CsrMatrix::Init, sparse_matrix.h:668-733).  Parallel and still stable: thread t counts its
// contiguous range of entries per row, and row i's entries of thread t land after those of
// threads < t, so every row keeps its entries in file order before the per-row column sort.
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
    bool bad = false;
#pragma omp parallel for reduction(|| : bad)
    for (long long k = 0; k < (long long)nnz; ++k)
        bad = bad || coo.r[k] < 0 || coo.r[k] >= m || coo.c[k] < 0 || coo.c[k] >= coo.cols;
    if (bad) {
        free(ro);
        free(ci);
        free(va);
        return MSPMV_ERR_IO;
    }
    // threads: enough entries each, and the per-thread row counters within ~1 GB
    int T = std::max(1, std::min(omp_get_max_threads(), (int)(nnz / 65536)));
    while (T > 1 && (size_t)T * ((size_t)m + 1) * sizeof(int) > (1ull << 30))
        --T;
    std::vector<int> cnt((size_t)T * ((size_t)m + 1), 0);
    auto range = [&](int t, size_t &b, size_t &e) {
        b = nnz * (size_t)t / T;
        e = nnz * (size_t)(t + 1) / T;
    };
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        size_t b, e;
        range(t, b, e);
        int *c = cnt.data() + (size_t)t * ((size_t)m + 1);
        for (size_t k = b; k < e; ++k)
            ++c[coo.r[k]];
    }
    // ro[i] = entries of rows < i; cnt[t][i] becomes thread t's first slot in row i
    std::vector<size_t> rowlen((size_t)m, 0);
#pragma omp parallel for
    for (long long i = 0; i < (long long)m; ++i) {
        size_t acc = 0;
        for (int t = 0; t < T; ++t) {
            const int c = cnt[(size_t)t * ((size_t)m + 1) + (size_t)i];
            cnt[(size_t)t * ((size_t)m + 1) + (size_t)i] = (int)acc;
            acc += (size_t)c;
        }
        rowlen[(size_t)i] = acc;
    }
    size_t run = 0;
    for (int i = 0; i < m; ++i) {
        ro[i] = (int)run;
        run += rowlen[(size_t)i];
    }
    ro[m] = (int)nnz;
    std::vector<size_t> order(nnz);
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        size_t b, e;
        range(t, b, e);
        int *c = cnt.data() + (size_t)t * ((size_t)m + 1);
        for (size_t k = b; k < e; ++k) {
            const int r = coo.r[k];
            order[(size_t)ro[r] + (size_t)c[r]++] = k;
        }
    }
#pragma omp parallel for schedule(dynamic, 4096)
    for (long long i = 0; i < (long long)m; ++i) {
        auto b = order.begin() + ro[i], e = order.begin() + ro[i + 1];
        std::stable_sort(b, e, [&](size_t x, size_t y) { return coo.c[x] < coo.c[y]; });
    }
#pragma omp parallel for
    for (long long k = 0; k < (long long)nnz; ++k) {
        ci[k] = coo.c[order[(size_t)k]];
        va[k] = coo.v[order[(size_t)k]];
    }
    *ro_out = ro;
    *ci_out = ci;
    *va_out = va;
    return MSPMV_OK;
}


// ---- MatrixMarket (CooMatrix::InitMarket, sparse_matrix.h:211-380) -------------------------
struct MarketState {
    bool array = false, symmetric = false, skew = false;
    long long cur = -1, declared = 0;
    double dflt = 1.0;
};

bool slurp(const char *path, std::vector<char> &buf)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return false;
    bool ok = fseek(f, 0, SEEK_END) == 0;
    const long size = ok ? ftell(f) : -1;
    ok = ok && size >= 0 && fseek(f, 0, SEEK_SET) == 0;
    if (ok) {
        buf.resize((size_t)size);
        ok = fread(buf.data(), 1, (size_t)size, f) == (size_t)size;
    }
    fclose(f);
    return ok;
}

// The reference's ifs.getline(line, 1024) + good() (:247-252): a line is taken only when it ends
// in '\n' and has at most 1022 characters; the first line that does not ends the parse.  Copies the
// line, NUL-terminated as getline leaves it (strtol must not run on into the next line).
inline bool take_line(const std::vector<char> &buf, size_t pos, char *line, size_t *next)
{
    if (pos >= buf.size())
        return false;
    const char *p = buf.data() + pos;
    const size_t avail = buf.size() - pos;
    const char *nl = (const char *)memchr(p, '\n', std::min<size_t>(avail, 1023));
    if (!nl)
        return false;
    const size_t len = (size_t)(nl - p);
    memcpy(line, p, len);
    line[len] = '\0';
    *next = pos + len + 1;
    return true;
}

// One coordinate entry "row col [val]" (:318-345): strtol base 0, strtod, pattern -> default.
inline bool parse_entry(const char *line, double dflt, int *row, int *col, double *val)
{
    char *t = nullptr;
    const char *l = line;
    *row = (int)strtol(l, &t, 0);
    if (t == l)
        return false;
    l = t;
    *col = (int)strtol(l, &t, 0);
    if (t == l)
        return false;
    l = t;
    *val = strtod(l, &t);
    if (t == l)
        *val = dflt;
    return true;
}

inline void push_entry(Coo &coo, const MarketState &S, int row, int col, double val)
{
    coo.r.push_back(row - 1);
    coo.c.push_back(col - 1);
    coo.v.push_back(val);
    if (S.symmetric && row != col) {  // mirror, skew-negated (:350-356)
        coo.r.push_back(col - 1);
        coo.c.push_back(row - 1);
        coo.v.push_back(val * (S.skew ? -1 : 1));
    }
}

// One accepted line of the reference's loop; false on a parse error (where it calls exit(1)).
bool market_line(const char *line, MarketState &S, Coo &coo)
{
    if (line[0] == '%') {
        if (line[1] == '%') {  // banner (:257-263)
            S.symmetric = strstr(line, "symmetric") != nullptr;
            S.skew = strstr(line, "skew") != nullptr;
            S.array = strstr(line, "array") != nullptr;
        }
        return true;
    }
    if (S.cur == -1) {  // problem description (:273-298)
        int nr = 0, nc = 0, nz = 0;
        const int nparsed = sscanf(line, "%d %d %d", &nr, &nc, &nz);
        if (!S.array && nparsed == 3)
            S.declared = S.symmetric ? 2LL * nz : nz;
        else if (S.array && nparsed == 2)
            S.declared = (long long)nr * nc;
        else
            return false;
        coo.rows = nr;
        coo.cols = nc;
        coo.r.reserve((size_t)S.declared);
        coo.c.reserve((size_t)S.declared);
        coo.v.reserve((size_t)S.declared);
        S.cur = 0;
        return true;
    }
    if (S.cur >= S.declared)  // more entries than declared (:303-307)
        return false;
    if (S.array) {  // column-major dense entries (:312-317)
        double val;
        if (sscanf(line, "%lf", &val) != 1)
            return false;
        const int col = (int)(S.cur / coo.rows);
        const int row = (int)(S.cur - (long long)coo.rows * col);
        coo.r.push_back(row);
        coo.c.push_back(col);
        coo.v.push_back(val);
        ++S.cur;
        if (S.symmetric && row != col) {
            coo.r.push_back(col);
            coo.c.push_back(row);
            coo.v.push_back(val * (S.skew ? -1 : 1));
            ++S.cur;
        }
        return true;
    }
    int row, col;
    double val;
    if (!parse_entry(line, S.dflt, &row, &col, &val))
        return false;
    const size_t before = coo.r.size();
    push_entry(coo, S, row, col, val);
    S.cur += (long long)(coo.r.size() - before);
    return true;
}

mspmv_status market_serial(const std::vector<char> &buf, size_t pos, MarketState &S, Coo &coo)
{
    char line[1024];
    size_t next;
    while (take_line(buf, pos, line, &next)) {
        pos = next;
        if (!market_line(line, S, coo))
            return MSPMV_ERR_IO;
    }
    return MSPMV_OK;
}

// Coordinate entries in parallel: the entry region is cut at line starts into one chunk per
// thread; each thread parses its lines into its own arrays exactly as market_line does, noting the
// first line that would end the reference's loop (stop), a parse error, or a banner ("%%" lines
// reset the format flags mid-file: then the whole region is redone serially).  Chunks are taken
// in order up to the first stop, so the entries, their order and every error decision are those
// of the serial loop: the declared-count check (:303-307) fails iff the last taken entry line
// starts at an entry count >= the declared one.  Returns false to ask for the serial parse.
// MSPMV_IO_MIN_CHUNK (bytes per thread, default 1 MiB) lets tests force many chunks.
bool market_entries_parallel(const std::vector<char> &buf, size_t pos, MarketState &S, Coo &coo, mspmv_status *st)
{
    const size_t region = buf.size() - pos;
    const char *mc = getenv("MSPMV_IO_MIN_CHUNK");
    const size_t min_chunk = std::max<size_t>(64, mc ? (size_t)atoll(mc) : (size_t)1 << 20);
    const int T = (int)std::min<size_t>((size_t)omp_get_max_threads(), region / min_chunk);
    if (T < 2)
        return false;
    std::vector<size_t> cut((size_t)T + 1, buf.size());
    cut[0] = pos;
    for (int t = 1; t < T; ++t) {  // the line start at or after the nominal cut
        size_t c = pos + region * (size_t)t / (size_t)T;
        const void *nl = memchr(buf.data() + c - 1, '\n', buf.size() - (c - 1));
        cut[(size_t)t] = nl ? (size_t)((const char *)nl - buf.data()) + 1 : buf.size();
    }
    for (int t = 1; t <= T; ++t)
        cut[(size_t)t] = std::max(cut[(size_t)t], cut[(size_t)t - 1]);
    struct Part {
        Coo coo;
        bool stop = false, err = false, banner = false, any = false;
        long long last_before = 0;  // entries of this chunk before its last entry line
    };
    std::vector<Part> part((size_t)T);
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        Part &P = part[(size_t)t];
        const size_t est = (cut[(size_t)t + 1] - cut[(size_t)t]) / 16 * (S.symmetric ? 2 : 1);
        P.coo.r.reserve(est);
        P.coo.c.reserve(est);
        P.coo.v.reserve(est);
        char line[1024];
        size_t p = cut[(size_t)t], next;
        while (p < cut[(size_t)t + 1]) {
            if (!take_line(buf, p, line, &next)) {
                P.stop = true;
                break;
            }
            p = next;
            if (line[0] == '%') {
                if (line[1] == '%') {
                    P.banner = true;
                    break;
                }
                continue;
            }
            int row, col;
            double val;
            if (!parse_entry(line, S.dflt, &row, &col, &val)) {
                P.err = true;
                break;
            }
            P.last_before = (long long)P.coo.r.size();
            P.any = true;
            push_entry(P.coo, S, row, col, val);
        }
    }
    long long total = 0, last_start = -1;
    int used = 0;
    for (int t = 0; t < T; ++t) {
        const Part &P = part[(size_t)t];
        if (P.banner)
            return false;
        if (P.any)
            last_start = total + P.last_before;
        if (P.err) {
            *st = MSPMV_ERR_IO;
            return true;
        }
        total += (long long)P.coo.r.size();
        used = t + 1;
        if (P.stop)
            break;
    }
    if (last_start >= S.declared) {
        *st = MSPMV_ERR_IO;
        return true;
    }
    coo.r.resize((size_t)total);
    coo.c.resize((size_t)total);
    coo.v.resize((size_t)total);
    std::vector<size_t> off((size_t)used + 1, 0);
    for (int t = 0; t < used; ++t)
        off[(size_t)t + 1] = off[(size_t)t] + part[(size_t)t].coo.r.size();
#pragma omp parallel for num_threads(T)
    for (int t = 0; t < used; ++t) {
        const Coo &c = part[(size_t)t].coo;
        std::copy(c.r.begin(), c.r.end(), coo.r.begin() + (long)off[(size_t)t]);
        std::copy(c.c.begin(), c.c.end(), coo.c.begin() + (long)off[(size_t)t]);
        std::copy(c.v.begin(), c.v.end(), coo.v.begin() + (long)off[(size_t)t]);
    }
    S.cur = total;
    *st = MSPMV_OK;
    return true;
}

}  // namespace

extern "C" {

void mspmv_host_free(void *p) { free(p); }

mspmv_status mspmv_market_read(const char *path, double default_value, int *num_rows, int *num_cols,
                               int *num_nonzeros, int **row_offsets, int **column_indices, double **values)
{
    if (!path || !num_rows || !num_cols || !num_nonzeros || !row_offsets || !column_indices || !values)
        return MSPMV_ERR_INVALID;
    std::vector<char> buf;
    if (!slurp(path, buf))
        return MSPMV_ERR_IO;
    MarketState S;
    Coo coo;
    S.dflt = default_value;
    // banner, comments and the size line: serial (they decide the format of what follows)
    size_t pos = 0;
    while (S.cur == -1) {
        char line[1024];
        size_t next;
        if (!take_line(buf, pos, line, &next))
            break;
        pos = next;
        if (!market_line(line, S, coo))
            return MSPMV_ERR_IO;
    }
    if (S.cur < 0)
        return MSPMV_ERR_IO;
    mspmv_status st = MSPMV_OK;
    if (S.array || !market_entries_parallel(buf, pos, S, coo, &st))
        st = market_serial(buf, pos, S, coo);  // array format (entry i's position is i), small files, banners mid-file
    if (st != MSPMV_OK)
        return st;
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
