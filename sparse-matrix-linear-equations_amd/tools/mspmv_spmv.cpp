// mspmv_spmv -- MI355X counterpart of the reference's cpu_spmv driver (cpu_spmv.cpp:747-991):
// same flags, same matrix sources, same x = 0.0019 input, same timing-iteration rule and the same
// DisplayPerf fields (cpu_spmv.cpp:715-742), so eval_csrmv.sh-style scripts parse its lines.
//
//   mspmv_spmv [--quiet] [--i=<timing iterations>] [--device=<d>] [--threads=<ignored>]
//              --mtx=<file.mtx> | --grid2d=<w> | --grid3d=<w> | --wheel=<spokes> | --dense=<cols>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mspmv.h"
#include "mspmv_io.h"

static bool flag(int argc, char **argv, const char *name)
{
    std::string f = std::string("--") + name;
    for (int i = 1; i < argc; ++i)
        if (f == argv[i])
            return true;
    return false;
}

static bool arg(int argc, char **argv, const char *name, std::string &out)
{
    std::string p = std::string("--") + name + "=";
    for (int i = 1; i < argc; ++i)
        if (strncmp(argv[i], p.c_str(), p.size()) == 0) {
            out = argv[i] + p.size();
            return true;
        }
    return false;
}

static void die(const char *what, mspmv_status s)
{
    fprintf(stderr, "%s failed (%d): %s\n", what, (int)s, mspmv_last_error());
    exit(1);
}

int main(int argc, char **argv)
{
    const bool quiet = flag(argc, argv, "quiet");
    std::string s_mtx, s;
    int grid2d = -1, grid3d = -1, wheel = -1, dense = -1, iters = -1, device = 0;
    arg(argc, argv, "mtx", s_mtx);
    if (arg(argc, argv, "grid2d", s)) grid2d = atoi(s.c_str());
    if (arg(argc, argv, "grid3d", s)) grid3d = atoi(s.c_str());
    if (arg(argc, argv, "wheel", s)) wheel = atoi(s.c_str());
    if (arg(argc, argv, "dense", s)) dense = atoi(s.c_str());
    if (arg(argc, argv, "i", s)) iters = atoi(s.c_str());
    if (arg(argc, argv, "device", s)) device = atoi(s.c_str());

    int m = 0, n = 0, nnz = 0, *ro = nullptr, *ci = nullptr;
    double *va = nullptr;
    mspmv_status st;
    char name[512];
    if (!s_mtx.empty()) {
        if ((st = mspmv_market_read(s_mtx.c_str(), 1.0, &m, &n, &nnz, &ro, &ci, &va)) != MSPMV_OK)
            die("mspmv_market_read", st);
        if (m == 1 || n == 1 || nnz == 1) {  // cpu_spmv.cpp:769-774
            if (!quiet)
                printf("Trivial dataset\n");
            return 0;
        }
        snprintf(name, sizeof(name), "%s", s_mtx.c_str());
    } else if (grid2d > 0) {
        st = mspmv_generate(MSPMV_GEN_GRID2D, grid2d, 0, 1.0, &m, &n, &nnz, &ro, &ci, &va);
        snprintf(name, sizeof(name), "grid2d_%d", grid2d);
    } else if (grid3d > 0) {
        st = mspmv_generate(MSPMV_GEN_GRID3D, grid3d, 0, 1.0, &m, &n, &nnz, &ro, &ci, &va);
        snprintf(name, sizeof(name), "grid3d_%d", grid3d);
    } else if (wheel > 0) {
        st = mspmv_generate(MSPMV_GEN_WHEEL, wheel, 0, 1.0, &m, &n, &nnz, &ro, &ci, &va);
        snprintf(name, sizeof(name), "wheel_%d", wheel);
    } else if (dense > 0) {
        st = mspmv_generate(MSPMV_GEN_DENSE, (1 << 24) / dense, dense, 1.0, &m, &n, &nnz, &ro, &ci, &va);
        snprintf(name, sizeof(name), "dense_%d_x_%d", (1 << 24) / dense, dense);
    } else {
        fprintf(stderr, "No graph type specified.\n");
        return 1;
    }
    if (s_mtx.empty() && st != MSPMV_OK)
        die("mspmv_generate", st);
    printf("%s, ", name);

    // row-length statistics, the CSV form of GraphStats::Display (sparse_matrix.h:59-103)
    double mean = (double)nnz / (m ? m : 1), var = 0, skew = 0;
    for (int i = 0; i < m; ++i) {
        const double d = (ro[i + 1] - ro[i]) - mean;
        var += d * d;
        skew += d * d * d;
    }
    const double sd = m > 1 ? std::sqrt(var / (m - 1)) : 0.0;
    const double sk = (m > 0 && sd > 0) ? (skew / m) / (sd * sd * sd) : 0.0;
    printf("%d, %d, %d, %.5f, %.5f, %.5f, %.5f, ", m, n, nnz, mean, sd, mean > 0 ? sd / mean : 0.0, sk);

    if (iters < 0)  // cpu_spmv.cpp:830-835
        iters = (int)std::min(200000ull, std::max(100ull, (16ull << 30) / (unsigned long long)std::max(nnz, 1)));

    mspmv_csr_d a{m, n, nnz, ro, ci, va};
    mspmv_handle h = nullptr;
    if ((st = mspmv_csr_create(&a, device, &h)) != MSPMV_OK)
        die("mspmv_csr_create", st);
    std::vector<double> x(n, 0.0019), y(m), gold(m), mag(m);  // cpu_spmv.cpp:855-859
    for (int r = 0; r < m; ++r) {  // SpmvGold with alpha 1, beta 0 (cpu_spmv.cpp:241-265)
        double p = 0.0 * 1.0, a = 0.0;
        for (int k = ro[r]; k < ro[r + 1]; ++k) {
            p += 1.0 * va[k] * x[ci[k]];
            a += std::fabs(va[k] * x[ci[k]]);
        }
        gold[r] = p;
        mag[r] = a;
    }
    void *dx = nullptr, *dy = nullptr;
    if ((st = mspmv_device_malloc(device, sizeof(double) * n, &dx)) != MSPMV_OK ||
        (st = mspmv_device_malloc(device, sizeof(double) * m, &dy)) != MSPMV_OK ||
        (st = mspmv_memcpy_h2d(dx, x.data(), sizeof(double) * n)) != MSPMV_OK)
        die("device buffers", st);
    if ((st = mspmv_dspmv_dev(h, (const double *)dx, (double *)dy)) != MSPMV_OK || (st = mspmv_sync(h)) != MSPMV_OK ||
        (st = mspmv_memcpy_d2h(y.data(), dy, sizeof(double) * m)) != MSPMV_OK)
        die("spmv", st);
    double maxrel = 0;
    for (int r = 0; r < m; ++r)
        maxrel = std::max(maxrel, std::fabs(y[r] - gold[r]) / std::max(mag[r], 1e-300));
    if (!quiet)  // |y - gold| against sum |a_k x_k|: the bound a reordered fp64 sum obeys
        printf("\n\n\t%s (max diff vs SpmvGold relative to |A||x| %.3g)\n", maxrel < 1e-12 ? "PASS" : "FAIL", maxrel);
    double avg_ms = 0;
    if ((st = mspmv_time_spmm_dev(h, (const double *)dx, (double *)dy, 1, iters, 0, &avg_ms)) != MSPMV_OK)
        die("timing", st);
    const double setup_ms = mspmv_setup_ms(h);
    // DisplayPerf (cpu_spmv.cpp:715-742)
    const size_t total_bytes = (size_t)nnz * (sizeof(double) * 2 + sizeof(int)) + (size_t)m * (sizeof(int) + sizeof(double));
    const double nz_throughput = (double)nnz / avg_ms / 1.0e6;
    const double eff_bw = (double)total_bytes / avg_ms / 1.0e6;
    printf("GPU Merge CsrMV, ");
    if (!quiet)
        printf("fp64: %.4f setup ms, %.4f avg ms, %.5f gflops, %.3lf effective GB/s\n", setup_ms, avg_ms,
               2 * nz_throughput, eff_bw);
    else
        printf("%.5f, %.5f, %.6f, %.3lf, \n", setup_ms, avg_ms, 2 * nz_throughput, eff_bw);
    mspmv_device_free(dx);
    mspmv_device_free(dy);
    mspmv_destroy(h);
    mspmv_host_free(ro);
    mspmv_host_free(ci);
    mspmv_host_free(va);
    return maxrel < 1e-12 ? 0 : 2;
}
