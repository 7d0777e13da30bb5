// mspmv_cg -- MI355X counterpart of the reference's CG drivers:
//   single (default): cpu_singlecg (cpu_singlecg.cpp:67-214): srand(42) RHS, L = 16 vectors
//     solved one after another, threshold = tol * ||B[0:n]|| (the reference's quirk), CSV
//     "matrix_name,kernel,num_vectors,min_ms,gflops,iterations" (:187-214).
//   --multi: cpu_multicg's CGSolveMultiple leg (cpu_multicg.cpp:106-210): L lock-step RHS,
//     "Min time / Iters / GFLOPS" line and the per-iteration max error CSV (:67-86).
//
//   mspmv_cg --mtx=<file> [--multi] [--num_vectors=16] [--max_iters=N] [--tolerance=1e-5]
//            [--timing_iters=1] [--output=<csv>] [--seed=42] [--device=0] [--quiet]
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
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

static std::string base_name(const std::string &f)  // GetMatrixBaseName, cpu_singlecg.cpp:39-49
{
    size_t sl = f.find_last_of("/\\");
    std::string b = sl == std::string::npos ? f : f.substr(sl + 1);
    size_t dot = b.find_last_of('.');
    return dot == std::string::npos ? b : b.substr(0, dot);
}

static void die(const char *what, mspmv_status s)
{
    fprintf(stderr, "%s failed (%d): %s\n", what, (int)s, mspmv_last_error());
    exit(1);
}

int main(int argc, char **argv)
{
    std::string mtx, out_csv, s;
    const bool multi = flag(argc, argv, "multi"), quiet = flag(argc, argv, "quiet");
    int L = 16, max_iters = multi ? 50000 : 10000, timing = 1, device = 0;
    unsigned seed = 42;
    double tol = 1e-5;
    arg(argc, argv, "mtx", mtx);
    arg(argc, argv, "output", out_csv);
    if (arg(argc, argv, "num_vectors", s)) L = atoi(s.c_str());
    if (arg(argc, argv, "max_iters", s)) max_iters = atoi(s.c_str());
    if (arg(argc, argv, "tolerance", s)) tol = atof(s.c_str());
    if (arg(argc, argv, "timing_iters", s)) timing = std::max(1, atoi(s.c_str()));
    if (arg(argc, argv, "seed", s)) seed = (unsigned)atoi(s.c_str());
    if (arg(argc, argv, "device", s)) device = atoi(s.c_str());
    if (mtx.empty()) {
        fprintf(stderr, "Usage: %s --mtx=<filename> [--multi] [options]\n", argv[0]);
        return 1;
    }
    int m, n, nnz, *ro, *ci;
    double *va;
    mspmv_status st = mspmv_market_read(mtx.c_str(), 1.0, &m, &n, &nnz, &ro, &ci, &va);
    if (st != MSPMV_OK)
        die("mspmv_market_read", st);
    mspmv_csr_d a{m, n, nnz, ro, ci, va};
    mspmv_handle h = nullptr;
    if ((st = mspmv_csr_create(&a, device, &h)) != MSPMV_OK)
        die("mspmv_csr_create", st);
    // RHS: srand(seed); B[i] = rand()/RAND_MAX over n*L (cpu_singlecg.cpp:87-90)
    std::vector<double> B((size_t)m * L), X((size_t)m * L);
    srand(seed);
    for (auto &b : B)
        b = (double)rand() / (double)RAND_MAX;
    double nb = 0;
    for (int i = 0; i < m; ++i)
        nb += B[i] * B[i];
    const double threshold = std::sqrt(nb) * tol;  // calculate_threshold, cpu_singlecg.cpp:22-34
    const double flops1 = 2.0 * nnz + 10.0 * m;
    const std::string name = base_name(mtx);
    double min_ms = std::numeric_limits<double>::max();
    long long iters_min = 0;
    std::vector<double> hist((size_t)max_iters);
    for (int t = 0; t < timing; ++t) {
        long long total = 0;
        const auto t0 = std::chrono::steady_clock::now();
        if (!multi) {
            for (int v = 0; v < L; ++v) {  // column blocks B[v*n .. ] (single_strategy.hpp:219-226)
                int it = 0;
                st = mspmv_dcg_single(h, &B[(size_t)v * m], &X[(size_t)v * m], max_iters, threshold, &it, nullptr, 0);
                if (st != MSPMV_OK && st != MSPMV_ERR_BREAKDOWN)
                    die("mspmv_dcg_single", st);
                total += it;
            }
        } else {
            int it = 0;
            st = mspmv_dcg_multi(h, B.data(), X.data(), L, max_iters, threshold, MSPMV_NONZERO_SPLIT, &it,
                                 t == 0 ? hist.data() : nullptr, t == 0 ? max_iters : 0);
            if (st != MSPMV_OK && st != MSPMV_ERR_BREAKDOWN)
                die("mspmv_dcg_multi", st);
            total = it;
            if (t == 0)
                hist.resize(std::min<size_t>(hist.size(), (size_t)it));
        }
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (!quiet)
            printf("\tTime: %.3f ms (Total Iters: %lld)\n", ms, total);
        if (ms < min_ms) {
            min_ms = ms;
            iters_min = total;
        }
    }
    if (!multi) {
        const double gflops = flops1 * (double)iters_min / (min_ms / 1000.0) / 1e9;
        printf("    %s, L=%d, method=GPU_SINGLE_LOOP: %.3f ms, %lld iters, %.2f GFLOPS\n", name.c_str(), L, min_ms,
               iters_min, gflops);
        if (out_csv.empty())
            out_csv = "data/simple_gflops/" + name + "_gflops.csv";
        if (FILE *f = fopen(out_csv.c_str(), "w")) {
            fprintf(f, "matrix_name,kernel,num_vectors,min_ms,gflops,iterations\n%s,GPU_SINGLE_LOOP,%d,%.3f,%.2f,%lld\n",
                    name.c_str(), L, min_ms, gflops, iters_min);
            fclose(f);
        } else {
            fprintf(stderr, "Error: Cannot open file %s for writing\n", out_csv.c_str());
        }
    } else {
        const double gflops = flops1 * L * (double)iters_min / (min_ms / 1000.0) / 1e9;
        printf("Min time: %8.3f ms, Iters: %6.1f, Overall GFLOPS/s: %6.2f\n", min_ms, (double)iters_min, gflops);
        if (out_csv.empty())
            out_csv = "data/error_data/" + name + "_cg_errors.csv";
        if (FILE *f = fopen(out_csv.c_str(), "w")) {
            fprintf(f, "iteration,max_error\n");
            for (size_t i = 0; i < hist.size(); ++i)
                fprintf(f, "%zu,%e\n", i, hist[i]);
            fclose(f);
        } else {
            fprintf(stderr, "Error: Cannot open file %s for writing\n", out_csv.c_str());
        }
    }
    mspmv_destroy(h);
    mspmv_host_free(ro);
    mspmv_host_free(ci);
    mspmv_host_free(va);
    return 0;
}
