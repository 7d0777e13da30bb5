// rw_probe.hip -- measurement tool (not product): read+write streaming passes of the split CG at
// the nlpkkt120 size, L = 8 (m * L = 28.3 M doubles per vector, 227 MB), in the product's
// grid-stride form and as one contiguous slice per workgroup with U pairs per thread in flight.
//   pupdate: x += alpha p, p = r + beta p   (reads r, p, x; writes p, x: 5 streams)
//   update : r += (-alpha) ap, acc += r.r    (reads r, ap; writes r: 3 streams)
//   hipcc --offload-arch=gfx950 -O3 -o tools/rw_probe tools/rw_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                                \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ v2d ld(const v2d *p)
{
    if (NT)
        return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v2d *p, v2d v)
{
    if (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

__global__ __launch_bounds__(256) void k_pu_stride(const v2d *r, v2d *p, v2d *x, long long n, double al, double be)
{
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const v2d rr = r[i];
        v2d q = p[i];
        v2d xx = x[i];
        xx = xx + al * q;
        x[i] = xx;
        p[i] = rr + be * q;
    }
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_pu_slice(const v2d *r, v2d *p, v2d *x, long long n, double al, double be)
{
    const long long per = ((n + gridDim.x - 1) / gridDim.x + 255) & ~255LL;
    const long long b = (long long)blockIdx.x * per;
    const long long e = b + per < n ? b + per : n;
    for (long long i = b + threadIdx.x; i < e; i += 256 * U) {
        v2d rr[U], q[U], xx[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long k = i + u * 256 < e ? i + u * 256 : e - 1;
            rr[u] = ld<NTL>(r + k);
            q[u] = ld<NTL>(p + k);
            xx[u] = ld<NTL>(x + k);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u * 256 < e) {
                st<NTS>(x + i + u * 256, xx[u] + al * q[u]);
                st<NTS>(p + i + u * 256, rr[u] + be * q[u]);
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_up_stride(v2d *r, const v2d *ap, long long n, double al, double *out)
{
    const long long stride = (long long)gridDim.x * 256;
    v2d acc = {0, 0};
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const v2d q = ap[i];
        v2d rr = r[i];
        rr = rr - al * q;
        r[i] = rr;
        acc += rr * rr;
    }
    if (acc.x == 1234.5)
        out[0] = acc.y;
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_up_slice(v2d *r, const v2d *ap, long long n, double al, double *out)
{
    const long long per = ((n + gridDim.x - 1) / gridDim.x + 255) & ~255LL;
    const long long b = (long long)blockIdx.x * per;
    const long long e = b + per < n ? b + per : n;
    v2d acc = {0, 0};
    for (long long i = b + threadIdx.x; i < e; i += 256 * U) {
        v2d rr[U], q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long k = i + u * 256 < e ? i + u * 256 : e - 1;
            rr[u] = ld<NTL>(r + k);
            q[u] = ld<NTL>(ap + k);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u * 256 < e) {
                const v2d v = rr[u] - al * q[u];
                st<NTS>(r + i + u * 256, v);
                acc += v * v;
            }
        }
    }
    if (acc.x == 1234.5)
        out[0] = acc.y;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const long long n = 3542400LL * 8 / 2;  // pairs
    const size_t bytes = (size_t)n * 16;
    v2d *r, *p, *x, *ap;
    double *out;
    CK(hipMalloc(&r, bytes));
    CK(hipMalloc(&p, bytes));
    CK(hipMalloc(&x, bytes));
    CK(hipMalloc(&ap, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(r, 0, bytes));
    CK(hipMemset(p, 0, bytes));
    CK(hipMemset(x, 0, bytes));
    CK(hipMemset(ap, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("== %lld pairs (%zu MB per vector), %d CUs\n", n, bytes >> 20, cus);
    auto run = [&](const char *name, int streams, auto launch) -> int {
        for (int w = 0; w < 4; ++w)
            launch();
        CK(hipDeviceSynchronize());
        const int iters = 20;
        double tot = 0;
        for (int it = 0; it < iters; ++it) {
            float ms = 0;
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        const double us = tot / iters * 1e3;
        printf("%-40s %9.2f us  %7.1f GB/s\n", name, us, (double)bytes * streams / us / 1e3);
        return 0;
    };
    char nm[96];
    const double al = 0.5, be = 0.25;
    run("pupdate stride grid=2048 (product)", 5, [&] { k_pu_stride<<<2048, 256>>>(r, p, x, n, al, be); });
    run("update  stride grid=2048 (product)", 3, [&] { k_up_stride<<<2048, 256>>>(r, ap, n, al, out); });
    for (int wpc : {2, 4, 8}) {
        const int g = cus * wpc;
        snprintf(nm, sizeof nm, "pupdate slice U2      grid=%dxCU", wpc);
        run(nm, 5, [&] { k_pu_slice<2, false, false><<<g, 256>>>(r, p, x, n, al, be); });
        snprintf(nm, sizeof nm, "pupdate slice U4      grid=%dxCU", wpc);
        run(nm, 5, [&] { k_pu_slice<4, false, false><<<g, 256>>>(r, p, x, n, al, be); });
        snprintf(nm, sizeof nm, "pupdate slice U4 ntl  grid=%dxCU", wpc);
        run(nm, 5, [&] { k_pu_slice<4, true, false><<<g, 256>>>(r, p, x, n, al, be); });
        snprintf(nm, sizeof nm, "pupdate slice U4 nt   grid=%dxCU", wpc);
        run(nm, 5, [&] { k_pu_slice<4, true, true><<<g, 256>>>(r, p, x, n, al, be); });
        snprintf(nm, sizeof nm, "update  slice U4      grid=%dxCU", wpc);
        run(nm, 3, [&] { k_up_slice<4, false, false><<<g, 256>>>(r, ap, n, al, out); });
        snprintf(nm, sizeof nm, "update  slice U8      grid=%dxCU", wpc);
        run(nm, 3, [&] { k_up_slice<8, false, false><<<g, 256>>>(r, ap, n, al, out); });
        snprintf(nm, sizeof nm, "update  slice U8 ntl  grid=%dxCU", wpc);
        run(nm, 3, [&] { k_up_slice<8, true, false><<<g, 256>>>(r, ap, n, al, out); });
        snprintf(nm, sizeof nm, "update  slice U8 nt   grid=%dxCU", wpc);
        run(nm, 3, [&] { k_up_slice<8, true, true><<<g, 256>>>(r, ap, n, al, out); });
    }
    return 0;
}
