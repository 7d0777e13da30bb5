// read_ceiling.hip -- measurement tool (not product): the HBM read ceiling on MI355X for the
// bench's `measured_read_GBps`.  One 1 GiB buffer (> the 256 MiB Infinity Cache) read whole per
// launch, event-timed, by several kernel shapes; and the single-launch ceiling at the headline's
// 142.6 MB (4 rotating copies, so every launch reads cold lines).
//   hipcc --offload-arch=gfx950 -O3 -o tools/read_ceiling tools/read_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>
#include <cstdlib>
#include <algorithm>

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

// A: grid-stride, U loads of 16 B per lane per iteration
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stride(const v2d *__restrict__ a, long long n16, double *out)
{
    const long long stride = (long long)gridDim.x * 256;
    v2d acc = {0, 0};
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        v2d t[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            t[u] = ld<NT>(a + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += t[u];
    }
    for (; i < n16; i += stride)
        acc += a[i];
    if (acc.x == 1234.5)
        out[0] = acc.y;
}

// B: persistent contiguous slice per workgroup, U x 16 B per lane in flight, next batch issued
// before the previous one is consumed (two register stages)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_slice(const v2d *__restrict__ a, long long n16, double *out)
{
    const long long per = (n16 + gridDim.x - 1) / gridDim.x;
    const long long b = (long long)blockIdx.x * per;
    const long long e = b + per < n16 ? b + per : n16;
    v2d acc = {0, 0};
    const long long step = 256LL * U;
    long long i = b + threadIdx.x;
    v2d t0[U], t1[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        t0[u] = i + u * 256 < e ? ld<NT>(a + i + u * 256) : v2d{0, 0};
    for (i += step; i < e + step; i += 2 * step) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            t1[u] = i + u * 256 < e ? ld<NT>(a + i + u * 256) : v2d{0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += t0[u];
#pragma unroll
        for (int u = 0; u < U; ++u)
            t0[u] = i + step + u * 256 < e ? ld<NT>(a + i + step + u * 256) : v2d{0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += t1[u];
    }
    if (acc.x == 1234.5)
        out[0] = acc.y;
}

// C: LDS-DMA (global_load_lds_dwordx4) ring: each wave streams its part of the workgroup's slice
// into its own 4 x 1 KiB LDS slots, R instructions in flight, nothing read back
template <int R, bool NT>
__global__ __launch_bounds__(256) void k_glds(const v2d *__restrict__ a, long long n16, double *out)
{
    __shared__ v2d ring[4][R][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long per = (n16 + gridDim.x - 1) / gridDim.x;
    const long long b = (long long)blockIdx.x * per;
    const long long e = b + per < n16 ? b + per : n16;
    const long long wper = (per + 3) / 4;
    const long long wb = b + wave * wper;
    const long long we = wb + wper < e ? wb + wper : e;
    int k = 0;
    for (long long i = wb + lane; i < we; i += 64, k = (k + 1) % R) {
        __builtin_amdgcn_global_load_lds((const void *)(a + i), (void *)&ring[wave][k][0], 16, 0, NT ? 2 : 0);
        if (k == R - 1)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R / 2) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ring[wave][0][lane].x == 1234.5)
        out[0] = 1.0;
}

int main(int argc, char **argv)
{
    std::vector<size_t> sizes = {(size_t)1 << 30, (size_t)142651548};
    if (argc > 1) {  // sizes in bytes (copies rotate through > 512 MiB, so every launch reads from HBM)
        sizes.clear();
        for (int i = 1; i < argc; ++i)
            sizes.push_back((size_t)atoll(argv[i]));
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double *out;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (size_t bytes : sizes) {
        const int NB = bytes < ((size_t)256 << 20) ? (int)std::max<size_t>(4, ((size_t)600 << 20) / bytes + 1) : 1;
        const long long n16 = (long long)(bytes / 16);
        std::vector<v2d *> bufs(NB);
        for (auto &p : bufs) {
            CK(hipMalloc(&p, bytes + 4096));
            CK(hipMemset(p, 0, bytes));
        }
        printf("== %zu bytes per launch (%d rotating copies), %d CUs\n", bytes, NB, cus);
        auto run = [&](const char *name, auto launch) -> int {
            for (int w = 0; w < 8; ++w)
                launch(bufs[w % NB]);
            CK(hipDeviceSynchronize());
            const int iters = 20;
            std::vector<float> t(iters);
            for (int it = 0; it < iters; ++it) {
                CK(hipEventRecord(e0));
                launch(bufs[it % NB]);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&t[it], e0, e1));
            }
            double tot = 0;
            for (float v : t)
                tot += v;
            const double us = tot / iters * 1e3;
            printf("%-36s %9.2f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);
            return 0;
        };
        char nm[96];
        for (int wpc : {4, 8}) {
            const int g = cus * wpc;
            snprintf(nm, sizeof nm, "stride U4 nt  grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_stride<4, true><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "stride U8 nt  grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_stride<8, true><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "stride U8     grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_stride<8, false><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "slice U4 nt   grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_slice<4, true><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "slice U8 nt   grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_slice<8, true><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "slice U8      grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_slice<8, false><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "glds R8 nt    grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_glds<8, true><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "glds R16 nt   grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_glds<16, true><<<g, 256>>>(p, n16, out); });
            snprintf(nm, sizeof nm, "glds R16      grid=%dxCU", wpc);
            run(nm, [&](v2d *p) { k_glds<16, false><<<g, 256>>>(p, n16, out); });
        }
        for (auto &p : bufs)
            CK(hipFree(p));
    }
    return 0;
}
