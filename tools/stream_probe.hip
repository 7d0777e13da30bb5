// stream_probe.hip -- measurement tool (not product): the HBM read ceiling for one launch of the
// SpMV headline's size.  Reads BYTES of int32+f64 streams (the cols/vals of a pwtk-shaped CSR,
// 142.6 MB) once per launch, rotating over 4 copies so every launch is cold (as in bench.py),
// with a few grid shapes / widths.  Prints per-launch kernel time and GB/s.
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const v2d *__restrict__ a, size_t n16, double *out)
{
    const size_t stride = (size_t)gridDim.x * 256;
    v2d acc = {0, 0};
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        v2d t[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            t[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += t[u];
    }
    for (; i < n16; i += stride)
        acc += a[i];
    if (acc.x == 1234.5)
        out[0] = acc.y;
}

// contiguous chunk per block (the tile kernel's access shape): block b reads [b*chunk, (b+1)*chunk)
template <bool NT>
__global__ __launch_bounds__(256) void k_read_chunk(const v2d *__restrict__ a, size_t n16, int chunk16, double *out)
{
    const int t = (blockIdx.x & 7) * ((gridDim.x + 7) >> 3) + (blockIdx.x >> 3);
    size_t b = (size_t)t * chunk16;
    v2d acc = {0, 0};
    v2d v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        size_t i = b + threadIdx.x + u * 256;
        v[u] = (u * 256 + (int)threadIdx.x < chunk16 && i < n16) ? (NT ? __builtin_nontemporal_load(a + i) : a[i]) : v2d{0, 0};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
        acc += v[u];
    if (acc.x == 1234.5)
        out[0] = acc.y;
}

int main()
{
    const size_t bytes = 142651548;
    const size_t n16 = bytes / 16;
    const int NB = 4;
    std::vector<v2d *> bufs(NB);
    for (auto &p : bufs) {
        CK(hipMalloc(&p, bytes + 4096));
        CK(hipMemset(p, 1, bytes));
    }
    double *out;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) -> int {
        for (int w = 0; w < 8; ++w)
            launch(bufs[w % NB]);
        CK(hipDeviceSynchronize());
        const int iters = 40;
        float tot = 0;
        for (int it = 0; it < iters; ++it) {
            CK(hipEventRecord(e0));
            launch(bufs[it % NB]);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        const double us = tot / iters * 1e3;
        printf("%-34s %8.2f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);
        return 0;
    };
    for (int g : {1024, 2048, 4096, 8192}) {
        char nm[64];
        snprintf(nm, sizeof nm, "grid-stride U4 grid=%d", g);
        run(nm, [&](v2d *p) { k_read<4, false><<<g, 256>>>(p, n16, out); });
        snprintf(nm, sizeof nm, "grid-stride U4 nt grid=%d", g);
        run(nm, [&](v2d *p) { k_read<4, true><<<g, 256>>>(p, n16, out); });
    }
    for (int chunk : {1024, 1536, 2048}) {
        const int grid = (int)((n16 + chunk - 1) / chunk);
        char nm[64];
        snprintf(nm, sizeof nm, "chunk %d x16B grid=%d", chunk, grid);
        run(nm, [&](v2d *p) { k_read_chunk<false><<<grid, 256>>>(p, n16, chunk, out); });
        snprintf(nm, sizeof nm, "chunk %d x16B nt grid=%d", chunk, grid);
        run(nm, [&](v2d *p) { k_read_chunk<true><<<grid, 256>>>(p, n16, chunk, out); });
    }
    return 0;
}
