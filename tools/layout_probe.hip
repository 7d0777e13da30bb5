// layout_probe.hip -- measurement tool (not product): does the SpMV tile stream read faster from
// one contiguous per-tile record ([vals | cols16] packed per tile) than from two separate arrays
// (vals[], cols16[]), and with 16-B instead of 8-B / 2-B lane loads?  Pure streaming, no gathers:
// each 256-thread block reads one tile of NZ nonzeros (the pwtk plan: ~1975 nnz per tile,
// 11.5 M nnz), rotating over 4 copies so every launch is cold.
//   hipcc --offload-arch=gfx950 -O3 -o tools/layout_probe tools/layout_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int NZ = 1976;        // nonzeros per tile (multiple of 8)
constexpr int REC = NZ * 10;    // bytes per packed tile record

__device__ __forceinline__ int xcd_map(int b, int n) { return (b & 7) * ((n + 7) >> 3) + (b >> 3); }

// two arrays, lane loads of 8 B (vals) and 2 B (cols), striped: lane l of round j takes l + 256 j
template <bool NT>
__global__ __launch_bounds__(256) void k_sep8(const double *__restrict__ v, const unsigned short *__restrict__ c,
                                              int tiles, double *out)
{
    const int t = xcd_map(blockIdx.x, gridDim.x);
    if (t >= tiles)
        return;
    const size_t n0 = (size_t)t * NZ;
    double acc = 0;
    double vv[8];
    int cc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = min((int)threadIdx.x + 256 * j, NZ - 1);
        cc[j] = NT ? __builtin_nontemporal_load(c + n0 + k) : c[n0 + k];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = min((int)threadIdx.x + 256 * j, NZ - 1);
        vv[j] = NT ? __builtin_nontemporal_load(v + n0 + k) : v[n0 + k];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        acc += vv[j] * cc[j];
    if (acc == 1234.5)
        out[0] = acc;
}

// one packed record per tile: [NZ doubles][NZ ushorts], same lane loads
template <bool NT>
__global__ __launch_bounds__(256) void k_pack8(const unsigned char *__restrict__ p, int tiles, double *out)
{
    const int t = xcd_map(blockIdx.x, gridDim.x);
    if (t >= tiles)
        return;
    const double *v = reinterpret_cast<const double *>(p + (size_t)t * REC);
    const unsigned short *c = reinterpret_cast<const unsigned short *>(p + (size_t)t * REC + NZ * 8);
    double acc = 0;
    double vv[8];
    int cc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = min((int)threadIdx.x + 256 * j, NZ - 1);
        cc[j] = NT ? __builtin_nontemporal_load(c + k) : c[k];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = min((int)threadIdx.x + 256 * j, NZ - 1);
        vv[j] = NT ? __builtin_nontemporal_load(v + k) : v[k];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        acc += vv[j] * cc[j];
    if (acc == 1234.5)
        out[0] = acc;
}

// packed record, 16-B lane loads over the whole record (REC/16 = 1235 per tile)
template <bool NT>
__global__ __launch_bounds__(256) void k_pack16(const unsigned char *__restrict__ p, int tiles, double *out)
{
    typedef double v2d __attribute__((ext_vector_type(2)));
    const int t = xcd_map(blockIdx.x, gridDim.x);
    if (t >= tiles)
        return;
    const v2d *q = reinterpret_cast<const v2d *>(p + (size_t)t * REC);
    constexpr int N16 = REC / 16;
    v2d acc = {0, 0};
    v2d vv[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int k = min((int)threadIdx.x + 256 * j, N16 - 1);
        vv[j] = NT ? __builtin_nontemporal_load(q + k) : q[k];
    }
#pragma unroll
    for (int j = 0; j < 5; ++j)
        acc += vv[j];
    if (acc.x == 1234.5)
        out[0] = acc.y;
}

int main()
{
    const int tiles = 5832;  // 11.5 M nnz / NZ
    const size_t nnz = (size_t)tiles * NZ;
    const int NB = 4;
    std::vector<double *> vb(NB);
    std::vector<unsigned short *> cb(NB);
    std::vector<unsigned char *> pb(NB);
    for (int i = 0; i < NB; ++i) {
        CK(hipMalloc(&vb[i], nnz * 8 + 4096));
        CK(hipMalloc(&cb[i], nnz * 2 + 4096));
        CK(hipMalloc(&pb[i], (size_t)tiles * REC + 4096));
        CK(hipMemset(vb[i], 1, nnz * 8));
        CK(hipMemset(cb[i], 1, nnz * 2));
        CK(hipMemset(pb[i], 1, (size_t)tiles * REC));
    }
    double *out;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)nnz * 10;
    auto run = [&](const char *name, auto launch) -> int {
        for (int w = 0; w < 8; ++w)
            launch(w % NB);
        CK(hipDeviceSynchronize());
        const int iters = 60;
        float tot = 0;
        for (int it = 0; it < iters; ++it) {
            CK(hipEventRecord(e0));
            launch(it % NB);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        const double us = tot / iters * 1e3;
        printf("%-28s %8.2f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);
        return 0;
    };
    for (int r = 0; r < 2; ++r) {
        run("separate 8B/2B", [&](int i) { k_sep8<false><<<tiles, 256>>>(vb[i], cb[i], tiles, out); });
        run("separate 8B/2B nt", [&](int i) { k_sep8<true><<<tiles, 256>>>(vb[i], cb[i], tiles, out); });
        run("packed 8B/2B", [&](int i) { k_pack8<false><<<tiles, 256>>>(pb[i], tiles, out); });
        run("packed 8B/2B nt", [&](int i) { k_pack8<true><<<tiles, 256>>>(pb[i], tiles, out); });
        run("packed 16B", [&](int i) { k_pack16<false><<<tiles, 256>>>(pb[i], tiles, out); });
        run("packed 16B nt", [&](int i) { k_pack16<true><<<tiles, 256>>>(pb[i], tiles, out); });
    }
    return 0;
}
