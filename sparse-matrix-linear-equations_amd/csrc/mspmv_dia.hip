// mspmv_dia.hip -- offset windows: SpMV / SpMM for structured-grid rows (round 5).
//
// A window is 64 consecutive rows.  Where the rows of a window list their columns at a few common
// offsets from the row index (col - row: a finite-difference or finite-volume stencil, the 27-point
// nlpkkt120-size shape, parabolic_fem's 7-point triangles), the window is stored as its sorted offset
// list D (K <= kDiaMaxK entries) and a K x 64 panel of values, lane-major: value k of the window's row
// l at vt[k][l] (0 where row l has no column at offset D[k]; a 64-bit presence mask per (window, k)
// then says which rows hold it).  One wave computes one window with lane = row: for k = 0 .. K-1 it
// loads vt[k][lane] (512 contiguous bytes) and x[row + D[k]] (64 consecutive rows: contiguous), so
// there is no column stream (8 B per nonzero from HBM instead of 10-12), no gather of scattered lines,
// no LDS and no cross-lane reduction.  Each row is summed from 0.0 in D order, which is its CSR order
// (the planner requires every row's columns strictly ascending), as mul then add: bit-identical to
// SpmvGold (cpu_spmv.cpp:241-265) and, per column, to the reference's row-by-row SpMM
// (work_2025/spmm/cpu_spmm.cpp), whose merge-path OmpMergeCsrmv / OmpMergeCsrmm
// (merge_based.hpp:46-153) differ from these only by the reordering of split rows.
//
// L-wide panels (row-major, row stride ld): lanes form groups of L/2 (one double2 of a panel row
// each); a wave instruction reads 64/(L/2) consecutive panel rows -- 1 KB contiguous -- and a lane
// holds L/2 rows of the window.
//
// The plan is all or nothing: every window of the matrix must fit (K <= kDiaMaxK, its nonzeros >=
// min_window_fill x rows x K) and the whole matrix fill its panels (nonzeros >= min_fill x 64 x sum K:
// the zeros of rows missing an offset -- grid boundaries -- are streamed too); anything else keeps
// the tile plans.
#include "mspmv_device.h"
#include "mspmv_internal.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace mspmv {

constexpr int kDiaThreads = 256;  // four windows per workgroup
constexpr int kDiaWaves = kDiaThreads / 64;

struct DiaArgs {
    const int4 *hdr;                 // [windows] {K, offset base, value base (x 64 doubles), mask base or -1}
    const int *off;                  // offsets, per window ascending
    const unsigned long long *mask;  // presence masks of the windows that need them
    const double *vt;                // [sum K][64]
    const double *x;
    double *y;
    const CgControl *ctrl;           // CG: return at once when ctrl->done
    int windows;
    int groups;                      // workgroups (windows / 4, rounded up)
    int m;
    int ld;                          // panel row stride (L-wide products)
};

template <bool NT>
__device__ __forceinline__ double dia_ld(const double *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// Values in flight per lane: U consecutive offsets of the window are loaded before any is summed.
constexpr int dia_unroll(int L) { return L <= 2 ? 8 : L <= 8 ? 4 : 2; }

// Lab forms of the L-wide kernel (MSPMV_DIA_FORM, A/B only; default 1): 0 lanes (column pair, row)
// with each lane's rows' values loaded directly, U = dia_unroll(L); 1 the values loaded once per offset
// (lane = row) and passed by shuffles; 2 one row per lane (L/2 double2 loads per offset); 3 form 2
// with half the unroll; 4 form 0 with half the unroll.  nlpkkt120 size, L = 8 (r05q): 497 / 470 / 586
// / 598 / 513 us -- value-load instructions and X lines per instruction both cost.
constexpr int dia_form_unroll(int L, int FORM) { return (FORM == 3 || FORM == 4) ? (dia_unroll(L) > 1 ? dia_unroll(L) / 2 : 1) : dia_unroll(L); }

template <int L, bool NT, int FORM = 0>
__global__ __launch_bounds__(kDiaThreads) void k_spmm_dia(DiaArgs a)
{
    constexpr int U = L == 1 ? dia_unroll(1) : dia_form_unroll(L, FORM);
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int w = xcd_tile(blockIdx.x, a.groups) * kDiaWaves + wv;
    if (w >= a.windows)
        return;
    if (a.ctrl && a.ctrl->done)
        return;
    const int lane = threadIdx.x & 63;
    const int4 hd = a.hdr[w];
    const int K = hd.x;
    const int *__restrict__ off = a.off + hd.y;
    const double *__restrict__ vt = a.vt + (size_t)hd.z * 64;
    const long long r0 = (long long)w * 64;
    const bool masked = hd.w >= 0;
    const unsigned long long *__restrict__ mk = a.mask + (masked ? hd.w : 0);

    if constexpr (L == 1) {
        const long long r = r0 + lane;
        double acc = 0.0;
        if (!masked) {  // every row of the window holds every offset: no selects, no clamps
            for (int k0 = 0; k0 < K; k0 += U) {
                double v[U], xv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int kk = min(k0 + u, K - 1);
                    v[u] = dia_ld<NT>(vt + (size_t)kk * 64 + lane);
                    xv[u] = a.x[r + off[kk]];
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (k0 + u < K)
                        acc += v[u] * xv[u];
            }
        } else {
            for (int k0 = 0; k0 < K; k0 += U) {
                double v[U], xv[U];
                bool on[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int kk = min(k0 + u, K - 1);
                    on[u] = (mk[kk] >> lane) & 1ull;
                    v[u] = dia_ld<NT>(vt + (size_t)kk * 64 + lane);
                    xv[u] = a.x[on[u] ? r + off[kk] : 0];
                }
                // acc starts at +0.0 and never becomes -0.0, so adding +0.0 for an absent entry is
                // the identity: the sum is the row's CSR-order sum bit for bit
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (k0 + u < K)
                        acc += on[u] ? v[u] * xv[u] : 0.0;
            }
        }
        if (r < a.m)
            __builtin_nontemporal_store(acc, a.y + r);
    } else if constexpr (FORM == 2 || FORM == 3) {
        constexpr int GL = L / 2;
        const long long r = r0 + lane;
        double2 acc[GL];
#pragma unroll
        for (int j = 0; j < GL; ++j)
            acc[j] = make_double2(0.0, 0.0);
        for (int k0 = 0; k0 < K; k0 += U) {
            double v[U];
            double2 xv[U][GL];
            bool on[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kk = min(k0 + u, K - 1);
                on[u] = masked ? ((mk[kk] >> lane) & 1ull) != 0 : true;
                v[u] = dia_ld<NT>(vt + (size_t)kk * 64 + lane);
                const double *xr = a.x + (on[u] ? r + off[kk] : 0) * a.ld;
#pragma unroll
                for (int j = 0; j < GL; ++j)
                    xv[u][j] = *reinterpret_cast<const double2 *>(xr + 2 * j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (k0 + u >= K)
                    break;
#pragma unroll
                for (int j = 0; j < GL; ++j) {
                    acc[j].x += on[u] ? v[u] * xv[u][j].x : 0.0;
                    acc[j].y += on[u] ? v[u] * xv[u][j].y : 0.0;
                }
            }
        }
        if (r < a.m) {
#pragma unroll
            for (int j = 0; j < GL; ++j)
                __builtin_nontemporal_store(v2d_t{acc[j].x, acc[j].y}, reinterpret_cast<v2d_t *>(a.y + r * a.ld + 2 * j));
        }
    } else {
        constexpr int GL = L / 2;    // lanes per panel row
        constexpr int RS = 64 / GL;  // panel rows per wave instruction
        const int c = lane % GL, rl = lane / GL;
        const double *__restrict__ xb = a.x + 2 * c;
        double2 acc[GL];
#pragma unroll
        for (int q = 0; q < GL; ++q)
            acc[q] = make_double2(0.0, 0.0);
        for (int k0 = 0; k0 < K; k0 += U) {
            double v[U][GL];
            double2 xv[U][GL];
            unsigned long long mw[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kk = min(k0 + u, K - 1);
                const long long d = off[kk];
                mw[u] = masked ? mk[kk] : ~0ull;
                double vl = 0.0;
                if constexpr (FORM == 1)
                    vl = dia_ld<NT>(vt + (size_t)kk * 64 + lane);
#pragma unroll
                for (int q = 0; q < GL; ++q) {
                    const int row = rl + RS * q;
                    if constexpr (FORM == 1)
                        v[u][q] = __shfl(vl, row);
                    else
                        v[u][q] = dia_ld<NT>(vt + (size_t)kk * 64 + row);
                    const long long xr = ((mw[u] >> row) & 1ull) ? r0 + row + d : 0;
                    xv[u][q] = *reinterpret_cast<const double2 *>(xb + xr * a.ld);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (k0 + u >= K)
                    break;
#pragma unroll
                for (int q = 0; q < GL; ++q) {
                    const bool on = (mw[u] >> (rl + RS * q)) & 1ull;
                    acc[q].x += on ? v[u][q] * xv[u][q].x : 0.0;
                    acc[q].y += on ? v[u][q] * xv[u][q].y : 0.0;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < GL; ++q) {
            const long long r = r0 + rl + RS * q;
            if (r < a.m)
                __builtin_nontemporal_store(v2d_t{acc[q].x, acc[q].y},
                                            reinterpret_cast<v2d_t *>(a.y + r * a.ld + 2 * c));
        }
    }
}

// Plan time: each window's values into its lane-major panel (the offsets were checked on the host:
// every row's offsets ascend and each is in the window's list).
__global__ __launch_bounds__(kDiaThreads) void k_dia_fill(const int *__restrict__ ro, const int *__restrict__ ci,
                                                         const double *__restrict__ vals, const int4 *__restrict__ hdr,
                                                         const int *__restrict__ off, int windows, int m,
                                                         double *__restrict__ vt)
{
    const int w = blockIdx.x * kDiaWaves + ((int)threadIdx.x >> 6);
    if (w >= windows)
        return;
    const int lane = threadIdx.x & 63;
    const int r = w * 64 + lane;
    if (r >= m)
        return;
    const int4 hd = hdr[w];
    const int *D = off + hd.y;
    int k = 0;
    for (int j = ro[r]; j < ro[r + 1]; ++j) {
        const int d = ci[j] - r;
        while (k < hd.x && D[k] < d)
            ++k;
        if (k < hd.x)
            vt[((size_t)hd.z + k) * 64 + lane] = vals[j];
        ++k;
    }
}

template <typename T>
static void dia_free(T *&p)
{
    if (p)
        (void)hipFree((void *)p);
    p = nullptr;
}

void free_dia(DiaData *d)
{
    if (!d)
        return;
    dia_free(d->d_hdr);
    dia_free(d->d_off);
    dia_free(d->d_mask);
    dia_free(d->d_vt);
    delete d;
}

template <typename T>
static mspmv_status dia_upload(T **d, const std::vector<T> &hsrc)
{
    const size_t bytes = sizeof(T) * hsrc.size();
    if (hipMalloc((void **)d, bytes ? bytes : sizeof(T)) != hipSuccess) {
        *d = nullptr;
        set_error("offset-window plan: hipMalloc failed");
        return MSPMV_ERR_HIP;
    }
    if (!hsrc.empty() && hipMemcpy(*d, hsrc.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
        set_error("offset-window plan: upload failed");
        return MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}

mspmv_status build_dia_plan(mspmv_handle_s *h, TilePlan &p, double min_fill, double min_window_fill)
{
    const int m = h->m;
    if (m <= 0 || h->nnz <= 0)
        return MSPMV_ERR_UNSUPPORTED;
    std::vector<int> ro((size_t)m + 1);
    if (hipMemcpy(ro.data(), h->d_row_offsets, sizeof(int) * ro.size(), hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("offset-window plan: row offsets download failed");
        return MSPMV_ERR_HIP;
    }
    for (int r = 0; r < m; ++r)  // a row longer than the list: no window can hold it
        if (ro[(size_t)r + 1] - ro[(size_t)r] > kDiaMaxK)
            return MSPMV_ERR_UNSUPPORTED;
    std::vector<int> ci((size_t)h->nnz);
    if (hipMemcpy(ci.data(), h->d_cols, sizeof(int) * ci.size(), hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("offset-window plan: column download failed");
        return MSPMV_ERR_HIP;
    }
    const int W = (m + 63) / 64;
    std::vector<int> kw((size_t)W, 0), dl((size_t)W * kDiaMaxK, 0);
    std::vector<unsigned char> full((size_t)W, 0);
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int w = 0; w < W; ++w) {
        if (bad)
            continue;
        const int r0 = w * 64, r1 = std::min(m, r0 + 64);
        std::vector<int> d;
        d.reserve((size_t)(ro[(size_t)r1] - ro[(size_t)r0]));
        bool ok = true;
        for (int r = r0; r < r1 && ok; ++r) {
            long long prev = -(1LL << 40);
            for (int j = ro[(size_t)r]; j < ro[(size_t)r + 1]; ++j) {
                const long long o = (long long)ci[(size_t)j] - r;
                if (o <= prev) {  // columns not strictly ascending: the D order would not be the CSR order
                    ok = false;
                    break;
                }
                prev = o;
                d.push_back((int)o);
            }
        }
        if (ok) {
            std::sort(d.begin(), d.end());
            d.erase(std::unique(d.begin(), d.end()), d.end());
            const int K = (int)d.size();
            const long long nz = ro[(size_t)r1] - ro[(size_t)r0];
            ok = K >= 1 && K <= kDiaMaxK && (double)nz >= min_window_fill * (double)(r1 - r0) * K;
            if (ok) {
                kw[(size_t)w] = K;
                std::copy(d.begin(), d.end(), dl.begin() + (size_t)w * kDiaMaxK);
                full[(size_t)w] = (r1 - r0 == 64 && nz == 64LL * K) ? 1 : 0;
            }
        }
        if (!ok)
            bad = 1;
    }
    if (bad)
        return MSPMV_ERR_UNSUPPORTED;
    long long sumk = 0, summ = 0;
    for (int w = 0; w < W; ++w)
        sumk += kw[(size_t)w];
    if (sumk > 0x7fffffffLL || (double)h->nnz < min_fill * 64.0 * (double)sumk)
        return MSPMV_ERR_UNSUPPORTED;  // the panels would stream too many zeros overall
    std::vector<int4> hdr((size_t)W);
    std::vector<int> offs;
    offs.reserve((size_t)sumk);
    sumk = 0;
    for (int w = 0; w < W; ++w) {
        const int K = kw[(size_t)w];
        hdr[(size_t)w] = make_int4(K, (int)sumk, (int)sumk, full[(size_t)w] ? -1 : (int)summ);
        offs.insert(offs.end(), dl.begin() + (size_t)w * kDiaMaxK, dl.begin() + (size_t)w * kDiaMaxK + K);
        sumk += K;
        if (!full[(size_t)w])
            summ += K;
    }
    std::vector<unsigned long long> masks((size_t)summ, 0ull);
#pragma omp parallel for schedule(static)
    for (int w = 0; w < W; ++w) {
        const int4 hd = hdr[(size_t)w];
        if (hd.w < 0)
            continue;
        const int *D = &offs[(size_t)hd.y];
        const int r0 = w * 64, r1 = std::min(m, r0 + 64);
        for (int r = r0; r < r1; ++r) {
            int k = 0;
            for (int j = ro[(size_t)r]; j < ro[(size_t)r + 1]; ++j) {
                const int o = ci[(size_t)j] - r;
                while (D[k] < o)
                    ++k;
                masks[(size_t)hd.w + k] |= 1ull << (r - r0);
                ++k;
            }
        }
    }
    auto *dd = new DiaData();
    p.dia = dd;
    dd->windows = W;
    dd->sum_k = sumk;
    dd->masked_windows = 0;
    for (int w = 0; w < W; ++w) {
        dd->max_k = std::max(dd->max_k, kw[(size_t)w]);
        dd->masked_windows += !full[(size_t)w];
    }
    dd->fill = (double)h->nnz / (64.0 * (double)sumk);
    mspmv_status st;
    if ((st = dia_upload(&dd->d_hdr, hdr)) != MSPMV_OK || (st = dia_upload(&dd->d_off, offs)) != MSPMV_OK ||
        (st = dia_upload(&dd->d_mask, masks)) != MSPMV_OK)
        return st;
    if (hipMalloc((void **)&dd->d_vt, sizeof(double) * 64 * (size_t)sumk) != hipSuccess) {
        dd->d_vt = nullptr;
        set_error("offset-window plan: value panel allocation failed");
        return MSPMV_ERR_OOM;
    }
    hipError_t e = hipMemsetAsync(dd->d_vt, 0, sizeof(double) * 64 * (size_t)sumk, h->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_dia_fill, dim3((unsigned)((W + kDiaWaves - 1) / kDiaWaves)), dim3(kDiaThreads), 0,
                           h->stream, h->d_row_offsets, h->d_cols, h->d_vals, dd->d_hdr, dd->d_off, W, m, dd->d_vt);
        e = hipGetLastError();
    }
    // the plan as the tile-plan queries see it: one "tile" per window, whole rows, every row summed in
    // CSR order (mode 1: bit-identical), no split rows
    std::vector<int2> hb((size_t)W + 1);
    for (int w = 0; w <= W; ++w) {
        const int r = std::min(m, w * 64);
        hb[(size_t)w] = make_int2(r, ro[(size_t)r]);
    }
    if (e == hipSuccess && hipMalloc((void **)&p.d_bounds, sizeof(int2) * hb.size()) != hipSuccess)
        e = hipErrorOutOfMemory;
    if (e == hipSuccess)
        e = hipMemcpy(p.d_bounds, hb.data(), sizeof(int2) * hb.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && hipMalloc((void **)&p.d_split, (size_t)W + 1) != hipSuccess)
        e = hipErrorOutOfMemory;
    if (e == hipSuccess)
        e = hipMemset(p.d_split, 0, (size_t)W + 1);
    for (int i = 0; i < 5 && e == hipSuccess; ++i) {
        if (hipMalloc((void **)&p.d_modes[i], (size_t)W) != hipSuccess)
            e = hipErrorOutOfMemory;
        else
            e = hipMemset(p.d_modes[i], 1, (size_t)W);
    }
    if (e == hipSuccess)
        e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        set_error(std::string("offset-window plan: ") + hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? MSPMV_ERR_OOM : MSPMV_ERR_HIP;
    }
    p.lanes = 64;
    p.tile_items = 64;
    p.num_tiles = W;
    p.snap = 0;
    return MSPMV_OK;
}

static int dia_form()
{
    static const int f = [] {
        const char *e = getenv("MSPMV_DIA_FORM");
        return e && *e ? atoi(e) : 1;
    }();
    return f;
}

template <int L, int FORM>
static void dia_launch_form(const DiaArgs &a, hipStream_t s, bool nt)
{
    const dim3 grid((unsigned)a.groups), block(kDiaThreads);
    if (nt)
        hipLaunchKernelGGL((k_spmm_dia<L, true, FORM>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((k_spmm_dia<L, false, FORM>), grid, block, 0, s, a);
}

template <int L>
static void dia_launch_L(const DiaArgs &a, hipStream_t s, bool nt)
{
    if constexpr (L == 1) {
        dia_launch_form<1, 0>(a, s, nt);
    } else {
        switch (dia_form()) {
        case 1: dia_launch_form<L, 1>(a, s, nt); break;
        case 2: dia_launch_form<L, 2>(a, s, nt); break;
        case 3: dia_launch_form<L, 3>(a, s, nt); break;
        case 4: dia_launch_form<L, 4>(a, s, nt); break;
        default: dia_launch_form<L, 0>(a, s, nt); break;
        }
    }
}

hipError_t launch_dia(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L, int ld,
                      const CgControl *ctrl)
{
    const DiaData *dd = plan.dia;
    if (!dd)
        return hipErrorInvalidValue;
    if (dd->windows == 0)
        return hipSuccess;
    DiaArgs a{};
    a.hdr = dd->d_hdr;
    a.off = dd->d_off;
    a.mask = dd->d_mask;
    a.vt = dd->d_vt;
    a.x = d_X;
    a.y = d_Y;
    a.ctrl = ctrl;
    a.windows = dd->windows;
    a.groups = (dd->windows + kDiaWaves - 1) / kDiaWaves;
    a.m = h->m;
    a.ld = ld > 0 ? ld : L;
    const bool nt = stream_nt(h);
    switch (L) {
    case 1: dia_launch_L<1>(a, h->stream, nt); break;
    case 2: dia_launch_L<2>(a, h->stream, nt); break;
    case 4: dia_launch_L<4>(a, h->stream, nt); break;
    case 8: dia_launch_L<8>(a, h->stream, nt); break;
    case 16: dia_launch_L<16>(a, h->stream, nt); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

std::string dia_kernel_name(const mspmv_handle_s *h, int L)
{
    const int f = L == 1 ? 0 : dia_form();
    return "k_spmm_dia<" + std::to_string(L) + "," + (stream_nt(h) ? "true" : "false") + "," + std::to_string(f) + ">";
}

}  // namespace mspmv
