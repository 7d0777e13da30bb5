// mspmv_dia.hip -- offset windows: SpMV / SpMM for structured-grid rows (round 5).
//
// A window is 64 consecutive rows.  Where the rows of a window list their columns at a few common
// offsets from the row index (col - row: a finite-difference or finite-volume stencil, the 27-point
// nlpkkt120-size shape, parabolic_fem's 7-point triangles), the window is stored as its sorted offset
// list D (K <= kDiaMaxK entries) and its values lane-major in pairs of offsets: values 2p and 2p+1 of
// the window's row l at vt[p][l][0..1] (0 where row l has no column at offset D[k]; a 64-bit presence
// mask per (window, k) then says which rows hold it).  One wave computes one window with lane = row:
// per two offsets it loads vt[p][lane] (16 B per lane, 1 KB per wave instruction: 8-B loads streamed
// the panels at 5.2 TB/s, r05u) and x[row + D[k]] (64 consecutive rows: contiguous), so there is no
// column stream (8 B per nonzero from HBM instead of 10-12), no gather of scattered lines, no LDS and
// no cross-lane reduction.  Each row is summed from 0.0 in D order, which is its CSR order
// (the planner requires every row's columns strictly ascending), as mul then add: bit-identical to
// SpmvGold (cpu_spmv.cpp:241-265) and, per column, to the reference's row-by-row SpMM
// (work_2025/spmm/cpu_spmm.cpp), whose merge-path OmpMergeCsrmv / OmpMergeCsrmm
// (merge_based.hpp:46-153) differ from these only by the reordering of split rows.
//
// L-wide panels (row-major, row stride ld): lanes form groups of L/2 (one double2 of a panel row
// each); a wave instruction reads 64/(L/2) consecutive panel rows -- 1 KB contiguous -- and a lane
// holds L/2 rows of the window.
//
// Windows plus a remainder (round 6; round 5's plan was all or nothing): each window keeps the offsets
// most of its rows hold (dia_plan_host: >= kDiaKeepRows rows, <= kDiaMaxK = 64 of them, its panels >=
// min_window_fill full), and every other entry -- an off-pattern column, a row longer than the list --
// goes to a remainder CSR over the same rows that the kernels add after the row's offsets.  The plan
// holds when the remainder is <= kDiaMaxRemFrac of the nonzeros and the kept entries fill >= min_fill
// of the panels (the zeros of rows missing an offset -- grid boundaries -- are streamed too); anything
// else keeps the tile plans.
#include "mspmv_device.h"
#include "mspmv_internal.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
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
    double *partials;                // dot mode: x.(A x) per column per window, [windows][L] (launch_fold_dot)
    const double *xr;                // dot mode: x at this matrix's rows (x + row_off * ld for a row-range view)
    // the remainder (entries off the window's offset list): a CSR over all rows, summed after the offsets
    const int *rem_ptr;
    const int *rem_col;
    const double *rem_val;
    int windows;
    int groups;                      // workgroups (windows / 4, rounded up)
    int m;
    int n;                           // columns (X rows)
    int ld;                          // panel row stride (L-wide products)
};

// Runs of consecutive offsets (d, d+1, ..., d+g-1; g <= kDiaRun) read the same X panel rows shifted by
// one row per offset: form 5 stages the run's 64 + g - 1 rows once in LDS.
constexpr int kDiaRun = 4;

template <bool NT>
__device__ __forceinline__ double dia_ld(const double *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <bool NT>
__device__ __forceinline__ v2d_t dia_ld2(const v2d_t *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// The window's metadata -- offsets, presence masks, run lengths -- is loaded once into lanes (lane k:
// offset k) and read as wave-uniform values with v_readlane: no memory operation per offset, so no
// scalar-load chain before each x load and no vmcnt wait that would drain a prefetch (r05s).
//
// L = 1: lane = row, U offsets in flight (U/2 pair loads of the panel, U x loads).
// L > 1 (X row-major, L/2 lanes per panel row, a lane holding L/2 rows of the window): the window's
// offsets taken run by run (d, d+1, ..., d+g-1, g <= kDiaRun: a stencil's x-line neighbours), each run's
// 64 + g - 1 panel rows loaded ONCE -- 1 KB contiguous per wave instruction -- and staged in LDS, where
// the g offsets read them shifted by one row each; the next run's rows and values are loaded while this
// run is summed.  A row's value for offset k comes from the lane holding the row (lane = row) by a
// shuffle.  nlpkkt120 size, L = 8 (r05q-r05t): 369-374 us against 440 on the
// merge tiles; gathering every offset's rows directly (no LDS) 460-497 us, one row per lane 586 us.
// DOT (the block CG's SpMM): each window also writes its rows' x.(A x) per column to a.partials (the x
// rows reloaded after the products -- they were staged moments before, cache hits), summed by
// launch_fold_dot, which replaces the separate p.Ap pass (k_pcg_dot) over p and Ap.
template <int L, bool NT, bool DOT = false>
__global__ __launch_bounds__(kDiaThreads) __attribute__((amdgpu_waves_per_eu(L == 1 ? 8 : 1))) void
k_spmm_dia(DiaArgs a)
{
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int w = xcd_tile(blockIdx.x, a.groups) * kDiaWaves + wv;
    if (w >= a.windows)
        return;
    if (a.ctrl && a.ctrl->done)
        return;
    const int lane = threadIdx.x & 63;
    const int4 hd = a.hdr[w];
    const int K = __builtin_amdgcn_readfirstlane(hd.x) & 0xffff;
    const bool has_rem = (__builtin_amdgcn_readfirstlane(hd.x) >> 16) != 0;
    const bool masked = __builtin_amdgcn_readfirstlane(hd.w) >= 0;
    const int lk = max(min(lane, K - 1), 0);
    const int offv = K ? a.off[__builtin_amdgcn_readfirstlane(hd.y) + lk] : 0;
    const unsigned long long mkv = masked && K ? a.mask[__builtin_amdgcn_readfirstlane(hd.w) + lk] : ~0ull;
    // value pairs of this window: pair p of lane l (offsets 2p, 2p+1 of row l) at vp[p * 64 + l]
    const v2d_t *__restrict__ vp = reinterpret_cast<const v2d_t *>(a.vt) + (size_t)__builtin_amdgcn_readfirstlane(hd.z) * 64;
    const int KP = (K + 1) >> 1;
    const long long r0 = (long long)w * 64;
    auto off_at = [&](int k) { return __builtin_amdgcn_readlane(offv, k); };
    auto mask_at = [&](int k) {
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)mkv, k);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(mkv >> 32), k);
        return ((unsigned long long)hi << 32) | lo;
    };
    auto pair_at = [&](int p) { return dia_ld2<NT>(vp + (size_t)min(p, KP - 1) * 64 + lane); };

    if constexpr (L == 1) {
        constexpr int U = 8;
        const long long r = r0 + lane;
        const long long nmax1 = (long long)a.n - 1;
        double acc = 0.0;
        // one batch of U offsets from k0.  MODE 0: every row holds every offset.  MODE 1 (EXACT, masked
        // windows): the absent entries selected out (acc starts at +0.0 and never becomes -0.0, so adding
        // +0.0 for them is the identity: the sum is the row's CSR-order sum bit for bit).  MODE 2 (masked
        // windows, first sweep): every offset summed at a clamped row -- an absent entry's panel value is 0.0,
        // so its product adds +-0.0, the identity, unless its x is Inf or NaN; a row that comes out non-finite
        // sends the window through MODE 1 again (the same bits as MODE 1 in every case, without its mask
        // tests).  GUARD stops at K (the last batch only).
        auto batch = [&](int k0, auto mode_c, auto guard_c, auto u_c) {
            constexpr int MODE = decltype(mode_c)::value;
            constexpr bool GUARD = decltype(guard_c)::value;
            constexpr int U = decltype(u_c)::value;
            v2d_t v[U / 2];
            double xv[U];
            bool on[U];
#pragma unroll
            for (int u = 0; u < U / 2; ++u)
                v[u] = pair_at((k0 >> 1) + u);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kk = GUARD ? min(k0 + u, K - 1) : k0 + u;
                on[u] = MODE == 1 ? ((mask_at(kk) >> lane) & 1ull) != 0 : true;
                const long long j = r + off_at(kk);
                xv[u] = a.x[MODE == 1 ? (on[u] ? j : 0) : MODE == 2 ? min(max(j, 0LL), nmax1) : j];
            }
            // (the guard is a select, not a break: a break let the compiler sink the loads under it and
            // issue them one round trip at a time -- K = 7 windows 8.0 -> 9.4 us, r05ab)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double pv = (u & 1 ? v[u >> 1].y : v[u >> 1].x) * xv[u];
                const bool use = (MODE != 1 || on[u]) && (!GUARD || k0 + u < K);
                acc += use ? pv : 0.0;
            }
        };
        // full batches of U, then the rest in one guarded batch of U or U/2 offsets (the 27-point stencil's
        // 3 left over would otherwise issue 5 clamped duplicate x loads and 2 pair loads per window)
        using U8 = std::integral_constant<int, U>;
        using U4 = std::integral_constant<int, U / 2>;
        const int kfull = K - K % U;
        auto windows = [&](auto mode_c) {
            acc = 0.0;
            for (int k0 = 0; k0 < kfull; k0 += U)
                batch(k0, mode_c, std::false_type{}, U8{});
            if (K - kfull > U / 2)
                batch(kfull, mode_c, std::true_type{}, U8{});
            else if (kfull < K)
                batch(kfull, mode_c, std::true_type{}, U4{});
        };
        if (!masked) {
            windows(std::integral_constant<int, 0>{});
        } else {
            windows(std::integral_constant<int, 2>{});
            if (__any(r < a.m && !__builtin_isfinite(acc)))  // wave-uniform
                windows(std::integral_constant<int, 1>{});
        }
        if (has_rem && r < a.m) {  // the row's remainder entries, in CSR order, after its offsets
            double ar = 0.0;
            for (int j = a.rem_ptr[r]; j < a.rem_ptr[r + 1]; ++j)
                ar += a.rem_val[j] * a.x[a.rem_col[j]];
            acc = acc + ar;  // + 0.0 for a row without any: acc is never -0.0, so the identity
        }
        if (r < a.m)
            __builtin_nontemporal_store(acc, a.y + r);
        if constexpr (DOT) {
            double d = r < a.m ? a.xr[r] * acc : 0.0;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1)
                d += __shfl_xor(d, off);
            if (lane == 0)
                a.partials[w] = d;
        }
    } else {
        constexpr int GL = L / 2;    // lanes per panel row
        constexpr int RS = 64 / GL;  // panel rows per wave instruction
        constexpr int SPAN = 64 + kDiaRun - 1;
        __shared__ v2d_t s_x[kDiaWaves][SPAN * GL];
        v2d_t *sx = s_x[wv];
        const int c = lane % GL, rl = lane / GL;
        const double *__restrict__ xb = a.x + 2 * c;
        const long long nmax = a.n - 1;
        // run length from each offset k (lane k): consecutive offsets, <= kDiaRun, within the list
        int runv = 1;
        {
            int step = 1;
#pragma unroll
            for (int j = 1; j < kDiaRun; ++j) {
                const int nxt = __shfl_down(offv, j);
                step = step && lane + j < K && nxt == offv + j;
                runv += step;
            }
        }
        v2d_t nx[GL], ne;
        double nv[kDiaRun];
        // offset k's value of row `lane`: one element of the pair panels (the L-wide products' values are a
        // small part of their traffic; 8-B loads keep the run's values in registers without pair selects)
        const double *__restrict__ vd = reinterpret_cast<const double *>(vp) + 2 * lane;
        const size_t lrow = (size_t)rl * a.ld;  // this lane's first span row, as an element offset
        auto fetch_vals = [&](int k, double (&dst)[kDiaRun]) {  // the values of the run from offset k
#pragma unroll
            for (int j = 0; j < kDiaRun; ++j) {
                const int kk = min(k + j, K - 1);
                dst[j] = dia_ld<NT>(vd + (size_t)(kk >> 1) * 128 + (kk & 1));
            }
        };
        auto fetch = [&](int k) {  // the run's panel span (clamped into X: rows outside it serve absent entries only)
            const long long d0 = off_at(k);
            const long long s0 = r0 + d0;  // the span's first row (wave-uniform)
            if (s0 >= 0 && s0 + 64 + kDiaRun - 2 <= nmax) {  // inside X: a scalar base and per-lane constants
                const size_t sb = (size_t)s0 * a.ld;
#pragma unroll
                for (int q = 0; q < GL; ++q) {
                    const size_t o = sb + lrow + (size_t)(RS * q) * a.ld;
                    nx[q] = *reinterpret_cast<const v2d_t *>(xb + o);
                }
                const size_t oe = sb + (size_t)(64 + min(rl, kDiaRun - 2)) * a.ld;
                ne = *reinterpret_cast<const v2d_t *>(xb + oe);
            } else {
#pragma unroll
                for (int q = 0; q < GL; ++q) {
                    const size_t o = (size_t)min(max(s0 + rl + RS * q, 0LL), nmax) * a.ld;
                    nx[q] = *reinterpret_cast<const v2d_t *>(xb + o);
                }
                const size_t oe = (size_t)min(max(s0 + 64 + min(rl, kDiaRun - 2), 0LL), nmax) * a.ld;
                ne = *reinterpret_cast<const v2d_t *>(xb + oe);
            }
            fetch_vals(k, nv);
        };
        // Lanes read panel rows other lanes of the wave wrote.  The hardware runs a wave's DS operations in
        // order; the compiler, reasoning per lane, could move a read of another lane's row above the write
        // (or the next run's writes above this run's reads): wave-scope fences around the hand-off.
        auto wave_sync = [] {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        v2d_t acc[GL];
        // EXACT: absent entries (presence mask bit clear) selected out of the sum.  Without it every offset is
        // summed as if all rows held it: an absent entry's panel value is 0.0, so its product is +-0.0 and adding
        // it leaves the row sum unchanged (a sum is never -0.0) -- unless the X element it meets is Inf or NaN.
        // Masked windows therefore run the plain sweep first and again EXACT only when a row came out
        // non-finite (whatever the cause): the same bits as the select form in every case, without its
        // 3 + 4 VALU per row per offset.
        auto sweep = [&](auto exact_c) {
            constexpr bool EXACT = decltype(exact_c)::value;
#pragma unroll
            for (int q = 0; q < GL; ++q)
                acc[q] = v2d_t{0.0, 0.0};
            // one run: its span to LDS, its values from buf; the next run's span and values in flight while it is
            // summed.  (Values loaded two runs ahead, two buffers alternating, measured even: L = 8 364-368 us
            // either way, r06l.)
            auto run = [&](int &k, double (&buf)[kDiaRun]) {
                wave_sync();
#pragma unroll
                for (int q = 0; q < GL; ++q)
                    sx[(rl + RS * q) * GL + c] = nx[q];
                if (rl < kDiaRun - 1)
                    sx[(64 + rl) * GL + c] = ne;
                wave_sync();
                double cv[kDiaRun];
#pragma unroll
                for (int j = 0; j < kDiaRun; ++j)
                    cv[j] = buf[j];
                const int gk = __builtin_amdgcn_readlane(runv, k), kc = k;
                k += gk;
                if (k < K)
                    fetch(k);
#pragma unroll
                for (int j = 0; j < kDiaRun; ++j) {
                    if (j >= gk)
                        break;
                    const unsigned long long mw = EXACT && masked ? mask_at(kc + j) : ~0ull;
                    if (mw == ~0ull) {  // every row holds this offset (wave-uniform), or the plain sweep
#pragma unroll
                        for (int q = 0; q < GL; ++q) {
                            const int row = rl + RS * q;
                            const double v = __shfl(cv[j], row);
                            const v2d_t xv = sx[(row + j) * GL + c];
                            acc[q].x += v * xv.x;
                            acc[q].y += v * xv.y;
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < GL; ++q) {
                            const int row = rl + RS * q;
                            const double v = __shfl(cv[j], row);
                            const v2d_t xv = sx[(row + j) * GL + c];
                            const bool on = (mw >> row) & 1ull;
                            acc[q].x += on ? v * xv.x : 0.0;
                            acc[q].y += on ? v * xv.y : 0.0;
                        }
                    }
                }
            };
            if (K > 0)
                fetch(0);
            for (int k = 0; k < K;)
                run(k, nv);
        };
        sweep(std::false_type{});
        if (masked) {
            bool bad = false;
#pragma unroll
            for (int q = 0; q < GL; ++q)
                bad |= !(__builtin_isfinite(acc[q].x) && __builtin_isfinite(acc[q].y));
            if (__any(bad))  // wave-uniform
                sweep(std::true_type{});
        }
        if (has_rem) {  // the rows' remainder entries, in CSR order, after their offsets
#pragma unroll
            for (int q = 0; q < GL; ++q) {
                const long long r = r0 + rl + RS * q;
                if (r >= a.m)
                    continue;
                v2d_t ar = v2d_t{0.0, 0.0};
                for (int j = a.rem_ptr[r]; j < a.rem_ptr[r + 1]; ++j) {
                    const double v = a.rem_val[j];
                    const size_t o = (size_t)a.rem_col[j] * a.ld;
                    const v2d_t xv = *reinterpret_cast<const v2d_t *>(xb + o);
                    ar[0] += v * xv[0];
                    ar[1] += v * xv[1];
                }
                acc[q][0] = acc[q][0] + ar[0];
                acc[q][1] = acc[q][1] + ar[1];
            }
        }
#pragma unroll
        for (int q = 0; q < GL; ++q) {
            const long long r = r0 + rl + RS * q;
            if (r < a.m)
                __builtin_nontemporal_store(acc[q], reinterpret_cast<v2d_t *>(a.y + r * a.ld + 2 * c));
        }
        if constexpr (DOT) {  // column pair c: the lane's rows in q order, then the wave's rows by a fixed butterfly
            v2d_t d = v2d_t{0.0, 0.0};
#pragma unroll
            for (int q = 0; q < GL; ++q) {
                const long long r = r0 + rl + RS * q;
                if (r < a.m) {
                    const v2d_t xv = *reinterpret_cast<const v2d_t *>(a.xr + 2 * c + r * a.ld);
                    d.x += xv.x * acc[q].x;
                    d.y += xv.y * acc[q].y;
                }
            }
#pragma unroll
            for (int off = 32; off >= GL; off >>= 1) {
                d.x += __shfl_xor(d.x, off);
                d.y += __shfl_xor(d.y, off);
            }
            if (rl == 0)
                *reinterpret_cast<v2d_t *>(a.partials + (size_t)w * L + 2 * c) = d;
        }
    }
}

// ---- pipelined single-RHS CG on the offset windows -----------------------------------------------
// The two-kernel pipelined CG (mspmv_kernels.hip: [SpMV MODE 1] -> [k_cg1_update]) with its SpMV on the
// windows instead of the merge tiles, for the single-RHS matrices the register-resident kernel does not
// hold: a 27-point stencil of pwtk's size runs the plain product in 20 us on the windows against 60 us on
// the tiles, and the tiles' CG form took 78 us (r06f).  One launch of iteration k:
//  * head: every workgroup sums the update's <= kUpdateMaxBlocks r.r partials in one fixed order
//    (part_sum), so all take the same stop test and beta = rs_k / rs_{k-1} (cg1_head; no ticket chain);
//  * products: x = p_k = r_k + beta p_{k-1}, formed at each load from the {r, p_{k-1}} pair (cg_rp: one
//    16-B load per lane, contiguous across the window's rows) -- UpdatePSingle fused into the SpMV as the
//    tile form does -- summed per row in D order then the remainder, as k_spmm_dia<1>;
//  * own rows: p_k stored into the next {r, p} buffer's p slot, Ap, and the deferred x += alpha_{k-1}
//    p_{k-1} (cg1_lag_*: alpha from scal[0].alpha, p_{k-1} the pair's second element);
//  * one p.Ap partial per workgroup (its four windows' rows by wave butterflies, then waves in order),
//    summed by k_cg1_update -- folded by group tickets first only beyond kConsumeTile workgroups.
struct Cg1DiaArgs {
    const double *rp;  // {r_k, p_{k-1}} interleaved
    double *rp_new;    // receives p_k at the odd slots (k_cg1_update then writes r_{k+1} at the even ones)
    double *xsol;
    double *ap;
    CgScalars *scal;
    CgControl *ctrl;
    const double *part_in;  // the update's (or init's) r.r partials
    int n_part_in;
    double *partials;       // [groups] p.Ap partials (+ fold levels beyond kConsumeTile)
    unsigned *gtickets;
    int parity;
    double tol;
    double *hist;
    int hist_cap;
};

template <bool NT>
__global__ __launch_bounds__(kDiaThreads) void k_cg1_dia(DiaArgs a, Cg1DiaArgs c)
{
    constexpr int U = 8;
    static_assert(kDiaThreads == kBlock, "block_sum / publish_partials assume kBlock threads");
    __shared__ double s_red[kBlock / 64];
    __shared__ double s_tmp[kBlock];
    __shared__ double s_out[1];
    __shared__ int s_flag;
    if (c.ctrl->done)  // block-uniform
        return;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int g = xcd_tile(blockIdx.x, a.groups);
    const int w = g * kDiaWaves + wv;
    const bool live = w < a.windows;  // a wave past the last window still joins the block's sums
    const int lane = threadIdx.x & 63;
    PartRegs<kUpdateMaxBlocks / kBlock> pin;
    part_load(c.part_in, c.n_part_in, pin);
    const long long r = (long long)w * 64 + lane;
    const bool own = live && r < a.m;
    const long long nmax1 = (long long)a.n - 1;
    const v2d_t *__restrict__ rp2 = reinterpret_cast<const v2d_t *>(c.rp);
    // the deferred x term's operands and this row's own {r_k, p_{k-1}}, loaded under the head's sum
    const int kit = c.ctrl->iter_par[c.parity];
    const double alpha_prev = c.scal[0].alpha;
    v2d_t rpo = v2d_t{0.0, 0.0};
    double xo = 0.0;
    if (own) {
        rpo = rp2[r];
        xo = c.xsol[r];
    }
    const int4 hd = live ? a.hdr[w] : make_int4(0, 0, 0, -1);
    const int K = __builtin_amdgcn_readfirstlane(hd.x) & 0xffff;
    const bool has_rem = (__builtin_amdgcn_readfirstlane(hd.x) >> 16) != 0;
    const bool masked = __builtin_amdgcn_readfirstlane(hd.w) >= 0;
    const int lk = max(min(lane, K - 1), 0);
    const int offv = K ? a.off[__builtin_amdgcn_readfirstlane(hd.y) + lk] : 0;
    const unsigned long long mkv = masked && K ? a.mask[__builtin_amdgcn_readfirstlane(hd.w) + lk] : ~0ull;
    const v2d_t *__restrict__ vp = reinterpret_cast<const v2d_t *>(a.vt) + (size_t)__builtin_amdgcn_readfirstlane(hd.z) * 64;
    const int KP = (K + 1) >> 1;
    auto off_at = [&](int k) { return __builtin_amdgcn_readlane(offv, k); };
    auto mask_at = [&](int k) {
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)mkv, k);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(mkv >> 32), k);
        return ((unsigned long long)hi << 32) | lo;
    };
    auto pair_at = [&](int p) { return dia_ld2<NT>(vp + (size_t)min(p, KP - 1) * 64 + lane); };
    double beta = 0.0;
    if (!cg1_head(c, part_sum(pin, s_red), beta))  // block-uniform: converged
        return;
    auto pk = [&](v2d_t q) { return q.x + beta * q.y; };  // p_k from {r_k, p_{k-1}}: one expression everywhere
    double acc = 0.0;
    // (k_spmm_dia<1>'s batches.  Issuing the first batch's loads ahead of the head's sum measured no faster:
    // 37.4 vs 37.0 us per iteration, r06h.)
    auto batch = [&](int k0, auto mode_c, auto guard_c, auto u_c) {  // MODE as k_spmm_dia<1>'s batches
        constexpr int MODE = decltype(mode_c)::value;
        constexpr bool GUARD = decltype(guard_c)::value;
        constexpr int UU = decltype(u_c)::value;
        v2d_t v[UU / 2];
        v2d_t xq[UU];
        bool on[UU];
#pragma unroll
        for (int u = 0; u < UU / 2; ++u)
            v[u] = pair_at((k0 >> 1) + u);
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            const int kk = GUARD ? min(k0 + u, K - 1) : k0 + u;
            on[u] = MODE == 1 ? ((mask_at(kk) >> lane) & 1ull) != 0 : true;
            const long long j = r + off_at(kk);
            xq[u] = rp2[MODE == 1 ? (on[u] ? j : 0) : MODE == 2 ? min(max(j, 0LL), nmax1) : j];
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            const double pv = (u & 1 ? v[u >> 1].y : v[u >> 1].x) * pk(xq[u]);
            const bool use = (MODE != 1 || on[u]) && (!GUARD || k0 + u < K);
            acc += use ? pv : 0.0;
        }
    };
    using U8 = std::integral_constant<int, U>;
    using U4 = std::integral_constant<int, U / 2>;
    const int kfull = K - K % U;
    auto windows = [&](auto mode_c) {
        acc = 0.0;
        for (int k0 = 0; k0 < kfull; k0 += U)
            batch(k0, mode_c, std::false_type{}, U8{});
        if (K - kfull > U / 2)
            batch(kfull, mode_c, std::true_type{}, U8{});
        else if (kfull < K)
            batch(kfull, mode_c, std::true_type{}, U4{});
    };
    if (!masked) {
        windows(std::integral_constant<int, 0>{});
    } else {  // the clamped sweep first, the exact one when a row came out non-finite (k_spmm_dia<1>)
        windows(std::integral_constant<int, 2>{});
        if (__any(own && !__builtin_isfinite(acc)))
            windows(std::integral_constant<int, 1>{});
    }
    if (has_rem && own) {
        double ar = 0.0;
        for (int j = a.rem_ptr[r]; j < a.rem_ptr[r + 1]; ++j)
            ar += a.rem_val[j] * pk(rp2[a.rem_col[j]]);
        acc = acc + ar;
    }
    double dot = 0.0;
    if (own) {
        const double p = pk(rpo);
        c.rp_new[2 * r + 1] = p;
        c.ap[r] = acc;
        dot = p * acc;
        if (kit >= 1)  // iteration 0: x = 0 and nothing is pending
            c.xsol[r] = xo + alpha_prev * rpo.y;
    }
    const double tsum = block_sum(dot, s_red);
    if (a.groups <= kConsumeTile) {  // k_cg1_update sums them: the launch boundary orders the store
        if (threadIdx.x == 0)
            c.partials[g] = tsum;
        return;
    }
    if (threadIdx.x == 0) {  // a ticket tree folds them first: published at agent scope, drained
        store_sc1(&c.partials[g], tsum);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    publish_partials<1>(c.partials, c.gtickets, g, a.groups, kConsumeTile, s_tmp, s_out, &s_flag, c.ctrl);
}

hipError_t launch_cg1_dia(mspmv_handle_s *h, const TilePlan &plan, const double *rp_old, double *rp_new, double *d_x,
                          int parity, int nblk, double tol, int *nslots)
{
    const DiaData *dd = plan.dia;
    if (!dd || dd->windows == 0 || nblk > kUpdateMaxBlocks)
        return hipErrorInvalidValue;
    DiaArgs a{};
    a.hdr = dd->d_hdr;
    a.off = dd->d_off;
    a.mask = dd->d_mask;
    a.vt = dd->d_vt;
    a.windows = dd->windows;
    a.rem_ptr = dd->d_rem_ptr;
    a.rem_col = dd->d_rem_col;
    a.rem_val = dd->d_rem_val;
    a.groups = (dd->windows + kDiaWaves - 1) / kDiaWaves;
    a.m = h->m;
    a.n = h->n;
    a.ld = 1;
    Cg1DiaArgs c{};
    c.rp = rp_old;
    c.rp_new = rp_new;
    c.xsol = d_x;
    c.ap = h->d_ap;
    c.scal = h->d_scal;
    c.ctrl = h->d_ctrl;
    c.part_in = h->d_partials_b;
    c.n_part_in = nblk;
    c.partials = h->d_partials;
    c.gtickets = h->d_gtickets;
    c.parity = parity;
    c.tol = tol;
    c.hist = h->d_hist;
    c.hist_cap = h->hist_cap;
    *nslots = a.groups;
    const dim3 grid((unsigned)a.groups), block(kDiaThreads);
    if (stream_nt(h))
        hipLaunchKernelGGL((k_cg1_dia<true>), grid, block, 0, h->stream, a, c);
    else
        hipLaunchKernelGGL((k_cg1_dia<false>), grid, block, 0, h->stream, a, c);
    return hipGetLastError();
}

// Plan time: each window's values into its lane-major panel.  One workgroup per window streams the
// window's CSR entries coalesced (its row offsets and offset list in LDS; an entry finds its row and its
// offset index by binary searches there); entries off the list are the remainder's (k_dia_rem_fill).  The
// round-5 form (one lane per row walking its own entries) read 64 scattered lines per wave instruction:
// 23.8 GB moved to fill 1.2 GB of panels on the nlpkkt120 size.
__global__ __launch_bounds__(kDiaThreads) void k_dia_fill(const int *__restrict__ ro, const int *__restrict__ ci,
                                                         const double *__restrict__ vals, const int4 *__restrict__ hdr,
                                                         const int *__restrict__ off, int windows, int m,
                                                         double *__restrict__ vt)
{
    __shared__ int s_ro[65];
    __shared__ int s_d[kDiaMaxK];
    const int w = blockIdx.x;
    const int r0 = w * 64, nr = min(m - r0, 64);
    const int4 hd = hdr[w];
    const int K = hd.x & 0xffff;
    const int tid = threadIdx.x;
    if (tid <= nr)
        s_ro[tid] = ro[r0 + tid];
    if (tid < K)
        s_d[tid] = off[hd.y + tid];
    __syncthreads();
    if (K == 0)
        return;
    double *__restrict__ panel = vt + (size_t)hd.z * 128;
    for (int j = s_ro[0] + tid; j < s_ro[nr]; j += kDiaThreads) {
        int lo = 0, hi = nr - 1;  // the row: the last i with s_ro[i] <= j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_ro[mid] <= j)
                lo = mid;
            else
                hi = mid - 1;
        }
        const int d = ci[j] - (r0 + lo);
        int a = 0, b = K;  // lower bound of d in the offset list
        while (a < b) {
            const int mid = (a + b) >> 1;
            if (s_d[mid] < d)
                a = mid + 1;
            else
                b = mid;
        }
        if (a < K && s_d[a] == d)
            panel[(size_t)(a >> 1) * 128 + 2 * lo + (a & 1)] = vals[j];
    }
}

__global__ void k_dia_rem_fill(const double *__restrict__ vals, const int *__restrict__ src, long long n,
                               double *__restrict__ out)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        out[i] = vals[src[i]];
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
    dia_free(d->d_rem_ptr);
    dia_free(d->d_rem_col);
    dia_free(d->d_rem_val);
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

// The planning itself, on host arrays (build_dia_plan after downloading them; mspmv_offset_windows for
// inspection).  false: the plan does not hold.
//
// Windows plus a remainder (round 6; the round-5 plan was all or nothing): a window keeps the offsets
// that at least kDiaKeepRows of its rows hold (all of its rows when it has fewer), the kDiaMaxK most
// frequent when more qualify (ties: the smaller offset), and drops its rarest kept offsets while its
// kept entries fill less than min_window_fill of rows x K.  Every other entry -- an off-pattern column,
// a row longer than the list, a whole window of scattered columns -- goes to the REMAINDER: a CSR of the
// same rows (rem_ptr over all rows, rem_col, rem_src = the entry's CSR position), summed after the
// window's offsets (rows with remainder entries are within the reordering bound; the others keep the
// CSR-order sum bit for bit).  The plan holds when every row's columns ascend strictly, the remainder is
// at most max_rem_frac of the nonzeros and the kept entries fill >= min_fill of 64 x sum K.
constexpr int kDiaKeepRows = 8;

struct DiaHostPlan {
    int windows = 0, max_k = 0, masked = 0, rem_windows = 0;
    long long sum_k = 0, sum_pairs = 0, rem = 0;
    std::vector<int> kw;                     // [windows] K
    std::vector<int4> hdr;                   // [windows] {K | has_rem << 16, offset base, pair panel base, mask base or -1}
    std::vector<int> offs;                   // [sum_k]
    std::vector<unsigned long long> masks;   // [K of the masked windows]
    std::vector<int> rem_ptr;                // [m + 1] (empty when rem == 0)
    std::vector<int> rem_col, rem_src;       // [rem]
};

// One window's kept offsets (ascending) and their entry count; false when some row's columns do not
// ascend strictly.  ci[j - cbase] is the column of CSR entry j.
static bool window_offsets(const int *ro, const int *ci, long long cbase, int r0, int r1, double min_window_fill,
                           std::vector<std::pair<int, int>> &keep, long long &kept, bool all_offsets)
{
    std::vector<int> d;
    d.reserve((size_t)(ro[r1] - ro[r0]));
    for (int r = r0; r < r1; ++r) {
        long long prev = -(1LL << 40);
        for (int j = ro[r]; j < ro[r + 1]; ++j) {
            const long long o = (long long)ci[j - cbase] - r;
            if (o <= prev)  // columns not strictly ascending: the D order would not be the CSR order
                return false;
            prev = o;
            d.push_back((int)o);
        }
    }
    // offsets with their row counts (a row holds an offset at most once: columns strictly ascend)
    std::sort(d.begin(), d.end());
    std::vector<std::pair<int, int>> cnt;  // (offset, rows)
    for (size_t i = 0; i < d.size();) {
        size_t e = i;
        while (e < d.size() && d[e] == d[i])
            ++e;
        cnt.emplace_back(d[i], (int)(e - i));
        i = e;
    }
    // all_offsets (the exact plan, dia_plan_host's first attempt): the window keeps its whole offset list
    const int keep_min = all_offsets ? 1 : std::min(kDiaKeepRows, r1 - r0);
    keep.clear();
    for (const auto &c : cnt)
        if (c.second >= keep_min)
            keep.push_back(c);
    // the most frequent first (ties: the smaller offset), at most kDiaMaxK, then drop the rarest while the
    // window's panels would be too empty
    std::stable_sort(keep.begin(), keep.end(),
                     [](const std::pair<int, int> &a, const std::pair<int, int> &b) { return a.second > b.second; });
    if ((int)keep.size() > kDiaMaxK)
        keep.resize(kDiaMaxK);
    kept = 0;
    for (const auto &c : keep)
        kept += c.second;
    while (!keep.empty() && (double)kept < min_window_fill * (double)(r1 - r0) * (double)keep.size()) {
        kept -= keep.back().second;
        keep.pop_back();
    }
    std::sort(keep.begin(), keep.end());  // ascending offsets: each row's kept entries in CSR order
    return true;
}

static bool dia_plan_host_pass(const int *ro, const int *ci, int m, long long nnz, double min_fill,
                               double min_window_fill, double max_rem_frac, bool all_offsets, DiaHostPlan &out);

// Two passes: first every window keeps its whole offset list (round 5's plan: no remainder, every row
// summed in CSR order); only when that plan does not hold are the rare offsets left to the remainder.
static bool dia_plan_host(const int *ro, const int *ci, int m, long long nnz, double min_fill, double min_window_fill,
                          double max_rem_frac, DiaHostPlan &out)
{
    return dia_plan_host_pass(ro, ci, m, nnz, min_fill, min_window_fill, 0.0, true, out) ||
           dia_plan_host_pass(ro, ci, m, nnz, min_fill, min_window_fill, max_rem_frac, false, out);
}

static bool dia_plan_host_pass(const int *ro, const int *ci, int m, long long nnz, double min_fill,
                               double min_window_fill, double max_rem_frac, bool all_offsets, DiaHostPlan &out)
{
    if (m <= 0 || nnz <= 0)
        return false;
    const int W = (m + 63) / 64;
    std::vector<int> kw((size_t)W, 0), dl((size_t)W * kDiaMaxK, 0);
    std::vector<long long> kept_nz((size_t)W, 0);
    std::vector<int> rem_rows((size_t)m, 0);  // remainder entries per row
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int w = 0; w < W; ++w) {
        if (bad)
            continue;
        const int r0 = w * 64, r1 = std::min(m, r0 + 64);
        std::vector<std::pair<int, int>> keep;
        long long nz = 0;
        if (!window_offsets(ro, ci, 0, r0, r1, min_window_fill, keep, nz, all_offsets)) {
            bad = 1;
            continue;
        }
        kw[(size_t)w] = (int)keep.size();
        kept_nz[(size_t)w] = nz;
        for (size_t k = 0; k < keep.size(); ++k)
            dl[(size_t)w * kDiaMaxK + k] = keep[k].first;
        // remainder entries per row
        const int *D = &dl[(size_t)w * kDiaMaxK];
        const int K = (int)keep.size();
        for (int r = r0; r < r1; ++r) {
            int k = 0, nrem = 0;
            for (int j = ro[r]; j < ro[r + 1]; ++j) {
                const int o = ci[j] - r;
                while (k < K && D[k] < o)
                    ++k;
                if (k < K && D[k] == o)
                    ++k;
                else
                    ++nrem;
            }
            rem_rows[(size_t)r] = nrem;
        }
    }
    if (bad)
        return false;
    long long sumk = 0, kept = 0, rem = 0;
    for (int w = 0; w < W; ++w) {
        sumk += kw[(size_t)w];
        kept += kept_nz[(size_t)w];
    }
    rem = nnz - kept;
    if (sumk == 0 || sumk > 0x7fffffffLL || (double)kept < min_fill * 64.0 * (double)sumk ||
        (double)rem > max_rem_frac * (double)nnz)
        return false;  // the panels would stream too many zeros overall, or too much would be left over
    out.hdr.assign((size_t)W, make_int4(0, 0, 0, 0));
    out.offs.clear();
    out.offs.reserve((size_t)sumk);
    long long summ = 0, sump = 0, sk = 0;  // value pair panels (64 x 16 B): (K + 1) / 2 per window
    std::vector<unsigned char> wrem((size_t)W, 0);
    for (int w = 0; w < W; ++w) {
        const int r0 = w * 64, r1 = std::min(m, r0 + 64);
        for (int r = r0; r < r1; ++r)
            wrem[(size_t)w] |= rem_rows[(size_t)r] > 0;
    }
    for (int w = 0; w < W; ++w) {
        const int K = kw[(size_t)w];
        const int r0 = w * 64, r1 = std::min(m, r0 + 64);
        if (sump > 0x7fffffffLL / 64)
            return false;
        const bool full = r1 - r0 == 64 && kept_nz[(size_t)w] == 64LL * K;
        out.hdr[(size_t)w] = make_int4(K | (wrem[(size_t)w] ? 1 << 16 : 0), (int)sk, (int)sump, full ? -1 : (int)summ);
        sump += (K + 1) / 2;
        out.offs.insert(out.offs.end(), dl.begin() + (size_t)w * kDiaMaxK, dl.begin() + (size_t)w * kDiaMaxK + K);
        sk += K;
        if (!full)
            summ += K;
        out.max_k = std::max(out.max_k, K);
        out.masked += !full;
        out.rem_windows += wrem[(size_t)w];
    }
    out.masks.assign((size_t)summ, 0ull);
    if (rem > 0) {
        out.rem_ptr.assign((size_t)m + 1, 0);
        for (int r = 0; r < m; ++r)
            out.rem_ptr[(size_t)r + 1] = out.rem_ptr[(size_t)r] + rem_rows[(size_t)r];
        out.rem_col.assign((size_t)rem, 0);
        out.rem_src.assign((size_t)rem, 0);
    }
    const std::vector<int4> &hdr = out.hdr;
    const std::vector<int> &offs = out.offs;
    std::vector<unsigned long long> &masks = out.masks;
#pragma omp parallel for schedule(static)
    for (int w = 0; w < W; ++w) {
        const int4 hd = hdr[(size_t)w];
        const int K = hd.x & 0xffff;
        const int *D = K ? &offs[(size_t)hd.y] : nullptr;
        const int r0 = w * 64, r1 = std::min(m, r0 + 64);
        if (hd.w < 0 && !(hd.x >> 16))
            continue;  // every row holds every offset and nothing is left over
        for (int r = r0; r < r1; ++r) {
            int k = 0;
            int q = rem > 0 ? out.rem_ptr[(size_t)r] : 0;
            for (int j = ro[r]; j < ro[r + 1]; ++j) {
                const int o = ci[j] - r;
                while (k < K && D[k] < o)
                    ++k;
                if (k < K && D[k] == o) {
                    if (hd.w >= 0)
                        masks[(size_t)hd.w + k] |= 1ull << (r - r0);
                    ++k;
                } else {
                    out.rem_col[(size_t)q] = ci[j];
                    out.rem_src[(size_t)q] = j;
                    ++q;
                }
            }
        }
    }
    out.windows = W;
    out.sum_k = sk;
    out.sum_pairs = sump;
    out.rem = rem;
    out.kw = std::move(kw);
    return true;
}

// The cheap test before the whole column array is copied to the host: up to kDiaSamples windows spread
// over the matrix, planned as dia_plan_host plans them (their columns downloaded alone); the plan is
// not attempted when their entries would leave twice the remainder allowed or fill the panels clearly
// less than min_fill (FEM node blocks, random bands and power-law rows fail here in microseconds).
constexpr int kDiaSamples = 64;
static mspmv_status dia_sample_ok(const mspmv_handle_s *h, const int *ro, const int *host_ci, double min_fill,
                                  double min_window_fill, double max_rem_frac, bool *ok)
{
    const int m = h->m, W = (m + 63) / 64;
    const int S = std::min(W, kDiaSamples);
    long long total = 0, kept = 0, slots = 0;
    std::vector<int> buf;
    std::vector<std::pair<int, int>> keep;
    for (int i = 0; i < S; ++i) {
        const int w = (int)((long long)i * W / S);
        const int r0 = w * 64, r1 = std::min(m, r0 + 64);
        const long long j0 = ro[(size_t)r0], j1 = ro[(size_t)r1];
        const int *cw = host_ci ? host_ci + j0 : nullptr;
        if (!host_ci) {
            buf.resize((size_t)std::max(j1 - j0, 1LL));
            if (j1 > j0 &&
                hipMemcpy(buf.data(), h->d_cols + j0, sizeof(int) * (size_t)(j1 - j0), hipMemcpyDeviceToHost) != hipSuccess) {
                set_error("offset-window plan: sample download failed");
                return MSPMV_ERR_HIP;
            }
            cw = buf.data();
        }
        long long kw = 0;
        if (!window_offsets(ro, cw, j0, r0, r1, min_window_fill, keep, kw, false)) {
            *ok = false;
            return MSPMV_OK;
        }
        total += j1 - j0;
        kept += kw;
        slots += 64LL * (long long)keep.size();
    }
    *ok = total > 0 && slots > 0 && (double)(total - kept) <= 2.0 * max_rem_frac * (double)total &&
          (double)kept >= 0.9 * min_fill * (double)slots;
    return MSPMV_OK;
}

mspmv_status build_dia_plan(mspmv_handle_s *h, TilePlan &p, double min_fill, double min_window_fill)
{
    const int m = h->m;
    if (m <= 0 || h->nnz <= 0)
        return MSPMV_ERR_UNSUPPORTED;
    const double max_rem = min_fill > 0.0 ? kDiaMaxRemFrac : 1.0;  // forced (MSPMV_DIA=1): any remainder
    const int *ro = nullptr, *ci = nullptr;
    bool sample_ok = true;
    if (host_pattern_resident(h)) {  // the caller's arrays (mspmv_csr_create) or a shared copy: sample there
        mspmv_status st0 = host_pattern(h, &ro, &ci);
        if (st0 != MSPMV_OK)
            return st0;
        st0 = dia_sample_ok(h, ro, ci, min_fill, min_window_fill, max_rem, &sample_ok);
        if (st0 != MSPMV_OK)
            return st0;
        if (!sample_ok)
            return MSPMV_ERR_UNSUPPORTED;
    } else {  // sample the device's columns first: non-stencils never copy the whole pattern
        std::vector<int> ros((size_t)m + 1);
        if (hipMemcpy(ros.data(), h->d_row_offsets, sizeof(int) * ros.size(), hipMemcpyDeviceToHost) != hipSuccess) {
            set_error("offset-window plan: row offsets download failed");
            return MSPMV_ERR_HIP;
        }
        mspmv_status st0 = dia_sample_ok(h, ros.data(), nullptr, min_fill, min_window_fill, max_rem, &sample_ok);
        if (st0 != MSPMV_OK)
            return st0;
        if (!sample_ok)
            return MSPMV_ERR_UNSUPPORTED;
        if ((st0 = host_pattern(h, &ro, &ci)) != MSPMV_OK)
            return st0;
    }
    DiaHostPlan hp;
    if (!dia_plan_host(ro, ci, m, h->nnz, min_fill, min_window_fill, max_rem, hp))
        return MSPMV_ERR_UNSUPPORTED;
    const int W = hp.windows;
    const std::vector<int4> &hdr = hp.hdr;
    const std::vector<int> &offs = hp.offs;
    const std::vector<unsigned long long> &masks = hp.masks;
    const long long sumk = hp.sum_k, sump = hp.sum_pairs;
    auto *dd = new DiaData();
    p.dia = dd;
    dd->windows = W;
    dd->sum_k = sumk;
    dd->sum_pairs = sump;
    dd->masked_windows = hp.masked;
    dd->max_k = hp.max_k;
    dd->rem = hp.rem;
    dd->rem_windows = hp.rem_windows;
    dd->fill = (double)(h->nnz - hp.rem) / (64.0 * (double)sumk);
    mspmv_status st;
    if ((st = dia_upload(&dd->d_hdr, hdr)) != MSPMV_OK || (st = dia_upload(&dd->d_off, offs)) != MSPMV_OK ||
        (st = dia_upload(&dd->d_mask, masks)) != MSPMV_OK)
        return st;
    if (hp.rem > 0) {
        if ((st = dia_upload(&dd->d_rem_ptr, hp.rem_ptr)) != MSPMV_OK ||
            (st = dia_upload(&dd->d_rem_col, hp.rem_col)) != MSPMV_OK)
            return st;
        int *d_src = nullptr;
        if ((st = dia_upload(&d_src, hp.rem_src)) != MSPMV_OK) {
            dia_free(d_src);
            return st;
        }
        if (hipMalloc((void **)&dd->d_rem_val, sizeof(double) * (size_t)hp.rem) != hipSuccess) {
            dd->d_rem_val = nullptr;
            dia_free(d_src);
            set_error("offset-window plan: remainder allocation failed");
            return MSPMV_ERR_OOM;
        }
        hipLaunchKernelGGL(k_dia_rem_fill, dim3(1024), dim3(256), 0, h->stream, h->d_vals, d_src, hp.rem, dd->d_rem_val);
        const hipError_t e = hipStreamSynchronize(h->stream);
        dia_free(d_src);
        if (e != hipSuccess) {
            set_error(std::string("offset-window plan: remainder fill: ") + hipGetErrorString(e));
            return MSPMV_ERR_HIP;
        }
    }
    if (hipMalloc((void **)&dd->d_vt, sizeof(double) * 128 * (size_t)sump) != hipSuccess) {
        dd->d_vt = nullptr;
        set_error("offset-window plan: value panel allocation failed");
        return MSPMV_ERR_OOM;
    }
    hipError_t e = hipMemsetAsync(dd->d_vt, 0, sizeof(double) * 128 * (size_t)sump, h->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_dia_fill, dim3((unsigned)W), dim3(kDiaThreads), 0, h->stream, h->d_row_offsets, h->d_cols,
                           h->d_vals, dd->d_hdr, dd->d_off, W, m, dd->d_vt);
        e = hipGetLastError();
    }
    // the plan as the tile-plan queries see it: one "tile" per window, whole rows, every row summed in
    // CSR order (mode 1: bit-identical) -- except in windows with remainder entries, summed after the
    // offsets (mode 255: within the reordering bound) -- and no split rows
    std::vector<int2> hb((size_t)W + 1);
    std::vector<unsigned char> modes((size_t)W);
    for (int w = 0; w <= W; ++w) {
        const int r = std::min(m, w * 64);
        hb[(size_t)w] = make_int2(r, ro[(size_t)r]);
        if (w < W)
            modes[(size_t)w] = (hdr[(size_t)w].x >> 16) ? 255 : 1;
    }
    if (e == hipSuccess && hipMalloc((void **)&p.d_bounds, sizeof(int2) * hb.size()) != hipSuccess)
        e = hipErrorOutOfMemory;
    if (e == hipSuccess)
        e = hipMemcpy(p.d_bounds, hb.data(), sizeof(int2) * hb.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && hipMalloc((void **)&p.d_split, (size_t)W + 1) != hipSuccess)
        e = hipErrorOutOfMemory;
    if (e == hipSuccess)
        e = memset_sync(p.d_split, 0, (size_t)W + 1);
    for (int i = 0; i < 5 && e == hipSuccess; ++i) {
        if (hipMalloc((void **)&p.d_modes[i], (size_t)W) != hipSuccess)
            e = hipErrorOutOfMemory;
        else
            e = hipMemcpy(p.d_modes[i], modes.data(), (size_t)W, hipMemcpyHostToDevice);
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

template <int L>
static void dia_launch_L(const DiaArgs &a, hipStream_t s, bool nt)
{
    const dim3 grid((unsigned)a.groups), block(kDiaThreads);
    if (a.partials) {
        if (nt)
            hipLaunchKernelGGL((k_spmm_dia<L, true, true>), grid, block, 0, s, a);
        else
            hipLaunchKernelGGL((k_spmm_dia<L, false, true>), grid, block, 0, s, a);
    } else if (nt) {
        hipLaunchKernelGGL((k_spmm_dia<L, true>), grid, block, 0, s, a);
    } else {
        hipLaunchKernelGGL((k_spmm_dia<L, false>), grid, block, 0, s, a);
    }
}

hipError_t launch_dia(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L, int ld,
                      const CgControl *ctrl, double *partials, long long row_off, hipStream_t stream)
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
    a.partials = partials;
    a.windows = dd->windows;
    a.rem_ptr = dd->d_rem_ptr;
    a.rem_col = dd->d_rem_col;
    a.rem_val = dd->d_rem_val;
    a.xr = d_X + row_off * (ld > 0 ? ld : L);
    a.groups = (dd->windows + kDiaWaves - 1) / kDiaWaves;
    a.m = h->m;
    a.n = h->n;
    a.ld = ld > 0 ? ld : L;
    const bool nt = stream_nt(h);
    hipStream_t s = stream ? stream : h->stream;
    switch (L) {
    case 1: dia_launch_L<1>(a, s, nt); break;
    case 2: dia_launch_L<2>(a, s, nt); break;
    case 4: dia_launch_L<4>(a, s, nt); break;
    case 8: dia_launch_L<8>(a, s, nt); break;
    case 16: dia_launch_L<16>(a, s, nt); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

std::string dia_kernel_name(const mspmv_handle_s *h, int L)
{
    return "k_spmm_dia<" + std::to_string(L) + "," + (stream_nt(h) ? "true" : "false") + ">";
}

}  // namespace mspmv

extern "C" mspmv_status mspmv_offset_windows(const mspmv_csr_d *a, double min_fill, double min_window_fill, int *ok,
                                            int *num_windows, long long *sum_offsets, int *masked_windows,
                                            int *k_per_window, long long *remainder)
{
    using namespace mspmv;
    if (!a || !ok || a->num_rows < 0 || a->num_cols < 0 || a->num_nonzeros < 0 || !a->row_offsets ||
        (a->num_nonzeros > 0 && !a->column_indices)) {
        set_error("offset_windows: bad matrix or null output");
        return MSPMV_ERR_INVALID;
    }
    const int m = a->num_rows;
    const int *ro = a->row_offsets;
    if (ro[0] != 0 || ro[m] != a->num_nonzeros) {
        set_error("offset_windows: row offsets must run from 0 to num_nonzeros");
        return MSPMV_ERR_INVALID;
    }
    for (int r = 0; r < m; ++r)
        if (ro[r + 1] < ro[r]) {
            set_error("offset_windows: row offsets not monotone");
            return MSPMV_ERR_INVALID;
        }
    for (long long j = 0; j < a->num_nonzeros; ++j)
        if (a->column_indices[j] < 0 || a->column_indices[j] >= a->num_cols) {
            set_error("offset_windows: column index out of range");
            return MSPMV_ERR_INVALID;
        }
    DiaHostPlan hp;
    *ok = dia_plan_host(ro, a->column_indices, m, a->num_nonzeros, min_fill, min_window_fill,
                        min_fill > 0.0 ? kDiaMaxRemFrac : 1.0, hp) ? 1 : 0;
    if (remainder)
        *remainder = *ok ? hp.rem : 0;
    if (num_windows)
        *num_windows = *ok ? hp.windows : 0;
    if (sum_offsets)
        *sum_offsets = *ok ? hp.sum_k : 0;
    if (masked_windows)
        *masked_windows = *ok ? hp.masked : 0;
    if (k_per_window && *ok)
        std::copy(hp.kw.begin(), hp.kw.end(), k_per_window);
    return MSPMV_OK;
}
