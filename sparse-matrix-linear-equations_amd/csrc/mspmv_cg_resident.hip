// mspmv_cg_resident.hip -- CGSolveSingle (work_2025/main/single_strategy.hpp:102-170) as ONE
// persistent launch whose matrix, x, r and p stay on chip for the whole solve.
//
// MI355X holds 128 MB of vector registers and 40 MB of LDS.  A matrix of a few million nonzeros
// (configs[3]: parabolic_fem, 3.67 M) fits in them, so instead of streaming 44 MB of CSR from the
// Infinity Cache twice per iteration (two kernels, two launch boundaries) every CU keeps its row
// block resident and the iteration costs two in-launch reductions plus the gathers of p:
//   * one 1024-thread workgroup per CU (cooperative launch: all resident); workgroup w owns a
//     contiguous row block (merge-path balanced on rows + nonzeros; blocks dealt XCD-contiguously
//     so an XCD's L2 serves its neighbours' p); thread t owns rows t, t + 1024, ... (<= RPT) with
//     their values in registers (ELL, NZR slots per row) and their columns in LDS;
//   * p_k = r_k + beta p_{k-1} is formed on the fly from the {r_k, p_{k-1}} pair the owner
//     published (the same expression the owner evaluates for its own rows: bit-identical), so
//     the SpMV needs no hand-off of its own;
//   * per iteration two hand-offs: p.Ap and r.r.  Each workgroup stores its partial in its own
//     slot (one 8-B sc1 store after every wave's payload stores drained), one wave of every
//     workgroup polls all G slots (sc1 loads) until none holds the empty pattern and sums them in
//     slot order -- every workgroup gets the same total bit for bit, so all take the same branch;
//   * payload ({r, p} pairs) is stored write-through (sc1) and gathered with sc1 loads, the
//     one-workgroup-per-CU hand-off of MI355X_MICROARCH.md (no acquire / release fences);
//   * slots form a ring of kResRing iterations; an owner resets its slot kResRing/2 iterations
//     ahead (nobody can still be reading it: every workgroup is within one iteration of every
//     other).  Every spin is bounded: a timeout raises an abort word that every poller checks,
//     and the solve reports MSPMV_ERR_STALL instead of hanging the GPU.
// Semantics are the pipelined CG's (mspmv_kernels.hip k_cg1_*): x = 0, r = p = b, b_norm =
// ||b|| (1 if 0), per iteration alpha = rs / p.Ap (a non-finite alpha stops before x and r
// change: MSPMV_ERR_BREAKDOWN), x += alpha p, r += (-alpha) Ap, hist[k] = sqrt(rs_new) / b_norm,
// stop when it is < tol (iterations = k + 1), beta = rs_new / rs.  Row sums are sequential in CSR
// order (SpmvGold's order); the dot products are fixed-order trees.
#include "mspmv_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#define RES_HIP_TRY(expr)                                                                          \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            set_error(std::string("resident CG: ") + #expr + ": " + hipGetErrorString(_e));        \
            return (_e == hipErrorOutOfMemory) ? MSPMV_ERR_OOM : MSPMV_ERR_HIP;                    \
        }                                                                                          \
    } while (0)

namespace mspmv {

namespace {

constexpr int kRB = 1024;    // threads per workgroup: 16 waves, the whole CU
constexpr int kResRing = 8;  // iterations of p.Ap / r.r slots before an owner reuses its slot
constexpr unsigned long long kSlotEmpty = ~0ull;  // all-ones NaN (memset 0xFF): no arithmetic on finite data makes it
constexpr unsigned kResSpinMax = 1u << 21;        // polls before a workgroup declares the solve stalled

typedef unsigned v4u_t __attribute__((ext_vector_type(4)));

struct ResArgs {
    const int *rb;         // [G + 1] row bounds of the row blocks
    const int *cols;       // ELL [G][RPT][NZR][kRB]
    const double *vals;    // ELL [G][RPT][NZR][kRB]
    const short *len;      // [G][RPT][kRB] row length, -1: no row
    const double *b;
    double *x;
    double *pair0, *pair1;  // {r, p} per row (2 m doubles each), iteration k reads pair[k & 1]
    unsigned pair_bytes;    // 16 m (buffer resource size)
    double *slots;          // [(1 + 2 kResRing) G]: b.b, then {p.Ap, r.r} per ring position
    unsigned *abort_word;
    CgControl *ctrl;
    double *hist;
    int hist_cap;
    int max_iters;
    double tol;
    int G;
    // diagnostic solves only (mspmv_cg_resident_stamps): wall_clock64() of every workgroup at the
    // phase boundaries of iterations k < stamp_iters, [k][w][kResStamps]; null in every other solve
    unsigned long long *stamps;
    int stamp_iters;
    int force_stall;  // test switch (MSPMV_CG_RESIDENT_STALL): the first hand-off reports a stall
};
constexpr int kResStamps = 5;
constexpr bool kResPipelinedDefault = true;  // configs[3]: 14.3 -> 9.45 us per iteration (r05i)  // iteration start | Ap done | p.Ap summed | r done | r.r summed

__device__ __forceinline__ void st_sc1(double *p, double v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Row block of workgroup w: blocks are dealt round-robin over the 8 XCDs, so XCD k gets the
// contiguous blocks [k G/8, (k+1) G/8) (bijective for any G).
__device__ __forceinline__ int res_block(int w, int G)
{
    const int q = G >> 3, r = G & 7;
    const int k = w & 7, i = w >> 3;
    return k * q + (k < r ? k : r) + i;
}

// Sum of a 1024-thread workgroup in a fixed order (wave butterflies, then waves in order);
// the result is left in thread 0.
__device__ __forceinline__ double res_block_sum(double v, double *s_red)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0)
        s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0) {
        t = s_red[0];
#pragma unroll
        for (int w = 1; w < kRB / 64; ++w)
            t += s_red[w];
    }
    return t;
}

// Publish this workgroup's partial for one phase: every wave's payload stores (sc1) drain, the
// workgroup meets, one lane stores the partial (sc1) -- the flag of the hand-off.
// A NaN partial is published as the canonical quiet NaN: a payload equal to kSlotEmpty (b memset
// to 0xFF) would otherwise read as "not published yet" and the solve would stall instead of
// reporting the breakdown.  DRAIN: every storing wave's payload stores complete before the flag --
// needed only where the flag hands payload over (r.r: the {r, p} pairs the next iteration gathers);
// the p.Ap hand-off carries none (the p stores it follows are drained by the r.r publish, which every
// reader waits for before its next gathers), so its partial goes out without waiting for them.
template <bool DRAIN>
__device__ __forceinline__ void res_publish(double part, double *slot, double *s_red)
{
    if (DRAIN)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its payload is out
    double t = res_block_sum(part, s_red);             // (contains the workgroup barrier)
    if (threadIdx.x == 0) {
        if (t != t)
            t = __longlong_as_double(0x7ff8000000000000ll);
        st_sc1(slot, t);
    }
}

// Diagnostic phase stamp (thread 0, stamped solves only): a plain vector store of wall_clock64().
__device__ __forceinline__ void res_stamp(const ResArgs &a, int k, int w, int phase)
{
    if (a.stamps && threadIdx.x == 0 && k < a.stamp_iters)
        a.stamps[((size_t)k * a.G + w) * kResStamps + phase] = wall_clock64();
}

// Wave 0 polls the G slots of one phase (NV arrays of them, slot + q G) until none holds the empty
// pattern (s_sleep between rounds, bounded), lane l sums slots l, l + 64, ... of each array in order, a
// fixed butterfly folds the lanes; the totals land in s_tot[q] for the whole workgroup.  false: the
// solve stalled (timeout / abort).
template <int NSL, int NV = 1>
__device__ __forceinline__ bool res_wait_sum(const double *slot, int G, unsigned *abort_word, double *s_tot,
                                             int *s_ok)
{
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        double v[NV][NSL];
        unsigned have = 0;
        bool ok = true;
#pragma unroll
        for (int q = 0; q < NV; ++q)
#pragma unroll
            for (int j = 0; j < NSL; ++j)
                v[q][j] = 0.0;
        for (unsigned spin = 0;; ++spin) {
            bool miss = false;
#pragma unroll
            for (int q = 0; q < NV; ++q)
#pragma unroll
                for (int j = 0; j < NSL; ++j) {
                    const int i = lane + 64 * j;
                    const unsigned bit = 1u << (q * NSL + j);
                    if (!(have & bit)) {
                        if (i < G) {
                            const double x = ld_sc1(slot + (size_t)q * G + i);
                            if ((unsigned long long)__double_as_longlong(x) != kSlotEmpty) {
                                v[q][j] = x;
                                have |= bit;
                            } else {
                                miss = true;
                            }
                        } else {
                            have |= bit;
                        }
                    }
                }
            if (!__any(miss))
                break;
            if ((spin & 63) == 63 &&
                __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                ok = false;
                break;
            }
            if (spin >= kResSpinMax) {
                if (lane == 0)
                    __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            double t = v[q][0];
#pragma unroll
            for (int j = 1; j < NSL; ++j)
                t += v[q][j];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1)
                t += __shfl_xor(t, off);
            if (lane == 0)
                s_tot[q] = t;
        }
        if (lane == 0)
            *s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    return *s_ok != 0;
}

// Two partials of one workgroup published together (the pipelined form's r.r and w.r): fixed-order
// block sums (wave butterflies, waves in order), every storing wave's payload drained first, then the
// two flags.  NaN partials as res_publish.
__device__ __forceinline__ void res_publish2(double g, double d, double *slot_g, double *slot_d, double2 *s_red2)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its payload (w) is out
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        g += __shfl_xor(g, off);
        d += __shfl_xor(d, off);
    }
    if ((threadIdx.x & 63) == 0)
        s_red2[threadIdx.x >> 6] = make_double2(g, d);
    __syncthreads();
    if (threadIdx.x == 0) {
        double2 t = s_red2[0];
#pragma unroll
        for (int w = 1; w < kRB / 64; ++w) {
            t.x += s_red2[w].x;
            t.y += s_red2[w].y;
        }
        if (t.x != t.x)
            t.x = __longlong_as_double(0x7ff8000000000000ll);
        if (t.y != t.y)
            t.y = __longlong_as_double(0x7ff8000000000000ll);
        st_sc1(slot_g, t.x);
        st_sc1(slot_d, t.y);
    }
}

// The pipelined (single-reduction) form: Ghysels & Vanroose's pipelined CG without preconditioner,
// i.e. the Chronopoulos-Gear recurrence with the SpMV moved next to the reduction.  Per iteration ONE
// hand-off carries both dot products, gamma = r.r and delta = w.r (w = A r), and the payload the next
// SpMV gathers (w, published before the partials): the classic form needs two (p.Ap, then r.r with
// the {r, p} payload), and each costs 3-4 us on 256 workgroups (r04 stamps), about half an iteration.
//   i = 0: alpha = gamma / delta;  i > 0: beta = gamma_i / gamma_{i-1},
//          alpha = gamma_i / (delta_i - beta gamma_i / alpha_{i-1})
//   n = A w;  z = n + beta z;  s = w + beta s;  p = r + beta p;
//   x += alpha p;  r += (-alpha) s;  w += (-alpha) z;  then gamma, delta of the new r, w
// Exactly CGSolveSingle's iterates in exact arithmetic (alpha = r.r / p.Ap, beta, x, r), with the same
// stop test (||r_i|| / ||b|| < tol -> i iterations, hist[i-1]), breakdown rule (a non-finite alpha stops
// before x changes) and b_norm; the rounding differs (r and Ap come from recurrences), so it is held to
// the oracle's CGSolveSingle by the same parity bars as the classic form (tests/test_gpu_cg_resident.py).
// LDS vectors of the pipelined form next to the columns: x and p always, z too where it fits.
template <int RPT, int NZR>
constexpr int res_nxp()
{
    const int free = 163840 - RPT * NZR * kRB * 4 - 1024;
    return free >= 3 * RPT * kRB * 8 ? 3 : 2;
}

template <int RPT, int NZR, int NSL>
__device__ __forceinline__ void res_pipelined(const ResArgs &a, const double (&v)[RPT][NZR], const int (&len)[RPT],
                                              const int (&s_col)[RPT][NZR][kRB],
                                              double (&s_xp)[res_nxp<RPT, NZR>()][RPT][kRB], double *s_red,
                                              double *s_tot, int *s_ok, int r0, int wgi)
{
    constexpr bool ZL = res_nxp<RPT, NZR>() >= 3;  // z in LDS
    const int t = threadIdx.x;
    const int G = a.G;
    const unsigned wbytes = a.pair_bytes / 2;  // w buffers: one double per row
    const __amdgpu_buffer_rsrc_t rb_b = __builtin_amdgcn_make_buffer_rsrc((void *)a.b, (short)0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw0 = __builtin_amdgcn_make_buffer_rsrc(a.pair0, (short)0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw1 = __builtin_amdgcn_make_buffer_rsrc(a.pair1, (short)0, (int)wbytes, 0x00020000);
    double2 *s_red2 = reinterpret_cast<double2 *>(s_red);  // 16 waves x 16 B: s_red's 128 B + the next 128 B
    // A src for this thread's rows (CSR-order sequential sums; padded slots gather row 0 and their
    // products are dropped by a select: acc starts at +0.0, so the sum is SpmvGold's)
    auto spmv = [&](const __amdgpu_buffer_rsrc_t src, int s) __attribute__((always_inline)) {
        double g[NZR];
#pragma unroll
        for (int kk = 0; kk < NZR; ++kk)
            g[kk] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(src, s_col[s][kk][t] * 8, 0, 16));
        double acc = 0.0;
#pragma unroll
        for (int kk = 0; kk < NZR; ++kk) {
            const double prod = v[s][kk] * g[kk];
            acc += kk < len[s] ? prod : 0.0;
        }
        return acc;
    };
    // r, w, s, z in registers; x and p (touched once per iteration each) in this thread's LDS slots, so
    // the form needs no more registers than the classic one
    double r[RPT], sv[RPT], z[RPT], w[RPT];
    double gam = 0.0, del = 0.0;
#pragma unroll
    for (int s = 0; s < RPT; ++s) {
        sv[s] = z[s] = w[s] = r[s] = 0.0;
#pragma unroll
        for (int q = 0; q < res_nxp<RPT, NZR>(); ++q)
            s_xp[q][s][t] = 0.0;
        if (len[s] >= 0) {
            const size_t R = (size_t)r0 + t + (size_t)s * kRB;
            r[s] = a.b[R];  // x = 0, r = b (single_strategy.hpp:117-124)
            w[s] = spmv(rb_b, s);  // w_0 = A b: b is complete from the start, no hand-off needed
            st_sc1(a.pair0 + R, w[s]);
            gam += r[s] * r[s];
            del += w[s] * r[s];
        }
    }
    __syncthreads();  // s_col complete (the loop above read it: every wave's columns are in)
    int iters = a.max_iters, brk = 0;
    res_publish2(gam, del, a.slots + (size_t)1 * G + wgi, a.slots + (size_t)2 * G + wgi, s_red2);
    if (!res_wait_sum<NSL, 2>(a.slots + (size_t)1 * G, G, a.abort_word, s_tot, s_ok) || a.force_stall) {
        iters = 0;
        brk = 2;
    } else {
        gam = s_tot[0];
        del = s_tot[1];
        const double bn = sqrt(gam);
        const double b_norm = bn == 0.0 ? 1.0 : bn;  // single_strategy.hpp:127-129
        double gam_prev = 0.0, alpha_prev = 0.0;
        for (int i = 0;; ++i) {
            // (gam, del) of r_i, w_i; w_i complete in buffer i & 1
            res_stamp(a, i, wgi, 0);
            if (i > 0) {
                const double rel = sqrt(gam) / b_norm;
                if (wgi == 0 && t == 0 && a.hist && i - 1 < a.hist_cap)
                    a.hist[i - 1] = rel;
                if (rel < a.tol) {
                    iters = i;
                    break;
                }
            }
            if (i == a.max_iters) {
                iters = i;
                break;
            }
            const double beta = i == 0 ? 0.0 : gam / gam_prev;
            const double alpha = i == 0 ? gam / del : gam / (del - beta * gam / alpha_prev);
            if (!(alpha == alpha && fabs(alpha) < HUGE_VAL)) {  // breakdown: stop before x and r change
                iters = i + 1;
                brk = 1;
                break;
            }
            const double nal = -alpha;
            const __amdgpu_buffer_rsrc_t cur = (i & 1) ? rw1 : rw0;
            double *nxt = (i & 1) ? a.pair0 : a.pair1;
            double g2 = 0.0, d2 = 0.0;
#pragma unroll
            for (int s = 0; s < RPT; ++s) {
                const double n = spmv(cur, s);  // n = A w_i
                if (len[s] >= 0) {
                    const size_t R = (size_t)r0 + t + (size_t)s * kRB;
                    double zs;
                    if constexpr (ZL) {
                        zs = n + beta * s_xp[ZL ? 2 : 0][s][t];
                        s_xp[ZL ? 2 : 0][s][t] = zs;
                    } else {
                        zs = z[s] = n + beta * z[s];
                    }
                    sv[s] = w[s] + beta * sv[s];
                    const double ps = r[s] + beta * s_xp[1][s][t];  // UpdatePSingle
                    s_xp[1][s][t] = ps;
                    s_xp[0][s][t] = s_xp[0][s][t] + alpha * ps;  // AxpySingle
                    r[s] = r[s] + nal * sv[s];   // AxpySingle(-alpha), s = A p by recurrence
                    w[s] = w[s] + nal * zs;
                    st_sc1(nxt + R, w[s]);
                    g2 += r[s] * r[s];
                    d2 += w[s] * r[s];
                }
            }
            if (a.stamps)
                __syncthreads();
            res_stamp(a, i, wgi, 1);
            res_stamp(a, i, wgi, 2);
            res_stamp(a, i, wgi, 3);
            double *sg = a.slots + (size_t)(1 + 2 * ((i + 1) % kResRing)) * G;
            res_publish2(g2, d2, sg + wgi, sg + G + wgi, s_red2);
            if (!res_wait_sum<NSL, 2>(sg, G, a.abort_word, s_tot, s_ok)) {
                iters = i;
                brk = 2;
                break;
            }
            res_stamp(a, i, wgi, 4);
            gam_prev = gam;
            alpha_prev = alpha;
            gam = s_tot[0];
            del = s_tot[1];
            if (t == 0) {  // this workgroup's slots of ring position i + 1 + kResRing/2: empty again
                double *ra = a.slots + (size_t)(1 + 2 * ((i + 1 + kResRing / 2) % kResRing)) * G + wgi;
                __hip_atomic_store((unsigned long long *)ra, kSlotEmpty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned long long *)(ra + G), kSlotEmpty, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
#pragma unroll
    for (int s = 0; s < RPT; ++s)
        if (len[s] >= 0)
            a.x[(size_t)r0 + t + (size_t)s * kRB] = s_xp[0][s][t];
    if (wgi == 0 && t == 0) {
        a.ctrl->iter = iters;
        a.ctrl->iters_out = iters;
        a.ctrl->done = 1;
        a.ctrl->breakdown = brk;
    }
}

template <int RPT, int NZR, int NSL, bool PIPE>
__global__ __launch_bounds__(kRB) void k_cg_resident(ResArgs a)
{
    __shared__ int s_col[RPT][NZR][kRB];
    __shared__ double s_red[2 * (kRB / 64)];  // (the pipelined form's two-value block sums use all of it)
    __shared__ double s_tot[2];
    __shared__ int s_ok;
    __shared__ double s_xp[PIPE ? res_nxp<RPT, NZR>() : 1][PIPE ? RPT : 1][kRB];  // the pipelined form's x, p (z)
    const int t = threadIdx.x;
    const int w = blockIdx.x;
    const int G = a.G;
    const int r0 = a.rb[res_block(w, G)];
    const __amdgpu_buffer_rsrc_t pr0 = __builtin_amdgcn_make_buffer_rsrc(a.pair0, (short)0, (int)a.pair_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t pr1 = __builtin_amdgcn_make_buffer_rsrc(a.pair1, (short)0, (int)a.pair_bytes, 0x00020000);

    // the row block: values to registers, columns to LDS (read once)
    double v[RPT][NZR];
    int len[RPT];
#pragma unroll
    for (int s = 0; s < RPT; ++s) {
        len[s] = a.len[((size_t)w * RPT + s) * kRB + t];
#pragma unroll
        for (int k = 0; k < NZR; ++k) {
            const size_t e = (((size_t)w * RPT + s) * NZR + k) * kRB + t;
            v[s][k] = a.vals[e];
            s_col[s][k][t] = a.cols[e];
        }
    }
    if constexpr (PIPE) {
        res_pipelined<RPT, NZR, NSL>(a, v, len, s_col, s_xp, s_red, s_tot, &s_ok, r0, w);
        return;
    }
    // x = 0, r = p = b (single_strategy.hpp:117-124); {r_0, p_-1} = {b, b} with beta = 0 gives p_0 = b
    double x[RPT], r[RPT], p[RPT];
    double bb = 0.0;
#pragma unroll
    for (int s = 0; s < RPT; ++s) {
        x[s] = r[s] = p[s] = 0.0;
        if (len[s] >= 0) {
            const size_t R = (size_t)r0 + t + (size_t)s * kRB;
            const double bv = a.b[R];
            r[s] = p[s] = bv;
            st_sc1(a.pair0 + 2 * R, bv);
            st_sc1(a.pair0 + 2 * R + 1, bv);
            bb += bv * bv;
        }
    }
    __syncthreads();  // s_col complete
    res_publish<true>(bb, a.slots + w, s_red);
    int iters = a.max_iters, brk = 0;
    if (!res_wait_sum<NSL>(a.slots, G, a.abort_word, s_tot, &s_ok) || a.force_stall) {
        iters = 0;
        brk = 2;
    } else {
        double rs = s_tot[0];
        const double bn = sqrt(rs);
        const double b_norm = bn == 0.0 ? 1.0 : bn;  // single_strategy.hpp:127-129
        double beta = 0.0;
        for (int k = 0; k < a.max_iters; ++k) {
            const __amdgpu_buffer_rsrc_t cur = (k & 1) ? pr1 : pr0;
            double *nxt = (k & 1) ? a.pair0 : a.pair1;
            double *slot_a = a.slots + (size_t)(1 + 2 * (k % kResRing)) * G;
            double *slot_b = slot_a + G;
            res_stamp(a, k, w, 0);
            // Ap = A p_k (OmpCsrSpmv, row by row in CSR order), p_k own rows, p.Ap partial
            double Ap[RPT];
            double dot = 0.0;
#pragma unroll
            for (int s = 0; s < RPT; ++s) {
                // every slot's pair is loaded (padded slots point at row 0) and the products of the
                // padding are dropped by a select: acc starts at +0.0 and adding +0.0 leaves it
                // unchanged, so the row sum is the CSR-order sequential sum
                double2 g[NZR];
#pragma unroll
                for (int kk = 0; kk < NZR; ++kk) {
                    const v4u_t q = __builtin_amdgcn_raw_buffer_load_b128(cur, s_col[s][kk][t] * 16, 0, 16);
                    __builtin_memcpy(&g[kk], &q, 16);
                }
                double acc = 0.0;
#pragma unroll
                for (int kk = 0; kk < NZR; ++kk) {
                    const double prod = v[s][kk] * (g[kk].x + beta * g[kk].y);
                    acc += kk < len[s] ? prod : 0.0;
                }
                Ap[s] = acc;
                if (len[s] >= 0) {
                    const size_t R = (size_t)r0 + t + (size_t)s * kRB;
                    p[s] = r[s] + beta * p[s];  // UpdatePSingle (single_strategy.hpp:89-97), as the gathers form it
                    st_sc1(nxt + 2 * R + 1, p[s]);
                    dot += p[s] * acc;
                }
            }
            if (a.stamps)
                __syncthreads();  // stamped solves: the phase ends when every wave's rows are done
            res_stamp(a, k, w, 1);
            res_publish<false>(dot, slot_a + w, s_red);
            if (!res_wait_sum<NSL>(slot_a, G, a.abort_word, s_tot, &s_ok)) {
                iters = k;
                brk = 2;
                break;
            }
            res_stamp(a, k, w, 2);
            const double alpha = rs / s_tot[0];
            if (!(alpha == alpha && fabs(alpha) < HUGE_VAL)) {  // breakdown: stop before x and r change
                iters = k + 1;
                brk = 1;
                break;
            }
            const double nal = -alpha;
            double rr = 0.0;
#pragma unroll
            for (int s = 0; s < RPT; ++s) {
                if (len[s] >= 0) {
                    const size_t R = (size_t)r0 + t + (size_t)s * kRB;
                    x[s] = x[s] + alpha * p[s];   // AxpySingle
                    r[s] = r[s] + nal * Ap[s];    // AxpySingle(-alpha)
                    st_sc1(nxt + 2 * R, r[s]);
                    rr += r[s] * r[s];
                }
            }
            if (a.stamps)
                __syncthreads();
            res_stamp(a, k, w, 3);
            res_publish<true>(rr, slot_b + w, s_red);
            if (!res_wait_sum<NSL>(slot_b, G, a.abort_word, s_tot, &s_ok)) {
                iters = k;
                brk = 2;
                break;
            }
            res_stamp(a, k, w, 4);
            const double rs_new = s_tot[0];
            const double rel = sqrt(rs_new) / b_norm;
            if (w == 0 && t == 0 && a.hist && k < a.hist_cap)
                a.hist[k] = rel;
            if (rel < a.tol) {
                iters = k + 1;
                break;
            }
            beta = rs_new / rs;
            rs = rs_new;
            if (t == 0) {  // this workgroup's slots of ring position k + kResRing/2: empty again
                double *ra = a.slots + (size_t)(1 + 2 * ((k + kResRing / 2) % kResRing)) * G + w;
                __hip_atomic_store((unsigned long long *)ra, kSlotEmpty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned long long *)(ra + G), kSlotEmpty, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
#pragma unroll
    for (int s = 0; s < RPT; ++s)
        if (len[s] >= 0)
            a.x[(size_t)r0 + t + (size_t)s * kRB] = x[s];
    if (w == 0 && t == 0) {
        a.ctrl->iter = iters;
        a.ctrl->iters_out = iters;
        a.ctrl->done = 1;
        a.ctrl->breakdown = brk;
    }
}

// ELL fill: workgroup w, thread t, row slot s -> row r0 + t + 1024 s of row block res_block(w).
template <int RPT, int NZR>
__global__ __launch_bounds__(kRB) void k_res_fill(const int *__restrict__ ro, const int *__restrict__ ci,
                                                  const double *__restrict__ va, const int *__restrict__ rb, int G,
                                                  int *cols, double *vals, short *len)
{
    const int t = threadIdx.x, w = blockIdx.x;
    const int blk = res_block(w, G);
    const int r0 = rb[blk], nr = rb[blk + 1] - r0;
    for (int s = 0; s < RPT; ++s) {
        const int lr = t + s * kRB;
        const bool has = lr < nr;
        const int b0 = has ? ro[r0 + lr] : 0;
        const int n = has ? ro[r0 + lr + 1] - b0 : 0;
        len[((size_t)w * RPT + s) * kRB + t] = has ? (short)n : (short)-1;
        for (int k = 0; k < NZR; ++k) {
            const size_t e = (((size_t)w * RPT + s) * NZR + k) * kRB + t;
            cols[e] = k < n ? ci[b0 + k] : 0;
            vals[e] = k < n ? va[b0 + k] : 0.0;
        }
    }
}

struct ResShape {
    int rpt, nzr;
};
// Instantiated (rows per thread, slots per row): values RPT x NZR doubles in registers next to the
// per-row x, r, p and one row's NZR gathered pairs -- at most 24 slots keeps the kernel at <= 128
// VGPRs (16 waves per CU).
constexpr ResShape kResShapes[] = {{1, 4}, {2, 4}, {1, 8}, {3, 4}, {2, 7}, {3, 7}, {2, 8}, {1, 16}, {3, 8}};

template <int RPT, int NZR>
hipError_t res_launch_t(const ResArgs &a, hipStream_t s, bool check_only, int *occ, bool pipe)
{
    const int nsl = (a.G + 63) / 64;
    void *args[] = {(void *)&a};
    auto go = [&](const void *kc, const void *kp) -> hipError_t {
        if (check_only) {  // both forms must fit one workgroup per CU
            int o1 = 0, o2 = 0;
            hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o1, kc, kRB, 0);
            if (e == hipSuccess)
                e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, kp, kRB, 0);
            *occ = std::min(o1, o2);
            return e;
        }
        // A plain launch: the grid is one workgroup per CU and the occupancy check above admitted
        // one, so every workgroup is resident -- the residency a cooperative launch would check,
        // without its per-launch host cost and its separate queue (whose teardown at process exit
        // crashed under rocprofv3: r03u).  Every spin in the kernel is bounded, so a grid that is
        // not co-resident after all ends in MSPMV_ERR_STALL (the caller then runs the pipelined
        // kernels), never a hang.
        return hipLaunchKernel(pipe ? kp : kc, dim3(a.G), dim3(kRB), args, 0, s);
    };
    if (nsl <= 4)
        return go((const void *)k_cg_resident<RPT, NZR, 4, false>, (const void *)k_cg_resident<RPT, NZR, 4, true>);
    if (nsl <= 8)
        return go((const void *)k_cg_resident<RPT, NZR, 8, false>, (const void *)k_cg_resident<RPT, NZR, 8, true>);
    return hipErrorInvalidValue;
}

hipError_t res_dispatch(int rpt, int nzr, const ResArgs &a, hipStream_t s, bool check_only, int *occ, bool pipe)
{
#define RES_CASE(R, Z)                                                                                       \
    if (rpt == R && nzr == Z)                                                                                \
        return res_launch_t<R, Z>(a, s, check_only, occ, pipe);
    RES_CASE(1, 4)
    RES_CASE(2, 4)
    RES_CASE(1, 8)
    RES_CASE(3, 4)
    RES_CASE(2, 8)
    RES_CASE(1, 16)
    RES_CASE(3, 8)
    RES_CASE(2, 7)
    RES_CASE(3, 7)
#undef RES_CASE
    return hipErrorInvalidValue;
}

hipError_t res_fill(int rpt, int nzr, const int *ro, const int *ci, const double *va, const int *rb, int G, int *cols,
                    double *vals, short *len, hipStream_t s)
{
#define RES_FILL(R, Z)                                                                                       \
    if (rpt == R && nzr == Z) {                                                                              \
        hipLaunchKernelGGL((k_res_fill<R, Z>), dim3(G), dim3(kRB), 0, s, ro, ci, va, rb, G, cols, vals, len); \
        return hipGetLastError();                                                                            \
    }
    RES_FILL(1, 4)
    RES_FILL(2, 4)
    RES_FILL(1, 8)
    RES_FILL(3, 4)
    RES_FILL(2, 8)
    RES_FILL(1, 16)
    RES_FILL(3, 8)
    RES_FILL(2, 7)
    RES_FILL(3, 7)
#undef RES_FILL
    return hipErrorInvalidValue;
}

}  // namespace

// The resident kernel's iteration: classic CGSolveSingle (two hand-offs) or the single-reduction
// form (one; res_pipelined).  MSPMV_CG_RESIDENT_FORM=single_reduction | classic, read per solve.
bool cg_resident_pipelined()
{
    const char *e = getenv("MSPMV_CG_RESIDENT_FORM");
    if (e && std::strcmp(e, "single_reduction") == 0)
        return true;
    if (e && std::strcmp(e, "classic") == 0)
        return false;
    return kResPipelinedDefault;
}

bool cg_resident_enabled()
{
    const char *e = getenv("MSPMV_CG_RESIDENT");  // read per solve (tests run both paths in one process)
    return !(e && std::strcmp(e, "0") == 0);
}

void resident_free(ResidentCg *r)
{
    if (!r)
        return;
    for (void *p : {(void *)r->d_rb, (void *)r->d_cols, (void *)r->d_vals, (void *)r->d_len, (void *)r->d_slots,
                    (void *)r->d_abort})
        if (p)
            (void)hipFree(p);
    delete r;
}

// Build (once per handle) the resident layout if the matrix fits: every row block <= RPT x 1024
// rows and every row <= NZR nonzeros for one instantiated shape, one 1024-thread workgroup
// resident per CU.  r->ok = false otherwise (the caller runs the pipelined CG).  The layout is
// attached to the handle only once it is complete; any failure while building it (allocation,
// fill) leaves a not-ok layout attached and returns MSPMV_OK, so this solve and every later one
// take the pipelined CG alike instead of the first one failing.
static bool resident_build(mspmv_handle_s *h, ResidentCg *r)
{
    int total = 0;
    if (hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess)
        return false;
    if (h->num_cus != total || h->m < 1 || h->m != h->n)  // CU-limited streams: residency is not the device's
        return false;
    const int G = total;
    std::vector<int> ro((size_t)h->m + 1);
    if (hipMemcpy(ro.data(), h->d_row_offsets, sizeof(int) * ro.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return false;
    // merge-path balanced row blocks: block j starts at the last row i with i + ro[i] <= j (m + nnz) / G
    std::vector<int> rb((size_t)G + 1);
    const long long tot = (long long)h->m + h->nnz;
    int maxrows = 0, maxlen = 0;
    for (int j = 0; j <= G; ++j) {
        const long long d = tot * j / G;
        int lo = 0, hi = h->m;
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (mid + (long long)ro[(size_t)mid] <= d)
                lo = mid;
            else
                hi = mid - 1;
        }
        rb[(size_t)j] = j == G ? h->m : lo;
    }
    for (int j = 0; j < G; ++j)
        maxrows = std::max(maxrows, rb[(size_t)j + 1] - rb[(size_t)j]);
    for (int i = 0; i < h->m; ++i)
        maxlen = std::max(maxlen, ro[(size_t)i + 1] - ro[(size_t)i]);
    const int rpt_need = (maxrows + kRB - 1) / kRB;
    int best = -1;
    for (int i = 0; i < (int)(sizeof(kResShapes) / sizeof(kResShapes[0])); ++i) {
        const ResShape &sh = kResShapes[i];
        if (sh.rpt >= std::max(rpt_need, 1) && sh.nzr >= maxlen &&
            (best < 0 || sh.rpt * sh.nzr < kResShapes[best].rpt * kResShapes[best].nzr))
            best = i;
    }
    if (best < 0)
        return false;
    const int rpt = kResShapes[best].rpt, nzr = kResShapes[best].nzr;
    ResArgs probe{};
    probe.G = G;
    int occ = 0;
    if (res_dispatch(rpt, nzr, probe, h->stream, true, &occ, false) != hipSuccess || occ < 1)
        return false;
    const size_t ell = (size_t)G * rpt * nzr * kRB;
    r->slot_bytes = sizeof(double) * (size_t)(1 + 2 * kResRing) * G;
    r->slot_bytes = (r->slot_bytes + 15) & ~(size_t)15;
    if (hipMalloc(&r->d_rb, sizeof(int) * rb.size()) != hipSuccess ||
        hipMalloc(&r->d_cols, sizeof(int) * ell) != hipSuccess ||
        hipMalloc(&r->d_vals, sizeof(double) * ell) != hipSuccess ||
        hipMalloc(&r->d_len, sizeof(short) * (size_t)G * rpt * kRB) != hipSuccess ||
        hipMalloc(&r->d_slots, r->slot_bytes) != hipSuccess || hipMalloc(&r->d_abort, 16) != hipSuccess)
        return false;
    if (hipMemcpyAsync(r->d_rb, rb.data(), sizeof(int) * rb.size(), hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        res_fill(rpt, nzr, h->d_row_offsets, h->d_cols, h->d_vals, r->d_rb, G, r->d_cols, r->d_vals, r->d_len,
                 h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess)
        return false;
    r->G = G;
    r->rpt = rpt;
    r->nzr = nzr;
    return true;
}

mspmv_status resident_prepare(mspmv_handle_s *h, ResidentCg **out)
{
    *out = h->rcg;
    if (h->rcg)
        return MSPMV_OK;
    auto *r = new ResidentCg();
    if (!resident_build(h, r)) {
        // a layout that does not fit or could not be built: release what was allocated, clear any
        // sticky error of the failed call, and remember "not resident" for this handle
        for (void *p : {(void *)r->d_rb, (void *)r->d_cols, (void *)r->d_vals, (void *)r->d_len, (void *)r->d_slots,
                        (void *)r->d_abort})
            if (p)
                (void)hipFree(p);
        *r = ResidentCg();
        (void)hipGetLastError();
    } else {
        r->ok = true;
    }
    h->rcg = r;
    *out = r;
    return MSPMV_OK;
}

hipError_t launch_cg_resident(mspmv_handle_s *h, ResidentCg *r, const double *d_b, double *d_x, int max_iters,
                              double tol, unsigned long long *d_stamps, int stamp_iters)
{
    hipError_t e = hipMemsetAsync(r->d_slots, 0xFF, r->slot_bytes, h->stream);  // every slot empty
    if (e == hipSuccess)
        e = hipMemsetAsync(r->d_abort, 0, 16, h->stream);
    if (e != hipSuccess)
        return e;
    ResArgs a{};
    a.rb = r->d_rb;
    a.cols = r->d_cols;
    a.vals = r->d_vals;
    a.len = r->d_len;
    a.b = d_b;
    a.x = d_x;
    a.pair0 = h->d_p0;
    a.pair1 = h->d_p1;
    a.pair_bytes = (unsigned)(16 * (size_t)h->m);
    a.slots = r->d_slots;
    a.abort_word = r->d_abort;
    a.ctrl = h->d_ctrl;
    a.hist = h->d_hist;
    a.hist_cap = h->hist_cap;
    a.max_iters = max_iters;
    a.tol = tol;
    a.G = r->G;
    a.stamps = d_stamps;
    a.stamp_iters = d_stamps ? stamp_iters : 0;
    // MSPMV_CG_RESIDENT_STALL=1 (test switch, read per solve): the first hand-off reports a stall, so
    // tests/test_gpu_cg_resident.py can check the caller's fallback to the two-kernel CG
    const char *fs = getenv("MSPMV_CG_RESIDENT_STALL");
    a.force_stall = fs && atoi(fs) != 0 && !d_stamps;
    const bool pipe = cg_resident_pipelined();
    char buf[80];
    snprintf(buf, sizeof buf, "k_cg_resident<%d,%d,%s> x %d", r->rpt, r->nzr, pipe ? "single_reduction" : "classic", r->G);
    r->name = buf;
    return res_dispatch(r->rpt, r->nzr, a, h->stream, false, nullptr, pipe);
}

}  // namespace mspmv
