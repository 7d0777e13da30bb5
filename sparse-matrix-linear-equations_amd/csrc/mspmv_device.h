// Device helpers shared by the tile kernels (mspmv_kernels.hip) and the column-slab SpMV
// (mspmv_slab.hip): agent-scope stores and loads, the XCD-contiguous tile mapping, and the closing of
// rows split between tiles.  Included by HIP sources only.
#pragma once
#include "mspmv_internal.h"

namespace mspmv {

typedef double v2d_t __attribute__((ext_vector_type(2)));  // 16-B nontemporal loads / stores

__device__ __forceinline__ int xcd_tile(int b, int T)
{
    // Blocks are dealt round-robin over the 8 XCDs; give XCD k (= b % 8, a label only) the
    // contiguous tile range [k*q + min(k,r), +q + (k<r)).  Bijective for any T (host check:
    // tests/test_abi.py mirrors this map).
    const int q = T >> 3, r = T & 7;
    const int k = b & 7, i = b >> 3;
    return k * q + (k < r ? k : r) + i;
}

__device__ __forceinline__ void store_sc1(double *p, double v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_sc1_2(double *p, double2 v)
{
    store_sc1(p, v.x);
    store_sc1(p + 1, v.y);
}

// One arrival on a self-resetting ticket (call from one thread; tickets guard the cross-workgroup folds:
// reduce_slots, publish_partials, close_split_rows, the slab kernels' column groups).  Every caller has
// written what the final arrival will read with agent-scope (sc1, write-through) stores and drained them
// (s_waitcnt vmcnt(0)) before arriving, and the final arrival reads with agent-scope loads.
// RELEASE: the fetch_add is also a release at agent scope, the memory model's own form of that order --
// on gfx950 a buffer_wbl2 (the XCD's whole L2 written back) per arrival.  The folds of few workgroups
// (k_fold_dot, rows split between tiles) take it; the streaming kernels, whose L2 holds the vectors they
// just wrote, keep the drained-store form (measured with the release on every arrival, r06a: configs[4]'s
// CG iteration +4.5 %, the sliced-ELL SpMV +10 %).  The arrival that draws `last` -- the group's final
// one -- takes an agent-scope acquire fence before it reads the others' stores; the other arrivals read
// nothing, so they skip it.  Tickets start at 0
// and the final arrival resets them, so a group draws exactly 0 .. last.  A draw > last means the ticket
// was not 0 when the group began -- its array not zeroed, or zeroed out of stream order, before the
// launch (round 5's 70-vs-43 iterations): the draw of `last` then falls on an arrival that
// is not the final one (a fold of partials not yet written) or on none (no fold: the consumer reads a
// stale total).  That draw raises kFaultTicket in *fault (nullable), which a solve returns as
// MSPMV_ERR_FAULT (a plain product: mspmv_check_faults).
// *faulted (nullable) tells the caller this arrival raised the fault.
template <bool RELEASE>
__device__ __forceinline__ bool ticket_arrive(unsigned *tk, unsigned last, unsigned *fault, bool *faulted = nullptr)
{
    const unsigned v = RELEASE ? __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT)
                               : __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v > last && fault)
        __hip_atomic_fetch_or(fault, kFaultTicket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (faulted)
        *faulted = v > last;
    if (v != last)
        return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return true;
}

// Split rows, closed inside the tile kernel (replaces r03's k_fixup launch).  A row longer than the
// snap distance spans consecutive tiles: each tile that ends inside it stores its partial as a carry,
// and the tile where it ends (its completing tile) stores the row's own part -- its row 0 -- to
// head_val instead of y (TileArgs::y0: one address select per row store, no branch).  The row's nc + 1
// tiles publish with agent scope (carries directly, the head copied to head_pub here) and take one
// ticket each on fix_cnt[completing tile]; whichever draws the last one -- no waiting: it is simply
// the last to finish -- closes the row: wave w takes columns j = w, w + TB/64, ...: lane l sums carries
// l, l + 64, ... in tile order, a fixed xor butterfly folds the wave, lane 0 adds the head and stores
// y's row (k_fixup's order, so reproducible), and the ticket is reset for the next launch.  fx =
// fix[t] (plan time): x = the completing tile of the row this tile ends inside (-1: none), y = that
// row's carry count, z = the carry count of the row this tile completes (0: none).  Call from every
// thread after the tile's rows and carry are stored and after any pass that reads its own rows back
// (the dot mode's).
template <typename A>
__device__ __forceinline__ int4 load_fix(const A &a, int t)  // block-uniform: kept in SGPRs
{
    if (!a.fix)
        return make_int4(-1, 0, 0, 0);
    const int4 f = a.fix[t];
    return make_int4(__builtin_amdgcn_readfirstlane(f.x), __builtin_amdgcn_readfirstlane(f.y),
                     __builtin_amdgcn_readfirstlane(f.z), 0);
}
template <int TB, typename A>
__device__ __forceinline__ void close_split_rows(const A &a, int t, int4 fx, int L, int ld)
{
    if (fx.x < 0 && fx.z == 0)  // block-uniform
        return;
    __shared__ int s_fin[2];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this tile's carry and head are out
    __syncthreads();
    if (fx.z > 0) {  // the head, stored by this workgroup: republished with agent scope
        for (int j = threadIdx.x; j < L; j += TB)
            store_sc1(&a.head_pub[(size_t)t * L + j], a.head_val[(size_t)t * L + j]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int f0 = -1, f1 = -1;
        if (fx.x >= 0 && ticket_arrive<true>(&a.fix_cnt[fx.x], (unsigned)fx.y, a.fault))
            f0 = fx.x;
        if (fx.z > 0 && ticket_arrive<true>(&a.fix_cnt[t], (unsigned)fx.z, a.fault))
            f1 = t;
        s_fin[0] = f0;
        s_fin[1] = f1;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int tc = s_fin[q], nc = q == 0 ? fx.y : fx.z;
        if (tc < 0)
            continue;
        const size_t R = (size_t)a.bounds[tc].x;
        for (int j = (int)threadIdx.x >> 6; j < L; j += TB / 64) {  // wave-uniform
            double sum = 0.0;
            for (int u = lane; u < nc; u += 64)
                sum += load_sc1(&a.carry_val[(size_t)(tc - nc + u) * L + j]);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1)
                sum += __shfl_xor(sum, off);
            if (lane == 0)
                a.y[R * ld + j] = sum + load_sc1(&a.head_pub[(size_t)tc * L + j]);
        }
        if (threadIdx.x == 0)
            __hip_atomic_store(&a.fix_cnt[tc], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace mspmv
