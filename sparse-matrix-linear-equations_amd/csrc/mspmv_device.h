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
// on gfx950 a buffer_wbl2 (the XCD's whole L2 written back) per arrival.  The fold of few workgroups
// (k_fold_dot) takes it; rows split between tiles do not (close_split_rows); the streaming kernels, whose L2 holds the vectors they
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
        // The drained-store form (the carries and the head were published with drained write-through stores
        // above): a release is a write-back of the XCD's whole L2 per arrival, and on the one-wave tiles of a
        // power-law matrix -- thousands of rows split over 2 to ~425 tiles -- releases took the skewed SpMV from
        // 80 to 525 us (r06t), still 291 us with releases kept for rows of <= 8 carries (r06u).
        auto arrive = [&](unsigned *tk, int carries) { return ticket_arrive<false>(tk, (unsigned)carries, a.fault); };
        int f0 = -1, f1 = -1;
        if (fx.x >= 0 && arrive(&a.fix_cnt[fx.x], fx.y))
            f0 = fx.x;
        if (fx.z > 0 && arrive(&a.fix_cnt[t], fx.z))
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

// ---- cross-workgroup sums shared by the tile kernels and the offset windows' CG (mspmv_dia.hip) ----
// Lane 0 of each wave holds a deterministic butterfly sum; wave totals are combined in
// wave order.  Call uniformly from every thread of the block; returns the total in all.
__device__ __forceinline__ double block_sum(double v, double *s_red)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v += __shfl_xor(v, off);
    __syncthreads();  // s_red may still be read by a previous call
    if ((threadIdx.x & 63) == 0)
        s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = s_red[0];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w)
        t += s_red[w];
    return t;
}

// Sum of column j over rows q, q + kBlock/L, ... < count of a [count][L] array written by
// other workgroups (agent-scope loads), in row order; eight loads in flight per batch.
template <int L>
__device__ __forceinline__ double fold_col_strided(const double *base, int count, int j, int q)
{
    constexpr int TPC = kBlock / L;
    double v = 0.0;
    int i = q;
    for (; i + 7 * TPC < count; i += 8 * TPC) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            t[u] = load_sc1(&base[(size_t)(i + u * TPC) * L + j]);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v += t[u];
    }
    for (; i < count; i += TPC)
        v += load_sc1(&base[(size_t)i * L + j]);
    return v;
}

// Column totals of a [count][L] partials array in a fixed order (per-thread strided rows,
// then threads in order) -> s_out[0..L).  Call uniformly from every thread.
template <int L>
__device__ __forceinline__ void fold_cols(const double *base, int count, double *s_tmp, double *s_out)
{
    constexpr int TPC = kBlock / L;
    const int tid = threadIdx.x;
    s_tmp[tid] = fold_col_strided<L>(base, count, tid % L, tid / L);
    __syncthreads();
    if (tid < L) {
        double w = s_tmp[tid];
        for (int u = 1; u < TPC; ++u)
            w += s_tmp[u * L + tid];
        s_out[tid] = w;
    }
    __syncthreads();
}

// One arrival on a fold group's ticket (thread 0 only; ticket_arrive).  A fault also stops a single-GPU
// solve (done); a sharded one does not (fault_no_stop: the ranks' stop decisions must stay identical, so
// its host stops on the all-reduced fault word at a batch boundary instead).
template <bool RELEASE>
__device__ __forceinline__ bool take_ticket(unsigned *tk, int gsize, CgControl *ctrl)
{
    bool faulted = false;
    if (ticket_arrive<RELEASE>(tk, (unsigned)gsize - 1, ctrl ? &ctrl->fault : nullptr, &faulted))
        return true;
    if (faulted && ctrl && !__hip_atomic_load(&ctrl->fault_no_stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        __hip_atomic_store(&ctrl->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
}

// Consumer-side reduction (single-RHS pipelined CG).  A producer kernel leaves one partial per
// workgroup; EVERY workgroup of the consumer kernel sums them itself, in one fixed order (thread
// tid adds elements tid, tid + 256, ... ascending, then block_sum's fixed tree), so all agree
// bit for bit and no ticket chain sits in the producer's tail.  The loads are issued early
// (part_load) and summed late (part_sum), under the consumer's own streaming loads.
template <int NR>
struct PartRegs {
    double v[NR];
};
template <int NR>
__device__ __forceinline__ void part_load(const double *p, int n, PartRegs<NR> &r)
{
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const int i = (int)threadIdx.x + j * kBlock;
        r.v[j] = i < n ? p[i] : 0.0;
    }
}
template <int NR>
__device__ __forceinline__ double part_sum(const PartRegs<NR> &r, double *s_red)
{
    double v = r.v[0];
#pragma unroll
    for (int j = 1; j < NR; ++j)
        v += r.v[j];
    return block_sum(v, s_red);
}

// Publish this workgroup's partial (already stored at partials[slot], agent scope, vmcnt
// drained, block synchronised) for a consumer kernel that sums at most `stop` of them: while
// more would remain, groups of kSlotGroup are folded into the next level by their last arriver
// (reduce_slots' tickets), down to the level consumer_level() names.
template <int L>
__device__ __forceinline__ void publish_partials(double *partials, unsigned *tickets, int slot, int nslots, int stop,
                                                 double *s_tmp, double *s_out, int *s_flag, CgControl *ctrl)
{
    const int tid = threadIdx.x;
    double *lvl = partials;
    int idx = slot, count = nslots;
    while (count > stop) {
        const int g = idx / kSlotGroup;
        const int ngroups = (count + kSlotGroup - 1) / kSlotGroup;
        const int gsize = min(kSlotGroup, count - g * kSlotGroup);
        unsigned *tk = &tickets[(size_t)g * kTicketStride];
        if (tid == 0)
            *s_flag = take_ticket<false>(tk, gsize, ctrl);
        __syncthreads();
        if (!*s_flag)
            return;
        fold_cols<L>(lvl + (size_t)g * kSlotGroup * L, gsize, s_tmp, s_out);
        if (tid == 0)
            __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        double *next = lvl + (size_t)count * L;
        if (tid < L) {
            store_sc1(&next[(size_t)g * L + tid], s_out[tid]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        tickets += (size_t)ngroups * kTicketStride;
        lvl = next;
        idx = g;
        count = ngroups;
    }
}

// Pipelined single-RHS CG, head of iteration k (MODE 1).  Every workgroup sums the previous
// update's r.r partials itself (rs_k; at k = 0 the init's b.b), so the stop test and beta need
// no ticket chain: the reference's check after iteration k-1 (single_strategy.hpp:150-156:
// sqrt(rs_new)/||b|| < tol -> iterations = k) is taken here, then beta = rs_k / rs_{k-1}
// (:158-160).  Workgroup 0 records the history and hands rs_k and k+1 on by parity.  Returns
// false when the solve has stopped (converged): the caller returns at once.
template <typename A>  // TileArgs (k_spmv_tile, k_spmv_blk) or Cg1DiaArgs (k_cg1_dia)
__device__ __forceinline__ bool cg1_head(const A &a, double rs, double &beta)
{
    CgScalars &s = a.scal[0];
    CgControl *c = a.ctrl;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    const int k = c->iter_par[a.parity];
    if (k == 0) {  // r = p = b: no stop test before the first iteration
        beta = 0.0;
        if (lead) {
            const double bn = sqrt(rs);
            s.b_norm = bn == 0.0 ? 1.0 : bn;  // single_strategy.hpp:124-129
            s.rs_par[0] = rs;
            c->iter_par[1] = 1;
        }
        return true;
    }
    const double rel = sqrt(rs) / s.b_norm;
    if (lead) {
        if (a.hist && k - 1 < a.hist_cap)
            a.hist[k - 1] = rel;
        c->iter = k;
    }
    if (rel < a.tol) {
        if (lead) {
            c->iters_out = k;
            c->done = 1;
        }
        return false;
    }
    beta = rs / s.rs_par[a.parity ^ 1];
    if (lead) {
        s.rs_par[a.parity] = rs;
        c->iter_par[a.parity ^ 1] = k + 1;
    }
    return true;
}

}  // namespace mspmv
