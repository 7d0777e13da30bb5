// mspmv_kernels.hip -- hand-written gfx950 (CDNA4) kernels for merge-path CSR SpMV/SpMM and
// the fused CG iteration.  Compiled with -ffp-contract=off: every a*b+c is two roundings, as
// in the reference built for the x86-64 baseline ISA, so rows that no tile/thread boundary
// splits are bit-identical to SpmvGold (cpu_spmv.cpp:241-265).
//
// Algorithm (Merrill & Garland merge-path, re-derived for 64-lane waves):
//   * the (row-end-offsets x nnz-index) merge path is cut into tiles of `tile_items` merge
//     items at setup (k_merge_coords + k_snap, once per matrix -- the matrix is immutable);
//   * one 256-thread workgroup per tile stages the tile's row end offsets and its
//     products val*x[col] (SpMV) or its (col, val) pairs (SpMM) in LDS with fully
//     coalesced loads, then every thread (SpMV) or every group of L/2 lanes (SpMM, one
//     double2 of the row-major panel per lane) runs its own merge-path search in LDS and
//     walks an equal share of merge items;
//   * rows split between threads are closed in LDS in thread order; rows split between
//     tiles (only inside rows longer than the snap distance) are closed by the tile that
//     completes them, in tile order (close_split_rows).  All reductions are fixed-order: results are run-to-run deterministic.
//   * tiles are dealt XCD-contiguously (blocks b and b+8 share an XCD), so each XCD's L2
//     sees one contiguous band of x / X.
#include "mspmv_internal.h"
#include "mspmv_device.h"

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace mspmv {

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------

template <typename... KArgs, typename... Args>
static void ggl(void (*kernel)(KArgs...), dim3 grid, dim3 block, hipStream_t s, Args... args)
{
    hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
}

// Streamed-once matrix arrays: nontemporal loads (don't displace x / X from the caches).
template <bool NT, typename T>
__device__ __forceinline__ T ld_stream(const T *p)
{
    if (NT)
        return __builtin_nontemporal_load(p);
    return *p;
}
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ int4 ld_stream(const int4 *p)
{
    if (NT) {
        const v4i_t t = __builtin_nontemporal_load(reinterpret_cast<const v4i_t *>(p));
        return make_int4(t.x, t.y, t.z, t.w);
    }
    return *p;
}
template <bool NT>
__device__ __forceinline__ double2 ld_stream(const double2 *p)
{
    if (NT) {
        const v2d_t t = __builtin_nontemporal_load(reinterpret_cast<const v2d_t *>(p));
        return make_double2(t.x, t.y);
    }
    return *p;
}

// Merge-path search (cpu_spmv.cpp:208-235 semantics) over an LDS copy of the tile's row
// end offsets, stored relative to the tile's first nonzero; list B is 0..b_len-1.
__device__ __forceinline__ void lds_search(int d, const int *s_rowend, int a_len, int b_len, int &x, int &y)
{
    int lo = d - b_len > 0 ? d - b_len : 0;
    int hi = d < a_len ? d : a_len;
    while (lo < hi) {
        const int pivot = (lo + hi) >> 1;
        if (s_rowend[pivot] <= d - pivot - 1)
            lo = pivot + 1;
        else
            hi = pivot;
    }
    x = lo;
    y = d - lo;
}

// Deterministic multi-level "last block done" reduction of per-slot column partials.  The
// caller has stored partials[slot][0..L) (agent scope, vmcnt drained) and synchronised.  Slots
// form groups of kSlotGroup; the last of a group to arrive (one agent-scope ticket per group)
// folds the group in slot order into the next level, whose groups fold the same way, until
// one group remains: its last arriver holds the totals in s_out and returns true (exactly one
// block does).  Tickets reset themselves for the next launch.  Why a tree of small groups on
// separate 256-B lines: agent-scope atomics on one address serialise at the memory side
// (~10 ns each), so 2 k blocks on one ticket cost ~22 us; fan-in 32 keeps each chain short.
// RELEASE: the arrivals are agent-scope releases (ticket_arrive; k_fold_dot), else the drained-store form.
template <int L, bool RELEASE = false>
__device__ __forceinline__ bool reduce_slots(double *partials, unsigned *tickets, int slot, int nslots,
                                             double *s_tmp, double *s_out, int *s_flag, CgControl *ctrl)
{
    const int tid = threadIdx.x;
    double *lvl = partials;
    int idx = slot, count = nslots;
    for (;;) {
        const int g = idx / kSlotGroup;
        const int ngroups = (count + kSlotGroup - 1) / kSlotGroup;
        const int gsize = min(kSlotGroup, count - g * kSlotGroup);
        unsigned *tk = &tickets[(size_t)g * kTicketStride];
        if (tid == 0)
            *s_flag = take_ticket<RELEASE>(tk, gsize, ctrl);
        __syncthreads();
        if (!*s_flag)
            return false;
        fold_cols<L>(lvl + (size_t)g * kSlotGroup * L, gsize, s_tmp, s_out);
        if (tid == 0)
            __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ngroups == 1)
            return true;
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

// ------------------------------------------------------------------------------------------
// partition: the reference's partition coordinates and the tile plan boundaries
// ------------------------------------------------------------------------------------------
__global__ void k_merge_coords(const int *__restrict__ row_offsets, int m, int nnz, long long step, int num_parts,
                               int2 *__restrict__ out)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > num_parts)
        return;
    const long long total = (long long)m + nnz;
    long long dl = step * (long long)t;
    const int d = (int)(dl < total ? dl : total);
    const int *a = row_offsets + 1;
    int lo = d - nnz > 0 ? d - nnz : 0;
    int hi = d < m ? d : m;
    while (lo < hi) {
        const int pivot = (lo + hi) >> 1;
        if (a[pivot] <= d - pivot - 1)
            lo = pivot + 1;
        else
            hi = pivot;
    }
    out[t] = make_int2(lo < m ? lo : m, d - lo);
}

__global__ void k_snap(const int *__restrict__ row_offsets, int m, int2 *__restrict__ b,
                       unsigned char *__restrict__ split, int T, int snap)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > T)
        return;
    int2 c = b[t];
    unsigned char s = 0;
    if (t > 0 && t < T && c.x < m) {
        const int start = row_offsets[c.x];
        if (c.y - start <= snap)
            c.y = start;  // row entered by <= snap nonzeros: the completing tile takes it whole
        else
            s = 1;        // deep inside a long row: exact merge coordinate, carry crosses it
    }
    b[t] = c;
    split[t] = s;
}

// 16-bit column offsets, one workgroup per tile: the tile's column range (block min / max), and
// when it spans < 65536 columns, cols16[k] = col[k] - colbase[t] for the tile's nonzeros.
__global__ __launch_bounds__(kBlock) void k_pack_cols16(const int *__restrict__ cols, const int2 *__restrict__ bounds,
                                                        int *__restrict__ colbase, unsigned short *__restrict__ cols16)
{
    __shared__ int s_min[kBlock / 64], s_max[kBlock / 64];
    const int t = blockIdx.x, tid = threadIdx.x;
    const int n0 = bounds[t].y, n1 = bounds[t + 1].y;
    int lo = 0x7fffffff, hi = -1;
    for (int k = n0 + tid; k < n1; k += kBlock) {
        const int c = cols[k];
        lo = min(lo, c);
        hi = max(hi, c);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off));
        hi = max(hi, __shfl_xor(hi, off));
    }
    if ((tid & 63) == 0) {
        s_min[tid >> 6] = lo;
        s_max[tid >> 6] = hi;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        lo = min(lo, s_min[w]);
        hi = max(hi, s_max[w]);
    }
    const int base = (n1 > n0 && hi - lo < 65536) ? lo : -1;
    if (tid == 0)
        colbase[t] = base;
    if (base >= 0)
        for (int k = n0 + tid; k < n1; k += kBlock)
            cols16[k] = (unsigned short)(cols[k] - base);
}

// Per-tile column dictionary (plan time, single-RHS plans): one workgroup per
// tile sorts the tile's column ids in LDS (bitonic, N = power of two >= the tile's nonzeros),
// keeps the distinct ones in ascending order -> dict[n0 + d], d < ndict[t] (stored in the tile's
// own nonzero range: ndict <= nnzt), and rewrites every nonzero as its dictionary position ->
// idx16[k].  The kernel then gathers each distinct x once per tile instead of once per nonzero.
// ratio < 0: a multi-RHS plan (k_spmm_tile parks the distinct panel rows in LDS): every tile
// whose nonzeros repeat its distinct columns at least twice and has at most dmax of them takes
// its dictionary, without the single-RHS line test.
template <int N>
__global__ __launch_bounds__(kBlock) void k_build_dict(const int *__restrict__ cols, const int2 *__restrict__ bounds,
                                                       int *__restrict__ dict, int *__restrict__ ndict,
                                                       unsigned short *__restrict__ idx16, int ratio, int dmax)
{
    __shared__ int keys[N];
    __shared__ int uniq[N];
    __shared__ int s_scan[kBlock];
    const int t = blockIdx.x, tid = threadIdx.x;
    const int n0 = bounds[t].y, nz = bounds[t + 1].y - n0;
    // Cache lines one gather instruction touches (64 consecutive entries, 16 doubles per 128-B
    // line), summed over the tile: first direct (nonzeros in CSR order, as the kernel stripes
    // them); a tile below 1 line per 2 nonzeros keeps direct gathers and skips the sort.
    constexpr int C = N / kBlock;
    int ld = 0;
    for (int c = 0; c < C; ++c) {
        const int i = tid * C + c;
        if (i < nz)
            ld += ((i & 63) == 0 || (cols[n0 + i] >> 4) != (cols[n0 + i - 1] >> 4)) ? 1 : 0;
    }
    s_scan[tid] = ld;
    __syncthreads();
    for (int off = kBlock / 2; off > 0; off >>= 1) {
        if (tid < off)
            s_scan[tid] += s_scan[tid + off];
        __syncthreads();
    }
    const int lines_direct = s_scan[0];
    // ratio >= 100 (MSPMV_SPMV_DICT=100, lab A/B): every tile takes its dictionary
    if (ratio == 0 || nz == 0 || (ratio > 0 && ratio < 100 && 2 * lines_direct < nz)) {
        if (tid == 0)
            ndict[t] = 0;
        return;
    }
    __syncthreads();
    for (int i = tid; i < N; i += kBlock)
        keys[i] = i < nz ? cols[n0 + i] : 0x7fffffff;
    __syncthreads();
    for (int k = 2; k <= N; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < N; i += kBlock) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int a = keys[i], b = keys[ixj];
                    if ((a > b) == ((i & k) == 0)) {
                        keys[i] = b;
                        keys[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    // distinct keys: thread tid scans its contiguous chunk [tid*C, (tid+1)*C)
    int cnt = 0;
    for (int c = 0; c < C; ++c) {
        const int i = tid * C + c;
        cnt += (i < nz && (i == 0 || keys[i] != keys[i - 1])) ? 1 : 0;
    }
    s_scan[tid] = cnt;
    __syncthreads();
    for (int off = 1; off < kBlock; off <<= 1) {  // inclusive Hillis-Steele scan
        const int v = tid >= off ? s_scan[tid - off] : 0;
        __syncthreads();
        s_scan[tid] += v;
        __syncthreads();
    }
    int pos = s_scan[tid] - cnt;
    for (int c = 0; c < C; ++c) {
        const int i = tid * C + c;
        if (i < nz && (i == 0 || keys[i] != keys[i - 1]))
            uniq[pos++] = keys[i];
    }
    const int nu = s_scan[kBlock - 1];
    __syncthreads();
    // ... then through the sorted dictionary.  The dictionary is taken only where direct gathers
    // are line-bound (>= 1 line per 2 nonzeros: scattered columns) and sorting saves >= 1/4 of
    // the lines; elsewhere (FEM blocks, stencils: ~0.2 lines per nonzero, served by L1/L2) its
    // LDS round trip measured a wash or a loss, and on random columns sorting saves nothing.
    int lu = 0;
    for (int c = 0; c < C; ++c) {
        const int i = tid * C + c;
        if (i < nu)
            lu += ((i & 63) == 0 || (uniq[i] >> 4) != (uniq[i - 1] >> 4)) ? 1 : 0;
    }
    s_scan[tid] = lu;
    __syncthreads();
    for (int off = kBlock / 2; off > 0; off >>= 1) {
        if (tid < off)
            s_scan[tid] += s_scan[tid + off];
        __syncthreads();
    }
    const int lines_dict = s_scan[0];
    const bool use = ratio >= 100 ? true : ratio > 0 ? 4 * lines_dict <= 3 * lines_direct : (nu <= dmax && 2 * nu <= nz);
    if (tid == 0)
        ndict[t] = use ? nu : 0;
    if (!use)
        return;
    for (int d = tid; d < nu; d += kBlock)
        dict[n0 + d] = uniq[d];
    for (int i = tid; i < nz; i += kBlock) {
        const int c = cols[n0 + i];
        int lo = 0, hi = nu - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (uniq[mid] < c)
                lo = mid + 1;
            else
                hi = mid;
        }
        idx16[n0 + i] = (unsigned short)lo;
    }
}

// ---- node blocks (plan time, single-RHS plans) --------------------------------------------
// FEM matrices store several unknowns per mesh node (pwtk: 6 DOF), and every row of a node lists
// the same columns.  A tile whose rows come in such runs -- consecutive rows whose column lists
// are prefixes of one list P (equal lists included; a row shortened by the matrix edge too) --
// stages them "column-owner" style: lane j reads P[j] once, gathers x[P[j]] once and multiplies
// it into every row of the run.  Only P's 16-bit column offsets cross HBM (1/h of the tile's
// column stream) and there is one gather per distinct (run, column) instead of one per nonzero.
// The products land in the same LDS slots as the striped staging writes, so the reduction --
// and every result bit -- is unchanged.
//
// Descriptor of one run chunk (16 B; at most kBlkMax per tile, tile t's at blk[t * stride ..], the
// plan's stride being the smallest of 16, 32, 64 that holds every tile's set):
//   x: vofs (nonzero offset of the run's first row in the tile, bits 0-15) | j0 (first pattern
//      column of this chunk, 16-23) | wc (chunk width <= 64, 24-31)
//   y: h (rows, 1..8, bits 0-3) | p (row holding P, 4-6) | nd (descriptor count, in entry 0 only,
//      8-15; 0 = the tile stages the plain way) | rofs (the run's first row in the tile, 16-31)
//   z, w: the h row lengths, 8 bits each (rows of a run are <= 255 long)
constexpr int kBlkMax = 64;  // descriptors a tile may have (the plan stores them at a stride of 16, 32 or 64)
constexpr int kBlkRows = 8;
// (kBlkRunRows, mspmv_internal.h: rows per run)
// (kBlkTileChunks, mspmv_internal.h: the chunks of a tile the LDS-staged and column-owner paths of
// k_spmv_tile take -- one round of its four waves, more measured slower than striped staging; tiles
// of up to kBlkPlanChunks run only in the column-pair kernel, which loops over rounds.)

__device__ __forceinline__ int blk_len(const uint4 &d, int i)
{
    return (int)(((i < 4 ? d.z : d.w) >> (8 * (i & 3))) & 255u);
}

// One thread per tile.  A tile qualifies when it holds whole rows only (no split boundary), is on
// the 16-bit column stream, fits in kBlkMax chunks, and its runs pay (below).  (Runs tolerating one
// row with one extra pattern column -- imperfect FEM rows -- measured 24.1 vs 24.4 us on the pwtk
// shape with 1 % such rows, and cost the regular shape: not kept, r04e.)
__global__ void k_build_blocks(const int *__restrict__ row_offsets, const int *__restrict__ cols,
                               const int2 *__restrict__ bounds, const unsigned char *__restrict__ split,
                               const int *__restrict__ colbase, int num_tiles, uint4 *__restrict__ blk,
                               int max_chunks)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= num_tiles)
        return;
    uint4 *out = blk + (size_t)t * kBlkMax;
    out[0] = make_uint4(0, 0, 0, 0);  // entry 0 (with the count) is written last, on success only
    uint4 d0 = make_uint4(0, 0, 0, 0);
    const int2 b0 = bounds[t], b1 = bounds[t + 1];
    const int r0 = b0.x, r1 = b1.x, n0 = b0.y, n1 = b1.y;
    if (split[t] || split[t + 1] || colbase[t] < 0 || n1 <= n0 || row_offsets[r0] != n0 || row_offsets[r1] != n1)
        return;
    int nd = 0, sum_w = 0, nruns = 0;
    int r = r0;
    while (r < r1) {
        const int g = r, gs = row_offsets[g];
        int p = g, plen = row_offsets[g + 1] - gs;
        unsigned lens[2] = {0u, 0u};
        int h = 0;
        for (; r < r1 && h < kBlkRunRows; ++r, ++h) {
            const int s = row_offsets[r], len = row_offsets[r + 1] - s;
            if (len > 255)
                return;
            if (h > 0) {  // a prefix of P, or P a prefix of it
                const int ps = row_offsets[p], m = min(len, plen);
                bool same = true;
                for (int q = 0; q < m && same; ++q)
                    same = cols[s + q] == cols[ps + q];
                // a row that would widen a pattern of <= 64 columns past 64 starts a new run: the run
                // stays one chunk (a register run tile) -- spmv_runs_decide's host restatement relies on it
                if (!same || (len > 64 && plen <= 64))
                    break;
                if (len > plen) {
                    p = r;
                    plen = len;
                }
            }
            lens[h >> 2] |= (unsigned)len << (8 * (h & 3));
        }
        sum_w += plen;
        ++nruns;
        const int vofs = gs - n0;
        for (int j0 = 0; j0 < plen || (j0 == 0 && plen == 0); j0 += 64) {
            if (nd == kBlkMax || j0 > 255)
                return;
            const int wc = min(64, plen - j0);
            const uint4 dd = make_uint4((unsigned)vofs | ((unsigned)j0 << 16) | ((unsigned)wc << 24),
                                        (unsigned)h | ((unsigned)(p - g) << 4) | ((unsigned)(g - r0) << 16),
                                        lens[0], lens[1]);
            if (nd == 0)
                d0 = dd;
            else
                out[nd] = dd;
            ++nd;
            if (plen == 0)
                break;
        }
    }
    // Pays only when (measured, tools/lab/narrow_probe.py): runs share columns (pattern columns
    // <= 3/5 of the nonzeros: mean run height >= ~1.7), are wide (mean pattern >= 32 columns: a
    // run's value loads use one lane per column, against 64 per load in the striped staging), and
    // the 4 waves take the tile in ONE round of two chunks each (nd <= 8): a second round waits
    // for the first's sums.  2-D Kronecker FEM matrices with 3, 4 and 6 unknowns per node (15-30
    // columns, ~11-20 runs per tile) ran 3.1x, 2.0x and 1.2x slower on node blocks than striped;
    // the pwtk shape (53 columns, ~7 runs per tile) 1.14x faster.  (Shifted runs -- rows whose columns
    // are the previous row's plus one, the 27-point stencil's x-lines -- in a 16-lane column-pair form
    // measured slower than the striped staging on the nlpkkt120 size: 266-268 vs 220-224 us, r04d.)
    if (5 * sum_w > 3 * (n1 - n0) || sum_w < 32 * nruns || nd > max_chunks)
        return;
    d0.y |= (unsigned)nd << 8;
    out[0] = d0;
}

// Per-tile choice of the in-tile reduction (one thread per tile, at plan time; gl = lanes per
// nonzero: 1 for SpMV, L/2 column-pair lanes for SpMM).  The tile's row segments -- its complete rows plus the trailing partial row of a
// split boundary -- are either summed by row groups of G = 2^lg lanes (mode lg + 1) or, when
// segment lengths are too uneven for that, by the per-thread merge walk (mode 0).  Cost model
// in latency steps of the slowest group: ceil(segments / groups) rounds of the longest
// segment's reads (SpMV: ceil(longest / G) LDS reads; SpMM: gather batches) plus the shuffle
// fold; the cheapest G wins if its cost is within max_cost (about the walk it replaces: IPT
// reads plus an 11-step search and two barriers for SpMV, IPTG/4 gather chunks for SpMM).
__global__ void k_tile_modes(const int *__restrict__ row_offsets, const int2 *__restrict__ bounds,
                             const unsigned char *__restrict__ split, int num_tiles, int gl, int max_cost,
                             int lanes, unsigned char *__restrict__ modes)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= num_tiles)
        return;
    const int2 b0 = bounds[t], b1 = bounds[t + 1];
    const int nrows = b1.x - b0.x;
    const bool tail = split[t + 1] != 0;
    const int nseg = nrows + (tail ? 1 : 0);
    int longest = 0, prev = b0.y;
    for (int r = 0; r < nrows; ++r) {
        const int e = row_offsets[b0.x + 1 + r];
        longest = max(longest, e - prev);
        prev = e;
    }
    if (tail)
        longest = max(longest, b1.y - prev);
    int best = 0, best_cost = max_cost + 1;
    for (int lg = 0; (gl << lg) <= 64; ++lg) {  // a row group stays inside one wave
        const int groups = lanes / (gl << lg), G = 1 << lg;
        const int rounds = (nseg + groups - 1) / groups;
        const int per_lane = (longest + G - 1) / G;
        // SpMV: LDS product reads, one step each, plus a 3-step shuffle per fold level.
        // SpMM: panel-row gathers in batches of 8 (about 4 steps of latency per batch).
        const int cost = gl == 1 ? rounds * (per_lane + 3 * lg) : rounds * (4 * ((per_lane + 7) / 8) + lg);
        if (cost < best_cost) {
            best_cost = cost;
            best = lg + 1;
        }
    }
    modes[t] = best_cost <= max_cost ? (unsigned char)best : (unsigned char)0;
}

// ------------------------------------------------------------------------------------------
// tile kernels
// ------------------------------------------------------------------------------------------
struct TileArgs {
    const int *__restrict__ row_offsets;
    const int *__restrict__ cols;
    const double *__restrict__ vals;
    const double *__restrict__ x;      // SpMV/SpMM: x / X.   CG: {r, p_old} interleaved (cg_rp)
    const double *__restrict__ xr;     // MODE 2: the rows' own x (row R at xr[R * ld]) for x.(Ax) --
                                       // x itself unless the handle is a row range of x's rows
    const double *__restrict__ p_old;  // (unused by the single-RHS CG: p_old rides with r in x)
    double *__restrict__ xsol;         // CG (MODE 1): the solution; iteration k applies x += alpha_{k-1} p_{k-1}
                                       // to the tile's rows (cg1_lag_*)
    double *__restrict__ p_new;        // CG: the {r, p} buffer of the next iteration; p = r + beta p_old
                                       // is written for the tile's rows at p_new[2 R + 1] (cg_pstore)
    double *__restrict__ y;            // SpMV/SpMM: y / Y.   CG: Ap
    const int2 *__restrict__ bounds;
    const unsigned char *__restrict__ split;
    const unsigned char *__restrict__ rmode;  // per-tile in-tile reduction (k_tile_modes)
    double *__restrict__ carry_val;    // [tile][L] split-row partials, agent-scope stores (close_split_rows)
    const int4 *fix;                   // TilePlan::d_fix / d_fix_cnt (null: the plan splits no row)
    unsigned *fix_cnt;
    unsigned *fault;                   // where a ticket overrun is raised (ticket_arrive): the CG's control word,
                                       // else the handle's fault word (mspmv_check_faults)
    double *head_val;                  // [tile][L]: the first row of a tile that completes a split row
    double *head_pub;                  // [tile][L]: the same, republished with agent scope (close_split_rows)
    double *y0;                        // per tile (set by the kernel): where row 0 of the tile goes --
                                       // y's row, or head_val when the tile completes a split row
    int num_tiles;
    CgScalars *scal;                   // CG: per-column scalars
    CgControl *ctrl;                   // CG: iteration control
    const unsigned char *conv;         // CG: per-column converged flags
    double *partials;                  // CG: per-slot partial dots [slot][L], then level 2 [group][L]
    unsigned *gtickets;                // CG: per-group tickets of reduce_slots (self-resetting)
    double *dot_out;                   // MODE 2: the reduced x.(Ax) per column [L]
    int m;                             // rows (row_offsets holds m + 1 entries)
    // MODE 1 (single-RHS pipelined CG): the previous update's r.r partials (summed by every
    // workgroup), the iteration parity, the stop test and the residual history
    const double *part_in;
    int n_part_in;
    int parity;
    double tol;
    double *hist;
    int hist_cap;
    // single-RHS plans: per-tile 16-bit column offsets (TilePlan::d_colbase / d_cols16; null: off)
    const int *colbase;
    const unsigned short *cols16;
    // single-RHS plans with node blocks (TilePlan::d_blk, k_build_blocks; null: off); all_reg:
    // every tile reduces in registers (host side: launch k_spmv_blk)
    const uint4 *blk;
    int blk_stride;
    int all_reg;
    // single-RHS plans with column dictionaries (TilePlan::d_dict; null: off)
    const int *dict;
    const int *ndict;
    const unsigned short *idx16;
    // SpMM: leading dimension of the x / y panels in doubles (L for whole panels; a column
    // chunk of a wider panel otherwise, mspmv_dspmm with L outside {1, 2, 4, 8, 16})
    int ld;
    // single-RHS tile kernel: load the tile's row ends with its stream (1) instead of after the
    // staging (0) -- one dependent round trip fewer per tile (SpmvTuning::early_re)
    int early_re;
    int blk_rows_max;  // node-block plans: the tallest run (TilePlan::blk_rows_max; k_spmm_blk's KR)
    unsigned long long *stamps;  // k_spmv_tile STAMP (diagnostic): [tile][kTileStamps]
    int tb;            // threads sharing one tile (the plan's lanes: 256, or 64 for one-wave SpMV plans)
    int blk_spmv;      // the plain SpMV runs k_spmv_blk on this plan (TilePlan::blk_spmv; mixed plans too)
    int n;             // columns (x holds n entries)
};

// Tile-kernel modes.
//   0: y = A x.
//   1: fused CG step: gather p = r + beta p_old, Ap = A p, write p for the tile's rows,
//      p.Ap by linearity, last block sets alpha (single GPU).
//   2: y = A x plus x.y over the rows (by linearity), last block writes dot_out (the
//      row-sharded CG, whose x = [p_own | p_halo] was updated and exchanged beforehand).
enum : int { kModeSpmv = 0, kModeCg = 1, kModeDot = 2 };

// Single-RHS pipelined CG keeps r and p interleaved, {r_i, p_i} per row (16 B): the fused
// p = r + beta p_old gather at every nonzero's column is one 16-B load instead of two 8-B loads
// on separate cache lines (the same operands, so the same rounding).  Two such buffers
// alternate by iteration parity: the SpMV reads {r_k, p_{k-1}} and writes p_k into the other
// one, the update reads r_k here and p_k there and writes r_{k+1} next to p_k.
__device__ __forceinline__ double2 cg_rp(const TileArgs &a, long long i)
{
    return reinterpret_cast<const double2 *>(a.x)[i];
}
__device__ __forceinline__ void cg_pstore(const TileArgs &a, long long i, double p) { a.p_new[2 * i + 1] = p; }

// LDS slot of tile-local product k: an XOR swizzle inside each aligned group of 8 doubles,
// so walkers 8 products apart hit different banks, while staging writes and row-group reads
// (consecutive k) stay conflict-free -- no padding, so the tile fits a smaller LDS footprint.
__device__ __forceinline__ int pslot(int k) { return k ^ ((k >> 3) & 7); }

// Stage products val*x[col] (or val*(r + beta p)[col] for CG) of the tile's nonzeros
// [n0, n0+nnzt) into LDS.  Striped: lane l of round j takes nonzero l + 256 j, so each
// gather instruction reads x at 64 CONSECUTIVE nonzeros' columns (runs of neighbouring
// columns share cache lines) -- measured 1.4x faster than 16-byte-per-lane blocked loads,
// whose gathers scatter over 4x more lines.  Every round's loads and gathers are issued
// before any is consumed (indices past the tile clamp to its last nonzero).
// Barrier over the threads that share a tile: the workgroup, or (one-wave workgroups) the wave,
// whose LDS accesses retire in order -- only compiler reordering has to be fenced.
template <int TB>
__device__ __forceinline__ void tile_sync()
{
    if (TB == 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

template <int NJ, bool CG>
struct StageRegs {
    int c[NJ];
    double v[NJ];
    double xv[NJ];
    double pv[CG ? NJ : 1];
};
template <int NJ, bool CG, bool NT, int TB = kBlock>
__device__ __forceinline__ void stage_issue(const TileArgs &a, int n0, int nnzt, int colbase, StageRegs<NJ, CG> &st)
{
    if (colbase >= 0) {  // block-uniform: the tile's 16-bit column offsets
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            st.c[j] = colbase + (int)ld_stream<NT>(a.cols16 + n0 + min((int)threadIdx.x + j * TB, nnzt - 1));
    } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            st.c[j] = ld_stream<NT>(a.cols + n0 + min((int)threadIdx.x + j * TB, nnzt - 1));
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        st.v[j] = ld_stream<NT>(a.vals + n0 + min((int)threadIdx.x + j * TB, nnzt - 1));
    if constexpr (CG) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const double2 v = cg_rp(a, st.c[j]);
            st.xv[j] = v.x;
            st.pv[j] = v.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            st.xv[j] = a.x[st.c[j]];
    }
}
template <int NJ, bool CG, int TB = kBlock>
__device__ __forceinline__ void stage_store(const StageRegs<NJ, CG> &st, int nnzt, double beta, double *s_prod)
{
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int k = (int)threadIdx.x + j * TB;
        double x = st.xv[j];
        if (CG)
            x = x + beta * st.pv[j];
        if (k < nnzt)
            s_prod[pslot(k)] = st.v[j] * x;
    }
}
// Grouped staging (plain SpMV on the 16-bit stream, W = 2: pairs):
// thread tid takes the ABSOLUTE nonzero groups q0 + tid + TB u of W consecutive nonzeros (q0 =
// n0 / W), each one aligned W*8-B value load (W/2 16-B loads) and one aligned W*2-B column load --
// 2/W of the striped form's column loads and 1/2 of its value loads for the same bytes (the stream
// instructions, not its bytes, are what the tile kernel spends here: the nlpkkt120-size SpMV ran
// 5 % faster with pairs, r03q).  Elements of a group outside the tile gather x[colbase] (always a
// valid column) and are not stored.  A tile with a group more than NP * TB (a start off the
// W-grid at the nominal size) issues one extra round (block-uniform).
// Measured and not kept (r03af, r03r): quads (W = 4) 245 vs 223 us and one 16-B x load per
// consecutive pair 261 vs 220 us at the nlpkkt120 size.
constexpr int kGroupW = 2;
typedef unsigned v2u_t __attribute__((ext_vector_type(2)));
template <int NP, int W>
struct GroupRegs {
    unsigned c[NP][W / 2];  // two 16-bit column offsets per word
    double2 v[NP][W / 2];
    double x[NP][W];
};
template <int NP, int W, bool NT, int TB>
__device__ __forceinline__ void group_issue(const TileArgs &a, int n0, int nnzt, int colbase, int ubase,
                                            GroupRegs<NP, W> &st)
{
    const int q0 = n0 / W, qlast = (n0 + nnzt - 1) / W;
    const double2 *v2 = reinterpret_cast<const double2 *>(a.vals);
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        const int q = min(q0 + (int)threadIdx.x + TB * (ubase + u), qlast);
        if constexpr (W == 2) {
            st.c[u][0] = ld_stream<NT>(reinterpret_cast<const unsigned *>(a.cols16) + q);
        } else {
            const v2u_t *c4 = reinterpret_cast<const v2u_t *>(a.cols16);
            const v2u_t cc = NT ? __builtin_nontemporal_load(c4 + q) : c4[q];
            st.c[u][0] = cc.x;
            st.c[u][1] = cc.y;
        }
#pragma unroll
        for (int h = 0; h < W / 2; ++h)
            st.v[u][h] = ld_stream<NT>(v2 + (size_t)q * (W / 2) + h);
    }
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        const int q = min(q0 + (int)threadIdx.x + TB * (ubase + u), qlast);
        const int k0 = W * q - n0;
#pragma unroll
        for (int e = 0; e < W; ++e) {
            const int off = (int)((st.c[u][e >> 1] >> (16 * (e & 1))) & 0xffffu);
            const bool in = k0 + e >= 0 && k0 + e < nnzt;
            st.x[u][e] = a.x[colbase + (in ? off : 0)];
        }
    }
}
template <int NP, int W, int TB>
__device__ __forceinline__ void group_store(const GroupRegs<NP, W> &st, int n0, int nnzt, int ubase, double *s_prod)
{
    const int q0 = n0 / W, qlast = (n0 + nnzt - 1) / W;
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        const int q = q0 + (int)threadIdx.x + TB * (ubase + u);
        if (q > qlast)
            continue;
        const int k0 = W * q - n0;
#pragma unroll
        for (int e = 0; e < W; ++e) {
            const double v = (e & 1) ? st.v[u][e >> 1].y : st.v[u][e >> 1].x;
            if (k0 + e >= 0 && k0 + e < nnzt)
                s_prod[pslot(k0 + e)] = v * st.x[u][e];
        }
    }
}

template <int NJ, bool CG, bool NT>
__device__ __forceinline__ void stage_products(const TileArgs &a, int n0, int nnzt, double beta, double *s_prod)
{
    StageRegs<NJ, CG> st;
    stage_issue<NJ, CG, NT>(a, n0, nnzt, -1, st);
    stage_store<NJ, CG>(st, nnzt, beta, s_prod);
}

// Dictionary staging (plain SpMV, plans built with MSPMV_SPMV_DICT=1): the tile's distinct
// columns are gathered once each (DJ per thread in flight, clamped), parked in LDS, and every
// nonzero's product reads its x there through its 16-bit dictionary position.  The products are
// the same values as the direct path (val * x[col]), so results are bit-identical to it.
template <int NJ, bool NT, int TB>
__device__ __forceinline__ void dict_stage(const TileArgs &a, double *s_prod, int nd, int n0, int nnzt)
{
    constexpr int DJ = 3;
    const int tid = threadIdx.x;
    int ix[NJ];
    double v[NJ];
    int dc[DJ];
    double dx[DJ];
#pragma unroll
    for (int u = 0; u < DJ; ++u)
        dc[u] = ld_stream<NT>(a.dict + n0 + min(tid + u * TB, nd - 1));
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        ix[j] = ld_stream<NT>(a.idx16 + n0 + min(tid + j * TB, nnzt - 1));
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        v[j] = ld_stream<NT>(a.vals + n0 + min(tid + j * TB, nnzt - 1));
#pragma unroll
    for (int u = 0; u < DJ; ++u)
        dx[u] = a.x[dc[u]];
    double *s_x = s_prod;  // nd <= nnzt: the dictionary's x fits the product slots
#pragma unroll
    for (int u = 0; u < DJ; ++u)
        if (tid + u * TB < nd)
            s_x[tid + u * TB] = dx[u];
    for (int d = tid + DJ * TB; d < nd; d += TB)  // rare: > DJ * TB distinct columns
        s_x[d] = a.x[a.dict[n0 + d]];
    tile_sync<TB>();
    double pr[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        pr[j] = v[j] * s_x[ix[j]];
    tile_sync<TB>();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int k = tid + j * TB;
        if (k < nnzt)
            s_prod[pslot(k)] = pr[j];
    }
}

// Node-block staging (k_build_blocks): wave w takes the tile's run chunks w, w + 4, ..., two per
// round.  Per chunk, lane l owns pattern column j = j0 + l: one 16-bit column offset of row P,
// one gather (x, or CG's {r, p}), and the values of that column in every row of the run that is
// long enough -- all of a round's loads issued before any is consumed.  The products
// val * x[col] (CG: val * (r + beta p)) go to the tile's usual LDS slots.  `head` runs once
// between the first round's loads and its products (CG: stop test + beta, as the striped path).
template <bool CG>
struct BlkRegs {
    int c[2];
    double v[2][kBlkRows];
    double xv[2];
    double pv[CG ? 2 : 1];
};

__device__ __forceinline__ uint4 blk_read(const uint4 &bd, int di)
{
    return make_uint4((unsigned)__builtin_amdgcn_readlane((int)bd.x, di),
                      (unsigned)__builtin_amdgcn_readlane((int)bd.y, di),
                      (unsigned)__builtin_amdgcn_readlane((int)bd.z, di),
                      (unsigned)__builtin_amdgcn_readlane((int)bd.w, di));
}

template <bool CG, bool NT, int TB, typename Head>
__device__ __forceinline__ void blk_stage(const TileArgs &a, const uint4 &bd, int nd, int n0, int colbase,
                                          double *s_prod, double &beta, Head &&head)
{
    constexpr int NW = TB / 64;  // waves sharing the tile
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (int round = 0; round * 2 * NW < nd; ++round) {
        BlkRegs<CG> st;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int di = wave + NW * (2 * round + s);
            st.c[s] = 0;
#pragma unroll
            for (int i = 0; i < kBlkRows; ++i)
                st.v[s][i] = 0.0;
            if (di < nd) {  // wave-uniform
                const uint4 d = blk_read(bd, di);
                const int vofs = d.x & 0xffff, j0 = (d.x >> 16) & 255, wc = d.x >> 24;
                const int h = d.y & 15, p = (d.y >> 4) & 7;
                const int j = j0 + lane;
                int start = 0, pstart = 0;
#pragma unroll
                for (int i = 0; i < kBlkRows; ++i) {
                    pstart = i == p ? start : pstart;
                    const int len = blk_len(d, i);
                    if (i < h && j < len)
                        st.v[s][i] = ld_stream<NT>(a.vals + n0 + vofs + start + j);
                    start += i < h ? len : 0;
                }
                if (lane < wc)
                    st.c[s] = colbase + (int)ld_stream<NT>(a.cols16 + n0 + vofs + pstart + j);
            }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (CG) {
                const double2 v = cg_rp(a, st.c[s]);
                st.xv[s] = v.x;
                st.pv[s] = v.y;
            } else {
                st.xv[s] = a.x[st.c[s]];
            }
        }
        if (round == 0 && !head())
            return;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int di = wave + NW * (2 * round + s);
            if (di < nd) {
                const uint4 d = blk_read(bd, di);
                const int vofs = d.x & 0xffff, j0 = (d.x >> 16) & 255;
                const int h = d.y & 15;
                const int j = j0 + lane;
                double x = st.xv[s];
                if (CG)
                    x = x + beta * st.pv[s];
                int start = 0;
#pragma unroll
                for (int i = 0; i < kBlkRows; ++i) {
                    const int len = blk_len(d, i);
                    if (i < h && j < len)
                        s_prod[pslot(vofs + start + j)] = st.v[s][i] * x;
                    start += i < h ? len : 0;
                }
            }
        }
    }
}

// Sum of 8 per-lane values over the wave by a reduce-scatter butterfly (xor 32, 16, 8 halve the
// values each lane carries, then xor 4, 2, 1 finish): lanes 8i .. 8i+7 end up holding row i's
// total (i = lane >> 3).  10 double shuffles for 8 sums instead of 48 for 8 full butterflies;
// the order is fixed, so results are bit-for-bit reproducible.
__device__ __forceinline__ double rows8_sum(const double (&p)[kBlkRows])
{
    const int lane = threadIdx.x & 63;
    const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
    double q4[4], q2[2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        q4[k] = (b5 ? p[k + 4] : p[k]) + __shfl_xor(b5 ? p[k] : p[k + 4], 32);
#pragma unroll
    for (int k = 0; k < 2; ++k)
        q2[k] = (b4 ? q4[k + 2] : q4[k]) + __shfl_xor(b4 ? q4[k] : q4[k + 2], 16);
    double v = (b3 ? q2[1] : q2[0]) + __shfl_xor(b3 ? q2[0] : q2[1], 8);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 1);
    return v;
}

// rows8_sum over the 32 lanes of a half-wave: row i's total lands in lanes 4i .. 4i + 3 of the
// half (i = (lane & 31) >> 2).  Shuffles with xor <= 16 never cross the halves, so the two halves
// fold two different runs with the same 10 shuffles.
__device__ __forceinline__ double rows8_sum32(const double (&p)[kBlkRows])
{
    const int lane = threadIdx.x & 63;
    const bool b4 = lane & 16, b3 = lane & 8, b2 = lane & 4;
    double q4[4], q2[2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        q4[k] = (b4 ? p[k + 4] : p[k]) + __shfl_xor(b4 ? p[k] : p[k + 4], 16);
#pragma unroll
    for (int k = 0; k < 2; ++k)
        q2[k] = (b3 ? q4[k + 2] : q4[k]) + __shfl_xor(b3 ? q4[k] : q4[k + 2], 8);
    double v = (b2 ? q2[1] : q2[0]) + __shfl_xor(b2 ? q2[0] : q2[1], 4);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 1);
    return v;
}

// Plain SpMV form of blk_rows with column PAIRS: each half-wave owns one run per round and its lane
// l owns pattern columns 2l and 2l + 1, so a row of the run arrives in ONE 16-B load per lane (half
// the value-load instructions of column-owner lanes; the loads may be 8-B aligned only -- gfx9's
// unaligned access mode), and one rows8_sum32 folds both halves' runs (half the shuffles).  A
// lane's two products are added before the half-wave tree: a fixed order, so rows stay
// reproducible and within the reordering bound (mode 255).  Column-owner lanes instead: pwtk shape
// 24.98 vs 22.6-23.1 us (r03t).  Per chunk (descriptor bit 7): pattern columns in consecutive pairs
// take ONE 16-B x load per lane.
template <bool NT, int KR>
__device__ __forceinline__ void blk_rows_pair(const TileArgs &a, const uint4 &bd, int nd, int r0, int n0,
                                              int colbase)
{
    constexpr int NW = kBlock / 64;
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5, hl = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (int round = 0; round * 2 * NW < nd; ++round) {
        const int di = wave + NW * (2 * round + half);
        const bool valid = di < nd;
        const int src = min(di, nd - 1);  // descriptor lane (every wave holds all of them in bd)
        const uint4 d = make_uint4((unsigned)__shfl((int)bd.x, src), (unsigned)__shfl((int)bd.y, src),
                                   (unsigned)__shfl((int)bd.z, src), (unsigned)__shfl((int)bd.w, src));
        const int vofs = d.x & 0xffff, wc = d.x >> 24;
        const int h = d.y & 15, p = (d.y >> 4) & 7, rofs = d.y >> 16;
        double2 v[KR];
        bool in0[KR], in1[KR];
        int start = 0, pstart = 0;
#pragma unroll
        for (int i = 0; i < KR; ++i) {
            pstart = i == p ? start : pstart;
            const int len = blk_len(d, i);
            in0[i] = valid && i < h && 2 * hl < len;
            in1[i] = valid && i < h && 2 * hl + 1 < len;
            v[i] = make_double2(0.0, 0.0);
            if (in0[i])
                v[i] = ld_stream<NT>(reinterpret_cast<const double2 *>(a.vals + n0 + vofs + start + 2 * hl));
            start += i < h ? len : 0;
        }
        // the lane's two pattern columns: ONE 4-B load of both 16-bit offsets (2-B aligned at worst; the
        // second belongs to the next position, in bounds by the stream's padding, and is replaced when
        // the lane has one column), then ONE 16-B x load (8-B aligned at worst) for an adjacent pair --
        // FEM nodes list their unknowns consecutively, so nearly every lane's pair is -- and a second
        // load only in lanes whose pair is not (an exec-masked load, skipped when no lane needs it).
        // The load starts at n - 2 at most and picks its half (the last column sits at n - 1 at most).
        unsigned cc = 0u;
        if (valid && 2 * hl < wc)
            cc = ld_stream<NT>(reinterpret_cast<const unsigned *>(a.cols16 + n0 + vofs + pstart + 2 * hl));
        const int c0 = colbase + (int)(cc & 0xffffu);
        const int c1 = (valid && 2 * hl + 1 < wc) ? colbase + (int)(cc >> 16) : c0 + 1;
        const int base = min(c0, a.n - 2);
        const double2 xx = *reinterpret_cast<const double2 *>(a.x + base);
        const double x0 = base == c0 ? xx.x : xx.y;
        double x1 = xx.y;  // c1 == c0 + 1 <= n - 1: base == c0
        if (c1 != c0 + 1)
            x1 = a.x[c1];
        double pr[kBlkRows];
#pragma unroll
        for (int i = 0; i < kBlkRows; ++i)
            pr[i] = i < KR ? (in0[i] ? v[i].x * x0 : 0.0) + (in1[i] ? v[i].y * x1 : 0.0) : 0.0;
        const double sum = rows8_sum32(pr);
        const int myrow = hl >> 2;
        if (valid && (hl & 3) == 0 && myrow < h)
            a.y[r0 + rofs + myrow] = sum;
    }
}

// Node-block tiles whose runs are at most 64 columns wide (one chunk each: FEM node rows) skip
// LDS altogether: lane j of the run's wave holds the products of pattern column j in every row
// of the run, rows8_sum folds them across the wave, and lane 8i stores row i (y; CG: p for the
// row, p.Ap; dot mode: x.(Ax)).  No row-end staging, no barrier, no LDS round trip -- the
// tile's life is its loads plus a few shuffles.  Rows are summed by a fixed lane tree, so they
// are reproducible and within 2 (len+1) eps (|A||x|)_i of the sequential CSR-order sum
// (mspmv_tile_modes reports these tiles as 255).
template <int MODE, bool NT, int TB, typename Head>
__device__ __forceinline__ void blk_rows(const TileArgs &a, const uint4 &bd, int nd, int r0, int n0, int colbase,
                                         double &beta, double &dot, Head &&head)
{
    constexpr bool CG = MODE == kModeCg;
    constexpr int NW = TB / 64;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int myrow = lane >> 3;  // the run row this lane stores (lanes 8i)
    for (int round = 0; round * 2 * NW < nd; ++round) {
        BlkRegs<CG> st;
        double2 ro[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int di = wave + NW * (2 * round + s);
            st.c[s] = 0;
            ro[s] = make_double2(0.0, 0.0);
#pragma unroll
            for (int i = 0; i < kBlkRows; ++i)
                st.v[s][i] = 0.0;
            if (di < nd) {  // wave-uniform
                const uint4 d = blk_read(bd, di);
                const int vofs = d.x & 0xffff, wc = d.x >> 24;
                const int h = d.y & 15, p = (d.y >> 4) & 7, rofs = d.y >> 16;
                int start = 0, pstart = 0;
#pragma unroll
                for (int i = 0; i < kBlkRows; ++i) {
                    pstart = i == p ? start : pstart;
                    const int len = blk_len(d, i);
                    if (i < h && lane < len)
                        st.v[s][i] = ld_stream<NT>(a.vals + n0 + vofs + start + lane);
                    start += i < h ? len : 0;
                }
                if (lane < wc)
                    st.c[s] = colbase + (int)ld_stream<NT>(a.cols16 + n0 + vofs + pstart + lane);
                if (MODE != kModeSpmv && (lane & 7) == 0 && myrow < h) {
                    const int R = r0 + rofs + myrow;
                    if constexpr (CG)
                        ro[s] = cg_rp(a, R);
                    else
                        ro[s].x = a.xr[R];
                }
            }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (CG) {
                const double2 v = cg_rp(a, st.c[s]);
                st.xv[s] = v.x;
                st.pv[s] = v.y;
            } else {
                st.xv[s] = a.x[st.c[s]];
            }
        }
        if (round == 0 && !head())
            return;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int di = wave + NW * (2 * round + s);
            if (di < nd) {
                const uint4 d = blk_read(bd, di);
                const int h = d.y & 15, rofs = d.y >> 16;
                double x = st.xv[s];
                if (CG)
                    x = x + beta * st.pv[s];
                double pr[kBlkRows];
#pragma unroll
                for (int i = 0; i < kBlkRows; ++i)
                    pr[i] = (i < h && lane < blk_len(d, i)) ? st.v[s][i] * x : 0.0;
                const double sum = rows8_sum(pr);
                if ((lane & 7) == 0 && myrow < h) {
                    const int R = r0 + rofs + myrow;
                    a.y[R] = sum;
                    if constexpr (CG) {
                        const double pn = ro[s].x + beta * ro[s].y;
                        cg_pstore(a, R, pn);
                        dot += pn * sum;
                    } else if constexpr (MODE == kModeDot) {
                        dot += ro[s].x * sum;
                    }
                }
            }
        }
    }
}

// Per-tile LDS of the single-RHS kernels.  Products and row ends share one buffer: a tile
// holds nrows + nnzt <= MAXI items, so the nnzt products (slots [0, nnzt) rounded up to the
// swizzle group) followed by the nrows int row ends always fit in MAXI + 8 doubles.
template <int IPT, int TB = kBlock>
struct SpmvSmem {
    static constexpr int TILE = TB * IPT;
    static constexpr int MAXI = TILE + TILE / kSnapDiv;
    static constexpr int MAXJ = (MAXI + TB - 1) / TB;
    double prod[MAXI + 8];
    double red[TB / 64];
    int last;
    __device__ __forceinline__ int *rowend(int nnzt) { return reinterpret_cast<int *>(prod + ((nnzt + 7) & ~7)); }
    // Once a tile's walk has consumed its products and row ends, the walkers' closing pass
    // (row ends reached, carries) reuses the front of prod as scratch: no separate arrays, so a
    // workgroup's LDS is the product buffer alone (18.5 KB at IPT = 8: 8 workgroups per CU).
    __device__ __forceinline__ double *scratch_val() { return prod; }
    __device__ __forceinline__ int *scratch_row() { return reinterpret_cast<int *>(prod + TB); }
    static_assert(MAXI + 8 >= TB + TB / 2, "scratch must fit the product buffer");
};

// Everything after staging, for one tile whose products and row ends are in LDS: one merge
// search per walker, the register walk, in-tile carries, the cross-tile carry, the row
// stores and (CG) the p.Ap contribution.  Called uniformly by all 256 threads; ends with the
// LDS free for the next tile.
template <int IPT, int MODE, int TB = kBlock, bool FIX = true>
__device__ __forceinline__ void walk_tile(const TileArgs &a, SpmvSmem<IPT, TB> &sm, int t, int r0, int n0, int nrows,
                                          int nnzt, bool tail, double beta, double &dot)
{
    constexpr int MAXJ = SpmvSmem<IPT, TB>::MAXJ;
    const int tid = threadIdx.x;
    const int *rend = sm.rowend(nnzt);
    const int items = nrows + nnzt;
    const int ipt = (items + TB - 1) / TB;
    const int d0 = min(tid * ipt, items);
    int cx, cy, ex = nrows, ey = nnzt;
    lds_search(d0, rend, nrows, nnzt, cx, cy);
    // The walker's end is the next walker's start: searched here too (no LDS exchange, so the
    // workgroup needs no scratch arrays beside the product buffer).
    if (tid + 1 < TB)
        lds_search(min(d0 + ipt, items), rend, nrows, nnzt, ex, ey);
    // Does this thread's first row hold nonzeros that earlier threads of the tile consumed?
    const bool need_cin = (cx < ex) && (cy > (cx == 0 ? 0 : rend[cx - 1]));
    // This walker's products, read from LDS up front (independent reads, no dependent chain).
    double pr[MAXJ];
    if (ey > cy) {
#pragma unroll
        for (int j = 0; j < MAXJ; ++j)
            pr[j] = sm.prod[pslot(min(cy + j, ey - 1))];
    }
    auto write_row = [&](int row, double val) {
        const int R = r0 + row;
        *(FIX && row == 0 ? a.y0 : &a.y[R]) = val;
        if (MODE == kModeCg) {
            const double2 v = cg_rp(a, R);
            const double pn = v.x + beta * v.y;
            cg_pstore(a, R, pn);
            dot += pn * val;
        } else if (MODE == kModeDot) {
            dot += a.xr[R] * val;
        }
    };
    double run = 0.0;
    bool first = true, pend = false;
    int prow = 0;
    double pval = 0.0;
    int next_end = cx < ex ? rend[cx] : 0x7fffffff;  // end of the row being accumulated
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        const int k = cy + j;
        if (k < ey) {
            while (next_end <= k) {
                if (first && need_cin) {
                    pend = true;
                    prow = cx;
                    pval = run;
                } else {
                    write_row(cx, run);
                }
                first = false;
                run = 0.0;
                ++cx;
                next_end = cx < ex ? rend[cx] : 0x7fffffff;
            }
            run += pr[j];
        }
    }
    while (cx < ex) {
        if (first && need_cin) {
            pend = true;
            prow = cx;
            pval = run;
        } else {
            write_row(cx, run);
        }
        first = false;
        run = 0.0;
        ++cx;
    }
    tile_sync<TB>();  // every walker is done with the products and row ends: scratch may reuse them
    int *s_row = sm.scratch_row();
    double *s_val = sm.scratch_val();
    s_row[tid] = ex;
    s_val[tid] = run;
    tile_sync<TB>();
    if (pend) {  // close the row begun by earlier threads, summing their carries in thread order
        int j0 = tid - 1;
        while (j0 > 0 && s_row[j0 - 1] == prow)
            --j0;
        double acc = s_val[j0];
        for (int u = j0 + 1; u < tid; ++u)
            acc += s_val[u];
        write_row(prow, acc + pval);
    }
    if (tid == TB - 1 && tail) {  // the tile's trailing partial row -> carry
        int j0 = TB - 1;
        while (j0 > 0 && s_row[j0 - 1] == nrows)
            --j0;
        double acc = s_val[j0];
        for (int u = j0 + 1; u < TB; ++u)
            acc += s_val[u];
        store_sc1(&a.carry_val[t], acc);
        const int R = r0 + nrows;
        if (MODE == kModeCg) {
            const double2 v = cg_rp(a, R);
            dot += (v.x + beta * v.y) * acc;
        }
        else if (MODE == kModeDot)
            dot += a.xr[R] * acc;
    }
    tile_sync<TB>();  // LDS free for the next tile
}

// Row-group reduction of one tile whose products and row ends are in LDS (mode lg + 1 of
// k_tile_modes): groups of G = 2^lg lanes take the tile's row segments round-robin; lane j of
// a group sums products j, j+G, ... of the segment in order from 0.0, then a fixed xor
// butterfly folds the group.  G = 1 is the sequential CSR-order sum of SpmvGold
// (cpu_spmv.cpp:241-265), bit for bit.  A few instructions per product, against the walk's
// merge search and per-item row-end test, for tiles whose rows are alike.
// The group's lane 0 stores the row (G = 1: thread r stores row r, one coalesced store per
// round, as a staged store would be); no LDS beyond the product buffer.  xr / pr: r and p_old
// (CG) or x (dot mode) of row r0 + tid, loaded by the caller for tid <= nrows -- the operands
// of the rows a G = 1 thread owns first; other rows load their own.
template <int IPT, int MODE, int TB = kBlock, bool FIX = true>
__device__ __forceinline__ void group_tile(const TileArgs &a, SpmvSmem<IPT, TB> &sm, int t, int r0, int nrows,
                                           int nnzt, bool tail, double beta, double &dot, int lg, double xr,
                                           double pr)
{
    const int G = 1 << lg;
    const int tid = threadIdx.x;
    const int *rend = sm.rowend(nnzt);
    const int lane = tid & (G - 1);
    const int nseg = nrows + (tail ? 1 : 0);
    auto seg_sum = [&](int r) {
        const int s0 = r == 0 ? 0 : rend[r - 1];
        const int e = r < nrows ? rend[r] : nnzt;
        double v = 0.0;
        int k = s0 + lane;
        for (; k + 3 * G < e; k += 4 * G) {  // four independent LDS reads in flight
            const double p0 = sm.prod[pslot(k)], p1 = sm.prod[pslot(k + G)];
            const double p2 = sm.prod[pslot(k + 2 * G)], p3 = sm.prod[pslot(k + 3 * G)];
            v += p0;
            v += p1;
            v += p2;
            v += p3;
        }
        for (; k < e; k += G)
            v += sm.prod[pslot(k)];
        for (int off = G >> 1; off > 0; off >>= 1)
            v += __shfl_xor(v, off);
        return v;
    };
    for (int r = tid >> lg; r < nseg; r += TB >> lg) {  // uniform within a group
        const double v = seg_sum(r);
        if (lane != 0)
            continue;
        const int R = r0 + r;
        double ox = xr, op = pr;  // the row's operands: preloaded when r is this thread's own row
        if (MODE != kModeSpmv && r != tid) {
            if constexpr (MODE == kModeCg) {
                const double2 w = cg_rp(a, R);
                ox = w.x;
                op = w.y;
            } else {
                ox = a.xr[R];
            }
        }
        if (r < nrows) {
            *(FIX && r == 0 ? a.y0 : &a.y[R]) = v;
            if (MODE == kModeCg) {
                const double pn = ox + beta * op;
                cg_pstore(a, R, pn);
                dot += pn * v;
            } else if (MODE == kModeDot) {
                dot += ox * v;
            }
        } else {  // the trailing partial row -> carry (close_split_rows adds the row's carries in order)
            store_sc1(&a.carry_val[t], v);
            if (MODE == kModeCg)
                dot += (ox + beta * op) * v;
            else if (MODE == kModeDot)
                dot += ox * v;
        }
    }
    tile_sync<TB>();  // LDS free for the next tile
}

// One tile's reduction, by its plan-time mode (a.rmode[t]); tail = a.split[t + 1].
template <int IPT, int MODE, int TB = kBlock, bool FIX = true>
__device__ __forceinline__ void reduce_tile(const TileArgs &a, SpmvSmem<IPT, TB> &sm, int t, int r0, int n0, int nrows,
                                            int nnzt, int mode, bool tail, double beta, double &dot, double xr,
                                            double pr)
{
    if (mode == 0)
        walk_tile<IPT, MODE, TB, FIX>(a, sm, t, r0, n0, nrows, nnzt, tail, beta, dot);
    else
        group_tile<IPT, MODE, TB, FIX>(a, sm, t, r0, nrows, nnzt, tail, beta, dot, mode - 1, xr, pr);
}

// x[r0 + tid] (dot mode), or r and p_old at r0 + tid (CG), for the row-group epilogue, tid <= nrows.
template <int MODE>
__device__ __forceinline__ void row_operands(const TileArgs &a, int r0, int nrows, double &xr, double &pr)
{
    xr = pr = 0.0;
    if (MODE != kModeSpmv && (int)threadIdx.x <= nrows) {
        const int R = min(r0 + (int)threadIdx.x, a.m - 1);
        if constexpr (MODE == kModeCg) {
            const double2 v = cg_rp(a, R);
            xr = v.x;
            pr = v.y;
        } else {
            xr = a.xr[R];
        }
    }
}

// Dot-mode epilogue (split multi-RHS / row-sharded CG): this block's x.(Ax) partial ->
// partials[slot], a plain store; k_fold_dot (a later launch) sums the partials in tile order.
template <typename SM>
__device__ __forceinline__ void dot_epilogue(const TileArgs &a, SM &sm, int slot, double dot)
{
    const double tsum = block_sum(dot, sm.red);
    if (threadIdx.x == 0)
        a.partials[slot] = tsum;
}

// Pipelined single-RHS CG, deferred solution update.  x += alpha_{k-1} p_{k-1} (AxpySingle,
// single_strategy.hpp:143-144, the same expression) is applied by iteration k's SpMV to the rows of
// its tile instead of by the update kernel of iteration k-1: the SpMV already holds p_{k-1} for
// those rows (it rides in the {r, p} buffer it reads), so the update kernel no longer reads p and
// x or writes x.  The last pending term is applied by k_cg1_xflush after the loop.  The operands of
// the tile's first rows are loaded at entry (one row per thread); alpha_{k-1} is scal[0].alpha.
struct CgLag {
    double x, p, alpha;
    int k;
};

template <int TB>
__device__ __forceinline__ void cg1_lag_load(const TileArgs &a, int r0, int nrows, CgLag &g)
{
    const int i = threadIdx.x;
    g.k = a.ctrl->iter_par[a.parity];  // the iteration cg1_head runs (not written by this launch)
    g.alpha = a.scal[0].alpha;
    g.x = g.p = 0.0;
    if (i < nrows) {
        g.x = a.xsol[r0 + i];
        g.p = a.x[2 * (size_t)(r0 + i) + 1];
    }
}

template <int TB>
__device__ __forceinline__ void cg1_lag_store(const TileArgs &a, int r0, int nrows, const CgLag &g)
{
    if (g.k < 1)  // iteration 0: x = 0 and nothing is pending
        return;
    const int i = threadIdx.x;
    if (i < nrows)
        a.xsol[r0 + i] = g.x + g.alpha * g.p;
    for (int j = i + TB; j < nrows; j += TB) {  // tiles of more rows than threads (empty rows)
        const size_t R = (size_t)r0 + j;
        a.xsol[R] = a.xsol[R] + g.alpha * a.x[2 * R + 1];
    }
}

// Pipelined single-RHS CG tail of the SpMV: this tile's p.Ap partial, for the update kernel
// to sum (folded by group tickets only beyond kConsumeTile tiles).
template <typename SM>
__device__ __forceinline__ void cg1_publish(const TileArgs &a, SM &sm, int slot, int nslots, double dot)
{
    const double tsum = block_sum(dot, sm.red);
    if (nslots <= kConsumeTile) {  // the update kernel sums them: the launch boundary orders the store
        if (threadIdx.x == 0)
            a.partials[slot] = tsum;
        return;
    }
    if (threadIdx.x == 0) {  // a ticket tree folds them: publish at agent scope, drained
        store_sc1(&a.partials[slot], tsum);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    publish_partials<1>(a.partials, a.gtickets, slot, nslots, kConsumeTile, sm.prod, sm.red, &sm.last, a.ctrl);
}

// Single right-hand side, one tile per workgroup of TB threads.  TILE = TB*IPT merge items
// nominal, up to 1.125*TILE after snapping.  CG: gathers p = r + beta*p_old on the fly
// (UpdatePSingle, single_strategy.hpp:89-97, fused into the SpMV), writes p for its rows, Ap, and
// p.Ap by linearity.  TB = 64 (one-wave workgroups, SpMV only): every wave owns its tile, so no
// workgroup barrier ties a wave's progress to its siblings' gather latencies.
// BLK = false: the plan has no node-block tiles (a.blk null), and the kernel is compiled without
// their staging paths -- the pipelined CG's form then needs far fewer registers (their run arrays
// set its VGPR count, so more workgroups fit per CU).
// FIX: the plan splits rows (close_split_rows); plans that split none -- FEM, CFD, stencils -- run
// the form without it (fewer SGPRs: 8 workgroups per CU).
// STAMP (diagnostic instantiation only, mspmv_spmv_tile_stamps): thread 0 records wall_clock64() at the
// tile's phase boundaries into a.stamps[t * kTileStamps + i]: 0 entry, 1 stream and gathers issued, 2 the
// staged products in LDS (stream and gathers landed), 3 row ends in LDS (after the barrier), 4 rows
// reduced and stored; slot 5 holds the CU (HW_ID) that ran the tile.
constexpr int kTileStamps = 6;
template <int IPT, int MODE, bool NT, int TB = kBlock, bool BLK = true, bool FIX = true, bool STAMP = false>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(STAMP ? 8 : 1))) void k_spmv_tile(TileArgs a)
{
    static_assert(TB == kBlock || MODE == kModeSpmv, "one-wave tiles run the plain SpMV only");
    constexpr bool CG = MODE == kModeCg;
    constexpr int TILE = SpmvSmem<IPT, TB>::TILE;
    constexpr int MAXJ = SpmvSmem<IPT, TB>::MAXJ;
    __shared__ SpmvSmem<IPT, TB> sm;
    const int tid = threadIdx.x;
    // CG: stop flag loaded now, tested after the stream and gathers are issued (see k_spmm_tile)
    const int stopped = (MODE != kModeSpmv || a.ctrl) ? a.ctrl->done : 0;  // MODE 0: a CG's plain SpMM
    const int t = xcd_tile(blockIdx.x, a.num_tiles);
    auto stamp = [&](int i) {
        if constexpr (STAMP) {
            if (tid == 0) {
                if (i == 0) {
                    unsigned hw;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                    a.stamps[(size_t)t * kTileStamps + 5] = hw;
                }
                a.stamps[(size_t)t * kTileStamps + i] = wall_clock64();
            }
        }
    };
    stamp(0);
    const int2 b0 = a.bounds[t];
    const int2 b1 = a.bounds[t + 1];
    const int r0 = b0.x, n0 = b0.y;
    const int nrows = b1.x - r0;
    const int nnzt = b1.y - n0;
    const int re_pre = a.early_re ? a.row_offsets[min(r0 + 1 + tid, a.m)] : 0;  // TileArgs::early_re
    const int4 fx = FIX ? load_fix(a, t) : make_int4(-1, 0, 0, 0);  // split rows (node-block tiles have none)
    if constexpr (FIX)
        a.y0 = fx.z > 0 ? a.head_val + t : a.y + r0;
    double beta = 0.0;
    bool go = true;
    // CG: the update's r.r partials are loaded first; summed (-> stop test, beta) once this
    // tile's stream and gathers are in flight.  Block-uniform, as is every branch on nnzt.
    PartRegs<CG ? kUpdateMaxBlocks / kBlock : 1> pin;
    CgLag lag{};
    if constexpr (CG) {
        part_load(a.part_in, a.n_part_in, pin);
        cg1_lag_load<TB>(a, r0, nrows, lag);
    }
    auto head = [&]() {  // the stop flag is tested before cg1_head records anything
        if (stopped)
            go = false;
        else if constexpr (CG)
            go = cg1_head(a, part_sum(pin, sm.red), beta);
    };
    const int colbase = a.cols16 ? a.colbase[t] : -1;
    // node-block descriptors of this tile, loaded beside its bounds (entry 0 holds the count)
    uint4 bd = make_uint4(0u, 0u, 0u, 0u);
    if (BLK && a.blk && (tid & 63) < a.blk_stride)
        bd = a.blk[(size_t)t * a.blk_stride + (tid & 63)];
    int nblk = (BLK && a.blk) ? (int)(((unsigned)__builtin_amdgcn_readfirstlane((int)bd.y) >> 8) & 255u) : 0;
    if (nblk > kBlkTileChunks)  // more than one round of runs: striped staging here (k_spmv_blk takes them)
        nblk = 0;
    bool staged = false;
    // every run one chunk wide (block-uniform: each wave holds all descriptors): no LDS at all
    const bool blk_reg = BLK && nblk > 0 && __ballot((tid & 63) < nblk && ((bd.x >> 16) & 255u) != 0) == 0;
    if constexpr (BLK) if (blk_reg) {
        double dot = 0.0;
        blk_rows<MODE, NT, TB>(a, bd, nblk, r0, n0, colbase, beta, dot, [&]() {
            head();
            return go;
        });
        if (!go)
            return;
        if constexpr (MODE == kModeCg) {
            cg1_lag_store<TB>(a, r0, nrows, lag);
            cg1_publish(a, sm, t, a.num_tiles, dot);
        } else if constexpr (MODE == kModeDot) {
            dot_epilogue(a, sm, t, dot);
        }
        return;
    }
    if (BLK && nblk > 0) {
        blk_stage<CG, NT, TB>(a, bd, nblk, n0, colbase, sm.prod, beta, [&]() {
            head();
            return go;
        });
        staged = true;
    } else if constexpr (MODE == kModeSpmv) {
        const int nd = a.dict ? a.ndict[t] : 0;  // > 0: this tile gathers through its dictionary
        if (nd > 0) {
            if (nnzt <= TILE)
                dict_stage<IPT, NT, TB>(a, sm.prod, nd, n0, nnzt);
            else
                dict_stage<MAXJ, NT, TB>(a, sm.prod, nd, n0, nnzt);
            staged = true;
        }
    }
    if (staged) {
    } else if (MODE == kModeSpmv && colbase >= 0 && nnzt > 0 && nnzt <= TILE) {
        constexpr int W = kGroupW;
        constexpr int NP = (TILE / TB + W - 1) / W;
        GroupRegs<NP, W> st;
        group_issue<NP, W, NT, TB>(a, n0, nnzt, colbase, 0, st);
        stamp(1);
        head();
        if (go) {
            group_store<NP, W, TB>(st, n0, nnzt, 0, sm.prod);
            if ((n0 + nnzt - 1) / W - n0 / W + 1 > NP * TB) {  // a start off the W-grid at the nominal size
                GroupRegs<1, W> ex;
                group_issue<1, W, NT, TB>(a, n0, nnzt, colbase, NP, ex);
                group_store<1, W, TB>(ex, n0, nnzt, NP, sm.prod);
            }
        }
    } else if (nnzt > 0 && nnzt <= TILE) {  // the common case: no snapped-in extra nonzeros
        StageRegs<IPT, CG> st;
        stage_issue<IPT, CG, NT, TB>(a, n0, nnzt, colbase, st);
        stamp(1);
        head();
        if (go)
            stage_store<IPT, CG, TB>(st, nnzt, beta, sm.prod);
    } else if (nnzt > TILE) {
        StageRegs<MAXJ, CG> st;
        stage_issue<MAXJ, CG, NT, TB>(a, n0, nnzt, colbase, st);
        head();
        if (go)
            stage_store<MAXJ, CG, TB>(st, nnzt, beta, sm.prod);
    } else {
        head();
    }
    if (!go)
        return;
    if constexpr (STAMP) {  // the staged products' stores are out (LDS): stamp after they complete
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp(2);
    }
    // Row ends: issued with the stream by default (TileArgs::early_re; with the pair staging 1-2 %
    // faster, r03ah/r03ai -- with the old striped staging it had measured +0.9 us on pwtk), or here.
    int *rend = sm.rowend(nnzt);
    if (a.early_re) {
        if (tid < nrows)
            rend[tid] = re_pre - n0;
        for (int i = tid + TB; i < nrows; i += TB)  // rare: more rows than threads
            rend[i] = a.row_offsets[r0 + 1 + i] - n0;
    } else {
        for (int i = tid; i < nrows; i += TB)
            rend[i] = a.row_offsets[r0 + 1 + i] - n0;
    }
    tile_sync<TB>();
    stamp(3);
    double dot = 0.0;
    double xr, pr;
    row_operands<MODE>(a, r0, nrows, xr, pr);
    reduce_tile<IPT, MODE, TB, FIX>(a, sm, t, r0, n0, nrows, nnzt, a.rmode[t], a.split[t + 1] != 0, beta, dot, xr, pr);
    if constexpr (STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows' stores have left
        stamp(4);
    }
    if constexpr (FIX)
        close_split_rows<TB>(a, t, fx, 1, 1);
    if constexpr (MODE == kModeCg) {
        cg1_lag_store<TB>(a, r0, nrows, lag);
        cg1_publish(a, sm, t, a.num_tiles, dot);
    } else if constexpr (MODE == kModeDot) {
        dot_epilogue(a, sm, t, dot);
    }
}

// Register fallback of the plain node-block SpMV for the tiles of a mixed plan that are not register
// run tiles (rows outside any run pattern, patterns wider than 64 columns, split boundaries): groups
// of G lanes take the tile's row segments round-robin (its whole rows, then the trailing partial row
// of a split boundary), lane j of a group sums products j, j + G, ... of its segment in order, a
// fixed xor butterfly folds the group and its lane 0 stores the row (the
// trailing partial row: the tile's carry, which the completing tile adds, close_split_rows).  No LDS, so the kernel keeps its
// register-only occupancy.  G is the smallest power of two with 4 G >= the tile's mean segment
// length.  Reproducible, and within the 2 (len+1) eps (|A||x|)_i reordering bound of the CSR-order
// sum (mspmv_tile_modes reports these tiles as 255).
template <bool NT>
__device__ __forceinline__ void tile_rows_reg(const TileArgs &a, int t, int r0, int n0, int colbase)
{
    const int2 b1 = a.bounds[t + 1];
    const int nrows = b1.x - r0, nnzt = b1.y - n0;
    const int nseg = nrows + (a.split[t + 1] ? 1 : 0);
    if (nseg == 0)
        return;
    const int mean = (nnzt + nseg - 1) / nseg;
    int lg = 0;
    while (lg < 6 && (4 << lg) < mean)
        ++lg;
    const int G = 1 << lg;
    const int lane = threadIdx.x & (G - 1);
    auto col = [&](int k) {
        return colbase >= 0 ? colbase + (int)ld_stream<NT>(a.cols16 + n0 + k) : ld_stream<NT>(a.cols + n0 + k);
    };
    for (int r = (int)threadIdx.x >> lg; r < nseg; r += kBlock >> lg) {  // uniform within a group
        const int s0 = r == 0 ? 0 : a.row_offsets[r0 + r] - n0;
        const int e = r < nrows ? a.row_offsets[r0 + r + 1] - n0 : nnzt;
        double v = 0.0;
        for (int k = s0 + lane; k < e; k += G)
            v += ld_stream<NT>(a.vals + n0 + k) * a.x[col(k)];
        for (int off = G >> 1; off > 0; off >>= 1)
            v += __shfl_xor(v, off);
        if (lane == 0) {
            if (r < nrows)
                *(r == 0 ? a.y0 : &a.y[r0 + r]) = v;
            else
                store_sc1(&a.carry_val[t], v);
        }
    }
}

// Single right-hand side, node-block plans (FEM matrices such as pwtk): the tile kernel without any
// LDS staging (only the CG / dot-mode epilogue's 2 KB), so occupancy is set by registers alone -- 8
// workgroups (32 waves) per CU instead of the 7 that k_spmv_tile's 22.6 KB of LDS allow.  Plain SpMV
// (MODE 0, column pairs): register run tiles through blk_rows_pair, every other tile of the plan
// through tile_rows_reg, so a plan whose tiles are mostly node blocks runs here whole (blk_spmv).
// Dot mode: plans whose EVERY tile is a register run tile, the per-tile work of k_spmv_tile's
// blk_rows path.
struct BlkSmem {
    double red[kBlock / 64];
    double cval[kBlock];
    int last;
};

// FB (plain SpMV): the plan has tiles that are not register run tiles, so the register fallback is
// compiled in; without it the kernel takes 62 SGPRs, with it 84 -- and 256-thread workgroups are
// admitted 8 per CU only up to .sgpr_count 80 (7 at 82-96, MI355X_MICROARCH.md "Residency"), so plans
// of run tiles only keep the lean form.
template <int MODE, bool NT, int KR = kBlkRows, bool FB = false>
__global__ __launch_bounds__(kBlock) void k_spmv_blk(TileArgs a)
{
    constexpr bool CG = MODE == kModeCg;
    __shared__ BlkSmem sm;
    const int tid = threadIdx.x;
    const int stopped = (MODE != kModeSpmv || a.ctrl) ? a.ctrl->done : 0;  // MODE 0: a CG's plain SpMM
    const int t = xcd_tile(blockIdx.x, a.num_tiles);
    const int2 b0 = a.bounds[t];
    const int colbase = a.colbase[t];
    const uint4 bd =
        (tid & 63) < a.blk_stride ? a.blk[(size_t)t * a.blk_stride + (tid & 63)] : make_uint4(0u, 0u, 0u, 0u);
    const int nblk = (int)(((unsigned)__builtin_amdgcn_readfirstlane((int)bd.y) >> 8) & 255u);
    double beta = 0.0, dot = 0.0;
    bool go = true;
    PartRegs<CG ? kUpdateMaxBlocks / kBlock : 1> pin;
    if constexpr (CG)
        part_load(a.part_in, a.n_part_in, pin);
    if constexpr (MODE == kModeSpmv && KR <= 6) {  // taller runs: 73 VGPRs, column owners
        if (stopped)
            return;
        // a register run tile: every chunk starts at pattern column 0 (wave-uniform: each wave holds
        // all descriptors)
        if constexpr (FB) {
            const bool reg = nblk > 0 && __ballot((tid & 63) < nblk && ((bd.x >> 16) & 255u) != 0) == 0;
            if (!reg) {
                const int4 fx = load_fix(a, t);
                a.y0 = fx.z > 0 ? a.head_val + t : a.y + b0.x;
                tile_rows_reg<NT>(a, t, b0.x, b0.y, a.cols16 ? colbase : -1);
                close_split_rows<kBlock>(a, t, fx, 1, 1);
                return;
            }
        }
        blk_rows_pair<NT, KR>(a, bd, nblk, b0.x, b0.y, colbase);
        return;
    }
    blk_rows<MODE, NT, kBlock>(a, bd, nblk, b0.x, b0.y, colbase, beta, dot, [&]() {
        if (stopped)
            go = false;
        else if constexpr (CG)
            go = cg1_head(a, part_sum(pin, sm.red), beta);
        return go;
    });
    if (!go)
        return;
    if constexpr (MODE == kModeCg)
        cg1_publish(a, sm, t, a.num_tiles, dot);
    else if constexpr (MODE == kModeDot)
        dot_epilogue(a, sm, t, dot);
}

// Row-group reduction of one multi-RHS tile (mode lgp + 1): a row group is GL column-pair
// lanes x Gp = 2^lgp nonzero lanes.  Lane (c, j) of a group sums, for its columns 2c, 2c+1,
// the products of nonzeros j, j+Gp, ... of the row in order from 0.0 (four panel-row gathers
// in flight), a fixed xor butterfly over j folds the group, and j = 0 writes the row.
// Gp = 1 is the row-by-row CSR-order sum of the reference's row-split SpMM, bit for bit.
// DICT: s_col holds each nonzero's position in the tile's column dictionary and the panel rows
// are read from s_panel (parked there by k_spmm_tile) -- the same operands, the same sums.
// Dot mode (MODE 2) of the row-group SpMM tiles: the x.(Ax) contribution of the tile's whole rows
// is taken after the row loop, from the Ap rows the workgroup has just stored and the rows' own x
// (both contiguous nrows x L slices, L2-resident: x[R] is a column of row R), instead of holding
// each row's x and the running dot in registers through the gathers -- the dot mode then needs
// no more registers than the plain SpMM, so it keeps the plain kernel's occupancy.

template <int L, bool DICT = false, bool FIX = true>
__device__ __forceinline__ void spmm_group_rows(const TileArgs &a, const int *s_col, const double *s_val,
                                                const int *rend, int t, int r0, int nrows, int nnzt, int lgp,
                                                const double2 *s_panel = nullptr)
{
    constexpr int GL = L / 2;
    const int Gp = 1 << lgp;
    const int tid = threadIdx.x;
    const int lane = tid % GL;
    const int sub = (tid / GL) & (Gp - 1);
    const int W = GL << lgp;
    const bool tail = a.split[t + 1] != 0;
    const int nseg = nrows + (tail ? 1 : 0);
    auto panel = [&](int c) {
        if constexpr (DICT)
            return s_panel[c * GL + lane];
        else
            return *reinterpret_cast<const double2 *>(a.x + (size_t)c * a.ld + 2 * lane);
    };
    for (int r = tid / W; r < nseg; r += kBlock / W) {  // uniform within a group
        const int s0 = r == 0 ? 0 : rend[r - 1];
        const int e = r < nrows ? rend[r] : nnzt;
        double2 acc = make_double2(0.0, 0.0);
        int k = s0 + sub;
        // batches of 8 panel-row gathers in flight per lane (the SpMM is gather-latency bound:
        // bytes in flight per CU set its rate), then 4, then singles; sums stay in order
        for (; k + 7 * Gp < e; k += 8 * Gp) {
            double v[8];
            double2 xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                v[u] = s_val[k + u * Gp];
                xv[u] = panel(s_col[k + u * Gp]);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                acc.x += v[u] * xv[u].x;
                acc.y += v[u] * xv[u].y;
            }
        }
        // the rest (< 8 per lane) as ONE batch, not a chain of single round trips: indices past
        // the row clamp to its last nonzero and their products are skipped by a select (acc
        // starts at +0.0 and never becomes -0.0, so adding +0.0 instead is the identity: the
        // sums stay bit-identical)
        auto rest = [&](auto nb) {
            constexpr int NB = decltype(nb)::value;
            double v[NB];
            double2 xv[NB];
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int kk = min(k + u * Gp, e - 1);
                v[u] = s_val[kk];
                xv[u] = panel(s_col[kk]);
            }
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const bool on = k + u * Gp < e;
                acc.x += on ? v[u] * xv[u].x : 0.0;
                acc.y += on ? v[u] * xv[u].y : 0.0;
            }
        };
        if (k + 3 * Gp < e)
            rest(std::integral_constant<int, 8>{});
        else if (k < e)
            rest(std::integral_constant<int, 4>{});
        for (int off = Gp >> 1; off > 0; off >>= 1) {
            acc.x += __shfl_xor(acc.x, off * GL);
            acc.y += __shfl_xor(acc.y, off * GL);
        }
        if (sub == 0) {
            const size_t off = (size_t)(r0 + r) * a.ld + 2 * lane;
            if (r < nrows)
                // nontemporal: Y does not displace the panel X from the caches (nlpkkt120 size, L = 8:
                // 476 -> 450 us per SpMM, r04n)
                __builtin_nontemporal_store(v2d_t{acc.x, acc.y},
                                            reinterpret_cast<v2d_t *>(FIX && r == 0 ? a.y0 + 2 * lane : a.y + off));
            else  // the trailing partial row -> carry (close_split_rows adds the row's carries in order)
                store_sc1_2(a.carry_val + (size_t)t * L + 2 * lane, acc);
        }
    }
}

// Multi right-hand side (L = 2..16, row-major panels).  A group of L/2 lanes owns one merge
// walk; each lane keeps a double2 of the L running totals (running_total[L],
// merge_based.hpp:84-127).  TILE = (256/(L/2)) groups * IPTG items.
// Workgroups per CU the multi-RHS tile's LDS allows, capped at 7: the register budget is pinned
// to it (the dot mode would otherwise need 90 VGPRs and fall to 5 workgroups at L = 8).
constexpr int spmm_waves_per_eu(int L, int IPTG, bool DICT = false)
{
    const int items = (kBlock / (L / 2)) * IPTG;
    const int lds = 16 * (items + items / kSnapDiv) + 6144 + (DICT ? spmm_dict_bytes(L) : 0);  // + s_crow, s_cval, s_red2
    const int w = 163840 / lds;
    return w < 1 ? 1 : w > 7 ? 7 : w;
}

// DICT: tiles with a column dictionary (multi-RHS plans, k_build_dict) gather each distinct
// panel row once, coalesced (the dictionary is sorted: neighbouring columns share lines), into
// LDS, and the row groups read the panel there: at L = 16 a FEM-blocked tile repeats each of
// its columns ~6 times.  Walk-mode tiles and tiles without one gather directly.  Measured
// (pwtk shape): L = 16 130 -> 102 us; at L = 4 and 8 it lost (47 -> 55, 63 -> 67 us; the
// 27-point nlpkkt120 size at L = 8 505 -> 590 us: the extra dependent round trip and the
// occupancy the 16 KB panel costs outweigh 64-B gathers), so only L = 16 plans build one.
// (Grouped staging, 4 nonzeros per lane: measured even, CG multi L = 8 0.915-0.920 vs 0.914 ms per
// iteration, r03z -- not kept.)
template <int L, int IPTG, int MODE, bool NT, bool DICT = false, bool FIX = true>  // FIX: as k_spmv_tile's
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(spmm_waves_per_eu(L, IPTG, DICT)))) void
k_spmm_tile(TileArgs a)
{
    static_assert(MODE != kModeCg, "multi-RHS CG runs the split iteration (MODE 2)");
    constexpr int GL = L / 2;
    constexpr int NG = kBlock / GL;
    constexpr int TILE = NG * IPTG;
    constexpr int MAXI = TILE + TILE / kSnapDiv;
    constexpr int MAXJ = (MAXI + NG - 1) / NG;
    constexpr int STG = (MAXI + kBlock - 1) / kBlock;
    __shared__ int s_rowend[MAXI];
    __shared__ int s_col[MAXI];
    __shared__ double s_val[MAXI];
    __shared__ int s_crow[NG];
    __shared__ double2 s_cval[NG * GL];
    __shared__ double2 s_red2[kBlock / 64][GL];
    constexpr int DMAX = DICT ? spmm_dict_max(L) : 1;
    constexpr int DJ = (DMAX + NG - 1) / NG;  // dictionary entries per lane group (4)
    __shared__ double2 s_panel[DICT ? DMAX * GL : 1];

    const int tid = threadIdx.x;
    const int g = tid / GL;
    const int lane = tid % GL;
    // CG: the stop flag is loaded now and tested once the tile's stream is in flight, so the
    // flag's round trip does not delay every workgroup's first load (MODE 2 writes only the
    // scratch Ap and partials: a stopped solve only needs the work skipped, not fenced)
    const int stopped = (MODE != kModeSpmv || a.ctrl) ? a.ctrl->done : 0;  // MODE 0: a CG's plain SpMM
    const int t = xcd_tile(blockIdx.x, a.num_tiles);
    const int2 b0 = a.bounds[t];
    const int2 b1 = a.bounds[t + 1];
    const int r0 = b0.x, n0 = b0.y;
    const int nrows = b1.x - r0;
    const int nnzt = b1.y - n0;
    const int items = nrows + nnzt;
    const int rmode = a.rmode[t];
    __shared__ int4 s_fix;  // parked in LDS until the epilogue: no registers held through the tile
    if constexpr (FIX) {
        if (tid == 0)
            s_fix = a.fix ? a.fix[t] : make_int4(-1, 0, 0, 0);
        a.y0 = a.fix && __builtin_amdgcn_readfirstlane(a.fix[t].z) > 0 ? a.head_val + (size_t)t * L
                                                                        : a.y + (size_t)r0 * a.ld;
    }
    int nd = 0;  // > 0: this tile reads its panel rows from s_panel
    if constexpr (DICT) {
        nd = a.ndict[t];
        if (nd > DMAX || rmode == 0)
            nd = 0;
    }
    int dcol[DJ];
    if constexpr (DICT) {  // the dictionary's columns first: the panel gathers wait on them
#pragma unroll
        for (int u = 0; u < DJ; ++u)
            dcol[u] = nd > 0 ? a.dict[n0 + min(g + u * NG, nd - 1)] : 0;
    }

    // Every round's loads are issued before any is stored to LDS (indices clamped into the
    // tile), the first round of row ends with them: one memory round trip per tile, not STG.
    const int re0 = a.row_offsets[min(r0 + 1 + min(tid, max(nrows - 1, 0)), a.m)];  // clamped: always issued
    if (!DICT && nnzt > 0) {  // block-uniform: aligned pairs (one 8-B column load and one 16-B value load
                              // per two nonzeros: half the stream instructions; pairs straddling the
                              // tile's ends load a neighbour's element and skip its store)
        constexpr int STG2 = (MAXI / 2 + 1 + kBlock - 1) / kBlock;
        const int q0 = n0 >> 1, qlast = (n0 + nnzt - 1) >> 1;
        int2 cp[STG2];
        double2 vp[STG2];
#pragma unroll
        for (int j = 0; j < STG2; ++j) {
            const int q = min(q0 + tid + j * kBlock, qlast);
            const v2i_t c = NT ? __builtin_nontemporal_load(reinterpret_cast<const v2i_t *>(a.cols) + q)
                               : reinterpret_cast<const v2i_t *>(a.cols)[q];
            cp[j] = make_int2(c.x, c.y);
        }
#pragma unroll
        for (int j = 0; j < STG2; ++j)
            vp[j] = ld_stream<NT>(reinterpret_cast<const double2 *>(a.vals) + min(q0 + tid + j * kBlock, qlast));
#pragma unroll
        for (int j = 0; j < STG2; ++j) {
            const int q = q0 + tid + j * kBlock;
            const int k = 2 * q - n0;
            if (q <= qlast) {
                if (k >= 0) {
                    s_col[k] = cp[j].x;
                    s_val[k] = vp[j].x;
                }
                if (k + 1 < nnzt) {
                    s_col[k + 1] = cp[j].y;
                    s_val[k + 1] = vp[j].y;
                }
            }
        }
    }
    if (DICT && nnzt > 0) {  // block-uniform
        int cst[STG];
        double vst[STG];
        if (DICT && nd > 0) {
#pragma unroll
            for (int j = 0; j < STG; ++j)
                cst[j] = (int)ld_stream<NT>(a.idx16 + n0 + min(tid + j * kBlock, nnzt - 1));
        } else {
#pragma unroll
            for (int j = 0; j < STG; ++j)
                cst[j] = ld_stream<NT>(a.cols + n0 + min(tid + j * kBlock, nnzt - 1));
        }
#pragma unroll
        for (int j = 0; j < STG; ++j)
            vst[j] = ld_stream<NT>(a.vals + n0 + min(tid + j * kBlock, nnzt - 1));
        if constexpr (DICT) {
            if (nd > 0) {  // each distinct panel row once: lane group g takes entries g, g + NG, ...
                double2 pv[DJ];
#pragma unroll
                for (int u = 0; u < DJ; ++u)
                    pv[u] = *reinterpret_cast<const double2 *>(a.x + (size_t)dcol[u] * a.ld + 2 * lane);
#pragma unroll
                for (int u = 0; u < DJ; ++u)
                    if (g + u * NG < nd)
                        s_panel[(g + u * NG) * GL + lane] = pv[u];
            }
        }
#pragma unroll
        for (int j = 0; j < STG; ++j) {
            const int k = tid + j * kBlock;
            if (k < nnzt) {
                s_col[k] = cst[j];
                s_val[k] = vst[j];
            }
        }
    }
    if (tid < nrows)
        s_rowend[tid] = re0 - n0;
    for (int i = kBlock + tid; i < nrows; i += kBlock)  // rare: > 256 rows in the tile
        s_rowend[i] = a.row_offsets[r0 + 1 + i] - n0;
    __syncthreads();
    if (stopped)
        return;

    double2 dot = make_double2(0.0, 0.0);
    if (rmode != 0) {
        if (DICT && nd > 0)
            spmm_group_rows<L, true, FIX>(a, s_col, s_val, s_rowend, t, r0, nrows, nnzt, rmode - 1, s_panel);
        else
            spmm_group_rows<L, false, FIX>(a, s_col, s_val, s_rowend, t, r0, nrows, nnzt, rmode - 1);
    } else {
    const int ipt = (items + NG - 1) / NG;
    const int d0 = min(g * ipt, items);
    const int d1 = min(d0 + ipt, items);
    int cx, cy, ex, ey;
    lds_search(d0, s_rowend, nrows, nnzt, cx, cy);
    lds_search(d1, s_rowend, nrows, nnzt, ex, ey);
    const bool need_cin = (cx < ex) && (cy > (cx == 0 ? 0 : s_rowend[cx - 1]));

    auto write_row = [&](int row, double2 val) {
        __builtin_nontemporal_store(v2d_t{val.x, val.y},  // nontemporal, as spmm_group_rows' row stores
                                    reinterpret_cast<v2d_t *>(FIX && row == 0 ? a.y0 + 2 * lane
                                                                              : a.y + (size_t)(r0 + row) * a.ld + 2 * lane));
    };

    double2 run = make_double2(0.0, 0.0);
    bool first = true, pend = false;
    int prow = 0;
    double2 pval = make_double2(0.0, 0.0);
    // The walk in chunks of WJ items: each chunk's panel rows are gathered together (WJ
    // independent 16-B loads in flight, indices clamped so every load is issued), then walked.
    constexpr int WJ = 4;
#pragma unroll
    for (int j0 = 0; j0 < MAXJ; j0 += WJ) {
        if (cy + j0 >= ey)
            break;
        double2 xr[WJ];
        double vv[WJ];
#pragma unroll
        for (int jj = 0; jj < WJ; ++jj) {
            const int k = min(cy + j0 + jj, ey - 1);
            vv[jj] = s_val[k];
            xr[jj] = *reinterpret_cast<const double2 *>(a.x + (size_t)s_col[k] * a.ld + 2 * lane);
        }
#pragma unroll
        for (int jj = 0; jj < WJ; ++jj) {
            const int k = cy + j0 + jj;
            if (j0 + jj < MAXJ && k < ey) {
                while (cx < ex && s_rowend[cx] <= k) {
                    if (first && need_cin) {
                        pend = true;
                        prow = cx;
                        pval = run;
                    } else {
                        write_row(cx, run);
                    }
                    first = false;
                    run = make_double2(0.0, 0.0);
                    ++cx;
                }
                run.x += vv[jj] * xr[jj].x;
                run.y += vv[jj] * xr[jj].y;
            }
        }
    }
    while (cx < ex) {
        if (first && need_cin) {
            pend = true;
            prow = cx;
            pval = run;
        } else {
            write_row(cx, run);
        }
        first = false;
        run = make_double2(0.0, 0.0);
        ++cx;
    }
    if (lane == 0)
        s_crow[g] = ex;
    s_cval[g * GL + lane] = run;
    __syncthreads();

    if (pend) {
        int j0 = g - 1;
        while (j0 > 0 && s_crow[j0 - 1] == prow)
            --j0;
        double2 acc = s_cval[j0 * GL + lane];
        for (int u = j0 + 1; u < g; ++u) {
            const double2 c = s_cval[u * GL + lane];
            acc.x += c.x;
            acc.y += c.y;
        }
        acc.x += pval.x;
        acc.y += pval.y;
        write_row(prow, acc);
    }
    if (g == NG - 1 && a.split[t + 1]) {
        int j0 = NG - 1;
        while (j0 > 0 && s_crow[j0 - 1] == nrows)
            --j0;
        double2 acc = s_cval[j0 * GL + lane];
        for (int u = j0 + 1; u < NG; ++u) {
            const double2 c = s_cval[u * GL + lane];
            acc.x += c.x;
            acc.y += c.y;
        }
        store_sc1_2(a.carry_val + (size_t)t * L + 2 * lane, acc);
    }
    }  // merge walk

    if (MODE == kModeDot) {
        // the tile's whole Ap rows, stored above by its own waves (either path): drained, then
        // visible to the workgroup after the barrier (one CU, and no wave read these lines before).
        // Pair e = (row e / GL, columns 2 (e % GL) + {0, 1}); kBlock % GL == 0, so a thread always
        // takes its own column pair `lane`, as the in-loop dot does.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // The trailing partial row (a carry, added to the row by the tile completing it) counts by
        // linearity: its x times the carry this tile stored.  (The row this tile completes is read
        // before close_split_rows adds the earlier tiles' carries to it: they count in their tiles.)
        const int npair = (nrows + (a.split[t + 1] ? 1 : 0)) * GL;
        for (int e = tid; e < npair; e += kBlock) {
            const int row = e / GL;
            const size_t off = (size_t)(r0 + row) * a.ld + 2 * lane;
            const double2 ap = *reinterpret_cast<const double2 *>(
                row < nrows ? (FIX && row == 0 ? a.y0 + 2 * lane : a.y + off) : a.carry_val + (size_t)t * L + 2 * lane);
            const double2 xx = *reinterpret_cast<const double2 *>(a.xr + off);
            dot.x += xx.x * ap.x;
            dot.y += xx.y * ap.y;
        }
    }
    if (MODE != kModeSpmv) {
        // Reduce the per-lane column partials over the groups (lanes with equal tid % GL).
#pragma unroll
        for (int off = 32; off >= GL; off >>= 1) {
            dot.x += __shfl_xor(dot.x, off);
            dot.y += __shfl_xor(dot.y, off);
        }
        if ((tid & 63) < GL)
            s_red2[tid >> 6][lane] = dot;
        __syncthreads();
        if (tid < GL) {
            double2 tsum = s_red2[0][tid];
#pragma unroll
            for (int w = 1; w < kBlock / 64; ++w) {
                tsum.x += s_red2[w][tid].x;
                tsum.y += s_red2[w][tid].y;
            }
            // plain stores: k_fold_dot (a later launch) sums the tiles' partials
            a.partials[(size_t)t * L + 2 * tid] = tsum.x;
            a.partials[(size_t)t * L + 2 * tid + 1] = tsum.y;
        }
    }
    if constexpr (FIX)
        close_split_rows<kBlock>(a, t, s_fix, L, a.ld);  // (s_fix: written before the staging barrier)
}

// ---- node-block SpMM (plans whose every single-RHS tile is a register node-block tile) --------
// Y = A X for L right-hand sides on the single-RHS plan's tiles and run descriptors.  A wave takes
// one run (<= 64 pattern columns) at a time; its lanes form 64/(L/2) column groups of L/2 lanes
// (one double2 of the panel row each).  Per pass a group owns pattern column j: it gathers panel
// row X[P[j]] ONCE and multiplies it into all h rows of the run, so the L2 -> CU gather traffic is
// one panel row per (run, column) instead of one per nonzero (1/6 of it on the pwtk shape).  The
// run's values and P arrive by coalesced loads (lane j holds column j) and reach the column groups
// by shuffles; the h row sums are folded across the groups by a reduce-scatter and group i stores
// row i (L/2 lanes x 16 B, contiguous).  No LDS, no carries (node-block tiles hold whole rows).
template <int GL>
__device__ __forceinline__ double2 rows8_sum2(const double2 (&p)[kBlkRows])
{
    const int lane = threadIdx.x & 63;
    const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
    auto sx = [](double2 v, int off) { return make_double2(__shfl_xor(v.x, off), __shfl_xor(v.y, off)); };
    auto add = [](double2 u, double2 v) { return make_double2(u.x + v.x, u.y + v.y); };
    double2 q4[4], q2[2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        q4[k] = add(b5 ? p[k + 4] : p[k], sx(b5 ? p[k] : p[k + 4], 32));
#pragma unroll
    for (int k = 0; k < 2; ++k)
        q2[k] = add(b4 ? q4[k + 2] : q4[k], sx(b4 ? q4[k] : q4[k + 2], 16));
    double2 v = add(b3 ? q2[1] : q2[0], sx(b3 ? q2[0] : q2[1], 8));
#pragma unroll
    for (int off = 4; off >= GL; off >>= 1)  // column groups inside the 8-lane row slot
        v = add(v, sx(v, off));
    return v;
}

// Waves per SIMD k_spmm_blk is compiled for: 8 (<= 64 VGPRs; with the pass fence below the L = 16
// kernel takes 60 and spills nothing).  Unconstrained the straight-line passes take 82 VGPRs (6
// waves): pwtk L = 16 58.5 vs 51-52 us hot at 8 waves (r03g).  The instantiations that fit 64 VGPRs
// without spilling (plain SpMM, runs of <= 6 rows, L >= 4); the others (L = 2, 8-row runs, dot
// mode) stay unconstrained rather than spill.
constexpr int spmm_blk_waves(int L, int MODE, int KR) { return MODE == 0 && KR <= 6 && L >= 4 ? 8 : 1; }
// KR: the plan's tallest run (rows of one node, <= kBlkRows); KR = 6 (6-DOF FEM such as pwtk)
// holds fewer accumulator and value registers than 8.
template <int L, int MODE, bool NT, int KR = kBlkRows>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(spmm_blk_waves(L, MODE, KR)))) void
k_spmm_blk(TileArgs a)
{
    static_assert(MODE != kModeCg, "multi-RHS CG runs the split iteration (MODE 2)");
    constexpr int GL = L / 2;      // lanes per panel row
    constexpr int NGW = 64 / GL;   // column groups per wave = pattern columns per pass
    // passes whose gathers are in flight together, measured on the pwtk shape: with the values in
    // registers (before LDSV) 4 was best at L = 16 and 2 at L = 4, 8 (r02z); with LDSV 2 is best at
    // every width (L = 16: 72.4-73.1 vs 74.4-74.8 us at 4 and 89.4 at 8; L = 4: 40-41 vs 50-51 and
    // 65 us; r02ah).  Fused multiply-adds instead of the guarded mul + add measured slower.
    // straight-line passes (r03g, pwtk, hot): L = 16 PB 2 50.9-51.7 us vs PB 1 53.4-54.6; L = 8 PB 1
    // 43.0-43.4 vs 43.6-45.6; L = 4 PB 1 37.3 vs 40.5-41.7
    constexpr int PB = L >= 16 ? 2 : 1;
    __shared__ double2 s_red2[MODE == kModeDot ? kBlock / 64 : 1][GL];
    // each wave parks its run's values (row-major, [row][column]) and pattern columns in its own LDS
    // slice, and a pass reads v[i][j] there (one broadcast read per (pass, row)) instead of holding
    // the rows in registers and shuffling them (two bpermutes per (pass, row)): r02ag
    __shared__ __attribute__((aligned(16))) double s_v[kBlock / 64][kBlkRows][64];
    __shared__ int s_c[kBlock / 64][64];
    const int stopped = (MODE != kModeSpmv || a.ctrl) ? a.ctrl->done : 0;  // MODE 0: a CG's plain SpMM
    const int tid = threadIdx.x, lane = tid & 63;
    const int g = lane / GL, c = lane % GL;
    const int t = xcd_tile(blockIdx.x, a.num_tiles);
    const int2 b0 = a.bounds[t];
    const int r0 = b0.x, n0 = b0.y;
    const int colbase = a.colbase[t];
    const uint4 bd = lane < a.blk_stride ? a.blk[(size_t)t * a.blk_stride + lane] : make_uint4(0u, 0u, 0u, 0u);
    const int nd = (int)(((unsigned)__builtin_amdgcn_readfirstlane((int)bd.y) >> 8) & 255u);
    const int wave = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
    double2 dot = make_double2(0.0, 0.0);
    // lane j: P[j] and the run's values in column j of chunk di, one coalesced load per row
    auto fetch = [&](int di, int &cj, double (&vr)[KR]) {
        const uint4 d = blk_read(bd, di);
        const int vofs = d.x & 0xffff, wc = d.x >> 24;
        const int h = d.y & 15, p = (d.y >> 4) & 7;
        int start[KR];
        int pstart = 0, acc_s = 0;
#pragma unroll
        for (int i = 0; i < KR; ++i) {
            start[i] = acc_s;
            pstart = i == p ? acc_s : pstart;
            acc_s += i < h ? blk_len(d, i) : 0;
        }
        cj = lane < wc ? colbase + (int)ld_stream<NT>(a.cols16 + n0 + vofs + pstart + lane) : 0;
#pragma unroll
        for (int i = 0; i < KR; ++i)
            vr[i] = (i < h && lane < blk_len(d, i)) ? ld_stream<NT>(a.vals + n0 + vofs + start[i] + lane) : 0.0;
    };
    for (int di = wave; di < nd && !stopped; di += kBlock / 64) {  // wave-uniform
        const uint4 d = blk_read(bd, di);
        const int wc = d.x >> 24;
        const int h = d.y & 15, rofs = d.y >> 16;
        {  // wave-private slice: the wave's LDS operations stay in order
            int colj;
            double vrow[KR];
            fetch(di, colj, vrow);
            s_c[wave][lane] = colj;
#pragma unroll
            for (int i = 0; i < KR; ++i)  // rows >= h too (0.0 from fetch): the passes read every row
                s_v[wave][i][lane] = vrow[i];
            __builtin_amdgcn_wave_barrier();
        }
        const int ri = lane >> 3;  // the run row this lane's slot stores
        const bool store = (lane & 7) < GL && ri < h;
        double2 xx = make_double2(0.0, 0.0);  // dot mode: the stored row's own x, issued early
        if (MODE == kModeDot && store)
            xx = *reinterpret_cast<const double2 *>(a.xr + (size_t)(r0 + rofs + ri) * a.ld + 2 * c);
        double2 acc[kBlkRows];  // rows KR.. stay 0.0 (compile-time constants: no registers)
#pragma unroll
        for (int i = 0; i < kBlkRows; ++i)
            acc[i] = make_double2(0.0, 0.0);
        // Straight-line passes: every LDS read and gather of a pass is unconditional, so a pass has
        // ONE dependent LDS round trip (its column indices) and one gather round trip, not one per
        // row (the per-row branches serialised six LDS round trips per pass: passes took 6 of a
        // chunk's 8.6 us, r03e stamps).  Lanes past the chunk width hold column 0 (a valid panel
        // row); rows >= h hold 0.0 (fetch) and are never stored.
        int minlen = 64;
#pragma unroll
        for (int i = 0; i < KR; ++i)
            minlen = i < h ? min(minlen, blk_len(d, i)) : minlen;
        int pb = 0;
        // groups of PB passes whose columns all lie in every row of the run: in-place fused
        // multiply-adds, no select, no merge of paths (the accumulators stay in place)
        for (; (pb + PB) * NGW <= minlen; pb += PB) {  // wave-uniform
            int cq[PB];
#pragma unroll
            for (int q = 0; q < PB; ++q)
                cq[q] = s_c[wave][((pb + q) * NGW + g) & 63];
            double2 xv[PB];
#pragma unroll
            for (int q = 0; q < PB; ++q)
                xv[q] = *reinterpret_cast<const double2 *>(a.x + (size_t)cq[q] * a.ld + 2 * c);
#pragma unroll
            for (int q = 0; q < PB; ++q) {
                const int j = (pb + q) * NGW + g;
#pragma unroll
                for (int i = 0; i < KR; ++i) {
                    const double v = s_v[wave][i][j & 63];
                    acc[i].x = __builtin_fma(v, xv[q].x, acc[i].x);
                    acc[i].y = __builtin_fma(v, xv[q].y, acc[i].y);
                }
                // pass q + 1's value reads stay behind pass q's FMAs: without the fence the
                // compiler hoists them and the kernel no longer fits 64 VGPRs (8 waves)
                asm volatile("" ::: "memory");
            }
        }
        // the remaining passes one at a time, each product kept or skipped by a select (the
        // reference's products exactly: a non-finite panel entry in a column a shorter row lacks
        // never reaches that row)
        for (; pb * NGW < wc; ++pb) {  // wave-uniform
            const int j = pb * NGW + g;
            const int cq = s_c[wave][j & 63];
            const double2 xv = *reinterpret_cast<const double2 *>(a.x + (size_t)cq * a.ld + 2 * c);
#pragma unroll
            for (int i = 0; i < KR; ++i) {
                const double v = s_v[wave][i][j & 63];
                const bool on = i < h && j < blk_len(d, i);
                acc[i].x += on ? v * xv.x : 0.0;
                acc[i].y += on ? v * xv.y : 0.0;
            }
        }
        const double2 row = rows8_sum2<GL>(acc);
        if (store) {
            *reinterpret_cast<double2 *>(a.y + (size_t)(r0 + rofs + ri) * a.ld + 2 * c) = row;
            if (MODE == kModeDot) {
                dot.x += xx.x * row.x;
                dot.y += xx.y * row.y;
            }
        }
    }
    if constexpr (MODE == kModeDot) {
        if (stopped)
            return;
        // this tile's x.(Ax) per column: lanes of one column pair (equal c) over the wave, then
        // the waves in order; a plain store (k_fold_dot sums the tiles' partials in a later launch)
#pragma unroll
        for (int off = 32; off >= GL; off >>= 1) {
            dot.x += __shfl_xor(dot.x, off);
            dot.y += __shfl_xor(dot.y, off);
        }
        if (lane < GL)
            s_red2[tid >> 6][lane] = dot;
        __syncthreads();
        if (tid < GL) {
            double2 tsum = s_red2[0][tid];
#pragma unroll
            for (int w = 1; w < kBlock / 64; ++w) {
                tsum.x += s_red2[w][tid].x;
                tsum.y += s_red2[w][tid].y;
            }
            a.partials[(size_t)t * L + 2 * tid] = tsum.x;
            a.partials[(size_t)t * L + 2 * tid + 1] = tsum.y;
        }
    }
}

// Per-column state in CgVecArgs::conv / TileArgs::conv: 0 iterating, 1 converged (the
// reference's converged[] mask), kConvBroken = p.Ap gave a non-finite alpha (frozen).
constexpr unsigned char kConvBroken = 2;

// What the fold's last block derives from the totals (k_fold_dot `mode`).
enum : int { kFoldDot = 0, kFoldCgAlpha = 1, kFoldPcgAlpha = 2, kFoldPcgBeta = 3, kFoldPcgInit = 4 };

// Split CG, after p.Ap of column j is known (one thread per column): the per-column breakdown
// (no_pretreatment.hpp:109-120 has no guard: a zero RHS column gives alpha = 0/0 and a NaN column
// that never converges).  The column is frozen (conv = kConvBroken: alpha = beta = 0 from here on,
// x and r keep their last finite values, left out of the max-error history as the reference's NaN
// is) and the other columns keep iterating.
__device__ __forceinline__ void cg_alpha_column(int j, double pAp, const CgScalars *scal, const unsigned char *conv,
                                                CgControl *ctrl)
{
    if (conv[j])
        return;
    const double alpha = scal[j].rs_old / pAp;
    if (!(alpha == alpha && fabs(alpha) < HUGE_VAL)) {
        const_cast<unsigned char *>(conv)[j] = kConvBroken;
        ctrl->breakdown = 1;
    }
}

// ... then (after a barrier, thread 0): the deferred x term was applied by the p update before
// this reduction (CgVecArgs::lazy_x), and every column converged or broken stops the solve here.
template <int L>
__device__ __forceinline__ void cg_alpha_finish(const unsigned char *conv, CgControl *ctrl)
{
    if (threadIdx.x != 0)
        return;
    ctrl->x_pending = 0;
    if (ctrl->breakdown) {
        int live = 0;
        for (int j = 0; j < L; ++j)
            live += conv[j] == 0;
        if (live == 0) {
            ctrl->done = 1;
            ctrl->iters_out = ctrl->iter + 1;
        }
    }
}

// x.(A x) per column from the tile kernels' MODE 2 partials [T][L], in a fixed order: block g
// folds tiles [g*q, g*q + q) (fold_cols), reduce_slots folds the block sums and its last block
// writes dot_out.  The tile kernels thus end without any ticket or store drain (a ticket per
// tile cost the L = 8 SpMM ~40 % on the nlpkkt120 shape).  scal given (single-GPU split CG): a
// non-finite alpha = rs_old / dot stops the solve before the update touches x and r.
template <int L>
__global__ __launch_bounds__(kBlock) void k_fold_dot(const double *part, int T, int q, double *lvl,
                                                     unsigned *tickets, double *dot_out, CgScalars *scal,
                                                     const unsigned char *conv, CgControl *ctrl, int mode)
{
    __shared__ double s_tmp[kBlock];
    __shared__ double s_out[L];
    __shared__ int s_last;
    const int tid = threadIdx.x;
    if (ctrl && ctrl->done)
        return;
    const int t0 = min((int)blockIdx.x * q, T);
    fold_cols<L>(part + (size_t)t0 * L, min(q, T - t0), s_tmp, s_out);
    if (tid < L) {
        store_sc1(&lvl[(size_t)blockIdx.x * L + tid], s_out[tid]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (!reduce_slots<L, true>(lvl, tickets, blockIdx.x, gridDim.x, s_tmp, s_out, &s_last, ctrl))
        return;
    if (tid < L) {
        const double d = s_out[tid];
        dot_out[tid] = d;
        if (mode == kFoldCgAlpha) {
            cg_alpha_column(tid, d, scal, conv, ctrl);
        } else if (mode == kFoldPcgAlpha) {  // sparse_approximate_inverse.hpp:131-138
            CgScalars &s = scal[tid];
            s.pAp = d;
            s.alpha = (!conv[tid] && d != 0.0) ? s.rs_old / d : 0.0;
        } else if (mode == kFoldPcgBeta) {  // :200-210 (rs_old <- rs_new for every column)
            CgScalars &s = scal[tid];
            s.beta = (!conv[tid] && s.rs_old != 0.0) ? d / s.rs_old : 0.0;
            s.rs_old = d;
        } else if (mode == kFoldPcgInit) {  // :99-100
            scal[tid].rs_old = d;
        }
    }
    if (mode == kFoldCgAlpha) {
        __syncthreads();
        cg_alpha_finish<L>(conv, ctrl);
    }
}

// ------------------------------------------------------------------------------------------
// CG: init and the fused update (x += alpha p; r += (-alpha) Ap; r.r; stop test; beta)
// ------------------------------------------------------------------------------------------
// Column-pair partial sums of a grid-stride loop over n*L elements viewed as pairs.  Each
// thread always meets the same column pair because the stride (in pairs) is a multiple of
// L/2 (L/2 divides 256).  For L == 1 the "pair" is two consecutive rows of one column.
template <int L>
__device__ __forceinline__ void colpair_block_reduce(double2 v, double2 (*s_red2)[L > 1 ? L / 2 : 1],
                                                     double *partials_row)
{
    constexpr int GL = L > 1 ? L / 2 : 1;
    const int tid = threadIdx.x;
    if (L == 1)
        v.x += v.y;
#pragma unroll
    for (int off = 32; off >= GL; off >>= 1) {
        v.x += __shfl_xor(v.x, off);
        if (L > 1)
            v.y += __shfl_xor(v.y, off);
    }
    if ((tid & 63) < GL)
        s_red2[tid >> 6][tid & 63] = v;
    __syncthreads();
    if (tid < GL) {
        double2 s = s_red2[0][tid];
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) {
            s.x += s_red2[w][tid].x;
            s.y += s_red2[w][tid].y;
        }
        if (L == 1) {
            store_sc1(&partials_row[0], s.x);
        } else {
            store_sc1(&partials_row[2 * tid], s.x);
            store_sc1(&partials_row[2 * tid + 1], s.y);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}


struct CgVecArgs {
    long long n_elems;       // n * L
    double *x;
    double *r;
    const double *p;         // CG init: b.  update: p_new
    double *p0;              // init: p0 = b
    const double *ap;
    CgScalars *scal;
    CgControl *ctrl;
    unsigned char *conv;
    double *partials;
    double *hist;
    int hist_cap;
    double tol;
    // Row-sharded CG (mspmv_dist.hip): red_in = all-reduced p.Ap per column (alpha is formed
    // from it in every block); red_out = where the last block leaves this rank's partial sums
    // (b.b at init, r.r at update) for the all-reduce, instead of finishing the scalars.
    const double *red_in;
    double *red_out;
    unsigned *gtickets;  // reduce_slots tickets
    int pcg;             // k_cg_update: SPAI-PCG (beta and rs_old come from R.Z, k_fold_dot)
    // Single-GPU split CG: x += alpha p is deferred from the update to the next p update (which
    // reads p anyway before overwriting it), so the update neither reads p nor reads / writes x.
    // k_cg_update stores each column's masked alpha in scal[j].alpha and raises ctrl->x_pending;
    // k_dist_pupdate applies the term; the fold after it clears the flag; k_cg_xflush applies the
    // term still pending when the solve ends.  Same expression x + alpha p: bit-identical x.
    int lazy_x;
    // Streaming passes of the split CG sweep their chunks of gridDim x kBlock elements last to
    // first (rev = 1) or first to last, alternately, so a pass starts on the lines the previous
    // pass touched last -- still in the 256 MiB Infinity Cache (every lane keeps its column pair).
    int rev;
    // Cache policy of the split CG's passes (the 256 MiB Infinity Cache holds about one L = 8 vector
    // of the nlpkkt120 size): a vector read for the last time before another pass streams over it is
    // loaded nontemporal -- Ap in the r update, p in the p.Ap pass (next read by the p update, two
    // passes on), r and x in the p update (x is touched once per iteration: stored nontemporal too) --
    // so the lines the NEXT pass starts on stay cached: 0.855 -> 0.793 ms per iteration (r04al-r04an;
    // r loaded nontemporal in the r update measured even).
};

// Chunk c (of kBlock x gridDim elements, element i = c * stride + i0) visited at step k: first to
// last, or last to first (CgVecArgs::rev).
__device__ __forceinline__ long long sweep_index(long long k, long long nchunks, long long stride, long long i0, int rev)
{
    return (rev ? nchunks - 1 - k : k) * stride + i0;
}

// The pairs a thread of a streaming CG kernel visits, in order: grid-stride chunks (the whole grid
// sweeps one chunk after another, rev: last chunk first).  (One contiguous slice per workgroup, the
// read ceiling's layout, measured even: CG multi L = 8 0.920-0.921 vs 0.916-0.919 ms, r03aa.)
template <int GL, typename F>
__device__ __forceinline__ void for_pairs(long long npairs, int rev, F &&f)
{
    const long long stride = (long long)gridDim.x * kBlock;
    const long long i0 = (long long)blockIdx.x * kBlock + threadIdx.x;
    const long long nch = (npairs + stride - 1) / stride;
    for (long long k = 0; k < nch; ++k) {
        const long long i = sweep_index(k, nch, stride, i0, rev);
        if (i < npairs)
            f(i);
    }
}

// x = 0, r = p0 = b; rs_old_j = r_j.r_j, b_norm_j = sqrt(b_j.b_j) (no_pretreatment.hpp:61-79,
// single_strategy.hpp:120-131).
template <int L>
__global__ __launch_bounds__(kBlock) void k_cg_init(CgVecArgs a)
{
    constexpr int GL = L > 1 ? L / 2 : 1;
    __shared__ double2 s_red2[kBlock / 64][GL];
    __shared__ double s_colred[kBlock];
    __shared__ double s_out[L];
    __shared__ int s_last;
    const int tid = threadIdx.x;
    const long long npairs = a.n_elems / 2;
    const long long stride = (long long)gridDim.x * kBlock;
    double2 acc = make_double2(0.0, 0.0);
    for (long long i = (long long)blockIdx.x * kBlock + tid; i < npairs; i += stride) {
        const double2 b = reinterpret_cast<const double2 *>(a.p)[i];
        reinterpret_cast<double2 *>(a.x)[i] = make_double2(0.0, 0.0);
        reinterpret_cast<double2 *>(a.r)[i] = b;
        reinterpret_cast<double2 *>(a.p0)[i] = b;
        acc.x += b.x * b.x;
        acc.y += b.y * b.y;
    }
    if ((a.n_elems & 1) && blockIdx.x == 0 && tid == 0) {  // L == 1 with odd n
        const long long i = a.n_elems - 1;
        const double b = a.p[i];
        a.x[i] = 0.0;
        a.r[i] = b;
        a.p0[i] = b;
        acc.x += b * b;
    }
    colpair_block_reduce<L>(acc, s_red2, a.partials + (size_t)blockIdx.x * L);
    if (!reduce_slots<L>(a.partials, a.gtickets, blockIdx.x, gridDim.x, s_colred, s_out, &s_last, a.ctrl))
        return;
    if (a.red_out) {
        if (tid < L)
            a.red_out[tid] = s_out[tid];
    } else {
        if (tid < L) {
            CgScalars &s = a.scal[tid];
            const double bb = s_out[tid];
            s.rs_old = bb;
            double bn = sqrt(bb);
            s.b_norm = bn == 0.0 ? 1.0 : bn;
            s.alpha = 0.0;
            s.beta = 0.0;
            s.pAp = 0.0;
            s.rs_new = 0.0;
            a.conv[tid] = 0;
        }
        if (tid == 0) {
            a.ctrl->iter = 0;
            a.ctrl->done = 0;
            a.ctrl->iters_out = 0;
            a.ctrl->breakdown = 0;
        }
    }
}

// x += alpha p (AxpySingle / axpy_multiple), r += (-alpha) Ap, rs_new = r.r, then on the last
// block: convergence with the reference's masks, history, beta, rs_old
// (single_strategy.hpp:143-163; no_pretreatment.hpp:122-182).
template <int L>
__global__ __launch_bounds__(kBlock) void k_cg_update(CgVecArgs a)
{
    constexpr int GL = L > 1 ? L / 2 : 1;
    __shared__ double2 s_red2[kBlock / 64][GL];
    __shared__ double s_colred[kBlock];
    __shared__ double s_out[L];
    __shared__ int s_last;
    const int tid = threadIdx.x;
    if (a.ctrl->done)
        return;
    const long long npairs = a.n_elems / 2;
    const long long stride = (long long)gridDim.x * kBlock;
    const long long i0 = (long long)blockIdx.x * kBlock + tid;
    double2 al;
    if (a.red_in) {  // alpha_j = rs_old_j / (reduced p.Ap)_j, masked (no_pretreatment.hpp:109-120)
        // A non-finite alpha (breakdown of column j) applies as 0: x_j and r_j stay finite and
        // the column is frozen (k_fold_dot on one GPU, k_dist_finish when sharded).
        auto masked = [&](int j) {
            const double al = a.conv[j] ? 0.0 : a.scal[j].rs_old / a.red_in[j];
            return (al == al && fabs(al) < HUGE_VAL) ? al : 0.0;
        };
        const int j0 = L == 1 ? 0 : 2 * (int)(i0 % GL);
        al.x = masked(j0);
        al.y = L == 1 ? al.x : masked(j0 + 1);
    } else if (L == 1) {
        al.x = a.scal[0].alpha;
        al.y = al.x;
    } else {
        const int cp = (int)(i0 % GL);
        al.x = a.scal[2 * cp].alpha;
        al.y = a.scal[2 * cp + 1].alpha;
    }
    const double2 nal = make_double2(-al.x, -al.y);
    double2 acc = make_double2(0.0, 0.0);
    if (a.lazy_x) {  // x += alpha p: deferred to the next p update (CgVecArgs::lazy_x)
        (void)stride;
        for_pairs<GL>(npairs, 0, [&](long long i) {
            const v2d_t qv = __builtin_nontemporal_load(reinterpret_cast<const v2d_t *>(a.ap) + i);
            const double2 q = make_double2(qv[0], qv[1]);
            double2 r = reinterpret_cast<double2 *>(a.r)[i];
            r.x = r.x + nal.x * q.x;
            r.y = r.y + nal.y * q.y;
            reinterpret_cast<double2 *>(a.r)[i] = r;
            acc.x += r.x * r.x;
            acc.y += r.y * r.y;
        });
    } else {
        for (long long i = i0; i < npairs; i += stride) {
            const double2 p = reinterpret_cast<const double2 *>(a.p)[i];
            const double2 q = reinterpret_cast<const double2 *>(a.ap)[i];
            double2 x = reinterpret_cast<double2 *>(a.x)[i];
            double2 r = reinterpret_cast<double2 *>(a.r)[i];
            x.x = x.x + al.x * p.x;
            x.y = x.y + al.y * p.y;
            r.x = r.x + nal.x * q.x;
            r.y = r.y + nal.y * q.y;
            reinterpret_cast<double2 *>(a.x)[i] = x;
            reinterpret_cast<double2 *>(a.r)[i] = r;
            acc.x += r.x * r.x;
            acc.y += r.y * r.y;
        }
    }
    if ((a.n_elems & 1) && blockIdx.x == 0 && tid == 0) {
        const long long i = a.n_elems - 1;
        if (!a.lazy_x)
            a.x[i] = a.x[i] + al.x * a.p[i];
        const double r = a.r[i] + nal.x * a.ap[i];
        a.r[i] = r;
        acc.x += r * r;
    }
    colpair_block_reduce<L>(acc, s_red2, a.partials + (size_t)blockIdx.x * L);
    if (!reduce_slots<L>(a.partials, a.gtickets, blockIdx.x, gridDim.x, s_colred, s_out, &s_last, a.ctrl))
        return;
    if (a.red_out) {
        if (tid < L)
            a.red_out[tid] = s_out[tid];
    } else {
        if (tid == 0) {
            if (a.lazy_x) {  // this iteration's alpha per column (as every block formed it above,
                             // before the masks below change), for the deferred x += alpha p
                for (int j = 0; j < L; ++j) {
                    const double aj = a.conv[j] ? 0.0 : a.scal[j].rs_old / a.red_in[j];
                    a.scal[j].alpha = (aj == aj && fabs(aj) < HUGE_VAL) ? aj : 0.0;
                }
                a.ctrl->x_pending = 1;
            }
            const int iter = a.ctrl->iter;
            int nconv = 0;
            double maxrel = 0.0;
            for (int j = 0; j < L; ++j) {
                CgScalars &s = a.scal[j];
                const double rs_new = s_out[j];
                s.rs_new = rs_new;
                const double rel = sqrt(rs_new) / s.b_norm;
                // std::max(max, rel): a NaN rel is skipped -- as is a broken-down column, whose
                // reference counterpart is NaN from its breakdown on
                if (a.conv[j] != kConvBroken)
                    maxrel = maxrel < rel ? rel : maxrel;  // std::max: a NaN rel is skipped
                if (!a.conv[j] && rel < a.tol)
                    a.conv[j] = 1;
                nconv += a.conv[j] != 0;
            }
            if (a.hist && iter < a.hist_cap)
                a.hist[iter] = maxrel;
            if (nconv == L) {
                a.ctrl->done = 1;
                a.ctrl->iters_out = iter + 1;
            } else if (!a.pcg) {  // PCG: beta and rs_old follow Z = M R (k_fold_dot kFoldPcgBeta)
                for (int j = 0; j < L; ++j) {
                    CgScalars &s = a.scal[j];
                    s.beta = a.conv[j] ? 0.0 : s.rs_new / s.rs_old;
                    s.rs_old = s.rs_new;
                }
            }
            a.ctrl->iter = iter + 1;
        }
    }
}

// ---- row-sharded CG helpers ------------------------------------------------------------
// After the all-reduce of b.b: rs_old_j = b_j.b_j, b_norm_j = sqrt (or 1), fresh control.
template <int L>
__global__ void k_dist_init_finish(CgVecArgs a)
{
    const int j = threadIdx.x;
    if (j < L) {
        CgScalars &s = a.scal[j];
        const double bb = a.red_in[j];
        s.rs_old = bb;
        const double bn = sqrt(bb);
        s.b_norm = bn == 0.0 ? 1.0 : bn;
        s.alpha = s.beta = s.pAp = s.rs_new = 0.0;
        a.conv[j] = 0;
    }
    if (j == 0) {
        a.ctrl->iter = 0;
        a.ctrl->done = 0;
        a.ctrl->iters_out = 0;
        a.ctrl->breakdown = 0;
    }
}

// p_own = r + beta p_own  (update_p_multiple, utils_multiple.hpp:43-59; beta = 0 on the first
// iteration gives p = r = b, the reference's P = B).
template <int L>
__global__ __launch_bounds__(kBlock) void k_dist_pupdate(CgVecArgs a, double *p)
{
    if (a.ctrl->done)
        return;
    const long long stride = (long long)gridDim.x * kBlock;
    const long long i0 = (long long)blockIdx.x * kBlock + threadIdx.x;
    const bool lag = a.lazy_x && a.ctrl->x_pending;  // the previous update's x += alpha p (lazy_x)
    if (L == 1) {
        const double beta = a.scal[0].beta, alpha = a.scal[0].alpha;
        for (long long i = i0; i < a.n_elems; i += stride) {
            const double q = p[i];
            if (lag)
                a.x[i] = a.x[i] + alpha * q;
            p[i] = a.r[i] + beta * q;
        }
        return;
    }
    // column pairs: the stride (in pairs) is a multiple of L/2, so a thread keeps its pair
    constexpr int GL = L > 1 ? L / 2 : 1;
    const int cp = (int)(i0 % GL);
    const double2 beta = make_double2(a.scal[2 * cp].beta, a.scal[2 * cp + 1].beta);
    const double2 alpha = make_double2(a.scal[2 * cp].alpha, a.scal[2 * cp + 1].alpha);
    const long long npairs = a.n_elems / 2;
    if (lag) {
        for_pairs<GL>(npairs, a.rev, [&](long long i) {
            const v2d_t rv = __builtin_nontemporal_load(reinterpret_cast<const v2d_t *>(a.r) + i);
            const double2 r = make_double2(rv[0], rv[1]);
            double2 q = reinterpret_cast<double2 *>(p)[i];
            const v2d_t xo = __builtin_nontemporal_load(reinterpret_cast<const v2d_t *>(a.x) + i);
            __builtin_nontemporal_store(v2d_t{xo[0] + alpha.x * q.x, xo[1] + alpha.y * q.y},
                                        reinterpret_cast<v2d_t *>(a.x) + i);
            q.x = r.x + beta.x * q.x;
            q.y = r.y + beta.y * q.y;
            reinterpret_cast<double2 *>(p)[i] = q;
        });
        return;
    }
    for (long long i = i0; i < npairs; i += stride) {
        const double2 r = reinterpret_cast<const double2 *>(a.r)[i];
        double2 q = reinterpret_cast<double2 *>(p)[i];
        q.x = r.x + beta.x * q.x;
        q.y = r.y + beta.y * q.y;
        reinterpret_cast<double2 *>(p)[i] = q;
    }
}

// After the split CG's loop: the deferred x += alpha p of the last update, if no p update applied
// it (CgVecArgs::lazy_x).  p still holds that iteration's p: the p updates after the stop return at
// once, and a stop in the fold (every column converged or broken) follows a p update that applied
// the term and a fold that cleared the flag.
template <int L>
__global__ __launch_bounds__(kBlock) void k_cg_xflush(CgVecArgs a, const double *p)
{
    if (!a.ctrl->x_pending)
        return;
    const long long stride = (long long)gridDim.x * kBlock;
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < a.n_elems; i += stride)
        a.x[i] = a.x[i] + a.scal[L == 1 ? 0 : (int)(i % L)].alpha * p[i];
}

// ---- IC(0) preconditioner apply: sync-free sparse triangular solves ---------------------------
// x = T^-1 b for a triangular CSR T, one wave per row: ForwardSolveMultiple (FWD, T = L lower, rows
// ascending) and BackwardSolveMultiple (T = L^T upper, rows descending),
// incomplete_cholesky_decomp.hpp:231-348.  Waves are dispatched in dependency-level order and wait
// only on rows of earlier levels, so every awaited row belongs to a wave already resident or
// finished: no deadlock.  Data-tagged values: the output starts filled with a NaN pattern no
// arithmetic produces (kTrsvPending, written by one 32-bit fill), a row's x values are stored by
// single 8-B write-through stores, and a consumer lane polls the very value it needs until the
// pattern is gone -- one memory round trip per dependency hop (ready flags: poll, load, store, drain,
// raise -- measured 9.8 vs 6.35 ms per iteration, round 1).  Bounded: after ~2^20 polls the solve
// reports a stall instead of hanging the GPU.  The partial sums are folded in a tree, not in CSR
// order (the reference's sequential sum): results agree to rounding.
constexpr unsigned kTrsvPendingWord = 0x7ff4deadu;
constexpr unsigned long long kTrsvPending = 0x7ff4dead7ff4deadull;

__device__ __forceinline__ bool wait_value(const double *p, double &out)
{
    for (int it = 0; it < (1 << 20); ++it) {
        const double v = load_sc1(p);
        if ((unsigned long long)__double_as_longlong(v) != kTrsvPending) {
            out = v;
            return true;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    out = 0.0;
    return false;
}

template <int L, bool FWD>
__global__ __launch_bounds__(kBlock) void k_trsv_tagged(const int *__restrict__ ro, const int *__restrict__ ci,
                                                        const double *__restrict__ va, int n,
                                                        const int *__restrict__ order, const double *b, double *x,
                                                        CgControl *ctrl)
{
    constexpr int NZ = 64 / L;
    const int w = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (w >= n || ctrl->done)  // done is set only by earlier launches: uniform here
        return;
    const int i = order[w];  // rows in (level, row) order: awaited rows belong to earlier waves
    const int lane = threadIdx.x & 63;
    const int v = lane % L, q = lane / L;
    const int k1 = ro[i + 1];
    double sum = 0.0, diag = 0.0;
    bool ok = true;
    for (int k0 = ro[i]; k0 < k1; k0 += NZ) {
        const int k = k0 + q;
        if (k < k1) {
            const int j = ci[k];
            const double a = va[k];
            if (j == i) {
                diag = a;
            } else {
                double xj;
                ok = wait_value(&x[(size_t)j * L + v], xj) && ok;
                sum += a * xj;
            }
        }
    }
#pragma unroll
    for (int off = L; off < 64; off <<= 1) {
        sum += __shfl_xor(sum, off);
        diag += __shfl_xor(diag, off);
    }
    if (q == 0) {
        const double bi = b[(size_t)i * L + v];
        const double xi = (!FWD && diag == 0.0) ? 0.0 : (bi - sum) / diag;
        store_sc1(&x[(size_t)i * L + v], xi);
    }
    if (__ballot(!ok) != 0 && lane == 0) {  // a dependency never arrived: MSPMV_ERR_STALL, never hung
        ctrl->breakdown = 2;
        __hip_atomic_store(&ctrl->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// R.Z per column and the PCG scalars after it (PCGSolveMultiple): mode 0 (init, :96-104)
// rs_old = R.Z; mode 1 (:171-185) beta = converged ? 0 : R.Z / rs_old, rs_old = R.Z.
// Mode 2 (split CG with a plain SpMM, cg_dot_pass): p.Ap per column into red_out, then the
// breakdown checks k_fold_dot makes in kFoldCgAlpha mode.
template <int L>
__global__ __launch_bounds__(kBlock) void k_pcg_dot(CgVecArgs a, int mode)
{
    constexpr int GL = L > 1 ? L / 2 : 1;
    __shared__ double2 s_red2[kBlock / 64][GL];
    __shared__ double s_colred[kBlock];
    __shared__ double s_out[L];
    __shared__ int s_last;
    const int tid = threadIdx.x;
    if (a.ctrl->done)
        return;
    const long long npairs = a.n_elems / 2;
    const long long stride = (long long)gridDim.x * kBlock;
    const long long i0 = (long long)blockIdx.x * kBlock + tid;
    double2 acc = make_double2(0.0, 0.0);
    (void)stride;
    (void)i0;
    if (mode == 2) {  // split CG: a.r = p (next read by the p update, two passes on): nontemporal
        for_pairs<GL>(npairs, a.rev, [&](long long i) {
            const v2d_t r = __builtin_nontemporal_load(reinterpret_cast<const v2d_t *>(a.r) + i);
            const double2 z = reinterpret_cast<const double2 *>(a.p)[i];
            acc.x += r[0] * z.x;
            acc.y += r[1] * z.y;
        });
    } else {
        for_pairs<GL>(npairs, a.rev, [&](long long i) {
            const double2 r = reinterpret_cast<const double2 *>(a.r)[i];
            const double2 z = reinterpret_cast<const double2 *>(a.p)[i];
            acc.x += r.x * z.x;
            acc.y += r.y * z.y;
        });
    }
    if ((a.n_elems & 1) && blockIdx.x == 0 && tid == 0)
        acc.x += a.r[a.n_elems - 1] * a.p[a.n_elems - 1];
    colpair_block_reduce<L>(acc, s_red2, a.partials + (size_t)blockIdx.x * L);
    if (!reduce_slots<L>(a.partials, a.gtickets, blockIdx.x, gridDim.x, s_colred, s_out, &s_last, a.ctrl))
        return;
    if (mode == 2) {  // split CG: p.Ap (a.r = p, a.p = Ap) -> red_out, breakdown per column
        if (tid < L) {
            a.red_out[tid] = s_out[tid];
            cg_alpha_column(tid, s_out[tid], a.scal, a.conv, a.ctrl);
        }
        __syncthreads();
        cg_alpha_finish<L>(a.conv, a.ctrl);
        return;
    }
    if (tid < L) {
        CgScalars &s = a.scal[tid];
        const double d = s_out[tid];
        if (mode == 1)
            s.beta = a.conv[tid] ? 0.0 : d / s.rs_old;
        s.rs_old = d;
    }
}

// Pack the owned entries other ranks need: send[e] = p[idx[e / L] * L + e % L].
__global__ void k_dist_pack(const double *__restrict__ p, const int *__restrict__ idx, long long n_elems, int L,
                            double *__restrict__ send, const CgControl *ctrl)
{
    if (ctrl && ctrl->done)
        return;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n_elems;
         e += (long long)gridDim.x * blockDim.x)
        send[e] = p[(size_t)idx[e / L] * L + e % L];
}

// One block, after the all-reduces of p.Ap (red_in) and r.r (red_out): breakdown test,
// convergence masks, max-residual history, beta, rs_old (no_pretreatment.hpp:109-182).
template <int L>
__global__ void k_dist_finish(CgVecArgs a)
{
    if (threadIdx.x != 0 || a.ctrl->done)
        return;
    const int iter = a.ctrl->iter;
    // The update (k_cg_update with red_in) already applied alpha = 0 to broken columns: their
    // x and r stay as they were; here they are marked and frozen (k_fold_dot's rule, per column).
    for (int j = 0; j < L; ++j) {
        if (a.conv[j])
            continue;
        const double alpha = a.scal[j].rs_old / a.red_in[j];
        if (!(alpha == alpha && fabs(alpha) < HUGE_VAL)) {
            a.ctrl->breakdown = 1;
            a.conv[j] = kConvBroken;
        }
    }
    int nconv = 0;
    double maxrel = 0.0;
    for (int j = 0; j < L; ++j) {
        CgScalars &s = a.scal[j];
        const double rs_new = a.red_out[j];
        s.rs_new = rs_new;
        const double rel = sqrt(rs_new) / s.b_norm;
        if (a.conv[j] != kConvBroken)
            maxrel = maxrel < rel ? rel : maxrel;  // std::max: a NaN rel is skipped
        if (!a.conv[j] && rel < a.tol)
            a.conv[j] = 1;
        nconv += a.conv[j] != 0;
    }
    if (a.hist && iter < a.hist_cap)
        a.hist[iter] = maxrel;
    if (nconv == L) {
        a.ctrl->done = 1;
        a.ctrl->iters_out = iter + 1;
    } else {
        for (int j = 0; j < L; ++j) {
            CgScalars &s = a.scal[j];
            s.beta = a.conv[j] ? 0.0 : s.rs_new / s.rs_old;
            s.rs_old = s.rs_new;
        }
    }
    a.ctrl->iter = iter + 1;
}

// Cache flush between cold calls: by default a READ sweep of a buffer larger than the L2s and
// the 256 MiB Infinity Cache, so the measured kernel finds its data evicted and the caches full
// of clean lines.  A write sweep (MSPMV_FLUSH=write, the first flush of every buffer) leaves them
// full of dirty lines instead, whose write-back the measured kernel then pays as it evicts them
// (measured: the cant-shaped SpMV 31.5 us after a write sweep against 15.5 us hot).
__global__ void k_flush(double *p, long long n, double v)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}
// STREAM-like read of n2 16-byte words (the practical HBM ceiling the roofline is read against,
// SURVEY 8(d)): grid-stride, four nontemporal 16-B loads in flight per thread per step.
// The practical HBM read ceiling (bench `roofline.measured_read_GBps`): every workgroup streams ONE
// contiguous slice of the buffer with nontemporal 16-B loads, two register stages of 8 loads per
// lane in flight.  Measured on MI355X (tools/read_ceiling.hip, r03b), 1 GiB per launch: 6.89-6.90
// TB/s for this shape at 4 or 8 workgroups per CU, against 5.5-5.6 TB/s for the grid-stride loop
// used before (which every workgroup walks across the whole buffer) and 6.4-6.7 TB/s for LDS-DMA.
__global__ __launch_bounds__(kBlock) void k_stream_read(const double2 *p, long long n2, double *sink)
{
    constexpr int U = 8;
    const long long per = (n2 + gridDim.x - 1) / gridDim.x;
    const long long b = (long long)blockIdx.x * per;
    const long long e = b + per < n2 ? b + per : n2;
    const long long step = (long long)kBlock * U;
    auto ld = [&](long long i) { return i < e ? ld_stream<true>(p + i) : make_double2(0.0, 0.0); };
    double acc = 0.0;
    double2 t0[U], t1[U];
    long long i = b + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
        t0[u] = ld(i + u * kBlock);
    for (i += step; i < e + step; i += 2 * step) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            t1[u] = ld(i + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += t0[u].x + t0[u].y;
#pragma unroll
        for (int u = 0; u < U; ++u)
            t0[u] = ld(i + step + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc += t1[u].x + t1[u].y;
    }
    if (acc == -1.0)  // never (the buffer holds zeros): keeps the loads live without a store
        *sink = acc;
}

hipError_t launch_stream_read(const double *p, size_t bytes, int num_cus, hipStream_t s)
{
    const long long n2 = (long long)(bytes / 16);
    hipLaunchKernelGGL(k_stream_read, dim3((unsigned)std::max(1, num_cus * 4)), dim3(kBlock), 0, s,
                       reinterpret_cast<const double2 *>(p), n2, const_cast<double *>(p));
    return hipGetLastError();
}

__global__ void k_flush_read(const double *p, long long n, double *sink)
{
    double acc = 0.0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load(p + i);
    if (acc == -1.0)  // never (the buffer holds +1.0): keeps the loads live without a store
        *sink = acc;
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------

// Tuning.  The shipped values are the measured best; variants measured and not kept are listed in
// DESIGN.md with their session tags.  Two switches stay, each with a GPU parity test of both
// settings: MSPMV_SPMV_BLOCKS=0 (no node blocks in single-RHS plans; test_gpu_blocks.py) and
// MSPMV_SPMM_BLK=0 (multi-RHS products on their own L-wide tiles instead of the node-block SpMM;
// test_gpu_blocks.py, test_gpu_dist.py).  Read once per process.
constexpr int kSpmvIpt = 8;     // merge items per thread of the single-RHS tiles (tile = 256 x 8)
constexpr int kSpmvRgCost = 48; // k_tile_modes budget for single-RHS row-group tiles
struct Switches {
    bool blocks = true;
    bool spmm_blk = true;
};
static const Switches &switches()
{
    static const Switches w = [] {
        Switches v;
        if (const char *e = getenv("MSPMV_SPMV_BLOCKS"))
            v.blocks = atoi(e) != 0;
        if (const char *e = getenv("MSPMV_SPMM_BLK"))
            v.spmm_blk = atoi(e) != 0;
        return v;
    }();
    return w;
}

// Nontemporal policy for the matrix stream: a matrix larger than kNtBytes cannot stay in the
// 256 MiB Infinity Cache across calls anyway, so its lines are not allowed to evict x / X.
constexpr double kNtBytes = 128.0 * 1024 * 1024;
bool stream_nt(const mspmv_handle_s *h) { return 12.0 * (double)h->nnz + 4.0 * (double)h->m > kNtBytes; }

// The node-block SpMV kernel's run height: the pair form holds KR = 6 rows of values per lane.
int blk_kr(const TilePlan &p) { return p.blk_rows_max <= 6 ? 6 : 8; }

std::string spmv_kernel_name(const mspmv_handle_s *h)
{
    if (h->dia == 1)
        return dia_kernel_name(h, 1);
    if (h->spmv_slab == 1)
        return slab_kernel_name(h);
    const std::string nt = stream_nt(h) ? "true" : "false";
    const auto it = h->plans.find(plan_key(1));
    if (h->spmv_onewave != 1 && it != h->plans.end() && it->second.blk_spmv)
        return "k_spmv_blk<0," + nt + (it->second.num_tiles_reg == it->second.num_tiles ? ",6,false>" : ",6,true>");
    if (h->spmv_onewave == 1)
        return "k_spmv_tile<" + std::to_string(kSpmvIpt) + ",0," + nt + ",64,true,true>";
    const bool fix = it != h->plans.end() && it->second.num_carries > 0;
    return "k_spmv_tile<" + std::to_string(kSpmvIpt) + ",0," + nt + ",256,true," + (fix ? "true>" : "false>");
}

int spmv_items_per_thread() { return kSpmvIpt; }

// SpMM tile depth: measured best 8 items per lane group for L <= 4 (fem-blocked pwtk shape,
// L = 4: 55.6 vs 74.8 us at 16), 24 for L = 8 (nlpkkt120 shape, L = 8: 1,536-item tiles of ~55 stencil
// rows -- one round of the 64 row groups -- 439 us vs 467 at 16, 455 at 28, 550 at 32, r04ai; pwtk
// shape flat) and 32 for L = 16 (cant shape: 39.2 -> 28.0 us -- half the tile start-ups at 6
// workgroups per CU instead of 7, r04aa).
int spmm_iptg_for(int L) { return L >= 16 ? 32 : L >= 8 ? 24 : 8; }

// The kernel a plain SpMM of native width L (1, 2, 4, 8, 16) launches on `plan` (get_plan's
// choice for L), spelled as rocprofv3 lists it: launch_spmm_L's dispatch, restated.
std::string spmm_kernel_name(const mspmv_handle_s *h, const TilePlan &plan, int L)
{
    if (L == 1)
        return spmv_kernel_name(h);
    if (plan.dia)
        return dia_kernel_name(h, L);
    if (plan.slab)
        return slab_mm_kernel_name(h, plan);
    const std::string nt = stream_nt(h) ? "true" : "false";
    if (plan.d_blk && plan.num_tiles_reg == plan.num_tiles && spmm_blk_enabled())
        return "k_spmm_blk<" + std::to_string(L) + ",0," + nt + "," + std::to_string(blk_kr(plan)) + ">";
    const int iptg = spmm_iptg_for(L);
    const bool dict = spmm_dict_max(L) > 0 && plan.d_dict;
    return "k_spmm_tile<" + std::to_string(L) + "," + std::to_string(iptg) + ",0," + nt +
           (dict ? ",true,true>" : plan.num_carries > 0 ? ",false,true>" : ",false,false>");
}

// Resident workgroups per CU of a kBlock-thread kernel from its own resources on gfx950: 160 KiB
// of LDS per CU, 512 VGPRs per SIMD lane (granule 8), at most 8 waves per SIMD, 4 SIMDs.
static int gfx950_blocks_per_cu(const void *fn)
{
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, fn) != hipSuccess)
        return 0;
    const int waves_per_block = kBlock / 64;
    const int vgpr = std::max(8, (fa.numRegs + 7) & ~7);
    const int waves_simd = std::min(8, 512 / vgpr);
    int by_waves = 4 * waves_simd / waves_per_block;
    int by_lds = fa.sharedSizeBytes > 0 ? (int)(160 * 1024 / fa.sharedSizeBytes) : by_waves;
    return std::max(0, std::min(by_waves, by_lds));
}

// Slots of the striped single-RHS tile kernels: the SpMV and the pipelined CG (its form without node
// blocks; FEM plans run the node-block kernels, whose tile counts are not near a generation
// boundary), from the kernels' own LDS / VGPR use (the runtime's occupancy query is the fallback
// without attributes).
int spmv_tile_blocks_per_cu()
{
    static const int occ = [] {
        const void *ks = (const void *)k_spmv_tile<kSpmvIpt, kModeSpmv, false, kBlock, true, false>;
        const void *kc = (const void *)k_spmv_tile<kSpmvIpt, kModeCg, false, kBlock, false>;
        const int c = std::min(gfx950_blocks_per_cu(ks), gfx950_blocks_per_cu(kc));
        if (c > 0)
            return c;
        int a = 0, b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_spmv_tile<kSpmvIpt, kModeSpmv, false, kBlock, true, false>,
                                                         kBlock, 0) !=
                hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_spmv_tile<kSpmvIpt, kModeCg, false, kBlock, false>,
                                                         kBlock, 0) != hipSuccess)
            return 0;
        return std::min(a, b);
    }();
    return occ;
}

int tile_items_for(int L)
{
    if (L == 1)
        return kBlock * kSpmvIpt;
    return (kBlock / (L / 2)) * spmm_iptg_for(L);
}

bool supported_L(int L) { return L == 1 || L == 2 || L == 4 || L == 8 || L == 16; }

hipError_t launch_merge_coords(const int *d_row_offsets, int m, int nnz, long long diag_step, int num_parts,
                               int2 *d_out, hipStream_t s)
{
    const int n = num_parts + 1;
    hipLaunchKernelGGL(k_merge_coords, dim3((n + 255) / 256), dim3(256), 0, s, d_row_offsets, m, nnz, diag_step,
                       num_parts, d_out);
    return hipGetLastError();
}

hipError_t launch_pack_cols16(const int *d_cols, const int2 *d_bounds, int num_tiles, int *d_colbase,
                              unsigned short *d_cols16, hipStream_t s)
{
    hipLaunchKernelGGL(k_pack_cols16, dim3(num_tiles), dim3(kBlock), 0, s, d_cols, d_bounds, d_colbase, d_cols16);
    return hipGetLastError();
}

bool spmv_blocks_enabled() { return switches().blocks; }
bool spmm_blk_enabled() { return switches().spmm_blk; }

hipError_t launch_build_blocks(const int *d_row_offsets, const int *d_cols, const int2 *d_bounds,
                               const unsigned char *d_split, const int *d_colbase, int num_tiles, uint4 *d_blk,
                               hipStream_t s, int max_chunks)
{
    static_assert(kBlkMax == kBlkPerTile, "descriptor capacity");
    if (num_tiles <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(k_build_blocks, dim3((num_tiles + 127) / 128), dim3(128), 0, s, d_row_offsets, d_cols, d_bounds,
                       d_split, d_colbase, num_tiles, d_blk, max_chunks);
    return hipGetLastError();
}

// multi: an L-wide plan (dictionaries of at most spmm_dict_max(L) entries: what its kernel parks in
// LDS; the kernel checks the limit again)
hipError_t launch_build_dict(const int *d_cols, const int2 *d_bounds, int num_tiles, int max_items, int *d_dict,
                             int *d_ndict, unsigned short *d_idx16, hipStream_t s, bool multi, int L)
{
    const int ratio = multi ? -1 : 1;
    const int dmax = multi ? spmm_dict_max(L) : 1 << 30;
    if (max_items <= 4096)
        hipLaunchKernelGGL(k_build_dict<4096>, dim3(num_tiles), dim3(kBlock), 0, s, d_cols, d_bounds, d_dict, d_ndict,
                           d_idx16, ratio, dmax);
    else if (max_items <= 8192)
        hipLaunchKernelGGL(k_build_dict<8192>, dim3(num_tiles), dim3(kBlock), 0, s, d_cols, d_bounds, d_dict, d_ndict,
                           d_idx16, ratio, dmax);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_snap(const int *d_row_offsets, int m, int2 *d_bounds, unsigned char *d_split, int num_tiles,
                       int snap, hipStream_t s)
{
    const int n = num_tiles + 1;
    hipLaunchKernelGGL(k_snap, dim3((n + 255) / 256), dim3(256), 0, s, d_row_offsets, m, d_bounds, d_split,
                       num_tiles, snap);
    return hipGetLastError();
}

hipError_t launch_tile_modes(const int *d_row_offsets, const int2 *d_bounds, const unsigned char *d_split,
                             int num_tiles, int L, unsigned char *d_modes, hipStream_t s, int lanes_in)
{
    if (num_tiles == 0)
        return hipSuccess;
    // SpMM budget: twice the walk's gather chunks (4 steps each) plus its search
    const int cost = L == 1 ? kSpmvRgCost : 2 * (4 * (spmm_iptg_for(L) / 4) + 2);
    const int lanes = L == 1 ? lanes_in : kBlock;  // threads sharing one tile
    hipLaunchKernelGGL(k_tile_modes, dim3((num_tiles + 255) / 256), dim3(256), 0, s, d_row_offsets, d_bounds, d_split,
                       num_tiles, L == 1 ? 1 : L / 2, cost, lanes, d_modes);
    return hipGetLastError();
}

static TileArgs make_args(mspmv_handle_s *h, const TilePlan &plan, const double *X, double *Y, int L)
{
    TileArgs a{};
    a.row_offsets = h->d_row_offsets;
    a.m = h->m;
    a.cols = h->d_cols;
    a.vals = h->d_vals;
    a.x = X;
    a.xr = X;
    a.y = Y;
    a.bounds = plan.d_bounds;
    a.split = plan.d_split;
    a.rmode = plan.d_modes[l_index(L)];
    a.carry_val = plan.d_carry_val;
    a.fix = plan.num_carries ? plan.d_fix : nullptr;  // split rows: closed by the tile kernels
    a.fix_cnt = plan.d_fix_cnt;
    a.fault = h->d_fault;
    a.head_val = plan.d_carry_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    a.head_pub = a.head_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    a.num_tiles = plan.num_tiles;
    if (L == 1 || plan.d_blk) {  // L > 1 on a node-block plan: k_spmm_blk (plan_for_L picked it)
        a.colbase = plan.d_colbase;
        a.cols16 = plan.d_cols16;
        a.blk = plan.d_blk;
        a.blk_stride = plan.blk_stride;
        // L > 1 runs the node-block plan only while k_spmm_blk is enabled (get_plan's gate): L = 2
        // shares the single-RHS tile size, so without this the switched-off plan would still be all-reg
        a.all_reg = plan.d_blk && plan.num_tiles_reg == plan.num_tiles && (L == 1 || spmm_blk_enabled());
        a.blk_spmv = L == 1 && plan.blk_spmv;
        a.blk_rows_max = plan.blk_rows_max;
    }
    a.dict = plan.d_dict;
    a.ndict = plan.d_ndict;
    a.idx16 = plan.d_idx16;
    a.ld = L;
    a.early_re = L == 1 ? 1 : 0;
    a.tb = L == 1 ? plan.lanes : kBlock;
    a.n = h->n;
    return a;
}

template <int LL, int I, int MODE>
static void launch_spmm_nt(const TileArgs &a, hipStream_t s, bool nt)
{
    if constexpr (MODE != kModeCg) {
        const dim3 grid(a.num_tiles), block(kBlock);
        if constexpr (spmm_dict_max(LL) > 0) {  // plans with column dictionaries (L = 16; L = 8 when enabled)
            if (a.dict) {
                if (nt)
                    ggl(k_spmm_tile<LL, I, MODE, true, true>, grid, block, s, a);
                else
                    ggl(k_spmm_tile<LL, I, MODE, false, true>, grid, block, s, a);
                return;
            }
        }
        if (MODE == kModeSpmv && !a.fix) {  // no split rows: the form without close_split_rows
            if (nt)
                ggl(k_spmm_tile<LL, I, MODE, true, false, false>, grid, block, s, a);
            else
                ggl(k_spmm_tile<LL, I, MODE, false, false, false>, grid, block, s, a);
        } else if (nt) {
            ggl(k_spmm_tile<LL, I, MODE, true>, grid, block, s, a);
        } else {
            ggl(k_spmm_tile<LL, I, MODE, false>, grid, block, s, a);
        }
    }
}

template <int LL, int MODE>
static void launch_spmm_L(const TileArgs &a, hipStream_t s, bool nt)
{
    if constexpr (MODE != kModeCg) {
        if (a.all_reg) {  // a node-block plan (single-RHS tiles): every tile a register run tile
            const dim3 grid(a.num_tiles), block(kBlock);
            if (a.blk_rows_max <= 6) {
                if (nt)
                    ggl(k_spmm_blk<LL, MODE, true, 6>, grid, block, s, a);
                else
                    ggl(k_spmm_blk<LL, MODE, false, 6>, grid, block, s, a);
            } else if (nt) {
                ggl(k_spmm_blk<LL, MODE, true>, grid, block, s, a);
            } else {
                ggl(k_spmm_blk<LL, MODE, false>, grid, block, s, a);
            }
            return;
        }
    }
    launch_spmm_nt<LL, (LL >= 16 ? 32 : LL >= 8 ? 24 : 8), MODE>(a, s, nt);
}

// MODE 1 (pipelined single-RHS CG) exists for L == 1 in the one-tile kernel only.
template <int MODE>
static hipError_t launch_tile(const TileArgs &a, int L, hipStream_t s, bool nt)
{
    const dim3 grid(a.num_tiles), block(kBlock);
    if (MODE == kModeCg && L != 1)
        return hipErrorInvalidValue;
    switch (L) {
    case 1:
        if (MODE == kModeSpmv && a.blk_spmv) {
            // a node-block plan (every tile, or most: the rest run the kernel's register fallback):
            // the LDS-free kernel, column pairs, runs of <= 6 rows
            if (a.all_reg)  // every tile a register run tile: no register fallback compiled in
                nt ? ggl(k_spmv_blk<kModeSpmv, true, 6>, grid, block, s, a)
                   : ggl(k_spmv_blk<kModeSpmv, false, 6>, grid, block, s, a);
            else
                nt ? ggl(k_spmv_blk<kModeSpmv, true, 6, true>, grid, block, s, a)
                   : ggl(k_spmv_blk<kModeSpmv, false, 6, true>, grid, block, s, a);
        } else if (MODE == kModeDot && a.all_reg) {
            // every tile a register node-block tile, dot mode (the row-sharded CG): column owners
            if (nt)
                ggl(k_spmv_blk<kModeDot, true>, grid, block, s, a);
            else
                ggl(k_spmv_blk<kModeDot, false>, grid, block, s, a);
        } else if (MODE == kModeSpmv && a.tb == 64) {  // one-wave tiles (skewed rows, spmv_plan)
            if (nt)
                ggl(k_spmv_tile<kSpmvIpt, kModeSpmv, true, 64>, grid, dim3(64), s, a);
            else
                ggl(k_spmv_tile<kSpmvIpt, kModeSpmv, false, 64>, grid, dim3(64), s, a);
        } else if (MODE == kModeCg && !a.blk) {  // the pipelined CG without node blocks: fewer VGPRs
            if (nt)
                ggl(k_spmv_tile<kSpmvIpt, MODE, true, kBlock, false>, grid, block, s, a);
            else
                ggl(k_spmv_tile<kSpmvIpt, MODE, false, kBlock, false>, grid, block, s, a);
        } else if (MODE == kModeSpmv && !a.fix) {  // no split rows: the form without close_split_rows
            if (nt)
                ggl(k_spmv_tile<kSpmvIpt, MODE, true, kBlock, true, false>, grid, block, s, a);
            else
                ggl(k_spmv_tile<kSpmvIpt, MODE, false, kBlock, true, false>, grid, block, s, a);
        } else if (nt) {
            ggl(k_spmv_tile<kSpmvIpt, MODE, true>, grid, block, s, a);
        } else {
            ggl(k_spmv_tile<kSpmvIpt, MODE, false>, grid, block, s, a);
        }
        break;
    case 2: launch_spmm_L<2, MODE>(a, s, nt); break;
    case 4: launch_spmm_L<4, MODE>(a, s, nt); break;
    case 8: launch_spmm_L<8, MODE>(a, s, nt); break;
    case 16: launch_spmm_L<16, MODE>(a, s, nt); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Diagnostic: the plain single-RHS SpMV of a plan that runs k_spmv_tile on 256-thread workgroups, in its
// stamped instantiation (mspmv_spmv_tile_stamps).  hipErrorNotSupported for plans that run another kernel.
hipError_t launch_spmv_tile_stamped(mspmv_handle_s *h, const TilePlan &plan, const double *d_x, double *d_y,
                                   unsigned long long *d_stamps)
{
    TileArgs a = make_args(h, plan, d_x, d_y, 1);
    if (a.blk_spmv || a.tb == 64 || plan.dia || plan.slab)
        return hipErrorNotSupported;
    a.stamps = d_stamps;
    const dim3 grid(a.num_tiles), block(kBlock);
    if (plan.num_tiles == 0)
        return hipSuccess;
    const bool nt = stream_nt(h);
    if (!a.fix)
        nt ? ggl(k_spmv_tile<kSpmvIpt, kModeSpmv, true, kBlock, true, false, true>, grid, block, h->stream, a)
           : ggl(k_spmv_tile<kSpmvIpt, kModeSpmv, false, kBlock, true, false, true>, grid, block, h->stream, a);
    else
        nt ? ggl(k_spmv_tile<kSpmvIpt, kModeSpmv, true, kBlock, true, true, true>, grid, block, h->stream, a)
           : ggl(k_spmv_tile<kSpmvIpt, kModeSpmv, false, kBlock, true, true, true>, grid, block, h->stream, a);
    return hipGetLastError();
}

hipError_t launch_spmm_tile_only(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                                 int ld)
{
    if (plan.num_tiles == 0)
        return hipSuccess;
    if (plan.dia)  // offset windows: every width on one plan
        return launch_dia(h, plan, d_X, d_Y, L, ld, nullptr);
    if (plan.slab) {  // a column-slab plan: the plain SpMV's (spmv_plan) or an L-wide SpMM's (get_plan)
        if (plan.slab->L != L)
            return hipErrorInvalidValue;
        return L == 1 ? launch_slab(h, plan, d_X, d_Y) : launch_slab_mm(h, plan, d_X, d_Y, L, ld, nullptr);
    }
    TileArgs a = make_args(h, plan, d_X, d_Y, L);
    if (ld > 0)
        a.ld = ld;
    return launch_tile<kModeSpmv>(a, L, h->stream, stream_nt(h));
}

// Column block copy between row-major panels: dst[i][j] = (j < cols ? src[i][j] : 0) for
// j < dcols (dcols > cols: the zero column of an odd-L panel padded to even width).  Gathers a
// column group out of a wider panel, scatters it back, pads and unpads.
__global__ void k_panel_copy(const double *__restrict__ src, int lds, double *__restrict__ dst, int ldd,
                             long long rows, int cols, int dcols)
{
    const long long total = rows * dcols;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const long long i = e / dcols;
        const int j = (int)(e - i * dcols);
        dst[i * ldd + j] = j < cols ? src[i * lds + j] : 0.0;
    }
}

hipError_t launch_panel_copy(const double *src, int lds, double *dst, int ldd, long long rows, int cols, int dcols,
                             hipStream_t s)
{
    const long long total = rows * dcols;
    if (total <= 0)
        return hipSuccess;
    const long long b = std::min<long long>((total + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_panel_copy, dim3((unsigned)b), dim3(kBlock), 0, s, src, lds, dst, ldd, rows, cols, dcols);
    return hipGetLastError();
}

hipError_t launch_spmm(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                       int *kernels_launched, int ld)
{
    const hipError_t e = launch_spmm_tile_only(h, plan, d_X, d_Y, L, ld);
    if (kernels_launched)
        *kernels_launched = plan.num_tiles ? 1 : 0;
    return e;
}

// Workgroups of the CG's streaming passes: ~12 pairs per thread, at most three per CU -- fewer,
// longer-lived workgroups stream faster here: configs[4] (nlpkkt120 size, L = 8) 0.915 -> 0.886 ms
// per iteration against the old 2,048 (~4 pairs per thread); 4 and 2 per CU 0.895 / 0.893 (r04ae,
// r04af).
int cg_update_blocks(long long elems, int /*num_cus*/)
{
    // ~12 pairs per thread on long vectors, capped at 768 workgroups (3 per CU of the whole chip).  Below that
    // (a single-RHS vector of a few hundred thousand rows: 70 workgroups at 12 pairs) one pair per thread up to
    // the cap instead: the passes are latency bound on a quarter of the CUs otherwise -- 15.4 us per pass on
    // the 427,500-row CG (r06e trace).  The grid -- and so every partial sum's order -- does not depend on the
    // handle's CU limit: a CU mask changes the speed of a solve, never its iterates (tests/test_parallel_
    // efficiency.py; round 5's cap of 3 per *available* CU made it depend on them).
    constexpr long long cap = 768;
    const long long pairs = (elems + 1) / 2;
    long long b = std::max((pairs + kBlock * 12 - 1) / (kBlock * 12), std::min((pairs + kBlock - 1) / kBlock, cap));
    if (b < 1)
        b = 1;
    if (b > cap)
        b = cap;
    return (int)b;
}

// Iterations per CG batch (one graph replay).  The host inspects batch b's control word while
// b + 1 runs, so a solve launches up to 2K - 1 iterations past its convergence (each returning
// early, but a multi-RHS SpMM still streams part of its tile before its stop test).  K = 32 wasted
// 48 of 96 launched iterations on the nlpkkt120-size 8-RHS solve (584 us each): size K so a batch
// lasts ~300 us at ~5 TB/s of the SURVEY 8(d) iteration bytes -- long enough to hide the host's
// check, short enough to bound the overshoot.  Even (the p buffers alternate by parity), 2..32.
// MSPMV_CG_BATCH overrides (lab).
int cg_batch_iters(long long m, long long nnz, int L)
{
    static const int forced = [] {
        const char *e = getenv("MSPMV_CG_BATCH");
        return e ? atoi(e) : 0;
    }();
    int k = forced;
    if (k <= 0) {
        const double est_us = (12.0 * (double)nnz + 88.0 * (double)m * L) / 5.0e6;
        k = (int)std::ceil(300.0 / std::max(est_us, 1.0));
    }
    k = (k + 1) & ~1;
    return std::min(32, std::max(2, k));
}

template <int L>
static void launch_vec(bool init, const CgVecArgs &a, int nblk, hipStream_t s)
{
    if (init)
        hipLaunchKernelGGL((k_cg_init<L>), dim3(nblk), dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL((k_cg_update<L>), dim3(nblk), dim3(kBlock), 0, s, a);
}

static hipError_t dispatch_vec(bool init, const CgVecArgs &a, int L, int nblk, hipStream_t s)
{
    switch (L) {
    case 1: launch_vec<1>(init, a, nblk, s); break;
    case 2: launch_vec<2>(init, a, nblk, s); break;
    case 4: launch_vec<4>(init, a, nblk, s); break;
    case 8: launch_vec<8>(init, a, nblk, s); break;
    case 16: launch_vec<16>(init, a, nblk, s); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_cg_init(mspmv_handle_s *h, const double *d_b, double *d_x, int L, double tol, int nblk)
{
    CgVecArgs a{};
    a.n_elems = (long long)h->m * L;
    a.x = d_x;
    a.r = h->d_r;
    a.p = d_b;
    a.p0 = h->d_p0;
    a.scal = h->d_scal;
    a.ctrl = h->d_ctrl;
    a.conv = h->d_conv;
    a.partials = h->d_partials;
    a.gtickets = h->d_gtickets;
    a.tol = tol;
    return dispatch_vec(true, a, L, nblk, h->stream);
}

hipError_t launch_dist_vec(int which, const CgVecArgs &a, int L, int nblk, double *p, hipStream_t s);

// ---- pipelined single-RHS CG (consumer-side reductions, no ticket chains) -------------------
// Iteration k = [k_spmv_tile MODE 1: stop test + beta from the r.r partials, p = r + beta p_old
// gathered, Ap, p.Ap partials] -> [k_cg1_update: alpha from the p.Ap partials, x, r, r.r
// partials].  Each kernel sums its producer's partials itself (part_load / part_sum), so no
// kernel ends on a chain of tickets and folds.
struct Cg1Args {
    long long m;
    double *x;
    double *rp;            // init: {r, p_0} = {b, b}.  update: {r_k, p_{k-1}} (r_k read at rp[2 i])
    double *rp_next;       // update: {., p_k} -> {r_{k+1}, p_k} (p_k read, r_{k+1} written)
    const double *b;       // init
    const double *ap;
    CgScalars *scal;
    CgControl *ctrl;
    const double *part_in;  // producer partials (update: the SpMV's p.Ap; finish: the update's r.r)
    int n_part_in;
    double *part_out;       // this kernel's per-block partials (r.r, or b.b at init)
    int parity;
    double *hist;
    int hist_cap;
};

// x = 0, {r, p_0} = {b, b} (interleaved, see cg_rp), and this block's b.b partial (the first
// SpMV sums them: rs_0, ||b||).
__global__ __launch_bounds__(kBlock) void k_cg1_init(Cg1Args a)
{
    __shared__ double s_red[kBlock / 64];
    double acc = 0.0;
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < a.m; i += (long long)gridDim.x * kBlock) {
        const double b = a.b[i];
        a.x[i] = 0.0;
        reinterpret_cast<double2 *>(a.rp)[i] = make_double2(b, b);
        acc += b * b;
    }
    const double t = block_sum(acc, s_red);
    if (threadIdx.x == 0)
        a.part_out[blockIdx.x] = t;
}

// Tail of iteration k (single_strategy.hpp:140-148): alpha = rs_k / p.Ap (every block sums the
// SpMV's partials in the same order), r += (-alpha) Ap, r.r partial per block; x += alpha p is
// deferred to the next SpMV (cg1_lag_*), which takes alpha from scal[0].alpha.  A non-finite
// alpha stops the solve before r changes (the reference keeps going on NaN).
__global__ __launch_bounds__(kBlock) void k_cg1_update(Cg1Args a)
{
    __shared__ double s_red[kBlock / 64];
    const int tid = threadIdx.x;
    if (a.ctrl->done)
        return;
    PartRegs<kConsumeTile / kBlock> pin;
    part_load(a.part_in, a.n_part_in, pin);
    const long long stride = (long long)gridDim.x * kBlock;
    const long long i0 = (long long)blockIdx.x * kBlock + tid;
    double q = 0.0, r = 0.0;  // the first element's operands, in flight under the sum
    if (i0 < a.m) {
        q = a.ap[i0];
        r = a.rp[2 * i0];
    }
    const double pAp = part_sum(pin, s_red);
    const double alpha = a.scal[0].rs_par[a.parity] / pAp;
    if (!(alpha == alpha && fabs(alpha) < HUGE_VAL)) {
        if (blockIdx.x == 0 && tid == 0) {
            a.ctrl->breakdown = 1;
            a.ctrl->iters_out = a.ctrl->iter_par[a.parity] + 1;
            a.ctrl->done = 1;
        }
        return;
    }
    if (blockIdx.x == 0 && tid == 0)
        a.scal[0].alpha = alpha;  // x += alpha p_k: the next SpMV's rows, or k_cg1_xflush
    const double nal = -alpha;
    double acc = 0.0;
    for (long long i = i0; i < a.m; i += stride) {
        if (i != i0) {
            q = a.ap[i];
            r = a.rp[2 * i];
        }
        r = r + nal * q;
        a.rp_next[2 * i] = r;
        acc += r * r;
    }
    const double t = block_sum(acc, s_red);
    if (tid == 0)
        a.part_out[blockIdx.x] = t;
}

// After max_iters iterations: the last iteration's stop test and history entry (the SpMV that
// would take it is not launched); iterations = max_iters either way (single_strategy.hpp:152-170).
__global__ __launch_bounds__(kBlock) void k_cg1_finish(Cg1Args a)
{
    __shared__ double s_red[kBlock / 64];
    if (a.ctrl->done)
        return;
    PartRegs<kUpdateMaxBlocks / kBlock> pin;
    part_load(a.part_in, a.n_part_in, pin);
    const double rs = part_sum(pin, s_red);
    if (threadIdx.x == 0) {
        CgControl *c = a.ctrl;
        const int k = c->iter_par[a.parity];
        if (a.hist && k >= 1 && k - 1 < a.hist_cap)
            a.hist[k - 1] = sqrt(rs) / a.scal[0].b_norm;
        c->iter = k;
        c->iters_out = k;
        c->done = 1;
    }
}

// After the loop (converged, max_iters or breakdown): the last deferred x += alpha p.  The solve
// reported j + 1 = iters_out iterations; the update of iteration j ran (it stored alpha_j) and no
// SpMV after it applied its term (the stop test that ended the solve returns before that, and
// max_iters launches none).  p_j was written into the {r, p} buffer of parity (j + 1) & 1.  A
// breakdown (non-finite alpha_j) leaves nothing pending: the update stopped before storing alpha_j
// and iteration j's SpMV had applied alpha_{j-1} p_{j-1} already.
__global__ __launch_bounds__(kBlock) void k_cg1_xflush(Cg1Args a)
{
    const CgControl *c = a.ctrl;
    if (c->breakdown || c->iters_out < 1)
        return;
    const int j = c->iters_out - 1;
    const double *rp = ((j + 1) & 1) ? a.rp_next : a.rp;  // rp: d_p0, rp_next: d_p1
    const double alpha = a.scal[0].alpha;
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < a.m; i += (long long)gridDim.x * kBlock)
        a.x[i] = a.x[i] + alpha * rp[2 * i + 1];
}

int cg1_blocks(long long m)
{
    // one element per thread up to kUpdateMaxBlocks (512 / 256 update blocks measured no faster, r02u)
    const long long b = (m + kBlock - 1) / kBlock;
    return (int)std::max<long long>(1, std::min<long long>(b, kUpdateMaxBlocks));
}

static Cg1Args cg1_args(mspmv_handle_s *h, double *d_x)
{
    Cg1Args a{};
    a.m = h->m;
    a.x = d_x;
    a.rp = h->d_p0;  // {r, p} of parity 0; the iterations alternate d_p0 / d_p1 (2 m doubles each)
    a.ap = h->d_ap;
    a.scal = h->d_scal;
    a.ctrl = h->d_ctrl;
    a.hist = h->d_hist;
    a.hist_cap = h->hist_cap;
    return a;
}

hipError_t launch_cg1_init(mspmv_handle_s *h, const double *d_b, double *d_x, int nblk)
{
    Cg1Args a = cg1_args(h, d_x);
    a.b = d_b;
    a.part_out = h->d_partials_b;
    hipLaunchKernelGGL(k_cg1_init, dim3(nblk), dim3(kBlock), 0, h->stream, a);
    return hipGetLastError();
}

hipError_t launch_cg1_finish(mspmv_handle_s *h, double *d_x, int parity, int nblk)
{
    Cg1Args a = cg1_args(h, nullptr);
    a.part_in = h->d_partials_b;
    a.n_part_in = nblk;
    a.parity = parity;
    hipLaunchKernelGGL(k_cg1_finish, dim3(1), dim3(kBlock), 0, h->stream, a);
    if (hipGetLastError() != hipSuccess)
        return hipErrorLaunchFailure;
    a.x = d_x;
    a.rp = h->d_p0;
    a.rp_next = h->d_p1;
    hipLaunchKernelGGL(k_cg1_xflush, dim3(nblk), dim3(kBlock), 0, h->stream, a);
    return hipGetLastError();
}


// Multi-RHS iteration, split: p = r + beta p (one streaming pass), then Y = A p with p.Ap by
// linearity (MODE 2, which also stops on a non-finite alpha), then the update with alpha from
// that p.Ap.  For L >= 2 the fused iteration would gather two L-wide panel rows (r and
// p_old) per nonzero, and the SpMM is gather-bound: measured 1.33 ms vs 0.62 + 0.14 ms split
// on the nlpkkt120-sized L = 8 case.
static hipError_t pcg_dot(const CgVecArgs &va, int L, int nblk, int mode, hipStream_t s);

// Split CG: p.Ap from the SpMM's dot mode (x.(Ax) partials per tile) or from a separate pass over
// p and Ap after the plain SpMM (MSPMV_CG_DOT=pass / fused; default: the pass).
static bool cg_dot_pass(int L)
{
    static const int mode = [] {
        const char *e = getenv("MSPMV_CG_DOT");
        return e && std::string(e) == "fused" ? 0 : 1;
    }();
    return mode != 0 && L >= 1;
}

// The block CG's SpMM on the offset windows takes p.Ap in its dot mode (MSPMV_DIA_DOT=0: the plain window
// SpMM and the separate pass, as the tiles do).
bool dia_dot_fused()
{
    const char *e = getenv("MSPMV_DIA_DOT");
    return !(e && *e && atoi(e) == 0);
}

// splan: the plan the solve chose for the plain L-wide product (cg_solve_native: the offset-window or
// column-slab plan, else null -> the tiles of `plan`); dot_fused: the window SpMM takes p.Ap in its dot
// mode (resolved once per solve, and part of the CG graph's key).
// The p update stays its own pass: fused into the window SpMM (the spans staged as r + beta p_old, the
// window's own rows written to a second p buffer) it measured 0.773-0.779 against 0.657-0.658 ms per
// configs[4] iteration (r06c): the SpMM then loads r's spans beside p's -- nine times per row through L2
// -- which costs the issue-bound kernel more than the pass it replaces.
static hipError_t launch_cg_iteration_split(mspmv_handle_s *h, const TilePlan &plan, const TilePlan *splan,
                                            bool dot_fused, double *d_x, int L, int nblk, double tol)
{
    CgVecArgs va{};
    va.n_elems = (long long)h->m * L;
    va.x = d_x;
    va.r = h->d_r;
    va.p = h->d_p0;
    va.ap = h->d_ap;
    va.scal = h->d_scal;
    va.ctrl = h->d_ctrl;
    va.conv = h->d_conv;
    va.partials = h->d_partials;
    va.gtickets = h->d_gtickets;
    va.hist = h->d_hist;
    va.hist_cap = h->hist_cap;
    va.tol = tol;
    va.lazy_x = 1;
    static const int rev = [] {  // measured knob: alternate sweep directions (CgVecArgs::rev)
        const char *e = getenv("MSPMV_CG_REV");
        return e ? atoi(e) : 1;
    }();
    va.rev = rev;  // the p update (after the forward update) sweeps backwards
    hipError_t e = launch_dist_vec(2, va, L, nblk, h->d_p0, h->stream);
    va.rev = 0;
    if (e != hipSuccess)
        return e;
    const TilePlan *dp = splan && splan->dia ? splan : nullptr;
    const TilePlan *sp = splan && splan->slab ? splan : nullptr;
    if (dp && dot_fused) {
        // offset windows (mspmv_dia.hip) in dot mode: Ap and one p.Ap partial per window, folded with the
        // non-finite-alpha stop -- no separate pass over p and Ap
        if ((e = launch_dia(h, *dp, h->d_p0, h->d_ap, L, L, h->d_ctrl, h->d_partials)) != hipSuccess)
            return e;
        if ((e = launch_fold_dot(dp->num_tiles, L, h->d_partials, h->d_gtickets, h->d_red, h->d_scal, h->d_conv,
                                 h->d_ctrl, -1, h->stream)) != hipSuccess)
            return e;
    } else if (cg_dot_pass(L)) {
        // the plain SpMM (its tile kernel holds fewer registers than the dot mode's, so more
        // workgroups per CU, and never spills), stopped by the control word, then p.Ap in one
        // streaming pass over p and Ap with the fold's breakdown checks (k_pcg_dot mode 2)
        // (on the offset-window or column-slab plan when the handle's plain L-wide product took one)
        if (dp) {
            if ((e = launch_dia(h, *dp, h->d_p0, h->d_ap, L, L, h->d_ctrl)) != hipSuccess)
                return e;
        } else if (sp) {
            if ((e = launch_slab_mm(h, *sp, h->d_p0, h->d_ap, L, L, h->d_ctrl)) != hipSuccess)
                return e;
        } else {
            TileArgs ta = make_args(h, plan, h->d_p0, h->d_ap, L);
            ta.ctrl = h->d_ctrl;
            ta.fault = &h->d_ctrl->fault;
            if ((e = launch_tile<kModeSpmv>(ta, L, h->stream, stream_nt(h))) != hipSuccess)
                return e;
        }
        CgVecArgs vd = va;
        vd.r = h->d_p0;
        vd.p = h->d_ap;
        vd.red_out = h->d_red;
        vd.rev = rev;  // ... the p.Ap pass backwards, so the update finds Ap's first lines cached
        if ((e = pcg_dot(vd, L, nblk, 2, h->stream)) != hipSuccess)
            return e;
    } else if ((e = launch_spmm_dot(h, plan, h->d_p0, h->d_ap, L, h->d_ctrl, h->d_partials, h->d_gtickets, h->d_red,
                                    h->d_scal, h->d_conv)) != hipSuccess) {
        return e;
    }
    va.red_in = h->d_red;
    return dispatch_vec(false, va, L, nblk, h->stream);
}

// After the split iteration's loop: the x += alpha p still pending (CgVecArgs::lazy_x).
hipError_t launch_cg_xflush(mspmv_handle_s *h, double *d_x, int L, int nblk)
{
    CgVecArgs va{};
    va.n_elems = (long long)h->m * L;
    va.x = d_x;
    va.scal = h->d_scal;
    va.ctrl = h->d_ctrl;
    switch (L) {
    case 1: hipLaunchKernelGGL((k_cg_xflush<1>), dim3(nblk), dim3(kBlock), 0, h->stream, va, h->d_p0); break;
    case 2: hipLaunchKernelGGL((k_cg_xflush<2>), dim3(nblk), dim3(kBlock), 0, h->stream, va, h->d_p0); break;
    case 4: hipLaunchKernelGGL((k_cg_xflush<4>), dim3(nblk), dim3(kBlock), 0, h->stream, va, h->d_p0); break;
    case 8: hipLaunchKernelGGL((k_cg_xflush<8>), dim3(nblk), dim3(kBlock), 0, h->stream, va, h->d_p0); break;
    case 16: hipLaunchKernelGGL((k_cg_xflush<16>), dim3(nblk), dim3(kBlock), 0, h->stream, va, h->d_p0); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Multi-RHS CG always runs the split iteration; single-RHS the pipelined one unless
// MSPMV_CG_SPLIT=1 asks for the split form (A/B runs, and its own parity test).
bool cg_split_iteration(int L)
{
    static const int mode = [] {
        const char *e = getenv("MSPMV_CG_SPLIT");
        return e ? atoi(e) : 0;
    }();
    return L >= 2 || mode != 0;
}

hipError_t launch_cg_iteration(mspmv_handle_s *h, const TilePlan &plan, const TilePlan *splan, bool dot_fused,
                               double *d_x, int L, int parity, int nblk, double tol)
{
    if (cg_split_iteration(L))
        return launch_cg_iteration_split(h, plan, splan, dot_fused, d_x, L, nblk, tol);
    double *rp_old = parity ? h->d_p1 : h->d_p0;  // {r_k, p_{k-1}} interleaved (cg_rp)
    double *rp_new = parity ? h->d_p0 : h->d_p1;  // receives p_k, then r_{k+1}
    int nslots = plan.num_tiles;                   // the SpMV's p.Ap partials
    hipError_t e = hipSuccess;
    if (splan && splan->dia) {  // the SpMV on the offset windows (mspmv_dia.hip, k_cg1_dia)
        e = launch_cg1_dia(h, *splan, rp_old, rp_new, d_x, parity, nblk, tol, &nslots);
    } else {
        TileArgs ta = make_args(h, plan, rp_old, h->d_ap, 1);
        ta.p_new = rp_new;
        ta.xsol = d_x;
        ta.scal = h->d_scal;
        ta.ctrl = h->d_ctrl;
        ta.fault = &h->d_ctrl->fault;
        ta.partials = h->d_partials;
        ta.gtickets = h->d_gtickets;
        ta.part_in = h->d_partials_b;
        ta.n_part_in = nblk;
        ta.parity = parity;
        ta.tol = tol;
        ta.hist = h->d_hist;
        ta.hist_cap = h->hist_cap;
        e = launch_tile<kModeCg>(ta, 1, h->stream, stream_nt(h));
    }
    if (e != hipSuccess)
        return e;
    Cg1Args a = cg1_args(h, d_x);
    a.rp = rp_old;
    a.rp_next = rp_new;
    long long off = 0;
    int count = 0;
    consumer_level(nslots, kConsumeTile, 1, &off, &count);
    a.part_in = h->d_partials + off;
    a.n_part_in = count;
    a.part_out = h->d_partials_b;
    a.parity = parity;
    hipLaunchKernelGGL(k_cg1_update, dim3(nblk), dim3(kBlock), 0, h->stream, a);
    return hipGetLastError();
}

// ---- row-sharded CG launchers --------------------------------------------------------------
template <int L>
static hipError_t dist_launch_L(int which, const CgVecArgs &a, int nblk, double *p, hipStream_t s)
{
    switch (which) {
    case 0: hipLaunchKernelGGL((k_cg_init<L>), dim3(nblk), dim3(kBlock), 0, s, a); break;
    case 1: hipLaunchKernelGGL((k_dist_init_finish<L>), dim3(1), dim3(64), 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_dist_pupdate<L>), dim3(nblk), dim3(kBlock), 0, s, a, p); break;
    case 3: hipLaunchKernelGGL((k_cg_update<L>), dim3(nblk), dim3(kBlock), 0, s, a); break;
    case 4: hipLaunchKernelGGL((k_dist_finish<L>), dim3(1), dim3(64), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_dist_vec(int which, const CgVecArgs &a, int L, int nblk, double *p, hipStream_t s)
{
    switch (L) {
    case 1: return dist_launch_L<1>(which, a, nblk, p, s);
    case 2: return dist_launch_L<2>(which, a, nblk, p, s);
    case 4: return dist_launch_L<4>(which, a, nblk, p, s);
    case 8: return dist_launch_L<8>(which, a, nblk, p, s);
    case 16: return dist_launch_L<16>(which, a, nblk, p, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_dist_pack(const double *p, const int *idx, long long n_elems, int L, double *send,
                            const CgControl *ctrl, hipStream_t s)
{
    if (n_elems <= 0)
        return hipSuccess;
    const long long nb = std::min<long long>((n_elems + 255) / 256, 4096);
    hipLaunchKernelGGL(k_dist_pack, dim3((unsigned)nb), dim3(256), 0, s, p, idx, n_elems, L, send, ctrl);
    return hipGetLastError();
}

// Y = A X with x.(AX) per column reduced into dot_out (MODE 2), plus the partials fold.  scal / conv (single-GPU split CG) add the non-finite-alpha stop.
// The dot-mode SpMM's tile kernel on stream s: Y = A X and one x.(AX) partial per tile
// at partials[t * L ..] (plain stores, summed by launch_fold_dot in a later launch).
hipError_t launch_spmm_dot_tiles(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                                 CgControl *ctrl, double *partials, hipStream_t s, long long row_off)
{
    if (plan.num_tiles == 0)
        return hipSuccess;
    TileArgs ta = make_args(h, plan, d_X, d_Y, L);
    ta.xr = d_X + row_off * L;  // the handle's rows start at row row_off of X
    ta.ctrl = ctrl;
    ta.fault = ctrl ? &ctrl->fault : h->d_fault;
    ta.partials = partials;
    return launch_tile<kModeDot>(ta, L, s, stream_nt(h));
}

// Sum T tiles' partials [T][L] in tile order into dot_out (k_fold_dot; partials_capacity() leaves
// room for the fold's levels after the T * L partials).
hipError_t launch_fold_dot(int T, int L, double *partials, unsigned *gtickets, double *dot_out, CgScalars *scal,
                           const unsigned char *conv, CgControl *ctrl, int fold_mode, hipStream_t s)
{
    const int mode = fold_mode >= 0 ? fold_mode : scal ? kFoldCgAlpha : kFoldDot;
    if (T == 0)  // no rows: contributes 0 (a rank's share of the all-reduce)
        return hipMemsetAsync(dot_out, 0, sizeof(double) * L, s);
    const int G = std::max(1, std::min(256, (T + 63) / 64));  // >= 64 tiles per fold block
    const int q = (T + G - 1) / G;
    double *lvl = partials + (size_t)T * L;
    switch (L) {
#define MSPMV_FOLD(LL)                                                                             \
    case LL:                                                                                       \
        hipLaunchKernelGGL((k_fold_dot<LL>), dim3(G), dim3(kBlock), 0, s, partials, T, q, lvl, gtickets, dot_out, \
                           scal, conv, ctrl, mode);                                                \
        break;
        MSPMV_FOLD(1)
        MSPMV_FOLD(2)
        MSPMV_FOLD(4)
        MSPMV_FOLD(8)
        MSPMV_FOLD(16)
#undef MSPMV_FOLD
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_spmm_dot(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                           CgControl *ctrl, double *partials, unsigned *gtickets, double *dot_out,
                           CgScalars *scal, const unsigned char *conv, int fold_mode)
{
    hipError_t e = launch_spmm_dot_tiles(h, plan, d_X, d_Y, L, ctrl, partials, h->stream, 0);
    if (e != hipSuccess)
        return e;
    return launch_fold_dot(plan.num_tiles, L, partials, gtickets, dot_out, scal, conv, ctrl, fold_mode, h->stream);
}

// Cold-cache flush between timed launches: a read sweep (caches left holding clean unrelated lines;
// a write sweep left them dirty and the timed kernel paid the write-back: cant 35.1 vs 19.2 us, r02n).
hipError_t launch_flush(void *p, size_t bytes, hipStream_t s, bool fresh)
{
    const long long n = (long long)(bytes / sizeof(double));
    if (fresh)
        hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, s, (double *)p, n, 1.0);
    else
        hipLaunchKernelGGL(k_flush_read, dim3(2048), dim3(256), 0, s, (const double *)p, n, (double *)p);
    return hipGetLastError();
}

}  // namespace mspmv

namespace mspmv {
hipError_t launch_dist_vec(int which, const CgVecArgs &a, int L, int nblk, double *p, hipStream_t s);


hipError_t launch_dist_vec_mirror(int which, const DistVecArgs &d, int L, int nblk, double *p, hipStream_t s)
{
    static_assert(sizeof(DistVecArgs) == sizeof(CgVecArgs), "DistVecArgs must mirror CgVecArgs");
    CgVecArgs a{};
    a.n_elems = d.n_elems;
    a.x = d.x;
    a.r = d.r;
    a.p = d.p;
    a.p0 = d.p0;
    a.ap = d.ap;
    a.scal = d.scal;
    a.ctrl = d.ctrl;
    a.conv = d.conv;
    a.partials = d.partials;
    a.hist = d.hist;
    a.hist_cap = d.hist_cap;
    a.tol = d.tol;
    a.red_in = d.red_in;
    a.red_out = d.red_out;
    a.gtickets = d.gtickets;
    a.pcg = d.pcg;
    return launch_dist_vec(which, a, L, nblk, p, s);
}

// ---- SPAI-preconditioned block CG (SPAISolveMultiple) ------------------------------------------
static CgVecArgs pcg_vec_args(mspmv_handle_s *h, double *d_x, int L, double tol)
{
    CgVecArgs va{};
    va.n_elems = (long long)h->m * L;
    va.x = d_x;
    va.r = h->d_r;
    va.p = h->d_p0;
    va.p0 = h->d_p0;
    va.ap = h->d_ap;
    va.scal = h->d_scal;
    va.ctrl = h->d_ctrl;
    va.conv = h->d_conv;
    va.partials = h->d_partials;
    va.gtickets = h->d_gtickets;
    va.hist = h->d_hist;
    va.hist_cap = h->hist_cap;
    va.tol = tol;
    va.pcg = 1;
    return va;
}

// X = 0, R = B, b_norms (sparse_approximate_inverse.hpp:59-78); Z = M R and rs_old = R.Z
// (:80-92, :99-100); P = Z (:94-97).  Z lives in h->d_p1, P in h->d_p0.
hipError_t launch_pcg_init(mspmv_handle_s *h, mspmv_handle_s *hm, const TilePlan &mplan, const double *d_b,
                           double *d_x, int L, double tol, int nblk)
{
    hipError_t e = launch_cg_init(h, d_b, d_x, L, tol, nblk);
    if (e != hipSuccess)
        return e;
    hipStream_t own = hm->stream;
    hm->stream = h->stream;
    e = launch_spmm_dot(hm, mplan, h->d_r, h->d_p1, L, h->d_ctrl, h->d_partials, h->d_gtickets, h->d_red,
                        h->d_scal, h->d_conv, kFoldPcgInit);
    hm->stream = own;
    if (e != hipSuccess)
        return e;
    return hipMemcpyAsync(h->d_p0, h->d_p1, sizeof(double) * (size_t)h->m * L, hipMemcpyDeviceToDevice, h->stream);
}

// One PCG iteration, four launches plus two folds: AP = A P with P.AP -> alpha (:111-138);
// X += alpha P, R -= alpha AP, R.R -> masks, max-residual history, stop (:140-181);
// Z = M R with R.Z -> beta, rs_old (:183-210); P = Z + beta P (:212-214).
hipError_t launch_pcg_iteration(mspmv_handle_s *h, mspmv_handle_s *hm, const TilePlan &plan, const TilePlan &mplan,
                                double *d_x, int L, int nblk, double tol)
{
    CgVecArgs va = pcg_vec_args(h, d_x, L, tol);
    hipError_t e = launch_spmm_dot(h, plan, h->d_p0, h->d_ap, L, h->d_ctrl, h->d_partials, h->d_gtickets, h->d_red,
                                   h->d_scal, h->d_conv, kFoldPcgAlpha);
    if (e != hipSuccess)
        return e;
    if ((e = dispatch_vec(false, va, L, nblk, h->stream)) != hipSuccess)
        return e;
    hipStream_t own = hm->stream;
    hm->stream = h->stream;
    e = launch_spmm_dot(hm, mplan, h->d_r, h->d_p1, L, h->d_ctrl, h->d_partials, h->d_gtickets, h->d_red,
                        h->d_scal, h->d_conv, kFoldPcgBeta);
    hm->stream = own;
    if (e != hipSuccess)
        return e;
    va.r = h->d_p1;  // P = Z + beta P
    return launch_dist_vec(2, va, L, nblk, h->d_p0, h->stream);
}
// ---- IC(0)-preconditioned block CG (PCGSolveMultiple) -------------------------------------------
template <int L>
static void trsv_L(const mspmv_ic0_s *ic, bool fwd, const double *b, double *x, CgControl *ctrl, hipStream_t s)
{
    const dim3 grid((ic->n + kBlock / 64 - 1) / (kBlock / 64)), block(kBlock);
    if (fwd)
        hipLaunchKernelGGL((k_trsv_tagged<L, true>), grid, block, 0, s, ic->d_lro, ic->d_lci, ic->d_lva, ic->n,
                           ic->d_fwd_order, b, x, ctrl);
    else
        hipLaunchKernelGGL((k_trsv_tagged<L, false>), grid, block, 0, s, ic->d_uro, ic->d_uci, ic->d_uva, ic->n,
                           ic->d_bwd_order, b, x, ctrl);
}

// Z = L^-T (L^-1 R): ForwardSolveMultiple into ic->d_y, then BackwardSolveMultiple
// (incomplete_cholesky.hpp:89-92, :166-167); the ready flags are cleared before each solve.
static hipError_t ic0_apply(mspmv_handle_s *h, mspmv_ic0_s *ic, int L, const double *r, double *z)
{
    if (ic->n == 0)
        return hipSuccess;
    for (int pass = 0; pass < 2; ++pass) {
        const bool fwd = pass == 0;
        const double *in = fwd ? r : ic->d_y;
        double *out = fwd ? ic->d_y : z;
        hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(out), kTrsvPendingWord,
                                         2 * (size_t)ic->n * L, h->stream);
        if (e != hipSuccess)
            return e;
        switch (L) {
        case 1: trsv_L<1>(ic, fwd, in, out, h->d_ctrl, h->stream); break;
        case 2: trsv_L<2>(ic, fwd, in, out, h->d_ctrl, h->stream); break;
        case 4: trsv_L<4>(ic, fwd, in, out, h->d_ctrl, h->stream); break;
        case 8: trsv_L<8>(ic, fwd, in, out, h->d_ctrl, h->stream); break;
        case 16: trsv_L<16>(ic, fwd, in, out, h->d_ctrl, h->stream); break;
        default: return hipErrorInvalidValue;
        }
        if ((e = hipGetLastError()) != hipSuccess)
            return e;
    }
    return hipSuccess;
}

static hipError_t pcg_dot(const CgVecArgs &va, int L, int nblk, int mode, hipStream_t s)
{
    switch (L) {
    case 1: hipLaunchKernelGGL((k_pcg_dot<1>), dim3(nblk), dim3(kBlock), 0, s, va, mode); break;
    case 2: hipLaunchKernelGGL((k_pcg_dot<2>), dim3(nblk), dim3(kBlock), 0, s, va, mode); break;
    case 4: hipLaunchKernelGGL((k_pcg_dot<4>), dim3(nblk), dim3(kBlock), 0, s, va, mode); break;
    case 8: hipLaunchKernelGGL((k_pcg_dot<8>), dim3(nblk), dim3(kBlock), 0, s, va, mode); break;
    case 16: hipLaunchKernelGGL((k_pcg_dot<16>), dim3(nblk), dim3(kBlock), 0, s, va, mode); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// X = 0, R = B, b_norms (incomplete_cholesky.hpp:66-85); Z = M^-1 R (:87-92); P = Z (:94-95);
// rs_old = R.Z (:97).  Z lives in h->d_p1, P in h->d_p0.
hipError_t launch_pcg_ic0_init(mspmv_handle_s *h, mspmv_ic0_s *ic, const double *d_b, double *d_x, int L, double tol,
                               int nblk)
{
    hipError_t e = launch_cg_init(h, d_b, d_x, L, tol, nblk);
    if (e == hipSuccess)
        e = ic0_apply(h, ic, L, h->d_r, h->d_p1);
    CgVecArgs va = pcg_vec_args(h, d_x, L, tol);
    va.p = h->d_p1;
    if (e == hipSuccess)
        e = pcg_dot(va, L, nblk, 0, h->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(h->d_p0, h->d_p1, sizeof(double) * (size_t)h->m * L, hipMemcpyDeviceToDevice, h->stream);
    return e;
}

// One iteration (:104-191): AP = A P with P.AP (fold: alpha = rs_old / P.AP, non-finite stops);
// X += alpha P, R -= alpha AP, R.R -> masks, history, stop; Z = M^-1 R; R.Z -> beta, rs_old;
// P = Z + beta P.
hipError_t launch_pcg_ic0_iteration(mspmv_handle_s *h, mspmv_ic0_s *ic, const TilePlan &plan, double *d_x, int L,
                                    int nblk, double tol)
{
    hipError_t e = launch_spmm_dot(h, plan, h->d_p0, h->d_ap, L, h->d_ctrl, h->d_partials, h->d_gtickets, h->d_red,
                                   h->d_scal, h->d_conv, kFoldCgAlpha);
    CgVecArgs va = pcg_vec_args(h, d_x, L, tol);
    va.red_in = h->d_red;  // alpha_j = converged ? 0 : rs_old_j / P.AP_j, in every block
    if (e == hipSuccess)
        e = dispatch_vec(false, va, L, nblk, h->stream);
    if (e == hipSuccess)
        e = ic0_apply(h, ic, L, h->d_r, h->d_p1);
    CgVecArgs vd = va;
    vd.p = h->d_p1;
    if (e == hipSuccess)
        e = pcg_dot(vd, L, nblk, 1, h->stream);
    va.r = h->d_p1;  // P = Z + beta P
    if (e == hipSuccess)
        e = launch_dist_vec(2, va, L, nblk, h->d_p0, h->stream);
    return e;
}

}  // namespace mspmv
