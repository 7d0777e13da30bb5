// Column-slab form of the plain single-RHS SpMV (y = A x) for matrices whose x gathers are
// line-bound: every nonzero of a tile gathers x from its own cache line (scattered columns inside a
// wide band), which the tile kernels serve one L2 line per nonzero.  Here the work is cut into a few
// large blocks (two resident per CU, merge-path balanced like the tiles: cpu_spmv.cpp:208-235), and
// each block's nonzeros are reordered at plan time by column slab -- kSlabCols columns of x, 32 KB --
// so the block stages each slab of x it touches into LDS once, with coalesced loads, and gathers
// from LDS.  A scattered band of +-10,000 columns then reads ~3 slabs of x per block instead of one L2
// line per nonzero.
//
// Per block: rows ending in the block accumulate in LDS (yacc); the reordered stream is cut into
// chunks of <= kSlabChunk nonzeros of one slab, each chunk's runs of one row listed as entries
// {offset, length, row}.  Per chunk: the products val * x[col] go to LDS (the chunk's stream and
// entries were loaded into registers two chunks earlier, its slab of x during the previous chunk), then groups of 2^lg lanes take the
// entries round-robin, lane j summing products j, j + 2^lg, ... of its run in order, a fixed xor
// butterfly folds the group and its lane 0 adds the run to yacc[row] -- a row has one run per chunk,
// and chunks run in order, so every sum is fixed-order (reproducible) and within the 2 (len+1) eps
// (|A||x|)_i reordering bound of the CSR-order sum (mspmv_tile_modes reports the blocks as 255).
// Rows split between blocks (longer than the snap distance) are closed as the tile kernels close
// them (close_split_rows, mspmv_device.h).
#include "mspmv_internal.h"
#include "mspmv_device.h"

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

namespace mspmv {

struct SlabArgs {
    const int4 *blk;            // SlabData::d_blk
    const int4 *chunk;          // SlabData::d_chunk (+ sentinel)
    const uint2 *ent;           // SlabData::d_ent
    const double *val;          // SlabData::d_val
    const unsigned short *col;  // SlabData::d_col
    const double *x;
    double *y;
    int n;
    int num_tiles;              // blocks
    int groups;                 // column groups (1: every block holds whole rows' nonzeros)
    int m;
    double *part;               // [groups][m] partial row sums (groups > 1)
    unsigned *gcnt;             // [row blocks] fold tickets
    const int4 *slice;          // sliced-ELL (k_spmv_sell): SlabData::d_slice, d_sent, d_long
    const unsigned short *sent;
    const int4 *lng;
    // split rows (close_split_rows reads these names)
    const int2 *bounds;
    const unsigned char *split;
    const int4 *fix;
    unsigned *fix_cnt;
    double *carry_val;
    double *head_val;
    double *head_pub;
    unsigned *fault;            // the handle's fault word (ticket_arrive)
};

template <bool NT, typename T>
__device__ __forceinline__ T slab_stream(const T *p)
{
    if (NT)
        return __builtin_nontemporal_load(p);
    return *p;
}

// A column group's partial row sums (agent scope), then, by the row block's last group to finish (a
// ticket per row block, reset by it), y = the groups' partials added in group order (fixed order).
template <int TB>
__device__ __forceinline__ void group_out(const SlabArgs &a, int b, int r0, int nrows, const double *yacc)
{
    const int tid = threadIdx.x;
    const int G = a.groups, g = b % G, rb = b / G;
    for (int i = tid; i < nrows; i += TB)
        store_sc1(&a.part[(size_t)g * a.m + r0 + i], yacc[i]);
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this group's partials are out
    __syncthreads();
    if (tid == 0)
        s_last = ticket_arrive<false>(&a.gcnt[rb], (unsigned)(G - 1), a.fault);
    __syncthreads();
    if (!s_last)
        return;
    // (agent-scope loads, all issued before the sum; __threadfence() pairs instead cost 100+ us, r05ao)
    for (int i = tid; i < nrows; i += TB) {
        double pv[kSlabMaxGroups];
#pragma unroll
        for (int q = 0; q < kSlabMaxGroups; ++q)
            pv[q] = q < G && q != g ? load_sc1(&a.part[(size_t)q * a.m + r0 + i]) : 0.0;
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < kSlabMaxGroups; ++q)
            if (q < G)
                s += q == g ? yacc[i] : pv[q];
        a.y[r0 + i] = s;
    }
    if (tid == 0)
        __hip_atomic_store(&a.gcnt[rb], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool NT, int CFG>
__global__ __launch_bounds__(kSlabCfgs[CFG].threads) void k_spmv_slab(SlabArgs a)
{
    constexpr SlabCfg C = kSlabCfgs[CFG];
    constexpr int TB = C.threads;
    constexpr int IPT = C.chunk / TB;    // stream items per thread and chunk
    constexpr int EPT = C.entries / TB;  // entries per thread and chunk
    __shared__ double xs[C.cols];
    __shared__ double yacc[C.rows + 1];
    __shared__ double prod[C.chunk];
    __shared__ uint2 sent[C.entries];
    __shared__ int4 schunk[kSlabMaxChunks + 1];
    const int tid = threadIdx.x;
    const int b = xcd_tile(blockIdx.x, a.num_tiles);
    const int4 bd = a.blk[b];  // {first row, rows ending here, chunk0, chunk1}
    // the block's chunk descriptors (and the next one's entry start) in LDS: a scalar load per chunk
    // would put its round trip at the head of every chunk
    for (int i = tid; i <= bd.w - bd.z; i += TB)
        schunk[i] = a.chunk[bd.z + i];
    __syncthreads();
    auto chunk = [&](int ci) {  // block-uniform
        const int4 c = schunk[ci - bd.z];
        return make_int4(__builtin_amdgcn_readfirstlane(c.x), __builtin_amdgcn_readfirstlane(c.y),
                         __builtin_amdgcn_readfirstlane(c.z), __builtin_amdgcn_readfirstlane(c.w));
    };
    const int4 fx = load_fix(a, b);
    const int nrows = bd.y;
    const bool tail = a.split[b + 1] != 0;
    for (int i = tid; i < nrows + (tail ? 1 : 0); i += TB)
        yacc[i] = 0.0;

    struct Regs {  // one chunk's stream and entries, in registers
        double v[IPT];
        unsigned short c[IPT];
        uint2 e[EPT];
    };
    auto fetch = [&](int ci, Regs &r) {
        const int4 cd = chunk(ci);
        const int len = cd.y & 0x1fff;
        const int e0 = cd.w, ne = chunk(ci + 1).w - e0;
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int k = min(tid + j * TB, len - 1);  // clamped: every load is issued
            r.v[j] = slab_stream<NT>(a.val + cd.x + k);
            r.c[j] = slab_stream<NT>(a.col + cd.x + k);
        }
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int k = tid + j * TB;
            r.e[j] = k < ne ? a.ent[e0 + k] : make_uint2(0u, 0u);
        }
    };
    constexpr int XPT = C.cols / TB;  // x values per thread and slab
    double xq[XPT];
    auto fetch_x = [&](int slab) {  // a slab of x, into registers (coalesced: lane-consecutive columns)
        const int c0 = slab * C.cols;
#pragma unroll
        for (int j = 0; j < XPT; ++j) {
            const int col = c0 + tid + j * TB;
            xq[j] = col < a.n ? a.x[col] : 0.0;
        }
    };
    int cur = -1;
    // One chunk: its slab (fetched during the previous chunk) into LDS when it changes, the products
    // and entries from registers into LDS, the registers refilled two chunks ahead (chunk ci + 2:
    // the stream's latency hides behind two chunks' sums, not one), the next slab fetched when the
    // next chunk changes it, then the runs summed into yacc.
    auto process = [&](int ci, Regs &r) {
        const int4 cd = chunk(ci);
        const int len = cd.y & 0x1fff, lg = (cd.y >> 13) & 7, nlong = cd.y >> 16;
        const int ne = chunk(ci + 1).w - cd.w;
        if (cd.z != cur) {  // block-uniform
            cur = cd.z;
            __syncthreads();  // the previous chunk's readers of xs are done
#pragma unroll
            for (int j = 0; j < XPT; ++j)
                xs[tid + j * TB] = xq[j];
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const int k = tid + j * TB;
            if (k < len)
                prod[k] = r.v[j] * xs[r.c[j]];
        }
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int k = tid + j * TB;
            if (k < ne)
                sent[k] = r.e[j];
        }
        if (ci + 2 < bd.w)
            fetch(ci + 2, r);
        if (ci + 1 < bd.w) {
            const int ns = chunk(ci + 1).z;
            if (ns != cur)
                fetch_x(ns);
        }
        __syncthreads();
        // long runs (listed first) by whole waves: a run thousands long (a power-law hub row) must not
        // sit on a few lanes of a group sized for the chunk's short runs
        for (int q = tid >> 6; q < nlong; q += TB >> 6) {  // wave-uniform
            const uint2 en = sent[q];
            const int off = (int)(en.x & 0xffffu), el = (int)(en.x >> 16);
            double s = 0.0;
            for (int k = off + (tid & 63); k < off + el; k += 64)
                s += prod[k];
            for (int o = 32; o > 0; o >>= 1)
                s += __shfl_xor(s, o);
            if ((tid & 63) == 0)
                yacc[en.y] += s;
        }
        const int G = 1 << lg, lane = tid & (G - 1);
        for (int q = nlong + (tid >> lg); q < ne; q += TB >> lg) {  // uniform within a group
            const uint2 en = sent[q];
            const int off = (int)(en.x & 0xffffu), el = (int)(en.x >> 16);
            double s = 0.0;
            for (int k = off + lane; k < off + el; k += G)
                s += prod[k];
            for (int o = G >> 1; o > 0; o >>= 1)
                s += __shfl_xor(s, o);
            if (lane == 0)
                yacc[en.y] += s;
        }
        __syncthreads();
    };
    Regs ra, rb;
    if (bd.z < bd.w) {
        fetch(bd.z, ra);
        fetch_x(chunk(bd.z).z);
        if (bd.z + 1 < bd.w)
            fetch(bd.z + 1, rb);
    }
    for (int ci = bd.z; ci < bd.w; ci += 2) {
        process(ci, ra);
        if (ci + 1 < bd.w)
            process(ci + 1, rb);
    }
    if (a.groups > 1) {  // block-uniform
        group_out<TB>(a, b, bd.x, nrows, yacc);
        return;
    }
    // rows ending in the block; its first row goes to the head slot when it completes a split row
    for (int i = tid; i < nrows; i += TB)
        *(i == 0 && fx.z > 0 ? a.head_val + b : a.y + bd.x + i) = yacc[i];
    if (tail && tid == 0)
        store_sc1(&a.carry_val[b], yacc[nrows]);
    close_split_rows<TB>(a, b, fx, 1, 1);
}

// Sliced-ELL form of the column-group blocks (kSlabCfgs[2]): per (block, slab) segment, the slab of x is
// staged in LDS once (the next segment's slab prefetched in registers meanwhile), then each wave takes
// slices of 64 runs -- lane = run, the run's values column-major in the slice, so every load of the
// stream is coalesced and no product passes through LDS; the next slice's values and the one after's
// header and runs are loaded while this one computes -- continuing its row's sum from yacc in the run's CSR order (a row's
// runs follow slab order: within a group the row sum is the CSR-order sum when its columns ascend).
// Runs longer than kSellLongRun come in pieces of <= 512 values, one wave each (8 loads per lane, xor
// butterfly) into lpart; after a barrier each run's pieces are added to its row in piece order.
#ifdef MSPMV_SELL_LAB_STAMPS
constexpr int kSellLabStampsEnd = 19;
// Lab build only (tools/lab/sell_stamps.sh): thread 0 of each block records wall_clock64() at entry, per segment
// (<= 6) after the x stage, after its wave's long pieces and after its wave's slices, and at exit.
constexpr int kSellLabStamps = 20, kSellLabBlocks = 1024;
__device__ unsigned long long g_sell_lab_stamps[kSellLabBlocks * kSellLabStamps];
#define SELL_STAMP(b, i)                                                                              \
    do {                                                                                              \
        if (threadIdx.x == 0 && (b) < kSellLabBlocks && (i) < kSellLabStamps)                         \
            g_sell_lab_stamps[(size_t)(b) * kSellLabStamps + (i)] = wall_clock64();                   \
    } while (0)
#else
#define SELL_STAMP(b, i) \
    do {                 \
    } while (0)
#endif

template <bool NT, bool PACK>
__global__ __launch_bounds__(kSlabCfgs[2].threads) void k_spmv_sell(SlabArgs a)
{
    constexpr SlabCfg C = kSlabCfgs[2];
    constexpr int TB = C.threads, NW = TB / 64, XPT = C.cols / TB;
    __shared__ double xs[C.cols];
    __shared__ double yacc[C.rows + 1];
    __shared__ double lpart[kSellMaxPieces];
    __shared__ int4 sseg[kSellMaxSegs + 1];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = xcd_tile(blockIdx.x, a.num_tiles);
    SELL_STAMP(b, 0);
    const int4 bd = a.blk[b];  // {first row, rows, segment0, segment1}
    const int nrows = bd.y;
    // the block's segment descriptors (and the next one's piece start) in LDS: a scalar load at each
    // segment's head put its round trip in every segment (~2 us each, r05ao)
    if (tid <= bd.w - bd.z)
        sseg[tid] = a.chunk[bd.z + tid];
    for (int i = tid; i < nrows; i += TB)
        yacc[i] = 0.0;
    __syncthreads();
    auto segd = [&](int sg) {  // block-uniform
        const int4 c = sseg[sg - bd.z];
        return make_int4(__builtin_amdgcn_readfirstlane(c.x), __builtin_amdgcn_readfirstlane(c.y),
                         __builtin_amdgcn_readfirstlane(c.z), __builtin_amdgcn_readfirstlane(c.w));
    };
    double xq[XPT];
    auto fetch_x = [&](int c0) {  // the segment's slab of x: C.cols columns from its first column c0
#pragma unroll
        for (int j = 0; j < XPT; ++j) {
            const int col = c0 + tid + j * TB;
            xq[j] = col < a.n ? a.x[col] : 0.0;
        }
    };
    struct Sl {
        double v[8];
        unsigned short c[8];
    };
    auto meta = [&](int qq) { return qq >= 0 ? a.slice[qq] : make_int4(0, 0, 0, 0); };  // qq < 0: none
    // this lane's run words (wave-uniform shape): K 16-bit words (short runs), or {row, length} of its
    // medium run (8 lanes each)
    auto runword = [&](const int4 &hq) {
        uint4 e = make_uint4(0u, 0u, 0u, 0u);
        const unsigned short *w = a.sent + hq.z;
        if (!PACK) {  // one {row, length} word per lane or per medium run: one load, no branches (r06hh: 5 % on bands)
            e.x = (hq.y & 0xffff) ? reinterpret_cast<const unsigned *>(w)[(hq.y >> 16) ? lane >> 3 : lane] : 0u;
            return e;
        }
        if (!(hq.y & 0xffff))
            return e;
        if (hq.y >> 16)
            e.x = reinterpret_cast<const unsigned *>(w)[lane >> 3];
        else if (hq.w == 8)
            e = reinterpret_cast<const uint4 *>(w)[lane];
        else if (hq.w == 4) {
            const uint2 u = reinterpret_cast<const uint2 *>(w)[lane];
            e.x = u.x;
            e.y = u.y;
        } else if (hq.w == 2)
            e.x = reinterpret_cast<const unsigned *>(w)[lane];
        else
            e.x = w[lane];
        return e;
    };
    auto load8 = [&](const int4 &hq, Sl &d) {  // slot pairs: one 16-B value load, one 4-B column load; an odd last slot alone
        const int Lm = hq.y & 0xffff, pairs = Lm >> 1;  // wave-uniform
        const v2d_t *vp = reinterpret_cast<const v2d_t *>(a.val + hq.x) + lane;
        const unsigned *cp = reinterpret_cast<const unsigned *>(a.col + hq.x) + lane;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            v2d_t v = v2d_t{0.0, 0.0};
            unsigned c = 0u;
            if (p < pairs) {
                v = slab_stream<NT>(vp + 64 * p);
                c = slab_stream<NT>(cp + 64 * p);
            } else if (p == pairs && (Lm & 1)) {
                v.x = slab_stream<NT>(a.val + hq.x + 128 * p + lane);
                c = slab_stream<NT>(a.col + hq.x + 128 * p + lane);
            }
            d.v[2 * p] = v.x;
            d.v[2 * p + 1] = v.y;
            d.c[2 * p] = (unsigned short)(c & 0xffffu);
            d.c[2 * p + 1] = (unsigned short)(c >> 16);
        }
    };
    // the wave's slice after slice q of segment s: q + NW in s, else its first one in s + 1 (-1: none)
    auto nxt = [&](int q, int s, int &qn, int &sn) {
        qn = -1;
        sn = s;
        if (q < 0)
            return;
        if (q + NW < segd(s).z) {
            qn = q + NW;
            return;
        }
        if (s + 1 < bd.w) {
            const int4 ns = segd(s + 1);
            if (ns.y + wave < ns.z) {
                qn = ns.y + wave;
                sn = s + 1;
            }
        }
    };
    int qa = -1, sa = -1, qb = -1, sb = -1;
    int4 h0 = make_int4(0, 0, 0, 0), h1 = make_int4(0, 0, 0, 0);
    uint4 e0 = make_uint4(0u, 0u, 0u, 0u);
    Sl d0, d1;
    if (bd.z < bd.w)
        fetch_x(segd(bd.z).x);
    for (int sg = bd.z; sg < bd.w; ++sg) {  // block-uniform
        const int4 seg = segd(sg);
        const int p0 = seg.w, p1 = segd(sg + 1).w;
        __syncthreads();  // the previous segment's readers of xs (and its folds) are done
#pragma unroll
        for (int j = 0; j < XPT; ++j)
            xs[tid + j * TB] = xq[j];
        __syncthreads();
        SELL_STAMP(b, 1 + 3 * (sg - bd.z));
        if (sg + 1 < bd.w)
            fetch_x(segd(sg + 1).x);
        // long runs first (their loads in flight behind the slices of other waves): pieces of <= 512 values
        for (int u = p0 + wave; u < p1; u += NW) {  // wave-uniform
            const int4 pc = a.lng[u];
            double v[8];
            unsigned short c[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = lane + 64 * j;
                v[j] = k < pc.y ? slab_stream<NT>(a.val + pc.x + k) : 0.0;
                c[j] = k < pc.y ? slab_stream<NT>(a.col + pc.x + k) : (unsigned short)0;
            }
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const double pv = v[j] * xs[c[j]];
                s += lane + 64 * j < pc.y ? pv : 0.0;
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1)
                s += __shfl_xor(s, o);
            if (lane == 0)
                lpart[u - p0] = s;
        }
        SELL_STAMP(b, 2 + 3 * (sg - bd.z));
        // slices, software-pipelined per wave and across segments: while slice qa computes, the wave's
        // next slice's values and run words and the one after's header are in flight -- at a segment's end
        // those are the next segment's first slices, so the pipeline refills during the x-stage barriers
        if (sa != sg) {  // prime: the wave's first slice of this segment
            qa = seg.y + wave < seg.z ? seg.y + wave : -1;
            sa = sg;
            h0 = meta(qa);
            load8(h0, d0);
            e0 = runword(h0);
            nxt(qa, sa, qb, sb);
            h1 = meta(qb);
        }
        while (qa >= 0 && sa == sg) {  // wave-uniform
            load8(h1, d1);
            const uint4 e1 = runword(h1);
            int qc, sc;
            nxt(qb, sb, qc, sc);
            const int4 h2 = meta(qc);
            // K short runs of <= ST slots per lane, each continuing its row's sum in CSR order
            auto short_runs = [&](auto KC, auto STC) {
                constexpr int K = decltype(KC)::value, ST = decltype(STC)::value;
                const unsigned ew[4] = {e0.x, e0.y, e0.z, e0.w};
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned wd = (ew[k >> 1] >> (16 * (k & 1))) & 0xffffu;
                    const int row = (int)(wd & 0xfffu), len = (int)(wd >> 12);
                    double acc = len > 0 ? yacc[row] : 0.0;
#pragma unroll
                    for (int j = 0; j < ST; ++j) {
                        const double pv = d0.v[k * ST + j] * xs[d0.c[k * ST + j]];
                        acc += j < len ? pv : 0.0;  // acc never -0.0 (sums start at +0.0): adding +0.0 is exact
                    }
                    if (len > 0)
                        yacc[row] = acc;
                }
            };
            const int row = (int)(e0.x & 0xffffu), len = (int)(e0.x >> 16);  // medium, or short unpacked
            if (!PACK && !(h0.y >> 16)) {  // wave-uniform: a slice of 64 short runs, lane = run, in CSR order
                double acc = len > 0 ? yacc[row] : 0.0;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const double pv = d0.v[j] * xs[d0.c[j]];
                    acc += j < len ? pv : 0.0;  // acc never -0.0 (sums start at +0.0): adding +0.0 is exact
                }
                if (len > 0)
                    yacc[row] = acc;
            } else if (!(h0.y >> 16)) {  // wave-uniform: a slice of short runs, K per lane, in CSR order
                const int pk = h0.w;
                if (pk == 8)
                    short_runs(std::integral_constant<int, 8>{}, std::integral_constant<int, 1>{});
                else if (pk == 4)
                    short_runs(std::integral_constant<int, 4>{}, std::integral_constant<int, 2>{});
                else if (pk == 2 && (h0.y & 0xffff) == 6)
                    short_runs(std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{});
                else if (pk == 2)
                    short_runs(std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{});
                else
                    short_runs(std::integral_constant<int, 1>{}, std::integral_constant<int, 8>{});
            } else {  // 8 medium runs, 8 lanes each: lane-strided sums, a fixed xor butterfly
                double s = 0.0;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const double pv = d0.v[j] * xs[d0.c[j]];
                    s += 8 * j + (lane & 7) < len ? pv : 0.0;
                }
                s += __shfl_xor(s, 1);
                s += __shfl_xor(s, 2);
                s += __shfl_xor(s, 4);
                if ((lane & 7) == 0 && len > 0)
                    yacc[row] += s;
            }
            qa = qb;
            sa = sb;
            h0 = h1;
            e0 = e1;
            d0 = d1;
            qb = qc;
            sb = sc;
            h1 = h2;
        }
        SELL_STAMP(b, 3 + 3 * (sg - bd.z));
        if (p1 > p0) {  // block-uniform: each run's pieces, in order, onto its row
            __syncthreads();
            for (int i = tid; i < p1 - p0; i += TB) {
                const int4 pc = a.lng[p0 + i];
                const int first = pc.w & 0xffff, np = pc.w >> 16;
                if (i == first) {
                    double s = yacc[pc.z];
                    for (int q = 0; q < np; ++q)
                        s += lpart[first + q];
                    yacc[pc.z] = s;
                }
            }
        }
    }
    __syncthreads();
    if (a.groups > 1) {  // block-uniform
        group_out<TB>(a, b, bd.x, nrows, yacc);
        SELL_STAMP(b, kSellLabStampsEnd);
        return;
    }
    for (int i = tid; i < nrows; i += TB)
        a.y[bd.x + i] = yacc[i];
    SELL_STAMP(b, kSellLabStampsEnd);
}

hipError_t launch_slab(mspmv_handle_s *h, const TilePlan &plan, const double *d_x, double *d_y)
{
    const SlabData &s = *plan.slab;
    SlabArgs a{};
    a.blk = s.d_blk;
    a.chunk = s.d_chunk;
    a.ent = s.d_ent;
    a.val = s.d_val;
    a.col = s.d_col;
    a.x = d_x;
    a.y = d_y;
    a.n = h->n;
    a.num_tiles = plan.num_tiles;
    a.bounds = plan.d_bounds;
    a.split = plan.d_split;
    a.fix = plan.num_carries ? plan.d_fix : nullptr;
    a.fix_cnt = plan.d_fix_cnt;
    a.fault = h->d_fault;
    a.carry_val = plan.d_carry_val;
    a.head_val = plan.d_carry_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    a.head_pub = a.head_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    a.groups = s.groups;
    a.m = h->m;
    a.part = s.d_part;
    a.gcnt = s.d_gcnt;
    a.slice = s.d_slice;
    a.sent = s.d_sent;
    a.lng = s.d_long;
    if (plan.num_tiles == 0)
        return hipSuccess;
    const bool nt = stream_nt(h);
    const dim3 grid(plan.num_tiles);
    if (s.cfg == 2) {
        const dim3 tb(kSlabCfgs[2].threads);
        if (nt && s.pack)
            hipLaunchKernelGGL((k_spmv_sell<true, true>), grid, tb, 0, h->stream, a);
        else if (nt)
            hipLaunchKernelGGL((k_spmv_sell<true, false>), grid, tb, 0, h->stream, a);
        else if (s.pack)
            hipLaunchKernelGGL((k_spmv_sell<false, true>), grid, tb, 0, h->stream, a);
        else
            hipLaunchKernelGGL((k_spmv_sell<false, false>), grid, tb, 0, h->stream, a);
        return hipGetLastError();
    }
    const dim3 b1(kSlabCfgs[1].threads), b0(kSlabCfgs[0].threads);
    if (s.cfg == 1 && nt)
        hipLaunchKernelGGL((k_spmv_slab<true, 1>), grid, b1, 0, h->stream, a);
    else if (s.cfg == 1)
        hipLaunchKernelGGL((k_spmv_slab<false, 1>), grid, b1, 0, h->stream, a);
    else if (nt)
        hipLaunchKernelGGL((k_spmv_slab<true, 0>), grid, b0, 0, h->stream, a);
    else
        hipLaunchKernelGGL((k_spmv_slab<false, 0>), grid, b0, 0, h->stream, a);
    return hipGetLastError();
}

#ifdef MSPMV_SELL_LAB_STAMPS
extern "C" __attribute__((visibility("default"))) int mspmv_lab_sell_stamps(unsigned long long *host, int n)
{
    const int m = std::min(n, kSellLabBlocks * kSellLabStamps);
    static const std::vector<unsigned long long> zero((size_t)kSellLabBlocks * kSellLabStamps, 0ull);
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sell_lab_stamps), sizeof(unsigned long long) * (size_t)m) != hipSuccess)
        return -1;
    // cleared for the next matrix (a block with fewer segments leaves the earlier matrix's slots otherwise)
    return hipMemcpyToSymbol(HIP_SYMBOL(g_sell_lab_stamps), zero.data(), sizeof(unsigned long long) * zero.size()) ==
                   hipSuccess
               ? m
               : -1;
}
#endif

std::string slab_kernel_name(const mspmv_handle_s *h)
{
    const auto it = h->plans.find(kSlabPlanKey);
    const SlabData *sd = it != h->plans.end() ? it->second.slab : nullptr;
    const int cfg = sd ? sd->cfg : 0;
    if (cfg == 2)
        return std::string("k_spmv_sell<") + (stream_nt(h) ? "true" : "false") + "," + (sd->pack ? "true" : "false") + ">";
    return std::string("k_spmv_slab<") + (stream_nt(h) ? "true" : "false") + "," + std::to_string(cfg) + ">";
}

template <typename T>
static void slab_free(T *&p)
{
    if (p)
        (void)hipFree(p);
    p = nullptr;
}

void free_slab(SlabData *s)
{
    if (!s)
        return;
    slab_free(s->d_blk);
    slab_free(s->d_chunk);
    slab_free(s->d_ent);
    slab_free(s->d_val);
    slab_free(s->d_col);
    slab_free(s->d_part);
    slab_free(s->d_gcnt);
    slab_free(s->d_slice);
    slab_free(s->d_sent);
    slab_free(s->d_long);
    delete s;
}

template <typename T>
static mspmv_status slab_upload(T **d, const std::vector<T> &hsrc, size_t pad = 0)
{
    const size_t bytes = sizeof(T) * (hsrc.size() + pad);
    if (hipMalloc((void **)d, bytes ? bytes : sizeof(T)) != hipSuccess) {
        *d = nullptr;
        set_error("column-slab plan: hipMalloc failed");
        return MSPMV_ERR_HIP;
    }
    hipError_t e = hsrc.empty() ? hipSuccess : hipMemcpy(*d, hsrc.data(), sizeof(T) * hsrc.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && pad)
        e = memset_sync(*d + hsrc.size(), 0, sizeof(T) * pad);
    if (e != hipSuccess) {
        set_error(std::string("column-slab plan upload: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}

// Per block: its nonzeros [n0, n1) with columns in [clo, chi) in slab-major order (stable within a
// slab: CSR order), placed at stream position base, cut into chunks of one slab, <= C.chunk nonzeros
// and <= C.entries runs of one row.
struct SlabBlockOut {
    std::vector<int4> chunks;  // entry0 relative to the block
    std::vector<uint2> ents;
    int slabs = 0;
};

static void slab_block(const std::vector<int> &ro, const std::vector<int> &ci, const std::vector<double> &va,
                       int r0, int n0, int r1, int n1, int clo, int chi, int base, const SlabCfg &C, double *oval,
                       unsigned short *ocol, SlabBlockOut &out)
{
    const int W = C.cols;
    const int rlast = n1 > ro[(size_t)r1] ? r1 : r1 - 1;  // the trailing partial row, when there is one
    std::vector<int> ks, kr;  // the block's nonzeros in the column range, CSR order, and their local rows
    for (int r = r0; r <= rlast; ++r) {
        const int k0 = std::max(ro[(size_t)r], n0), k1 = std::min(ro[(size_t)r + 1], n1);
        for (int k = k0; k < k1; ++k)
            if (ci[(size_t)k] >= clo && ci[(size_t)k] < chi) {
                ks.push_back(k);
                kr.push_back(r - r0);
            }
    }
    const int cnt = (int)ks.size();
    if (cnt <= 0)
        return;
    int smin = 0x7fffffff, smax = -1;
    for (int k : ks) {
        const int s = ci[(size_t)k] / W;
        smin = std::min(smin, s);
        smax = std::max(smax, s);
    }
    const int ns = smax - smin + 1;
    std::vector<int> off((size_t)ns + 1, 0);
    for (int k : ks)
        ++off[(size_t)(ci[(size_t)k] / W - smin) + 1];
    for (int s = 0; s < ns; ++s) {
        out.slabs += off[(size_t)s + 1] > 0;
        off[(size_t)s + 1] += off[(size_t)s];
    }
    std::vector<int> row((size_t)cnt);  // local row of each reordered nonzero
    std::vector<int> put(off.begin(), off.end() - 1);
    for (int i = 0; i < cnt; ++i) {
        const int k = ks[(size_t)i];
        const int s = ci[(size_t)k] / W;
        const int q = put[(size_t)(s - smin)]++;
        oval[(size_t)base + q] = va[(size_t)k];
        ocol[(size_t)base + q] = (unsigned short)(ci[(size_t)k] - s * W);
        row[(size_t)q] = kr[(size_t)i];
    }
    for (int s = 0; s < ns; ++s) {
        int q = off[(size_t)s];
        const int qe = off[(size_t)s + 1];
        while (q < qe) {  // chunks of this slab
            const int start = q, e0 = (int)out.ents.size();
            int ne = 0;
            while (q < qe && q - start < C.chunk) {
                int k = q;
                while (k < qe && k - start < C.chunk && row[(size_t)k] == row[(size_t)q])
                    ++k;
                if (ne == C.entries)
                    break;
                out.ents.push_back(make_uint2((unsigned)(q - start) | ((unsigned)(k - q) << 16), (unsigned)row[(size_t)q]));
                ++ne;
                q = k;
            }
            const int len = q - start;
            // runs longer than kSlabLongRun first (whole waves sum them), then the short ones
            std::stable_partition(out.ents.begin() + e0, out.ents.end(),
                                  [](const uint2 &e) { return (int)(e.x >> 16) > kSlabLongRun; });
            int nlong = 0, slen = 0;
            for (int i = e0; i < (int)out.ents.size(); ++i) {
                const int el = (int)(out.ents[(size_t)i].x >> 16);
                nlong += el > kSlabLongRun;
                slen += el > kSlabLongRun ? 0 : el;
            }
            const int ns_ = ne - nlong;
            // lanes per short run: the fewest latency steps -- rounds of runs over the workgroup x (the
            // run's products per lane + its butterfly + ~8 steps of LDS round trips); the older rule, the
            // smallest G with 4 G >= the mean run, took two rounds where one does (44 -> 40 us, r04w)
            const int mean = ns_ > 0 ? (slen + ns_ - 1) / ns_ : 1;
            int lg = 0, best = 1 << 30;
            for (int l = 0; l <= 6; ++l) {
                const int rounds = (ns_ + (C.threads >> l) - 1) / (C.threads >> l);
                const int cost = rounds * ((mean + (1 << l) - 1) / (1 << l) + 2 * l + 8);
                if (cost < best) {
                    best = cost;
                    lg = l;
                }
            }
            out.chunks.push_back(make_int4(base + start, len | (lg << 13) | (nlong << 16), smin + s, e0));
        }
    }
}

// Merge-path blocks of (rows + nonzeros) for a slab plan: at least g0 of them (one resident generation
// of the slab kernel), more -- x 9/8 at a time, up to max_g -- while a block would end more than rows_cap
// rows (its row sums sit in LDS).  Fills p.d_bounds / p.d_split, their host copies and the step.
static mspmv_status slab_bounds(mspmv_handle_s *h, long long g0, long long max_g, int rows_cap, TilePlan &p,
                                std::vector<int2> &hb, std::vector<unsigned char> &hs, long long &step)
{
    const long long total = (long long)h->m + h->nnz;
    long long G = std::max(g0, ((long long)h->m + rows_cap - 1) / rows_cap);
    for (;; G = G + std::max(1LL, G / 8)) {
        if (G > max_g)
            return MSPMV_ERR_UNSUPPORTED;
        step = (total + G - 1) / G;
        if (step > (1LL << 30))
            return MSPMV_ERR_UNSUPPORTED;
        const int T = (int)((total + step - 1) / step);
        if (p.d_bounds)
            (void)hipFree(p.d_bounds);
        if (p.d_split)
            (void)hipFree(p.d_split);
        p.d_bounds = nullptr;
        p.d_split = nullptr;
        if (hipMalloc((void **)&p.d_bounds, sizeof(int2) * ((size_t)T + 1)) != hipSuccess ||
            hipMalloc((void **)&p.d_split, (size_t)T + 1) != hipSuccess) {
            set_error("column-slab plan: hipMalloc failed");
            return MSPMV_ERR_HIP;
        }
        hipError_t e = launch_merge_coords(h->d_row_offsets, h->m, h->nnz, step, T, p.d_bounds, h->stream);
        if (e == hipSuccess)
            e = launch_snap(h->d_row_offsets, h->m, p.d_bounds, p.d_split, T, (int)(step / kSnapDiv), h->stream);
        hb.assign((size_t)T + 1, make_int2(0, 0));
        hs.assign((size_t)T + 1, 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(hb.data(), p.d_bounds, sizeof(int2) * hb.size(), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(hs.data(), p.d_split, hs.size(), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) {
            set_error(std::string("column-slab plan: ") + hipGetErrorString(e));
            return MSPMV_ERR_HIP;
        }
        if (hb[0].x != 0 || hb[0].y != 0 || hb[(size_t)T].x != h->m || hb[(size_t)T].y != h->nnz) {
            set_error("column-slab plan: bad end boundaries");
            return MSPMV_ERR_INVALID;
        }
        int rows_max = 0;
        bool ok = true;
        for (int t = 0; t < T; ++t) {
            const int nr = hb[(size_t)t + 1].x - hb[(size_t)t].x, nz = hb[(size_t)t + 1].y - hb[(size_t)t].y;
            ok = ok && nr >= 0 && nz >= 0;
            rows_max = std::max(rows_max, nr);
        }
        if (!ok) {
            set_error("column-slab plan: non-monotone boundaries");
            return MSPMV_ERR_INVALID;
        }
        p.num_tiles = T;
        if (rows_max <= rows_cap)
            return MSPMV_OK;
    }
}

// The matrix back on the host (the plan builders reorder it block by block).
static mspmv_status slab_host_matrix(mspmv_handle_s *h, std::vector<int> &ro, std::vector<int> &ci,
                                     std::vector<double> &va)
{
    ro.resize((size_t)h->m + 1);
    ci.resize((size_t)h->nnz);
    va.resize((size_t)h->nnz);
    hipError_t e = hipMemcpy(ro.data(), h->d_row_offsets, sizeof(int) * ro.size(), hipMemcpyDeviceToHost);
    if (e == hipSuccess)
        e = hipMemcpy(ci.data(), h->d_cols, sizeof(int) * ci.size(), hipMemcpyDeviceToHost);
    if (e == hipSuccess)
        e = hipMemcpy(va.data(), h->d_vals, sizeof(double) * va.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        set_error(std::string("column-slab plan: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}

// The blocks' reordered streams, chunks and entries to the device, then the plan's split rows (their
// carries and heads: three [T][16] slots, as the tile plans) and tile modes 255.
static mspmv_status slab_finish(mspmv_handle_s *h, TilePlan &p, int cfg, int groups,
                                const std::vector<int4> &blk, const std::vector<SlabBlockOut> &outs,
                                const std::vector<double> &oval, const std::vector<unsigned short> &ocol,
                                const std::vector<int2> &hb, const std::vector<unsigned char> &hs)
{
    const int T = p.num_tiles;
    std::vector<int4> dblk(blk), chunks;
    std::vector<uint2> ents;
    long long staged = 0;
    for (int t = 0; t < T; ++t) {
        const SlabBlockOut &o = outs[(size_t)t];
        if ((int)o.chunks.size() > kSlabMaxChunks)  // more chunks than one block's LDS table holds
            return MSPMV_ERR_UNSUPPORTED;
        const int c0 = (int)chunks.size(), ebase = (int)ents.size();
        for (int4 c : o.chunks) {
            c.w += ebase;
            chunks.push_back(c);
        }
        ents.insert(ents.end(), o.ents.begin(), o.ents.end());
        dblk[(size_t)t].z = c0;
        dblk[(size_t)t].w = (int)chunks.size();
        staged += (long long)o.slabs * kSlabCfgs[cfg].cols * 8;
    }
    chunks.push_back(make_int4(0, 0, 0, (int)ents.size()));  // sentinel: the last chunk's entry end
    SlabData *s = new SlabData();
    s->cfg = cfg;
    s->groups = groups;
    s->num_chunks = (int)chunks.size() - 1;
    s->num_entries = (int)ents.size();
    s->x_bytes_per_nnz = (double)staged / (double)h->nnz;
    p.slab = s;
    mspmv_status st;
    if ((st = slab_upload(&s->d_blk, dblk)) != MSPMV_OK || (st = slab_upload(&s->d_chunk, chunks)) != MSPMV_OK ||
        (st = slab_upload(&s->d_ent, ents)) != MSPMV_OK || (st = slab_upload(&s->d_val, oval, kNnzPad)) != MSPMV_OK ||
        (st = slab_upload(&s->d_col, ocol, kNnzPad)) != MSPMV_OK)
        return st;
    if (groups > 1) {
        const std::vector<unsigned> zero((size_t)T / groups, 0u);
        if ((st = slab_upload(&s->d_gcnt, zero)) != MSPMV_OK)
            return st;
        if (hipMalloc((void **)&s->d_part, sizeof(double) * (size_t)groups * h->m) != hipSuccess) {
            s->d_part = nullptr;
            set_error("column-slab plan: hipMalloc failed");
            return MSPMV_ERR_HIP;
        }
    }
    p.carry_L = 16;
    if (hipMalloc((void **)&p.d_carry_val, sizeof(double) * (size_t)T * 16 * 3) != hipSuccess ||
        hipMalloc((void **)&p.d_modes[0], (size_t)T) != hipSuccess) {
        set_error("column-slab plan: hipMalloc failed");
        return MSPMV_ERR_HIP;
    }
    if (memset_sync(p.d_modes[0], 255, (size_t)T) != hipSuccess) {
        set_error("column-slab plan: memset failed");
        return MSPMV_ERR_HIP;
    }
    return plan_split_rows(p, hb, hs);
}

// Sliced-ELL layout of one column-group block (rows [r0, r1), columns [lo, hi)): per slab touched, in
// slab order, its runs of one row (CSR order); runs longer than kSellLongRun stored contiguously and
// listed apart in pieces of <= 512 values, the others sorted by length (longest first, rows ascending among equals) and cut into
// slices of 64, value j of the slice's run i at slot j of lane i -- slots in pairs, pair p of lane i at
// 2 (64 p + i): one 16-B value load and one 4-B column load per pair; an odd last slot alone, lane i at
// 128 p + i (slots past a run's length: zeros, never added).  With `pack` (the skewed plans' column groups;
// a band's runs are mostly medium, and its kernel measured 5 % slower with the unpacking) short runs of
// length <= 4 are packed K to a lane (kSellPack: 1 -> 8 runs of 1 slot, 2 -> 4 of 2, 3 -> 2 of 3, 4 -> 2 of 4; run k of lane i in slots
// [k stride, (k + 1) stride)), so a slice of 64 K runs still fills ~8 slots per lane: a power-law block's
// slices then hold 3x the bytes each and a wave's pipeline keeps that much more in flight.  Each slice's
// header {value base, slots per lane | medium << 16, run-word base, K}; run words are 16-bit: packed short
// runs row | length << 12, lane i's K words at i K + k; unpacked short runs and medium runs two per run,
// {row, length}.  Bases
// relative to the block; run-word bases multiples of 8 (the K = 8 words are one 16-B load).
struct SellBlockOut {
    std::vector<int4> segs;
    std::vector<int4> slices;
    std::vector<unsigned short> sents;
    std::vector<int4> longs;
    std::vector<double> val;
    std::vector<unsigned short> col;
    long long staged = 0;
    bool too_many = false;  // a segment with more long-run pieces than the kernel's LDS table holds
};

static void sell_block(const std::vector<int> &ro, const std::vector<int> &ci, const std::vector<double> &va, int r0,
                       int r1, int lo, int hi, bool pack, SellBlockOut &o)
{
    // Slabs are cut from the block's own first column (round 6), not from column 0: a band block's
    // 2 x band + rows columns then take ceil(width / W) slabs, where globally aligned ones took one more about
    // half the time.
    const int W = kSlabCfgs[2].cols;
    std::vector<int> ks, kr;
    int cmin = 0x7fffffff, cmax = -1;
    for (int r = r0; r < r1; ++r)
        for (int k = ro[(size_t)r]; k < ro[(size_t)r + 1]; ++k)
            if (ci[(size_t)k] >= lo && ci[(size_t)k] < hi) {
                ks.push_back(k);
                kr.push_back(r - r0);
                cmin = std::min(cmin, ci[(size_t)k]);
                cmax = std::max(cmax, ci[(size_t)k]);
            }
    if (ks.empty())
        return;
    auto slab_of = [&](int c) { return (c - cmin) / W; };
    const int ns = slab_of(cmax) + 1;
    std::vector<int> off((size_t)ns + 1, 0);
    for (int k : ks)
        ++off[(size_t)slab_of(ci[(size_t)k]) + 1];
    for (int s = 0; s < ns; ++s)
        off[(size_t)s + 1] += off[(size_t)s];
    std::vector<int> ord(ks.size()), put(off.begin(), off.end() - 1);
    for (size_t i = 0; i < ks.size(); ++i)
        ord[(size_t)put[(size_t)slab_of(ci[(size_t)ks[i]])]++] = (int)i;  // stable: CSR order per slab
    struct Run {
        int row, first, len;
    };
    for (int s = 0; s < ns; ++s) {
        const int q0 = off[(size_t)s], q1 = off[(size_t)s + 1];
        if (q0 == q1)
            continue;
        std::vector<Run> runs;
        for (int q = q0; q < q1;) {
            int e = q;
            while (e < q1 && kr[(size_t)ord[(size_t)e]] == kr[(size_t)ord[(size_t)q]])
                ++e;
            runs.push_back({kr[(size_t)ord[(size_t)q]], q, e - q});
            q = e;
        }
        const int base = cmin + s * W;  // the segment's first column
        auto put_val = [&](size_t at, int q) {
            const int k = ks[(size_t)ord[(size_t)q]];
            o.val[at] = va[(size_t)k];
            o.col[at] = (unsigned short)(ci[(size_t)k] - base);
        };
        // slot s of lane i in a slice of Lm slots per lane: pairs, then an odd last slot alone
        auto slot_at = [](size_t b, int Lm, int s, int i) {
            const int pairs = Lm >> 1;
            return s < 2 * pairs ? b + (size_t)(s >> 1) * 128 + 2 * i + (s & 1) : b + (size_t)pairs * 128 + i;
        };
        const int slice0 = (int)o.slices.size(), long0 = (int)o.longs.size();
        std::vector<Run> shorts, mediums;
        for (const Run &r : runs) {
            if (r.len > kSellShortRun && r.len <= kSellLongRun) {
                mediums.push_back(r);
            } else if (r.len > kSellLongRun) {  // pieces of <= 512 values: {base, length, row, first | count << 16}
                const size_t base = o.val.size();
                o.val.resize(base + r.len + (r.len & 1), 0.0);  // even bases: the slices' pair loads
                o.col.resize(base + r.len + (r.len & 1), 0);
                for (int j = 0; j < r.len; ++j)
                    put_val(base + j, r.first + j);
                const int np = (r.len + 511) / 512, first = (int)o.longs.size() - long0;
                for (int q = 0; q < np; ++q)
                    o.longs.push_back(make_int4((int)base + 512 * q, std::min(512, r.len - 512 * q), r.row,
                                                first | (np << 16)));
            } else {
                shorts.push_back(r);
            }
        }
        if ((int)o.longs.size() - long0 > kSellMaxPieces)
            o.too_many = true;
        std::stable_sort(shorts.begin(), shorts.end(), [](const Run &x, const Run &y) { return x.len > y.len; });
        for (size_t i0 = 0; i0 < shorts.size();) {
            const int Lmax = shorts[i0].len;
            const bool pk = pack && Lmax <= 4;
            const int K = pk ? kSellPack[Lmax].x : 1, stride = pk ? kSellPack[Lmax].y : Lmax;
            const int S = K * stride;  // slots per lane
            const int n = (int)std::min<size_t>((size_t)64 * K, shorts.size() - i0);
            o.sents.resize((o.sents.size() + 7) & ~(size_t)7, 0);
            const int e0 = (int)o.sents.size();
            o.sents.resize(o.sents.size() + (size_t)64 * (pack ? K : 2), 0);
            const size_t base = o.val.size();
            o.val.resize(base + (size_t)S * 64, 0.0);
            o.col.resize(base + (size_t)S * 64, 0);
            for (int t = 0; t < n; ++t) {  // run t: lane t % 64, its k = t / 64
                const Run &r = shorts[i0 + (size_t)t];
                const int i = t % 64, k = t / 64;
                for (int j = 0; j < r.len; ++j)
                    put_val(slot_at(base, S, k * stride + j, i), r.first + j);
                if (pack) {
                    o.sents[(size_t)e0 + (size_t)i * K + k] = (unsigned short)(r.row | (r.len << 12));
                } else {  // {row, length}, as the medium runs' words
                    o.sents[(size_t)e0 + 2 * (size_t)i] = (unsigned short)r.row;
                    o.sents[(size_t)e0 + 2 * (size_t)i + 1] = (unsigned short)r.len;
                }
            }
            o.slices.push_back(make_int4((int)base, S, e0, K));
            i0 += (size_t)n;
        }
        // medium runs: 8 per slice, 8 lanes each (slots as above) -- value j of the slice's run r at slot j / 8, lane
        // 8 r + j % 8 (header length | 1 << 16: slots per lane, the medium flag)
        std::stable_sort(mediums.begin(), mediums.end(), [](const Run &x, const Run &y) { return x.len > y.len; });
        for (size_t i0 = 0; i0 < mediums.size(); i0 += 8) {
            const int n = (int)std::min<size_t>(8, mediums.size() - i0);
            const int Lm = (mediums[i0].len + 7) / 8;
            o.sents.resize((o.sents.size() + 7) & ~(size_t)7, 0);
            const int e0 = (int)o.sents.size();
            const size_t base = o.val.size();
            o.val.resize(base + (size_t)Lm * 64, 0.0);
            o.col.resize(base + (size_t)Lm * 64, 0);
            for (int i = 0; i < 8; ++i) {
                const Run *r = i < n ? &mediums[i0 + (size_t)i] : nullptr;
                if (r)
                    for (int j = 0; j < r->len; ++j)
                        put_val(slot_at(base, Lm, j / 8, 8 * i + j % 8), r->first + j);
                o.sents.push_back(r ? (unsigned short)r->row : (unsigned short)0);
                o.sents.push_back(r ? (unsigned short)r->len : (unsigned short)0);
            }
            o.slices.push_back(make_int4((int)base, Lm | (1 << 16), e0, 1));
        }
        o.segs.push_back(make_int4(base, slice0, (int)o.slices.size(), long0));
        o.staged += (long long)W * 8;
    }
}

static mspmv_status sell_finish(mspmv_handle_s *h, TilePlan &p, const std::vector<int> &rbs, int G, int spg,
                                const std::vector<int> &ro, const std::vector<int> &ci, const std::vector<double> &va,
                                const std::vector<int2> &hb, const std::vector<unsigned char> &hs)
{
    const int W = kSlabCfgs[2].cols, T = p.num_tiles;
    std::vector<SellBlockOut> outs((size_t)T);
#pragma omp parallel for schedule(dynamic, 2)
    for (int t = 0; t < T; ++t) {
        const int rb = t / G, g = t % G;
        // groups of equal column counts (the blocks' slabs start at their own first column, so a group need
        // not be whole slabs; with whole slabs the last group of the power-law variant held 0.8 of the others'
        // nonzeros and the others set the time)
        (void)spg;
        (void)W;
        const int lo = (int)((long long)g * h->n / G), hi = g == G - 1 ? 0x7fffffff : (int)((long long)(g + 1) * h->n / G);
        sell_block(ro, ci, va, rbs[(size_t)rb], rbs[(size_t)rb + 1], lo, hi, G > 1, outs[(size_t)t]);
    }
    std::vector<int4> blk((size_t)T), segs, longs, slices;
    std::vector<unsigned short> sents;
    std::vector<double> val;
    std::vector<unsigned short> col;
    long long staged = 0;
    for (int t = 0; t < T; ++t) {
        const SellBlockOut &o = outs[(size_t)t];
        if (o.too_many || (int)o.segs.size() > kSellMaxSegs || val.size() + o.val.size() > (size_t)0x7fffff00 ||
            sents.size() + o.sents.size() > (size_t)0x7fffff00)
            return MSPMV_ERR_UNSUPPORTED;
        const int vb = (int)val.size(), sb = (int)slices.size(), lb = (int)longs.size(), g0 = (int)segs.size();
        sents.resize((sents.size() + 7) & ~(size_t)7, 0);  // run-word bases stay multiples of 8
        const int eb = (int)sents.size();
        for (int4 s : o.segs)
            segs.push_back(make_int4(s.x, s.y + sb, s.z + sb, s.w + lb));
        for (int4 s : o.slices)
            slices.push_back(make_int4(s.x + vb, s.y, s.z + eb, s.w));
        for (int4 l : o.longs)
            longs.push_back(make_int4(l.x + vb, l.y, l.z, l.w));
        sents.insert(sents.end(), o.sents.begin(), o.sents.end());
        val.insert(val.end(), o.val.begin(), o.val.end());
        col.insert(col.end(), o.col.begin(), o.col.end());
        const int rb = t / G;
        blk[(size_t)t] = make_int4(rbs[(size_t)rb], rbs[(size_t)rb + 1] - rbs[(size_t)rb], g0, (int)segs.size());
        staged += o.staged;
    }
    segs.push_back(make_int4(0, 0, 0, (int)longs.size()));  // sentinel: the last segment's long-run end
    SlabData *s = new SlabData();
    s->cfg = 2;
    s->groups = G;
    s->pack = G > 1;
    s->num_chunks = (int)segs.size() - 1;
    s->num_entries = (int)longs.size();
    s->x_bytes_per_nnz = (double)staged / (double)h->nnz;
    p.slab = s;
    mspmv_status st;
    if ((st = slab_upload(&s->d_blk, blk)) != MSPMV_OK || (st = slab_upload(&s->d_chunk, segs)) != MSPMV_OK ||
        (st = slab_upload(&s->d_slice, slices)) != MSPMV_OK || (st = slab_upload(&s->d_sent, sents)) != MSPMV_OK ||
        (st = slab_upload(&s->d_long, longs)) != MSPMV_OK || (st = slab_upload(&s->d_val, val, kNnzPad)) != MSPMV_OK ||
        (st = slab_upload(&s->d_col, col, kNnzPad)) != MSPMV_OK)
        return st;
    if (G > 1) {
        const std::vector<unsigned> zero((size_t)T / G, 0u);
        if ((st = slab_upload(&s->d_gcnt, zero)) != MSPMV_OK)
            return st;
        if (hipMalloc((void **)&s->d_part, sizeof(double) * (size_t)G * h->m) != hipSuccess) {
            s->d_part = nullptr;
            set_error("column-slab plan: hipMalloc failed");
            return MSPMV_ERR_HIP;
        }
    }
    p.carry_L = 16;
    if (hipMalloc((void **)&p.d_carry_val, sizeof(double) * (size_t)T * 16 * 3) != hipSuccess ||
        hipMalloc((void **)&p.d_modes[0], (size_t)T) != hipSuccess) {
        set_error("column-slab plan: hipMalloc failed");
        return MSPMV_ERR_HIP;
    }
    if (memset_sync(p.d_modes[0], 255, (size_t)T) != hipSuccess) {
        set_error("column-slab plan: memset failed");
        return MSPMV_ERR_HIP;
    }
    return plan_split_rows(p, hb, hs);
}

// Column-group blocks (kSlabCfgs[1]): whole-row blocks of ~(m + nnz) / R merge items (<= C.rows rows),
// R = the resident blocks / groups, each crossed with the groups' column ranges (consecutive slabs);
// block t = row block t / G, group t % G.  The reported bounds give each row block to its first group
// (the others span nothing), so the plan reads as monotone merge-path tiles.
static mspmv_status build_slab_group_plan(mspmv_handle_s *h, TilePlan &p, double min_nnz_per_block, int cfg,
                                          int num_groups)
{
    const SlabCfg &C = kSlabCfgs[cfg];
    const int nslabs = (h->n + C.cols - 1) / C.cols;
    const char *ge = getenv("MSPMV_SLAB_GROUPS");  // lab: the column-group count (over num_groups too)
    const int want = ge && *ge ? atoi(ge) : num_groups > 0 ? num_groups : kSlabGroups;
    const int G = std::max(1, std::min(std::min(want, kSlabMaxGroups), nslabs));
    const int spg = (nslabs + G - 1) / G;  // slabs per group
    const long long R0 = std::max(1, h->num_cus * C.per_cu / G);
    std::vector<int> ro, ci;
    std::vector<double> va;
    mspmv_status st0;
    ro.resize((size_t)h->m + 1);
    if (hipMemcpy(ro.data(), h->d_row_offsets, sizeof(int) * ro.size(), hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("column-slab plan: row offsets download failed");
        return MSPMV_ERR_HIP;
    }
    // whole-row blocks of at most C.rows rows, R0 of them with the smallest possible largest block (in
    // rows + nonzeros): the least bound B whose greedy cut needs <= R0 blocks (binary search), so a hub
    // row sets B only as far as its own length
    auto cut = [&](long long B, std::vector<int> *out) {
        long long items = 0, blocks = 1;
        int rows = 0;
        for (int r = 0; r < h->m; ++r) {
            const long long it = 1 + (long long)ro[(size_t)r + 1] - ro[(size_t)r];
            if (rows > 0 && (rows == C.rows || items + it > B)) {
                if (out)
                    out->push_back(r);
                ++blocks;
                items = 0;
                rows = 0;
            }
            items += it;
            ++rows;
        }
        return blocks;
    };
    long long lo_b = ((long long)h->m + h->nnz + R0 - 1) / R0, hi_b = (long long)h->m + h->nnz;
    for (int r = 0; r < h->m; ++r)
        lo_b = std::max(lo_b, 1 + (long long)ro[(size_t)r + 1] - ro[(size_t)r]);
    while (lo_b < hi_b) {
        const long long mid = lo_b + (hi_b - lo_b) / 2;
        if (cut(mid, nullptr) <= R0)
            hi_b = mid;
        else
            lo_b = mid + 1;
    }
    const long long target = lo_b;
    std::vector<int> rbs{0};
    cut(target, &rbs);
    rbs.push_back(h->m);
    const int R = (int)rbs.size() - 1;
    const long long Tl = (long long)R * G;
    if (Tl > 64LL * h->num_cus || (double)h->nnz < min_nnz_per_block * (double)Tl)  // before the copy
        return MSPMV_ERR_UNSUPPORTED;
    const int T = (int)Tl;
    if ((st0 = slab_host_matrix(h, ro, ci, va)) != MSPMV_OK)
        return st0;
    std::vector<int2> hb((size_t)T + 1);
    for (int t = 0; t < T; ++t) {
        const int r = rbs[(size_t)(t / G) + (t % G == 0 ? 0 : 1)];
        hb[(size_t)t] = make_int2(r, ro[(size_t)r]);
    }
    hb[(size_t)T] = make_int2(h->m, h->nnz);
    const std::vector<unsigned char> hs((size_t)T + 1, 0);
    if (hipMalloc((void **)&p.d_bounds, sizeof(int2) * hb.size()) != hipSuccess ||
        hipMalloc((void **)&p.d_split, hs.size()) != hipSuccess) {
        set_error("column-slab plan: hipMalloc failed");
        return MSPMV_ERR_HIP;
    }
    if (hipMemcpy(p.d_bounds, hb.data(), sizeof(int2) * hb.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p.d_split, hs.data(), hs.size(), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("column-slab plan: upload failed");
        return MSPMV_ERR_HIP;
    }
    p.num_tiles = T;
    p.lanes = C.threads;
    p.tile_items = (int)std::min<long long>(target, 0x7fffffff);
    p.snap = 0;
    if (cfg == 2)
        return sell_finish(h, p, rbs, G, spg, ro, ci, va, hb, hs);
    auto crange = [&](int g, int &lo, int &hi) {
        lo = std::min(h->n, g * spg * C.cols);
        hi = g == G - 1 ? 0x7fffffff : std::min(h->n, (g + 1) * spg * C.cols);
    };
    // stream positions: block t's nonzeros after those of blocks 0 .. t-1
    std::vector<long long> cnt((size_t)T + 1, 0);
#pragma omp parallel for schedule(dynamic, 4)
    for (int rb = 0; rb < R; ++rb) {
        for (int k = ro[(size_t)rbs[(size_t)rb]]; k < ro[(size_t)rbs[(size_t)rb + 1]]; ++k) {
            const int g = std::min(G - 1, ci[(size_t)k] / (spg * C.cols));
            ++cnt[(size_t)rb * G + g + 1];
        }
    }
    for (int t = 0; t < T; ++t)
        cnt[(size_t)t + 1] += cnt[(size_t)t];
    std::vector<double> oval((size_t)h->nnz);
    std::vector<unsigned short> ocol((size_t)h->nnz);
    std::vector<SlabBlockOut> outs((size_t)T);
    std::vector<int4> blk((size_t)T);
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < T; ++t) {
        const int rb = t / G, g = t % G, r0 = rbs[(size_t)rb], r1 = rbs[(size_t)rb + 1];
        int lo, hi;
        crange(g, lo, hi);
        slab_block(ro, ci, va, r0, ro[(size_t)r0], r1, ro[(size_t)r1], lo, hi, (int)cnt[(size_t)t], C, oval.data(),
                   ocol.data(), outs[(size_t)t]);
        blk[(size_t)t] = make_int4(r0, r1 - r0, 0, 0);
    }
    return slab_finish(h, p, cfg, G, blk, outs, oval, ocol, hb, hs);
}

mspmv_status build_slab_plan(mspmv_handle_s *h, TilePlan &p, double min_nnz_per_block, int cfg, bool groups,
                             int num_groups)
{
    if (h->m <= 0 || h->nnz <= 0)
        return MSPMV_ERR_UNSUPPORTED;
    if (cfg >= 1 || groups)
        return build_slab_group_plan(h, p, min_nnz_per_block, cfg, num_groups);
    std::vector<int2> hb;
    std::vector<unsigned char> hs;
    long long step = 0;
    mspmv_status st0 = slab_bounds(h, (long long)kSlabBlocksPerCu * h->num_cus, 64LL * h->num_cus, kSlabRows, p, hb,
                                   hs, step);
    if (st0 != MSPMV_OK)
        return st0;
    const int T = p.num_tiles;
    if ((double)h->nnz < min_nnz_per_block * T)  // before the matrix is copied or anything allocated
        return MSPMV_ERR_UNSUPPORTED;
    p.lanes = kSlabThreads;
    p.tile_items = (int)step;
    p.snap = (int)(step / kSnapDiv);
    p.num_tiles = T;

    // the matrix on the host, reordered block by block
    std::vector<int> ro, ci;
    std::vector<double> va;
    if ((st0 = slab_host_matrix(h, ro, ci, va)) != MSPMV_OK)
        return st0;
    std::vector<double> oval((size_t)h->nnz);
    std::vector<unsigned short> ocol((size_t)h->nnz);
    std::vector<SlabBlockOut> outs((size_t)T);
    std::vector<int4> blk((size_t)T);
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < T; ++t) {
        const int2 b0 = hb[(size_t)t], b1 = hb[(size_t)t + 1];
        slab_block(ro, ci, va, b0.x, b0.y, b1.x, b1.y, 0, 0x7fffffff, b0.y, kSlabCfgs[0], oval.data(), ocol.data(),
                   outs[(size_t)t]);
        blk[(size_t)t] = make_int4(b0.x, b1.x - b0.x, 0, 0);
    }
    return slab_finish(h, p, 0, 1, blk, outs, oval, ocol, hb, hs);
}


// ---- column-slab SpMM (Y = A X, L = 8 or 16) ------------------------------------------------------
// The L-wide tile kernels gather one L x 8-B panel row per nonzero from L2 (k_spmm_tile): on matrices
// that are not node-blocked that is 64-128 B of L2 -> CU traffic per 12 B of matrix, and a CU takes in
// ~70 GB/s of such gathers, so the gathers, not HBM, set the time (configs[2] cant-shaped L = 16: 513 MB
// of panel lines for 64 MB of HBM bytes; configs[4]'s 27-point L = 8 SpMM: 6 GB per product).  Here a
// block of rows stages each panel row it touches into LDS once, with coalesced loads, and the runs of
// one row read it there: the reference's OmpMergeCsrmm (work_2025/spmm/merge_based.hpp:46-153) computes
// the same y_i = sum_k a_ik X[c_k][:], its merge-path row/nonzero balance (the partition, :62-75)
// re-derived at block granularity.
//
// Plan (build_slab_mm_plan): merge-path blocks of <= cfg.rows rows; a block's distinct columns, sorted,
// are cut greedily into segments of <= cfg.cols consecutive column ids (a segment starts at its first
// touched column, so the gaps between a stencil's planes or a band's ends cost nothing); the block's
// nonzeros are reordered by segment, CSR order within it (rows ascending), and cut into chunks of
// <= cfg.chunk nonzeros and <= cfg.entries runs of one row.  Per chunk: its stream and runs go to LDS
// (loaded two chunks earlier), its segment's panel rows too when the segment changes (loaded during the
// previous chunk); groups of L/2 column-pair lanes x 2^lg nonzero lanes take the runs round-robin, lane
// (c, j) sums products j, j + 2^lg, ... of its run for columns 2c, 2c + 1 in order, a fixed xor
// butterfly folds the group and lane (c, 0) adds the run to the row's sums in LDS.  A row has one run
// per chunk and chunks run in order, so every sum is fixed-order (reproducible) and within the 2 (len+1)
// eps (|A||X|)_i reordering bound of the CSR-order sum (mspmv_tile_modes reports the blocks as 255).
// Rows split between blocks are closed as the tile kernels close them (close_split_rows).
struct SlabMmArgs {
    const int4 *blk;
    const int4 *chunk;
    const uint2 *ent;
    const double *val;
    const unsigned short *col;
    const double *x;  // panel X, row stride ld
    double *y;        // panel Y, row stride ld
    int ld;
    int num_tiles;
    const CgControl *ctrl;
    // split rows (close_split_rows reads these names)
    const int2 *bounds;
    const unsigned char *split;
    const int4 *fix;
    unsigned *fix_cnt;
    double *carry_val;
    double *head_val;
    double *head_pub;
    unsigned *fault;            // the handle's fault word (ticket_arrive)
};

// Configurations (one kernel instance each): LDS = 2 x cols x L x 8 (two segment buffers) + (rows + 1) x
// L x 8 (row sums) + 10 x chunk (stream) + 8 x entries + the chunk table.
constexpr SlabMmCfg kSlabMmCfgs[] = {
    {8, 512, 384, 256, 1024, 256},     // 0: L = 8, 71 KB, two blocks per CU
    {8, 1024, 768, 512, 2048, 512},    // 1: L = 8, 139 KB, one block per CU
    {16, 1024, 256, 320, 2048, 512},   // 2: L = 16, 139 KB, one block per CU
    {16, 512, 192, 128, 1024, 256},    // 3: L = 16, 71 KB, two blocks per CU
};
constexpr int kSlabMmNumCfgs = (int)(sizeof(kSlabMmCfgs) / sizeof(kSlabMmCfgs[0]));
constexpr int kSlabMmSets = 4;  // stream chunks in flight per block (register sets)

static int slab_mm_lab_cfg()  // lab: MSPMV_SPMM_SLAB_CFG picks a configuration by index (A/B runs)
{
    static const int v = [] {
        const char *e = getenv("MSPMV_SPMM_SLAB_CFG");
        return e && *e ? atoi(e) : -1;
    }();
    return v;
}

const SlabMmCfg &slab_mm_cfg(int L, int which)
{
    if (which < 0)
        which = slab_mm_lab_cfg();
    if (which >= 0 && which < kSlabMmNumCfgs && kSlabMmCfgs[which].L == L)
        return kSlabMmCfgs[which];
    return L == 8 ? kSlabMmCfgs[0] : kSlabMmCfgs[2];
}

static int slab_mm_cfg_index(const SlabMmCfg &c) { return (int)(&c - kSlabMmCfgs); }

typedef __attribute__((address_space(3))) void lds_void_t;

// One 16-B-per-lane LDS-DMA load (global_load_lds_dwordx4): lane l's 16 bytes from its own gsrc land at
// LDS byte address lds_base + 16 l.  Inline asm, so the compiler neither tracks it (with the builtin it
// treats the DMA as a pending LDS write and waits vmcnt(0) before the kernel's LDS reads, in both wave
// roles) nor keeps M0 (saved and restored here; the callers retire the DMA with their own vmcnt wait).
__device__ __forceinline__ void glds16(const void *gsrc, unsigned lds_base)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_base)
                 : "memory");
}

// Two wave roles per block, so that each load kind waits on its own counter (vmcnt is per wave and
// in order: a block whose waves issued both kinds had to drain every older stream load to use a fresh
// panel load, which capped the stream at ~2 chunks in flight and ~2 TB/s, r05c-r05e):
//  * stream waves (the first half) hold the chunk stream kSlabMmSets chunks ahead in registers and
//    write each chunk's values, columns and runs into LDS; compiler-counted waits, __syncthreads;
//  * panel waves (the second half) stage each segment's panel rows by LDS-DMA (global_load_lds_dwordx4,
//    no registers) into one of two LDS buffers, one segment ahead: a segment's DMA is retired by the
//    panel waves' own vmcnt(0) before the barrier that opens the segment to readers, and the next one
//    is issued into the buffer whose readers passed the previous barrier; raw s_barrier with
//    lgkmcnt(0) only (a __syncthreads would drain the DMA in flight).
// Every wave then sums runs.  Both roles run the same chunk loop, so they meet at every barrier.
template <int CFG, bool NT>
__global__ __launch_bounds__(kSlabMmCfgs[CFG].threads) void k_spmm_slab(SlabMmArgs a)
{
    constexpr SlabMmCfg C = kSlabMmCfgs[CFG];
    constexpr int L = C.L, TB = C.threads, GL = L / 2;
    constexpr int LGL = GL == 4 ? 2 : 3;                  // log2 GL
    constexpr int TS = TB / 2;                            // stream threads
    constexpr int XW = (TB - TS) / 64;                    // panel waves
    constexpr int IPT = (C.chunk + TS - 1) / TS;          // stream items per stream thread and chunk
    constexpr int EPT = (C.entries + TS - 1) / TS;        // entries per stream thread and chunk
    constexpr int NS = kSlabMmSets;
    static_assert(GL == 4 || GL == 8, "L = 8 or 16");
    static_assert((C.cols * GL) % 64 == 0, "whole 1-KB DMA pieces per segment buffer");
    __shared__ double2 xs[2][C.cols * GL];
    __shared__ double2 yacc[(C.rows + 1) * GL];
    __shared__ double s_val[C.chunk];
    __shared__ unsigned short s_col[C.chunk];
    __shared__ uint2 sent[C.entries];
    __shared__ int4 schunk[kSlabMmMaxChunks + 1];
    const int tid = threadIdx.x;
    // CG: the stop flag is loaded first and tested once the block's table is in
    const int stopped = a.ctrl ? a.ctrl->done : 0;
    const int b = xcd_tile(blockIdx.x, a.num_tiles);
    const int4 bd = a.blk[b];  // {first row, rows ending here, chunk0, chunk1}
    for (int i = tid; i <= bd.w - bd.z; i += TB)
        schunk[i] = a.chunk[bd.z + i];
    const int4 fx = load_fix(a, b);
    const int nrows = bd.y;
    const bool tail = a.split[b + 1] != 0;
    for (int i = tid; i < (nrows + (tail ? 1 : 0)) * GL; i += TB)
        yacc[i] = make_double2(0.0, 0.0);
    __syncthreads();
    if (stopped)  // block-uniform (every block of the launch reads the same word)
        return;
    auto chunk = [&](int ci) __attribute__((always_inline)) {  // block-uniform
        const int4 c = schunk[ci - bd.z];
        return make_int4(__builtin_amdgcn_readfirstlane(c.x), __builtin_amdgcn_readfirstlane(c.y),
                         __builtin_amdgcn_readfirstlane(c.z), __builtin_amdgcn_readfirstlane(c.w));
    };
    const int last = bd.w - 1;
    // The runs of chunk ci over the segment in xb: groups of GL column-pair lanes x 2^lg nonzero lanes
    // take the runs round-robin, lane (c, j) sums products j, j + 2^lg, ... in order, a fixed xor
    // butterfly folds the group, lane (c, 0) adds the run to its row in yacc.
    auto runs = [&](int ci, const double2 *xb) __attribute__((always_inline)) {
        const int4 cd = chunk(ci);
        const int lg = (cd.y >> 13) & 7;
        const int ne = chunk(ci + 1).w - cd.w;
        const int lgg = LGL + lg, Gp = 1 << lg;
        const int c = tid & (GL - 1), j = (tid >> LGL) & (Gp - 1);
        for (int q = tid >> lgg; q < ne; q += TB >> lgg) {  // uniform within a group
            const uint2 en = sent[q];
            const int off = (int)(en.x & 0xffffu), e = off + (int)(en.x >> 16);
            double2 acc = make_double2(0.0, 0.0);
            int k = off + j;
            for (; k + 3 * Gp < e; k += 4 * Gp) {  // 4 panel reads in flight per lane, summed in order
                double v[4];
                double2 xv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    v[u] = s_val[k + u * Gp];
                    xv[u] = xb[(int)s_col[k + u * Gp] * GL + c];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc.x += v[u] * xv[u].x;
                    acc.y += v[u] * xv[u].y;
                }
            }
            if (k < e) {  // the rest (< 4 per lane) as one batch: clamped reads, skipped products
                double v[3];
                double2 xv[3];
#pragma unroll
                for (int u = 0; u < 3; ++u) {
                    const int kk = min(k + u * Gp, e - 1);
                    v[u] = s_val[kk];
                    xv[u] = xb[(int)s_col[kk] * GL + c];
                }
#pragma unroll
                for (int u = 0; u < 3; ++u) {
                    const bool on = k + u * Gp < e;      // acc starts at +0.0 and never becomes -0.0:
                    acc.x += on ? v[u] * xv[u].x : 0.0;  // adding +0.0 is the identity
                    acc.y += on ? v[u] * xv[u].y : 0.0;
                }
            }
            for (int o = Gp >> 1; o > 0; o >>= 1) {
                acc.x += __shfl_xor(acc.x, o * GL);
                acc.y += __shfl_xor(acc.y, o * GL);
            }
            if (j == 0) {
                double2 &yr = yacc[(int)en.y * GL + c];
                yr.x += acc.x;
                yr.y += acc.y;
            }
        }
    };
    if (bd.z < bd.w && tid < TS) {  // ---- stream waves (wave-uniform branch)
        struct Regs {
            double v[IPT];
            unsigned short c[IPT];
            uint2 e[EPT];
        };
        auto fetch = [&](int ci, Regs &r) __attribute__((always_inline)) {
            ci = min(ci, last);  // past the block's end: a repeat of its last chunk, never used (every
                                 // chunk issues the same loads, so the compiler's waits stay counted)
            const int4 cd = chunk(ci);
            const int len = cd.y & 0x1fff;
            const int e0 = cd.w, ne = chunk(ci + 1).w - e0;
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const int k = min(tid + j * TS, len - 1);  // clamped: every load is issued
                r.v[j] = slab_stream<NT>(a.val + cd.x + k);
                r.c[j] = slab_stream<NT>(a.col + cd.x + k);
            }
#pragma unroll
            for (int j = 0; j < EPT; ++j)
                r.e[j] = a.ent[e0 + min(tid + j * TS, ne - 1)];
        };
        Regs rs[NS];
#pragma unroll
        for (int u = 0; u < NS; ++u)
            fetch(bd.z + u, rs[u]);
        int cur = -1, seg = -1;
        for (int ci = bd.z; ci < bd.w; ci += NS) {
#pragma unroll
            for (int u = 0; u < NS; ++u) {
                const int c = ci + u;
                const bool valid = c <= last;
                const int4 cd = chunk(min(c, last));
                if (valid) {
                    if (cd.z != cur) {
                        cur = cd.z;
                        ++seg;
                    }
                    const int len = cd.y & 0x1fff, ne = chunk(c + 1).w - cd.w;
#pragma unroll
                    for (int j = 0; j < IPT; ++j) {
                        const int k = tid + j * TS;
                        if (k < len) {
                            s_val[k] = rs[u].v[j];
                            s_col[k] = rs[u].c[j];
                        }
                    }
#pragma unroll
                    for (int j = 0; j < EPT; ++j) {
                        const int k = tid + j * TS;
                        if (k < ne)
                            sent[k] = rs[u].e[j];
                    }
                }
                fetch(c + NS, rs[u]);
                __syncthreads();
                if (valid)
                    runs(c, xs[seg & 1]);
                __syncthreads();
            }
        }
    } else if (bd.z < bd.w) {  // ---- panel waves
        const int xw = (tid - TS) >> 6, lane = tid & 63;
        auto stage = [&](int c0, int ncols, int buf) __attribute__((always_inline)) {
            const int n2 = ncols * GL;  // double2s of the segment
            for (int p = xw; p * 64 < n2; p += XW) {  // wave-uniform; the DMA writes lane-linear 1-KB pieces
                const int e = min(p * 64 + lane, n2 - 1);
                const unsigned dst = (unsigned)(uintptr_t)(lds_void_t *)&xs[buf][p * 64];
                glds16(a.x + (size_t)(c0 + (e >> LGL)) * a.ld + 2 * (e & (GL - 1)), __builtin_amdgcn_readfirstlane(dst));
            }
        };
        stage(chunk(bd.z).z, chunk(bd.z).y >> 16, 0);
        int cur = -1, seg = -1;
        for (int ci = bd.z; ci < bd.w; ci += NS) {
#pragma unroll
            for (int u = 0; u < NS; ++u) {
                const int c = ci + u;
                const bool valid = c <= last;
                const int4 cd = chunk(min(c, last));
                if (valid && cd.z != cur) {  // chunk c opens the next segment
                    cur = cd.z;
                    ++seg;
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // its DMA has landed
                    int n = c + 1;  // the following segment, into the other buffer (its readers are done)
                    while (n <= last && chunk(n).z == cur)
                        ++n;
                    if (n <= last)
                        stage(chunk(n).z, chunk(n).y >> 16, (seg + 1) & 1);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (valid)
                    runs(c, xs[seg & 1]);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
        }
    }
    // rows ending in the block (row 0 to the head slot when it completes a split row), nontemporal so
    // Y does not displace the panel X from the caches; the trailing partial row -> its carry
    const int r0 = bd.x;
    for (int e = tid; e < nrows * GL; e += TB) {
        const int row = e >> LGL, cp = e & (GL - 1);
        const double2 v = yacc[e];
        double *dst = row == 0 && fx.z > 0 ? a.head_val + (size_t)b * L + 2 * cp : a.y + (size_t)(r0 + row) * a.ld + 2 * cp;
        __builtin_nontemporal_store(v2d_t{v.x, v.y}, reinterpret_cast<v2d_t *>(dst));
    }
    if (tail)
        for (int cp = tid; cp < GL; cp += TB)
            store_sc1_2(a.carry_val + (size_t)b * L + 2 * cp, yacc[nrows * GL + cp]);
    close_split_rows<TB>(a, b, fx, L, a.ld);
}

template <int CFG>
static void launch_slab_mm_cfg(const SlabMmArgs &a, bool nt, hipStream_t s)
{
    const dim3 grid(a.num_tiles), block(kSlabMmCfgs[CFG].threads);
    if (nt)
        hipLaunchKernelGGL((k_spmm_slab<CFG, true>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((k_spmm_slab<CFG, false>), grid, block, 0, s, a);
}

hipError_t launch_slab_mm(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L, int ld,
                          const CgControl *ctrl)
{
    const SlabData &s = *plan.slab;
    if (s.L != L || L != kSlabMmCfgs[s.cfg].L)
        return hipErrorInvalidValue;
    SlabMmArgs a{};
    a.blk = s.d_blk;
    a.chunk = s.d_chunk;
    a.ent = s.d_ent;
    a.val = s.d_val;
    a.col = s.d_col;
    a.x = d_X;
    a.y = d_Y;
    a.ld = ld > 0 ? ld : L;
    a.num_tiles = plan.num_tiles;
    a.ctrl = ctrl;
    a.bounds = plan.d_bounds;
    a.split = plan.d_split;
    a.fix = plan.num_carries ? plan.d_fix : nullptr;
    a.fix_cnt = plan.d_fix_cnt;
    a.fault = ctrl ? &const_cast<CgControl *>(ctrl)->fault : h->d_fault;
    a.carry_val = plan.d_carry_val;
    a.head_val = plan.d_carry_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    a.head_pub = a.head_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    if (plan.num_tiles == 0)
        return hipSuccess;
    const bool nt = stream_nt(h);
    switch (s.cfg) {
    case 0: launch_slab_mm_cfg<0>(a, nt, h->stream); break;
    case 1: launch_slab_mm_cfg<1>(a, nt, h->stream); break;
    case 2: launch_slab_mm_cfg<2>(a, nt, h->stream); break;
    case 3: launch_slab_mm_cfg<3>(a, nt, h->stream); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

std::string slab_mm_kernel_name(const mspmv_handle_s *h, const TilePlan &plan)
{
    return "k_spmm_slab<" + std::to_string(plan.slab ? plan.slab->cfg : 0) + "," + (stream_nt(h) ? "true" : "false") +
           ">";
}

// Per block: its nonzeros [n0, n1) reordered by column segment (CSR order within it), cut into chunks
// of one segment, <= cfg.chunk nonzeros and <= cfg.entries runs of one row.  chunk.x is relative to n0.
struct SlabMmBlockOut {
    std::vector<int4> chunks;  // entry0 relative to the block
    std::vector<uint2> ents;
    long long staged_cols = 0;
    bool ok = true;
};

static void slab_mm_block(const SlabMmCfg &cfg, const std::vector<int> &ro, const std::vector<int> &ci,
                          const std::vector<double> &va, int r0, int n0, int r1, int n1, double *oval,
                          unsigned short *ocol, SlabMmBlockOut &out)
{
    const int cnt = n1 - n0;
    if (cnt <= 0)
        return;
    std::vector<int> u(ci.begin() + n0, ci.begin() + n1);  // distinct columns, ascending
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    std::vector<int> seg_lo, seg_n;  // greedy segments: [lo, lo + n), n <= cfg.cols
    for (size_t i = 0; i < u.size();) {
        const int lo = u[i];
        size_t k = i;
        while (k < u.size() && u[k] < lo + cfg.cols)
            ++k;
        seg_lo.push_back(lo);
        seg_n.push_back(u[k - 1] - lo + 1);
        out.staged_cols += u[k - 1] - lo + 1;
        i = k;
    }
    const int ns = (int)seg_lo.size();
    auto seg_of = [&](int c) { return (int)(std::upper_bound(seg_lo.begin(), seg_lo.end(), c) - seg_lo.begin()) - 1; };
    std::vector<int> off((size_t)ns + 1, 0);
    for (int k = n0; k < n1; ++k)
        ++off[(size_t)seg_of(ci[(size_t)k]) + 1];
    for (int s = 0; s < ns; ++s)
        off[(size_t)s + 1] += off[(size_t)s];
    std::vector<int> row((size_t)cnt);
    std::vector<int> put(off.begin(), off.end() - 1);
    const int rlast = n1 > ro[(size_t)r1] ? r1 : r1 - 1;  // the trailing partial row, when there is one
    for (int r = r0; r <= rlast; ++r) {
        const int k0 = std::max(ro[(size_t)r], n0), k1 = std::min(ro[(size_t)r + 1], n1);
        for (int k = k0; k < k1; ++k) {
            const int s = seg_of(ci[(size_t)k]);
            const int q = put[(size_t)s]++;
            oval[(size_t)n0 + q] = va[(size_t)k];
            ocol[(size_t)n0 + q] = (unsigned short)(ci[(size_t)k] - seg_lo[(size_t)s]);
            row[(size_t)q] = r - r0;
        }
    }
    constexpr int kGL[2] = {4, 8};
    const int GL = kGL[cfg.L == 16 ? 1 : 0];
    int lg_max = 0;
    while ((GL << (lg_max + 1)) <= 64)  // a run's lanes stay inside one wave (xor butterfly)
        ++lg_max;
    for (int s = 0; s < ns; ++s) {
        int q = off[(size_t)s];
        const int qe = off[(size_t)s + 1];
        while (q < qe) {  // chunks of this segment
            const int start = q, e0 = (int)out.ents.size();
            int ne = 0;
            while (q < qe && q - start < cfg.chunk && ne < cfg.entries) {
                int k = q;
                while (k < qe && k - start < cfg.chunk && row[(size_t)k] == row[(size_t)q])
                    ++k;
                out.ents.push_back(make_uint2((unsigned)(q - start) | ((unsigned)(k - q) << 16), (unsigned)row[(size_t)q]));
                ++ne;
                q = k;
            }
            const int len = q - start;
            // nonzero lanes per run: the fewest latency steps -- rounds of runs over the block's groups
            // x (the run's products per lane + its butterfly + ~8 steps of LDS round trips)
            const int mean = (len + ne - 1) / ne;
            int lg = 0, best = 1 << 30;
            for (int l = 0; l <= lg_max; ++l) {
                const int groups = cfg.threads / (GL << l);
                const int rounds = (ne + groups - 1) / groups;
                const int cost = rounds * ((mean + (1 << l) - 1) / (1 << l) + 2 * l + 8);
                if (cost < best) {
                    best = cost;
                    lg = l;
                }
            }
            out.chunks.push_back(make_int4(start, len | (lg << 13) | (seg_n[(size_t)s] << 16), seg_lo[(size_t)s], e0));
        }
    }
    out.ok = (int)out.chunks.size() <= kSlabMmMaxChunks;
}

mspmv_status build_slab_mm_plan(mspmv_handle_s *h, int L, TilePlan &p)
{
    const SlabMmCfg &cfg = slab_mm_cfg(L);
    if (h->m <= 0 || h->nnz <= 0 || (L != 8 && L != 16) || cfg.chunk > 0x1fff || cfg.cols > 0xffff)
        return MSPMV_ERR_UNSUPPORTED;
    const int per_cu = 163840 / (2 * cfg.cols * L * 8 + (cfg.rows + 1) * L * 8 + 10 * cfg.chunk + 8 * cfg.entries + 2048);
    std::vector<int2> hb;
    std::vector<unsigned char> hs;
    long long step = 0;
    mspmv_status st = slab_bounds(h, (long long)std::max(per_cu, 1) * h->num_cus,
                                  (long long)h->m + h->nnz, cfg.rows, p, hb, hs, step);
    if (st != MSPMV_OK)
        return st;
    const int T = p.num_tiles;
    p.lanes = cfg.threads;
    p.tile_items = (int)step;
    p.snap = (int)(step / kSnapDiv);
    std::vector<int> ro, ci;
    std::vector<double> va;
    if ((st = slab_host_matrix(h, ro, ci, va)) != MSPMV_OK)
        return st;
    std::vector<double> oval((size_t)h->nnz);
    std::vector<unsigned short> ocol((size_t)h->nnz);
    std::vector<SlabMmBlockOut> outs((size_t)T);
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < T; ++t) {
        const int2 b0 = hb[(size_t)t], b1 = hb[(size_t)t + 1];
        slab_mm_block(cfg, ro, ci, va, b0.x, b0.y, b1.x, b1.y, oval.data(), ocol.data(), outs[(size_t)t]);
    }
    std::vector<int4> blk((size_t)T), chunks;
    std::vector<uint2> ents;
    long long staged = 0;
    for (int t = 0; t < T; ++t) {
        const SlabMmBlockOut &o = outs[(size_t)t];
        if (!o.ok)  // more segments x chunks than one block's LDS table holds
            return MSPMV_ERR_UNSUPPORTED;
        const int c0 = (int)chunks.size(), ebase = (int)ents.size();
        for (int4 c : o.chunks) {
            c.x += hb[(size_t)t].y;
            c.w += ebase;
            chunks.push_back(c);
        }
        ents.insert(ents.end(), o.ents.begin(), o.ents.end());
        blk[(size_t)t] = make_int4(hb[(size_t)t].x, hb[(size_t)t + 1].x - hb[(size_t)t].x, c0, (int)chunks.size());
        staged += o.staged_cols;
    }
    chunks.push_back(make_int4(0, 0, 0, (int)ents.size()));  // sentinel: the last chunk's entry end
    SlabData *s = new SlabData();
    s->L = L;
    s->cfg = slab_mm_cfg_index(cfg);
    s->num_chunks = (int)chunks.size() - 1;
    s->num_entries = (int)ents.size();
    s->x_bytes_per_nnz = (double)staged * 8.0 * L / (double)h->nnz;
    p.slab = s;
    if ((st = slab_upload(&s->d_blk, blk)) != MSPMV_OK || (st = slab_upload(&s->d_chunk, chunks)) != MSPMV_OK ||
        (st = slab_upload(&s->d_ent, ents)) != MSPMV_OK || (st = slab_upload(&s->d_val, oval, kNnzPad)) != MSPMV_OK ||
        (st = slab_upload(&s->d_col, ocol, kNnzPad)) != MSPMV_OK)
        return st;
    // split rows, their carries and heads (three [T][16] slots, as the tile plans), block modes 255
    p.carry_L = 16;
    if (hipMalloc((void **)&p.d_carry_val, sizeof(double) * (size_t)T * 16 * 3) != hipSuccess ||
        hipMalloc((void **)&p.d_modes[l_index(L)], (size_t)T) != hipSuccess) {
        set_error("column-slab SpMM plan: hipMalloc failed");
        return MSPMV_ERR_HIP;
    }
    if (memset_sync(p.d_modes[l_index(L)], 255, (size_t)T) != hipSuccess) {
        set_error("column-slab SpMM plan: memset failed");
        return MSPMV_ERR_HIP;
    }
    return plan_split_rows(p, hb, hs);
}

}  // namespace mspmv
