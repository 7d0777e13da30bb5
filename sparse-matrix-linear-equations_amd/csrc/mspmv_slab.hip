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
#include <cstring>
#include <string>
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
    // split rows (close_split_rows reads these names)
    const int2 *bounds;
    const unsigned char *split;
    const int4 *fix;
    unsigned *fix_cnt;
    double *carry_val;
    double *head_val;
    double *head_pub;
};

template <bool NT, typename T>
__device__ __forceinline__ T slab_stream(const T *p)
{
    if (NT)
        return __builtin_nontemporal_load(p);
    return *p;
}

template <bool NT>
__global__ __launch_bounds__(kSlabThreads) void k_spmv_slab(SlabArgs a)
{
    constexpr int TB = kSlabThreads;
    constexpr int IPT = kSlabChunk / TB;    // stream items per thread and chunk
    constexpr int EPT = kSlabEntries / TB;  // entries per thread and chunk
    __shared__ double xs[kSlabCols];
    __shared__ double yacc[kSlabRows + 1];
    __shared__ double prod[kSlabChunk];
    __shared__ uint2 sent[kSlabEntries];
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
        const int len = cd.y & 0xffff;
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
    constexpr int XPT = kSlabCols / TB;  // x values per thread and slab
    double xq[XPT];
    auto fetch_x = [&](int slab) {  // a slab of x, into registers (coalesced: lane-consecutive columns)
        const int c0 = slab * kSlabCols;
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
        const int len = cd.y & 0xffff, lg = cd.y >> 16;
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
        const int G = 1 << lg, lane = tid & (G - 1);
        for (int q = tid >> lg; q < ne; q += TB >> lg) {  // uniform within a group
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
    // rows ending in the block; its first row goes to the head slot when it completes a split row
    for (int i = tid; i < nrows; i += TB)
        *(i == 0 && fx.z > 0 ? a.head_val + b : a.y + bd.x + i) = yacc[i];
    if (tail && tid == 0)
        store_sc1(&a.carry_val[b], yacc[nrows]);
    close_split_rows<TB>(a, b, fx, 1, 1);
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
    a.carry_val = plan.d_carry_val;
    a.head_val = plan.d_carry_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    a.head_pub = a.head_val + (size_t)std::max(plan.num_tiles, 1) * plan.carry_L;
    if (plan.num_tiles == 0)
        return hipSuccess;
    if (stream_nt(h))
        hipLaunchKernelGGL(k_spmv_slab<true>, dim3(plan.num_tiles), dim3(kSlabThreads), 0, h->stream, a);
    else
        hipLaunchKernelGGL(k_spmv_slab<false>, dim3(plan.num_tiles), dim3(kSlabThreads), 0, h->stream, a);
    return hipGetLastError();
}

std::string slab_kernel_name(const mspmv_handle_s *h)
{
    return std::string("k_spmv_slab<") + (stream_nt(h) ? "true" : "false") + ">";
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
        e = hipMemset(*d + hsrc.size(), 0, sizeof(T) * pad);
    if (e != hipSuccess) {
        set_error(std::string("column-slab plan upload: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}

// Per block: its nonzeros [n0, n1) in slab-major order (stable within a slab: CSR order), cut into
// chunks of one slab, <= kSlabChunk nonzeros and <= kSlabEntries runs of one row.
struct SlabBlockOut {
    std::vector<int4> chunks;  // entry0 relative to the block
    std::vector<uint2> ents;
    int slabs = 0;
};

static void slab_block(const std::vector<int> &ro, const std::vector<int> &ci, const std::vector<double> &va,
                       int r0, int n0, int r1, int n1, double *oval, unsigned short *ocol, SlabBlockOut &out)
{
    const int cnt = n1 - n0;
    if (cnt <= 0)
        return;
    int smin = 0x7fffffff, smax = -1;
    for (int k = n0; k < n1; ++k) {
        const int s = ci[(size_t)k] / kSlabCols;
        smin = std::min(smin, s);
        smax = std::max(smax, s);
    }
    const int ns = smax - smin + 1;
    std::vector<int> off((size_t)ns + 1, 0);
    for (int k = n0; k < n1; ++k)
        ++off[(size_t)(ci[(size_t)k] / kSlabCols - smin) + 1];
    for (int s = 0; s < ns; ++s) {
        out.slabs += off[(size_t)s + 1] > 0;
        off[(size_t)s + 1] += off[(size_t)s];
    }
    std::vector<int> row((size_t)cnt);  // local row of each reordered nonzero
    std::vector<int> put(off.begin(), off.end() - 1);
    const int rlast = n1 > ro[(size_t)r1] ? r1 : r1 - 1;  // the trailing partial row, when there is one
    for (int r = r0; r <= rlast; ++r) {
        const int k0 = std::max(ro[(size_t)r], n0), k1 = std::min(ro[(size_t)r + 1], n1);
        for (int k = k0; k < k1; ++k) {
            const int s = ci[(size_t)k] / kSlabCols;
            const int q = put[(size_t)(s - smin)]++;
            oval[(size_t)n0 + q] = va[(size_t)k];
            ocol[(size_t)n0 + q] = (unsigned short)(ci[(size_t)k] - s * kSlabCols);
            row[(size_t)q] = r - r0;
        }
    }
    for (int s = 0; s < ns; ++s) {
        int q = off[(size_t)s];
        const int qe = off[(size_t)s + 1];
        while (q < qe) {  // chunks of this slab
            const int start = q, e0 = (int)out.ents.size();
            int ne = 0;
            while (q < qe && q - start < kSlabChunk) {
                int k = q;
                while (k < qe && k - start < kSlabChunk && row[(size_t)k] == row[(size_t)q])
                    ++k;
                if (ne == kSlabEntries)
                    break;
                out.ents.push_back(make_uint2((unsigned)(q - start) | ((unsigned)(k - q) << 16), (unsigned)row[(size_t)q]));
                ++ne;
                q = k;
            }
            const int len = q - start;
            // lanes per run: the fewest latency steps -- rounds of runs over the workgroup x (the run's
            // products per lane + its butterfly + ~8 steps of LDS round trips); the older rule, the
            // smallest G with 4 G >= the mean run, took two rounds where one does (44 -> 40 us, r04w)
            const int mean = (len + ne - 1) / ne;
            int lg = 0, best = 1 << 30;
            for (int l = 0; l <= 6; ++l) {
                const int rounds = (ne + (kSlabThreads >> l) - 1) / (kSlabThreads >> l);
                const int cost = rounds * ((mean + (1 << l) - 1) / (1 << l) + 2 * l + 8);
                if (cost < best) {
                    best = cost;
                    lg = l;
                }
            }
            out.chunks.push_back(make_int4(n0 + start, len | (lg << 16), smin + s, e0));
        }
    }
}

mspmv_status build_slab_plan(mspmv_handle_s *h, TilePlan &p)
{
    if (h->m <= 0 || h->nnz <= 0)
        return MSPMV_ERR_UNSUPPORTED;
    const long long total = (long long)h->m + h->nnz;
    std::vector<int2> hb;
    std::vector<unsigned char> hs;
    int T = 0;
    long long step = 0;
    for (int G = kSlabBlocksPerCu * h->num_cus;; G *= 2) {  // one resident generation; more when rows are short
        if (G > 64 * h->num_cus)
            return MSPMV_ERR_UNSUPPORTED;
        step = (total + G - 1) / G;
        if (step > (1LL << 30))
            return MSPMV_ERR_UNSUPPORTED;
        T = (int)((total + step - 1) / step);
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
        if (rows_max <= kSlabRows)
            break;
    }
    p.lanes = kSlabThreads;
    p.tile_items = (int)step;
    p.snap = (int)(step / kSnapDiv);
    p.num_tiles = T;

    // the matrix on the host, reordered block by block
    std::vector<int> ro((size_t)h->m + 1), ci((size_t)h->nnz);
    std::vector<double> va((size_t)h->nnz);
    hipError_t e = hipMemcpy(ro.data(), h->d_row_offsets, sizeof(int) * ro.size(), hipMemcpyDeviceToHost);
    if (e == hipSuccess)
        e = hipMemcpy(ci.data(), h->d_cols, sizeof(int) * ci.size(), hipMemcpyDeviceToHost);
    if (e == hipSuccess)
        e = hipMemcpy(va.data(), h->d_vals, sizeof(double) * va.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        set_error(std::string("column-slab plan: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    std::vector<double> oval((size_t)h->nnz);
    std::vector<unsigned short> ocol((size_t)h->nnz);
    std::vector<SlabBlockOut> outs((size_t)T);
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < T; ++t) {
        const int2 b0 = hb[(size_t)t], b1 = hb[(size_t)t + 1];
        slab_block(ro, ci, va, b0.x, b0.y, b1.x, b1.y, oval.data(), ocol.data(), outs[(size_t)t]);
    }
    SlabData *s = new SlabData();
    std::vector<int4> blk((size_t)T), chunks;
    std::vector<uint2> ents;
    long long staged = 0;
    for (int t = 0; t < T; ++t) {
        const SlabBlockOut &o = outs[(size_t)t];
        const int c0 = (int)chunks.size(), ebase = (int)ents.size();
        for (int4 c : o.chunks) {
            c.w += ebase;
            chunks.push_back(c);
        }
        ents.insert(ents.end(), o.ents.begin(), o.ents.end());
        blk[(size_t)t] = make_int4(hb[(size_t)t].x, hb[(size_t)t + 1].x - hb[(size_t)t].x, c0, (int)chunks.size());
        if ((int)o.chunks.size() > kSlabMaxChunks) {  // more slabs than one block's LDS table holds
            delete s;
            return MSPMV_ERR_UNSUPPORTED;
        }
        staged += (long long)o.slabs * kSlabCols * 8;
    }
    chunks.push_back(make_int4(0, 0, 0, (int)ents.size()));  // sentinel: the last chunk's entry end
    s->num_chunks = (int)chunks.size() - 1;
    s->num_entries = (int)ents.size();
    s->x_bytes_per_nnz = (double)staged / (double)h->nnz;
    p.slab = s;
    mspmv_status st;
    if ((st = slab_upload(&s->d_blk, blk)) != MSPMV_OK || (st = slab_upload(&s->d_chunk, chunks)) != MSPMV_OK ||
        (st = slab_upload(&s->d_ent, ents)) != MSPMV_OK || (st = slab_upload(&s->d_val, oval, kNnzPad)) != MSPMV_OK ||
        (st = slab_upload(&s->d_col, ocol, kNnzPad)) != MSPMV_OK)
        return st;
    // split rows, their carries and heads (three [T][16] slots, as the tile plans), tile modes 255
    p.carry_L = 16;
    if (hipMalloc((void **)&p.d_carry_val, sizeof(double) * (size_t)T * 16 * 3) != hipSuccess ||
        hipMalloc((void **)&p.d_modes[0], (size_t)T) != hipSuccess) {
        set_error("column-slab plan: hipMalloc failed");
        return MSPMV_ERR_HIP;
    }
    if (hipMemset(p.d_modes[0], 255, (size_t)T) != hipSuccess) {
        set_error("column-slab plan: memset failed");
        return MSPMV_ERR_HIP;
    }
    return plan_split_rows(p, hb, hs);
}

}  // namespace mspmv
