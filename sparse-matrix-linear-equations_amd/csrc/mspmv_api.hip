// mspmv_api.hip -- the C-ABI (include/mspmv.h): matrix handles, tile plans, SpMV/SpMM
// entry points, and the CG drivers.  Host C++17 over the HIP runtime.
#include "mspmv_internal.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace mspmv {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }

hipError_t launch_flush(void *p, size_t bytes, hipStream_t s, bool fresh);

}  // namespace mspmv

unsigned long long mspmv_next_generation()
{
    static std::atomic<unsigned long long> next{1};
    return next.fetch_add(1, std::memory_order_relaxed);
}

using namespace mspmv;

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                          \
            return (_e == hipErrorOutOfMemory) ? MSPMV_ERR_OOM : MSPMV_ERR_HIP;                    \
        }                                                                                          \
    } while (0)

#define ST_TRY(expr)                                                                               \
    do {                                                                                           \
        mspmv_status _s = (expr);                                                                  \
        if (_s != MSPMV_OK)                                                                        \
            return _s;                                                                             \
    } while (0)

static mspmv_status invalid(const std::string &msg)
{
    set_error(msg);
    return MSPMV_ERR_INVALID;
}

template <typename T>
static mspmv_status dev_alloc(T **p, size_t count)
{
    *p = nullptr;
    if (count == 0)
        count = 1;
    hipError_t e = hipMalloc((void **)p, count * sizeof(T));
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc(") + std::to_string(count * sizeof(T)) + " B): " + hipGetErrorString(e));
        *p = nullptr;
        return e == hipErrorOutOfMemory ? MSPMV_ERR_OOM : MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}

template <typename T>
static void dev_free(T *&p)
{
    if (p)
        (void)hipFree((void *)p);
    p = nullptr;
}

__global__ void k_check_cols(const int *__restrict__ cols, long long nnz, int n, int *bad)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += (long long)gridDim.x * blockDim.x) {
        const int c = cols[i];
        if (c < 0 || c >= n)
            atomicOr(bad, 1);
    }
}

static void free_plan(TilePlan &p)
{
    dev_free(p.d_bounds);
    dev_free(p.d_split);
    for (auto &m : p.d_modes)
        dev_free(m);
    dev_free(p.d_fix);
    dev_free(p.d_fix_cnt);
    dev_free(p.d_carry_val);
    dev_free(p.d_colbase);
    dev_free(p.d_cols16);
    dev_free(p.d_dict);
    dev_free(p.d_ndict);
    dev_free(p.d_idx16);
    dev_free(p.d_blk);
    free_slab(p.slab);
    p.slab = nullptr;
    free_dia(p.dia);
    p.dia = nullptr;
}

// Build (once) the tile plan for L right-hand sides, validating on the host every bound the
// kernels rely on (monotone boundaries, <= 1.25 * tile_items merge items per tile) before any
// tile kernel can run on it.
static mspmv_status build_plan(mspmv_handle_s *h, int L, const TilePlan **out, int lanes = 0,
                               const std::vector<int2> *fixed = nullptr);

// The in-tile reduction modes of a plan for L right-hand sides, built on first use.
static mspmv_status ensure_modes(mspmv_handle_s *h, TilePlan &p, int L)
{
    unsigned char *&m = p.d_modes[l_index(L)];
    if (m)
        return MSPMV_OK;
    mspmv_status st = dev_alloc(&m, (size_t)std::max(p.num_tiles, 1));
    if (st != MSPMV_OK)
        return st;
    hipError_t e = launch_tile_modes(h->d_row_offsets, p.d_bounds, p.d_split, p.num_tiles, L, m, h->stream, p.lanes);
    if (e == hipSuccess)
        e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        set_error(std::string("tile modes: ") + hipGetErrorString(e));
        dev_free(m);
        m = nullptr;
        return MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}

static mspmv_status spmv_plan(mspmv_handle_s *h, const TilePlan **out);
static mspmv_status spmm_slab_decide(mspmv_handle_s *h, int L);
static mspmv_status spmv_runs_decide(mspmv_handle_s *h, const TilePlan *wg);

// Offset-window plan (mspmv_dia.hip) for the plain SpMV / SpMM of every width and the split CG's SpMM:
// taken when every 64-row window of the matrix lists its columns at <= kDiaMaxK common offsets col - row
// and the nonzeros fill >= kDiaAutoFill of the windows' rows x offsets overall (>= kDiaWindowFill in each
// window): structured-grid stencils, whose boundary planes miss a third of the offsets.  MSPMV_DIA=0
// never, =1 whenever every window fits at any fill; read at each handle's decision.
constexpr double kDiaAutoFill = 0.85;
constexpr double kDiaWindowFill = 0.3;
static int dia_switch()
{
    const char *e = getenv("MSPMV_DIA");
    return e && *e ? (atoi(e) != 0 ? 1 : 0) : -1;
}

static mspmv_status dia_decide(mspmv_handle_s *h)
{
    h->dia = 0;
    const int sw = dia_switch();
    if (sw == 0)
        return MSPMV_OK;
    TilePlan p;
    const mspmv_status st = build_dia_plan(h, p, sw == 1 ? 0.0 : kDiaAutoFill, sw == 1 ? 0.0 : kDiaWindowFill);
    if (st != MSPMV_OK) {
        free_plan(p);
        if (sw < 0 || st == MSPMV_ERR_UNSUPPORTED) {  // optional plan: the tile plans stay
            set_error("");
            (void)hipGetLastError();
            return MSPMV_OK;
        }
        return st;
    }
    h->plans.emplace(kDiaPlanKey, p);
    h->dia = 1;
    return MSPMV_OK;
}

// The L-wide products take the windows too unless MSPMV_DIA_SPMM=0: with the offsets taken run by run
// through LDS they beat the merge tiles at every width on the stencil shapes (nlpkkt120 size L = 2 / 4 / 8
// / 16: 268 / 295 / 372 / 677 us against 336 / 375 / 441 / 753; parabolic_fem shape 10.5 / 13.5 / 19.2 /
// 37 against 15.4 / 16 / 21.8 / 37.5 us; configs[4]'s CG 0.786 -> 0.704 ms per iteration, r05x).
bool mspmv::dia_spmm_enabled()
{
    const char *e = getenv("MSPMV_DIA_SPMM");
    return !(e && *e && atoi(e) == 0);
}

// The offset-window plan for a product of width L when the handle takes one (deciding on first use),
// else null.
static mspmv_status dia_plan(mspmv_handle_s *h, const TilePlan **out, int L = 1)
{
    *out = nullptr;
    if (L > 1 && !dia_spmm_enabled())
        return MSPMV_OK;
    if (h->dia < 0)
        ST_TRY(dia_decide(h));
    if (h->dia == 1)
        *out = &h->plans.find(kDiaPlanKey)->second;
    return MSPMV_OK;
}

// plain: the caller runs the plain product (y = A x / Y = A X), whose single-RHS form may take a
// one-wave plan of its own (spmv_plan); CG, dot-mode and sharded callers use the workgroup plan.
bool mspmv::host_pattern_resident(const mspmv_handle_s *h) { return h->pat_ro_ext || !h->pat_ro.empty(); }

mspmv_status mspmv::host_pattern(mspmv_handle_s *h, const int **ro, const int **ci)
{
    if (h->pat_ro_ext) {
        *ro = h->pat_ro_ext;
        *ci = h->pat_ci_ext;
        return MSPMV_OK;
    }
    if (h->pat_ro.empty()) {
        std::vector<int> r((size_t)h->m + 1), c((size_t)std::max(h->nnz, 1));
        HIP_TRY(hipMemcpy(r.data(), h->d_row_offsets, sizeof(int) * r.size(), hipMemcpyDeviceToHost));
        if (h->nnz)
            HIP_TRY(hipMemcpy(c.data(), h->d_cols, sizeof(int) * (size_t)h->nnz, hipMemcpyDeviceToHost));
        h->pat_ro.swap(r);
        h->pat_ci.swap(c);
    }
    *ro = h->pat_ro.data();
    *ci = h->pat_ci.data();
    return MSPMV_OK;
}

static mspmv_status get_plan(mspmv_handle_s *h, int L, const TilePlan **out, bool plain = false)
{
    std::unique_ptr<PatternScope> scope;  // the plain product's decisions share one host copy of the pattern
    if (plain)
        scope.reset(new PatternScope(h));
    if (plain) {
        const TilePlan *dp = nullptr;
        ST_TRY(dia_plan(h, &dp, L));
        if (dp) {
            *out = dp;
            return MSPMV_OK;
        }
    }
    if (plain && L == 1)
        return spmv_plan(h, out);
    if (L > 1 && spmm_blk_enabled()) {
        // a matrix of node blocks only (every single-RHS tile a register run tile: FEM node rows)
        // multiplies L columns on that plan with k_spmm_blk -- one panel-row gather per (run,
        // column) -- instead of its own L-wide merge tiles
        auto one = h->plans.find(plan_key(1));
        if (one != h->plans.end() && one->second.d_blk && one->second.num_tiles_reg == one->second.num_tiles) {
            if (plain) {  // the plain product on the run-balanced plan, as the plain SpMV (spmv_runs_decide)
                if (h->spmv_runs < 0)
                    ST_TRY(spmv_runs_decide(h, &one->second));
                auto rp = h->spmv_runs == 1 ? h->plans.find(kRunPlanKey) : h->plans.end();
                if (rp != h->plans.end()) {
                    ST_TRY(ensure_modes(h, rp->second, L));
                    *out = &rp->second;
                    return MSPMV_OK;
                }
            }
            ST_TRY(ensure_modes(h, one->second, L));
            *out = &one->second;
            return MSPMV_OK;
        }
    }
    if (plain && (L == 8 || L == 16)) {
        // the plain L-wide product on a column-slab plan when one was chosen (spmm_slab_decide, after the
        // node-block check: FEM matrices keep k_spmm_blk)
        const TilePlan *tp = nullptr;
        ST_TRY(get_plan(h, L, &tp, false));
        if (tp->d_blk && tp->num_tiles_reg == tp->num_tiles && spmm_blk_enabled()) {
            *out = tp;
            return MSPMV_OK;
        }
        if (h->spmm_slab[l_index(L)] < 0)
            ST_TRY(spmm_slab_decide(h, L));
        auto it = h->spmm_slab[l_index(L)] == 1 ? h->plans.find(slab_mm_key(L)) : h->plans.end();
        *out = it != h->plans.end() ? &it->second : tp;
        return MSPMV_OK;
    }
    const int key = plan_key(L);
    auto it = h->plans.find(key);
    if (it == h->plans.end()) {
        const TilePlan *np = nullptr;
        mspmv_status st = build_plan(h, L, &np);
        if (st != MSPMV_OK)
            return st;
        it = h->plans.find(key);
    }
    mspmv_status st = ensure_modes(h, it->second, L);
    if (st != MSPMV_OK)
        return st;
    *out = &it->second;
    return MSPMV_OK;
}

namespace mspmv {
// Split rows of a plan (boundaries hb, split flags hs; p.num_tiles set): the tiles t0 .. t1 - 1 that
// end inside one row carry into the tile t1 that completes it (the first tile after them with no
// carry into the same row; the last tile always ends on m) -- TilePlan::d_fix / d_fix_cnt, closed by
// close_split_rows.  No arrays when nothing is split.
mspmv_status plan_split_rows(TilePlan &p, const std::vector<int2> &hb, const std::vector<unsigned char> &hs)
{
    const int T = p.num_tiles;
    std::vector<int4> fix((size_t)T, make_int4(-1, 0, 0, 0));
    int carries = 0;
    for (int t = 0; t < T;) {
        if (!hs[(size_t)t + 1]) {
            ++t;
            continue;
        }
        const int t0 = t;
        while (t < T && hs[(size_t)t + 1] && hb[(size_t)t + 1].x == hb[(size_t)t0 + 1].x)
            ++t;
        if (t >= T) {
            set_error("tile plan: split row past the last tile");
            return MSPMV_ERR_INVALID;
        }
        for (int u = t0; u < t; ++u) {
            fix[(size_t)u].x = t;
            fix[(size_t)u].y = t - t0;
        }
        fix[(size_t)t].z = t - t0;
        carries += t - t0;
    }
    p.num_carries = carries;
    if (carries == 0)
        return MSPMV_OK;
    mspmv_status st;
    if ((st = dev_alloc(&p.d_fix, (size_t)T)) != MSPMV_OK || (st = dev_alloc(&p.d_fix_cnt, (size_t)T)) != MSPMV_OK)
        return st;
    hipError_t e = hipMemcpy(p.d_fix, fix.data(), sizeof(int4) * fix.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = memset_sync(p.d_fix_cnt, 0, sizeof(unsigned) * T);
    if (e != hipSuccess) {
        set_error(std::string("tile plan upload: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}
}  // namespace mspmv

static mspmv_status build_plan(mspmv_handle_s *h, int L, const TilePlan **out, int lanes,
                               const std::vector<int2> *fixed)
{
    // lanes: 64 builds the one-wave single-RHS plan (tile = 64 x items per thread, keyed by minus
    // that size); 0 the default plan for L.  fixed: the run-balanced single-RHS plan's boundaries
    // (whole rows, no split; spmv_run_plan), keyed kRunPlanKey -- run by the node-block SpMV only,
    // whose tiles have no LDS item bound
    const bool onewave = L == 1 && lanes == 64;
    const int tile = onewave ? 64 * spmv_items_per_thread() : tile_items_for(L);
    TilePlan p;
    p.lanes = onewave ? 64 : kBlock;
    const long long total = (long long)h->m + h->nnz;
    int step = tile, snap = tile / kSnapDiv;
    if (L == 1 && !onewave) {
        // A grid a few tiles over a whole number of resident generations of workgroups takes one
        // tile lifetime more (the parabolic_fem shape: 2,052 tiles on 2,048 slots).  Stretch the
        // tiles into the snap slack so they fit one generation fewer: MAXI (step + snap) is
        // unchanged, rows entered by more than the smaller snap distance stay split (carries,
        // close_split_rows).  (Measured against nominal tiles in round 3: kept.)
        const long long slots = (long long)h->num_cus * spmv_tile_blocks_per_cu();
        const long long t0 = (total + tile - 1) / tile;
        // Below one generation (cant: 1,988 tiles on 2,048 slots; rma10: 1,183) the nominal tiles stay: cut
        // into exactly one tile per slot they measured the same (r06e).
        if (slots > 0 && t0 > slots) {
            const long long fewer = (t0 + slots - 1) / slots - 1;  // generations after stretching
            const long long fit = (total + fewer * slots - 1) / (fewer * slots);
            if (fit + 16 <= tile + tile / kSnapDiv) {
                step = (int)fit;
                snap = tile + tile / kSnapDiv - step;  // >= 16
            }
        }
    }
    if (fixed) {
        int most = 0;
        for (size_t t = 0; t + 1 < fixed->size(); ++t)
            most = std::max(most, ((*fixed)[t + 1].x - (*fixed)[t].x) + ((*fixed)[t + 1].y - (*fixed)[t].y));
        step = most;
        snap = 0;
    }
    p.tile_items = step;
    p.snap = snap;
    p.num_tiles = fixed ? (int)fixed->size() - 1 : (int)((total + step - 1) / step);
    const int T = p.num_tiles;
    mspmv_status st;
    if ((st = dev_alloc(&p.d_bounds, (size_t)T + 1)) != MSPMV_OK ||
        (st = dev_alloc(&p.d_split, (size_t)T + 1)) != MSPMV_OK ||
        (st = dev_alloc(&p.d_carry_val, (size_t)std::max(T, 1) * 16 * 3)) != MSPMV_OK) {  // carries, heads x 2
        free_plan(p);
        return st;
    }
    p.carry_L = 16;
    auto fail = [&](mspmv_status s) {
        free_plan(p);
        return s;
    };
    hipError_t e = hipSuccess;
    if (fixed) {
        e = hipMemcpyAsync(p.d_bounds, fixed->data(), sizeof(int2) * (T + 1), hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess)
            e = hipMemsetAsync(p.d_split, 0, (size_t)T + 1, h->stream);
    } else {
        e = launch_merge_coords(h->d_row_offsets, h->m, h->nnz, step, T, p.d_bounds, h->stream);
        if (e == hipSuccess)
            e = launch_snap(h->d_row_offsets, h->m, p.d_bounds, p.d_split, T, p.snap, h->stream);
    }
    std::vector<int2> hb((size_t)T + 1);
    std::vector<unsigned char> hs((size_t)T + 1);
    if (e == hipSuccess)
        e = hipMemcpyAsync(hb.data(), p.d_bounds, sizeof(int2) * (T + 1), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(hs.data(), p.d_split, T + 1, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        set_error(std::string("tile plan: ") + hipGetErrorString(e));
        return fail(MSPMV_ERR_HIP);
    }
    const int maxi = fixed ? step : tile + tile / kSnapDiv;
    if (hb[0].x != 0 || hb[0].y != 0 || hb[T].x != h->m || hb[T].y != h->nnz) {
        set_error("tile plan: bad end boundaries");
        return fail(MSPMV_ERR_INVALID);
    }
    for (int t = 0; t < T; ++t) {
        const int nr = hb[t + 1].x - hb[t].x, nz = hb[t + 1].y - hb[t].y;
        if (nr < 0 || nz < 0 || nr + nz > maxi) {
            set_error("tile plan: tile " + std::to_string(t) + " violates the merge bound");
            return fail(MSPMV_ERR_INVALID);
        }
    }
    if ((st = plan_split_rows(p, hb, hs)) != MSPMV_OK)
        return fail(st);
    // the single-RHS kernels' 16-bit column stream; keyed on the tile size, not L, because the
    // L = 2 SpMM shares the single-RHS plan.  (The SpMM itself keeps int32 columns: it is gather
    // bound, and the 16-bit stream measured 0% at L = 4/8 and 7% slower at L = 16.)
    const bool single = L == 1;  // a single-RHS plan
    if (single && T > 0 && h->nnz > 0) {
        if ((st = dev_alloc(&p.d_colbase, (size_t)T)) != MSPMV_OK ||
            (st = dev_alloc(&p.d_cols16, (size_t)h->nnz + kNnzPad)) != MSPMV_OK)
            return fail(st);
        e = hipMemsetAsync(p.d_cols16, 0, sizeof(unsigned short) * ((size_t)h->nnz + kNnzPad), h->stream);
        if (e == hipSuccess)
            e = launch_pack_cols16(h->d_cols, p.d_bounds, T, p.d_colbase, p.d_cols16, h->stream);
        std::vector<int> hbase((size_t)T);
        if (e == hipSuccess)
            e = hipMemcpyAsync(hbase.data(), p.d_colbase, sizeof(int) * T, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) {
            set_error(std::string("16-bit columns: ") + hipGetErrorString(e));
            return fail(MSPMV_ERR_HIP);
        }
        for (int b : hbase)
            p.num_tiles16 += b >= 0;
        if (p.num_tiles16 == 0) {  // nothing fits: keep the plan on int32 columns only
            dev_free(p.d_colbase);
            dev_free(p.d_cols16);
            p.d_colbase = nullptr;
            p.d_cols16 = nullptr;
        }
    }
    // node blocks: single-RHS plan on the 16-bit stream only (the runs' pattern columns are read there)
    if (single && !onewave && p.d_cols16 && spmv_blocks_enabled()) {
        if ((st = dev_alloc(&p.d_blk, (size_t)T * kBlkPerTile)) != MSPMV_OK)
            return fail(st);
        e = launch_build_blocks(h->d_row_offsets, h->d_cols, p.d_bounds, p.d_split, p.d_colbase, T, p.d_blk,
                                h->stream, kBlkPlanChunks);
        std::vector<uint4> hd((size_t)T * kBlkPerTile);
        if (e == hipSuccess)
            e = hipMemcpyAsync(hd.data(), p.d_blk, sizeof(uint4) * hd.size(), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) {
            set_error(std::string("node blocks: ") + hipGetErrorString(e));
            return fail(MSPMV_ERR_HIP);
        }
        p.h_blk_reg.assign((size_t)T, 0);
        int maxnd = 0, maxh = 0;
        std::vector<unsigned char> reg((size_t)T, 0);
        for (int t = 0; t < T; ++t) {
            const uint4 *d = &hd[(size_t)t * kBlkPerTile];
            const int nd = (int)((d[0].y >> 8) & 255u);
            if (nd == 0)
                continue;
            ++p.num_tiles_blk;
            maxnd = std::max(maxnd, nd);
            for (int i = 0; i < nd; ++i)
                maxh = std::max(maxh, (int)(d[i].y & 15u));
            bool one = true;  // the kernels' own test: every chunk starts at pattern column 0
            for (int i = 0; i < nd; ++i)
                one = one && ((d[i].x >> 16) & 255u) == 0;
            reg[(size_t)t] = one;
            p.num_tiles_reg += one;
        }
        // the plain SpMV runs the column-pair node-block kernel (its register fallback taking the
        // other tiles) when most tiles are register run tiles; otherwise k_spmv_tile, whose register
        // path takes the run tiles of one round (<= kBlkTileChunks chunks)
        p.blk_spmv = p.num_tiles_reg > 0 && 2LL * p.num_tiles_reg >= T;
        for (int t = 0; t < T; ++t) {
            const int nd = (int)((hd[(size_t)t * kBlkPerTile].y >> 8) & 255u);
            p.h_blk_reg[(size_t)t] = p.blk_spmv || (reg[(size_t)t] && nd <= kBlkTileChunks);
            p.blk_two_rounds += nd > kBlkTileChunks;
        }
        dev_free(p.d_blk);
        p.d_blk = nullptr;
        p.blk_rows_max = maxh > 0 ? maxh : 8;
        if (p.num_tiles_blk > 0) {  // repack at the smallest stride that holds every tile's set
            p.blk_stride = maxnd <= 16 ? 16 : maxnd <= 32 ? 32 : 64;
            std::vector<uint4> packed((size_t)T * p.blk_stride, make_uint4(0u, 0u, 0u, 0u));
            for (int t = 0; t < T; ++t)
                for (int i = 0, nd = (int)((hd[(size_t)t * kBlkPerTile].y >> 8) & 255u); i < nd; ++i)
                    packed[(size_t)t * p.blk_stride + i] = hd[(size_t)t * kBlkPerTile + i];
            if ((st = dev_alloc(&p.d_blk, packed.size())) != MSPMV_OK)
                return fail(st);
            if (hipMemcpy(p.d_blk, packed.data(), sizeof(uint4) * packed.size(), hipMemcpyHostToDevice) != hipSuccess) {
                set_error("node blocks: upload failed");
                return fail(MSPMV_ERR_HIP);
            }
        }
    }
    // multi-RHS: only the L = 16 plan (k_spmm_tile's DICT path runs at L = 16 only); not the run-
    // balanced plan (its kernel gathers x directly)
    const bool multi = !single;
    const bool want = fixed ? false : multi ? spmm_dict_max(L) > 0 : true;
    if (T > 0 && h->nnz > 0 && want) {
        if ((st = dev_alloc(&p.d_dict, (size_t)h->nnz + kNnzPad)) != MSPMV_OK ||
            (st = dev_alloc(&p.d_ndict, (size_t)T)) != MSPMV_OK ||
            (st = dev_alloc(&p.d_idx16, (size_t)h->nnz + kNnzPad)) != MSPMV_OK)
            return fail(st);
        e = hipMemsetAsync(p.d_dict, 0, sizeof(int) * ((size_t)h->nnz + kNnzPad), h->stream);
        if (e == hipSuccess)
            e = hipMemsetAsync(p.d_idx16, 0, sizeof(unsigned short) * ((size_t)h->nnz + kNnzPad), h->stream);
        if (e == hipSuccess)
            e = launch_build_dict(h->d_cols, p.d_bounds, T, maxi, p.d_dict, p.d_ndict, p.d_idx16, h->stream, multi, L);
        std::vector<int> hnd((size_t)T);
        if (e == hipSuccess)
            e = hipMemcpyAsync(hnd.data(), p.d_ndict, sizeof(int) * T, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) {
            set_error(std::string("column dictionaries: ") + hipGetErrorString(e));
            return fail(MSPMV_ERR_HIP);
        }
        for (int v : hnd)
            p.num_tiles_dict += v > 0;
        if (p.num_tiles_dict == 0) {  // no tile takes one: drop the arrays, the kernel skips the test
            dev_free(p.d_dict);
            dev_free(p.d_ndict);
            dev_free(p.d_idx16);
            p.d_dict = nullptr;
            p.d_ndict = nullptr;
            p.d_idx16 = nullptr;
        }
    }
    auto res = h->plans.emplace(fixed ? kRunPlanKey : p.lanes == 64 ? -tile : plan_key(L), p);  // one-wave: negative keys
    *out = &res.first->second;
    return MSPMV_OK;
}

// The plan the plain single-RHS SpMV runs on.  Decided once per handle on first use: a matrix
// whose workgroup plan is mostly merge-walk tiles (row lengths uneven inside most tiles: skewed,
// power-law rows) runs one-wave tiles instead (k_spmv_tile<.., 64>: 512 merge items, wave
// barriers only), so a tile's hub-row closing and its walkers' latencies stall one wave, not four.
// Measured on the skewed pwtk-sized variant 100.1 -> 78.3 us; on row-group plans (banded, FEM,
// stencils) one-wave tiles lost 1-15 % (r03r), so those keep the workgroup plan.
// Column-slab plan (mspmv_slab.hip) for the plain SpMV: MSPMV_SPMV_SLAB=1 takes it for every matrix
// it can hold, =0 never; by default a matrix takes it when its workgroup plan gathers through column
// dictionaries on most tiles (x gathers line-bound: scattered columns) and the slab plan stages at
// most kSlabAutoBytes of x per nonzero (the columns of a block lie in a few slabs: a band, not the
// whole width).  Scattered band at pwtk size: 58.9 -> 40 us per launch (r04w).
constexpr double kSlabAutoBytes = 16.0;
// ... and its blocks hold >= kSlabAutoNnzPerBlock nonzeros: a block's fixed costs (its descriptors,
// yacc, the first slab, the write-out) then spread over >= 6 chunks.  cant (7,800 per block) took the
// slab plan without it and lost: 0.396 against 0.43 on tiles (r04x).
constexpr double kSlabAutoNnzPerBlock = 12288.0;
constexpr bool kSlabAuto = true;
static int slab_switch()  // read at each handle's decision (tests set it per matrix); 2: column groups
{
    const char *e = getenv("MSPMV_SPMV_SLAB");
    return e && *e ? (atoi(e) >= 2 && atoi(e) <= 4 ? atoi(e) : atoi(e) != 0 ? 1 : 0) : -1;
}

// Most of the workgroup plan's tiles are merge walks (row lengths uneven inside most tiles: skewed,
// power-law rows): the one-wave plan's and the sliced-ELL plan's test.
static mspmv_status mostly_walks(const TilePlan *wg, bool *out)
{
    *out = false;
    if (wg->lanes != kBlock || wg->num_tiles < 64 || wg->d_blk)
        return MSPMV_OK;
    std::vector<unsigned char> hm((size_t)wg->num_tiles);
    HIP_TRY(hipMemcpy(hm.data(), wg->d_modes[0], hm.size(), hipMemcpyDeviceToHost));
    long long walk = 0;
    for (unsigned char v : hm)
        walk += v == 0;
    *out = 2 * walk >= (long long)wg->num_tiles;
    return MSPMV_OK;
}

// Skewed rows (mostly merge walks) with at least kSellAutoNnzPerBlock nonzeros per column-group block
// take the sliced-ELL plan (k_spmv_sell) when it stages at most kSlabAutoBytes of x per nonzero: the
// power-law variant at pwtk size 80 -> 55 us per launch (r05ao-r05as); smaller skewed matrices keep
// the one-wave tiles (their blocks would be a few chunks of work each).
constexpr double kSellAutoNnzPerBlock = 12288.0;

static mspmv_status spmv_slab_decide(mspmv_handle_s *h, const TilePlan *wg)
{
    const int sw = slab_switch();
    bool cand = sw >= 1;
    if (sw < 0 && kSlabAuto)
        cand = wg->lanes == kBlock && wg->num_tiles >= 64 && !wg->blk_spmv && 2 * wg->num_tiles_dict >= wg->num_tiles;
    h->spmv_slab = 0;
    if (!cand && sw < 0 && kSlabAuto) {  // skewed rows: the sliced-ELL plan, when it pays
        bool skew = false;
        ST_TRY(mostly_walks(wg, &skew));
        if (skew && (double)h->nnz >= kSellAutoNnzPerBlock * h->num_cus) {
            TilePlan p;
            const mspmv_status st = build_slab_plan(h, p, kSellAutoNnzPerBlock, 2, true);
            if (st == MSPMV_OK && p.slab->x_bytes_per_nnz <= kSlabAutoBytes) {
                h->plans.emplace(kSlabPlanKey, p);
                h->spmv_slab = 1;
                return MSPMV_OK;
            }
            free_plan(p);  // optional plan: any failure keeps the tiles
            set_error("");
            (void)hipGetLastError();
        }
        return MSPMV_OK;
    }
    if (!cand)
        return MSPMV_OK;
    if (sw < 0 && (double)h->nnz >= kSlabAutoNnzPerBlock * kSlabBlocksPerCu * h->num_cus) {
        // line-bound gathers over a band (rows whose columns scatter within a window of a few slabs): the
        // sliced-ELL kernel with ONE column group -- whole-row blocks, each staging only its band's slabs --
        // before the merge-path slab blocks: bench's scattered band 41.5-42.0 -> 36.3 us (r06r / r06t, with slabs
        // cut from each block's first column; with the power-law variant's 4 groups three of every four blocks of
        // a band would be empty: 118 us, r05).  At the slab blocks' own size bar (cant, 4 M nonzeros, stays on the
        // tiles: 14.2 us on these against 13.9)
        TilePlan q;
        const mspmv_status st = build_slab_plan(h, q, kSellAutoNnzPerBlock, 2, true, 1);
        if (st == MSPMV_OK && q.slab->x_bytes_per_nnz <= kSlabAutoBytes) {
            h->plans.emplace(kSlabPlanKey, q);
            h->spmv_slab = 1;
            return MSPMV_OK;
        }
        free_plan(q);  // optional plan: any failure keeps trying the slab blocks, then the tiles
        set_error("");
        (void)hipGetLastError();
    }
    TilePlan p;
    // automatic: the blocks-per-nonzero test runs inside the builder before anything past the bounds is
    // copied or allocated, and any failure (an allocation near capacity included) means "no slab plan":
    // the workgroup plan is ready, so the product must not fail for an optional plan
    const mspmv_status st = build_slab_plan(h, p, sw < 0 ? kSlabAutoNnzPerBlock : 0.0, sw == 2 ? 1 : sw == 4 ? 2 : 0, sw >= 2);
    if (st != MSPMV_OK && (sw < 0 || st == MSPMV_ERR_UNSUPPORTED)) {
        free_plan(p);
        set_error("");
        (void)hipGetLastError();
        return MSPMV_OK;
    }
    if (st != MSPMV_OK) {
        free_plan(p);
        return st;
    }
    if (sw < 0 && p.slab->x_bytes_per_nnz > kSlabAutoBytes) {
        free_plan(p);
        return MSPMV_OK;
    }
    h->plans.emplace(kSlabPlanKey, p);
    h->spmv_slab = 1;
    return MSPMV_OK;
}

// Column-slab plan for the plain SpMM of width L = 8 or 16 (mspmv_slab.hip k_spmm_slab): MSPMV_SPMM_SLAB=1
// takes it for every matrix it can hold, =0 never; by default a matrix whose L-wide product runs the
// merge tiles (not the node-block SpMM) takes it when the plan stages at most kSlabMmAutoFrac of the
// panel bytes the tiles gather (L x 8 B per nonzero): a band or a stencil, whose blocks reuse each staged
// panel row several times, not scattered columns.
constexpr double kSlabMmAutoFrac = 0.5;
constexpr long long kSlabMmAutoMinNnz = 1 << 20;
// Off by default until it beats the L-wide tiles on the BASELINE shapes: cant-shaped L = 16 48 vs 27 us,
// nlpkkt120-size L = 8 715 vs 460 us (r05f).
constexpr bool kSlabMmAuto = false;
static int slab_mm_switch()
{
    const char *e = getenv("MSPMV_SPMM_SLAB");
    return e && *e ? (atoi(e) != 0 ? 1 : 0) : -1;
}

static mspmv_status spmm_slab_decide(mspmv_handle_s *h, int L)
{
    int &dec = h->spmm_slab[l_index(L)];
    const int sw = slab_mm_switch();
    dec = 0;
    if (!(sw == 1 || (sw < 0 && kSlabMmAuto && h->nnz >= kSlabMmAutoMinNnz)))
        return MSPMV_OK;
    TilePlan p;
    const mspmv_status st = build_slab_mm_plan(h, L, p);
    if (st != MSPMV_OK && (sw < 0 || st == MSPMV_ERR_UNSUPPORTED)) {  // optional: never fail the product
        free_plan(p);
        set_error("");
        (void)hipGetLastError();
        return MSPMV_OK;
    }
    if (st != MSPMV_OK) {
        free_plan(p);
        return st;
    }
    if (sw < 0 && p.slab->x_bytes_per_nnz > kSlabMmAutoFrac * 8.0 * L) {
        free_plan(p);
        return MSPMV_OK;
    }
    h->plans.emplace(slab_mm_key(L), p);
    dec = 1;
    return MSPMV_OK;
}

// Run-balanced plan for the node-block SpMV / SpMM (round 5).  The merge-path tiles of a node-block plan hold
// ~2,048 items: 6-7 runs on the pwtk shape, one round of k_spmv_blk's eight half-wave run slots.  On
// imperfect FEM (odd-size nodes, off-pattern rows: more, shorter runs) a quarter of the tiles need 9-14
// slots, i.e. a second round after the first has returned (24.2 vs 21.1 us per launch, r04).  This plan
// cuts the tiles at run starts instead, each holding whole runs of <= kBlkTileChunks chunks (the
// runs k_build_blocks forms, restated here on the host: <= kBlkRunRows rows whose column lists are
// prefixes of the run's longest, <= 64 pattern columns per chunk), so every tile is one round.  Only
// the plain SpMV on an all-register node-block plan runs it (k_spmv_blk has no LDS item bound); CG,
// dot-mode callers keep the merge-path plan; the plain L-wide node-block SpMM (k_spmm_blk: the same
// per-round run slots) takes it too.  MSPMV_SPMV_RUNS=0/1 forces it off / on.
static int runs_switch()
{
    const char *e = getenv("MSPMV_SPMV_RUNS");
    return e && *e ? (atoi(e) != 0 ? 1 : 0) : -1;
}

static mspmv_status spmv_runs_decide(mspmv_handle_s *h, const TilePlan *wg)
{
    h->spmv_runs = 0;
    const int sw = runs_switch();
    if (sw == 0 || !wg->blk_spmv || wg->num_tiles_reg != wg->num_tiles || h->m <= 0)
        return MSPMV_OK;
    const int *ro = nullptr, *ci = nullptr;
    if (host_pattern(h, &ro, &ci) != MSPMV_OK) {
        (void)hipGetLastError();
        set_error("");
        return MSPMV_OK;  // optional plan: the merge-path plan stays
    }
    // tiles of whole runs: <= kBlkTileChunks chunks and about the merge-path plan's items, and always
    // at least one run
    // (caps measured, r05l: 112 / 125 / 150 / 200 % of the merge-path tile's items within 1 % on pwtk,
    // 7 chunks per tile slower on the imperfect shape)
    const long long items_cap = (long long)wg->tile_items + wg->tile_items / 4;
    std::vector<int2> hb;
    hb.push_back(make_int2(0, 0));
    int chunks = 0;
    long long items = 0;
    for (int r = 0; r < h->m;) {
        const int g = r;
        int p = g, plen = ro[(size_t)g + 1] - ro[(size_t)g], hgt = 0;
        for (; r < h->m && hgt < kBlkRunRows; ++r, ++hgt) {
            const int s0 = ro[(size_t)r], len = ro[(size_t)r + 1] - s0;
            if (hgt > 0) {
                const int ps = ro[(size_t)p], mm = std::min(len, plen);
                bool same = true;
                for (int q = 0; q < mm && same; ++q)
                    same = ci[(size_t)s0 + q] == ci[(size_t)ps + q];
                if (!same || (len > 64 && plen <= 64))  // (k_build_blocks' rules, incl. its 64-column stop)
                    break;
                if (len > plen) {
                    p = r;
                    plen = len;
                }
            }
        }
        const int c = std::max(1, (plen + 63) / 64);
        const long long it = (long long)(r - g) + (ro[(size_t)r] - ro[(size_t)g]);
        if (chunks > 0 && (chunks + c > kBlkTileChunks || items + it > items_cap)) {
            hb.push_back(make_int2(g, ro[(size_t)g]));
            chunks = 0;
            items = 0;
        }
        chunks += c;
        items += it;
    }
    hb.push_back(make_int2(h->m, h->nnz));
    if (hb.size() > 2 && hb[hb.size() - 2].x == h->m)
        hb.erase(hb.end() - 2);
    const TilePlan *np = nullptr;
    const mspmv_status st = build_plan(h, 1, &np, 0, &hb);
    if (st != MSPMV_OK) {
        auto it = h->plans.find(kRunPlanKey);
        if (it != h->plans.end()) {
            free_plan(it->second);
            h->plans.erase(it);
        }
        (void)hipGetLastError();
        set_error("");
        return MSPMV_OK;
    }
    TilePlan &rp = h->plans.find(kRunPlanKey)->second;
    if (ensure_modes(h, rp, 1) != MSPMV_OK || !rp.blk_spmv || rp.num_tiles_reg != rp.num_tiles) {
        // the runs must all be register tiles
        auto it = h->plans.find(kRunPlanKey);
        free_plan(it->second);
        h->plans.erase(it);
        (void)hipGetLastError();
        set_error("");
        return MSPMV_OK;
    }
    h->spmv_runs = 1;
    return MSPMV_OK;
}

static mspmv_status spmv_plan(mspmv_handle_s *h, const TilePlan **out)
{
    ST_TRY(dia_plan(h, out));
    if (*out)
        return MSPMV_OK;
    const TilePlan *wg = nullptr;
    ST_TRY(get_plan(h, 1, &wg));
    if (h->spmv_slab < 0)
        ST_TRY(spmv_slab_decide(h, wg));
    if (h->spmv_slab == 1) {
        *out = &h->plans.find(kSlabPlanKey)->second;
        return MSPMV_OK;
    }
    if (h->spmv_onewave < 0) {
        bool want = false;
        ST_TRY(mostly_walks(wg, &want));
        if (want) {
            const TilePlan *np = nullptr;
            const int key = -64 * spmv_items_per_thread();  // build_plan's key for one-wave plans
            if (h->plans.find(key) == h->plans.end())
                ST_TRY(build_plan(h, 1, &np, 64));
            ST_TRY(ensure_modes(h, h->plans.find(key)->second, 1));
        }
        h->spmv_onewave = want ? 1 : 0;
    }
    if (h->spmv_onewave == 1) {
        *out = &h->plans.find(-64 * spmv_items_per_thread())->second;
        return MSPMV_OK;
    }
    if (h->spmv_runs < 0)
        ST_TRY(spmv_runs_decide(h, wg));
    *out = h->spmv_runs == 1 ? &h->plans.find(kRunPlanKey)->second : wg;
    return MSPMV_OK;
}

namespace mspmv {
mspmv_status plan_for(mspmv_handle_s *h, int L, const TilePlan **out) { return get_plan(h, L, out); }
mspmv_status dia_plan_for(mspmv_handle_s *h, int L, const TilePlan **out) { return dia_plan(h, out, L); }
}  // namespace mspmv

static mspmv_status validate_host_csr(const mspmv_csr_d *a)
{
    if (!a)
        return invalid("null matrix");
    if (a->num_rows < 0 || a->num_cols < 0 || a->num_nonzeros < 0)
        return invalid("negative dimension");
    if ((long long)a->num_rows + a->num_nonzeros > 0x7fffffffLL)
        return invalid("num_rows + num_nonzeros must fit in int32 (merge-path diagonals)");
    if (!a->row_offsets || (a->num_nonzeros > 0 && (!a->column_indices || !a->values)))
        return invalid("null CSR array");
    return MSPMV_OK;
}

static mspmv_status check_offsets_host(const int *ro, int m, int nnz)
{
    if (ro[0] != 0)
        return invalid("row_offsets[0] != 0");
    for (int i = 0; i < m; ++i)
        if (ro[i + 1] < ro[i])
            return invalid("row_offsets not monotone at row " + std::to_string(i));
    if (ro[m] != nnz)
        return invalid("row_offsets[num_rows] != num_nonzeros");
    return MSPMV_OK;
}

// view_of: a row range of another handle on the same device -- a->row_offsets (host, rebased to 0)
// are uploaded, the columns and values are the parent's from nonzero view_off on (not copied, not
// owned; the parent validated them), a->column_indices / values are ignored.
static mspmv_status create_common(const mspmv_csr_d *a, int device, bool from_device, mspmv_handle *out,
                                  hipStream_t on_stream = nullptr, const mspmv_handle_s *view_of = nullptr,
                                  long long view_off = 0)
{
    if (view_of) {
        if (!a || a->num_rows < 0 || a->num_nonzeros < 0 || !a->row_offsets || view_off < 0 ||
            view_off + a->num_nonzeros > view_of->nnz || a->num_cols != view_of->n)
            return invalid("row-range view outside its parent");
    } else {
        ST_TRY(validate_host_csr(a));
    }
    if (!out)
        return invalid("null out handle");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device visible");
        return MSPMV_ERR_HIP;
    }
    if (device < 0 || device >= ndev)
        return invalid("device index out of range");
    HIP_TRY(hipSetDevice(device));
    const auto t0 = std::chrono::steady_clock::now();
    auto *h = new mspmv_handle_s();
    h->device = device;
    h->m = a->num_rows;
    h->n = a->num_cols;
    h->nnz = a->num_nonzeros;
    auto fail = [&](mspmv_status s) {
        mspmv_destroy(h);
        return s;
    };
    if (hipDeviceGetAttribute(&h->num_cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        h->num_cus < 1)
        h->num_cus = 256;
    if (on_stream) {  // a stream owned by the caller (mspmv_comm: one stream per rank)
        h->stream = on_stream;
        h->own_stream = false;
    } else if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        set_error("hipStreamCreate failed");
        return fail(MSPMV_ERR_HIP);
    }
    mspmv_status st;
    // Column / value arrays are padded (zero column index, zero value) so the kernels' aligned
    // 16-byte group reads past the last nonzero stay inside the allocation.
    const size_t padded = (size_t)h->nnz + kNnzPad;
    if ((st = dev_alloc(&h->d_row_offsets, (size_t)h->m + 1)) != MSPMV_OK)
        return fail(st);
    if (view_of) {  // the parent's arrays (padded past its last nonzero, so past this range's too)
        h->own_arrays = false;
        h->d_cols = view_of->d_cols + view_off;
        h->d_vals = view_of->d_vals + view_off;
    } else {
        if ((st = dev_alloc(&h->d_cols, padded)) != MSPMV_OK || (st = dev_alloc(&h->d_vals, padded)) != MSPMV_OK)
            return fail(st);
        if (memset_sync(h->d_cols, 0, sizeof(int) * padded) != hipSuccess ||
            memset_sync(h->d_vals, 0, sizeof(double) * padded) != hipSuccess) {
            set_error("hipMemset of padded CSR arrays failed");
            return fail(MSPMV_ERR_HIP);
        }
    }
    if ((st = dev_alloc(&h->d_fault, 1)) != MSPMV_OK)
        return fail(st);
    if (memset_sync(h->d_fault, 0, sizeof(unsigned)) != hipSuccess) {
        set_error("hipMemset of the fault word failed");
        return fail(MSPMV_ERR_HIP);
    }
    const hipMemcpyKind kind = from_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    std::vector<int> host_ro;
    const int *ro = a->row_offsets;
    if (from_device) {
        host_ro.resize((size_t)h->m + 1);
        if (hipMemcpy(host_ro.data(), a->row_offsets, sizeof(int) * (h->m + 1), hipMemcpyDeviceToHost) != hipSuccess) {
            set_error("copy of device row_offsets failed");
            return fail(MSPMV_ERR_HIP);
        }
        ro = host_ro.data();
    }
    if ((st = check_offsets_host(ro, h->m, h->nnz)) != MSPMV_OK)
        return fail(st);
    if (hipMemcpy(h->d_row_offsets, a->row_offsets, sizeof(int) * (h->m + 1), kind) != hipSuccess ||
        (!view_of && h->nnz &&
         hipMemcpy(h->d_cols, a->column_indices, sizeof(int) * (size_t)h->nnz, kind) != hipSuccess) ||
        (!view_of && h->nnz && hipMemcpy(h->d_vals, a->values, sizeof(double) * (size_t)h->nnz, kind) != hipSuccess)) {
        set_error("CSR upload failed");
        return fail(MSPMV_ERR_HIP);
    }
    if (h->nnz && !view_of) {  // column range check on the device (a bad index would fault a gather)
        int *d_bad = nullptr;
        if ((st = dev_alloc(&d_bad, 1)) != MSPMV_OK)
            return fail(st);
        int bad = 0;
        hipError_t e = memset_sync(d_bad, 0, sizeof(int));
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_check_cols, dim3(1024), dim3(256), 0, h->stream, h->d_cols, (long long)h->nnz, h->n,
                               d_bad);
            e = hipGetLastError();
        }
        if (e == hipSuccess)
            e = hipStreamSynchronize(h->stream);
        if (e == hipSuccess)
            e = hipMemcpy(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost);
        dev_free(d_bad);
        if (e != hipSuccess) {
            set_error(std::string("column check: ") + hipGetErrorString(e));
            return fail(MSPMV_ERR_HIP);
        }
        if (bad)
            return fail(invalid("column index out of [0, num_cols)"));
    }
    // The plain product's plan is decided here, from the caller's host arrays when there are any (no
    // download): a matrix that takes the offset windows never builds the merge tile plan (VERDICT r05:
    // 0.66 ms of unused k_build_dict / k_pack_cols16 / k_build_blocks on the nlpkkt120 size); any other
    // path that needs tiles builds them on first use.
    {
        PatternScope scope(h);
        if (!from_device && !view_of) {
            h->pat_ro_ext = a->row_offsets;
            h->pat_ci_ext = a->column_indices;
        }
        const TilePlan *plan = nullptr;
        st = get_plan(h, 1, &plan, true);
        h->pat_ro_ext = h->pat_ci_ext = nullptr;
        if (st != MSPMV_OK)
            return fail(st);
    }
    if (hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
        set_error("hipEventCreate failed");
        return fail(MSPMV_ERR_HIP);
    }
    if (hipStreamSynchronize(h->stream) != hipSuccess) {
        set_error("setup sync failed");
        return fail(MSPMV_ERR_HIP);
    }
    h->setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *out = h;
    return MSPMV_OK;
}

static mspmv_status check_handle(mspmv_handle h)
{
    if (!h)
        return invalid("null handle");
    HIP_TRY(hipSetDevice(h->device));
    return MSPMV_OK;
}

static bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

extern "C" {

const char *mspmv_last_error(void) { return g_err.c_str(); }

const char *mspmv_cg_kernel_name(mspmv_handle h) { return h ? h->last_cg_kernel.c_str() : ""; }

const char *mspmv_spmv_kernel_name(mspmv_handle h)
{
    thread_local std::string name;
    if (!h)
        return "";
    const TilePlan *plan = nullptr;  // settles the handle's plain-SpMV plan (one-wave or not)
    if (h->m > 0 && spmv_plan(h, &plan) != MSPMV_OK)
        return "";
    name = spmv_kernel_name(h);
    return name.c_str();
}

const char *mspmv_spmm_kernel_name(mspmv_handle h, int L)
{
    thread_local std::string name;
    if (!h || L < 1)
        return "";
    // widths outside 1, 2, 4, 8, 16 run as column chunks (odd L on a zero-padded panel): the
    // widest chunk's kernel
    int w = 16;
    const int lp = (L > 1 && (L & 1)) ? L + 1 : L;
    while (w > lp)
        w >>= 1;
    const TilePlan *plan = nullptr;
    if (get_plan(h, w, &plan, true) != MSPMV_OK)
        return "";
    name = spmm_kernel_name(h, *plan, w);
    return name.c_str();
}

const char *mspmv_version(void) { return "mspmv 0.1.0 (gfx950, merge-path fp64)"; }

int mspmv_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

mspmv_status mspmv_csr_create(const mspmv_csr_d *host, int device, mspmv_handle *out)
{
    return create_common(host, device, false, out);
}

mspmv_status mspmv_csr_create_dev(const mspmv_csr_d *dev, int device, mspmv_handle *out)
{
    return create_common(dev, device, true, out);
}

}  // extern "C"

mspmv_status mspmv::csr_create_on_stream(const mspmv_csr_d *host, int device, hipStream_t stream, mspmv_handle *out)
{
    return create_common(host, device, false, out, stream);
}

mspmv_status mspmv::csr_create_view(mspmv_handle parent, int row_lo, int row_hi, const int *host_row_offsets,
                                    mspmv_handle *out)
{
    if (!parent || row_lo < 0 || row_hi < row_lo || row_hi > parent->m || !host_row_offsets)
        return invalid("csr_create_view: bad row range");
    const long long off = host_row_offsets[row_lo];
    std::vector<int> ro((size_t)(row_hi - row_lo) + 1);
    for (int r = row_lo; r <= row_hi; ++r)
        ro[(size_t)(r - row_lo)] = (int)(host_row_offsets[r] - off);
    const mspmv_csr_d v{row_hi - row_lo, parent->n, ro.back(), ro.data(), nullptr, nullptr};
    return create_common(&v, parent->device, false, out, nullptr, parent, off);
}

extern "C" {

mspmv_status mspmv_destroy(mspmv_handle h)
{
    if (!h)
        return MSPMV_OK;
    (void)hipSetDevice(h->device);
    if (h->stream)
        (void)hipStreamSynchronize(h->stream);
    for (auto &kv : h->plans)
        free_plan(kv.second);
    dev_free(h->d_row_offsets);
    if (h->own_arrays) {
        dev_free(h->d_cols);
        dev_free(h->d_vals);
    }
    dev_free(h->d_r);
    dev_free(h->d_p0);
    dev_free(h->d_p1);
    dev_free(h->d_ap);
    dev_free(h->d_partials);
    dev_free(h->d_partials_b);
    dev_free(h->d_gtickets);
    dev_free(h->d_scal);
    dev_free(h->d_red);
    dev_free(h->d_conv);
    dev_free(h->d_ctrl);
    dev_free(h->d_hist);
    dev_free(h->d_fault);
    if (h->cg_exec)
        (void)hipGraphExecDestroy(h->cg_exec);
    if (h->cg_graph)
        (void)hipGraphDestroy(h->cg_graph);
    if (h->d_flush)
        (void)hipFree(h->d_flush);
    if (h->h_ctrl)
        (void)hipHostFree(h->h_ctrl);
    if (h->ev0)
        (void)hipEventDestroy(h->ev0);
    if (h->ev1)
        (void)hipEventDestroy(h->ev1);
    resident_free(h->rcg);
    if (h->stream && h->own_stream)
        (void)hipStreamDestroy(h->stream);
    delete h;
    return MSPMV_OK;
}

mspmv_status mspmv_shape(mspmv_handle h, int *num_rows, int *num_cols, int *num_nonzeros)
{
    if (!h)
        return invalid("null handle");
    if (num_rows)
        *num_rows = h->m;
    if (num_cols)
        *num_cols = h->n;
    if (num_nonzeros)
        *num_nonzeros = h->nnz;
    return MSPMV_OK;
}

double mspmv_setup_ms(mspmv_handle h) { return h ? h->setup_ms : 0.0; }

mspmv_status mspmv_sync(mspmv_handle h)
{
    ST_TRY(check_handle(h));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MSPMV_OK;
}

// One CU-masked stream per (device, CU count) for the whole process, shared by every handle
// limited to that count and never destroyed: a masked stream holds a hardware queue of its own,
// and creating one per handle / per call ran a process out of its few queues (a launch on a
// third masked stream never started).
static std::mutex g_cu_mu;
static std::map<std::pair<int, int>, hipStream_t> g_cu_streams;

mspmv_status mspmv_set_cu_limit(mspmv_handle h, int num_cus)
{
    ST_TRY(check_handle(h));
    HIP_TRY(hipSetDevice(h->device));
    int total = 0;
    HIP_TRY(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, h->device));
    const int n = (num_cus <= 0 || num_cus >= total) ? total : num_cus;
    hipStream_t s = nullptr;
    bool own = true;
    if (n == total) {
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    } else {
        std::lock_guard<std::mutex> lk(g_cu_mu);
        auto it = g_cu_streams.find({h->device, n});
        if (it != g_cu_streams.end()) {
            s = it->second;
        } else {
            // CU i joins when floor((i+1) n / total) steps: n of the total, evenly spaced
            std::vector<uint32_t> mask((size_t)(total + 31) / 32, 0u);
            for (int i = 0; i < total; ++i)
                if ((long long)(i + 1) * n / total > (long long)i * n / total)
                    mask[(size_t)i / 32] |= 1u << (i % 32);
            HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
            g_cu_streams[{h->device, n}] = s;
        }
        own = false;
    }
    if (s == h->stream)
        return MSPMV_OK;
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        if (own)
            (void)hipStreamDestroy(s);
        set_error(std::string("set_cu_limit: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    // the CG graph was captured on the old stream with the old launch sizing
    if (h->cg_exec)
        (void)hipGraphExecDestroy(h->cg_exec);
    if (h->cg_graph)
        (void)hipGraphDestroy(h->cg_graph);
    h->cg_exec = nullptr;
    h->cg_graph = nullptr;
    h->cg_graph_key.clear();
    if (h->own_stream)
        (void)hipStreamDestroy(h->stream);
    h->stream = s;
    h->own_stream = own;
    if (n != h->num_cus) {
        // the register-resident CG layout is one workgroup per CU of the whole device: a CU-limited
        // stream cannot hold it (and one built while limited is "does not fit") -- rebuilt on demand
        resident_free(h->rcg);
        h->rcg = nullptr;
        // the single-RHS plan's tile stretch is sized to num_cus x resident workgroups (build_plan):
        // drop every cached plan so the next call plans for the CUs it will actually run on
        for (auto &kv : h->plans)
            free_plan(kv.second);
        h->plans.clear();
        h->spmv_onewave = -1;
        h->spmv_slab = -1;
        h->spmv_runs = -1;
        h->dia = -1;
        for (int &v : h->spmm_slab)
            v = -1;
        h->num_cus = n;
        const TilePlan *plan = nullptr;
        ST_TRY(get_plan(h, 1, &plan));
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return MSPMV_OK;
}

mspmv_status mspmv_merge_coords(mspmv_handle h, int num_parts, mspmv_coord *coords)
{
    ST_TRY(check_handle(h));
    if (num_parts < 1 || !coords)
        return invalid("num_parts must be >= 1 and coords non-null");
    const long long total = (long long)h->m + h->nnz;
    const long long step = (total + num_parts - 1) / num_parts;  // cpu_spmv.cpp:379
    int2 *d = nullptr;
    ST_TRY(dev_alloc(&d, (size_t)num_parts + 1));
    hipError_t e = launch_merge_coords(h->d_row_offsets, h->m, h->nnz, step, num_parts, d, h->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(coords, d, sizeof(int2) * (num_parts + 1), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize(h->stream);
    dev_free(d);
    if (e != hipSuccess) {
        set_error(std::string("merge coords: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    return MSPMV_OK;
}

// Widest native width (the tile kernels' L in {1, 2, 4, 8, 16}) that fits `left` columns.
static int native_chunk(int left)
{
    int w = 16;
    while (w > left)
        w >>= 1;
    return w;
}

// Even L outside the native set (6, 32, 1024, ... -- the reference's OmpMergeCsrmm takes any
// num_vectors, eval_vectors.sh sweeps 1..1024): column chunks of 16, 8, 4, 2 at even offsets of
// the same panels, the kernels reading and writing with panel stride L.  Each column's sum is
// the chunk kernel's, so the result equals the native-width one up to the tile plan's split
// rows (the SpMM tolerance of the tests).
static mspmv_status spmm_chunks(mspmv_handle_s *h, const double *d_X, double *d_Y, int L)
{
    const TilePlan *dp = nullptr;  // the offset-window plan serves every width it is enabled for
    ST_TRY(dia_plan(h, &dp, 2));
    for (int c0 = 0; c0 < L;) {
        const int w = native_chunk(L - c0);
        const TilePlan *plan = dp;
        if (!plan)
            ST_TRY(get_plan(h, w, &plan));
        HIP_TRY(launch_spmm(h, *plan, d_X + c0, d_Y + c0, w, nullptr, L));
        c0 += w;
    }
    return MSPMV_OK;
}

mspmv_status mspmv_dspmm_dev(mspmv_handle h, const double *d_X, double *d_Y, int L)
{
    ST_TRY(check_handle(h));
    if (L < 1)
        return invalid("L must be >= 1");
    if (h->m > 0 && (!d_X || !d_Y))
        return invalid("null vector");
    if (L > 1 && L % 2 == 0 && (!aligned16(d_X) || !aligned16(d_Y)))
        return invalid("multi-vector panels must be 16-byte aligned");
    if (h->m == 0)
        return MSPMV_OK;
    if (supported_L(L)) {
        const TilePlan *plan = nullptr;
        ST_TRY(get_plan(h, L, &plan, true));
        int nk = 0;
        HIP_TRY(launch_spmm(h, *plan, d_X, d_Y, L, &nk));
        return MSPMV_OK;
    }
    if (L % 2 == 0)
        return spmm_chunks(h, d_X, d_Y, L);
    // odd L > 1: through panels padded with a zero column to L + 1 (16-byte aligned rows)
    const int Lp = L + 1;
    double *xp = nullptr, *yp = nullptr;
    ST_TRY(dev_alloc(&xp, (size_t)h->n * Lp));
    mspmv_status st = dev_alloc(&yp, (size_t)h->m * Lp);
    hipError_t e = hipSuccess;
    if (st == MSPMV_OK)
        e = launch_panel_copy(d_X, L, xp, Lp, h->n, L, Lp, h->stream);
    if (st == MSPMV_OK && e == hipSuccess)
        st = spmm_chunks(h, xp, yp, Lp);
    if (st == MSPMV_OK && e == hipSuccess)
        e = launch_panel_copy(yp, Lp, d_Y, L, h->m, L, L, h->stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize(h->stream);  // before the padded panels are released
    dev_free(xp);
    dev_free(yp);
    if (st == MSPMV_OK && e != hipSuccess) {
        set_error(std::string("padded SpMM: ") + hipGetErrorString(e));
        st = MSPMV_ERR_HIP;
    }
    return st;
}

mspmv_status mspmv_dspmv_dev(mspmv_handle h, const double *d_x, double *d_y)
{
    return mspmv_dspmm_dev(h, d_x, d_y, 1);
}

mspmv_status mspmv_dspmm(mspmv_handle h, const double *X, double *Y, int L)
{
    ST_TRY(check_handle(h));
    if (L < 1)
        return invalid("L must be >= 1");
    if (h->m == 0)
        return MSPMV_OK;
    if (!X || !Y)
        return invalid("null vector");
    double *dX = nullptr, *dY = nullptr;
    ST_TRY(dev_alloc(&dX, (size_t)h->n * L));
    mspmv_status st = dev_alloc(&dY, (size_t)h->m * L);
    if (st == MSPMV_OK) {
        hipError_t e = hipMemcpyAsync(dX, X, sizeof(double) * h->n * L, hipMemcpyHostToDevice, h->stream);
        if (e != hipSuccess) {
            set_error(hipGetErrorString(e));
            st = MSPMV_ERR_HIP;
        }
    }
    if (st == MSPMV_OK)
        st = mspmv_dspmm_dev(h, dX, dY, L);
    if (st == MSPMV_OK) {
        hipError_t e = hipMemcpyAsync(Y, dY, sizeof(double) * h->m * L, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) {
            set_error(hipGetErrorString(e));
            st = MSPMV_ERR_HIP;
        }
    }
    if (st == MSPMV_OK)
        st = mspmv_check_faults(h);
    dev_free(dX);
    dev_free(dY);
    return st;
}

mspmv_status mspmv_dspmv(mspmv_handle h, const double *x, double *y) { return mspmv_dspmm(h, x, y, 1); }

mspmv_status mspmv_spmv_tile_stamps(mspmv_handle h, const double *d_x, double *d_y, size_t flush_bytes,
                                    unsigned long long *stamps, int *num_tiles)
{
    ST_TRY(check_handle(h));
    const TilePlan *p = nullptr;
    ST_TRY(get_plan(h, 1, &p, true));
    if (num_tiles)
        *num_tiles = p->num_tiles;
    if (!stamps)
        return MSPMV_OK;
    if (h->m > 0 && (!d_x || !d_y))
        return invalid("null vector");
    unsigned long long *d_st = nullptr;
    ST_TRY(dev_alloc(&d_st, (size_t)std::max(p->num_tiles, 1) * 6));
    hipError_t e = hipMemsetAsync(d_st, 0, sizeof(unsigned long long) * (size_t)std::max(p->num_tiles, 1) * 6, h->stream);
    if (e == hipSuccess && flush_bytes && flush_bytes > h->flush_cap) {  // the cold protocol's read sweep first
        if (h->d_flush)
            (void)hipFree(h->d_flush);
        h->d_flush = nullptr;
        h->flush_cap = 0;
        e = hipMalloc(&h->d_flush, flush_bytes);
        if (e == hipSuccess) {
            h->flush_cap = flush_bytes;
            e = launch_flush(h->d_flush, flush_bytes, h->stream, true);
        }
    }
    if (e == hipSuccess && flush_bytes)
        e = launch_flush(h->d_flush, flush_bytes, h->stream, false);
    if (e == hipSuccess)
        e = launch_spmv_tile_stamped(h, *p, d_x, d_y, d_st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess && p->num_tiles)
        e = hipMemcpy(stamps, d_st, sizeof(unsigned long long) * (size_t)p->num_tiles * 6, hipMemcpyDeviceToHost);
    dev_free(d_st);
    if (e == hipErrorNotSupported) {
        (void)hipGetLastError();
        set_error("spmv_tile_stamps: this matrix's plain SpMV does not run k_spmv_tile on 256-thread tiles");
        return MSPMV_ERR_UNSUPPORTED;
    }
    HIP_TRY(e);
    return MSPMV_OK;
}

mspmv_status mspmv_check_faults(mspmv_handle h)
{
    ST_TRY(check_handle(h));
    HIP_TRY(hipStreamSynchronize(h->stream));
    unsigned f = 0;
    HIP_TRY(hipMemcpy(&f, h->d_fault, sizeof f, hipMemcpyDeviceToHost));
    if (!f)
        return MSPMV_OK;
    HIP_TRY(memset_sync(h->d_fault, 0, sizeof f));
    set_error("a fold ticket drew past its group (its array was not zero when the launch began): the products "
              "since the last check are invalid");
    return MSPMV_ERR_FAULT;
}

mspmv_status mspmv_test_poison_tickets(mspmv_handle h, unsigned value, int flags)
{
    ST_TRY(check_handle(h));
    if (flags & ~(MSPMV_POISON_FILL | MSPMV_POISON_LATE_ZERO | MSPMV_POISON_NO_STOP))
        return invalid("test_poison_tickets: unknown flag");
    h->poison_value = value;
    h->poison_flags = flags;
    return MSPMV_OK;
}

// ---- CG ------------------------------------------------------------------------------------
static mspmv_status ensure_cg_workspace(mspmv_handle_s *h, int L, int nblk, int num_tiles, int hist_cap)
{
    // L = 1: the pipelined CG's p buffers hold {r, p} interleaved (2 m doubles each)
    const size_t elems = (size_t)h->m * std::max(L, 2);
    if (elems > h->cg_cap_elems) {
        dev_free(h->d_r);
        dev_free(h->d_p0);
        dev_free(h->d_p1);
        dev_free(h->d_ap);
        h->cg_cap_elems = 0;
        ST_TRY(dev_alloc(&h->d_r, elems));
        ST_TRY(dev_alloc(&h->d_p0, elems));
        ST_TRY(dev_alloc(&h->d_p1, elems));
        ST_TRY(dev_alloc(&h->d_ap, elems));
        h->cg_cap_elems = elems;
    }
    const size_t slots = (size_t)std::max(nblk, num_tiles);
    const size_t pcap = partials_capacity(slots, L);
    if (pcap > h->partials_cap) {
        dev_free(h->d_partials);
        h->partials_cap = 0;
        ST_TRY(dev_alloc(&h->d_partials, pcap));
        h->partials_cap = pcap;
    }
    if (!h->d_partials_b)
        ST_TRY(dev_alloc(&h->d_partials_b, (size_t)kUpdateMaxBlocks));
    if (gtickets_capacity(slots) > h->gtickets_cap) {
        dev_free(h->d_gtickets);
        h->gtickets_cap = 0;
        ST_TRY(dev_alloc(&h->d_gtickets, gtickets_capacity(slots)));
        // on the handle's stream: it is non-blocking, so a null-stream memset is not ordered before the
        // folds queued on it next
        HIP_TRY(hipMemsetAsync(h->d_gtickets, 0, sizeof(unsigned) * gtickets_capacity(slots), h->stream));
        h->gtickets_cap = gtickets_capacity(slots);
    }
    if (L > h->scal_cap) {
        dev_free(h->d_scal);
        dev_free(h->d_conv);
        h->scal_cap = 0;
        dev_free(h->d_red);
        ST_TRY(dev_alloc(&h->d_scal, (size_t)L));
        ST_TRY(dev_alloc(&h->d_conv, (size_t)L));
        ST_TRY(dev_alloc(&h->d_red, (size_t)L));
        h->scal_cap = L;
    }
    if (!h->d_ctrl)
        ST_TRY(dev_alloc(&h->d_ctrl, 1));
    if (!h->h_ctrl)
        HIP_TRY(hipHostMalloc((void **)&h->h_ctrl, sizeof(CgControl) * 2, hipHostMallocDefault));
    if (hist_cap > h->hist_cap) {
        dev_free(h->d_hist);
        h->hist_cap = 0;
        ST_TRY(dev_alloc(&h->d_hist, (size_t)hist_cap));
        h->hist_cap = hist_cap;
    }
    return MSPMV_OK;
}

// Register-resident single-RHS CG: one launch runs the whole solve.  d_stamps: the diagnostic
// phase stamps (mspmv_cg_resident_stamps), null in ordinary solves.
static mspmv_status cg_solve_resident(mspmv_handle_s *h, ResidentCg *rc, const double *d_b, double *d_x,
                                      int max_iters, double tol, int *iters, double *hist, int use_cap,
                                      unsigned long long *d_stamps = nullptr, int stamp_iters = 0)
{
    const int saved_cap = h->hist_cap;
    h->hist_cap = use_cap;
    hipError_t e = hipMemsetAsync(h->d_ctrl, 0, sizeof(CgControl), h->stream);
    if (e == hipSuccess)
        e = launch_cg_resident(h, rc, d_b, d_x, max_iters, tol, d_stamps, stamp_iters);
    h->hist_cap = saved_cap;
    if (e != hipSuccess) {
        set_error(std::string("resident CG launch: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    h->last_cg_kernel = rc->name;
    CgControl fin{};
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(&fin, h->d_ctrl, sizeof(CgControl), hipMemcpyDeviceToHost));
    const int it = fin.iters_out;
    if (iters)
        *iters = it;
    if (hist && use_cap > 0) {
        const int nh = std::min(it, use_cap);
        if (nh > 0)
            HIP_TRY(hipMemcpy(hist, h->d_hist, sizeof(double) * nh, hipMemcpyDeviceToHost));
    }
    if (fin.breakdown == 2) {
        set_error("resident CG: a reduction hand-off never completed (solve stalled; workgroups not co-resident?)");
        return MSPMV_ERR_STALL;
    }
    if (fin.breakdown) {
        set_error("CG breakdown: p.Ap gave a non-finite alpha at iteration " + std::to_string(it));
        return MSPMV_ERR_BREAKDOWN;
    }
    return MSPMV_OK;
}

// The resident layout of h when the next single-RHS solve may use it: built for this handle's
// current CU count (all of the device's CUs), matrix fits.  nullptr otherwise.
static mspmv_status resident_for(mspmv_handle_s *h, ResidentCg **out)
{
    *out = nullptr;
    if (!cg_resident_enabled())
        return MSPMV_OK;
    ResidentCg *rc = nullptr;
    ST_TRY(resident_prepare(h, &rc));
    if (rc->ok && rc->G == h->num_cus)
        *out = rc;
    return MSPMV_OK;
}

// CG; SPAI-preconditioned CG with the preconditioner's handle hm; or IC(0)-preconditioned CG
// with the factor ic.
static mspmv_status cg_solve_native(mspmv_handle_s *h, const double *d_b, double *d_x, int L, int max_iters,
                                    double tol, int *iters, double *hist, int hist_cap, mspmv_handle_s *hm,
                                    mspmv_ic0_s *ic)
{
    if (h->m != h->n)
        return invalid("CG needs a square matrix");
    if (hm && (hm->m != h->m || hm->n != h->n || hm->device != h->device))
        return invalid("the preconditioner must match the matrix's shape and device");
    if (ic && (ic->n != h->m || ic->device != h->device))
        return invalid("the IC(0) factor must match the matrix's shape and device");
    if (ic && (size_t)h->m * L > ic->y_cap) {
        if (ic->d_y)
            (void)hipFree(ic->d_y);
        ic->d_y = nullptr;
        ic->y_cap = 0;
        HIP_TRY(hipSetDevice(h->device));
        if (hipMalloc(&ic->d_y, sizeof(double) * (size_t)h->m * L) != hipSuccess)
            return (set_error("IC(0) workspace allocation failed"), MSPMV_ERR_OOM);
        ic->y_cap = (size_t)h->m * L;
    }
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    if (max_iters < 0)
        return invalid("max_iters < 0");
    if (h->m > 0 && (!d_b || !d_x))
        return invalid("null vector");
    if (!aligned16(d_b) || !aligned16(d_x))
        return invalid("CG vectors must be 16-byte aligned");
    if (iters)
        *iters = 0;
    if (h->m == 0)
        return MSPMV_OK;
    const TilePlan *plan = nullptr, *mplan = nullptr, *splan = nullptr;
    if (!hm && !ic) {
        // the split iteration's plain SpMM runs on the handle's offset-window or column-slab plan when
        // the plain product takes one, the pipelined single-RHS iteration's SpMV on its offset windows
        // (k_cg1_dia): decided here, before any graph capture (it may copy the matrix to the host)
        ST_TRY(get_plan(h, L, &splan, true));
        if (!(splan->dia || (splan->slab && cg_split_iteration(L))))
            splan = nullptr;
    }
    if (splan && splan->dia && !cg_split_iteration(L))
        plan = splan;  // the pipelined form on the windows needs no merge tiles
    else
        ST_TRY(get_plan(h, L, &plan));
    const bool dot_fused = dia_dot_fused();  // once per solve (an environment switch; in the graph key)
    if (hm) {
        ST_TRY(get_plan(hm, L, &mplan));
        HIP_TRY(hipStreamSynchronize(hm->stream));  // hm's SpMMs are enqueued on h's stream
    }
    const bool pipelined = !hm && !ic && !cg_split_iteration(L);  // single RHS: consumer-side reductions
    bool stalled = false;
    const int nblk = pipelined ? cg1_blocks(h->m) : cg_update_blocks((long long)h->m * L, h->num_cus);
    const int cap = hist ? std::max(hist_cap, 0) : 0;
    // partials: one per tile of the plan, or per window of the offset-window plan (its dot mode)
    ST_TRY(ensure_cg_workspace(h, L, nblk,
                               std::max({plan->num_tiles, mplan ? mplan->num_tiles : 0, splan ? splan->num_tiles : 0}),
                               cap));
    const int use_cap = hist ? cap : 0;
    if (pipelined) {
        // the whole solve as one register-resident launch, where the matrix fits (mspmv_cg_resident.hip)
        ResidentCg *rc = nullptr;
        ST_TRY(resident_for(h, &rc));
        if (rc) {
            const mspmv_status rs = cg_solve_resident(h, rc, d_b, d_x, max_iters, tol, iters, hist, use_cap);
            if (rs != MSPMV_ERR_STALL)
                return rs;
            // A hand-off never completed: the one-workgroup-per-CU grid was not co-resident (work on
            // another stream or process held CUs).  The solve is run again on the pipelined kernels,
            // whose init resets x, r and p; nothing of the stalled launch is kept.
            set_error("");
            stalled = true;
        }
    }
    const bool on_windows = pipelined && splan && splan->dia;
    h->last_cg_kernel = pipelined ? std::string(on_windows ? "pipelined (k_cg1_dia + k_cg1_update)"
                                                           : "pipelined (k_spmv_tile MODE 1 + k_cg1_update)") +
                                        (stalled ? " after a resident-CG stall" : "")
                        : hm      ? "SPAI-PCG (split)"
                        : ic      ? "IC0-PCG (split)"
                                  : "split (p update, SpMM, p.Ap, update)";
    const int saved_cap = h->hist_cap;
    h->hist_cap = use_cap;  // kernels record only what the caller asked for
    HIP_TRY(hipMemsetAsync(h->d_ctrl, 0, sizeof(CgControl), h->stream));
    // test hook (mspmv_test_poison_tickets): dirty fold tickets at the first fold, as an unordered zeroing
    // of freshly allocated (recycled) memory leaves them
    const int poison = h->poison_flags;
    h->poison_flags = 0;
    // the fold tickets reset themselves, but a solve that stopped early or faulted may leave some
    // raised: every solve starts from zeroed ones (a few KB, on the solve's stream)
    HIP_TRY(hipMemsetAsync(h->d_gtickets, 0, sizeof(unsigned) * h->gtickets_cap, h->stream));
    if (poison & MSPMV_POISON_NO_STOP)
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)&h->d_ctrl->fault_no_stop, 1, 1, h->stream));
    // Split-row tickets reset themselves when every tile sharing a row reaches close_split_rows; a CG
    // SpMM returns at its stop test before that (all tiles alike, but an aborted launch might not), so
    // every solve starts from zeroed tickets
    for (const TilePlan *tp : {plan, splan, mplan})
        if (tp && tp->d_fix_cnt)
            HIP_TRY(hipMemsetAsync(tp->d_fix_cnt, 0, sizeof(unsigned) * (size_t)tp->num_tiles, h->stream));
    if (hm)
        HIP_TRY(launch_pcg_init(h, hm, *mplan, d_b, d_x, L, tol, nblk));
    else if (ic)
        HIP_TRY(launch_pcg_ic0_init(h, ic, d_b, d_x, L, tol, nblk));
    else if (pipelined)
        HIP_TRY(launch_cg1_init(h, d_b, d_x, nblk));
    else
        HIP_TRY(launch_cg_init(h, d_b, d_x, L, tol, nblk));
    if (poison & MSPMV_POISON_FILL)  // test hook: the iterations' folds meet dirty tickets (after the init's)
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)h->d_gtickets, (int)h->poison_value, h->gtickets_cap, h->stream));
    auto iterate = [&](int i) -> hipError_t {
        if (hm)
            return launch_pcg_iteration(h, hm, *plan, *mplan, d_x, L, nblk, tol);
        if (ic)
            return launch_pcg_ic0_iteration(h, ic, *plan, d_x, L, nblk, tol);
        return launch_cg_iteration(h, *plan, splan, dot_fused, d_x, L, i & 1, nblk, tol);
    };
    int iterations_enqueued = 0;
    auto iterate_hook = [&](int i) -> hipError_t {
        hipError_t e = iterate(i);
        if (e == hipSuccess && (poison & MSPMV_POISON_LATE_ZERO) && ++iterations_enqueued == 1)
            e = hipMemsetAsync(h->d_gtickets, 0, sizeof(unsigned) * h->gtickets_cap, h->stream);  // the late zeroing
        return e;
    };

    const int K = cg_batch_iters(h->m, h->nnz, L);  // iterations per graph replay (even: p buffers alternate)
    mspmv_status st = MSPMV_OK;
    hipGraphExec_t exec = nullptr;
    if (max_iters >= K && !(poison & MSPMV_POISON_LATE_ZERO)) {
        // The graph bakes in every buffer, the plan, L, the tolerance and the history size:
        // reuse the handle's graph while all of them are unchanged (instantiation costs ms).
        const void *tk = nullptr;
        static_assert(sizeof(tk) == sizeof(tol), "tolerance bits as a key word");
        std::memcpy(&tk, &tol, sizeof tk);
        const std::vector<const void *> key = {
            d_x, h->d_r, h->d_p0, h->d_p1, h->d_ap, h->d_partials, h->d_partials_b, h->d_gtickets, h->d_scal,
            h->d_conv, h->d_red, h->d_ctrl, h->d_hist, h->stream, plan, splan, tk,
            reinterpret_cast<const void *>((intptr_t)L), reinterpret_cast<const void *>((intptr_t)nblk),
            reinterpret_cast<const void *>((intptr_t)use_cap), hm, mplan,
            hm ? (const void *)hm->d_vals : nullptr, ic, ic ? (const void *)ic->d_y : nullptr,
            ic ? (const void *)ic->d_lva : nullptr,
            reinterpret_cast<const void *>((uintptr_t)(hm ? hm->gen : 0)),
            reinterpret_cast<const void *>((uintptr_t)(ic ? ic->gen : 0)),
            reinterpret_cast<const void *>((intptr_t)K), reinterpret_cast<const void *>((intptr_t)dot_fused)};
        if (!h->cg_exec || h->cg_graph_key != key) {
            if (h->cg_exec)
                (void)hipGraphExecDestroy(h->cg_exec);
            if (h->cg_graph)
                (void)hipGraphDestroy(h->cg_graph);
            h->cg_exec = nullptr;
            h->cg_graph = nullptr;
            h->cg_graph_key.clear();
            hipError_t e = hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal);
            for (int i = 0; i < K && e == hipSuccess; ++i)
                e = iterate(i);
            hipGraph_t graph = nullptr;
            hipError_t e2 = hipStreamEndCapture(h->stream, &graph);
            if (e == hipSuccess)
                e = e2;
            h->cg_graph = graph;
            if (e == hipSuccess)
                e = hipGraphInstantiate(&h->cg_exec, graph, nullptr, nullptr, 0);
            if (e != hipSuccess) {
                set_error(std::string("CG graph capture: ") + hipGetErrorString(e));
                st = MSPMV_ERR_HIP;
            } else {
                h->cg_graph_key = key;
            }
        }
        exec = h->cg_exec;
    }
    hipEvent_t evs[2] = {nullptr, nullptr};
    if (st == MSPMV_OK && (hipEventCreateWithFlags(&evs[0], hipEventDisableTiming) != hipSuccess ||
                           hipEventCreateWithFlags(&evs[1], hipEventDisableTiming) != hipSuccess)) {
        set_error("hipEventCreate failed");
        st = MSPMV_ERR_HIP;
    }
    // Pipelined: batch b+1 is queued before batch b's control word is inspected, so the GPU
    // never idles on the host check; after convergence at most one batch of kernels runs,
    // each returning at its first instruction (the `done` test).
    int launched = 0, pending = 0, oldest = 0, slot = 0;
    while (st == MSPMV_OK) {
        const int k = std::min(K, max_iters - launched);
        if (k > 0) {
            hipError_t e = hipSuccess;
            if (k == K && exec)
                e = hipGraphLaunch(exec, h->stream);
            else
                for (int i = 0; i < k && e == hipSuccess; ++i)
                    e = iterate_hook(i);
            if (e == hipSuccess)
                e = hipMemcpyAsync(&h->h_ctrl[slot], h->d_ctrl, sizeof(CgControl), hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess)
                e = hipEventRecord(evs[slot], h->stream);
            if (e != hipSuccess) {
                set_error(std::string("CG launch: ") + hipGetErrorString(e));
                st = MSPMV_ERR_HIP;
                break;
            }
            launched += k;
            ++pending;
            slot ^= 1;
        }
        if (pending == 0)
            break;
        if (pending == 2 || k <= 0) {
            if (hipEventSynchronize(evs[oldest]) != hipSuccess) {
                set_error("CG event sync failed");
                st = MSPMV_ERR_HIP;
                break;
            }
            --pending;
            const bool done = h->h_ctrl[oldest].done != 0;
            oldest ^= 1;
            if (done)
                break;
        }
    }
    if (st == MSPMV_OK && max_iters > 0 && !hm && !ic) {
        // pipelined: the last iteration's stop test (a no-op once the solve has stopped); both
        // forms: the deferred x += alpha p of the last update
        hipError_t ef = pipelined ? launch_cg1_finish(h, d_x, max_iters & 1, nblk) : launch_cg_xflush(h, d_x, L, nblk);
        if (ef != hipSuccess) {
            set_error(std::string("CG finish launch: ") + hipGetErrorString(ef));
            st = MSPMV_ERR_HIP;
        }
    }
    hipError_t e = hipStreamSynchronize(h->stream);
    CgControl fin{};
    if (e == hipSuccess)
        e = hipMemcpy(&fin, h->d_ctrl, sizeof(CgControl), hipMemcpyDeviceToHost);
    if (st == MSPMV_OK && e != hipSuccess) {
        set_error(std::string("CG finish: ") + hipGetErrorString(e));
        st = MSPMV_ERR_HIP;
    }
    for (auto &ev : evs)
        if (ev)
            (void)hipEventDestroy(ev);
    h->hist_cap = saved_cap;
    if (st != MSPMV_OK)
        return st;
    const int it = fin.done ? fin.iters_out : fin.iter;
    if (iters)
        *iters = it;
    if (hist && use_cap > 0) {
        const int nh = std::min(it, use_cap);
        if (nh > 0)
            HIP_TRY(hipMemcpy(hist, h->d_hist, sizeof(double) * nh, hipMemcpyDeviceToHost));
    }
    if (fin.fault) {
        set_error("CG: a reduction ticket drew past its group (the ticket array was not zero when a fold began): "
                  "the solve stopped, X is not a solution");
        return MSPMV_ERR_FAULT;
    }
    if (fin.breakdown == 2) {
        if (iters)
            *iters = fin.iter;
        set_error("IC(0) apply: a triangular-solve dependency never became ready (solve stalled)");
        return MSPMV_ERR_STALL;
    }
    if (fin.breakdown) {
        set_error(L == 1 ? "CG breakdown: p.Ap gave a non-finite alpha at iteration " + std::to_string(it)
                         : "CG breakdown: p.Ap gave a non-finite alpha in at least one column (frozen; the "
                           "other columns were solved)");
        return MSPMV_ERR_BREAKDOWN;
    }
    return MSPMV_OK;
}

// Any L: the reference's L lock-step recurrences are independent per column (per-column alpha,
// beta and converged masks, no_pretreatment.hpp:109-120,163-176), so a panel of width outside
// {1, 2, 4, 8, 16} (the reference's preconditioner_benchmark runs num_vectors = 32) is solved as
// column groups of native widths, each copied into a contiguous panel and back.  The iteration
// count is the groups' maximum; the history is the max over groups, a finished group's columns
// frozen at their last residual (alpha = 0 leaves r unchanged), as the reference records them.
static mspmv_status cg_solve_dev(mspmv_handle_s *h, const double *d_b, double *d_x, int L, int max_iters,
                                 double tol, int *iters, double *hist, int hist_cap, mspmv_handle_s *hm = nullptr,
                                 mspmv_ic0_s *ic = nullptr)
{
    if (L < 1)
        return invalid("L must be >= 1");
    if (supported_L(L) || h->m == 0)
        return cg_solve_native(h, d_b, d_x, supported_L(L) ? L : 1, max_iters, tol, iters, hist, hist_cap, hm, ic);
    if (!d_b || !d_x)
        return invalid("null vector");
    const size_t m = (size_t)h->m;
    const int cap = hist ? std::max(hist_cap, 0) : 0;
    double *gb = nullptr, *gx = nullptr;
    ST_TRY(dev_alloc(&gb, m * 16));
    mspmv_status st = dev_alloc(&gx, m * 16);
    std::vector<std::vector<double>> gh;
    std::vector<int> git;
    int total = 0;
    bool faulted = false;  // a group's solve met a ticket fault (reported at the end)
    bool broke = false;  // a group's CG broke down: keep solving the other groups, report it at the end
    for (int c0 = 0; c0 < L && st == MSPMV_OK;) {
        const int w = native_chunk(L - c0);
        hipError_t e = launch_panel_copy(d_b + c0, L, gb, w, (long long)m, w, w, h->stream);
        if (e != hipSuccess) {
            set_error(std::string("column group copy: ") + hipGetErrorString(e));
            st = MSPMV_ERR_HIP;
            break;
        }
        std::vector<double> hg((size_t)cap);
        int it = 0;
        st = cg_solve_native(h, gb, gx, w, max_iters, tol, &it, cap ? hg.data() : nullptr, cap, hm, ic);
        if (st == MSPMV_ERR_BREAKDOWN) {
            broke = true;
            st = MSPMV_OK;
        } else if (st == MSPMV_ERR_FAULT) {  // the other groups still run (each solve re-zeroes its tickets)
            faulted = true;
            st = MSPMV_OK;
        }
        if (st == MSPMV_OK) {
            e = launch_panel_copy(gx, w, d_x + c0, L, (long long)m, w, w, h->stream);
            if (e == hipSuccess)
                e = hipStreamSynchronize(h->stream);
            if (e != hipSuccess) {
                set_error(std::string("column group copy: ") + hipGetErrorString(e));
                st = MSPMV_ERR_HIP;
            }
        }
        total = std::max(total, it);
        gh.push_back(std::move(hg));
        git.push_back(it);
        c0 += w;
    }
    dev_free(gb);
    dev_free(gx);
    if (st == MSPMV_OK && faulted) {
        set_error("CG: a reduction ticket drew past its group in at least one column group: X is not a solution");
        st = MSPMV_ERR_FAULT;
    } else if (st == MSPMV_OK && broke) {
        set_error("CG breakdown: p.Ap gave a non-finite alpha in at least one column (frozen; the other "
                  "columns were solved)");
        st = MSPMV_ERR_BREAKDOWN;
    }
    if (iters)
        *iters = total;
    for (int k = 0; k < std::min(total, cap); ++k) {
        double v = 0.0;
        for (size_t g = 0; g < gh.size(); ++g)
            if (git[g] > 0)
                v = std::max(v, gh[g][(size_t)std::min(k, git[g] - 1)]);
        hist[k] = v;
    }
    return st;
}

static mspmv_status cg_solve_host(mspmv_handle h, const double *B, double *X, int L, int max_iters, double tol,
                                  int *iters, double *hist, int hist_cap, mspmv_handle hm = nullptr,
                                  mspmv_ic0 ic = nullptr)
{
    ST_TRY(check_handle(h));
    if (h->m == 0) {
        if (iters)
            *iters = 0;
        return MSPMV_OK;
    }
    if (!B || !X)
        return invalid("null vector");
    double *dB = nullptr, *dX = nullptr;
    const size_t bytes = sizeof(double) * (size_t)h->m * L;
    ST_TRY(dev_alloc(&dB, (size_t)h->m * L));
    mspmv_status st = dev_alloc(&dX, (size_t)h->m * L);
    if (st == MSPMV_OK && hipMemcpy(dB, B, bytes, hipMemcpyHostToDevice) != hipSuccess) {
        set_error("B upload failed");
        st = MSPMV_ERR_HIP;
    }
    if (st == MSPMV_OK)
        st = cg_solve_dev(h, dB, dX, L, max_iters, tol, iters, hist, hist_cap, hm, ic);
    if ((st == MSPMV_OK || st == MSPMV_ERR_BREAKDOWN) && hipMemcpy(X, dX, bytes, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("X download failed");
        st = MSPMV_ERR_HIP;
    }
    dev_free(dB);
    dev_free(dX);
    return st;
}

mspmv_status mspmv_dcg_single_dev(mspmv_handle h, const double *d_b, double *d_x, int max_iters, double tolerance,
                                  int *iters, double *resid_hist, int hist_cap)
{
    ST_TRY(check_handle(h));
    return cg_solve_dev(h, d_b, d_x, 1, max_iters, tolerance, iters, resid_hist, hist_cap);
}

mspmv_status mspmv_cg_resident_stamps(mspmv_handle h, const double *d_b, double *d_x, int max_iters, double tolerance,
                                      int *iters, unsigned long long *stamps, int stamp_iters, int *workgroups)
{
    ST_TRY(check_handle(h));
    if (!d_b || !d_x || !stamps || stamp_iters < 1 || max_iters < 0)
        return invalid("cg_resident_stamps: vectors, stamps and stamp_iters >= 1 required");
    if (!aligned16(d_b) || !aligned16(d_x))
        return invalid("CG vectors must be 16-byte aligned");
    if (h->m < 1 || h->m != h->n)
        return invalid("CG needs a non-empty square matrix");
    HIP_TRY(hipSetDevice(h->device));
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, 1, &plan));
    ST_TRY(ensure_cg_workspace(h, 1, cg1_blocks(h->m), plan->num_tiles, 0));
    ResidentCg *rc = nullptr;
    ST_TRY(resident_for(h, &rc));
    if (!rc)
        return (set_error("cg_resident_stamps: this matrix does not take the register-resident CG"),
                MSPMV_ERR_UNSUPPORTED);
    const size_t n = (size_t)stamp_iters * rc->G * 5;
    unsigned long long *d_st = nullptr;
    ST_TRY(dev_alloc(&d_st, n));
    mspmv_status st = MSPMV_OK;
    if (hipMemsetAsync(d_st, 0, sizeof(unsigned long long) * n, h->stream) != hipSuccess) {
        set_error("cg_resident_stamps: memset failed");
        st = MSPMV_ERR_HIP;
    }
    if (st == MSPMV_OK)
        st = cg_solve_resident(h, rc, d_b, d_x, max_iters, tolerance, iters, nullptr, 0, d_st, stamp_iters);
    if (st == MSPMV_OK && hipMemcpy(stamps, d_st, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("cg_resident_stamps: download failed");
        st = MSPMV_ERR_HIP;
    }
    dev_free(d_st);
    if (workgroups)
        *workgroups = rc->G;
    return st;
}

mspmv_status mspmv_dcg_single(mspmv_handle h, const double *b, double *x, int max_iters, double tolerance,
                              int *iters, double *resid_hist, int hist_cap)
{
    return cg_solve_host(h, b, x, 1, max_iters, tolerance, iters, resid_hist, hist_cap);
}

mspmv_status mspmv_dcg_multi_dev(mspmv_handle h, const double *d_B, double *d_X, int L, int max_iters,
                                 double tolerance, mspmv_spmm_kernel kernel, int *iters, double *max_err_hist,
                                 int hist_cap)
{
    (void)kernel;  // the GPU always runs the merge-path SpMM
    ST_TRY(check_handle(h));
    return cg_solve_dev(h, d_B, d_X, L, max_iters, tolerance, iters, max_err_hist, hist_cap);
}

mspmv_status mspmv_dcg_multi(mspmv_handle h, const double *B, double *X, int L, int max_iters, double tolerance,
                             mspmv_spmm_kernel kernel, int *iters, double *max_err_hist, int hist_cap)
{
    (void)kernel;
    return cg_solve_host(h, B, X, L, max_iters, tolerance, iters, max_err_hist, hist_cap);
}

mspmv_status mspmv_dpcg_spai_multi_dev(mspmv_handle a, mspmv_handle m, const double *d_B, double *d_X, int L,
                                       int max_iters, double tolerance, mspmv_spmm_kernel kernel, int *iters,
                                       double *max_err_hist, int hist_cap)
{
    (void)kernel;  // the GPU always runs the merge-path SpMM
    ST_TRY(check_handle(a));
    ST_TRY(check_handle(m));
    return cg_solve_dev(a, d_B, d_X, L, max_iters, tolerance, iters, max_err_hist, hist_cap, m);
}

mspmv_status mspmv_dpcg_spai_multi(mspmv_handle a, mspmv_handle m, const double *B, double *X, int L, int max_iters,
                                   double tolerance, mspmv_spmm_kernel kernel, int *iters, double *max_err_hist,
                                   int hist_cap)
{
    (void)kernel;
    ST_TRY(check_handle(m));
    return cg_solve_host(a, B, X, L, max_iters, tolerance, iters, max_err_hist, hist_cap, m);
}

// ---- IC(0) factor on the device --------------------------------------------------------------
mspmv_status mspmv_ic0_create(const mspmv_csr_d *l, int device, mspmv_ic0 *out)
{
    if (!out)
        return invalid("null output");
    *out = nullptr;
    ST_TRY(validate_host_csr(l));
    if (l->num_rows != l->num_cols)
        return invalid("IC(0) factor must be square");
    const int n = l->num_rows, nnz = l->num_nonzeros;
    for (int r = 0; r < n; ++r)
        if (l->row_offsets[r + 1] < l->row_offsets[r])
            return invalid("row_offsets not monotone");
    if (l->row_offsets[0] != 0 || l->row_offsets[n] != nnz)
        return invalid("row_offsets inconsistent with num_nonzeros");
    for (int k = 0; k < nnz; ++k)
        if (l->column_indices[k] < 0 || l->column_indices[k] >= n)
            return invalid("column index out of range");
    // A lower-triangular factor with every diagonal present (IncompleteCholesky keeps A's lower
    // pattern, diagonal included): an entry above the diagonal would make the forward solve wait
    // on a row of a later level, a missing diagonal would divide by zero -- reject both here
    // rather than stall on the GPU.
    for (int r = 0; r < n; ++r) {
        bool diag = false;
        for (int k = l->row_offsets[r]; k < l->row_offsets[r + 1]; ++k) {
            if (l->column_indices[k] > r)
                return invalid("IC(0) factor has an entry above the diagonal in row " + std::to_string(r));
            diag = diag || l->column_indices[k] == r;
        }
        if (!diag)
            return invalid("IC(0) factor row " + std::to_string(r) + " has no diagonal entry");
    }
    // TransposeCsr (incomplete_cholesky_decomp.hpp:11-78): counting sort by column, rows in order
    std::vector<int> uro((size_t)n + 1, 0), uci((size_t)std::max(nnz, 1));
    std::vector<double> uva((size_t)std::max(nnz, 1));
    for (int k = 0; k < nnz; ++k)
        ++uro[(size_t)l->column_indices[k] + 1];
    for (int c = 0; c < n; ++c)
        uro[(size_t)c + 1] += uro[c];
    {
        std::vector<int> pos(uro.begin(), uro.end() - 1);
        for (int r = 0; r < n; ++r)
            for (int k = l->row_offsets[r]; k < l->row_offsets[r + 1]; ++k) {
                const int d = pos[l->column_indices[k]]++;
                uci[d] = r;
                uva[d] = l->values[k];
            }
    }
    // Level sets: a row's level is 1 + the deepest level among the rows it reads (L: columns
    // below the diagonal, solved ascending; L^T: columns above it, solved descending).  Waves
    // take rows in (level, row) order, so every awaited row is in an earlier level, hence an
    // earlier-dispatched wave, and a whole level's rows are solved concurrently (natural order
    // would chain every row to its left neighbour: ~15x slower on a 2-D stencil).
    auto order_by_level = [&](const int *rp, const int *cp, bool fwd, std::vector<int> &order) {
        std::vector<int> lev((size_t)n, 0);
        int maxlev = 0;
        for (int s = 0; s < n; ++s) {
            const int i = fwd ? s : n - 1 - s;
            int lv = 0;
            for (int k = rp[i]; k < rp[i + 1]; ++k) {
                const int j = cp[k];
                if (fwd ? j < i : j > i)
                    lv = std::max(lv, lev[j] + 1);
            }
            lev[i] = lv;
            maxlev = std::max(maxlev, lv);
        }
        std::vector<int> cnt((size_t)maxlev + 2, 0);
        for (int i = 0; i < n; ++i)
            ++cnt[(size_t)lev[i] + 1];
        for (int l2 = 0; l2 <= maxlev; ++l2)
            cnt[(size_t)l2 + 1] += cnt[l2];
        order.assign((size_t)std::max(n, 1), 0);
        for (int s = 0; s < n; ++s) {
            const int i = fwd ? s : n - 1 - s;
            order[(size_t)cnt[lev[i]]++] = i;
        }
        return n ? maxlev + 1 : 0;
    };
    std::vector<int> fwd_order, bwd_order;
    const int lf = order_by_level(l->row_offsets, l->column_indices, true, fwd_order);
    const int lb = order_by_level(uro.data(), uci.data(), false, bwd_order);
    HIP_TRY(hipSetDevice(device));
    mspmv_ic0_s *m = new mspmv_ic0_s;
    m->levels_fwd = lf;
    m->levels_bwd = lb;
    m->device = device;
    m->n = n;
    m->nnz = nnz;
    mspmv_status st = MSPMV_OK;
    auto up = [&](auto **d, const auto *src, size_t cnt) {
        if (st != MSPMV_OK)
            return;
        st = dev_alloc(d, std::max<size_t>(cnt, 1));
        if (st == MSPMV_OK && cnt && hipMemcpy(*d, src, sizeof(**d) * cnt, hipMemcpyHostToDevice) != hipSuccess) {
            set_error("IC(0) upload failed");
            st = MSPMV_ERR_HIP;
        }
    };
    up(&m->d_lro, l->row_offsets, (size_t)n + 1);
    up(&m->d_lci, l->column_indices, (size_t)nnz);
    up(&m->d_lva, l->values, (size_t)nnz);
    up(&m->d_uro, uro.data(), (size_t)n + 1);
    up(&m->d_uci, uci.data(), (size_t)nnz);
    up(&m->d_uva, uva.data(), (size_t)nnz);
    up(&m->d_fwd_order, fwd_order.data(), (size_t)n);
    up(&m->d_bwd_order, bwd_order.data(), (size_t)n);
    if (st == MSPMV_OK)
        st = dev_alloc(&m->d_ready, (size_t)std::max(n, 1));
    if (st != MSPMV_OK) {
        mspmv_ic0_destroy(m);
        return st;
    }
    *out = m;
    return MSPMV_OK;
}

mspmv_status mspmv_ic0_destroy(mspmv_ic0 m)
{
    if (!m)
        return MSPMV_OK;
    (void)hipSetDevice(m->device);
    dev_free(m->d_lro);
    dev_free(m->d_lci);
    dev_free(m->d_lva);
    dev_free(m->d_uro);
    dev_free(m->d_uci);
    dev_free(m->d_uva);
    dev_free(m->d_fwd_order);
    dev_free(m->d_bwd_order);
    dev_free(m->d_ready);
    if (m->d_y)
        (void)hipFree(m->d_y);
    delete m;
    return MSPMV_OK;
}

mspmv_status mspmv_dpcg_ic0_multi_dev(mspmv_handle a, mspmv_ic0 m, const double *d_B, double *d_X, int L,
                                      int max_iters, double tolerance, mspmv_spmm_kernel kernel, int *iters,
                                      double *max_err_hist, int hist_cap)
{
    (void)kernel;
    ST_TRY(check_handle(a));
    if (!m)
        return invalid("null IC(0) factor");
    return cg_solve_dev(a, d_B, d_X, L, max_iters, tolerance, iters, max_err_hist, hist_cap, nullptr, m);
}

mspmv_status mspmv_dpcg_ic0_multi(mspmv_handle a, mspmv_ic0 m, const double *B, double *X, int L, int max_iters,
                                  double tolerance, mspmv_spmm_kernel kernel, int *iters, double *max_err_hist,
                                  int hist_cap)
{
    (void)kernel;
    if (!m)
        return invalid("null IC(0) factor");
    return cg_solve_host(a, B, X, L, max_iters, tolerance, iters, max_err_hist, hist_cap, nullptr, m);
}

// ---- measurement ---------------------------------------------------------------------------
mspmv_status mspmv_time_stream_read(int device, size_t bytes, int reps, double *gbps)
{
    if (!gbps || reps < 1 || bytes < (1u << 20))
        return invalid("time_stream_read: gbps non-null, reps >= 1, bytes >= 1 MiB");
    HIP_TRY(hipSetDevice(device));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    bytes &= ~(size_t)15;
    double *buf = nullptr;
    HIP_TRY(hipMalloc(&buf, bytes));
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = memset_sync(buf, 0, bytes);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipEventCreate(&e0);
    if (e == hipSuccess)
        e = hipEventCreate(&e1);
    if (e == hipSuccess)
        e = launch_stream_read(buf, bytes, cus, s);  // warm-up
    if (e == hipSuccess)
        e = hipEventRecord(e0, s);
    for (int r = 0; r < reps && e == hipSuccess; ++r)
        e = launch_stream_read(buf, bytes, cus, s);
    if (e == hipSuccess)
        e = hipEventRecord(e1, s);
    if (e == hipSuccess)
        e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess)
        e = hipEventElapsedTime(&ms, e0, e1);
    if (e1)
        (void)hipEventDestroy(e1);
    if (e0)
        (void)hipEventDestroy(e0);
    if (s)
        (void)hipStreamDestroy(s);
    (void)hipFree(buf);
    if (e != hipSuccess) {
        set_error(std::string("time_stream_read: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    *gbps = ms > 0.f ? (double)bytes * reps / (ms * 1e-3) / 1e9 : 0.0;
    return MSPMV_OK;
}

mspmv_status mspmv_time_spmm_dev(mspmv_handle h, const double *d_X, double *d_Y, int L, int reps,
                                 size_t flush_bytes, double *avg_ms)
{
    ST_TRY(check_handle(h));
    if (reps < 1 || !avg_ms)
        return invalid("reps >= 1 and avg_ms required");
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    if (L > 1 && (!aligned16(d_X) || !aligned16(d_Y)))
        return invalid("multi-vector panels must be 16-byte aligned");
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, L, &plan, true));
    if (flush_bytes && flush_bytes > h->flush_cap) {
        if (h->d_flush)
            (void)hipFree(h->d_flush);
        h->d_flush = nullptr;
        h->flush_cap = 0;
        HIP_TRY(hipMalloc(&h->d_flush, flush_bytes));
        h->flush_cap = flush_bytes;
        HIP_TRY(launch_flush(h->d_flush, flush_bytes, h->stream, true));  // defined contents (+1.0)
    }
    // Hot (flush_bytes == 0): reps launches back to back, events around the region only; per launch
    // = region / reps (the launch gap included, ~0.2 us: r04i's headline 21.06 us against 21.09 in the
    // trace).  Cold: blocks of n (flush, launch) pairs, each beside a control block of n flushes alone;
    // per launch = the median over blocks of (pairs - control) / n.  Per-launch events (stream events,
    // or hipExtLaunchKernel's kernel-boundary ones) measured 4.7 us over the traced kernel on cant and
    // rma10 (r04i_frac_check.md); one control region for all reps left rma10 at 7.4 us against 9.5 in
    // the trace (r04m).  avg_ms: the timed regions per launch (flushes included).
    const bool run = plan->num_tiles > 0;
    const int nblk = flush_bytes && run ? std::min(reps, 8) : 1;
    std::vector<hipEvent_t> ev((size_t)nblk * 4, nullptr);
    for (auto &x : ev)
        HIP_TRY(hipEventCreate(&x));
    hipError_t e = hipSuccess;
    std::vector<int> nper((size_t)nblk);
    for (int b = 0, done = 0; b < nblk && e == hipSuccess; ++b) {
        const int n = (reps - done) / (nblk - b);
        nper[(size_t)b] = n;
        done += n;
        hipEvent_t *q = &ev[(size_t)b * 4];
        if (flush_bytes && run) {  // the control: n flushes alone
            e = hipEventRecord(q[2], h->stream);
            for (int i = 0; i < n && e == hipSuccess; ++i)
                e = launch_flush(h->d_flush, flush_bytes, h->stream, false);
            if (e == hipSuccess)
                e = hipEventRecord(q[3], h->stream);
        }
        if (e == hipSuccess)
            e = hipEventRecord(q[0], h->stream);
        for (int i = 0; i < n && e == hipSuccess && run; ++i) {
            if (flush_bytes)
                e = launch_flush(h->d_flush, flush_bytes, h->stream, false);
            if (e == hipSuccess)
                e = launch_spmm_tile_only(h, *plan, d_X, d_Y, L);
        }
        if (e == hipSuccess)
            e = hipEventRecord(q[1], h->stream);
    }
    if (e == hipSuccess)
        e = hipEventSynchronize(ev[(size_t)nblk * 4 - 3]);
    double total = 0.0;
    std::vector<double> per;
    for (int b = 0; b < nblk && e == hipSuccess; ++b) {
        float t = 0.f, c = 0.f;
        e = hipEventElapsedTime(&t, ev[(size_t)b * 4], ev[(size_t)b * 4 + 1]);
        if (e == hipSuccess && flush_bytes && run)
            e = hipEventElapsedTime(&c, ev[(size_t)b * 4 + 2], ev[(size_t)b * 4 + 3]);
        total += t;
        per.push_back(nper[(size_t)b] > 0 ? (double)(t - c) / nper[(size_t)b] : 0.0);
    }
    for (auto &x : ev)
        (void)hipEventDestroy(x);
    if (e != hipSuccess) {
        set_error(std::string("timing: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    std::sort(per.begin(), per.end());
    const double med = per.empty() ? 0.0 : per.size() % 2 ? per[per.size() / 2]
                                                         : 0.5 * (per[per.size() / 2 - 1] + per[per.size() / 2]);
    h->last_tile_kernel_ms = std::max(0.0, med);
    h->last_kernels_per_call = run ? 1 : 0;
    *avg_ms = total / reps;
    return MSPMV_OK;
}

mspmv_status mspmv_time_spmm_batch_dev(int count, const mspmv_handle *hs, const double *const *d_X,
                                       double *const *d_Y, int L, int reps, double *step_ms, double *tile_kernel_ms,
                                       int *kernels_per_step)
{
    if (count < 1 || !hs || !d_X || !d_Y || reps < 1 || !step_ms)
        return invalid("bad batch timing arguments");
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    for (int i = 0; i < count; ++i) {
        ST_TRY(check_handle(hs[i]));
        if (hs[i]->device != hs[0]->device)
            return invalid("batch handles must share a device");
        if (L > 1 && (!aligned16(d_X[i]) || !aligned16(d_Y[i])))
            return invalid("multi-vector panels must be 16-byte aligned");
    }
    ST_TRY(check_handle(hs[0]));
    std::vector<const TilePlan *> plans(count);
    int kps = 0;
    for (int i = 0; i < count; ++i) {
        ST_TRY(get_plan(hs[i], L, &plans[i], true));
        kps += plans[i]->num_tiles ? 1 : 0;
    }
    hipStream_t s = hs[0]->stream;
    for (int i = 0; i < count; ++i)  // everything after this point is ordered on hs[0]'s stream
        HIP_TRY(hipStreamSynchronize(hs[i]->stream));
    // The timed steps: launches back to back, events only around the whole region (one kernel per
    // product: split rows are closed inside the tile kernel).
    hipEvent_t ev[2] = {nullptr, nullptr};
    for (auto &x : ev)
        HIP_TRY(hipEventCreate(&x));
    hipError_t e = hipEventRecord(ev[0], s);
    for (int r = 0; r < reps && e == hipSuccess; ++r)
        for (int i = 0; i < count && e == hipSuccess; ++i) {
            hipStream_t own = hs[i]->stream;
            hs[i]->stream = s;
            e = launch_spmm_tile_only(hs[i], *plans[i], d_X[i], d_Y[i], L);
            hs[i]->stream = own;
        }
    if (e == hipSuccess)
        e = hipEventRecord(ev[1], s);
    if (e == hipSuccess)
        e = hipEventSynchronize(ev[1]);
    float total = 0.f;
    if (e == hipSuccess)
        e = hipEventElapsedTime(&total, ev[0], ev[1]);
    const double sum = (double)total;
    for (auto &x : ev)
        (void)hipEventDestroy(x);
    if (e != hipSuccess) {
        set_error(std::string("batch timing: ") + hipGetErrorString(e));
        return MSPMV_ERR_HIP;
    }
    *step_ms = (double)total / reps;
    if (tile_kernel_ms)
        *tile_kernel_ms = sum / ((double)reps * count);
    if (kernels_per_step)
        *kernels_per_step = kps;
    return MSPMV_OK;
}

mspmv_status mspmv_last_kernel_ms(mspmv_handle h, double *tile_kernel_ms, int *kernels_per_call)
{
    if (!h)
        return invalid("null handle");
    if (tile_kernel_ms)
        *tile_kernel_ms = h->last_tile_kernel_ms;
    if (kernels_per_call)
        *kernels_per_call = h->last_kernels_per_call;
    return MSPMV_OK;
}

mspmv_status mspmv_tile_plan(mspmv_handle h, int L, int *num_tiles, int *tile_items, int *num_carries,
                             mspmv_coord *bounds)
{
    ST_TRY(check_handle(h));
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, L, &plan, true));
    if (num_tiles)
        *num_tiles = plan->num_tiles;
    if (tile_items)
        *tile_items = plan->tile_items;
    if (num_carries)
        *num_carries = plan->num_carries;
    if (bounds)
        HIP_TRY(hipMemcpy(bounds, plan->d_bounds, sizeof(int2) * (plan->num_tiles + 1), hipMemcpyDeviceToHost));
    return MSPMV_OK;
}

mspmv_status mspmv_tile_modes(mspmv_handle h, int L, unsigned char *modes)
{
    ST_TRY(check_handle(h));
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    if (!modes)
        return invalid("null modes");
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, L, &plan, true));
    if (plan->num_tiles)
        HIP_TRY(hipMemcpy(modes, plan->d_modes[l_index(L)], plan->num_tiles, hipMemcpyDeviceToHost));
    // node-block tiles reduced in registers (lane tree, not the plan's mode): L = 1 on any plan
    // with node blocks, L > 1 when get_plan chose the node-block plan (k_spmm_blk)
    if (plan->d_blk && (L == 1 || plan->num_tiles_reg == plan->num_tiles))
        for (int t = 0; t < plan->num_tiles; ++t)
            if (plan->h_blk_reg[(size_t)t])
                modes[t] = 255;
    return MSPMV_OK;
}

mspmv_status mspmv_tile_lanes(mspmv_handle h, int L, int *lanes)
{
    ST_TRY(check_handle(h));
    if (!lanes)
        return invalid("null out pointer");
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, L, &plan, true));
    *lanes = L == 1 ? plan->lanes : kBlock;
    return MSPMV_OK;
}

mspmv_status mspmv_tile_streams(mspmv_handle h, int *tiles_cols16, int *tiles_dict)
{
    ST_TRY(check_handle(h));
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, 1, &plan, true));
    if (tiles_cols16)
        *tiles_cols16 = plan->d_cols16 ? plan->num_tiles16 : 0;
    if (tiles_dict)
        *tiles_dict = plan->d_dict ? plan->num_tiles_dict : 0;
    return MSPMV_OK;
}

mspmv_status mspmv_plan_block_tiles(mspmv_handle h, int L, int *tiles_blk)
{
    ST_TRY(check_handle(h));
    if (!tiles_blk)
        return invalid("null out pointer");
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, L, &plan, true));
    *tiles_blk = plan->d_blk ? plan->num_tiles_blk : 0;
    return MSPMV_OK;
}

mspmv_status mspmv_plan_dict_tiles(mspmv_handle h, int L, int *tiles_dict)
{
    ST_TRY(check_handle(h));
    if (!tiles_dict)
        return invalid("null out pointer");
    if (!supported_L(L))
        return (set_error("L must be one of 1, 2, 4, 8, 16"), MSPMV_ERR_UNSUPPORTED);
    const TilePlan *plan = nullptr;
    ST_TRY(get_plan(h, L, &plan, true));
    *tiles_dict = plan->d_dict && (L == 1 || L == 16) ? plan->num_tiles_dict : 0;
    return MSPMV_OK;
}

// ---- device memory helpers -----------------------------------------------------------------
mspmv_status mspmv_device_malloc(int device, size_t bytes, void **d_ptr)
{
    if (!d_ptr)
        return invalid("null out pointer");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipMalloc(d_ptr, bytes ? bytes : 1));
    return MSPMV_OK;
}

mspmv_status mspmv_device_free(void *d_ptr)
{
    if (d_ptr)
        HIP_TRY(hipFree(d_ptr));
    return MSPMV_OK;
}

mspmv_status mspmv_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes)
{
    HIP_TRY(hipMemcpy(d_dst, h_src, bytes, hipMemcpyHostToDevice));
    return MSPMV_OK;
}

mspmv_status mspmv_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes)
{
    HIP_TRY(hipMemcpy(h_dst, d_src, bytes, hipMemcpyDeviceToHost));
    return MSPMV_OK;
}

mspmv_status mspmv_memcpy_d2d(void *d_dst, const void *d_src, size_t bytes)
{
    HIP_TRY(hipMemcpy(d_dst, d_src, bytes, hipMemcpyDeviceToDevice));
    return MSPMV_OK;
}

mspmv_status mspmv_memset_dev(void *d_dst, int byte_value, size_t bytes)
{
    HIP_TRY(memset_sync(d_dst, byte_value, bytes));
    return MSPMV_OK;
}

}  // extern "C"
