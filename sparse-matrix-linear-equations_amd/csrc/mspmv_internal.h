// mspmv_internal.h -- shared between the HIP kernels (mspmv_kernels.hip) and the C-ABI
// implementation (mspmv_api.hip).  Not installed; the public boundary is include/mspmv.h.
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

#include "mspmv.h"

// hipMemset on the legacy null stream, then wait for it: every handle's stream is non-blocking, so a
// null-stream fill is not ordered before the next launch on it otherwise (a fold's tickets or a plan's
// modes could be read before they are written)
static inline hipError_t memset_sync(void *p, int value, size_t bytes)
{
    const hipError_t e = hipMemset(p, value, bytes);
    return e == hipSuccess ? hipStreamSynchronize(nullptr) : e;
}

namespace mspmv {

constexpr int kBlock = 256;  // 4 x 64-lane waves per workgroup
constexpr unsigned kFaultTicket = 1u;  // fault word bit: a fold ticket drew past its group (ticket_arrive)
constexpr int kNnzPad = 16;  // padding elements after the last nonzero of the device arrays
constexpr int kSnapDiv = 8;
constexpr int kSlotGroup = 32;     // fan-in of the CG partial-reduction tree (reduce_slots)
constexpr int kTicketStride = 64;  // tickets 256 B apart: one per memory line
// Single-RHS pipelined CG (consumer-side reductions): the update kernel sums at most
// kConsumeTile of the SpMV's p.Ap partials (more are folded by group tickets first), the
// SpMV sums the update's <= kUpdateMaxBlocks r.r partials.
constexpr int kConsumeTile = 4096;
constexpr int kUpdateMaxBlocks = 1024;

// Column-slab form of the plain single-RHS SpMV (mspmv_slab.hip): the plan's tiles are large blocks
// (two per CU), each block's nonzeros reordered by column slab (kSlabCols columns of x, staged in LDS
// once per block and slab) and cut into chunks of <= kSlabChunk nonzeros of one slab; a chunk's
// entries are its runs of one row.
constexpr int kSlabThreads = 512;
constexpr int kSlabCols = 4096;     // columns per slab: 32 KB of x in LDS
constexpr int kSlabRows = 2047;     // rows ending in one block (+ a trailing partial row)
constexpr int kSlabChunk = 2048;    // nonzeros per chunk (4 per thread)
constexpr int kSlabEntries = 1024;  // row runs per chunk
constexpr int kSlabBlocksPerCu = 2; // resident blocks per CU (LDS: 76 KB per block)
constexpr int kSlabMaxChunks = 255; // chunks per block (their descriptors sit in LDS)
// The SpMV's block shapes: 0 the band configuration above (merge-path blocks, two per CU); 1 the
// column-group configuration for x too wide for any block to reuse a slab (power-law rows over random
// columns): one block per CU, each block a (row block, column group) pair -- whole rows, the columns of
// kSlabGroups consecutive slab ranges -- so a block stages a quarter of x, not all of it; the groups'
// partial row sums are folded by the row block's last block to finish.
struct SlabCfg {
    int threads;  // per block
    int cols;     // columns per slab (LDS: cols x 8 B)
    int rows;     // rows ending in one block
    int chunk;    // nonzeros per chunk
    int entries;  // row runs per chunk
    int per_cu;   // resident blocks per CU
};
// 2: the column-group blocks of 1 in sliced-ELL form (k_spmv_sell): per (block, slab) the short runs, sorted
// by length, in slices of 64 whose values sit column-major (lane = run), long runs apart.
constexpr SlabCfg kSlabCfgs[3] = {{kSlabThreads, kSlabCols, kSlabRows, kSlabChunk, kSlabEntries, kSlabBlocksPerCu},
                                  {1024, 8192, 4095, 4096, 2048, 1},
                                  {1024, 14336, 4095, 0, 0, 1}};
constexpr int kSlabGroups = 4;
constexpr int kSlabMaxGroups = 8;
constexpr int kSellShortRun = 8;     // sliced-ELL: runs up to this long sit one per lane in slices of 64,
constexpr int kSellLongRun = 64;     // up to this long 8 per slice (8 lanes each), longer ones by whole waves
                                     // in pieces of <= 512
constexpr int kSellMaxPieces = 1024;  // long-run pieces per (block, slab) segment (their sums sit in LDS)
constexpr int kSellMaxSegs = 255;     // segments per block (their descriptors sit in LDS)
// short runs packed per lane by the slice's longest run (<= 4): {runs per lane K, slots per run}
constexpr int2 kSellPack[5] = {{1, 1}, {8, 1}, {4, 2}, {2, 3}, {2, 4}};
constexpr int kSlabLongRun = 64;  // runs longer than this are summed by whole waves (listed first in a chunk)
struct SlabData {
    int L = 1;                          // 1: the SpMV's plan (k_spmv_slab); 8 / 16: an SpMM plan (k_spmm_slab)
    int cfg = 0;                        // the kernel configuration the plan was cut for (SpMV: kSlabCfgs;
                                        // SpMM: slab_mm_cfg)
    int groups = 1;                     // SpMV column groups (cfg 1): blocks = row blocks x groups
    bool pack = false;                  // sliced-ELL: short runs packed per lane (column groups > 1; k_spmv_sell<., true>)
    double *d_part = nullptr;           // [groups][m] the groups' partial row sums (groups > 1)
    unsigned *d_gcnt = nullptr;         // [row blocks] tickets of the fold (self-resetting)
    // sliced-ELL (cfg 2): d_chunk holds the (block, slab) segments {first column, slice0, slice1, piece0} (+ sentinel)
    int4 *d_slice = nullptr;            // [slices] {value base, slots per lane | medium << 16, run-word base, 0}
    unsigned short *d_sent = nullptr;   // 16-bit run words (mspmv_slab.hip sell_block; 0: no run)
    int4 *d_long = nullptr;             // [long-run pieces] {value base, length <= 512, row in block,
                                        //  the run's first piece in the segment | pieces << 16}
    int num_chunks = 0, num_entries = 0;
    int4 *d_blk = nullptr;              // [blocks] {first row, rows ending in the block, chunk0, chunk1}
    int4 *d_chunk = nullptr;            // [chunks + 1] SpMV: {stream start, length | lanes_log2 << 13 | long runs << 16,
                                        // slab, entry0};
                                        // SpMM: {stream start, length | lanes_log2 << 13 | columns << 16,
                                        // first column of the chunk's segment, entry0}
    uint2 *d_ent = nullptr;             // [entries] {offset in chunk | length << 16, row in block}
    double *d_val = nullptr;            // [nnz + pad] values, slab-major within each block
    unsigned short *d_col = nullptr;    // [nnz + pad] column - slab * kSlabCols (SpMM: - segment's first column)
    double x_bytes_per_nnz = 0.0;       // x (SpMM: panel rows, all L columns) staged per nonzero (plan statistic)
};

// Column-slab SpMM (Y = A X, L = 8 or 16; mspmv_slab.hip): blocks of rows (merge-path balanced), each
// block's nonzeros reordered by column segment (a greedy cut of the block's sorted columns into ranges
// of <= cols panel rows, gaps between them skipped), the segment's panel rows staged in LDS once, and
// the block's rows accumulated in LDS.  One configuration per launch shape.
struct SlabMmCfg {
    int L;        // right-hand sides
    int threads;  // per block
    int rows;     // rows ending in one block (+ a trailing partial row)
    int cols;     // panel rows per segment (LDS: cols x L x 8 B)
    int chunk;    // nonzeros per chunk
    int entries;  // row runs per chunk
};
constexpr int kSlabMmMaxChunks = 127;  // chunks per block (their descriptors sit in LDS)

// Offset windows (mspmv_dia.hip): 64-row windows whose rows list their columns at <= kDiaMaxK common
// offsets col - row, values lane-major per window.
constexpr double kDiaMaxRemFrac = 0.05;  // at most this share of the nonzeros in the windows' remainder
constexpr int kDiaMaxK = 64;  // one offset per lane of the window's wave (metadata read by v_readlane)
struct DiaData {
    int windows = 0;
    int max_k = 0;
    int masked_windows = 0;                  // windows with a row missing some offset (presence masks)
    long long sum_k = 0;                     // offsets over the windows
    long long sum_pairs = 0;                 // value pair panels: (K + 1) / 2 per window
    double fill = 0.0;                       // nonzeros / (64 sum_k)
    int4 *d_hdr = nullptr;                   // [windows] {K, offset base, pair panel base, mask base or -1}
    int *d_off = nullptr;                    // [sum_k]
    unsigned long long *d_mask = nullptr;    // [K of the masked windows]
    double *d_vt = nullptr;                  // [sum_pairs][64 lanes][2]: offsets 2p, 2p+1 of each row
    long long rem = 0;                       // remainder entries (off the windows' offset lists)
    int rem_windows = 0;                     // windows holding some
    int *d_rem_ptr = nullptr;                // [m + 1] (null when rem == 0)
    int *d_rem_col = nullptr;                // [rem]
    double *d_rem_val = nullptr;             // [rem]
};

// A merge-path tile plan for one nominal tile size (merge items per tile).
//
// Tile t covers the merge-path diagonals between boundary t and t+1.  A boundary whose
// row was entered by at most `snap` nonzeros is moved back to that row's start ("row
// snapped"): the row is then computed whole by the tile that completes it, so no carry
// crosses that boundary.  Boundaries deeper inside a long row stay exact merge-path
// coordinates ("split"): the tiles that end inside such a row store carries, the tile that completes
// it stores the row's own part, and the last of them to finish adds the carries in tile order
// (close_split_rows: one ticket per row, no fix-up launch).  Every tile holds at most tile_items +
// tile_items/kSnapDiv items.
struct TilePlan {
    int lanes = kBlock;                 // threads sharing one tile: 256, or 64 (one-wave plain-SpMV plan)
    int tile_items = 0;
    int snap = 0;
    int num_tiles = 0;
    int2 *d_bounds = nullptr;           // [num_tiles+1] (row, nnz) boundary coordinates
    unsigned char *d_split = nullptr;   // [num_tiles+1] 1 = split boundary (carry crosses it)
    // [log2 L][num_tiles] in-tile reduction per right-hand-side count (plans are shared by
    // tile size across L): 0 merge walk, lg+1 row groups of 2^lg nonzero lanes (k_tile_modes)
    unsigned char *d_modes[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    int num_carries = 0;                // tiles whose trailing boundary is split
    double *d_carry_val = nullptr;      // [3][num_tiles][carry_L]: carries, then the split rows' heads
                                        // (TileArgs::head_val, head_pub)
    // Split rows (null when num_carries == 0): fix[t] = {the tile completing the row tile t ends inside
    // (-1: t ends on a row boundary), that row's carry count, the carry count of the row tile t
    // completes (0: none), 0}; fix_cnt[t] = tickets of the row tile t completes (reset by its closer).
    int4 *d_fix = nullptr;              // [num_tiles]
    unsigned *d_fix_cnt = nullptr;      // [num_tiles]
    int carry_L = 0;                    // capacity (columns) of d_carry_val
    // Single-RHS plans: 16-bit column offsets.  A tile whose columns span < 65536 stores
    // col - colbase[t] in cols16 (2 B per nonzero instead of 4 in the HBM stream); colbase[t]
    // = -1 keeps the tile on the int32 columns.  Null when not built.
    int *d_colbase = nullptr;           // [num_tiles]
    unsigned short *d_cols16 = nullptr; // [nnz + kNnzPad]
    int num_tiles16 = 0;                // tiles on the 16-bit stream
    // Single-RHS plans: per-tile column dictionaries (k_build_dict) where they pay.  Tile t's
    // distinct columns ascending in dict[n0 ..] (ndict[t] of them), each nonzero's position in
    // that list in idx16[k].  Null when not built.
    int *d_dict = nullptr;              // [nnz + kNnzPad]
    int *d_ndict = nullptr;             // [num_tiles]
    unsigned short *d_idx16 = nullptr;  // [nnz + kNnzPad]
    int num_tiles_dict = 0;             // tiles that gather through their dictionary
    // Single-RHS plans: node-block run descriptors (k_build_blocks), blk_stride (16, 32 or 64) per
    // tile, entry 0 of a tile holding its count (0: striped staging).  Null when no tile qualifies.
    uint4 *d_blk = nullptr;             // [num_tiles * blk_stride]
    int blk_stride = 0;
    int num_tiles_blk = 0;              // tiles staged by node blocks
    int num_tiles_reg = 0;              // of those, tiles reduced in registers (h_blk_reg)
    int blk_rows_max = 8;               // the tallest run (rows of one node) over the descriptors
    bool blk_spmv = false;              // the plain SpMV runs k_spmv_blk (most tiles register run tiles;
                                        // the rest take its register fallback)
    int blk_two_rounds = 0;             // node-block tiles of more than one round of run slots (> kBlkTileChunks)
    std::vector<unsigned char> h_blk_reg;  // [num_tiles] 1: the plain SpMV reduces the tile in registers
                                           // (a reordered sum: mspmv_tile_modes reports 255)
    SlabData *slab = nullptr;           // column-slab plan (tiles = blocks; mspmv_slab.hip), else null
    DiaData *dia = nullptr;             // offset-window plan (tiles = 64-row windows; mspmv_dia.hip), else null
};

// Device-resident CG scalars (one set per right-hand side column).
struct CgScalars {
    double rs_old;
    double b_norm;
    double alpha;
    double beta;
    double pAp;
    double rs_new;
    double rs_par[2];  // single-RHS pipelined CG: r.r of iteration k at [k & 1] (k_spmv_tile MODE 1)
};

struct CgControl {
    int iter;        // iterations completed
    int done;        // 1 once every column converged (or breakdown)
    int iters_out;   // iteration count to report (the reference's return value)
    int breakdown;   // 1 if p.Ap <= 0 or non-finite was met
    int iter_par[2]; // single-RHS pipelined CG: iteration index handed to the next SpMV, by parity
    int x_pending;   // multi-RHS split CG: x += alpha p of the last update not applied yet (k_cg_update
                     // sets it, the next p update applies the term, the fold after it clears it)
    unsigned fault;          // kFault* bits raised by the kernels (take_ticket): the solve's result is invalid
    unsigned fault_no_stop;  // sharded CG: a fault does not set done on the device (the host stops on the
                             // all-reduced fault word, so every rank stops at the same batch)
};


// Register-resident single-RHS CG (mspmv_cg_resident.hip): the ELL layout of the matrix's row
// blocks, one per CU, built once per handle when the matrix fits (ok).
struct ResidentCg {
    bool ok = false;
    int G = 0, rpt = 0, nzr = 0;
    int *d_rb = nullptr;
    int *d_cols = nullptr;
    double *d_vals = nullptr;
    short *d_len = nullptr;
    double *d_slots = nullptr;  // hand-off slots, reset to the empty pattern before every solve
    size_t slot_bytes = 0;
    unsigned *d_abort = nullptr;
    std::string name;  // "k_cg_resident<RPT,NZR> x G" (mspmv_cg_kernel_name)
};

}  // namespace mspmv

// Every handle and IC(0) factor gets a process-unique generation number at creation, so a cached
// CG graph that baked in another object's buffers is never replayed against a new object the
// allocator happened to place at the same address (mspmv_api.hip, cg_solve_native).
unsigned long long mspmv_next_generation();

struct mspmv_handle_s {
    unsigned long long gen = mspmv_next_generation();
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    bool own_stream = true;  // false: a shared CU-masked stream (mspmv_set_cu_limit)
    bool own_arrays = true;  // false: d_cols / d_vals are a row range of another handle's (csr_create_view)
    int m = 0, n = 0, nnz = 0;
    int *d_row_offsets = nullptr;
    int *d_cols = nullptr;
    double *d_vals = nullptr;
    double setup_ms = 0.0;
    std::map<int, mspmv::TilePlan> plans;  // by nominal tile size
    // CG workspace (grown on demand)
    size_t cg_cap_elems = 0;
    double *d_r = nullptr, *d_p0 = nullptr, *d_p1 = nullptr, *d_ap = nullptr;
    double *d_partials = nullptr;
    size_t partials_cap = 0;
    double *d_partials_b = nullptr;  // single-RHS pipelined CG: r.r partials of init / update (<= kUpdateMaxBlocks)
    unsigned *d_gtickets = nullptr;  // reduce_slots group tickets (zeroed once, self-resetting)
    size_t gtickets_cap = 0;
    mspmv::CgScalars *d_scal = nullptr;
    double *d_red = nullptr;  // [L] p.Ap of the split multi-RHS iteration (k_spmm_tile MODE 2 -> k_cg_update)
    unsigned char *d_conv = nullptr;   // per-column converged flags
    mspmv::CgControl *d_ctrl = nullptr;
    mspmv::CgControl *h_ctrl = nullptr;  // pinned mirror
    double *d_hist = nullptr;
    int hist_cap = 0;
    int scal_cap = 0;
    // kFault* bits the plain products raise (ticket_arrive: split-row and column-group tickets), read
    // and cleared by mspmv_check_faults (the host-pointer products call it; CG solves use d_ctrl's)
    unsigned *d_fault = nullptr;
    // The CSR pattern on the host for the plan builders (host_pattern): the caller's arrays while
    // mspmv_csr_create runs (no copy), else one download shared by every builder of one plan decision and
    // released after it (PatternScope; ADVICE r05: the window, run and slab builders each copied it)
    const int *pat_ro_ext = nullptr, *pat_ci_ext = nullptr;
    std::vector<int> pat_ro, pat_ci;
    bool pat_scope = false;
    // test hook (mspmv_test_poison_tickets): the next CG solve fills its fold tickets with this value
    unsigned poison_value = 0;
    int poison_flags = 0;  // 0: none pending; MSPMV_POISON_* bits
    // CG iteration graph (K iterations), reused while everything it was captured with is unchanged
    hipGraph_t cg_graph = nullptr;
    hipGraphExec_t cg_exec = nullptr;
    std::vector<const void *> cg_graph_key;
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_tile_kernel_ms = 0.0;
    int last_kernels_per_call = 1;
    void *d_flush = nullptr;
    size_t flush_cap = 0;
    mspmv::ResidentCg *rcg = nullptr;  // register-resident CG layout (built on the first single-RHS CG)
    std::string last_cg_kernel;        // the CG path the last solve ran (mspmv_cg_kernel_name)
    // plain single-RHS SpMV on one-wave tiles (a plan of its own, TilePlan::lanes = 64): -1 not
    // decided yet, 0 no, 1 yes (mspmv_api.hip spmv_plan: skewed rows, most tiles merge walks)
    int spmv_onewave = -1;
    // plain single-RHS SpMV on the column-slab plan (mspmv_slab.hip, plan key kSlabPlanKey): -1 not
    // decided yet, 0 no, 1 yes (spmv_plan; MSPMV_SPMV_SLAB)
    int spmv_slab = -1;
    // plain single-RHS SpMV on the run-balanced node-block plan (key kRunPlanKey; mspmv_api.hip
    // spmv_runs_decide): -1 not decided yet, 0 no, 1 yes
    int spmv_runs = -1;
    // plain SpMM of width L (index l_index(L)) on a column-slab plan (key slab_mm_key(L)): -1 not
    // decided yet, 0 no, 1 yes (mspmv_api.hip spmm_slab_decide; MSPMV_SPMM_SLAB)
    int spmm_slab[5] = {-1, -1, -1, -1, -1};
    // plain SpMV / SpMM (every width) and the split CG's SpMM on the offset-window plan (key kDiaPlanKey;
    // mspmv_api.hip dia_decide): -1 not decided yet, 0 no, 1 yes
    int dia = -1;
};

namespace mspmv {
// The handle's CSR pattern on the host (see mspmv_handle_s::pat_*): *ro [m + 1], *ci [nnz]
mspmv_status host_pattern(mspmv_handle_s *h, const int **ro, const int **ci);
bool host_pattern_resident(const mspmv_handle_s *h);  // available without a download
// Holds a downloaded pattern for the duration of one plan decision (the outermost scope releases it).
struct PatternScope {
    mspmv_handle_s *h;
    bool own;
    explicit PatternScope(mspmv_handle_s *hh) : h(hh), own(!hh->pat_scope) { hh->pat_scope = true; }
    ~PatternScope()
    {
        if (own) {
            h->pat_scope = false;
            std::vector<int>().swap(h->pat_ro);
            std::vector<int>().swap(h->pat_ci);
        }
    }
};
}  // namespace mspmv

// IC(0) factor on the device (mspmv_ic0_create): L and its transpose for the two sync-free
// triangular solves of the preconditioner apply, their ready flags and the intermediate Y.
struct mspmv_ic0_s {
    unsigned long long gen = mspmv_next_generation();
    int device = 0;
    int n = 0, nnz = 0;
    int *d_lro = nullptr, *d_lci = nullptr;  // L (lower, diagonal last in each row)
    double *d_lva = nullptr;
    int *d_uro = nullptr, *d_uci = nullptr;  // L^T (upper, diagonal first)
    double *d_uva = nullptr;
    int *d_fwd_order = nullptr;              // [n] rows of L by dependency level (then row): wave w solves row fwd_order[w]
    int *d_bwd_order = nullptr;              // [n] rows of L^T by backward level
    int levels_fwd = 0, levels_bwd = 0;
    int *d_ready = nullptr;                  // [n] per-row ready flags of the running solve
    double *d_y = nullptr;                   // [n * L] forward-solve result
    size_t y_cap = 0;
};

namespace mspmv {

// ---- column-slab SpMV (mspmv_slab.hip) ---------------------------------------------
constexpr int kSlabPlanKey = -1;
constexpr int kRunPlanKey = -2;  // the run-balanced node-block SpMV plan (mspmv_api.hip spmv_runs_decide)
// Builds the column-slab plan into *p (blocks, split rows, reordered stream); MSPMV_ERR_UNSUPPORTED
// when the matrix does not fit the form (rows per block) or its blocks would hold fewer than
// min_nnz_per_block nonzeros on average; p is freed by the caller on any error.
// cfg: the block shape (kSlabCfgs); groups (always for cfg 1): column-group blocks instead of merge-path ones.
mspmv_status build_slab_plan(mspmv_handle_s *h, TilePlan &p, double min_nnz_per_block = 0.0, int cfg = 0,
                             bool groups = false, int num_groups = 0);  // num_groups 0: MSPMV_SLAB_GROUPS or kSlabGroups
void free_slab(SlabData *s);
hipError_t launch_slab(mspmv_handle_s *h, const TilePlan &plan, const double *d_x, double *d_y);
std::string slab_kernel_name(const mspmv_handle_s *h);  // the handle's plain-SpMV slab plan's kernel
// Column-slab SpMM plans (L = 8, 16), keyed apart from every tile plan.
inline int slab_mm_key(int L) { return -(1 << 20) - L; }
const SlabMmCfg &slab_mm_cfg(int L, int which = -1);  // which < 0: the shipped configuration for L
mspmv_status build_slab_mm_plan(mspmv_handle_s *h, int L, TilePlan &p);
// ctrl (CG): the launch returns at once when ctrl->done is set; ld: panel stride (0: L)
hipError_t launch_slab_mm(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L, int ld,
                          const CgControl *ctrl);
std::string slab_mm_kernel_name(const mspmv_handle_s *h, const TilePlan &plan);
mspmv_status plan_split_rows(TilePlan &p, const std::vector<int2> &hb, const std::vector<unsigned char> &hs);

// ---- offset windows (mspmv_dia.hip) -------------------------------------------------
constexpr int kDiaPlanKey = -3;
// Builds the offset-window plan into *p; MSPMV_ERR_UNSUPPORTED when some window does not fit (a row
// longer than kDiaMaxK, more distinct offsets than that, fewer than min_window_fill x rows x K
// nonzeros, or columns not strictly ascending) or the matrix's nonzeros fill less than min_fill of the
// panels; p is freed by the caller on any error.
mspmv_status build_dia_plan(mspmv_handle_s *h, TilePlan &p, double min_fill, double min_window_fill);
void free_dia(DiaData *d);
// Y = A X (L = 1, 2, 4, 8, 16; ld: panel stride, 0 = L); ctrl (CG): return at once when ctrl->done;
// partials (dot mode): also X.(A X) per column per window into partials[windows][L] (launch_fold_dot),
// with the matrix's rows at X row row_off (a row-range view); stream: 0 = the handle's
hipError_t launch_dia(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L, int ld,
                      const CgControl *ctrl, double *partials = nullptr, long long row_off = 0,
                      hipStream_t stream = nullptr);
std::string dia_kernel_name(const mspmv_handle_s *h, int L);
// The pipelined single-RHS CG's SpMV (iteration `parity`) on the windows of `plan` (k_cg1_dia): reads
// {r_k, p_{k-1}} from rp_old, writes p_k into rp_new, Ap into h->d_ap, the deferred x term into d_x and one
// p.Ap partial per workgroup into h->d_partials; *nslots = that count, for k_cg1_update's consumer level.
hipError_t launch_cg1_dia(mspmv_handle_s *h, const TilePlan &plan, const double *rp_old, double *rp_new, double *d_x,
                          int parity, int nblk, double tol, int *nslots);
bool dia_spmm_enabled();  // the L-wide products on the windows too unless MSPMV_DIA_SPMM=0 (mspmv_api.hip)
// The handle's offset-window plan for width L (decided on first use), or null (mspmv_api.hip)
mspmv_status dia_plan_for(mspmv_handle_s *h, int L, const TilePlan **out);
bool dia_dot_fused();     // the window SpMM takes p.Ap in its dot mode unless MSPMV_DIA_DOT=0 (mspmv_kernels.hip)

// ---- launchers (mspmv_kernels.hip) --------------------------------------------------
void set_error(const std::string &msg);
hipError_t launch_merge_coords(const int *d_row_offsets, int m, int nnz, long long diag_step, int num_parts,
                               int2 *d_out, hipStream_t s);
hipError_t launch_tile_modes(const int *d_row_offsets, const int2 *d_bounds, const unsigned char *d_split,
                             int num_tiles, int L, unsigned char *d_modes, hipStream_t s, int lanes = kBlock);
// Items per thread of the single-RHS tiles (the nominal tile is lanes x this)
int spmv_items_per_thread();
inline int l_index(int L) { return L == 1 ? 0 : L == 2 ? 1 : L == 4 ? 2 : L == 8 ? 3 : 4; }
hipError_t launch_snap(const int *d_row_offsets, int m, int2 *d_bounds, unsigned char *d_split, int num_tiles,
                       int snap, hipStream_t s);
// Per-tile 16-bit column offsets (TilePlan::d_colbase / d_cols16); whether plans get them.
hipError_t launch_pack_cols16(const int *d_cols, const int2 *d_bounds, int num_tiles, int *d_colbase,
                              unsigned short *d_cols16, hipStream_t s);
// Node blocks (runs of rows sharing one column list) for the single-RHS plan; needs cols16.
bool spmv_blocks_enabled();
// SpMM (L >= 2) through the single-RHS node-block plan (k_spmm_blk) when all its tiles are register tiles.
bool spmm_blk_enabled();
// Rows per run: at most 6, the column-pair SpMV kernel's value registers (k_spmv_blk<.., 6>); a node
// of 7 or 8 unknowns becomes two runs (a 6-DOF FEM node, pwtk's, is one).
constexpr int kBlkRunRows = 6;
constexpr int kBlkPerTile = 64;  // == kBlkMax in the kernels: descriptor capacity of a tile
// Chunks per tile k_build_blocks may describe for the plain SpMV's column-pair kernel (two rounds of
// its eight half-wave run slots), and the one-round limit of k_spmv_tile's node-block paths.
constexpr int kBlkPlanChunks = 16;
constexpr int kBlkTileChunks = 8;
hipError_t launch_build_blocks(const int *d_row_offsets, const int *d_cols, const int2 *d_bounds,
                               const unsigned char *d_split, const int *d_colbase, int num_tiles, uint4 *d_blk,
                               hipStream_t s, int max_chunks = 8);
hipError_t launch_build_dict(const int *d_cols, const int2 *d_bounds, int num_tiles, int max_items, int *d_dict,
                             int *d_ndict, unsigned short *d_idx16, hipStream_t s, bool multi, int L = 1);
// Multi-RHS column dictionaries: the distinct panel rows a tile parks in LDS, 8 KB per workgroup
// (L = 16: 64 rows), which keeps 7 workgroups per CU; 16 KB (5 per CU) measured 105 vs 102 us and
// 24 KB 119 us on the pwtk shape.
constexpr int kSpmmDictBytes = 16384;  // L = 16: 128 distinct panel rows per 1,024-item tile
constexpr int kSpmmDict8Bytes = 0;     // L = 8 (0: no dictionaries at L = 8)
constexpr int spmm_dict_bytes(int L) { return L == 16 ? kSpmmDictBytes : L == 8 ? kSpmmDict8Bytes : 0; }
constexpr int spmm_dict_max(int L) { return spmm_dict_bytes(L) / (8 * L); }
// y = A x (L == 1) or Y = A X (row-major panels), tile kernel + optional carry fix-up.
hipError_t launch_spmm(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                       int *kernels_launched, int ld = 0);
// dst[i][j] = (j < cols ? src[i][j] : 0) for i < rows, j < dcols (row-major, strides lds / ldd).
hipError_t launch_panel_copy(const double *src, int lds, double *dst, int ldd, long long rows, int cols, int dcols,
                             hipStream_t s);
// ld: panel leading dimension in doubles (0: L, whole panels)
hipError_t launch_spmm_tile_only(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                                 int ld = 0);
// Nominal tile size (merge items per tile) used for L right-hand sides.
int tile_items_for(int L);
// Map key of the default plan for L (one-wave plans are keyed by minus their tile size: 512 is also
// the L = 16 tile size)
// Plans are shared by tile size (the L = 2 SpMM runs on the single-RHS plan), except that the L = 16
// plan, whose 1,024-item tiles equal L = 4's, keeps its own (its column dictionaries).
inline int plan_key(int L) { return L == 16 ? tile_items_for(16) + 1 : tile_items_for(L); }
// Resident single-RHS tile workgroups per CU at the default tile shape (0: non-default tuning).
int spmv_tile_blocks_per_cu();
// STREAM-like nontemporal read of `bytes` (16-B words) on stream s (mspmv_time_stream_read).
hipError_t launch_stream_read(const double *p, size_t bytes, int num_cus, hipStream_t s);
std::string spmv_kernel_name(const mspmv_handle_s *h);
std::string spmm_kernel_name(const mspmv_handle_s *h, const TilePlan &plan, int L);
bool stream_nt(const mspmv_handle_s *h);
bool supported_L(int L);

// CG pieces
hipError_t launch_cg_init(mspmv_handle_s *h, const double *d_b, double *d_x, int L, double tol, int nblk);
// Diagnostic: the plain SpMV's k_spmv_tile in its stamped instantiation (hipErrorNotSupported for plans
// that run another kernel); d_stamps [num_tiles][6] (mspmv_spmv_tile_stamps)
hipError_t launch_spmv_tile_stamped(mspmv_handle_s *h, const TilePlan &plan, const double *d_x, double *d_y,
                                   unsigned long long *d_stamps);
// splan / dot_fused: the split iteration's plain-product plan and window dot mode, resolved once per
// solve by cg_solve_native (launch_cg_iteration_split)
hipError_t launch_cg_iteration(mspmv_handle_s *h, const TilePlan &plan, const TilePlan *splan, bool dot_fused,
                               double *d_x, int L, int parity, int nblk, double tol);
int cg_update_blocks(long long elems, int num_cus);
// Iterations per CG batch / graph replay for an m-row, nnz-nonzero matrix and L columns (mspmv_api.hip).
int cg_batch_iters(long long m, long long nnz, int L);
// Pipelined single-RHS CG (L == 1 unless MSPMV_CG_SPLIT=1): init (x = 0, r = p0 = b, b.b
// partials) and, after the loop, the last stop test (after max_iters iterations) and the last deferred
// x += alpha p (k_cg1_xflush, always); grid of cg1_blocks(m).
bool cg_split_iteration(int L);
int cg1_blocks(long long m);
hipError_t launch_cg1_init(mspmv_handle_s *h, const double *d_b, double *d_x, int nblk);
hipError_t launch_cg1_finish(mspmv_handle_s *h, double *d_x, int parity, int nblk);
// Register-resident single-RHS CG (one launch for the whole solve; MSPMV_CG_RESIDENT=0
// turns it off): the layout is built on first use; r->ok false when the matrix does not fit.
bool cg_resident_enabled();
bool cg_resident_pipelined();  // the resident kernel's iteration form (MSPMV_CG_RESIDENT_FORM)
mspmv_status resident_prepare(mspmv_handle_s *h, ResidentCg **out);
void resident_free(ResidentCg *r);
// d_stamps (diagnostic solves, mspmv_cg_resident_stamps): [stamp_iters][G][5] wall_clock64() phase
// stamps of every workgroup; null otherwise.
hipError_t launch_cg_resident(mspmv_handle_s *h, ResidentCg *r, const double *d_b, double *d_x, int max_iters,
                              double tol, unsigned long long *d_stamps = nullptr, int stamp_iters = 0);
// Split (multi-RHS) CG: the last deferred x += alpha p after the loop (a no-op when none is pending).
hipError_t launch_cg_xflush(mspmv_handle_s *h, double *d_x, int L, int nblk);
// Offset (doubles) and count of the partials level a consumer sums: levels of a fan-in
// kSlotGroup tree are folded while more than `stop` partials would remain.
inline void consumer_level(int nslots, int stop, int L, long long *off, int *count)
{
    long long o = 0;
    int c = nslots;
    while (c > stop) {
        o += (long long)c * L;
        c = (c + kSlotGroup - 1) / kSlotGroup;
    }
    *off = o;
    *count = c;
}

// Row-sharded CG (mspmv_dist.hip).  CgVecArgs lives in the kernels file; the dist code builds
// it through this mirror.
struct DistVecArgs {
    long long n_elems;
    double *x;
    double *r;
    const double *p;
    double *p0;
    const double *ap;
    CgScalars *scal;
    CgControl *ctrl;
    unsigned char *conv;
    double *partials;
    double *hist;
    int hist_cap;
    double tol;
    const double *red_in;
    double *red_out;
    unsigned *gtickets;
    int pcg;
    int lazy_x;  // (single-GPU split CG only: 0 here)
    int rev;
};
// which: 0 init partial sums (b.b -> red_out), 1 init finish (red_in = all-reduced b.b),
// 2 p update, 3 x/r update (alpha from red_in = all-reduced p.Ap; r.r -> red_out),
// 4 finish (red_in = p.Ap, red_out = all-reduced r.r)
hipError_t launch_dist_vec_mirror(int which, const DistVecArgs &a, int L, int nblk, double *p, hipStream_t s);
hipError_t launch_dist_pack(const double *p, const int *idx, long long n_elems, int L, double *send,
                            const CgControl *ctrl, hipStream_t s);
hipError_t launch_spmm_dot(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                           CgControl *ctrl, double *partials, unsigned *gtickets, double *dot_out,
                           CgScalars *scal = nullptr, const unsigned char *conv = nullptr, int fold_mode = -1);
// The two halves of launch_spmm_dot, for SpMMs split over several handles (the row-sharded CG's
// head | interior | tail): each part's tiles write their partials at its offset, one fold sums all.
hipError_t launch_spmm_dot_tiles(mspmv_handle_s *h, const TilePlan &plan, const double *d_X, double *d_Y, int L,
                                 CgControl *ctrl, double *partials, hipStream_t s, long long row_off);
hipError_t launch_fold_dot(int T, int L, double *partials, unsigned *gtickets, double *dot_out, CgScalars *scal,
                           const unsigned char *conv, CgControl *ctrl, int fold_mode, hipStream_t s);
// The tile plan a handle's kernels use for L right-hand sides (built on first use).
mspmv_status plan_for(mspmv_handle_s *h, int L, const TilePlan **out);
// mspmv_csr_create on a stream the caller owns (kept; the handle never destroys it)
mspmv_status csr_create_on_stream(const mspmv_csr_d *host, int device, hipStream_t stream, mspmv_handle *out);
// Rows [row_lo, row_hi) of `parent` as a handle of their own (own stream, row offsets and plans) whose
// columns and values ARE the parent's (no copy; destroy it before the parent).  host_row_offsets: the
// parent's row offsets on the host.
mspmv_status csr_create_view(mspmv_handle parent, int row_lo, int row_hi, const int *host_row_offsets,
                             mspmv_handle *out);
// SPAI-preconditioned block CG (SPAISolveMultiple, work_2025/main/sparse_approximate_inverse.hpp:
// 30-230) on A's handle h with the preconditioner's handle hm (same shape and device): init
// (X = 0, R = B, Z = M R, P = Z, rs_old = R.Z) and one iteration (AP = A P -> alpha; X, R update
// and stop test; Z = M R -> beta; P = Z + beta P).  hm's SpMMs run on h's stream.
hipError_t launch_pcg_init(mspmv_handle_s *h, mspmv_handle_s *hm, const TilePlan &mplan, const double *d_b,
                           double *d_x, int L, double tol, int nblk);
hipError_t launch_pcg_iteration(mspmv_handle_s *h, mspmv_handle_s *hm, const TilePlan &plan, const TilePlan &mplan,
                                double *d_x, int L, int nblk, double tol);
// IC(0)-preconditioned block CG (PCGSolveMultiple, work_2025/main/incomplete_cholesky.hpp:33-199):
// Z = L^-T L^-1 R by two sync-free triangular solves (k_trsv); ic->d_y must hold m * L.
hipError_t launch_pcg_ic0_init(mspmv_handle_s *h, mspmv_ic0_s *ic, const double *d_b, double *d_x, int L, double tol,
                               int nblk);
hipError_t launch_pcg_ic0_iteration(mspmv_handle_s *h, mspmv_ic0_s *ic, const TilePlan &plan, double *d_x, int L,
                                    int nblk, double tol);
// Partials capacity (doubles) and group-ticket count for `slots` partial slots of L columns.
// (every level of the tree: slots, slots/32, ... -> <= slots * 32/31 + one per level)
inline size_t partials_capacity(size_t slots, int L) { return (slots + slots / (kSlotGroup - 1) + 8) * L; }
inline size_t gtickets_capacity(size_t slots) { return (slots / (kSlotGroup - 1) + 8) * kTicketStride; }

}  // namespace mspmv
