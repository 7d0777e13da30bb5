/*
 * mspmv.h -- C-ABI of the MI355X-native merge-path CSR SpMV/SpMM + CG library (libmspmv.so).
 *
 * This is the drop-in boundary for the reference's hot path
 * (YuyaW-0118/Sparse-Matrix-Linear-Equations).  Each entry point names the reference
 * interface it replaces (file:line in the reference checkout).  Plain pointers and sizes
 * only; no C++ or torch types.  The header-only C++ facade in mspmv.hpp re-exposes the
 * reference's own template names (CsrMatrix, OmpMergeCsrmv, OmpMergeCsrmm, CGSolveSingle,
 * CGSolveMultiple) on top of these.
 *
 * Types: values fp64, indices int32 -- CsrMatrix<double,int> (sparse_matrix.h:633-653).
 * Dense multi-vector panels are ROW-MAJOR n x L (X[c*L + j]), the layout of
 * OmpMergeCsrmm / CGSolveMultiple (merge_based.hpp:97-100, utils_multiple.hpp:17).
 *
 * Threading: one handle per host thread.  Work is enqueued on the handle's own HIP
 * stream; *_dev calls are asynchronous with respect to the host (use mspmv_sync);
 * host-pointer calls copy in, compute, copy out and return synchronously.  There is no
 * global mutable state except the thread-local last-error string.
 *
 * Errors: every call returns an mspmv_status; nothing calls exit() (unlike
 * sparse_matrix.h:232,297,305).  mspmv_last_error() describes the last failure on the
 * calling thread.
 */
#ifndef MSPMV_H
#define MSPMV_H

#include <stddef.h>

#ifndef MSPMV_API
#define MSPMV_API __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef enum mspmv_status {
    MSPMV_OK = 0,
    MSPMV_ERR_INVALID = 1,       /* bad argument / shape */
    MSPMV_ERR_HIP = 2,           /* a HIP runtime call failed */
    MSPMV_ERR_OOM = 3,           /* device allocation failed */
    MSPMV_ERR_BREAKDOWN = 4,     /* CG: p.Ap <= 0 or non-finite (the reference has no guard) */
    MSPMV_ERR_RCCL = 5,          /* a collective failed */
    MSPMV_ERR_UNSUPPORTED = 6,   /* e.g. L outside the compiled set */
    MSPMV_ERR_IO = 7,            /* MatrixMarket read/parse failure */
    MSPMV_ERR_STALL = 8,         /* IC(0) apply: a triangular-solve dependency never became ready
                                    (the solve stopped; X is not a solution) */
    MSPMV_ERR_FAULT = 9          /* a cross-workgroup fold ticket drew past its group: its array was
                                    not zero when the launch began, so a fold summed partials not yet
                                    written or never ran (results invalid; a CG solve stops) */
} mspmv_status;

/* Mirror of CsrMatrix<double,int> fields, sparse_matrix.h:648-653.  row_offsets has
 * num_rows+1 entries; column indices sorted within each row as CsrMatrix::Init leaves
 * them (stable_sort by (row,col), sparse_matrix.h:680); duplicates allowed. */
typedef struct mspmv_csr_d {
    int num_rows;
    int num_cols;
    int num_nonzeros;
    const int *row_offsets;
    const int *column_indices;
    const double *values;
} mspmv_csr_d;

typedef struct mspmv_handle_s *mspmv_handle;
/* An IC(0) factor resident on a device (mspmv_ic0_create). */
typedef struct mspmv_ic0_s *mspmv_ic0;

/* Merge-path coordinate (CUB CoordinateT / the reference's int2, types.hpp:3-7). */
typedef struct mspmv_coord {
    int x; /* row index (merge list A = row end offsets) */
    int y; /* nonzero index (merge list B = 0..nnz-1) */
} mspmv_coord;

/* SpmmKernel (work_2025/types.hpp:11-16).  Accepted for signature compatibility; the GPU
 * always runs its merge-path kernel. */
typedef enum mspmv_spmm_kernel { MSPMV_SIMPLE = 0, MSPMV_MERGE = 1, MSPMV_NONZERO_SPLIT = 2 } mspmv_spmm_kernel;

/* ---- library / errors -------------------------------------------------------------- */
MSPMV_API const char *mspmv_last_error(void);
MSPMV_API const char *mspmv_version(void);
/* Number of visible HIP devices (0 when none; never an error). */
MSPMV_API int mspmv_device_count(void);

/* ---- matrix handle ------------------------------------------------------------------ */
/* Upload the CSR once to HBM on `device` and build its merge-path tile plans.  Replaces
 * the per-call partitioning of OmpMergeCsrmv (cpu_spmv.cpp:379-389) and CUB's
 * DeviceSpmvSearchKernel (dispatch_spmv_orig.cuh:99-143): the matrix is immutable, so the
 * partition is computed once.  `host` arrays are only read during the call. */
MSPMV_API mspmv_status mspmv_csr_create(const mspmv_csr_d *host, int device, mspmv_handle *out);
/* Same, from arrays already resident in HBM (copied device-to-device). */
MSPMV_API mspmv_status mspmv_csr_create_dev(const mspmv_csr_d *dev, int device, mspmv_handle *out);
MSPMV_API mspmv_status mspmv_destroy(mspmv_handle h);
MSPMV_API mspmv_status mspmv_shape(mspmv_handle h, int *num_rows, int *num_cols, int *num_nonzeros);
/* Milliseconds spent in mspmv_csr_create (upload + partition), the reference's setup_ms
 * (cpu_spmv.cpp:715-742). */
MSPMV_API double mspmv_setup_ms(mspmv_handle h);
/* Block until all work enqueued on the handle's stream has finished. */
MSPMV_API mspmv_status mspmv_sync(mspmv_handle h);
/* Confine the handle's work to num_cus compute units (spread evenly over the device's CUs, so
 * over its XCDs), or to all of them when num_cus <= 0 or >= the device's count: the handle's
 * stream is replaced by a CU-masked one (hipExtStreamCreateWithCUMask) and launch sizing follows
 * the new count.  The GPU counterpart of the thread count that OpenMP runs take
 * (parallel_efficiency.cpp:67-113 sets omp_set_num_threads per point); tools/parallel_efficiency.py
 * sweeps it, one CU count per process.  One masked stream per (device, count) is created per
 * process and shared by all handles limited to that count (a masked stream holds a hardware
 * queue of its own; a process has few).  Synchronizes the handle first. */
MSPMV_API mspmv_status mspmv_set_cu_limit(mspmv_handle h, int num_cus);

/* ---- merge-path partition ----------------------------------------------------------- */
/* Coordinates of the num_parts+1 partition boundaries exactly as OmpMergeCsrmv computes
 * them: diagonal_t = min(ceil((m+nnz)/P) * t, m+nnz), MergePathSearch over
 * (row_offsets+1, 0..nnz-1) (cpu_spmv.cpp:208-235, :379-389).  Computed on the GPU, one
 * lane per diagonal; bit-exact with the reference.  `coords` has num_parts+1 entries. */
MSPMV_API mspmv_status mspmv_merge_coords(mspmv_handle h, int num_parts, mspmv_coord *coords);

/* ---- SpMV / SpMM -------------------------------------------------------------------- */
/* y = A x   (OmpMergeCsrmv, cpu_spmv.cpp:357-421; cub::DeviceSpmv::CsrMV with alpha=1,
 * beta=0, device_spmv.cuh:129-164).  Host pointers: x[num_cols], y[num_rows]. */
MSPMV_API mspmv_status mspmv_dspmv(mspmv_handle h, const double *x, double *y);
/* Device pointers, asynchronous on the handle's stream. */
MSPMV_API mspmv_status mspmv_dspmv_dev(mspmv_handle h, const double *d_x, double *d_y);
/* Y = A X for L right-hand sides, row-major panels (OmpMergeCsrmm, merge_based.hpp:46-153).
 * Any L >= 1: the tile kernels run widths 1, 2, 4, 8, 16; other even L run as column chunks of
 * those widths over the same panels (stride L), odd L > 1 through a copy padded to L + 1
 * columns.  Even-L panels must be 16-byte aligned. */
MSPMV_API mspmv_status mspmv_dspmm(mspmv_handle h, const double *X, double *Y, int L);
MSPMV_API mspmv_status mspmv_dspmm_dev(mspmv_handle h, const double *d_X, double *d_Y, int L);

/* ---- CG ----------------------------------------------------------------------------- */
/* Single-RHS CG, CGSolveSingle (work_2025/main/single_strategy.hpp:102-170): x0 = 0,
 * r = p = b; stop after the update of r when sqrt(r.r)/||b|| < tolerance, counting that
 * iteration; ||b|| == 0 -> 1.  `tolerance` has the reference's meaning (callers such as
 * cpu_singlecg.cpp:92,101 pass tol*||b||; that quirk is the caller's).  Returns the
 * iteration count in *iters.  resid_hist (optional, capacity hist_cap) receives
 * sqrt(r.r)/||b|| per iteration.  Host pointers b[n], x[n]. */
MSPMV_API mspmv_status mspmv_dcg_single(mspmv_handle h, const double *b, double *x, int max_iters, double tolerance,
                              int *iters, double *resid_hist, int hist_cap);
MSPMV_API mspmv_status mspmv_dcg_single_dev(mspmv_handle h, const double *d_b, double *d_x, int max_iters, double tolerance,
                                  int *iters, double *resid_hist, int hist_cap);
/* Diagnostic (measurement of configs[3]'s kernel): one register-resident single-RHS solve, as
 * mspmv_dcg_single_dev on device vectors, that also records wall_clock64() (a constant 100 MHz
 * clock) at five phase boundaries of every workgroup's iterations k < stamp_iters:
 * stamps[(k * G + w) * 5 + i], i = 0 iteration start, 1 the workgroup's rows of Ap done, 2 the
 * p.Ap total received, 3 the workgroup's r update done, 4 the r.r total received (entries of
 * iterations not run stay 0).  stamps holds stamp_iters * G * 5 values; *workgroups = G.
 * MSPMV_ERR_UNSUPPORTED when the matrix does not take the resident path.  No reference
 * counterpart (CGSolveSingle has no instrumentation). */
MSPMV_API mspmv_status mspmv_cg_resident_stamps(mspmv_handle h, const double *d_b, double *d_x, int max_iters,
                                                double tolerance, int *iters, unsigned long long *stamps,
                                                int stamp_iters, int *workgroups);
/* Block multi-RHS CG, CGSolveMultiple (work_2025/main/no_pretreatment.hpp:32-197): L
 * lock-step recurrences on interleaved n x L panels, per-column converged masks
 * (alpha = beta = 0 once converged), stop when all columns converged.  Breakdown is per
 * column: a column whose p.Ap gives a non-finite alpha (e.g. a zero RHS column, 0/0) is frozen
 * at its last finite iterate and left out of the history (the reference's column turns NaN and
 * never converges); the other columns keep iterating, and the call returns
 * MSPMV_ERR_BREAKDOWN with X holding every column's result.  max_err_hist
 * (optional) receives the per-iteration max over ALL columns of sqrt(r.r)/||b||
 * (:132-155).  Any L >= 1: widths outside {1, 2, 4, 8, 16} are solved as independent column
 * groups of those widths (the recurrences are per column), iteration count = the groups'
 * maximum, history = the max over groups with finished groups frozen, as the reference's. */
MSPMV_API mspmv_status mspmv_dcg_multi(mspmv_handle h, const double *B, double *X, int L, int max_iters, double tolerance,
                             mspmv_spmm_kernel kernel, int *iters, double *max_err_hist, int hist_cap);
MSPMV_API mspmv_status mspmv_dcg_multi_dev(mspmv_handle h, const double *d_B, double *d_X, int L, int max_iters,
                                 double tolerance, mspmv_spmm_kernel kernel, int *iters, double *max_err_hist,
                                 int hist_cap);

/* ---- SPAI-preconditioned block CG ---------------------------------------------------- */
/* SPAI preconditioner M with A's own pattern, SparseApproximateInversion
 * (work_2025/cg/sparse_approximate_inversion.hpp:40-321): column k of M minimises
 * ||A(I,J) m - e_k(I)||_2 (J = rows of A's column k, I = rows those columns touch; Householder
 * QR where the reference calls LAPACKE_dgels; a rank-deficient column gives zeros, as the
 * reference's info != 0 fallback), then M = (M + M^T)/2 over the pattern.  Host setup
 * (OpenMP), like the reference's; m_values[num_nonzeros] receives M's values in A's CSR order,
 * so M's CSR is (A.row_offsets, A.column_indices, m_values).  Square A only. */
MSPMV_API mspmv_status mspmv_spai_values(const mspmv_csr_d *a, double *m_values);
/* SPAISolveMultiple (work_2025/main/sparse_approximate_inverse.hpp:30-230) on the GPU: X = 0,
 * R = B, Z = M R, P = Z, rs_old = R.Z; per iteration AP = A P, alpha = rs_old/P.AP (0 when
 * converged or P.AP == 0), X += alpha P, R -= alpha AP, stop test on sqrt(R.R)/||B_j|| with the
 * per-column masks and the max-over-columns history, Z = M R, beta = R.Z/rs_old (0 when converged
 * or rs_old == 0), P = Z + beta P.  `m` is M's handle (same shape and device as `a`); both SpMMs
 * are merge-path tile kernels.  Any L >= 1 (column groups as mspmv_dcg_multi); interleaved
 * n x L panels. */
MSPMV_API mspmv_status mspmv_dpcg_spai_multi(mspmv_handle a, mspmv_handle m, const double *B, double *X, int L,
                                             int max_iters, double tolerance, mspmv_spmm_kernel kernel, int *iters,
                                             double *max_err_hist, int hist_cap);
MSPMV_API mspmv_status mspmv_dpcg_spai_multi_dev(mspmv_handle a, mspmv_handle m, const double *d_B, double *d_X,
                                                 int L, int max_iters, double tolerance, mspmv_spmm_kernel kernel,
                                                 int *iters, double *max_err_hist, int hist_cap);

/* ---- IC(0)-preconditioned block CG --------------------------------------------------- */
/* IncompleteCholesky (work_2025/cg/incomplete_cholesky_decomp.hpp:84-201) on the host, as in the
 * reference: L has A's lower-triangle pattern (diagonal included, A's CSR order); on a
 * non-positive pivot the factorization restarts with the diagonal shifted by 1e-3, x10 per
 * attempt, 20 attempts (MSPMV_ERR_BREAKDOWN after that).  mspmv_ic0_nnz gives L's nonzero count;
 * l_row_offsets[n+1], l_cols / l_vals[nnz_l] receive L; *shift (nullable) the shift used. */
MSPMV_API mspmv_status mspmv_ic0_nnz(const mspmv_csr_d *a, int *nnz_l);
MSPMV_API mspmv_status mspmv_ic0_factor(const mspmv_csr_d *a, int *l_row_offsets, int *l_cols, double *l_vals,
                                        double *shift);
/* TransposeCsr (work_2025/cg/incomplete_cholesky_decomp.hpp:11-78) on the host: out_row_offsets
 * [num_cols+1], out_cols / out_vals [num_nonzeros] receive A^T in CSR, each row's entries in
 * ascending column order (the reference's counting sort). */
MSPMV_API mspmv_status mspmv_csr_transpose(const mspmv_csr_d *in, int *out_row_offsets, int *out_cols,
                                           double *out_vals);
/* Upload L and its transpose (TransposeCsr, :11-78) for the GPU triangular solves. */
MSPMV_API mspmv_status mspmv_ic0_create(const mspmv_csr_d *l, int device, mspmv_ic0 *out);
MSPMV_API mspmv_status mspmv_ic0_destroy(mspmv_ic0 m);
/* PCGSolveMultiple (work_2025/main/incomplete_cholesky.hpp:33-199) on the GPU: Z = L^-T L^-1 R by
 * two sync-free triangular solves per application (one wave per row, per-row ready flags),
 * merge-path SpMM for A P, the reference's masks and max-residual history.  A stalled solve
 * (a dependency never ready) stops the iteration and is reported as MSPMV_ERR_STALL, never a
 * hang.  mspmv_ic0_create rejects a factor with an entry above the diagonal or a row without
 * its diagonal (either would make a solve wait forever). */
MSPMV_API mspmv_status mspmv_dpcg_ic0_multi(mspmv_handle a, mspmv_ic0 m, const double *B, double *X, int L,
                                            int max_iters, double tolerance, mspmv_spmm_kernel kernel, int *iters,
                                            double *max_err_hist, int hist_cap);
MSPMV_API mspmv_status mspmv_dpcg_ic0_multi_dev(mspmv_handle a, mspmv_ic0 m, const double *d_B, double *d_X, int L,
                                                int max_iters, double tolerance, mspmv_spmm_kernel kernel,
                                                int *iters, double *max_err_hist, int hist_cap);

/* ---- measurement helpers (HIP events on the handle's stream) ------------------------ */
/* Enqueue `reps` back-to-back SpMV (L == 1) or SpMM launches on device buffers and return
 * the average milliseconds per call measured by hipEvents on the handle's stream.
 * flush_bytes > 0 sweeps a scratch buffer of that many bytes before every call (outside the
 * timed events) to evict the 256 MiB Infinity Cache ("cold" protocol): a
 * nontemporal read sweep, so the caches hold clean unrelated lines (MSPMV_FLUSH=write: a write
 * sweep, whose dirty lines the timed call would pay to write back). */
MSPMV_API mspmv_status mspmv_time_spmm_dev(mspmv_handle h, const double *d_X, double *d_Y, int L, int reps,
                                 size_t flush_bytes, double *avg_ms);
/* Batch form for benchmarks: `reps` steps, each step one SpMM launch per handle (all handles
 * on one device), every launch enqueued back to back on hs[0]'s stream, HIP events only
 * around the whole region.  *step_ms = average event time per step; *tile_kernel_ms =
 * average duration of one merge tile kernel launch: region time / launches when a step holds
 * only tile kernels (the launch boundary included), else from a second pass that brackets
 * every tile launch with events; *kernels_per_step = launches per step (tile + fix-up). */
MSPMV_API mspmv_status mspmv_time_spmm_batch_dev(int count, const mspmv_handle *hs, const double *const *d_X,
                                                 double *const *d_Y, int L, int reps, double *step_ms,
                                                 double *tile_kernel_ms, int *kernels_per_step);
/* The practical HBM ceiling the roofline fraction is read against: a STREAM-like
 * nontemporal read of a `bytes` buffer (>= 1 MiB; use >> 256 MiB so the Infinity Cache cannot hold
 * it) on `device`, one contiguous slice per workgroup (the fastest read shape measured: ~6.9 TB/s
 * at 1 GiB), `reps` timed passes after one warm-up, HIP events around the timed region.
 * *gbps = bytes x reps / time. */
MSPMV_API mspmv_status mspmv_time_stream_read(int device, size_t bytes, int reps, double *gbps);
/* Per-kernel average duration (ms) of the dominant (merge tile) kernel over the last
 * mspmv_time_spmm_dev call, and the number of kernels per SpMV/SpMM call. */
MSPMV_API mspmv_status mspmv_last_kernel_ms(mspmv_handle h, double *tile_kernel_ms, int *kernels_per_call);

/* ---- diagnostics ---------------------------------------------------------------------- */
/* The tile plan the L-column kernels use: *num_tiles tiles of nominal *tile_items merge
 * items; `bounds` (nullable, num_tiles+1 entries) receives the boundary coordinates after
 * row snapping, *num_carries the number of boundaries a carry crosses.  Lets tests locate
 * exactly which rows are split between threads (those are within tolerance, the rest are
 * bit-identical to SpmvGold). */
MSPMV_API mspmv_status mspmv_tile_plan(mspmv_handle h, int L, int *num_tiles, int *tile_items, int *num_carries,
                                       mspmv_coord *bounds);
/* Single-RHS plan: how many tiles stream 16-bit column offsets (*tiles_cols16) and how many
 * gather x through a per-tile column dictionary (*tiles_dict: tiles whose scattered columns
 * make direct gathers line-bound; the sorted distinct columns are gathered once into LDS).
 * Either output may be null. */
MSPMV_API mspmv_status mspmv_tile_streams(mspmv_handle h, int *tiles_cols16, int *tiles_dict);
/* The L-column plan's tiles that carry a column dictionary (*tiles_dict).  L = 1: as
 * mspmv_tile_streams.  L = 16: the SpMM parks each such tile's distinct panel rows in LDS and
 * reads them there (row-group tiles with at most 64 distinct columns, each repeated >= 2
 * times on average); other widths build none (0). */
MSPMV_API mspmv_status mspmv_plan_dict_tiles(mspmv_handle h, int L, int *tiles_dict);
/* Tiles of the L-column plan staged by node blocks (*tiles_blk): runs of consecutive rows whose
 * column lists are prefixes of one list (FEM unknowns of one mesh node) read that list once and
 * gather each of its x entries once for all the run's rows.  Runs <= 64 columns wide are summed
 * in registers by a fixed lane tree (tile mode 255); wider ones go through the striped path's
 * LDS slots and reduction (bit-identical to it).  Tiles that hold whole rows only, <= 16 run
 * chunks, mean run height >= ~1.7 (others: 0). */
MSPMV_API mspmv_status mspmv_plan_block_tiles(mspmv_handle h, int L, int *tiles_blk);
/* Each tile's in-tile reduction for L right-hand sides (num_tiles entries; 255 = a node-block
 * tile summed in registers by a fixed lane tree, see mspmv_plan_block_tiles): 0 = merge walk
 * (one walker per thread, or per L/2 lanes), g > 0 = row groups with 2^(g-1) nonzero-parallel
 * lanes per row (times L/2 column-pair lanes for L > 1).  g = 1 sums each row sequentially in
 * CSR order -> bit-identical to SpmvGold / the row-split SpMM for rows the tile holds whole. */
MSPMV_API mspmv_status mspmv_tile_modes(mspmv_handle h, int L, unsigned char *modes);
/* Threads that share one tile of the plan the plain L-column product runs on (*lanes): 256, or 64
 * for a single-RHS matrix whose rows are skewed (most workgroup tiles would be merge walks), which
 * the plain SpMV runs on one-wave tiles of 512 merge items.  A merge-walk tile gives each of its
 * lanes (L = 1) ceil(items / lanes) consecutive merge items -- what mspmv_tile_plan's readers
 * need to tell the rows summed sequentially from the split ones. */
MSPMV_API mspmv_status mspmv_tile_lanes(mspmv_handle h, int L, int *lanes);
/* Offset windows (host planning only, no device needed): whether a CSR matrix fits the plan the plain
 * SpMV takes by default for structured-grid rows -- 64-row windows, each keeping the offsets col - row
 * that at least 8 of its rows hold (all rows when it has fewer; <= 64 offsets, the most frequent),
 * dropping its rarest while its kept entries fill less than min_window_fill of rows x offsets; every
 * other entry goes to the plan's remainder (summed after the row's offsets).  Every row's columns
 * must ascend strictly.  The plan holds when the kept entries fill >= min_fill of the
 * windows' 64 x sum K slots and the remainder is at most 5 % of the nonzeros (any share when min_fill
 * is 0: the forced plan).  The library's automatic choice uses 0.85 / 0.30.  *ok = 1 when the plan
 * holds; then *num_windows = ceil(m / 64), *sum_offsets = the offsets over all windows,
 * *masked_windows = windows where some row lacks a kept offset (or that hold fewer than 64 rows),
 * *remainder (nullable) = the remainder's entries; k_per_window (nullable, num_windows entries)
 * receives each window's offset count.  Outputs other than *ok are 0 when the plan does not hold. */
MSPMV_API mspmv_status mspmv_offset_windows(const mspmv_csr_d *a, double min_fill, double min_window_fill, int *ok,
                                            int *num_windows, long long *sum_offsets, int *masked_windows,
                                            int *k_per_window, long long *remainder);
/* Diagnostic (the small-matrix SpMV's per-tile phases): one plain SpMV y = A x on device
 * vectors through the stamped instantiation of the merge-tile kernel k_spmv_tile, whose thread 0 records
 * wall_clock64() (a constant 100 MHz clock) per tile: stamps[t * 6 + i], i = 0 entry, 1 stream and x
 * gathers issued, 2 staged products in LDS (stream and gathers landed), 3 row ends in LDS, 4 rows reduced
 * and stored, 5 the HW_ID register of the CU that ran it.  flush_bytes > 0: the cold protocol's read
 * sweep of that many bytes first (as mspmv_time_spmm_dev).  stamps NULL: only *num_tiles.
 * MSPMV_ERR_UNSUPPORTED when the matrix's plain SpMV runs another kernel (node blocks, windows, slabs,
 * one-wave tiles).  No reference counterpart. */
MSPMV_API mspmv_status mspmv_spmv_tile_stamps(mspmv_handle h, const double *d_x, double *d_y, size_t flush_bytes,
                                              unsigned long long *stamps, int *num_tiles);
/* The single-RHS SpMV kernel instantiation launched for this matrix (tuning read once from
 * the MSPMV_SPMV_* environment; nontemporal matrix loads above 128 MiB), e.g.
 * "k_spmv_tile<8,0,true>" -- the name rocprofv3 reports.  Valid until the next call on this
 * thread. */
MSPMV_API const char *mspmv_spmv_kernel_name(mspmv_handle h);
/* The same for a plain SpMM with L right-hand sides (builds the plan for L if needed): e.g.
 * "k_spmm_blk<16,0,false,6>" on a node-block plan, "k_spmm_tile<8,16,0,true>" elsewhere; widths
 * outside 1, 2, 4, 8, 16 name their widest column chunk's kernel.  "" on error. */
MSPMV_API const char *mspmv_spmm_kernel_name(mspmv_handle h, int L);
/* The CG path the last solve on this handle ran: "k_cg_resident<RPT,NZR> x G" (single RHS, the
 * matrix register/LDS-resident on every CU, one cooperative launch per solve), "pipelined (...)"
 * (single RHS, two kernels per iteration), or the split multi-RHS / PCG forms.  "" before any. */
MSPMV_API const char *mspmv_cg_kernel_name(mspmv_handle h);

/* ---- fault detection ----------------------------------------------------------------- */
/* The kernels' cross-workgroup folds (CG dot products, rows split between tiles, column groups) are
 * closed by the last arrival on a self-resetting ticket.  An arrival that draws past its group (the
 * ticket was not 0 when the launch began) raises a fault word.  CG solves return MSPMV_ERR_FAULT
 * themselves; for products, the host-pointer calls check after their copy-back and *_dev callers
 * call this: it synchronizes the handle's stream, clears the word and returns MSPMV_ERR_FAULT if any
 * product since the last check raised it.  No reference counterpart (OpenMP reductions need none). */
MSPMV_API mspmv_status mspmv_check_faults(mspmv_handle h);
/* Test hook: the next CG solve on h fills its fold tickets with `value` after its init, before its first
 * iteration (MSPMV_POISON_FILL), optionally zeroes them again after the first iteration is enqueued
 * (MSPMV_POISON_LATE_ZERO: the ordering of round 5's unordered null-stream memset) and optionally
 * records the fault without stopping (MSPMV_POISON_NO_STOP: the solve runs to its stop test and then
 * returns MSPMV_ERR_FAULT with the iteration count it reached).  One solve only. */
enum { MSPMV_POISON_FILL = 1, MSPMV_POISON_LATE_ZERO = 2, MSPMV_POISON_NO_STOP = 4 };
MSPMV_API mspmv_status mspmv_test_poison_tickets(mspmv_handle h, unsigned value, int flags);

/* ---- device memory helpers (so hosts need no HIP headers) ---------------------------- */
MSPMV_API mspmv_status mspmv_device_malloc(int device, size_t bytes, void **d_ptr);
MSPMV_API mspmv_status mspmv_device_free(void *d_ptr);
MSPMV_API mspmv_status mspmv_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes);
MSPMV_API mspmv_status mspmv_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes);
MSPMV_API mspmv_status mspmv_memcpy_d2d(void *d_dst, const void *d_src, size_t bytes);
MSPMV_API mspmv_status mspmv_memset_dev(void *d_dst, int byte_value, size_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* MSPMV_H */
