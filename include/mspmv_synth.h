/*
 * mspmv_synth.h -- deterministic synthetic CSR generators for the benchmark shapes
 * (SURVEY 8(d)): SuiteSparse matrices are not available offline, so bench.py and the
 * tests build matrices of the same shapes.  Host-only (OpenMP), part of libmspmv.so.
 * Every value is a pure function of (seed, index) via splitmix64, independent of the
 * thread count.
 */
#ifndef MSPMV_SYNTH_H
#define MSPMV_SYNTH_H

#include "mspmv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Banded non-symmetric pattern (cant / pwtk / rma10 shapes): exactly `nnz` nonzeros, row i
 * holding floor((i+1)nnz/m) - floor(i nnz/m) of them, one per equal slice of the band
 * [i-half_band, i+half_band] (clamped), so columns are unique and sorted; values
 * U(0.5, 1.5).  Arrays: row_offsets[m+1], cols[nnz], vals[nnz] (caller-allocated).
 * Requires half_band >= the longest row. */
MSPMV_API mspmv_status mspmv_synth_banded(int m, long long nnz, int half_band, unsigned long long seed, int *row_offsets,
                                int *cols, double *vals);

/* Node-blocked FEM pattern (pwtk / cant / rma10 are FEM/CFD matrices with several unknowns
 * per mesh node): rows are grouped in nodes of `block` consecutive rows; every row of node I
 * couples to the same set of neighbour nodes, chosen one per equal slice of the node band
 * [I - half_band_nodes, I + half_band_nodes] (own node always included), and takes all
 * `block` columns of each neighbour, so columns come in runs of `block` consecutive indices.
 * Exactly `nnz` nonzeros (row i holds floor((i+1)nnz/m) - floor(i nnz/m), the last
 * neighbour block truncated); values U(0.5, 1.5).  Requires half_band_nodes*2+1 >= the
 * number of blocks the longest row needs. */
MSPMV_API mspmv_status mspmv_synth_fem_blocked(int m, long long nnz, int block, int half_band_nodes,
                                               unsigned long long seed, int *row_offsets, int *cols, double *vals);

/* Rows [row_lo, row_hi) of the same matrix, for row-block sharding without building the whole
 * matrix on every rank: row_offsets[row_hi - row_lo + 1] rebased to 0, GLOBAL column ids, every
 * (row, position) holding the value mspmv_synth_fem_blocked gives it.  cols / vals may be NULL
 * to size (row_offsets only). */
MSPMV_API mspmv_status mspmv_synth_fem_blocked_rows(int m, long long nnz, int block, int half_band_nodes,
                                                    unsigned long long seed, int row_lo, int row_hi,
                                                    int *row_offsets, int *cols, double *vals);

/* An imperfect node-blocked FEM pattern (real FEM matrices are not all regular): nodes of `block`
 * unknowns, a fraction odd_node_frac of them with block - 1 or block + 1 instead (half each); node
 * I's pattern is every unknown of its neighbour nodes (chosen as mspmv_synth_fem_blocked chooses
 * them, in node-index space), row i takes the first min(floor((i+1)nnz/m) - floor(i nnz/m),
 * |pattern|) of them, and a fraction extra_row_frac of rows gets one more column of the node band
 * that the pattern lacks, in order.  Columns unique and sorted per row; values U(0.5, 1.5).
 * Call with cols/vals NULL to size (row_offsets and *nnz_out). */
MSPMV_API mspmv_status mspmv_synth_fem_perturbed(int m, long long nnz, int block, int half_band_nodes,
                                                 double odd_node_frac, double extra_row_frac,
                                                 unsigned long long seed, int *row_offsets, int *cols,
                                                 double *vals, long long *nnz_out);

/* Power-law row lengths with the same contract as mspmv_synth_banded: row lengths drawn
 * from a Zipf-like law (a handful of rows hold a large share of nnz), columns spread over
 * the whole matrix.  Exercises merge-path load balance and long-row carries. */
MSPMV_API mspmv_status mspmv_synth_powerlaw(int m, int n, long long nnz, double exponent, unsigned long long seed,
                                  int *row_offsets, int *cols, double *vals);

/* SPD stencils (symmetric pattern, off-diagonals -U(0,1) symmetric in (i,j), diagonal =
 * sum|off| + diag_shift -> strictly diagonally dominant for diag_shift > 0; a small shift
 * gives the FEM-like condition numbers (hundreds to thousands of CG iterations).
 *   kind 0: 2-D 7-point triangular-mesh stencil (P1 FEM; parabolic_fem shape) on a grid
 *           `dim0` wide with m points in row-major order (last grid row may be partial);
 *   kind 1: 3-D 27-point stencil on dim0 x dim1 x dim2 (nlpkkt120-sized, made SPD).
 * Call with row_offsets only (cols/vals NULL) to size: fills row_offsets and *nnz_out. */
MSPMV_API mspmv_status mspmv_synth_stencil(int kind, int m, int dim0, int dim1, int dim2, unsigned long long seed,
                                           double diag_shift, int *row_offsets, int *cols, double *vals,
                                           long long *nnz_out);

/* The kind-1 27-point SPD stencil on dim0 x dim1 x dim2 made imperfect (a shape the
 * offset windows were not designed on): each row gains one column at a random position within
 * +-2 dim0 dim1 of the diagonal with probability extra_frac, and eight such columns with probability
 * long_frac (rows of up to 36 entries); added values -U(0,1), columns sorted per row.  Not symmetric. */
MSPMV_API mspmv_status mspmv_synth_stencil_perturbed(int dim0, int dim1, int dim2, unsigned long long seed,
                                                     double diag_shift, double extra_frac, double long_frac,
                                                     int *row_offsets, int *cols, double *vals, long long *nnz_out);

/* KKT-shaped saddle-point matrix, nlpkkt120's block structure [[H, B^T], [B, -eps I]] with grid blocks:
 * H = the SPD 27-point stencil (kind 1, diag_shift) on the N = dim0 dim1 dim2 grid, B = a 7-point grid
 * operator (diagonal 1 + U(0,1), neighbours -U(0,1)/6).  m = 2 N (120 x 120 x 123: nlpkkt120's
 * 3,542,400 rows); rows < N hold 27 + 7 entries, rows >= N 7 + 1.  Symmetric indefinite. */
MSPMV_API mspmv_status mspmv_synth_kkt(int dim0, int dim1, int dim2, unsigned long long seed, double diag_shift,
                                       double eps, int *row_offsets, int *cols, double *vals, long long *nnz_out);

#ifdef __cplusplus
}
#endif

#endif /* MSPMV_SYNTH_H */
