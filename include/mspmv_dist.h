/*
 * mspmv_dist.h -- row-block sharded SpMV/SpMM and block CG over several GPUs (one process per
 * GPU), RCCL over xGMI.  Part of libmspmv.so.
 *
 * The reference is single-process OpenMP and has no multi-GPU code; this is the
 * north-star's "matrices shard by row-block across the node's 8 GPUs with an RCCL all-reduce of
 * the CG dot products over xGMI".  Per CG iteration (CGSolveMultiple's recurrence,
 * no_pretreatment.hpp:32-197, unchanged):
 *   p_own = r + beta p_own; pack the owned p rows other ranks reference; grouped
 *   ncclSend/ncclRecv into this rank's halo rows; Ap = A_local [p_own | p_halo] with the
 *   local p.Ap; ncclAllReduce(L doubles); x += alpha p, r -= alpha Ap with the local r.r;
 *   ncclAllReduce(L doubles); one-block convergence / beta step.
 * Everything is stream-ordered on the local handle's stream; the host only polls the
 * convergence flag once per batch of iterations.
 */
#ifndef MSPMV_DIST_H
#define MSPMV_DIST_H

#include "mspmv.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MSPMV_UNIQUE_ID_BYTES 128

typedef struct mspmv_dist_s *mspmv_dist;

/* ---- host planning (no GPU needed) ------------------------------------------------------ */
/* Contiguous row blocks balanced by merge path: row_begin[g] (g = 0..nranks) is the row
 * coordinate of diagonal min(ceil((m+nnz)/nranks) * g, m+nnz) (MergePathSearch,
 * cpu_spmv.cpp:208-235, at GPU granularity), so every rank gets equal rows + nonzeros. */
MSPMV_API mspmv_status mspmv_dist_partition(const int *row_offsets, int num_rows, int num_nonzeros, int nranks,
                                            int *row_begin);

/* Localize rank `rank`'s rows (CSR with GLOBAL column ids, local_row_offsets rebased to 0):
 * columns in [row_begin[rank], row_begin[rank+1]) become 0..n_own-1, every other column
 * n_own + its position among the sorted distinct halo columns.  The nonzero order is kept
 * (so each row is summed in the reference's CSR order).  halo_global (capacity halo_cap;
 * NULL to size) receives the halo columns in that order -- grouped by owner rank, since
 * ranks own ascending row ranges -- and halo_counts[g] how many rank g owns.  Requires a
 * square matrix (columns partitioned like rows). */
MSPMV_API mspmv_status mspmv_dist_localize(const int *row_begin, int nranks, int rank, const int *local_row_offsets,
                                           const int *global_cols, int *local_cols, int *n_halo, int *halo_global,
                                           int halo_cap, int *halo_counts);

/* ---- communicator and sharded matrix ------------------------------------------------------ */
/* Rank 0 creates the RCCL id and the host broadcasts it (torch.distributed, MPI, ...). */
MSPMV_API mspmv_status mspmv_comm_unique_id(unsigned char id[MSPMV_UNIQUE_ID_BYTES]);
/* One communicator per rank (collective: RCCL init), shared by every sharded object on the rank.
 * It owns ONE stream: every object created on it runs its local kernels and all of its collectives
 * there, so a rank's collectives form one sequence in program order -- call the objects' collective
 * functions in the same order on every rank.  (Several communicators with collectives in flight at
 * once can deadlock under RCCL/NCCL; one communicator per rank rules that out.)  Destroy it after
 * every object created on it (MSPMV_ERR_INVALID before). */
typedef struct mspmv_comm_s *mspmv_comm;
MSPMV_API mspmv_status mspmv_comm_create(const unsigned char id[MSPMV_UNIQUE_ID_BYTES], int nranks, int rank,
                                         int device, mspmv_comm *out);
MSPMV_API mspmv_status mspmv_comm_destroy(mspmv_comm c);
/* Collective over all ranks of `c`: localization of this rank's row block (`local_rows`: num_rows =
 * rows owned, num_cols = global columns, GLOBAL column ids), upload, and the halo-exchange plan
 * (request lists exchanged once with RCCL). */
MSPMV_API mspmv_status mspmv_dist_create_on(mspmv_comm c, const int *row_begin, const mspmv_csr_d *local_rows,
                                            mspmv_dist *out);
/* The same on a private communicator (mspmv_comm_create + mspmv_dist_create_on; destroyed with the
 * object).  For one sharded object per rank; several objects on one rank share one mspmv_comm. */
MSPMV_API mspmv_status mspmv_dist_create(const unsigned char id[MSPMV_UNIQUE_ID_BYTES], int nranks, int rank,
                                         int device, const int *row_begin, const mspmv_csr_d *local_rows,
                                         mspmv_dist *out);
MSPMV_API mspmv_status mspmv_dist_destroy(mspmv_dist d);
/* n_own rows owned, n_halo remote rows referenced, n_send owned rows other ranks reference. */
MSPMV_API mspmv_status mspmv_dist_info(mspmv_dist d, int *n_own, int *n_halo, int *n_send);
/* Y_own = (A X)_own with the halo exchange (collective).  Row-major n_own x L panels on the
 * device, any L >= 1.  Where the local rows have an interior (rows referencing owned columns
 * only, >= half the local nonzeros: banded / FEM row blocks), it is multiplied on its own stream
 * while the halo is packed and exchanged, and the rows next to the block ends follow the
 * exchange.  Asynchronous on the local stream (every part joined into it).  Passing
 * mspmv_dist_x_ext's buffer as d_X_own skips the copy of X_own into it. */
MSPMV_API mspmv_status mspmv_dist_spmm_dev(mspmv_dist d, const double *d_X_own, double *d_Y_own, int L);
/* The (n_own + n_halo) x L extended panel the SpMM reads: rows [0, n_own) are X_own (a caller
 * writes them there directly), the rest receives the halo.  Valid until a call with a larger L. */
MSPMV_API mspmv_status mspmv_dist_x_ext(mspmv_dist d, int L, double **d_x_ext);
/* Block until the local stream (and every part joined into it) is idle. */
MSPMV_API mspmv_status mspmv_dist_sync(mspmv_dist d);
/* Local-only SpMM timing, no exchange: `reps` repetitions of the local multiply
 * Y_own = A_local [X_own | X_halo] (whatever the halo rows hold) -- the same head / interior / tail
 * launches the overlapped SpMM makes, back to back on one stream, HIP events around the region;
 * *avg_ms per repetition (the per-rank SpMV time the bench's roofline uses at N > 1). */
MSPMV_API mspmv_status mspmv_dist_time_local_dev(mspmv_dist d, double *d_Y_own, int L, int reps, double *avg_ms);
/* Sharded CGSolveMultiple (collective): B_own / X_own are this rank's rows of the interleaved
 * n x L panels.  Iteration count, history and breakdown semantics as mspmv_dcg_multi, any L >= 1
 * (widths outside 1, 2, 4, 8, 16 as independent column groups, every rank the same groups). */
MSPMV_API mspmv_status mspmv_dist_cg_dev(mspmv_dist d, const double *d_B_own, double *d_X_own, int L,
                                         int max_iters, double tolerance, int *iters, double *max_err_hist,
                                         int hist_cap);
/* Test hook, as mspmv_test_poison_tickets (mspmv.h) for the next sharded CG solve on this rank.  A
 * ticket fault does not stop a rank's kernels; the fault word is all-reduced (max) after every batch
 * of iterations, so every rank stops at the same batch and returns MSPMV_ERR_FAULT. */
MSPMV_API mspmv_status mspmv_dist_test_poison_tickets(mspmv_dist d, unsigned value, int flags);

#ifdef __cplusplus
}
#endif

#endif /* MSPMV_DIST_H */
