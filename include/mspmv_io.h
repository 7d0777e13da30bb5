/*
 * mspmv_io.h -- host-side CSR construction with the reference's exact semantics (part of
 * libmspmv.so, no GPU needed).  Output arrays are malloc'ed; release them with mspmv_host_free.
 */
#ifndef MSPMV_IO_H
#define MSPMV_IO_H

#include "mspmv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* CooMatrix::InitMarket (sparse_matrix.h:211-380) + CsrMatrix::Init (:668-733): banner
 * "symmetric"/"skew"/"array" detection, symmetric expansion without duplicating the diagonal,
 * skew negation, pattern entries = default_value, array format column-major, 1-based ->
 * 0-based, stable (row, col) order with duplicates kept.  Returns MSPMV_ERR_IO where the
 * reference calls exit(1).  Line handling follows std::istream::getline(line, 1024): a line of
 * 1023+ characters or a last line without '\n' ends the parse (:247-252). */
MSPMV_API mspmv_status mspmv_market_read(const char *path, double default_value, int *num_rows, int *num_cols,
                                         int *num_nonzeros, int **row_offsets, int **column_indices,
                                         double **values);

enum { MSPMV_GEN_GRID2D = 0, MSPMV_GEN_GRID3D = 1, MSPMV_GEN_WHEEL = 2, MSPMV_GEN_DENSE = 3 };
/* The reference's generators (sparse_matrix.h:385-623) through CsrMatrix::Init:
 * GRID2D(width, self_loop), GRID3D(width, self_loop), WHEEL(spokes, -), DENSE(rows, cols). */
MSPMV_API mspmv_status mspmv_generate(int kind, int p0, int p1, double default_value, int *num_rows, int *num_cols,
                                      int *num_nonzeros, int **row_offsets, int **column_indices, double **values);

MSPMV_API void mspmv_host_free(void *p);

#ifdef __cplusplus
}
#endif

#endif /* MSPMV_IO_H */
