"""World-1 DistCsr: local SpMV timing vs a plain GpuCsr on the same pwtk-shaped matrix."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "sparse-matrix-linear-equations_amd")]
import mspmv  # noqa: E402

M, NNZ = 217918, 11524432
a = mspmv.CsrMatrix.synth_fem_blocked(M, NNZ, 6, 1700, seed=1)
x = np.random.default_rng(2).uniform(0, 1, M)
with mspmv.GpuCsr(a) as g:
    dx, dy = mspmv.DeviceBuffer.from_array(x), mspmv.DeviceBuffer(8 * M)
    mspmv.time_spmm_batch([g], [dx], [dy], 1, 20)
    st, k, _ = mspmv.time_spmm_batch([g], [dx], [dy], 1, 50)
    print("GpuCsr hot", st, k, g.kernel_name(), g.plan_block_tiles(1), flush=True)
ro = a.row_offsets
rb = mspmv.dist_partition(a, 1)
loc = mspmv.CsrMatrix.synth_fem_blocked_rows(M, NNZ, 6, 1700, 1, 0, M)
d = mspmv.DistCsr(mspmv.comm_unique_id(), 1, 0, 0, rb, loc)
xp = d.x_ext(1)
mspmv.memcpy_h2d_ptr(xp, x)
dy2 = mspmv.DeviceBuffer(8 * M)
for _ in range(3):
    print("dist time_local", d.time_local(dy2, 1, 50), flush=True)
d.spmm_dev(xp, dy2, 1)
with mspmv.GpuCsr(a) as g:
    y = g.spmv(x)
print("dist y == GpuCsr y:", np.array_equal(dy2.download((M,)), y))
d.close()
