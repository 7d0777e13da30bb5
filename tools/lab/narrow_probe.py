"""Node blocks on narrow runs: SpMV kernel time with blocks on/off (run twice, MSPMV_SPMV_BLOCKS=0/1)."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "sparse-matrix-linear-equations_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests")]
import mspmv  # noqa: E402
from test_gpu_blocks import kron_fem, kron_fem9  # noqa: E402

for name, make in (("kron5pt_3", lambda: kron_fem(600, 600, 3)), ("kron5pt_6", lambda: kron_fem(400, 400, 6)),
                   ("kron9pt_5", lambda: kron_fem9(330, 330, 5)), ("kron9pt_6", lambda: kron_fem9(300, 300, 6))):
    a = make()
    dof = name
    x = np.random.default_rng(1).uniform(0, 1, a.num_cols)
    with mspmv.GpuCsr(a) as g:
        dx, dy = mspmv.DeviceBuffer.from_array(x, 0), mspmv.DeviceBuffer(8 * a.num_rows, 0)
        g.time_spmm(dx, dy, 1, 20)
        _, k, _ = g.time_spmm(dx, dy, 1, 200)
        print(f"blocks={os.environ.get('MSPMV_SPMV_BLOCKS', '1')} dof={dof} m={a.num_rows} nnz={a.num_nonzeros} "
              f"blk_tiles={g.plan_block_tiles(1)}/{g.tile_plan(1)['num_tiles']} kernel={g.kernel_name()} us={k*1e3:.2f} "
              f"GBps={(12*a.num_nonzeros+20*a.num_rows)/k/1e6:.0f}", flush=True)
