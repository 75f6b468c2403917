"""Make tests/golden/laplace_3d_grid.npz: the data of the reference's demos/laplace_3d.grid (an
output of utils/create_3d_laplace.py — firedrake P1, 12^3 cells, anisotropic D, Dirichlet nodes
removed): its CSR arrays, interior node coordinates and the generator parameters from 'extra'.
Read with mlamg.gridio (opcode walk, nothing from the file is executed). Data only: the GPU box
has no /root/reference.

  python tests/golden/make_grid_fixture.py [/root/reference/demos/laplace_3d.grid]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "ml-amg_amd"))

from mlamg import gridio  # noqa: E402


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/demos/laplace_3d.grid"
    A, x, extra = gridio.load_grid(src)
    out = os.path.join(HERE, "laplace_3d_grid.npz")
    np.savez_compressed(out, data=A.data, indices=A.indices.astype(np.int32),
                        indptr=A.indptr.astype(np.int32), x=np.asarray(x, dtype=np.float64),
                        **{k: float(extra[k]) for k in ("theta_y", "theta_z", "eps_x", "eps_y",
                                                        "eps_z", "dim")})
    print(out, A.shape, A.nnz, {k: v for k, v in extra.items() if k != "filename"})


if __name__ == "__main__":
    main()
