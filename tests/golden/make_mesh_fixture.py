"""Make tests/golden/cylflow_highres_mesh.npz: the node coordinates and element connectivity of
the reference's mesh/cylflow-highres.msh (the C3 input), parsed with this
repo's gmsh reader (mlamg.mesh.read_gmsh). Data only: the GPU box has no /root/reference.

  python tests/golden/make_mesh_fixture.py [/root/reference/mesh/cylflow-highres.msh]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "ml-amg_amd"))

from mlamg import mesh  # noqa: E402


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/mesh/cylflow-highres.msh"
    m = mesh.read_gmsh(src)
    out = os.path.join(HERE, "cylflow_highres_mesh.npz")
    np.savez_compressed(out, points=m.points, triangle=m.cells["triangle"].astype(np.int32),
                        line=m.cells["line"].astype(np.int32))
    print(out, m.points.shape, {k: v.shape for k, v in m.cells.items()})


if __name__ == "__main__":
    main()
