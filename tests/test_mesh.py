"""CPU: gmsh reader, P1 assembly and red refinement for the C3/C5 inputs (mlamg.mesh).
The assembled matrix itself is "parity unpinned" against pyamg.gallery.fem (pyamg absent): the
checks here are the finite-element identities and the reference's own mesh counts (SURVEY.md §8a:
13,072 nodes, 25,600 triangles, 544 boundary nodes, 12,528 interior DoF)."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "cylflow_highres_mesh.npz")
REF_MSH = "/root/reference/mesh/cylflow-highres.msh"


def _area(tri):
    d1, d2 = tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]
    return 0.5 * np.abs(d1[:, 0] * d2[:, 1] - d1[:, 1] * d2[:, 0]).sum()

SQUARE = """$MeshFormat
4.1 0 8
$EndMeshFormat
$Nodes
2 4 1 4
2 1 0 3
1
2
4
0 0 0
1 0 0
0 1 0
0 0 0 1
3
1 1 0
$EndNodes
$Elements
2 6 1 6
1 1 1 4
1 1 2
2 2 3
3 3 4
4 4 1
2 1 2 2
5 1 2 3
6 1 3 4
$EndElements
"""


def test_unit_square_stiffness():
    from mlamg import mesh
    m = mesh.read_gmsh(SQUARE)
    # node tags 1,2,4,3 in file order -> indices 0,1,2,3; tag 3 = (1,1) is index 3
    assert np.allclose(m.points[:, :2], [[0, 0], [1, 0], [0, 1], [1, 1]])
    assert m.cells["triangle"].tolist() == [[0, 1, 3], [0, 3, 2]]
    assert len(m.cells["line"]) == 4
    K = mesh.p1_stiffness(m.points, m.cells["triangle"]).toarray()
    # (0,0) (1,0) (0,1) (1,1): the diagonal split through (0,0)-(1,1)
    ref = np.array([[1.0, -0.5, -0.5, 0.0], [-0.5, 1.0, 0.0, -0.5],
                    [-0.5, 0.0, 1.0, -0.5], [0.0, -0.5, -0.5, 1.0]])
    assert np.allclose(K, ref, atol=1e-15)
    # all nodes are boundary nodes -> empty Dirichlet system
    A, pts = mesh.poisson_dirichlet(m)
    assert A.shape == (0, 0) and pts.shape == (0, 2)


def test_cylflow_fixture_counts_and_fem_identities():
    from mlamg import mesh
    m = mesh.load_npz(FIXTURE)
    assert m.points.shape == (13072, 3)
    assert m.cells["triangle"].shape == (25600, 3)
    assert len(np.unique(m.cells["line"])) == 544
    K = mesh.p1_stiffness(m.points, m.cells["triangle"])
    assert abs(K - K.T).max() <= 1e-12
    assert np.abs(K @ np.ones(K.shape[0])).max() <= 1e-12          # constants in the kernel
    xy = m.points[:, :2]
    # sum over elements of |T| equals the domain area = x^T K x / |grad x|^2 for x = linear fn
    lin = xy[:, 0]
    area = lin @ (K @ lin)
    tri = xy[m.cells["triangle"]]
    ref_area = _area(tri)
    assert abs(area - ref_area) <= 1e-12 * ref_area
    A, pts = mesh.poisson_dirichlet(m)
    assert A.shape == (12528, 12528) and pts.shape == (12528, 2)
    assert A.indices.dtype == np.int32 and A.has_sorted_indices
    w = np.linalg.eigvalsh(A.toarray()[:400, :400])  # a principal block of an SPD matrix
    assert w.min() > 0


@pytest.mark.skipif(not os.path.exists(REF_MSH), reason="reference mesh not present")
def test_fixture_matches_reference_msh():
    from mlamg import mesh
    m = mesh.read_gmsh(REF_MSH)
    f = mesh.load_npz(FIXTURE)
    assert np.array_equal(m.points, f.points)
    assert np.array_equal(m.cells["triangle"], f.cells["triangle"])
    assert np.array_equal(m.cells["line"], f.cells["line"])


def test_refine_counts_and_consistency():
    from mlamg import mesh
    m = mesh.load_npz(FIXTURE)
    r = mesh.refine(m)
    n_edges = len(np.unique(np.sort(np.concatenate([m.cells["triangle"][:, [0, 1]],
                                                    m.cells["triangle"][:, [1, 2]],
                                                    m.cells["triangle"][:, [2, 0]]]), 1), axis=0))
    assert r.points.shape[0] == 13072 + n_edges
    assert r.cells["triangle"].shape == (4 * 25600, 3)
    assert r.cells["line"].shape == (2 * 544, 2)
    # refinement keeps the domain area and the constants-in-kernel identity
    K = mesh.p1_stiffness(r.points, r.cells["triangle"])
    assert np.abs(K @ np.ones(K.shape[0])).max() <= 1e-11
    xy = r.points[:, :2]
    tri = xy[r.cells["triangle"]]
    area = _area(tri)
    tri0 = m.points[:, :2][m.cells["triangle"]]
    area0 = _area(tri0)
    assert abs(area - area0) <= 1e-12 * area0
    A, _ = mesh.poisson_dirichlet(r)
    assert A.shape[0] == r.points.shape[0] - len(np.unique(r.cells["line"]))


def test_jump_and_anisotropic_coefficients():
    from mlamg import mesh
    m = mesh.load_npz(FIXTURE)
    jumps = np.array([[1.0, 0.5, 1e-3], [3.0, 0.5, 1e3]])
    A, _ = mesh.poisson_dirichlet_jumps(m, jumps)
    assert abs(A - A.T).max() <= 1e-9 * abs(A).max()
    # coefficient 1e3 on the right half: those rows are ~1e6x the left ones
    xy = mesh.poisson_dirichlet(m)[1]
    d = A.diagonal()
    assert d[xy[:, 0] > 3.2].min() > 1e4 * d[xy[:, 0] < 0.8].max()
    Aa, _ = mesh.poisson_dirichlet(m, epsilon=0.01, theta=np.pi / 6)
    assert abs(Aa - Aa.T).max() <= 1e-12
    assert np.all(np.linalg.eigvalsh(Aa.toarray()[:300, :300]) > 0)


GRID3D = os.path.join(HERE, "golden", "laplace_3d_grid.npz")


def test_aniso_laplace_3d_matches_reference_grid():
    """mesh.aniso_laplace_3d (utils/create_3d_laplace.py:35-76 without firedrake) against the
    reference's own output demos/laplace_3d.grid (fixture: tests/golden/make_grid_fixture.py):
    after matching DoFs by coordinates, the same sparsity and the same values to assembly
    rounding (different element summation order: 1e-14 of max|a_ij|)."""
    g = np.load(GRID3D)
    Aref = sp.csr_matrix((g["data"], g["indices"], g["indptr"]))
    N = 12  # 11^3 = 1331 interior nodes
    from mlamg import mesh
    A, xyz = mesh.aniso_laplace_3d(N, N, N, float(g["theta_y"]), float(g["theta_z"]),
                                   float(g["eps_x"]), float(g["eps_y"]))
    assert A.shape == Aref.shape and A.nnz == Aref.nnz
    assert A.indices.dtype == np.int32 and A.has_sorted_indices

    def key(c):
        return np.rint(c * N).astype(np.int64) @ np.array([1, 100, 10000])
    mine = {k: i for i, k in enumerate(key(xyz))}
    p = np.array([mine[k] for k in key(g["x"])])
    assert len(set(p.tolist())) == A.shape[0]
    B = A[p][:, p].tocsr()
    B.sort_indices()
    Ar = Aref.copy()
    Ar.sort_indices()
    assert np.array_equal(B.indptr, Ar.indptr) and np.array_equal(B.indices, Ar.indices)
    assert np.abs(B.data - Ar.data).max() <= 1e-14 * np.abs(Ar.data).max()
    # the other diagonal orientations give a different operator: the split is pinned
    pts, tets = mesh.unit_cube_tets(N, N, N, flip=(1, 0, 0))
    K = mesh.p1_stiffness_3d(pts, tets, mesh.aniso_tensor_3d(
        float(g["theta_y"]), float(g["theta_z"]), float(g["eps_x"]), float(g["eps_y"])))
    assert abs(K.sum() - 0.0) < 1e-10  # Neumann operator annihilates constants
    interior = np.all((pts > 1e-12) & (pts < 1 - 1e-12), axis=1)
    Kf = K[interior][:, interior].tocsr()
    assert np.abs((Kf[p][:, p] - Ar)).max() > 1e-3


def test_random_aniso_laplace_3d_family():
    from mlamg import mesh
    A, xyz, extra = mesh.random_aniso_laplace_3d(np.random.RandomState(0))
    Nx, Ny, Nz = extra["Nx"], extra["Ny"], extra["Nz"]
    assert all(8 <= v < 15 for v in (Nx, Ny, Nz))
    assert A.shape[0] == (Nx - 1) * (Ny - 1) * (Nz - 1) == xyz.shape[0]
    assert abs(A - A.T).max() <= 1e-12 * abs(A).max()
    # SPD after the Dirichlet reduction: Cholesky-free check via the smallest eigenvalue
    w = np.linalg.eigvalsh(A.toarray())
    assert w.min() > 0
