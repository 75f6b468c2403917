"""Unstructured P1 inputs for the C3/C5 configurations.

The reference reads gmsh files with meshio and assembles with pyamg.gallery.fem:
  meshio_2d_poisson_dirichlet(mesh, epsilon, theta)      ns/model/data.py:301-344
  meshio_2d_poisson_dirichlet_jump_coeffs(mesh, jumps)   ns/model/data.py:346-394
  Dirichlet rows removed: R = I[interior], A_d = R A R^T, eliminate_zeros (data.py:328-342);
  boundary nodes = nodes of the gmsh 'line' elements (data.py:328-333).
Neither meshio nor pyamg is in this image, so both are restated here:
  * read_gmsh: gmsh MSH 4.1 ASCII ($Nodes / $Elements entity blocks; element types 1 = line,
    2 = triangle, 15 = point), points in file order, node tags mapped to 0-based indices (what
    meshio's `points` / `cells_dict` expose);
  * p1_stiffness: standard P1 grad-grad form, K_e = |T| * G_e kappa(centroid) G_e^T with G_e the
    constant gradients of the barycentric basis; kappa a 2x2 tensor or a scalar. For the
    isotropic C3 case (kappa = I) every quadrature rule gives the same K_e; for jump and
    anisotropic coefficients the centroid rule is a documented deviation from pyamg's quadrature.
    Assembly order (element order, local row-major 3x3, duplicates summed by scipy's coo->csr)
    is this module's own: parity of the ASSEMBLED MATRIX against pyamg is unpinned; everything
    downstream (hierarchy, cycle) is pinned against the oracle on the same matrix.
  * refine: uniform red refinement (each triangle -> 4 through its edge midpoints; boundary lines
    split in two), the "x4^r" C3 variants.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp


@dataclass
class Mesh:
    points: np.ndarray                     # (n, 3) float64, file order
    cells: dict = field(default_factory=dict)  # 'line' (m, 2), 'triangle' (t, 3), int64

    @property
    def cells_dict(self):  # meshio's name
        return self.cells


_NODES_PER_TYPE = {1: 2, 2: 3, 15: 1, 3: 4, 4: 4, 8: 3, 9: 6}
_TYPE_NAME = {1: "line", 2: "triangle", 15: "vertex", 3: "quad", 4: "tetra", 8: "line3",
              9: "triangle6"}


def _sections(lines):
    out, i = {}, 0
    while i < len(lines):
        ln = lines[i].strip()
        if ln.startswith("$") and not ln.startswith("$End"):
            name = ln[1:]
            j = i + 1
            while not lines[j].strip().startswith("$End" + name):
                j += 1
            out[name] = lines[i + 1:j]
            i = j + 1
        else:
            i += 1
    return out


def read_gmsh(path_or_text):
    """Parse a gmsh MSH 4.1 ASCII file (path or its text) into a Mesh."""
    if "\n" in path_or_text:
        text = path_or_text
    else:
        with open(path_or_text) as fh:
            text = fh.read()
    sec = _sections(text.splitlines())
    fmt = sec["MeshFormat"][0].split()
    if not fmt[0].startswith("4") or fmt[1] != "0":
        raise ValueError(f"only gmsh 4.x ASCII is supported (got version {fmt[0]}, "
                         f"file-type {fmt[1]})")
    nl = sec["Nodes"]
    n_blocks, n_nodes = (int(v) for v in nl[0].split()[:2])
    tags = np.empty(n_nodes, dtype=np.int64)
    pts = np.empty((n_nodes, 3), dtype=np.float64)
    k, p = 0, 1
    for _ in range(n_blocks):
        _dim, _tag, parametric, cnt = (int(v) for v in nl[p].split())
        p += 1
        tags[k:k + cnt] = [int(nl[p + q]) for q in range(cnt)]
        p += cnt
        for q in range(cnt):
            pts[k + q] = [float(v) for v in nl[p + q].split()[:3]]
        p += cnt
        k += cnt
        if parametric:
            raise ValueError("parametric node coordinates are not supported")
    index = {int(t): i for i, t in enumerate(tags)}
    el = sec["Elements"]
    n_eblocks = int(el[0].split()[0])
    cells = {}
    p = 1
    for _ in range(n_eblocks):
        _dim, _tag, etype, cnt = (int(v) for v in el[p].split())
        p += 1
        npe = _NODES_PER_TYPE.get(etype)
        if npe is None:
            raise ValueError(f"unsupported gmsh element type {etype}")
        conn = np.empty((cnt, npe), dtype=np.int64)
        for q in range(cnt):
            f = el[p + q].split()
            conn[q] = [index[int(v)] for v in f[1:1 + npe]]
        p += cnt
        name = _TYPE_NAME[etype]
        cells[name] = np.concatenate([cells[name], conn]) if name in cells else conn
    return Mesh(pts, cells)


def load_npz(path):
    """Mesh saved as arrays (points, triangle, line), e.g. tests/golden/cylflow_highres_mesh.npz."""
    z = np.load(path)
    return Mesh(np.array(z["points"], dtype=np.float64),
                {"triangle": np.array(z["triangle"], dtype=np.int64),
                 "line": np.array(z["line"], dtype=np.int64)})


def refine(mesh):
    """Uniform red refinement: new nodes at edge midpoints (appended after the old ones in order
    of first appearance), each triangle -> 4, each boundary line -> 2."""
    tri = mesh.cells["triangle"]
    e = np.concatenate([tri[:, [0, 1]], tri[:, [1, 2]], tri[:, [2, 0]]])
    lines = mesh.cells.get("line", np.zeros((0, 2), np.int64))
    e_all = np.sort(np.concatenate([e, lines]), axis=1)
    uniq, first, inv = np.unique(e_all, axis=0, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")         # number midpoints by first appearance
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    n0 = mesh.points.shape[0]
    mid_id = n0 + rank[inv.ravel()]
    pts = np.concatenate([mesh.points, 0.5 * (mesh.points[uniq[order, 0]] +
                                              mesh.points[uniq[order, 1]])])
    t = len(tri)
    m01, m12, m20 = mid_id[:t], mid_id[t:2 * t], mid_id[2 * t:3 * t]
    a, b, c = tri[:, 0], tri[:, 1], tri[:, 2]
    new_tri = np.concatenate([np.stack([a, m01, m20], 1), np.stack([m01, b, m12], 1),
                              np.stack([m20, m12, c], 1), np.stack([m01, m12, m20], 1)])
    cells = dict(mesh.cells)
    cells["triangle"] = new_tri
    if len(lines):
        ml = mid_id[3 * t:]
        cells["line"] = np.concatenate([np.stack([lines[:, 0], ml], 1),
                                        np.stack([ml, lines[:, 1]], 1)])
    return Mesh(pts, cells)


def p1_stiffness(points, triangles, kappa=None):
    """Global P1 grad-grad matrix (n x n CSR, duplicates summed, sorted columns).

    kappa: None (identity), a scalar, a (2, 2) tensor, or a callable kappa(x, y) returning
    either, evaluated at each element centroid."""
    xy = points[:, :2]
    P = xy[triangles]                                   # (t, 3, 2)
    d1 = P[:, 1] - P[:, 0]
    d2 = P[:, 2] - P[:, 0]
    det = d1[:, 0] * d2[:, 1] - d1[:, 1] * d2[:, 0]
    area = 0.5 * np.abs(det)
    # gradients of the barycentric functions: rows of inv([[d1],[d2]])^T mapped to 3 nodes
    inv = np.empty((len(det), 2, 2))
    inv[:, 0, 0] = d2[:, 1] / det
    inv[:, 0, 1] = -d1[:, 1] / det
    inv[:, 1, 0] = -d2[:, 0] / det
    inv[:, 1, 1] = d1[:, 0] / det
    G = np.empty((len(det), 3, 2))
    G[:, 1] = inv[:, :, 0]
    G[:, 2] = inv[:, :, 1]
    G[:, 0] = -G[:, 1] - G[:, 2]
    if kappa is None:
        KG = G
    else:
        c = P.mean(axis=1)
        if callable(kappa):
            kv = [np.asarray(kappa(cx, cy), dtype=np.float64) for cx, cy in c]
            K = np.stack([k * np.eye(2) if k.ndim == 0 else k for k in kv])
        else:
            k = np.asarray(kappa, dtype=np.float64)
            K = np.broadcast_to(k * np.eye(2) if k.ndim == 0 else k, (len(det), 2, 2))
        KG = np.einsum("tij,tkj->tki", K, G)           # (kappa g_k) for each node k
    Ke = area[:, None, None] * np.einsum("tki,tli->tkl", G, KG)
    rows = np.repeat(triangles, 3, axis=1).ravel()
    cols = np.tile(triangles, (1, 3)).ravel()
    n = points.shape[0]
    A = sp.coo_matrix((Ke.ravel(), (rows, cols)), shape=(n, n)).tocsr()
    A.sort_indices()
    return A


def _dirichlet(A, mesh):
    bnd = np.unique(mesh.cells.get("line", np.zeros((0, 2), np.int64)).ravel())
    interior = np.ones(mesh.points.shape[0], dtype=bool)
    interior[bnd] = False
    R = sp.eye(mesh.points.shape[0], format="csr")[interior]
    A_d = (R @ A @ R.T).tocsr()
    A_d.eliminate_zeros()
    A_d.sort_indices()
    A_d.indices = A_d.indices.astype(np.int32)
    A_d.indptr = A_d.indptr.astype(np.int32)
    return A_d, (R @ mesh.points)[:, :2]


def poisson_dirichlet(mesh, epsilon=1.0, theta=0.0):
    """meshio_2d_poisson_dirichlet (ns/model/data.py:301-344): kappa = Q diag(1, eps) Q^T."""
    c, s = np.cos(theta), np.sin(theta)
    Q = np.array([[c, -s], [s, c]])
    kap = Q @ np.diag([1.0, epsilon]) @ Q.T
    kappa = None if (epsilon == 1.0 and theta == 0.0) else kap
    return _dirichlet(p1_stiffness(mesh.points, mesh.cells["triangle"], kappa), mesh)


def unit_cube_tets(Nx, Ny, Nz, flip=(0, 0, 0)):
    """Tetrahedral mesh of [0,1]^3 with Nx x Ny x Nz cells, each split into the 6 tetrahedra
    that share one main diagonal of the cell (firedrake UnitCubeMesh, the mesh of
    utils/create_3d_laplace.py:36). Nodes are numbered lexicographically, x fastest:
    p = i + (Nx+1) (j + (Ny+1) k). flip[a] = 1 reflects the shared diagonal along axis a; the
    default (0,0,0)-(1,1,1) diagonal is the one the reference's laplace_3d.grid was built on
    (tests/test_mesh.py pins it)."""
    nxp, nyp = Nx + 1, Ny + 1
    i, j, k = np.meshgrid(np.arange(Nx + 1), np.arange(Ny + 1), np.arange(Nz + 1), indexing="ij")
    pts = np.stack([i.ravel(order="F") / Nx, j.ravel(order="F") / Ny, k.ravel(order="F") / Nz],
                   axis=1)
    ci, cj, ck = np.meshgrid(np.arange(Nx), np.arange(Ny), np.arange(Nz), indexing="ij")
    ci, cj, ck = ci.ravel(order="F"), cj.ravel(order="F"), ck.ravel(order="F")
    f = np.asarray(flip, dtype=np.int64)
    tets = []
    for perm in ((0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1), (2, 1, 0)):
        o = np.zeros(3, dtype=np.int64)
        verts = []
        for step in range(4):
            if step:
                o = o.copy()
                o[perm[step - 1]] = 1
            oo = o ^ f
            verts.append((ci + oo[0]) + nxp * ((cj + oo[1]) + nyp * (ck + oo[2])))
        tets.append(np.stack(verts, axis=1))
    return pts, np.concatenate(tets).astype(np.int64)


def p1_stiffness_3d(points, tets, D=None):
    """Global P1 grad-grad matrix inner(D grad u, grad v) dx on tetrahedra (n x n CSR, duplicates
    summed, sorted columns); D a constant (3, 3) tensor or None (identity). Exact for P1."""
    P = points[tets]                                    # (t, 4, 3)
    J = P[:, 1:] - P[:, :1]                             # rows p_k - p_0
    det = np.linalg.det(J)
    Jinv = np.linalg.inv(J)                             # grad lambda_k = column k of J^-1
    G = np.empty((len(tets), 4, 3))
    G[:, 1:] = np.transpose(Jinv, (0, 2, 1))
    G[:, 0] = -G[:, 1:].sum(axis=1)
    KG = G if D is None else np.einsum("ij,tkj->tki", np.asarray(D, dtype=np.float64), G)
    Ke = (np.abs(det) / 6.0)[:, None, None] * np.einsum("tki,tli->tkl", G, KG)
    rows = np.repeat(tets, 4, axis=1).ravel()
    cols = np.tile(tets, (1, 4)).ravel()
    n = points.shape[0]
    A = sp.coo_matrix((Ke.ravel(), (rows, cols)), shape=(n, n)).tocsr()
    A.sort_indices()
    return A


def aniso_tensor_3d(theta_y, theta_z, eps_x, eps_y):
    """D = R^T diag(eps_x, eps_y, 1) R with R = R_y(theta_y) R_z(theta_z)
    (utils/create_3d_laplace.py:45-57)."""
    cz, sz, cy, sy = np.cos(theta_z), np.sin(theta_z), np.cos(theta_y), np.sin(theta_y)
    R_z = np.array([[cz, -sz, 0.0], [sz, cz, 0.0], [0.0, 0.0, 1.0]])
    R_y = np.array([[cy, 0.0, sy], [0.0, 1.0, 0.0], [-sy, 0.0, cy]])
    R = R_y @ R_z
    return R.T @ np.diag([eps_x, eps_y, 1.0]) @ R


def aniso_laplace_3d(Nx, Ny, Nz, theta_y=0.0, theta_z=0.0, eps_x=1.0, eps_y=1.0):
    """gen_aniso_laplace (utils/create_3d_laplace.py:35-76) restated without firedrake: P1 on
    unit_cube_tets, D = aniso_tensor_3d, the 6 cube faces' nodes removed (R A R^T, :68-76).
    Returns (A, xyz) with A (interior nodes in lexicographic order, int32 CSR, sorted columns,
    exact zeros dropped as scipy's SpGEMM does) and the interior node coordinates. The reference
    numbers DoFs in firedrake's order; tests/test_mesh.py matches its laplace_3d.grid by
    coordinates."""
    pts, tets = unit_cube_tets(Nx, Ny, Nz)
    A = p1_stiffness_3d(pts, tets, aniso_tensor_3d(theta_y, theta_z, eps_x, eps_y))
    eps = 1e-12
    interior = np.all((pts > eps) & (pts < 1.0 - eps), axis=1)
    R = sp.eye(pts.shape[0], format="csr")[interior]
    A_d = (R @ A @ R.T).tocsr()
    A_d.eliminate_zeros()
    A_d.sort_indices()
    A_d.indices = A_d.indices.astype(np.int32)
    A_d.indptr = A_d.indptr.astype(np.int32)
    return A_d, pts[interior]


def random_aniso_laplace_3d(rand, anisotropic=True):
    """One grid of create_3d_laplace.py's loop (:79-95): N in [8, 15) per axis; theta_y, theta_z
    ~ U[0, 2 pi), eps_x, eps_y ~ 10^U[-4, 4] when anisotropic. Draw order follows the
    reference (Nx, Ny, Nz, theta_z, theta_y, eps_x, eps_y). Returns (A, xyz, extra)."""
    Nx, Ny, Nz = rand.randint(8, 15), rand.randint(8, 15), rand.randint(8, 15)
    if anisotropic:
        theta_z = rand.uniform(0, 2 * np.pi)
        theta_y = rand.uniform(0, 2 * np.pi)
        eps_x = 10.0 ** rand.uniform(-4.0, 4.0)
        eps_y = 10.0 ** rand.uniform(-4.0, 4.0)
    else:
        theta_z = theta_y = 0.0
        eps_x = eps_y = 1.0
    A, xyz = aniso_laplace_3d(Nx, Ny, Nz, theta_y, theta_z, eps_x, eps_y)
    extra = {"theta_z": theta_z, "theta_y": theta_y, "eps_x": eps_x, "eps_y": eps_y,
             "eps_z": 1.0, "dim": 3, "Nx": Nx, "Ny": Ny, "Nz": Nz}
    return A, xyz, extra


def poisson_dirichlet_jumps(mesh, jumps):
    """meshio_2d_poisson_dirichlet_jump_coeffs (ns/model/data.py:346-394): scalar coefficient of
    the nearest jump seed (rows [x, y, d]), evaluated at the element centroid."""
    jumps = np.asarray(jumps, dtype=np.float64)

    def kappa(x, y):
        return jumps[np.argmin(np.hypot(jumps[:, 0] - x, jumps[:, 1] - y)), -1]

    return _dirichlet(p1_stiffness(mesh.points, mesh.cells["triangle"], kappa), mesh)
