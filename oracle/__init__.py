"""TEST INFRASTRUCTURE ONLY — CPU oracle of the reference AMG V-cycle path.

This package restates nicknytko/ml-amg's hot path (ns/lib/multigrid.py, ns/lib/graph.py,
ns/preconditioner/MLAMG.py) and the third-party pieces it calls (scipy sparsetools, pyamg 4.x
gauss_seidel / lloyd_cluster) on the CPU. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it, and only as the checker. The product (ml-amg_amd/mlamg) never
imports it and has no CPU fallback.

Pinning: the scipy-level restatements are checked against golden vectors produced by running the
reference functions themselves in the build container (tests/golden/make_golden.py, which imports
/root/reference with empty stubs for its absent imports). pyamg is not installed anywhere here,
so the pyamg pieces (gauss_seidel, lloyd_cluster) are restatements of pyamg 4.x amg_core from its
published algorithm: parity at that boundary is unpinned.
"""
