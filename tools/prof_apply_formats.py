"""cProfile of Hierarchy.apply_formats (the setup's format autotune) on the C4 hierarchy."""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ml-amg_amd")]

import torch  # noqa: E402

from mlamg import problems  # noqa: E402
from mlamg.hierarchy import Hierarchy  # noqa: E402

A = problems.poisson_3d_7pt(int(sys.argv[1]) if len(sys.argv) > 1 else 216)
H = Hierarchy.build(A, alpha=0.1, max_coarse=2000, aggregation="reference",
                    coarse_order="sorted", finalize=False)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
H.apply_formats("autotune", "auto")
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())
