"""GPU: unchanged callers through the amg_2_v broker (mlamg/broker.py, MLAMG_BROKER=1). Worker
processes that never touch the GPU call mlamg.multigrid.amg_2_v exactly as the reference's pool
workers call ns.lib.multigrid.amg_2_v (utils/evaluate_dataset.py:96, utils/train_dataset.py:114);
ONE broker process, started by the first of them, runs the calls — concurrent ones coalesced into
fused batch launches. Every result is bitwise the direct single call's (both tolerance modes,
both smoothers, grids whose coarse operator takes the fused kernel and grids beyond it)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/ml-amg_amd"]
from tests.test_gpu_broker import problem
from mlamg import multigrid
rank, nprocs, count = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
out = {}
for i in range(rank, count, nprocs):
    A, P, b, x, kw = problem(i)
    xo, c, e, it = multigrid.amg_2_v(A, P, b, x, **kw)
    out[i] = [np.asarray(xo).tolist(), float(c), np.asarray(e).tolist(), int(it)]
print(json.dumps(out))
'''


def problem(i):
    """Grids 24^2 - 128^2 (n_c 64 - 1849: the fused kernel's batch limit is 1024), alternating
    the reference's two call shapes and both smoothers."""
    from mlamg import problems
    from oracle import restated as orc
    m = (24, 32, 48, 64, 96, 128)[i % 6]
    A = problems.poisson_2d_5pt(m)
    P, _ = orc.smoothed_aggregation_jacobi(A, problems.box_aggregates_2d(m, m, 3),
                                           omega=2.0 / 3.0)
    x = np.random.RandomState(i).randn(A.shape[0])
    b = np.zeros(A.shape[0]) if i % 3 else np.random.RandomState(50 + i).randn(A.shape[0])
    kw = {"res_tol": 1e-10} if i % 2 == 0 else {"error_tol": 1e-6}
    if i % 4 == 3:
        kw["smoother"] = "jacobi"
    return A, P, b, x, kw


def test_broker_results_bitwise_single_calls(oracle, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mlamg import broker, multigrid
    count, nprocs = 24, 6
    env = dict(os.environ, MLAMG_BROKER="1", MLAMG_BROKER_DIR=str(tmp_path),
               MLAMG_BROKER_IDLE="30", OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, "-c", WORKER, ROOT, str(r), str(nprocs),
                               str(count)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True, env=env) for r in range(nprocs)]
    got = {}
    try:
        for p in procs:
            out, err = p.communicate(timeout=240)
            assert p.returncode == 0, err[-3000:]
            got.update({int(k): v for k, v in json.loads(out.strip().splitlines()[-1]).items()})
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        os.environ["MLAMG_BROKER_DIR"] = str(tmp_path)
        try:
            stopped = broker.shutdown()
        finally:
            del os.environ["MLAMG_BROKER_DIR"]
    assert stopped
    assert len(got) == count
    for i in range(count):
        A, P, b, x, kw = problem(i)
        xd, cd, ed, itd = multigrid.amg_2_v(A, P, b, x, **kw)
        xb, cb, eb, itb = got[i]
        assert itb == itd and np.array_equal(np.array(eb), ed), i
        assert np.array_equal(np.array(xb), xd), i
        assert cb == float(cd) or (np.isnan(cb) and np.isnan(cd)), i
