"""CPU: the autotune's pruning bound (Hierarchy._lower_bound_us) — the most compact formats come
first and no candidate is skipped unless its bytes could not move in the best time so far."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ml-amg_amd", "mlamg", "libmlamg_hip.so")


class _Op:
    def __init__(self, n_rows, n_cols, nnz):
        self.shape = (n_rows, n_cols)
        self.nnz = nnz


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmlamg_hip.so not built")
def test_lower_bound_order_and_values():
    sys.path.insert(0, os.path.join(ROOT, "ml-amg_amd"))
    from mlamg.hierarchy import Hierarchy
    A0 = _Op(10077696, 10077696, 70263936)  # C4 fine operator
    lb = {f: Hierarchy._lower_bound_us(A0, "A", f)
          for f in ("rowpat", "sell_dict", "sorted", "csr_stream", "sell", "long")}
    assert lb["rowpat"] < lb["sell_dict"] < lb["sorted"] < lb["csr_stream"] == lb["sell"]
    # x, y and b at 7 TB/s: 34.6 us; CSR adds 12 B per nonzero: 120.5 us more
    assert abs(lb["rowpat"] - 34.552) < 0.01
    assert abs(lb["csr_stream"] - lb["rowpat"] - 120.452) < 0.01
    # below every time the C4 autotune has measured for that format (profiles/r03, r04: rowpat
    # 44.6 us cold, sorted and SELL above 100 us, dictionary SELL 95 us)
    assert lb["rowpat"] < 44.0 and lb["csr_stream"] < 160.0 and lb["sorted"] < 100.0
    assert lb["sell_dict"] < 77.0
    P = _Op(1008, 10078, 878932)  # R_3
    assert Hierarchy._lower_bound_us(P, "R", "vector") < 8.0
