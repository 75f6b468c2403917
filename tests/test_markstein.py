"""CPU: the division of the device's Gauss-Seidel chains (csrc/common.hpp mk_recip / mk_div:
q = RN(a y) with y = RN(1/b), corrected by one exact fma remainder — Markstein's theorem) equals
the IEEE quotient bit for bit, which is what keeps the sweeps bitwise pyamg's. The same code in C
(oracle/markstein_check.c) on 1e7 random operand pairs over several exponent spreads (including
the guard boundaries) and all pairs of special values."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_markstein_division_is_ieee(tmp_path):
    exe = str(tmp_path / "mk")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "oracle", "markstein_check.c"), "-lm"], check=True)
    r = subprocess.run([exe, "10000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert "0 mismatches" in r.stdout
