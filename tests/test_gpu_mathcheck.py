"""The arithmetic contract's short sqrt / reciprocal sequences (csrc/mcpt_math.h sqrt_rn,
rcp_rn, normalize's rsqrt_rn(x) = RN(1/RN(sqrt(x)))) equal the correctly rounded results for all 2^32
binary32 inputs on this device (tools/mathcheck/exhaustive.hip, built by build())."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tools", "mathcheck", "exhaustive")


def test_sqrt_rcp_exhaustive():
    assert os.path.exists(BIN), "build() compiles tools/mathcheck/exhaustive"
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    res = json.loads(out.stdout)
    assert res["inputs"] == 1 << 32
    for k in ("sqrt_rn", "rcp_rn", "rsqrt_rn"):
        assert res[k]["mismatches"] == 0, (k, res[k])
    assert res["contract_exact"] and out.returncode == 0
    # the raw hardware instructions alone are not correctly rounded (why the sequences exist)
    assert res["hw v_sqrt_f32"]["mismatches"] > 0 and res["hw v_rcp_f32"]["mismatches"] > 0


DIV_BIN = os.path.join(REPO, "tools", "mathcheck", "div_exhaustive")


def test_division_exhaustive():
    """div_core (y = RN(1/b), q0 = RN(a y), q1 = RN(q0 + (a - b q0) y)) equals the correctly
    rounded a / b on all 2^46 pairs of binary32 significands, and div_rn (with its range check
    and IEEE fallback) on 2^32 random pairs of signs and exponents (tools/mathcheck/div_exhaustive.hip)."""
    assert os.path.exists(DIV_BIN), "build() compiles tools/mathcheck/div_exhaustive"
    out = subprocess.run([DIV_BIN], capture_output=True, text=True, timeout=600)
    res = json.loads(out.stdout)
    assert res["significand_pairs"] == 1 << 46
    assert res["div_core_mismatches"] == 0, res
    assert res["div_rn_mismatches"] == 0 and res["random_in_range"] > 0, res
    assert res["exact"] and out.returncode == 0
