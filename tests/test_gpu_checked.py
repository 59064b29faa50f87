"""The bounds-checked build on the paths that index past the work items (verdict r05 item 1).

Round 5's first tail-piece form read ``item_perm[blockIdx.x]`` for every workgroup of a grid of
``n_items + tail_m (K - 1)`` workgroups; at 1080p the over-read landed in allocation slack and
``test_tail_pieces_same_bits`` passed with the bug, and at the C5 shape (3840x2160, four
segments per item) it faulted the *next* call.  The checked build (``make checked``,
``-DMCPT_CHECKED``: mcpt_internal.h ``idx_ok``) tests every work-item-order, split-item and
segment-slot index against its array's length, counts and skips a violation, and waits for every
sub-launch, so a violation or a fault fails the render call that caused it with the sub-launch
named.  Here it renders, each in its own process (a process loads one libmcpt):

* the C5 shape with MCPT_SEG_PER_ITEM=4 (tail pieces), per-lane and wave-coherent walks;
* the mesh workload (split items);

and the results must equal the shipped build's bit for bit with the work-item order off.  A
last case injects round 5's read pattern (MCPT_CHECKED_INJECT=1: every workgroup id tested
against n_items, no access made) and requires the checked build to report it at the first
ordered launch, as site CK_PERM_HEAD.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECKED = os.path.join(REPO, "montecarlo-pathtracing_amd", "mcpt", "variants", "libmcpt_checked.so")
SCRIPT = os.path.join(REPO, "tools", "checked_render.py")
CK_PERM_HEAD = 4   # mcpt_internal.h CheckSite


def _run(case, out, lib=None, **env_over):
    env = dict(os.environ)
    env.pop("MCPT_LIB", None)
    if lib is not None:
        env["MCPT_LIB"] = lib
    env.update({k: str(v) for k, v in env_over.items()})
    return subprocess.run([sys.executable, "-u", SCRIPT, case, out], env=env, capture_output=True, text=True,
                          timeout=300)


def _load(out, case):
    return {f[len(case) + 1:-4]: np.load(os.path.join(out, f)) for f in sorted(os.listdir(out)) if f.endswith(".npy")}


@pytest.fixture(scope="module")
def checked_lib():
    assert os.path.exists(CHECKED), f"build the checked variant first (make -C montecarlo-pathtracing_amd/csrc checked): {CHECKED}"
    return CHECKED


@pytest.mark.parametrize("case,env", [("c5", {"MCPT_SEG_PER_ITEM": 4}), ("mesh", {})])
def test_checked_build_same_bits(checked_lib, tmp_path, case, env):
    r = _run(case, str(tmp_path / "checked"), checked_lib, **env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "build_flags 1" in r.stdout, r.stdout   # the checked build ran (MCPT_BUILD_CHECKED)
    s = _run(case, str(tmp_path / "plain"), None, MCPT_ITEM_ORDER=0, **env)
    assert s.returncode == 0, s.stdout[-2000:] + s.stderr[-3000:]
    assert "build_flags 0" in s.stdout, s.stdout
    got, ref = _load(str(tmp_path / "checked"), case), _load(str(tmp_path / "plain"), case)
    assert got.keys() == ref.keys() and got
    for k in got:
        assert np.array_equal(got[k].view(np.uint32), ref[k].view(np.uint32)), f"{case} {k}"


def test_checked_build_reports_round5_pattern(checked_lib, tmp_path):
    """The checker catches the round-5 read pattern at the launch that makes it."""
    r = _run("c5", str(tmp_path / "inject"), checked_lib, MCPT_SEG_PER_ITEM=4, MCPT_CHECKED_INJECT=1)
    assert r.returncode != 0, r.stdout[-2000:]
    msg = r.stderr
    assert "checked build: sub-launch 0 of 1" in msg, msg[-3000:]
    assert f"first at site {CK_PERM_HEAD} index" in msg, msg[-3000:]
    # the first call runs in dispatch order (no tail pieces, grid = n_items): clean; the second
    # call is the first with tail pieces and its spare workgroups are what the injected test sees
    assert "LANE passes" not in r.stdout
