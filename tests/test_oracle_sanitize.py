"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer.

tests/cpp/oracle_sanitize.cpp links oracle/oracle.cpp directly, built with
-fsanitize=address,undefined -fno-sanitize-recover=all, and exercises every entry point the
tests use (8 scenes, 3 variants, both accumulation orders, ray queries, sampler, mesh BVH).
Any sanitizer report aborts the run; its results must also equal the normal oracle build's
bit for bit (sanitizers must not change the arithmetic).
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sanitized_output(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("asan")
    exe = str(d / "oracle_sanitize")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", "-ffp-contract=off", "-fno-fast-math", "-mfma",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                    os.path.join(REPO, "oracle", "oracle.cpp"), os.path.join(REPO, "tests", "cpp", "oracle_sanitize.cpp"),
                    "-o", exe], check=True, timeout=600)
    out = str(d / "out.bin")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, out], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return np.fromfile(out, np.float32)


def _expected(orc):
    W, H = 16, 12
    ipv, iv = orc.camera(W, H)
    parts = []
    for s in range(1, 9):
        prims, nodes, leaves, d, _ = orc.scene(s, 1.2)
        B = 3 if s == 1 else (12 if s == 8 else 8)
        for variant in range(3):
            if variant > 0 and s != 6:
                continue
            acc, _ = orc.render(prims, nodes, leaves, d, ipv, iv, W, H, 1, 2, 0.0, B, 1.5 if s == 6 else 1.0,
                                variant, n_threads=2)
            parts.append(acc.ravel())
        xy = np.array([[0, 0], [7, 5], [15, 11]], np.int32)
        for per_pass in (False, True):
            parts.append(orc.render_pixels(prims, nodes, leaves, d, ipv, iv, W, H, xy, 5, 40, 0.0, B, 1.0, 0,
                                           per_pass=per_pass, n_threads=2).ravel())
        O = np.array([[0.0, -347.0, 61.0], [10.0, 20.0, 30.0]], np.float32)
        D = np.array([[0.0, 0.98, -0.17], [0.3, -0.5, -0.8]], np.float32)
        for any_hit in (False, True):
            _, of = orc.trace(prims, nodes, leaves, d, O, D, any_hit=any_hit)
            parts.append(of.ravel())
    parts.append(orc.sample_hemisphere([0.2, 0.3, 0.9], [0.25, 3.5, 0.75], 64, 0.7, 3).ravel())
    verts = np.array([[i, j, 0.1 * np.float32(i * j)] for j in range(5) for i in range(5)], np.float32)
    tris = []
    for j in range(4):
        for i in range(4):
            a = j * 5 + i
            tris += [[a, a + 1, a + 5], [a + 1, a + 6, a + 5]]
    _, mnodes, _ = orc.mesh_bvh(verts, np.array(tris, np.int32))
    parts.append(mnodes.ravel())
    return np.concatenate(parts).astype(np.float32)


def test_oracle_clean_under_asan_ubsan(sanitized_output, oracle_mod):
    ref = _expected(oracle_mod)
    assert sanitized_output.size == ref.size
    assert np.array_equal(sanitized_output.view(np.uint32), ref.view(np.uint32))
