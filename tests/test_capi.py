"""The C-ABI library loads and exports every symbol include/mcpt.h declares; without a
GPU the device half fails loudly (status code), never silently."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(REPO, "include", "mcpt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mcpt_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported(mcpt_mod):
    L = ctypes.CDLL(mcpt_mod.lib_path())
    names = declared()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


VARIANTS = os.path.join(REPO, "montecarlo-pathtracing_amd", "mcpt", "variants")


@pytest.mark.parametrize("name", ["checked", "stamps", "lanestats", "blocktimes", "drvmath1", "drvmath2", "drvmath4",
                                  "drvmath7"])
def test_diagnostic_builds_current(name):
    """The in-tree diagnostic builds the GPU tests and tools load (round 6: a stale round-5 build
    lacked a symbol the binding declares): each exports every header symbol and says which build
    it is (mcpt_build_flags)."""
    path = os.path.join(VARIANTS, f"libmcpt_{name}.so")
    assert os.path.exists(path), f"make -C montecarlo-pathtracing_amd/csrc {name}: {path}"
    L = ctypes.CDLL(path)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, (name, missing)
    want = {"checked": 1, "stamps": 2, "lanestats": 4, "blocktimes": 8}.get(name, 16)
    assert L.mcpt_build_flags() == want


def test_shipped_build_flags(mcpt_mod):
    assert mcpt_mod.build_flags() == 0   # the shipped library is no diagnostic build


def test_python_binding_covers_header(mcpt_mod):
    L = mcpt_mod.lib()
    for n in declared():
        assert getattr(L, n).argtypes is not None, f"{n} not bound in mcpt/__init__.py"


def test_status_strings(mcpt_mod):
    L = mcpt_mod.lib()
    for code in (0, -1, -2, -3, -4, -5, -6):
        assert L.mcpt_error_string(code)
    assert L.mcpt_event_bytes(0) == 48 and L.mcpt_event_bytes(99) < 0


def test_no_gpu_fails_loudly(mcpt_mod):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(mcpt_mod.MCPTError):
        mcpt_mod.Renderer(0)


def test_invalid_arguments_rejected(mcpt_mod):
    L = mcpt_mod.lib()
    assert L.mcpt_upload_scene(None, None, 0, None, None, 0, 0) == -1
    assert L.mcpt_render(None, None, None, 1, 1, 0.0, 3, 1.0, 0) == -1
    assert L.mcpt_camera_canonical(0, 10, None, None) == -1


# The reference's own arrays, as numpy record types (scene.h:15-19 BB, scene.h:64-73 PrimData;
# GLMat4 = Eigen::Matrix4f column-major, GLVec3/GLVec4 = packed floats): what an adapter passes
# straight to mcpt_upload_scene.  Field offsets must be the texel layout the
# library reads.
PRIMDATA = __import__("numpy").dtype([("transfo_", "<f4", (4, 4)), ("inv_transfo_", "<f4", (4, 4)),
                                      ("inv_mesh_bb_transfo_", "<f4", (4, 4)), ("type_", "<f4", 4),
                                      ("color_", "<f4", 4), ("mat_info", "<f4", 4), ("padding2_", "<f4", 4)])
BB = __import__("numpy").dtype([("min_", "<f4", 3), ("max_", "<f4", 3)])


def test_reference_record_layouts(mcpt_mod):
    import numpy as np
    assert PRIMDATA.itemsize == 256 and BB.itemsize == 24
    sc = mcpt_mod.Scene.reference(6)
    prims, nodes, leaves = sc.buffers()
    rec = np.frombuffer(np.ascontiguousarray(prims, np.float32).tobytes(), PRIMDATA)
    bb = np.frombuffer(np.ascontiguousarray(nodes, np.float32).tobytes(), BB)
    assert rec.shape[0] == sc.nb_prim() == 6 and bb.shape[0] == 2 ** (sc.depth() + 1) - 1
    # the light (emissive first): an oriented quad (type 5) with emissivity 20 * 1.2
    assert rec["type_"][0, 0] == 5.0 and np.isclose(rec["mat_info"][0, 2], 24.0)
    assert (rec["type_"][1:, 0] != 5.0).all() and (rec["mat_info"][1:, 2] == 0.0).all()
    # Eigen column-major: transfo_ rows are [col][row]; transfo · inverse = identity (affine)
    for r in rec:
        T, Ti = r["transfo_"].T.astype(np.float64), r["inv_transfo_"].T.astype(np.float64)
        assert np.allclose(T @ Ti, np.eye(4), atol=1e-4)
        assert np.array_equal(T[3], [0, 0, 0, 1])
    # spheres' opacities (colour .a) as in montecarlo.cpp:756-770
    assert np.allclose(np.sort(rec["color_"][rec["type_"][:, 0] == 1.0, 3]), [0.01, 0.05, 0.15, 0.25])
    # BB: the root box contains every node box, min <= max where a subtree holds a primitive
    assert (bb["min_"][0] <= bb["min_"].min(0)).all() and (bb["max_"][0] >= bb["max_"].max(0)).all()
    assert (bb["min_"] <= bb["max_"]).all()
    assert leaves.dtype == np.int32 and set(leaves.tolist()) <= set(range(-1, 6))
