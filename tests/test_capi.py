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
