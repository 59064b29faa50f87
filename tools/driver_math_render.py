#!/usr/bin/env python3
"""Render the C2 and C3 parity frames with one library build (MCPT_LIB) and save the averaged
images (tests/test_gpu_driver_math.py runs it once per build, each in its own process, since a
process loads one libmcpt).

    MCPT_LIB=.../libmcpt_drvmath7.so python tools/driver_math_render.py OUT_DIR

C2: scene 6, 1920x1080, passes 1..256, B 8, IOR 1.0.  C3: the same frame at 1,024 passes, IOR 1.5,
roughness 0.5 on every non-emissive primitive.  Per-lane walk, one render call each.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import mcpt  # noqa: E402

W, H = 1920, 1080
CASES = {"C2": dict(spp=256, bounces=8, ior=1.0, rough=None),
         "C3": dict(spp=1024, bounces=8, ior=1.5, rough=0.5)}


def scene(rough):
    sc = mcpt.Scene.reference(6)
    if rough is not None:
        prims, _, _ = sc.buffers()
        for i in range(sc.nb_prim()):
            rec = prims[i]
            if rec[58] > 0:   # emissive: untouched
                continue
            sc.set_material(i, np.concatenate([rec[52:56], [rec[56], rough, rec[58]]]).astype(np.float32))
    return sc


def main(out):
    os.makedirs(out, exist_ok=True)
    r = mcpt.Renderer(0)
    r.set_traversal(mcpt.TRAVERSAL_LANE)
    ipv, iv = mcpt.camera_canonical(W, H)
    for name, c in CASES.items():
        r.upload_scene(scene(c["rough"]))
        r.set_target(W, H)
        r.render(ipv, iv, 1, c["spp"], 0.0, c["bounces"], c["ior"], mcpt.MONTECARLO)
        acc, n = r.read_accum()
        assert n == c["spp"]
        np.save(os.path.join(out, f"{name}.npy"), acc / np.float32(n))
    r.close()
    print("ok", mcpt.lib_path(), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
