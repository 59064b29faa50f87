#!/usr/bin/env python3
"""Throughput of the triangle-mesh test scene (tests/test_meshes.py mesh_scene) at 1080p, B 8."""
import sys, os, json
sys.path[:0] = ['tests', 'montecarlo-pathtracing_amd', '.']
import torch  # noqa
import numpy as np
import mcpt
from test_meshes import mesh_scene
r = mcpt.Renderer(0)
W, H = 1920, 1080
sc = mesh_scene(mcpt)
r.upload_scene(sc)
r.set_target(W, H)
ipv, iv = mcpt.camera_canonical(W, H)
knobs = [(1, -1, -1), (2, -1, -1), (1, 0, 8), (1, 16, 8), (1, 16, 0), (1, 8, 4), (1, 24, 16)]
for flat in (False,):
    r.set_flat_face(flat)
    for mode, wx, lb in knobs:
        r.set_traversal(mode)
        r.set_walk_exit(wx)
        r.set_leaf_batch(lb)
        r.render(ipv, iv, 1, 32, 0.0, 8, 1.0, 0)
        ms = 0.0
        for k in range(3):
            r.render(ipv, iv, 33 + 32 * k, 32, 0.0, 8, 1.0, 0)
            ms += r.last_kernel_ms()[0]
        print(json.dumps({"scene": "mesh_scene (tests/test_meshes.py)", "triangles": int(sum(len(t) for t in [mcpt.meshes.cube()[2], mcpt.meshes.uv_sphere(20, 10)[2], mcpt.meshes.torus(24, 12)[2]])),
                          "flat_face": flat, "mode": mode, "walk_exit": wx, "leaf_batch": lb,
                          "msamples_s": round(W * H * 96 / ms / 1e3, 1)}))
