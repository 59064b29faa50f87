#!/usr/bin/env python3
"""Kernel A/B timing: one library (MCPT_LIB) × traversal modes × scenes.

Prints one JSON line per (scene, mode): average path-tracing kernel ms over `--reps`
launches of `--spp` passes at W×H (HIP events on the launch stream), Msamples/s.

    MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_w4.so \
        python tools/ab_time.py --scenes 6 8 --modes 1 2
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import mcpt  # noqa: E402

BOUNCES = {0: 8, 1: 3, 2: 8, 3: 8, 4: 8, 5: 8, 6: 8, 7: 8, 8: 12}   # scene 0: the mesh workload


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, nargs="+", default=[6])
    ap.add_argument("--modes", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default=os.path.basename(mcpt.lib_path()))
    ap.add_argument("--walk-exit", type=int, nargs="+", default=[-1])
    ap.add_argument("--mesh-tris", type=int, default=1_000_000, help="scene 0: mcpt.meshes.big_mesh_scene(N)")
    a = ap.parse_args()
    r = mcpt.Renderer(0)
    r.set_target(a.width, a.height)
    ipv, iv = mcpt.camera_canonical(a.width, a.height)
    for sid in a.scenes:
        if sid == 0:
            from mcpt import meshes
            r.upload_scene(meshes.big_mesh_scene(a.mesh_tris)[0])
        else:
            r.upload_scene(mcpt.Scene.reference(sid))
        for mode, wx in [(m, w) for m in a.modes for w in (a.walk_exit if m == 1 else [-1])]:
            r.set_traversal(mode)
            if hasattr(r, "set_walk_exit"):
                r.set_walk_exit(wx)
            B = BOUNCES[sid]
            r.render(ipv, iv, 1, a.spp, 0.0, B, 1.0, 0)   # warm-up
            ms = []
            for k in range(a.reps):
                r.render(ipv, iv, 1 + (k + 1) * a.spp, a.spp, 0.0, B, 1.0, 0)
                ms.append(r.last_kernel_ms()[0])
            t = float(np.mean(ms))
            extra = {"stream_iterations": r.stream_iterations()} if mode == 3 else {}
            print(json.dumps({"lib": a.tag, "scene": sid, "mode": mode, "walk_exit": wx, "bounces": B, "spp": a.spp,
                              **extra,
                              "kernel_ms": round(t, 3),
                              "msamples_s": round(a.width * a.height * a.spp / t / 1e3, 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
