#!/usr/bin/env python3
"""Interleaved A/B timing of several libmcpt builds in ONE process (finer than tools/ab_time.py,
whose candidates run one after another): every library gets its own context on the same GPU and
the same scene buffers, and the timed launches alternate library by library, `--reps` rounds, so
clock and cache drift hit every candidate alike.  Kernel time from each library's HIP events.

    python tools/ab_interleave.py --scene 0 --libs main variants/libmcpt_mw5.so --walk-exit 16 40

--scene 0 is the mesh workload (mcpt.meshes.big_mesh_scene), -1 the four-mesh workload
(big_mesh4_scene), 1..8 the reference scenes.
Prints one JSON line per (library, walk exit): median / mean / min kernel ms and Msamples/s.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import mcpt  # noqa: E402

BOUNCES = {-1: 8, 0: 8, 1: 3, 2: 8, 3: 8, 4: 8, 5: 8, 6: 8, 7: 8, 8: 12}
MAIN = os.path.join(REPO, "montecarlo-pathtracing_amd", "mcpt", "libmcpt.so")


def lib_path(name):
    if name == "main":
        return MAIN
    p = name if os.path.isabs(name) else os.path.join(REPO, "montecarlo-pathtracing_amd", "mcpt", name)
    if not p.endswith(".so"):
        p = os.path.join(REPO, "montecarlo-pathtracing_amd", "mcpt", "variants", f"libmcpt_{name}.so")
    return p


class Ctx:
    """One library's context with the scene uploaded and the target set."""

    def __init__(self, path, bufs, mb, W, H):
        self.L = ctypes.CDLL(path)
        mcpt._declare(self.L)
        h = ctypes.c_void_p()
        self._ok(self.L.mcpt_create(0, ctypes.byref(h)))
        self.h = h
        prims, nodes, leaves, depth, nbe = bufs
        fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
        ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))    # noqa: E731
        self._ok(self.L.mcpt_upload_scene(h, fp(prims), prims.shape[0], fp(nodes), ip(leaves), depth, nbe))
        if mb is not None:
            self._ok(self.L.mcpt_upload_meshes(h, mb["info"].shape[0], ip(mb["info"]), mb["nodes"].shape[0],
                                               fp(mb["nodes"]), mb["leaves"].size, ip(mb["leaves"]),
                                               mb["tris"].shape[0], ip(mb["tris"]), mb["verts"].shape[0],
                                               fp(mb["verts"]), fp(mb["normals"])))
        self._ok(self.L.mcpt_set_target(h, W, H, 8, 1, 0))

    def _ok(self, st):
        if st != 0:
            raise RuntimeError(self.L.mcpt_error_string(st).decode())

    def render(self, ipv, iv, first, n, B):
        fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
        self._ok(self.L.mcpt_render(self.h, fp(ipv), fp(iv), first, n, 0.0, B, 1.0, 0))

    def kernel_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        self._ok(self.L.mcpt_last_kernel_ms(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value

    def close(self):
        self.L.mcpt_destroy(self.h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=0)
    ap.add_argument("--libs", nargs="+", default=["main"])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--traversal", type=int, default=1)
    ap.add_argument("--walk-exit", type=int, nargs="+", default=[-1])
    ap.add_argument("--leaf-batch", type=int, nargs="+", default=[-1])
    ap.add_argument("--mesh-tris", type=int, default=1_000_000)
    a = ap.parse_args()
    W, H, S, B = a.width, a.height, a.spp, BOUNCES[a.scene]
    if a.scene == 0:
        from mcpt import meshes
        sc = meshes.big_mesh_scene(a.mesh_tris)[0]
    elif a.scene == -1:   # bench.py --config mesh_big
        from mcpt import meshes
        sc = meshes.big_mesh4_scene(a.mesh_tris)[0]
    else:
        sc = mcpt.Scene.reference(a.scene)
    prims, nodes, leaves = sc.buffers()
    bufs = (np.ascontiguousarray(prims), np.ascontiguousarray(nodes), np.ascontiguousarray(leaves, np.int32),
            sc.depth(), sc.nb_emissives())
    mb = sc.mesh_buffers()
    if mb is not None:
        mb = {k: np.ascontiguousarray(v) for k, v in mb.items()}
    ipv, iv = mcpt.camera_canonical(W, H)
    ctxs = [Ctx(lib_path(n), bufs, mb, W, H) for n in a.libs]
    for c in ctxs:
        c._ok(c.L.mcpt_set_traversal(c.h, a.traversal))
    for wx, lb in [(x, b) for x in a.walk_exit for b in a.leaf_batch]:
        for c in ctxs:
            c._ok(c.L.mcpt_set_walk_exit(c.h, wx))
            c._ok(c.L.mcpt_set_leaf_batch(c.h, lb))
            c.render(ipv, iv, 1, S, B)   # warm-up
            c.kernel_ms()
        ms = [[] for _ in ctxs]
        for r in range(a.reps):
            order = range(len(ctxs)) if r % 2 == 0 else reversed(range(len(ctxs)))
            for k in order:
                ctxs[k].render(ipv, iv, 1 + (r + 1) * S, S, B)
                ms[k].append(ctxs[k].kernel_ms())
        for n, m in zip(a.libs, ms):
            m = np.array(m)
            print(json.dumps({"lib": n, "scene": a.scene, "walk_exit": wx, "leaf_batch": lb, "spp": S, "reps": a.reps,
                              "kernel_ms_median": round(float(np.median(m)), 3), "kernel_ms_mean": round(float(m.mean()), 3),
                              "kernel_ms_min": round(float(m.min()), 3),
                              "msamples_s_median": round(W * H * S / float(np.median(m)) / 1e3, 1)}), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
