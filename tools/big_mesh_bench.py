#!/usr/bin/env python3
"""Large triangle-mesh scenes ("the only route to HBM-sized scenes").

The mesh test scene of tests/test_meshes.py with its sphere instance replaced by a UV sphere of
N triangles (10 K ... 1 M: mesh BVH depth 14 ... 20, up to 100 MB of mesh nodes + 24 MB of
triangles / vertices / normals in HBM), 1920x1080, B 8, per-lane and wave-coherent walks.
Per size: Msamples/s (kernel time, HIP events), the counting build's algorithmic bytes per
sample (SURVEY §8d model incl. the mesh events) and the achieved algorithmic GB/s.

    python tools/big_mesh_bench.py [--sizes 10000 100000 1000000] [--spp 32]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "montecarlo-pathtracing_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import mcpt  # noqa: E402
from mcpt import meshes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[10_000, 100_000, 1_000_000])
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--walk-exit", type=int, nargs="+", default=[-1], help="per-lane walk suspension (mcpt_set_walk_exit)")
    ap.add_argument("--leaf-batch", type=int, nargs="+", default=[-1], help="batched leaf visits (mcpt_set_leaf_batch)")
    a = ap.parse_args()
    W, H, B, S = 1920, 1080, a.bounces, a.spp
    r = mcpt.Renderer(0)
    r.set_target(W, H)
    ipv, iv = mcpt.camera_canonical(W, H)
    eb = mcpt.Renderer.event_bytes()
    for n in a.sizes:
        sc, n_tris = meshes.big_mesh_scene(n)
        r.upload_scene(sc)
        mb = sc.mesh_buffers()
        mesh_mb = sum(x.nbytes for x in mb.values()) / 1e6
        ev = r.render_counted(ipv, iv, 1, S, 0.0, B, 1.0, 0)
        bps = float((ev.astype(np.float64) * eb).sum() / max(float(ev[6]), 1.0))
        for mode, wx, lb in [(1, x, b) for x in a.walk_exit for b in a.leaf_batch] + [(2, -1, -1)]:
            r.set_traversal(mode)
            r.set_walk_exit(wx)
            r.set_leaf_batch(lb)
            r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)   # warm-up
            ms = []
            for k in range(2):
                r.render(ipv, iv, 1 + (k + 1) * S, S, 0.0, B, 1.0, 0)
                ms.append(r.last_kernel_ms()[0])
            t = float(np.mean(ms))
            sps = W * H * S / (t / 1e3)
            print(json.dumps({"triangles_per_instance": n_tris, "instances": 2, "mesh_buffers_mb": round(mesh_mb, 1),
                              "traversal": "lane" if mode == 1 else "wave", "walk_exit": wx, "leaf_batch": lb, "spp": S, "bounces": B,
                              "kernel_ms": round(t, 2), "msamples_s": round(sps / 1e6, 1),
                              "algorithmic_bytes_per_sample": round(bps, 1),
                              "algorithmic_gb_s": round(bps * sps / 1e9, 1),
                              "events_per_sample": {k: round(float(v) / max(float(ev[6]), 1.0), 2)
                                                    for k, v in zip(mcpt.EVENT_NAMES, ev)}}), flush=True)
        r.set_traversal(0)
        r.set_walk_exit(-1)
        r.set_leaf_batch(-1)
    r.close()


if __name__ == "__main__":
    main()
