#!/usr/bin/env python3
"""Per-sample kernel cost of one frame's samples under different launch shapes (scene 6,
1080p, B 8): full frame vs a 1/8-row shard, 256 passes per launch vs one launch of all
passes.  The weak-scaling bench at N GPUs renders a 1/N-row shard with 256·N passes in one
launch per step; its per-sample cost against the full-frame 256-pass launch is the
single-GPU part of the N-GPU efficiency.

    python tools/launch_shape_cost.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import torch  # noqa: E402,F401

import mcpt  # noqa: E402
from mcpt.dist import local_rows  # noqa: E402


def main():
    W, H, B = 1920, 1080, 8
    r = mcpt.Renderer(0)
    r.set_traversal(1)
    r.upload_scene(mcpt.Scene.reference(6))
    ipv, iv = mcpt.camera_canonical(W, H)
    shard = local_rows(H, 8, 8, 0, "balanced")
    cases = [("full", None, 256, 1), ("full", None, 2048, 1), ("full", None, 256, 8),
             ("shard1/8", shard, 2048, 1), ("shard1/8", shard, 256, 8), ("shard1/8", shard, 512, 4),
             ("shard1/8", shard, 1024, 2), ("shard1/4", local_rows(H, 8, 4, 0, "balanced"), 1024, 1)]
    for name, rows, per_launch, launches in cases:
        if rows is None:
            r.set_target(W, H)
        else:
            r.set_target_rows(W, H, rows)
        r.render(ipv, iv, 1, per_launch, 0.0, B, 1.0, 0)   # warm-up
        r.clear_accum()
        best = None
        for rep in range(2):
            tot = 0.0
            for k in range(launches):
                r.render(ipv, iv, k * per_launch + 1, per_launch, 0.0, B, 1.0, 0)
                tot += r.last_kernel_ms()[0]
            best = tot if best is None else min(best, tot)
        n = r.n_local_rows * W * per_launch * launches
        print(json.dumps({"case": name, "rows": r.n_local_rows, "passes_per_launch": per_launch, "launches": launches,
                          "kernel_ms": round(best, 3), "ns_per_ksample": round(best * 1e9 / n, 3),
                          "msamples_s": round(n / best / 1e3, 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
