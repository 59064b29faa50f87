#!/usr/bin/env python3
"""Kernel time of the C2 frame (scene 6, 1080p, B 8) per 256-pass launch across pass ranges
1..256, 257..512, ..., 1793..2048: the weak-scaling bench at N GPUs renders passes up to
256·N, so a cost that drifts with the pass number shows up as apparent scaling loss.

    python tools/pass_range_cost.py [--ranges 8] [--reps 2]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import torch  # noqa: E402,F401

import mcpt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranges", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--scene", type=int, default=6)
    ap.add_argument("--bounces", type=int, default=8)
    a = ap.parse_args()
    W, H, S = 1920, 1080, 256
    r = mcpt.Renderer(0)
    r.set_traversal(1)
    r.upload_scene(mcpt.Scene.reference(a.scene))
    r.set_target(W, H)
    ipv, iv = mcpt.camera_canonical(W, H)
    r.render(ipv, iv, 1, S, 0.0, a.bounces, 1.0, 0)   # warm-up
    for k in range(a.ranges):
        ms = []
        for _ in range(a.reps):
            r.render(ipv, iv, k * S + 1, S, 0.0, a.bounces, 1.0, 0)
            ms.append(r.last_kernel_ms()[0])
        print(json.dumps({"scene": a.scene, "first_pass": k * S + 1, "passes": S, "kernel_ms": [round(x, 3) for x in ms],
                          "msamples_s": round(W * H * S / min(ms) / 1e3, 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
