#!/usr/bin/env python3
"""Projected strong scaling of the default N-GPU bench (bench.py --gpus N, C2: ONE 1080p x 256-spp
frame split N ways) from one GPU: every rank's shard is run as that rank would run it — its own
context, AUTO's trials on its shard's launches, warm-up, then K timed steps back to back (render
+ combine; wall time bracketed by synchronisations) — one rank after another on this GPU.  The
N-GPU step is the slowest rank's; the RCCL gather of the frame (3.1 MB per rank at N = 8) is not
included.  Efficiency = projected N-GPU rate / (N x the 1-rank rate).

    python tools/strong_scaling_projection.py [--worlds 1 2 4 8] [--steps 10] [--config c2|c4|c5]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import torch  # noqa: E402,F401  (HIP runtime first)

import mcpt  # noqa: E402
from mcpt.dist import local_rows  # noqa: E402

CASES = {"c2": (6, 1920, 1080, 256, 8), "c4": (8, 1920, 1080, 512, 12), "c5": (6, 3840, 2160, 1024, 8)}


def rank_step_ms(sc, W, H, S, B, world, rank, steps, warmup, band):
    r = mcpt.Renderer(0)
    try:
        r.upload_scene(sc)
        r.set_target_rows(W, H, local_rows(H, band, world, rank, "balanced"))
        ipv, iv = mcpt.camera_canonical(W, H)
        for _ in range(mcpt.AUTO_TRIALS):
            r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
        r.clear_accum()
        for k in range(warmup):
            r.render(ipv, iv, k * S + 1, S, 0.0, B, 1.0, 0)
        r.synchronize()
        t0 = time.perf_counter()
        for k in range(warmup, warmup + steps):
            r.render(ipv, iv, k * S + 1, S, 0.0, B, 1.0, 0)
        r.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        return ms, r.n_local_rows, r.schedule(), r.last_kernel_ms()[0]
    finally:
        r.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--config", choices=sorted(CASES), default="c2")
    a = ap.parse_args()
    sid, W, H, S, B = CASES[a.config]
    sc = mcpt.Scene.reference(sid)
    base = None
    for world in a.worlds:
        per = [rank_step_ms(sc, W, H, S, B, world, rk, a.steps, a.warmup, a.band_rows) for rk in range(world)]
        slow = max(p[0] for p in per)
        rate = W * H * S / slow / 1e3   # Msamples/s of the projected N-GPU step
        if world == 1:
            base = rate
        print(json.dumps({"config": a.config.upper(), "scaling": "strong", "world": world, "spp_per_step": S,
                          "rank_step_ms": [round(p[0], 3) for p in per], "rank_rows": [p[1] for p in per],
                          "rank_kernel_ms": [round(p[3], 3) for p in per],
                          "rank_schedule": [p[2] for p in per],
                          "projected_step_ms": round(slow, 3), "projected_msamples_s": round(rate, 1),
                          "speedup": round(rate / base, 3) if base else None,
                          "efficiency": round(rate / base / world, 3) if base else None,
                          "note": "one rank after another on one GPU, each its own context; excludes the gather"}),
              flush=True)


if __name__ == "__main__":
    main()
