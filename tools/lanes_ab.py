#!/usr/bin/env python3
"""Render lanes on / off (mcpt_set_render_lanes), measured the way bench.py runs: blocks of K
consecutive render calls of one workload, wall time per call between synchronisations, the two
settings alternating block by block for R rounds in one context (interleaving single calls would
defeat the overlap, which is between consecutive calls of one context).  The accumulator after a
block with lanes equals the one without, bit for bit (checked on the first round).

    python tools/lanes_ab.py [--cases c2 c2_shard8 c4 mesh c5] [--calls 10] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import mcpt  # noqa: E402
from mcpt.dist import local_rows  # noqa: E402

# name: (scene id (0: mesh workload), W, H, passes per call, bounces, shard of N (1: whole frame))
CASES = {"c2": (6, 1920, 1080, 256, 8, 1), "c2_shard8": (6, 1920, 1080, 256, 8, 8),
         "c2_shard4": (6, 1920, 1080, 256, 8, 4), "c4": (8, 1920, 1080, 512, 12, 1),
         "c4_shard8": (8, 1920, 1080, 512, 12, 8), "mesh": (0, 1920, 1080, 64, 8, 1),
         "c5": (6, 3840, 2160, 1024, 8, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", nargs="+", default=["c2", "c2_shard8", "c4", "mesh"])
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    for name in a.cases:
        sid, W, H, S, B, shard = CASES[name]
        if sid == 0:
            from mcpt import meshes
            sc = meshes.big_mesh_scene(1_000_000)[0]
        else:
            sc = mcpt.Scene.reference(sid)
        r = mcpt.Renderer(0)
        r.upload_scene(sc)
        if shard > 1:
            r.set_target_rows(W, H, local_rows(H, 8, shard, 0, "balanced"))
        else:
            r.set_target(W, H)
        ipv, iv = mcpt.camera_canonical(W, H)
        for _ in range(mcpt.AUTO_TRIALS):   # AUTO settles
            r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
        p = 1
        ms = {1: [], 0: []}
        bits = {}
        for rnd in range(a.rounds):
            for on in ((1, 0) if rnd % 2 == 0 else (0, 1)):
                r.set_render_lanes(on)
                r.clear_accum()
                first = p if rnd else 1
                r.synchronize()
                t0 = time.perf_counter()
                q = first
                for _ in range(a.calls):
                    r.render(ipv, iv, q, S, 0.0, B, 1.0, 0)
                    q += S
                r.synchronize()
                ms[on].append((time.perf_counter() - t0) * 1e3 / a.calls)
                if rnd == 0:
                    bits[on] = r.read_accum()[0]
            p += a.calls * S
        same = bool(np.array_equal(bits[1].view(np.uint32), bits[0].view(np.uint32)))
        med = {k: float(np.median(v)) for k, v in ms.items()}
        print(json.dumps({"case": name, "scene": sid, "width": W, "height": H, "spp_per_call": S, "bounces": B,
                          "shard_of": shard, "calls": a.calls, "rounds": a.rounds, "schedule": r.schedule(),
                          "ms_per_call_lanes": [round(x, 3) for x in ms[1]],
                          "ms_per_call_in_order": [round(x, 3) for x in ms[0]],
                          "median_lanes": round(med[1], 3), "median_in_order": round(med[0], 3),
                          "gain": round(med[0] / med[1] - 1.0, 4), "bit_equal": same}), flush=True)
        r.close()


if __name__ == "__main__":
    main()
