#!/usr/bin/env python3
"""Segments per work item (MCPT_SEG_PER_ITEM) A/B under the bench's execution: blocks of K
consecutive render calls of one workload (render lanes on), the settings alternating block by block
for R rounds in one context; wall time per call between synchronisations.

    python tools/seg_ab.py [--case c2] [--segs 1 2 4] [--calls 10] [--rounds 4]
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

CASES = {"c2": (6, 1920, 1080, 256, 8), "c3": (6, 1920, 1080, 1024, 8), "c5": (6, 3840, 2160, 1024, 8),
         "c4": (8, 1920, 1080, 512, 12)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", choices=sorted(CASES), default="c2")
    ap.add_argument("--segs", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    sid, W, H, S, B = CASES[a.case]
    r = mcpt.Renderer(0)
    r.upload_scene(mcpt.Scene.reference(sid))
    r.set_target(W, H)
    r.set_traversal(mcpt.TRAVERSAL_LANE)
    ipv, iv = mcpt.camera_canonical(W, H)
    ms = {k: [] for k in a.segs}
    p = 1
    for rnd in range(a.rounds + 1):   # round 0: warm-up of every setting (its work-item order)
        for k in (a.segs if rnd % 2 == 0 else list(reversed(a.segs))):
            os.environ["MCPT_SEG_PER_ITEM"] = str(k)
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                r.render(ipv, iv, p, S, 0.0, B, 1.0, 0)
                p += S
            r.synchronize()
            if rnd:
                ms[k].append((time.perf_counter() - t0) * 1e3 / a.calls)
    os.environ.pop("MCPT_SEG_PER_ITEM", None)
    r.close()
    med = {k: float(np.median(v)) for k, v in ms.items()}
    best = min(med, key=med.get)
    print(json.dumps({"case": a.case, "calls": a.calls, "rounds": a.rounds,
                      "ms_per_call": {str(k): [round(x, 3) for x in v] for k, v in ms.items()},
                      "median_ms": {str(k): round(v, 3) for k, v in med.items()},
                      "msamples_s": {str(k): round(W * H * S / v / 1e3, 1) for k, v in med.items()},
                      "best_seg_per_item": best}), flush=True)


if __name__ == "__main__":
    main()
