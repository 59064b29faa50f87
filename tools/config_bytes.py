#!/usr/bin/env python3
"""Algorithmic bytes per sample (SURVEY.md §8d texel-fetch model) of each BASELINE config,
counted by the CPU oracle's event counters on a row/pass sample of the config's workload
(every 8th row of the full-size frame, 8 passes from the config's first pass).

    python tools/config_bytes.py > profiles/r01_config_bytes.jsonl
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from oracle import oracle as orc  # noqa: E402

# (config, scene, W, H, B, ior, first pass)
CONFIGS = [("C1", 1, 256, 256, 3, 1.0, 1), ("C2", 6, 1920, 1080, 8, 1.0, 1), ("C3", 6, 1920, 1080, 8, 1.5, 1),
           ("C4", 8, 1920, 1080, 12, 1.0, 1), ("C5", 6, 3840, 2160, 8, 1.0, 83969)]


def main():
    for name, sid, W, H, B, ior, first in CONFIGS:
        prims, nodes, leaves, d, _ = orc.scene(sid)
        ipv, iv = orc.camera(W, H)
        step = 1 if H <= 256 else 8
        acc = np.zeros((H, W, 3), np.float32)
        _, ev = orc.render(prims, nodes, leaves, d, ipv, iv, W, H, first, 8, 0.0, B, ior, 0, row_step=step,
                           accum=acc)
        n = float(ev[6])
        bps = float((ev.astype(np.float64) * orc.EV_BYTES[:len(ev)]).sum() / n)
        print(json.dumps({"config": name, "scene": sid, "width": W, "height": H, "bounces": B, "ior": ior,
                          "sample": f"every {step}th row, passes {first}..{first + 7}", "samples": int(n),
                          "algorithmic_bytes_per_sample": round(bps, 1),
                          "events_per_sample": {k: round(float(v) / n, 3) for k, v in zip(orc.EV_NAMES, ev)}}),
              flush=True)


if __name__ == "__main__":
    main()
