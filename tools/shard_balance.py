#!/usr/bin/env python3
"""Row-band shard balance: every rank's shard of an N-GPU frame rendered on this GPU, one
after another, for several band heights (mcpt_set_target band_rows).

The N-GPU step time is the slowest shard's (max over ranks), so the balance min/max of the
shard kernel times bounds the scaling efficiency the row-band split can reach.

    python tools/shard_balance.py [--world 8] [--bands 1 2 4 8] [--cases bench c4]
                                  [--partitions balanced bands]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import torch  # noqa: E402,F401

import mcpt  # noqa: E402
from mcpt.dist import local_rows  # noqa: E402

# bench: bench.py's weak-scaling step at N GPUs (256·N passes per step); c4: BASELINE config C4
CASES = {"bench": (6, 1920, 1080, 256, 8, True), "c4": (8, 1920, 1080, 512, 12, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--bands", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--cases", nargs="+", default=["bench", "c4"])
    ap.add_argument("--partitions", nargs="+", default=["balanced", "bands"])
    a = ap.parse_args()
    r = mcpt.Renderer(0)
    r.set_traversal(1)   # the per-lane walk AUTO picks for both scenes (no per-shape trials)
    for case in a.cases:
        sid, W, H, spp, B, weak = CASES[case]
        S = spp * a.world if weak else spp
        r.upload_scene(mcpt.Scene.reference(sid))
        ipv, iv = mcpt.camera_canonical(W, H)
        for part, band in [(pt, b) for pt in a.partitions for b in a.bands]:
            ms = []
            for rank in range(a.world):
                if part == "bands":
                    r.set_target(W, H, band, a.world, rank)
                else:
                    r.set_target_rows(W, H, local_rows(H, band, a.world, rank, part))
                if rank == 0:   # warm-up
                    r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
                r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
                ms.append(r.last_kernel_ms()[0])
            print(json.dumps({"case": case, "scene": sid, "width": W, "height": H, "spp": S, "bounces": B,
                              "world": a.world, "partition": part, "band_rows": band, "shard_ms": [round(x, 2) for x in ms],
                              "slowest_ms": round(max(ms), 2), "balance": round(min(ms) / max(ms), 4),
                              "projected_msamples_s": round(W * H * S / max(ms) / 1e3, 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
