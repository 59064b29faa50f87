#!/usr/bin/env python3
"""BASELINE config C5 at its full target: scene 6, 3840x2160, 84,000 spp, B 8, the 8 row
shards of an 8-GPU run (the balanced partition bench.py uses, mcpt_balanced_rows), each rendered on this GPU as ONE mcpt_render call of 84,000 passes
(the library cuts it into chunk-aligned launches within its segment-sum budget).

Whole frame (round 6, verdict r05 #6): the 3840x2160 frame accumulated progressively in 1,024-pass
calls (C5's step) up to 84,000 passes on this GPU — the measured one-GPU time to target — and
`--oracle-pixels` pixels of its
accumulator checked bit for bit against the CPU oracle's sums of the same 84,000 passes
(oracle.render_pixels, the chunked accumulation contract), so the last passes are covered too.

Per shard: kernel time (sum over the call's launches, HIP events), wall time of the call,
launch count.  The slowest shard is the 8-GPU time to 84,000 spp (shards are independent;
the one RCCL gather of the 99.5 MB frame is not included).  Rank 0 is also rendered as the
progressive sequence of 1,024-pass calls C5 describes, which must give the same bits.

    python tools/c5_full.py [--passes 84000] [--ranks 0 1 ... 7] [--no-progressive-check]
                            [--no-whole] [--oracle-pixels 256]
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

W, H, B, WORLD, BAND = 3840, 2160, 8, 8, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=84000)
    ap.add_argument("--ranks", type=int, nargs="+", default=list(range(WORLD)))
    ap.add_argument("--no-progressive-check", action="store_true")
    ap.add_argument("--traversal", type=int, default=0, help="0 AUTO (trials on 256-pass launches), 1 lane, 2 wave")
    ap.add_argument("--seg-per-item", type=int, default=0, help="> 0: MCPT_SEG_PER_ITEM for every launch")
    ap.add_argument("--no-whole", action="store_true", help="skip the whole-frame one-GPU run")
    ap.add_argument("--step", type=int, default=1024, help="whole frame: passes per progressive call (C5's step)")
    ap.add_argument("--one-call", action="store_true", help="whole frame: one call of all the passes")
    ap.add_argument("--oracle-pixels", type=int, default=256, help="whole-frame pixels checked against the oracle")
    a = ap.parse_args()
    if a.seg_per_item > 0:
        os.environ["MCPT_SEG_PER_ITEM"] = str(a.seg_per_item)
    ipv, iv = mcpt.camera_canonical(W, H)
    whole = None
    if not a.no_whole:
        # the whole frame on this GPU, as C5 defines it: progressive accumulation in calls of
        # `--step` passes (bench.py --config c5's step) up to the target — the one-GPU time to target,
        # measured (with --one-call: ONE call of all the passes instead)
        r = mcpt.Renderer(0)   # its own context: AUTO settles on this target's launches
        r.set_traversal(a.traversal)
        r.upload_scene(mcpt.Scene.reference(6))
        r.set_target(W, H)
        step = a.passes if a.one_call else a.step
        for _ in range(mcpt.AUTO_TRIALS):   # AUTO's trials on this target's step-sized launches
            r.render(ipv, iv, 1, min(step, 1024), 0.0, B, 1.0, 0)
        r.clear_accum()
        r.synchronize()
        t0 = time.perf_counter()
        p, calls = 1, 0
        while p <= a.passes:
            k = min(step, a.passes - p + 1)
            r.render(ipv, iv, p, k, 0.0, B, 1.0, 0)
            p += k
            calls += 1
        r.synchronize()
        wall = time.perf_counter() - t0
        acc, n = r.read_accum()
        assert n == a.passes and np.isfinite(acc).all()
        whole = {"config": "C5", "whole_frame": True, "width": W, "height": H, "spp": a.passes, "bounces": B,
                 "calls": calls, "passes_per_call": step, "time_to_target_s": round(wall, 3),
                 "msamples_s_wall": round(W * H * a.passes / wall / 1e6, 1), "schedule": r.schedule(),
                 "mean_radiance": [round(float(v), 5) for v in (acc.reshape(-1, 3).mean(0) / a.passes)]}
        if a.oracle_pixels > 0:
            sys.path.insert(0, REPO)
            from oracle import oracle as orc   # the checker (test infrastructure), after the timed call
            rng = np.random.default_rng(84000)
            xs = rng.integers(0, W, a.oracle_pixels)
            ys = rng.integers(0, H, a.oracle_pixels)
            prims, nodes, leaves, depth, _ = orc.scene(6)
            oipv, oiv = orc.camera(W, H)
            t1 = time.perf_counter()
            ref = orc.render_pixels(prims, nodes, leaves, depth, oipv, oiv, W, H, np.stack([xs, ys], 1), 1, a.passes,
                                    0.0, B, 1.0, 0, n_threads=16)
            got = acc[ys, xs]
            diff = int((got.view(np.uint32) != ref.view(np.uint32)).sum())
            whole["oracle_check"] = {"pixels": int(a.oracle_pixels), "passes": f"1..{a.passes}",
                                     "channels_differing": diff, "bit_equal": diff == 0,
                                     "oracle_s": round(time.perf_counter() - t1, 1),
                                     "pixels_seed": 84000}
        print(json.dumps(whole), flush=True)
        r.close()
    r = mcpt.Renderer(0)
    r.set_traversal(a.traversal)
    r.upload_scene(mcpt.Scene.reference(6))
    r.set_target_rows(W, H, local_rows(H, BAND, WORLD, 0, "balanced"))
    # AUTO traversal trials on this launch shape first (same bits either way)
    for _ in range(mcpt.AUTO_TRIALS):
        r.render(ipv, iv, 1, 256, 0.0, B, 1.0, 0)
    shard_ms = []
    for rank in a.ranks:
        r.set_target_rows(W, H, local_rows(H, BAND, WORLD, rank, "balanced"))
        r.synchronize()
        t0 = time.perf_counter()
        r.render(ipv, iv, 1, a.passes, 0.0, B, 1.0, 0)
        r.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        kms, cms = r.last_kernel_ms()
        acc, n = r.read_accum()
        assert n == a.passes and np.isfinite(acc).all()
        rec = {"config": "C5", "scene": 6, "width": W, "height": H, "spp": a.passes, "bounces": B, "world": WORLD,
               "rank": rank, "shard_rows": r.n_local_rows, "launches": r.last_launch_count(),
               "kernel_ms": round(kms, 1), "combine_ms": round(cms, 2), "wall_ms": round(wall, 1),
               "msamples_s_wall": round(r.n_local_rows * W * a.passes / wall / 1e3, 1),
               "mean_radiance": [round(float(v), 5) for v in (acc.reshape(-1, 3).mean(0) / a.passes)]}
        if rank == a.ranks[0] and not a.no_progressive_check:
            one = acc.copy()
            r.clear_accum()
            p = 1
            while p <= a.passes:
                k = min(1024, a.passes - p + 1)
                r.render(ipv, iv, p, k, 0.0, B, 1.0, 0)
                p += k
            prog, n2 = r.read_accum()
            rec["progressive_1024_bit_equal"] = bool(n2 == a.passes and np.array_equal(one.view(np.uint32),
                                                                                       prog.view(np.uint32)))
        shard_ms.append(wall)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"config": "C5", "summary": True, "spp": a.passes, "ranks": a.ranks,
                      "traversal": a.traversal, "seg_per_item": a.seg_per_item,
                      "slowest_shard_wall_s": round(max(shard_ms) / 1e3, 2),
                      "shard_balance": round(min(shard_ms) / max(shard_ms), 3),
                      "one_gpu_time_to_target_s": whole["time_to_target_s"] if whole else None,
                      "one_gpu_oracle_bit_equal": whole.get("oracle_check", {}).get("bit_equal") if whole else None,
                      "projected_8gpu_msamples_s": round(W * H * a.passes / max(shard_ms) / 1e3, 1),
                      "note": "8-GPU time to target = slowest shard (independent shards, measured one after "
                              "another on one GPU); excludes the one RCCL gather of the 99.5 MB frame"}),
          flush=True)
    r.close()


if __name__ == "__main__":
    main()
