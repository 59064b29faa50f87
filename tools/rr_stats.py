#!/usr/bin/env python3
"""random_ray job statistics of the rr_jobs compaction (diagnostic build, MCPT_RR_STATS):

    MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_rrstats.so python tools/rr_stats.py

Per scene: shading rounds per wave, jobs per round (first / total), active lanes per round,
batches per round and the share of rounds whose jobs exceed the active lanes."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
import torch  # noqa: E402,F401
import mcpt  # noqa: E402

W, H, S = 1920, 1080, 64
r = mcpt.Renderer(0)
r.set_target(W, H)
ipv, iv = mcpt.camera_canonical(W, H)
for sid, B in [(6, 8), (1, 3), (3, 8), (8, 12)]:
    r.upload_scene(mcpt.Scene.reference(sid))
    r.set_traversal(1)
    r.debug_counters(reset=True)
    r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
    c = r.debug_counters(reset=True).astype(float)
    calls, batches, jobs, active, over, jobs1, waves = c[0:7]
    print(json.dumps({"scene": sid, "waves": int(waves), "rounds_per_wave": round(calls / waves, 1),
                      "jobs_per_round": round(jobs / calls, 2), "ray_jobs_per_round": round(jobs1 / calls, 2),
                      "active_per_round": round(active / calls, 2), "batches_per_round": round(batches / calls, 3),
                      "share_rounds_over": round(over / calls, 3)}), flush=True)
