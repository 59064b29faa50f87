#!/usr/bin/env python3
"""Section shares from the diagnostic stamp build (MCPT_LIB=.../libmcpt_stamps.so).

Per scene/traversal mode (--mesh: the mesh workload, "scene" 0): wave-cycles in the primary-ray prelude, in traversal rounds and
in shading rounds, and the lane utilisation of the rounds (participating lanes /
(64 x rounds)).  Shares only: stamps perturb timing.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
import torch  # noqa: E402,F401
import mcpt  # noqa: E402

W, H, S = 1920, 1080, 32
r = mcpt.Renderer(0)
if "--stream" in sys.argv:
    # the stream schedule's trace kernel (persistent waves): walk-loop iterations and lanes per
    # block over the kernel's whole life, scene 8 at B 12 (its iterations reset nothing in between)
    r.set_target(W, H)
    ipv, iv = mcpt.camera_canonical(W, H)
    r.upload_scene(mcpt.Scene.reference(8))
    r.set_traversal(mcpt.TRAVERSAL_STREAM)
    r.debug_counters(reset=True)
    r.render(ipv, iv, 1, 64, 0.0, 12, 1.0, 0)
    c = r.debug_counters(reset=True).astype(float)
    lit, wit, nl, nw, ll, lw = c[9:15]
    print(json.dumps({"scene": 8, "mode": "stream", "spp": 64, "wave_lives": int(c[6]),
                      "walk_loop_simd_util": round(lit / (64 * wit), 3) if wit else None,
                      "node_block_lane_util": round(nl / (64 * nw), 3) if nw else None,
                      "leaf_block_lane_util": round(ll / (64 * lw), 3) if lw else None,
                      "node_iters": nw, "leaf_iters": lw, "iters": wit,
                      "lane_node_visits": nl, "lane_leaf_visits": ll}), flush=True)
    r.close()
    sys.exit(0)
r.set_target(W, H)
ipv, iv = mcpt.camera_canonical(W, H)
CASES = [(6, 8), (3, 8), (8, 12)]
if "--mesh" in sys.argv:   # the mesh workload (bench.py --config mesh), per-lane walk
    from mcpt import meshes
    CASES = [(0, 8)]
for sid, B in CASES:
    r.upload_scene(meshes.big_mesh_scene(1_000_000)[0] if sid == 0 else mcpt.Scene.reference(sid))
    for mode in (1,):
        r.set_traversal(mode)
        r.debug_counters(reset=True)
        r.render(ipv, iv, 1, S, 0.0, B, 1.0, 0)
        c = r.debug_counters(reset=True).astype(float)
        tot, pre, trav, rest, it, lane_it, waves, leaf, lane_tr, t_lit, t_wit, nl, nw, ll, lw = c[:15]
        print(json.dumps({"scene": sid, "mode": mode, "waves": int(waves),
                          "share_prelude": round(pre / tot, 3), "share_traverse_rounds": round(trav / tot, 3),
                          "share_shade_rounds": round(rest / tot, 3),
                          "share_leaf_blocks": round(leaf / tot, 3),
                          "rounds_per_wave": round(it / waves, 1),
                          "lane_util": round(lane_it / (64 * it), 3),
                          "trav_lane_util": round(lane_tr / (64 * it), 3) if lane_tr else None,
                          "trav_loop_simd_util": round(t_lit / (64 * t_wit), 3) if t_wit else None,
                          "trav_loop_iters_per_wave": round(t_wit / waves, 1),
                          "node_block_lane_util": round(nl / (64 * nw), 3) if nw else None,
                          "leaf_block_lane_util": round(ll / (64 * lw), 3) if lw else None,
                          "node_block_iters_per_wave": round(nw / waves, 1),
                          "leaf_block_iters_per_wave": round(lw / waves, 1),
                          "cycles_per_round": round((trav + rest) / it, 1)}), flush=True)
r.close()
