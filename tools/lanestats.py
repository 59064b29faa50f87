#!/usr/bin/env python3
"""Lane accounting of the render kernel (diagnostic build MCPT_LANESTATS, never timed).

MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_lanestats.so python tools/lanestats.py

For each workload: how many wave iterations run each block of the walk loop (node block,
the box tests' face and cull stages, leaf block, primitive types) and the shading block, and
how many lanes take part: lanes / (64 x wave iterations) is the block's lane utilisation.
The counts come from ballots at the block entries (mcpt_kernel.hip ls_* helpers).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
import torch  # noqa: E402,F401
import mcpt  # noqa: E402

NAMES = ["node_it", "node_ln", "ne_wv", "ne_ln", "out_wv", "out_ln", "val_wv", "val_ln",
         "leaf_it", "leaf_ln", "prim_ln", "sph_wv", "sph_ln", "cube_wv", "cube_ln", "cyl_wv",
         "cyl_ln", "quad_wv", "quad_ln", "walk_it", "walk_ln", "walk_calls", "rounds", "round_ln",
         "shade_wv", "shade_ln", "rr2_wv", "rr2_ln", "waves", "fit_it", "two_it",
         "snode_it", "snode_ln", "sleaf_it", "sleaf_ln", "exit_ln"]


def util(ln, wv):
    return round(ln / (64.0 * wv), 3) if wv else None


def run(sid, B, spp, seg, leaf_batch, walk_exit, W=1920, H=1080):
    os.environ["MCPT_SEG_PER_ITEM"] = str(seg)
    os.environ["MCPT_LEAF_BATCH"] = str(leaf_batch)   # read when a context is created
    r = mcpt.Renderer(0)
    r.set_traversal(1)
    if sid in (0, -1):   # the mesh workloads (walk_run_mesh: node / leaf = mesh-node / mesh-leaf steps)
        from mcpt import meshes
        r.upload_scene((meshes.big_mesh_scene if sid == 0 else meshes.big_mesh4_scene)(1_000_000)[0])
    else:
        r.upload_scene(mcpt.Scene.reference(sid))
    r.set_target(W, H)
    if walk_exit is not None:
        r.set_walk_exit(walk_exit)
    ipv, iv = mcpt.camera_canonical(W, H)
    r.debug_counters(reset=True)
    r.render(ipv, iv, 1, spp, 0.0, B, 1.0, 0)
    c = r.debug_counters(reset=True).astype(float)[16:16 + len(NAMES)]
    d = dict(zip(NAMES, c))
    out = {"scene": sid, "B": B, "spp": spp, "seg_per_item": seg, "leaf_batch": leaf_batch, "walk_exit": walk_exit,
           "waves": int(d["waves"]),
           "per_wave": {k: round(d[k] / d["waves"], 1) for k in ("rounds", "walk_calls", "walk_it", "node_it",
                                                               "leaf_it", "shade_wv", "rr2_wv")},
           "util": {"round": util(d["round_ln"], d["rounds"]), "walk_loop": util(d["walk_ln"], d["walk_it"]),
                    "node_block": util(d["node_ln"], d["node_it"]),
                    "child_nonempty": util(d["ne_ln"], d["ne_wv"]), "face_stage": util(d["out_ln"], d["out_wv"]),
                    "cull_stage": util(d["val_ln"], d["val_wv"]), "leaf_block": util(d["leaf_ln"], d["leaf_it"]),
                    "sphere": util(d["sph_ln"], d["sph_wv"]), "cube": util(d["cube_ln"], d["cube_wv"]),
                    "cylinder": util(d["cyl_ln"], d["cyl_wv"]), "quad": util(d["quad_ln"], d["quad_wv"]),
                    "shade": util(d["shade_ln"], d["shade_wv"]), "reflect_rr": util(d["rr2_ln"], d["rr2_wv"]),
                    "scene_node": util(d["snode_ln"], d["snode_it"]), "scene_leaf": util(d["sleaf_ln"], d["sleaf_it"])},
           "walk_lanes_at_exit": round(d["exit_ln"] / max(d["walk_calls"], 1), 2),
           "walk_it_share": {k: round(d[k] / max(d["walk_it"], 1), 3) for k in ("node_it", "leaf_it", "snode_it", "sleaf_it")},
           "node_it_share": {"face_jobs_fit_one_round": round(d["fit_it"] / max(d["node_it"], 1), 3),
                             "some_lane_two_face_jobs": round(d["two_it"] / max(d["node_it"], 1), 3),
                             "face_jobs_per_walking_lane": round(d["out_ln"] / max(d["walk_ln"] * d["node_it"] / max(d["walk_it"], 1), 1), 3)},
           "child_tests_per_node_it": {"nonempty_wv": round(d["ne_wv"] / max(d["node_it"], 1), 3),
                                       "face_wv": round(d["out_wv"] / max(d["node_it"], 1), 3),
                                       "cull_wv": round(d["val_wv"] / max(d["node_it"], 1), 3)},
           "raw": {k: int(v) for k, v in d.items()}}
    print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "mesh":   # the mesh workloads (walk_run_mesh) at walk exit 24
        run(0, 8, 64, 1, -1, 24)
        run(-1, 8, 64, 1, -1, 24)
        sys.exit(0)
    run(8, 12, 256, 8, 16, 40)      # C4 shape: deep knobs, eight segments per item
    run(8, 12, 256, 1, 16, 40)
    run(8, 12, 256, 8, 8, 16)       # the depth >= 8 defaults
    run(3, 8, 256, 4, 8, 16)
    run(6, 8, 256, 2, 0, 0)         # C2
