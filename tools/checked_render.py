#!/usr/bin/env python3
"""Render the work-item-order paths that index past the work items (tail pieces, split items)
with one library build (MCPT_LIB) and save the accumulators (tests/test_gpu_checked.py runs it
once with the checked build, libmcpt_checked.so, and once with the shipped build).

    MCPT_LIB=.../variants/libmcpt_checked.so python tools/checked_render.py CASE OUT_DIR

CASE c5:   scene 6, 3840x2160, B 8, three 128-pass calls (1..384) per traversal (per lane,
           wave-coherent) with MCPT_SEG_PER_ITEM=4 set by the caller: the shape round 5's
           fault ran (bench.py --config c5, four segments per item); from the second call the
           launch runs the sorted order with one workgroup-generation of tail pieces.
CASE mesh: the mesh workload (mcpt.meshes.big_mesh_scene, two instances of a 1 M-triangle
           sphere), 1920x1080, B 8, three 64-pass calls: from the second call the costliest items
           run as split items (kSplitPieces pass ranges each).
Prints the build flags, the launches' split count (mesh) and "ok".  A checked build fails the
render call (non-zero exit) on any out-of-range index or fault, naming the sub-launch.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)
import mcpt  # noqa: E402

CASES = {
    "c5": dict(W=3840, H=2160, B=8, calls=(128, 128, 128), traversals=("LANE", "WAVE")),
    "mesh": dict(W=1920, H=1080, B=8, calls=(64, 64, 64), traversals=("LANE",)),
}


def main(case, out):
    os.makedirs(out, exist_ok=True)
    c = CASES[case]
    print("lib", mcpt.lib_path(), "build_flags", mcpt.build_flags(), flush=True)
    if case == "mesh":
        from mcpt import meshes
        sc = meshes.big_mesh_scene(1_000_000)[0]
    else:
        sc = mcpt.Scene.reference(6)
    r = mcpt.Renderer(0)
    try:
        r.upload_scene(sc)
        ipv, iv = mcpt.camera_canonical(c["W"], c["H"])
        for tname in c["traversals"]:
            r.set_traversal(getattr(mcpt, f"TRAVERSAL_{tname}"))
            r.set_target(c["W"], c["H"])
            first = 1
            for n in c["calls"]:
                r.render(ipv, iv, first, n, 0.0, c["B"], 1.0, mcpt.MONTECARLO)
                first += n
            acc, npass = r.read_accum()
            assert npass == first - 1
            np.save(os.path.join(out, f"{case}_{tname}.npy"), acc)
            dbg = r.debug_counters(reset=False)
            print(tname, "passes", npass, "split items of the last sort", int(dbg[63]), flush=True)
    finally:
        r.close()
    print("ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
