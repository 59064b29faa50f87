#!/usr/bin/env python3
"""The reference's only published numbers (ImGui FPS in captures/, 1280x1000,
9 bounces, light 0.443, IOR 1, one path per pixel per frame, unstated GPU) next to this
renderer on the same settings, one MI355X:
  * fps_1pass: one pass per launch, launch + synchronize per frame (wall clock), like the
    reference's one-path frames (its FPS also includes the display pass and ImGui);
  * msamples_s: 64-pass launches, kernel time.
    python tools/captures_bench.py > profiles/r01_vs_captures.jsonl
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import torch  # noqa: E402,F401  (HIP runtime first)

import mcpt  # noqa: E402

REF_FPS = {1: 26.96, 2: 15.63, 3: 18.73, 4: 21.54, 5: 65.35, 7: 10.16, 8: 5.12}
W, H, B, LIGHT = 1280, 1000, 9, 0.443


def main():
    r = mcpt.Renderer(0)
    r.set_target(W, H)
    ipv, iv = mcpt.camera_canonical(W, H)
    for sid in (1, 2, 3, 4, 5, 6, 7, 8):
        r.upload_scene(mcpt.Scene.reference(sid, LIGHT))
        for k in range(mcpt.AUTO_TRIALS):         # warm-up incl. AUTO's timing trials
            r.render(ipv, iv, 1 + 64 * k, 64, 0.0, B, 1.0, 0)
        r.synchronize()
        kms = 0.0
        for k in range(4):
            r.render(ipv, iv, 1 + 64 * (mcpt.AUTO_TRIALS + k), 64, 0.0, B, 1.0, 0)
            kms += r.last_render_ms()
        rate = W * H * 256 / kms / 1e3
        frames = 50
        r.synchronize()
        t0 = time.perf_counter()
        for f in range(frames):
            r.render(ipv, iv, 449 + f, 1, 0.0, B, 1.0, 0)
            r.synchronize()
        fps = frames / (time.perf_counter() - t0)
        rec = {"scene": sid, "width": W, "height": H, "bounces": B, "light": LIGHT, "fps_1pass": round(fps, 1),
               "msamples_s": round(rate, 1)}
        if sid in REF_FPS:
            rec["reference_fps"] = REF_FPS[sid]
            rec["reference_msamples_s"] = round(REF_FPS[sid] * W * H / 1e6, 1)
            rec["x_vs_reference_fps"] = round(fps / REF_FPS[sid], 1)
            rec["x_vs_reference_msamples_s"] = round(rate / (REF_FPS[sid] * W * H / 1e6), 1)
        print(json.dumps(rec), flush=True)
    r.close()


if __name__ == "__main__":
    main()
