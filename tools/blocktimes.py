#!/usr/bin/env python3
"""Occupancy of one render launch over time, from the MCPT_BLOCKTIMES diagnostic build
(``make -C montecarlo-pathtracing_amd/csrc blocktimes``; never timed): every wave's start and end
on the 100 MHz real-time clock.  Per workload: the launch span, the waves' summed lifetimes
against (peak concurrent waves x span) = how full the launch kept the chip, the tail (the time
from the moment the running-wave count falls below 90 % of its peak for good to the end), and
each XCD group's (blockIdx % 8) last end.

    MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_blocktimes.so \\
        python tools/blocktimes.py [c2] [c4] [mesh] [--seg K] [--auto] [--shard N]

--shard N: rank 0's shard of an N-GPU strong run (mcpt_balanced_rows, 8-row bands) instead of the
whole frame.
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import mcpt  # noqa: E402

CASES = {"c2": (6, 256, 8), "c4": (8, 512, 12), "mesh": (0, 64, 8)}
CLOCK_HZ = 100e6


def analyse(t: np.ndarray, waves_per_item: int = 4) -> dict:
    t = t.reshape(-1, 2)
    live = t[:, 1] > 0
    idx = np.nonzero(live)[0]
    st, en = t[live, 0].astype(np.float64), t[live, 1].astype(np.float64)
    t0 = st.min()
    st, en = (st - t0) / CLOCK_HZ * 1e3, (en - t0) / CLOCK_HZ * 1e3   # ms
    span = en.max()
    ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    run = np.cumsum(ev[:, 1])
    peak = run.max()
    below = np.nonzero(run >= 0.9 * peak)[0]
    t_drop = ev[below[-1] + 1, 0] if len(below) and below[-1] + 1 < len(ev) else span
    life = en - st
    items = idx // waves_per_item
    xcd = items % 8
    xcd_end = [round(float(en[xcd == k].max()), 3) for k in range(8) if (xcd == k).any()]
    # running waves (fraction of the peak) at 20 evenly spaced instants of the launch
    grid = np.linspace(0.0, span, 21)[:-1] + span / 40
    prof = [round(float(((st <= g) & (en > g)).sum()) / peak, 3) for g in grid]
    return {"waves": int(live.sum()), "span_ms": round(float(span), 3), "peak_waves": int(peak),
            "occupancy_profile": prof,
            "fill": round(float(life.sum() / (peak * span)), 4),
            "tail_ms": round(float(span - t_drop), 3), "tail_frac": round(float((span - t_drop) / span), 4),
            "wave_life_ms": {"mean": round(float(life.mean()), 3), "p50": round(float(np.median(life)), 3),
                             "p99": round(float(np.percentile(life, 99)), 3), "max": round(float(life.max()), 3)},
            "last_start_ms": round(float(st.max()), 3), "xcd_group_end_ms": xcd_end}


def main():
    names = [a for a in sys.argv[1:] if a in CASES] or ["c2", "c4", "mesh"]
    seg = int(sys.argv[sys.argv.index("--seg") + 1]) if "--seg" in sys.argv else 0
    L = mcpt.lib()
    if not hasattr(L, "mcpt_debug_blocktimes"):
        sys.exit("blocktimes.py needs the MCPT_BLOCKTIMES build (MCPT_LIB=.../libmcpt_blocktimes.so)")
    L.mcpt_debug_blocktimes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_longlong]
    W, H = 1920, 1080
    ipv, iv = mcpt.camera_canonical(W, H)
    for name in names:
        sid, S, B = CASES[name]
        r = mcpt.Renderer(0)
        if sid == 0:
            from mcpt import meshes
            r.upload_scene(meshes.big_mesh_scene(1_000_000)[0])
        else:
            r.upload_scene(mcpt.Scene.reference(sid))
        shard = int(sys.argv[sys.argv.index("--shard") + 1]) if "--shard" in sys.argv else 1
        if shard > 1:
            from mcpt.dist import local_rows
            r.set_target_rows(W, H, local_rows(H, 8, shard, 0, "balanced"))
        else:
            r.set_target(W, H)
        auto = "--auto" in sys.argv
        r.set_traversal(mcpt.TRAVERSAL_AUTO if auto else mcpt.TRAVERSAL_LANE)
        if seg:
            os.environ["MCPT_SEG_PER_ITEM"] = str(seg)
        # warm-up (first touch of the scene; with --auto, AUTO's timing trials until it settles)
        for k in range(12 if auto else 1):   # (LANE: one warm-up; the timed launch is the 13th pass range either way)
            r.render(ipv, iv, 1 + k * S, S, 0.0, B, 1.0, 0)
        n = 8 << 20
        buf = (ctypes.c_ulonglong * n)()
        L.mcpt_debug_blocktimes(r._h, buf, n)   # (zeroes the slots)
        r.render(ipv, iv, 1 + 12 * S, S, 0.0, B, 1.0, 0)
        L.mcpt_debug_blocktimes(r._h, buf, n)
        sched = r.schedule()
        t = np.frombuffer(buf, dtype=np.uint64)
        res = {"workload": name, "scene": sid, "spp": S, "bounces": B, "seg_per_item_env": seg or None,
               "traversal": "AUTO" if auto else "LANE", "schedule": sched, "shard_of": shard}
        res.update(analyse(t, waves_per_item=1 if sid == 0 else 2))   # waves per workgroup (tile_w_for; records by workgroup)
        print(json.dumps(res), flush=True)
        r.close()


if __name__ == "__main__":
    main()
