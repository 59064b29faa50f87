#!/usr/bin/env python3
"""All five BASELINE.json configs on one MI355X (bench.py measures configs[1] only).

    python tools/configs_bench.py [--quick] > profiles/r01_configs.jsonl

One JSON line per measurement, Msamples/s from HIP-event kernel time (`kernel_ms`) and from
wall time around synchronised launches (`wall_ms`):
  C1  scene 1, 256x256, 4 spp, B 3      GPU, and the CPU oracle on the whole config (16 threads)
  C2  scene 6, 1920x1080, 256 spp, B 8  (= bench.py's workload)
  C3  scene 6, 1920x1080, 1024 spp, B 8, IOR 1.5, roughness of every non-emissive primitive
      swept over 0, 0.5, 0.9, 0.99, 1
  C4  scene 8, 1920x1080, 512 spp, B 12, 8-GPU balanced row shards: each of the 8 shards measured in
      turn on this GPU (world 8, rank r); projected 8-GPU rate = all samples / slowest shard
  C5  scene 6, 3840x2160, 8-GPU balanced row shards, progressive: 1024 spp per shard measured (of the
      84,000 spp target); projected time to 84,000 spp on 8 GPUs from the slowest shard
Synthetic inputs: the reference scenes built by the C++ scene producer, canonical camera.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import mcpt  # noqa: E402
from mcpt.dist import local_rows  # noqa: E402


def timed_render(r, ipv, iv, first, spp, B, ior, chunk=256):
    """Render spp passes in launches of `chunk`; returns (kernel ms, wall ms)."""
    kms = 0.0
    r.synchronize()
    t0 = time.perf_counter()
    done = 0
    while done < spp:
        n = min(chunk, spp - done)
        r.render(ipv, iv, first + done, n, 0.0, B, ior, mcpt.MONTECARLO)
        kms += r.last_render_ms()
        done += n
    r.synchronize()
    return kms, (time.perf_counter() - t0) * 1e3


def tune(r, ipv, iv, B, ior, chunk=256):
    """AUTO schedule timing trials (after each scene upload), outside the measurements,
    on launches of the measured shape (timed_render's chunk)."""
    for _ in range(mcpt.AUTO_TRIALS):
        r.render(ipv, iv, 1, chunk, 0.0, B, ior, mcpt.MONTECARLO)
    r.clear_accum()


def emit(rec):
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="fewer passes (smoke run)")
    a = ap.parse_args()
    q = 4 if a.quick else 1
    r = mcpt.Renderer(0)

    # C1 (GPU + the CPU oracle on the whole configuration)
    from oracle import oracle as orc
    W, H, S, B = 256, 256, 4, 3
    r.upload_scene(mcpt.Scene.reference(1))
    r.set_target(W, H)
    ipv, iv = mcpt.camera_canonical(W, H)
    timed_render(r, ipv, iv, 1, S, B, 1.0)   # warm-up
    r.clear_accum()
    kms, wms = timed_render(r, ipv, iv, 1, S, B, 1.0)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    prims, nodes, leaves, depth, _ = orc.scene(1)
    oipv, oiv = orc.camera(W, H)
    t0 = time.perf_counter()
    orc.render(prims, nodes, leaves, depth, oipv, oiv, W, H, 1, S, 0.0, B, 1.0, 0, n_threads=threads)
    cpu_s = time.perf_counter() - t0
    n = W * H * S
    emit({"config": "C1", "scene": 1, "width": W, "height": H, "spp": S, "bounces": B, "kernel_ms": round(kms, 3),
          "wall_ms": round(wms, 3), "msamples_s_kernel": round(n / kms / 1e3, 1),
          "msamples_s_wall": round(n / wms / 1e3, 1), "cpu_oracle_s": round(cpu_s, 3),
          "cpu_oracle_msamples_s": round(n / cpu_s / 1e6, 2), "cpu_threads": threads,
          "note": "tiny launch: wall time is launch/sync overhead"})

    # C2
    W, H, S, B = 1920, 1080, 256 // q, 8
    r.upload_scene(mcpt.Scene.reference(6))
    r.set_target(W, H)
    ipv, iv = mcpt.camera_canonical(W, H)
    tune(r, ipv, iv, B, 1.0)
    timed_render(r, ipv, iv, 1, S, B, 1.0)
    kms, wms = timed_render(r, ipv, iv, S + 1, S, B, 1.0)
    n = W * H * S
    emit({"config": "C2", "scene": 6, "width": W, "height": H, "spp": S, "bounces": B, "kernel_ms": round(kms, 3),
          "wall_ms": round(wms, 3), "msamples_s_kernel": round(n / kms / 1e3, 1),
          "msamples_s_wall": round(n / wms / 1e3, 1)})

    # C3: IOR 1.5, roughness sweep over the non-emissive primitives
    S = 1024 // q
    for rough in (0.0, 0.5, 0.9, 0.99, 1.0):
        sc = mcpt.Scene.reference(6)
        prims, _, _ = sc.buffers()
        for i in range(sc.nb_prim()):
            rec = prims[i]
            if rec[58] > 0:
                continue
            sc.set_material(i, np.concatenate([rec[52:56], [rec[56], rough, rec[58]]]).astype(np.float32))
        r.upload_scene(sc)
        tune(r, ipv, iv, B, 1.5)
        timed_render(r, ipv, iv, 1, 64, B, 1.5)
        kms, wms = timed_render(r, ipv, iv, 65, S, B, 1.5)
        n = W * H * S
        emit({"config": "C3", "scene": 6, "width": W, "height": H, "spp": S, "bounces": B, "ior": 1.5,
              "roughness": rough, "kernel_ms": round(kms, 3), "wall_ms": round(wms, 3),
              "msamples_s_kernel": round(n / kms / 1e3, 1), "msamples_s_wall": round(n / wms / 1e3, 1)})

    # C4 / C5: the 8 row-band shards of the 8-GPU runs, each measured on this GPU
    for cfg, sid, W, H, S, B in (("C4", 8, 1920, 1080, 512 // q, 12), ("C5", 6, 3840, 2160, 1024 // q, 8)):
        r.upload_scene(mcpt.Scene.reference(sid))
        ipv, iv = mcpt.camera_canonical(W, H)
        shard_ms = []
        for rank in range(8):
            r.set_target_rows(W, H, local_rows(H, 8, 8, rank, "balanced"))   # = bench.py's partition
            if rank == 0:   # one call of all S passes per shard, as an N-GPU run makes it
                tune(r, ipv, iv, B, 1.0, chunk=S)
                timed_render(r, ipv, iv, 1, 32, B, 1.0)
                r.clear_accum()
            kms, wms = timed_render(r, ipv, iv, 1, S, B, 1.0, chunk=S)
            shard_ms.append(kms)
            emit({"config": cfg, "scene": sid, "width": W, "height": H, "spp": S, "bounces": B, "world": 8,
                  "rank": rank, "shard_rows": r.n_local_rows, "kernel_ms": round(kms, 3), "wall_ms": round(wms, 3),
                  "msamples_s_kernel": round(r.n_local_rows * W * S / kms / 1e3, 1)})
        n = W * H * S
        rec = {"config": cfg, "scene": sid, "width": W, "height": H, "spp": S, "bounces": B, "world": 8,
               "summary": True, "slowest_shard_ms": round(max(shard_ms), 3),
               "projected_8gpu_msamples_s": round(n / max(shard_ms) / 1e3, 1),
               "shard_balance": round(min(shard_ms) / max(shard_ms), 3),
               "note": "projection from per-shard kernel times measured on one GPU; excludes the RCCL gather"}
        if cfg == "C5":
            rec["projected_8gpu_s_to_84000spp"] = round(max(shard_ms) / 1e3 * 84000 / S, 1)
        emit(rec)
    r.close()


if __name__ == "__main__":
    main()
