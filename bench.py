#!/usr/bin/env python3
"""bench.py — north-star benchmark of the MI355X path tracer.

Workload (BASELINE.json configs[1], "C2"): scene 6 (scene_4boules), 1920×1080, 256 spp per
step, 8 bounces, IOR 1.0, light intensity 1.2, date 0, canonical camera, variant
montecarlo.frag.  A *step* = one full C2 frame: passes [k·256+1, (k+1)·256] accumulated
into the device framebuffer, then the frame gathered to rank 0 (RCCL gather for N>1).
Scene buffers and the framebuffer are resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Multi-GPU: weak scaling — per-GPU work fixed at one C2 frame's worth of samples: at N GPUs
a step accumulates 256·N passes of the 1080p frame (progressive accumulation, as configs
C4/C5 do), the frame split into balanced row shards across ranks (mcpt_balanced_rows:
rotated 8-row bands; each rank H/N rows × 256·N passes = one C2 frame of samples), then one
RCCL gather of the fp32 RGB shards to rank 0 inside the timed region.  Bit-identical to rendering the same passes on one GPU.

Prints ONE JSON line (rank 0) with `roofline` (dominant kernel = the path-tracing
kernel; achieved = algorithmic bytes per launch, counted exactly by the counting build
of the same kernel over the same pass range (SURVEY.md §8d byte model), ÷ its average
launch time from HIP events on its stream) and `cpu_baseline` (the C++ oracle on a
bounded row/pass sample of the same workload, host threads stated).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (loads the HIP runtime first; libmcpt binds to the same one)
import torch.distributed as dist  # noqa: E402

import mcpt  # noqa: E402
from mcpt.dist import ShardedRenderer  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_T = 78.64     # 256 CUs x 4 SIMD x 32 lanes/clk x 2.4 GHz (wave64 VALU = 2 clk/SIMD)
METRIC = "Msamples/s (W×H×spp/s) + achieved HBM GB/s, 1080p scene6, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", type=int, default=6)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--ior", type=float, default=1.0)
    ap.add_argument("--light", type=float, default=1.2)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the algorithmic-byte counting launch")
    return ap.parse_args()


def cpu_baseline(args, seconds: float):
    """Oracle (C++ restatement, same arithmetic) on a bounded sample of the C2 workload:
    every 2nd row of the frame, 1-pass launches of increasing pass number (1..256) until
    the budget is spent (≈10 s on the box's 16 host threads).  Threads = the host share of one GPU on the box (OMP_NUM_THREADS,
    16 there), else nproc."""
    from oracle import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or threads))
    prims, nodes, leaves, depth, _ = orc.scene(args.scene, args.light)
    ipv, iv = orc.camera(args.width, args.height)
    W, H, row_step = args.width, args.height, 2
    rows = len(range(0, H, row_step))
    acc = np.zeros((H, W, 3), np.float32)
    samples, t0, p = 0, time.perf_counter(), 1
    while True:
        orc.render(prims, nodes, leaves, depth, ipv, iv, W, H, p, 1, 0.0, args.bounces, args.ior, 0,
                   row_step=row_step, row_offset=0, n_threads=threads, accum=acc)
        samples += rows * W
        p += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or p > args.spp:
            break
    return {"value": round(samples / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/oracle.cpp, scene {args.scene} {W}x{H} every {row_step}th row ({rows} rows), "
                      f"passes 1..{p - 1} ({samples} samples, {dt:.1f} s), B={args.bounces}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MCPT_DIST_BACKEND") == "gloo":
        local_rank = local_rank % max(torch.cuda.device_count(), 1)   # ranks may share a GPU
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local_rank)
    if world > 1:
        backend = os.environ.get("MCPT_DIST_BACKEND", "nccl")   # "gloo": N>1 rehearsal on one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    W, H, B = args.width, args.height, args.bounces
    S = args.spp * world          # passes per step: per-GPU work = one C2 frame of samples
    scene = mcpt.Scene.reference(args.scene, args.light)
    sr = ShardedRenderer(W, H, args.band_rows, world, rank, local_rank)
    sr.upload_scene(scene)
    ipv, iv = mcpt.camera_canonical(W, H)

    def step(k: int):
        sr.render(ipv, iv, k * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
        return sr.gather()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # AUTO times its candidate schedules (per-lane / wave-coherent walk, two or four pass
    # segments per work item) on the first sizeable launches of a scene: run those before the
    # warm-up so that every warm-up and timed step uses the pick
    for k in range(4):
        sr.render(ipv, iv, 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
    sr.r.clear_accum()
    for k in range(args.warmup):
        step(k)
    barrier()
    trace_ms = []
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
        trace_ms.append(sr.r.last_kernel_ms())   # HIP events of this launch (waits for its stop event)
    barrier()
    elapsed = time.perf_counter() - t0
    stat_dev = sr.device if os.environ.get("MCPT_DIST_BACKEND", "nccl") == "nccl" else torch.device("cpu")
    t = torch.tensor([elapsed], dtype=torch.float64, device=stat_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # exact algorithmic bytes of one launch: the counting build over the first timed pass range
    ev_local = np.zeros(len(mcpt.EVENT_NAMES), np.uint64)
    if not args.no_count:
        ev_local = sr.r.render_counted(ipv, iv, args.warmup * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
    bytes_local = float((ev_local.astype(np.float64) * mcpt.Renderer.event_bytes()).sum())
    avg_trace_ms = float(np.mean([a for a, _ in trace_ms]))
    avg_combine_ms = float(np.mean([b for _, b in trace_ms]))
    stats = torch.tensor([bytes_local, avg_trace_ms, avg_combine_ms, float(ev_local[6])], dtype=torch.float64,
                         device=stat_dev)
    if world > 1:
        allstats = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allstats, stats)
        allstats = torch.stack(allstats).cpu().numpy()
    else:
        allstats = stats.cpu().numpy()[None]

    if rank == 0:
        samples = float(W) * H * S * args.steps
        value = samples / elapsed / 1e6
        # dominant kernel = path-tracing kernel, rank 0's launches (the others are alike)
        achieved = allstats[0, 0] / (allstats[0, 1] / 1e3) / 1e9 if allstats[0, 1] > 0 else 0.0
        bytes_per_sample = allstats[:, 0].sum() / max(allstats[:, 3].sum(), 1.0)
        traffic, valu = None, None
        pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc) and world == 1:
            try:
                with open(pmc) as f:
                    rec = json.load(f)
                if rec.get("workload") == f"scene{args.scene}_{W}x{H}_{S}spp_B{B}":
                    traffic = rec.get("hbm_bytes_per_launch")
                    n_valu = rec.get("counters_per_launch", {}).get("SQ_INSTS_VALU")
                    if n_valu and avg_trace_ms > 0:
                        # VALU issue roofline: wave64 instructions x 64 lanes over this run's
                        # kernel time; peak = 256 CUs x 4 SIMD x 32 lanes/clk x 2.4 GHz
                        ach = n_valu * 64 / (avg_trace_ms / 1e3) / 1e12
                        valu = {"achieved": round(ach, 2), "peak": VALU_PEAK_T, "unit": "T lane-instr/s",
                                "frac": round(ach / VALU_PEAK_T, 4), "instructions_per_launch": n_valu,
                                "source": rec.get("source")}
                        if rec.get("valu_lane_utilisation") is not None:
                            valu["lane_utilisation"] = round(rec["valu_lane_utilisation"], 4)
                        if rec.get("f32_flop_per_launch_upper"):
                            # fp32 ops against the 157.3 TFLOP/s vector peak (upper
                            # bound: counts every lane of an issued instruction)
                            tf = rec["f32_flop_per_launch_upper"] / (avg_trace_ms / 1e3) / 1e12
                            valu["f32_tflops_upper"] = round(tf, 2)
                            valu["f32_peak_tflops"] = 157.3
            except Exception:
                traffic, valu = None, None
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference scene 6 built by the C++ scene producer; deterministic RNG seeds)",
            "config": {
                "workload": f"scene{args.scene}_{W}x{H}_{S}spp_B{B}",
                "scene": args.scene, "width": W, "height": H, "spp_per_step": S,
                "spp_per_gpu_step": args.spp, "bounces": B,
                "ior": args.ior, "light_intensity": args.light, "variant": "montecarlo.frag",
                "parallelism": f"balanced row shards ({args.band_rows}-row bands) x{world} + RCCL gather" if world > 1
                               else "single GPU",
            },
            "kernel_ms": {"trace_avg": round(avg_trace_ms, 3), "combine_avg": round(avg_combine_ms, 3)},
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": allstats[0, 0],
                "algorithmic_bytes_per_sample": round(float(bytes_per_sample), 2),
                "note": ("achieved = the reference's texel-fetch bytes (SURVEY §8d model) / kernel time; "
                         "scene records live in SGPRs/L1/L2 and primary hits are cached per pixel, so "
                         "actual HBM bytes are `traffic` and the kernel is VALU-issue bound: see `valu`"),
                "valu": valu,
            },
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    sr.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
