#!/usr/bin/env python3
"""bench.py — north-star benchmark of the MI355X path tracer.

Workload (BASELINE.json configs[1], "C2", the default): scene 6 (scene_4boules), 1920×1080,
256 spp per step, 8 bounces, IOR 1.0, light intensity 1.2, date 0, canonical camera, variant
montecarlo.frag.  A *step* = one full C2 frame: passes [k·256+1, (k+1)·256] accumulated
into the device framebuffer, then the frame gathered to rank 0 (RCCL gather for N>1).
Scene buffers and the framebuffer are resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c4]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Multi-GPU, C2: weak scaling — per-GPU work fixed at one C2 frame's worth of samples: at N GPUs
a step accumulates 256·N passes of the 1080p frame (progressive accumulation, as configs
C4/C5 do), the frame split into balanced row shards across ranks (mcpt_balanced_rows:
rotated 8-row bands; each rank H/N rows × 256·N passes = one C2 frame of samples), then one
RCCL gather of the fp32 RGB shards to rank 0 inside the timed region.  Bit-identical to
rendering the same passes on one GPU; rank 0 checks that after the timed region (`self_check`:
rows owned by every rank of the gathered frame against a single-rank render of those rows).
``--config c4`` (BASELINE configs[3]): scene 8, 1080p, 512 spp, B 12, the same frame split
over N ranks — strong scaling.  ``--config c1`` (configs[0], the reference's CPU case): scene 1,
256², 4 spp, B 3 — launch-bound on the GPU; its `cpu_baseline` times the whole config.

Prints ONE JSON line (rank 0) with
* `roofline` for the dominant kernel (the path-tracing kernel).  Its limiter is VALU issue,
  not HBM, so `bound` = "valu": `achieved` = wave64 VALU instructions per
  launch × 64 lanes ÷ the launch's average time from HIP events on its stream, against the
  78.64 T lane-instr/s issue peak (256 CUs × 4 SIMD-32 × 2.4 GHz); `lane_utilisation` = active
  lanes per issued VALU instruction, `useful_frac` = frac × lane_utilisation.  The HBM side is
  `traffic` (PMC FETCH_SIZE×2 + WRITE_SIZE bytes per launch) ÷ the same time against 8 TB/s.
  Instruction and byte counts come from rocprofv3 --pmc passes of the SAME libmcpt.so
  (`profiles/pmc_records.json`, keyed by workload and the library's sha256): with no record
  for this build the PMC-derived fields are null, never stale.  `reference_equivalent_bytes`
  is the SURVEY §8d texel-fetch model of the reference (counted exactly by the counting build
  of the same kernel): reference-equivalent work, not HBM traffic, and never divided by the
  HBM peak.
* `cpu_baseline` (the C++ oracle on a bounded row/pass sample of the same workload, host
  threads stated).
"""
from __future__ import annotations

import argparse
import hashlib
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
from mcpt.dist import ShardedRenderer, local_rows  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_T = 78.64     # 256 CUs x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz (a wave64 VALU op = 2 clk)
METRIC = "Msamples/s (W×H×spp/s) + achieved HBM GB/s, 1080p scene6, 1/2/4/8 GPU"
PMC_RECORDS = os.path.join(REPO, "profiles", "pmc_records.json")

CONFIGS = {   # BASELINE.json configs[0] / configs[1] / configs[3]
    "c1": dict(scene=1, width=256, height=256, spp=4, bounces=3, ior=1.0, scaling="weak"),
    "c2": dict(scene=6, width=1920, height=1080, spp=256, bounces=8, ior=1.0, scaling="weak"),
    "c4": dict(scene=8, width=1920, height=1080, spp=512, bounces=12, ior=1.0, scaling="strong"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--light", type=float, default=1.2)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the reference-byte counting launch")
    ap.add_argument("--no-check", action="store_true", help="skip rank 0's post-run self check")
    a = ap.parse_args()
    for k, v in CONFIGS[a.config].items():
        setattr(a, k, v)
    return a


def workload_key(args, passes_per_step: int) -> str:
    return f"scene{args.scene}_{args.width}x{args.height}_{passes_per_step}spp_B{args.bounces}"


def lib_sha256() -> str:
    with open(mcpt.lib_path(), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_record(workload: str, sha: str):
    """The PMC record of this workload measured on this exact library build, or None."""
    try:
        with open(PMC_RECORDS) as f:
            recs = json.load(f)["records"]
    except (OSError, ValueError, KeyError):
        return None
    for rec in recs:
        if rec.get("workload") == workload and rec.get("lib_sha256") == sha:
            return rec
    return None


def cpu_baseline(args, seconds: float):
    """Oracle (C++ restatement, same arithmetic) on a bounded sample of the workload:
    every 2nd row of the frame, 1-pass launches of increasing pass number (1..spp) until
    the budget is spent (≈10 s on the box's 16 host threads).  Threads = the host share of
    one GPU on the box (OMP_NUM_THREADS, 16 there), else nproc."""
    from oracle import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or threads))
    prims, nodes, leaves, depth, _ = orc.scene(args.scene, args.light)
    ipv, iv = orc.camera(args.width, args.height)
    # C1 (65,536 pixels x 4 passes) is timed whole; larger frames on every 2nd row
    W, H = args.width, args.height
    row_step = 1 if W * H <= (1 << 17) else 2
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
            "sample": f"oracle/oracle.cpp, scene {args.scene} {W}x{H} "
                      f"{'every row' if row_step == 1 else f'every {row_step}nd row'} ({rows} rows), "
                      f"passes 1..{p - 1} ({samples} samples, {dt:.3g} s), B={args.bounces}"}


def check_rows(H: int, band_rows: int, world: int):
    """Rows for rank 0's self check: the first two local rows of every rank's shard (so every
    rank's contribution to the gathered frame is checked) plus the frame's last row."""
    rows = set()
    for r in range(world):
        lr = local_rows(H, band_rows, world, r, "balanced")
        rows.update(int(y) for y in lr[:2])
    rows.add(H - 1)
    return sorted(rows)


def self_check(args, scene, ipv, iv, frame: torch.Tensor, n_calls: int, S: int, device: int):
    """Single-rank render of `check_rows` with the run's own call sequence (passes [k·S+1,
    (k+1)·S] for k < n_calls: a call that splits a 32-pass accumulation chunk adds its own
    partial sum, DESIGN.md §3.3, so C1's 4-pass steps need the same split) against the same
    rows of the gathered frame."""
    rows = check_rows(args.height, args.band_rows, max(args.world, 1))
    r = mcpt.Renderer(device)
    try:
        r.upload_scene(scene)
        r.set_target_rows(args.width, args.height, rows)
        r.set_traversal(mcpt.TRAVERSAL_LANE)   # no AUTO trials on this small target
        for k in range(n_calls):
            r.render(ipv, iv, k * S + 1, S, 0.0, args.bounces, args.ior, mcpt.MONTECARLO)
        ref, n = r.read_accum()
    finally:
        r.close()
    got = frame[torch.as_tensor(rows, device=frame.device)].cpu().numpy()
    diff = int((got.view(np.uint32) != ref.view(np.uint32)).sum())
    return {"rows": len(rows), "passes": int(n), "bit_equal": diff == 0, "channels_differing": diff}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    args.world = world
    if os.environ.get("MCPT_DIST_BACKEND") == "gloo":
        local_rank = local_rank % max(torch.cuda.device_count(), 1)   # ranks may share a GPU
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local_rank)
    backend = os.environ.get("MCPT_DIST_BACKEND", "nccl")   # "gloo": N>1 rehearsal on one GPU
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    W, H, B = args.width, args.height, args.bounces
    # passes per step: weak (C2) = one frame of samples per GPU; strong (C4) = one frame in total
    S = args.spp * world if args.scaling == "weak" else args.spp
    scene = mcpt.Scene.reference(args.scene, args.light)
    sr = ShardedRenderer(W, H, args.band_rows, world, rank, local_rank)
    sr.upload_scene(scene)
    ipv, iv = mcpt.camera_canonical(W, H)
    stream = sr.stream   # the renderer's kernels, its D2D copy and the gather run on it

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # AUTO times its candidate schedules (per-lane / wave-coherent walk, two or four pass
    # segments per work item) on the first sizeable launches of a scene: run those before the
    # warm-up so that every warm-up and timed step uses the pick
    for k in range(mcpt.AUTO_TRIALS):
        sr.render(ipv, iv, 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
    sr.r.clear_accum()
    frame = None
    for k in range(args.warmup):
        sr.render(ipv, iv, k * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
        frame = sr.gather()
    barrier()
    kernel_ms, gather_ev = [], []
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        sr.render(ipv, iv, k * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        frame = sr.gather()
        e1.record(stream)
        gather_ev.append((e0, e1))
        kernel_ms.append(sr.r.last_kernel_ms())   # HIP events of this launch (waits for its stop event)
    barrier()
    elapsed = time.perf_counter() - t0
    sched = sr.r.schedule()   # what AUTO picked for this rank's timed launches
    stat_dev = sr.device if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([elapsed], dtype=torch.float64, device=stat_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    gather_ms = float(np.mean([a.elapsed_time(b) for a, b in gather_ev]))

    # reference-equivalent bytes of one launch: the counting build over the first timed pass range
    ev_local = np.zeros(len(mcpt.EVENT_NAMES), np.uint64)
    if not args.no_count:
        ev_local = sr.r.render_counted(ipv, iv, args.warmup * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
    bytes_local = float((ev_local.astype(np.float64) * mcpt.Renderer.event_bytes()).sum())
    avg_trace_ms = float(np.mean([a for a, _ in kernel_ms]))
    avg_combine_ms = float(np.mean([b for _, b in kernel_ms]))
    stats = torch.tensor([bytes_local, avg_trace_ms, avg_combine_ms, float(ev_local[6]), gather_ms,
                          float(sr.g.n_local)], dtype=torch.float64, device=stat_dev)
    if world > 1:
        allstats = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allstats, stats)
        allstats = torch.stack(allstats).cpu().numpy()
    else:
        allstats = stats.cpu().numpy()[None]

    check = None
    if rank == 0 and not args.no_check:
        check = self_check(args, scene, ipv, iv, frame, args.warmup + args.steps, S, local_rank)

    if rank == 0:
        samples = float(W) * H * S * args.steps
        value = samples / elapsed / 1e6
        workload = workload_key(args, S)
        sha = lib_sha256()
        rec = pmc_record(workload, sha) if world == 1 else None
        t_s = avg_trace_ms / 1e3
        ref_bytes = allstats[0, 0]
        bytes_per_sample = allstats[:, 0].sum() / max(allstats[:, 3].sum(), 1.0)
        roof = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_T, "unit": "T lane-instr/s", "frac": None,
                "lane_utilisation": None, "useful_frac": None, "traffic": None,
                "hbm": {"achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None},
                "kernel_ms": round(avg_trace_ms, 3),
                "pmc": {"lib_sha256": sha, "matched": rec is not None,
                        "source": rec.get("source") if rec else None,
                        "note": None if rec else "no rocprofv3 PMC record of this workload for this libmcpt.so "
                                                 "build (profiles/pmc_records.json): PMC fields left null"}}
        if rec is not None and t_s > 0:
            c = rec["counters_per_launch"]
            ach = c["SQ_INSTS_VALU"] * 64 / t_s / 1e12
            roof["achieved"] = round(ach, 3)
            roof["frac"] = round(ach / VALU_PEAK_T, 4)
            lu = rec.get("valu_lane_utilisation")
            if lu is not None:
                roof["lane_utilisation"] = round(lu, 4)
                roof["useful_frac"] = round(ach / VALU_PEAK_T * lu, 4)
            roof["valu_instructions_per_launch"] = c["SQ_INSTS_VALU"]
            traffic = rec.get("hbm_bytes_per_launch")
            roof["traffic"] = traffic
            if traffic is not None:
                gbs = traffic / t_s / 1e9
                roof["hbm"].update(achieved=round(gbs, 2), frac=round(gbs / HBM_PEAK_GBS, 5))
            if rec.get("wave_cycle_split"):
                roof["wave_cycle_split"] = {k: round(v, 4) for k, v in rec["wave_cycle_split"].items()}
        roof["reference_equivalent_bytes"] = {
            "per_launch": ref_bytes, "per_sample": round(float(bytes_per_sample), 2),
            "rate_GBs": round(ref_bytes / t_s / 1e9, 1) if t_s > 0 else None,
            "note": ("SURVEY §8d texel-fetch model: the bytes the reference's shader would fetch for the "
                     "same work (event counts of the counting build). Scene records are served from "
                     "LDS/L1/L2 here, so this is NOT HBM traffic and is never divided by the HBM peak")}
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (reference scene {args.scene} built by the C++ scene producer; "
                    "deterministic RNG seeds)",
            "config": {
                "workload": workload,
                "baseline_config": args.config.upper(),
                "scene": args.scene, "width": W, "height": H, "spp_per_step": S,
                "spp_per_gpu_step": S // world if args.scaling == "weak" else S, "bounces": B,
                "ior": args.ior, "light_intensity": args.light, "variant": "montecarlo.frag",
                "parallelism": f"balanced row shards ({args.band_rows}-row bands) x{world} + RCCL gather"
                               if world > 1 else "single GPU",
            },
            "kernel_ms": {"trace_avg": round(avg_trace_ms, 3), "combine_avg": round(avg_combine_ms, 3),
                          "gather_avg": round(gather_ms, 3),
                          "per_rank_trace_avg": [round(float(x), 3) for x in allstats[:, 1]],
                          "per_rank_rows": [int(x) for x in allstats[:, 5]],
                          "schedule_rank0": sched},
            "roofline": roof,
            "self_check": check,
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
    if check is not None and not check["bit_equal"]:
        sys.exit(f"self check failed: {check}")


if __name__ == "__main__":
    main()
