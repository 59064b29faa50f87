#!/usr/bin/env python3
"""bench.py — north-star benchmark of the MI355X path tracer.

Workload (BASELINE.json configs[1], "C2", the default): scene 6 (scene_4boules), 1920×1080,
256 spp per step, 8 bounces, IOR 1.0, light intensity 1.2, date 0, canonical camera, variant
montecarlo.frag.  A *step* = one full C2 frame: passes [k·256+1, (k+1)·256] accumulated
into the device framebuffer, then the frame gathered to rank 0 (RCCL gather for N>1).
Scene buffers and the framebuffer are resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W] [--config c1|c2|c3|c4|c5|mesh] [--rough R]
                    [--scaling weak|strong] [--deadline S]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Launch: with ``--gpus N > 1`` and no launcher (``WORLD_SIZE`` unset) the process starts N
child ranks itself (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, rendezvous
on 127.0.0.1) before touching the GPU, waits for them, and prints rank 0's line after checking
that it reports N GPUs; a failed rank stops the others and the run exits non-zero with no
line.  A rank whose world size differs from ``--gpus``, or that sees fewer GPUs than ranks
(RCCL), exits non-zero before rendering.  ``MCPT_DIST_BACKEND=gloo`` rehearses the N>1 path
with ranks sharing the visible GPUs (host-staged gloo gather; the line says so).

Configs (BASELINE.json ``configs``):
* c2 (configs[1], default) — strong scaling (round 6; verdict r05 #4): a step renders ONE fixed
  1080p × 256-spp frame; at N GPUs the frame's rows are split into balanced row shards across
  ranks (mcpt_balanced_rows: rotated 8-row bands, H/N rows each, all 256 passes), then one RCCL
  gather of the fp32 RGB shards to rank 0 inside the timed region, so launch, AUTO-trial, gather
  and tail overheads count against the N-GPU figure.  ``--scaling weak`` keeps one C2 frame's
  worth of samples per GPU instead (256·N passes per step, progressive accumulation).
  Bit-identical to rendering the same passes on one GPU; rank 0 checks that after the timed
  region (`self_check`: rows owned by every rank of the gathered frame against a single-rank
  render of those rows).
* c3 (configs[2]) — scene 6, 1080p, 1024 spp per step, B 8, IOR 1.5, roughness sweep: the
  roughness (material .y) of every non-emissive primitive set to each of 0, 0.5, 0.9, 0.99, 1
  (SURVEY §8d), one measurement per point (``--rough R`` runs one point); `value` = the
  sweep's samples ÷ its timed seconds, each point listed under ``config.roughness_points``.  Strong
  scaling like c2 (``--scaling weak``: 1024·N passes per step).
* c4 (configs[3]) — scene 8, 1080p, 512 spp, B 12, the same frame split over N ranks: strong.
* c5 (configs[4]) — scene 6, 3840×2160, B 8, progressive accumulation toward 84,000 spp: a
  step = 1,024 passes (a bounded slice of the target), the 4K frame split over N ranks
  (strong); ``config.time_to_target_s`` extrapolates the measured rate to 84,000 spp (labelled
  as an extrapolation, not a measured run of the whole target).
* c1 (configs[0], the reference's CPU case) — scene 1, 256², 4 spp, B 3: launch-bound on the
  GPU; its `cpu_baseline` times the whole config.
* mesh (round 5; SURVEY §8 (f)2, the triangle-mesh row) — two instances of one 1 M-triangle UV
  sphere (mesh BVH depth 20, 128 MB of mesh records: mcpt.meshes.big_mesh_scene), a ground
  cube, a glass sphere and a light quad; 1080p, 64 spp, B 8, strong.  Its walk is a chain of
  dependent mesh-record fetches from the Infinity Cache / HBM, so its `roofline.bound` is
  "hbm": `achieved` = the §8d algorithmic bytes (counting build of the same kernel) ÷ the
  launch time, `traffic` = the PMC fabric bytes, `traffic_ratio` = traffic ÷ algorithmic, the
  VALU figures under `roofline.valu`.
* mesh_big (round 6; verdict r05 #2) — the mesh workload past the 256 MiB Infinity Cache: four
  distinct ~1 M-triangle meshes (two UV spheres, two tori), one instance each
  (mcpt.meshes.big_mesh4_scene), 1080p, 64 spp, B 8, strong; roofline as for mesh.
``--scaling weak`` runs c2 / c3 with one frame's worth of samples per GPU; the line's `scaling`
says which.  ``--deadline S`` bounds every rank's wall time (and the launcher's, + 15 s; default
600 s + 30 s per step and roughness point, <= 0 no limit): a rank past it prints its current
phase (``PHASES``) and exits 124, and the launcher names the least advanced rank and its phase.

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
* `cpu_baseline` (the C++ oracle on a bounded row/pass sample of the same workload; threads
  used, the host's CPU count and CPU model stated).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import signal
import socket
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (loads the HIP runtime library; no HIP call until a rank runs)
import torch.distributed as dist  # noqa: E402

import mcpt  # noqa: E402  (libmcpt.so is loaded lazily, on the first call)
from mcpt.dist import ShardedRenderer, local_rows  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_T = 78.64     # 256 CUs x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz (a wave64 VALU op = 2 clk)
# fabric requests per second that lanes running dependent chains of random 64-B record reads (the
# mesh walk's access pattern, without its arithmetic) sustain at 5 waves per SIMD, by working set
# (tools/microbench/gather_ceiling.hip, profiles/r06_gather_ceiling.json: one 128-B request per
# record; 128 MB: 3.53 / 3.66 TB/s of records in two sessions, 640 MB: 3.59 TB/s)
GATHER_CEILING_REQ_S = {"mesh1000k": 56.2e9, "mesh4x1000k": 56.1e9}
METRIC = "Msamples/s (W×H×spp/s) + achieved HBM GB/s, 1080p scene6, 1/2/4/8 GPU"
PMC_RECORDS = os.path.join(REPO, "profiles", "pmc_records.json")
C3_ROUGHNESS = (0.0, 0.5, 0.9, 0.99, 1.0)
C5_TARGET_SPP = 84000

CONFIGS = {   # BASELINE.json configs[0..4]
    "c1": dict(scene=1, width=256, height=256, spp=4, bounces=3, ior=1.0, scaling="weak"),
    "c2": dict(scene=6, width=1920, height=1080, spp=256, bounces=8, ior=1.0, scaling="strong"),
    "c3": dict(scene=6, width=1920, height=1080, spp=1024, bounces=8, ior=1.5, scaling="strong",
               rough_sweep=C3_ROUGHNESS),
    "c4": dict(scene=8, width=1920, height=1080, spp=512, bounces=12, ior=1.0, scaling="strong"),
    "c5": dict(scene=6, width=3840, height=2160, spp=1024, bounces=8, ior=1.0, scaling="strong",
               target_spp=C5_TARGET_SPP),
    # the HBM-roofline workload (verdict r04 #1; SURVEY §8f row 2, "the only route to HBM-sized
    # scenes"): two instances of a 1 M-triangle UV sphere (mesh BVH depth 20, 2^21 - 1 mesh nodes,
    # ~130 MB of device mesh records), 1080p, B 8 (mcpt.meshes.big_mesh_scene)
    "mesh": dict(scene="mesh", width=1920, height=1080, spp=64, bounces=8, ior=1.0, scaling="strong",
                 mesh_tris=1_000_000),
    # past the 256 MiB Infinity Cache (verdict r05 #2): four distinct ~1 M-triangle meshes, one
    # instance each (mcpt.meshes.big_mesh4_scene), 1080p, 64 spp, B 8
    "mesh_big": dict(scene="mesh4", width=1920, height=1080, spp=64, bounces=8, ior=1.0, scaling="strong",
                     mesh_tris=1_000_000),
}
# the phases a rank stamps on stderr, in order (the launcher names the rank that stalls, and where)
PHASES = ("start", "init", "upload", "auto", "warmup", "timed", "stats", "count", "self_check", "cpu_baseline",
          "done")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--rough", type=float, default=None, help="c3: one roughness point instead of the sweep")
    ap.add_argument("--light", type=float, default=1.2)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the reference-byte counting launch")
    ap.add_argument("--no-check", action="store_true", help="skip rank 0's post-run self check")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="c2/c3: strong (default: one fixed frame split over the N GPUs) or weak (one C2 frame "
                         "of samples per GPU)")
    ap.add_argument("--deadline", type=float, default=None,
                    help="wall-clock limit (s) of every rank (and of the launcher, +15 s): a rank past it names "
                         "its phase on stderr and exits 124.  Default: 600 s + 30 s per warm-up or timed step "
                         "and roughness point; <= 0: no limit")
    ap.add_argument("--drill-stall", default=None, metavar="RANK:PHASE[:SECONDS]",
                    help="launcher drill (CPU only, MCPT_DIST_BACKEND=gloo): the ranks walk the phases with "
                         "gloo barriers and no GPU work; RANK sleeps SECONDS (default 3600) before PHASE")
    a = ap.parse_args(argv)
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.deadline is None:
        n_pts = 1 if a.config != "c3" or a.rough is not None else len(C3_ROUGHNESS)
        a.deadline = 600.0 + 30.0 * (a.steps + a.warmup) * n_pts
    elif a.deadline <= 0:
        a.deadline = None   # no limit
    scaling = a.scaling
    for k, v in CONFIGS[a.config].items():
        setattr(a, k, v)
    if scaling is not None:
        if a.config not in ("c2", "c3"):
            ap.error("--scaling applies to --config c2 / c3 (c1 is weak, c4 / c5 / mesh are strong)")
        a.scaling = scaling
    if not hasattr(a, "mesh_tris"):
        a.mesh_tris = 0
    if a.drill_stall is not None:
        parts = a.drill_stall.split(":")
        if len(parts) not in (2, 3) or parts[1] not in PHASES:
            ap.error(f"--drill-stall RANK:PHASE[:SECONDS], PHASE one of {PHASES}")
        a.drill_stall = (int(parts[0]), parts[1], float(parts[2]) if len(parts) == 3 else 3600.0)
    if not hasattr(a, "target_spp"):
        a.target_spp = None
    if a.config == "c3":
        a.rough_points = (a.rough,) if a.rough is not None else tuple(a.rough_sweep)
    else:
        if a.rough is not None:
            ap.error("--rough applies to --config c3 only")
        a.rough_points = (None,)
    return a


# ------------------------------------------------------------------------------------------
# launcher: `python bench.py --gpus N` without torchrun starts its own N ranks
# ------------------------------------------------------------------------------------------
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


PHASE_TAG = "bench-phase"


def stamp(rank: int, phase: str, t0: float) -> None:
    """One phase stamp on stderr: `bench-phase rank=R phase=P t=S` (S = seconds since the rank
    started).  The launcher keeps each rank's last stamp to name the rank and phase that stall."""
    print(f"{PHASE_TAG} rank={rank} phase={phase} t={time.time() - t0:.2f}", file=sys.stderr, flush=True)


def parse_stamp(line: str):
    """(rank, phase) of a phase-stamp line, else None."""
    if not line.startswith(PHASE_TAG):
        return None
    kv = dict(f.split("=", 1) for f in line.split()[1:] if "=" in f)
    try:
        return int(kv["rank"]), kv["phase"]
    except (KeyError, ValueError):
        return None


def stall_report(last: dict, alive: set, world: int) -> str:
    """Which rank stalled in which phase: every rank's last stamp, and the rank(s) least advanced
    in PHASES (a rank blocked in a collective waits for the least advanced one; a rank that
    failed early is the least advanced too)."""
    order = {p: i for i, p in enumerate(PHASES)}
    parts = []
    for r in range(world):
        ph, t = last.get(r, ("(none)", None))
        state = "running" if r in alive else "exited"
        parts.append(f"rank {r} {state}, last phase {ph}" + (f" ({time.time() - t:.1f} s ago)" if t else ""))
    idx = {r: order.get(last.get(r, ("", 0))[0], -1) for r in range(world)}
    lo = min(idx.values())
    slow = [r for r in range(world) if idx[r] == lo]
    nxt = PHASES[lo + 1] if lo + 1 < len(PHASES) else "-"
    return ("; ".join(parts) + f". Stalled: rank(s) {', '.join(map(str, slow))} in phase "
            f"{PHASES[lo] if lo >= 0 else '(no stamp yet)'} (next: {nxt})")


def spawn_ranks(cmd, world: int, base_env=None, poll_s: float = 0.2, grace_s: float = 10.0,
                deadline_s: float = None):
    """Run `cmd` as `world` child processes (rank r gets RANK/LOCAL_RANK = r, WORLD_SIZE = world,
    MASTER_ADDR 127.0.0.1 and a free port).  Rank 0's stdout is captured; the others' stdout
    passes through; every rank's stderr is relayed line by line, and its phase stamps kept.
    As soon as one rank exits non-zero the others are stopped (SIGTERM, then SIGKILL after
    `grace_s`), since they would block in a collective; so are all of them once `deadline_s`
    passes (status 124).  Either way the stderr report names each rank's last phase and the
    rank that stalled.  Returns (exit status: 0, the first failing rank's non-zero status or 124;
    rank 0's stdout)."""
    base = dict(os.environ if base_env is None else base_env)
    port = free_port()
    procs, out0, readers = [], [], []
    last = {}   # rank -> (phase, time of its stamp)
    lock = threading.Lock()

    def relay(r, pipe):
        for ln in pipe:
            st = parse_stamp(ln)
            if st is not None:
                with lock:
                    last[st[0]] = (st[1], time.time())
            sys.stderr.write(ln)
            sys.stderr.flush()

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        t_end = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def on_term(signum, _frame):   # the parent being stopped stops its ranks too
        stop_all()
        sys.exit(128 + signum)

    old = signal.signal(signal.SIGTERM, on_term) if threading.current_thread() is threading.main_thread() else None
    t_start = time.time()
    try:
        for r in range(world):
            procs.append(subprocess.Popen(cmd, env=rank_env(base, r, world, port),
                                          stdout=subprocess.PIPE if r == 0 else None,
                                          stderr=subprocess.PIPE, text=True))
            th = threading.Thread(target=relay, args=(r, procs[-1].stderr), daemon=True)
            th.start()
            readers.append(th)
        reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
        reader.start()
        status, why = 0, None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                status, why = bad[0][1], f"rank {bad[0][0]} exited with status {bad[0][1]}"
                break
            if all(c == 0 for c in codes):
                break
            if deadline_s is not None and time.time() - t_start > deadline_s:
                status, why = 124, f"deadline of {deadline_s:g} s passed"
                break
            time.sleep(poll_s)
        if status:
            alive = {r for r, p in enumerate(procs) if p.poll() is None}
            with lock:
                rep = stall_report(last, alive, world)
            print(f"bench: {why}: {rep}", file=sys.stderr, flush=True)
            stop_all()
        reader.join(timeout=grace_s)
        for th in readers:
            th.join(timeout=grace_s)
    finally:
        if old is not None:
            signal.signal(signal.SIGTERM, old)
    return status, (out0[0] if out0 else "")


def rank0_line(stdout: str, world: int):
    """Rank 0's JSON line if it reports `world` GPUs, else None."""
    for ln in reversed(stdout.strip().splitlines()):
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                d = json.loads(ln)
            except ValueError:
                return None
            return ln if d.get("n_gpus") == world else None
    return None


def launch(args) -> int:
    """Parent of a plain `python bench.py --gpus N` (N > 1).  No HIP call happens here: the
    children are fresh processes, and this process only waits and relays rank 0's line."""
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench: starting {args.gpus} ranks (one process per GPU)", file=sys.stderr, flush=True)
    # the ranks stop themselves at --deadline (naming their phase); the launcher's own limit is a
    # little later, for a rank that cannot
    status, out = spawn_ranks(cmd, args.gpus, deadline_s=None if args.deadline is None else args.deadline + 15.0)
    if status:
        print(f"bench: a rank failed (exit {status}); no result", file=sys.stderr, flush=True)
        return status if status > 0 else 1
    line = rank0_line(out, args.gpus)
    if line is None:
        print(f"bench: rank 0 did not report a {args.gpus}-GPU result:\n{out}", file=sys.stderr, flush=True)
        return 1
    print(line, flush=True)
    return 0


def check_world(gpus: int, world: int, backend: str, n_devices: int, local_world: int):
    """Why this rank must not run (str), or None.  Every rank of an N-GPU run must see the
    --gpus N it was asked for, and with RCCL one GPU of its own."""
    if world != gpus:
        return f"--gpus {gpus} but {world} rank(s) joined (WORLD_SIZE)"
    if backend == "nccl" and n_devices < local_world:
        return f"{local_world} ranks on this node but only {n_devices} visible GPU(s)"
    if n_devices < 1:
        return "no visible GPU"
    return None


# ------------------------------------------------------------------------------------------
# workload
# ------------------------------------------------------------------------------------------
def workload_key(args, passes_per_step: int, rough=None) -> str:
    scene = (f"mesh{args.mesh_tris // 1000}k" if args.scene == "mesh" else
             f"mesh4x{args.mesh_tris // 1000}k" if args.scene == "mesh4" else f"scene{args.scene}")
    k = f"{scene}_{args.width}x{args.height}_{passes_per_step}spp_B{args.bounces}"
    if getattr(args, "ior", 1.0) != 1.0:
        k += f"_ior{args.ior:g}"
    if rough is not None:
        k += f"_rough{rough:g}"
    return k


def build_scene(args, rough=None) -> "mcpt.Scene":
    """The reference scene (or the HBM-sized mesh scene); for a C3 point, every non-emissive
    primitive's roughness = rough."""
    if args.scene == "mesh":
        from mcpt import meshes
        return meshes.big_mesh_scene(args.mesh_tris)[0]
    if args.scene == "mesh4":
        from mcpt import meshes
        return meshes.big_mesh4_scene(args.mesh_tris)[0]
    sc = mcpt.Scene.reference(args.scene, args.light)
    if rough is not None:
        prims, _, _ = sc.buffers()
        for i in range(sc.nb_prim()):
            rec = prims[i]
            if rec[58] > 0:   # emissive (material .z): untouched
                continue
            sc.set_material(i, np.concatenate([rec[52:56], [rec[56], rough, rec[58]]]).astype(np.float32))
    return sc


def lib_sha256() -> str:
    with open(mcpt.lib_path(), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_record(workload: str, sha: str, sched=None):
    """The PMC record of this workload measured on this exact library build, or None.  A workload
    may hold records of several schedules (AUTO can settle on either of two close candidates):
    with `sched` ({"traversal", "seg_per_item"}) the record of that schedule is preferred."""
    try:
        with open(PMC_RECORDS) as f:
            recs = json.load(f)["records"]
    except (OSError, ValueError, KeyError):
        return None
    mine = [r for r in recs if r.get("workload") == workload and r.get("lib_sha256") == sha]
    if sched is not None:
        want = {"traversal": sched.get("traversal"), "seg_per_item": sched.get("seg_per_item")}
        for rec in mine:
            if rec.get("schedule") == want:
                return rec
    return mine[0] if mine else None


def host_cpu():
    """(logical CPUs of the host, CPU model string)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count() or 1, model


def cpus_available() -> int:
    """CPUs this process may run on (its affinity mask): the host cores the CPU baseline uses."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_quota():
    """CPUs' worth of time the process's cgroup grants (cpu.max quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_threads() -> int:
    """Host cores the process's time is granted on: the CPUs of the affinity mask, capped by
    the cgroup's CPU quota when one is set (on the GPU box 256 CPUs are visible but the quota
    grants 16: 256 workers then share 16 CPUs' time and run slower than 16)."""
    avail, quota = cpus_available(), cpu_quota()
    return max(1, min(avail, math.ceil(quota))) if quota else avail


def cpu_baseline_run(args, seconds: float, rough=None, threads=None, scene=None):
    """Oracle (C++ restatement, same arithmetic) on a bounded sample of the workload: every
    2nd row of the frame (every row for C1), 1-pass launches of increasing pass number
    (1..spp) until the budget is spent, std::thread over rows on `threads` workers."""
    from oracle import oracle as orc
    nproc, model = host_cpu()
    mv = None
    if args.scene in ("mesh", "mesh4"):   # the mesh workloads: buffers from the scene producer, oracle mesh walk
        prims, nodes, leaves = scene.buffers()
        depth = scene.depth()
        mv = orc.MeshView(scene.mesh_buffers())
    else:
        prims, nodes, leaves, depth, _ = orc.scene(args.scene, args.light)
    if rough is not None:   # build_scene's override: material .y of every non-emissive record
        prims = np.array(prims, copy=True)
        prims[~(prims[:, 58] > 0), 57] = rough
    ipv, iv = orc.camera(args.width, args.height)
    W, H = args.width, args.height
    row_step = 1 if W * H <= (1 << 17) else 2
    rows = len(range(0, H, row_step))
    acc = np.zeros((H, W, 3), np.float32)
    samples, t0, p = 0, time.perf_counter(), 1
    while True:
        orc.render(prims, nodes, leaves, depth, ipv, iv, W, H, p, 1, 0.0, args.bounces, args.ior, 0,
                   row_step=row_step, row_offset=0, n_threads=threads, accum=acc, meshes=mv)
        samples += rows * W
        p += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or p > args.spp:
            break
    scene_name = {"mesh": "the mesh workload (mcpt.meshes.big_mesh_scene)",
                  "mesh4": "the four-mesh workload (mcpt.meshes.big_mesh4_scene)"}.get(args.scene, f"scene {args.scene}")
    return {"value": round(samples / dt / 1e6, 4), "threads": threads,
            "sample": f"oracle/oracle.cpp, {scene_name} {W}x{H} "
                      f"{'every row' if row_step == 1 else f'every {row_step}nd row'} ({rows} rows), "
                      f"passes 1..{p - 1} ({samples} samples, {dt:.3g} s), B={args.bounces}, IOR {args.ior:g}"
                      + (f", roughness {rough:g}" if rough is not None else "")
                      + ("" if row_step == 1 and p > args.spp else "; extrapolated rate, not the whole config"),
            "nproc": nproc, "model": model}


def cpu_baseline(args, seconds: float, rough=None, scene=None):
    """The CPU figure of the line: the oracle run with one worker per CPU of the process's
    affinity mask and, when the cgroup's CPU quota grants fewer CPUs' time than that (the GPU
    box: 256 CPUs visible, 16 granted), again with one worker per granted CPU; `value` is the
    faster run and `cores` its thread count, the other run beside it (verdict / advisor r04)."""
    avail, quota = cpus_available(), cpu_quota()
    counts = [avail]
    nq = cpu_threads()
    if nq != avail:
        counts.append(nq)
    share = seconds / len(counts)
    runs = [cpu_baseline_run(args, share, rough, threads=n, scene=scene) for n in counts]
    best = max(runs, key=lambda r: r["value"])
    others = [r for r in runs if r is not best]
    return {"value": best["value"], "unit": "Msamples/s", "cores": best["threads"], "kind": "port",
            "threads_used": best["threads"], "cores_available": avail, "cgroup_cpu_quota": quota,
            "host_logical_cpus": best["nproc"], "cpu_model": best["model"], "sample": best["sample"],
            "other_runs": [{"threads": r["threads"], "value": r["value"], "sample": r["sample"]} for r in others],
            "threads_note": ("std::thread workers over rows. Run with one worker per CPU of the affinity mask "
                             "(os.sched_getaffinity) and, when the cgroup quota (cpu.max quota/period) grants "
                             "fewer CPUs' time, with one per granted CPU; value = the faster run, cores = its "
                             "thread count, the other under other_runs"),
            "algorithm_note": ("Same integrator and arithmetic as the GPU path, with one difference in work: the "
                               "GPU traverses each pixel's camera ray once per 32-pass segment and reuses the primary hit "
                               "(exact: raytracer.vert has no jitter and the walk draws no random number); the CPU "
                               "port, like the reference's shader, re-traverses it every pass")}


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


def roofline(workload: str, sha: str, avg_trace_ms: float, ref_bytes: float, bytes_per_sample: float, world: int,
             launches: int = 1, bound: str = "valu", sched=None):
    """`avg_trace_ms` is one timed call's kernel time, summed over its `launches` sub-launches; a
    PMC record is used only if it sums the same number of launches.
    bound "valu" (the LDS/L2-resident reference scenes): achieved = VALU lane-instructions / s
    from the same-build PMC record, against the issue peak; the HBM side under `hbm`.
    bound "hbm" (the mesh workload, whose records stream from HBM / the Infinity Cache):
    achieved = the SURVEY §8d algorithmic bytes of one launch (counting build) / its time,
    against 8 TB/s; `traffic` = the PMC fabric bytes of one launch, `traffic_ratio` = traffic /
    algorithmic (> 1: re-reads); the VALU side under `valu`."""
    rec = pmc_record(workload, sha, sched) if world == 1 else None
    if rec is not None and int(rec.get("launches_summed", 1)) != int(launches):
        rec = None
    # (a record states the schedule its counter passes ran, tools/pmc_summary.py: used only for the
    # same schedule as this run's timed launches; None there = its passes ran different ones)
    other_sched = False
    if rec is not None and sched is not None and "schedule" in rec:
        mine = {"traversal": sched.get("traversal"), "seg_per_item": sched.get("seg_per_item")}
        if rec["schedule"] != mine:
            rec, other_sched = None, True
    t_s = avg_trace_ms / 1e3
    valu = {"achieved": None, "peak": VALU_PEAK_T, "unit": "T lane-instr/s", "frac": None,
            "lane_utilisation": None, "useful_frac": None}
    hbm = {"achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None}
    traffic = None
    if rec is not None and t_s > 0:
        c = rec["counters_per_launch"]
        ach = c["SQ_INSTS_VALU"] * 64 / t_s / 1e12
        valu.update(achieved=round(ach, 3), frac=round(ach / VALU_PEAK_T, 4), valu_instructions_per_launch=c["SQ_INSTS_VALU"])
        lu = rec.get("valu_lane_utilisation")
        if lu is not None:
            valu.update(lane_utilisation=round(lu, 4), useful_frac=round(ach / VALU_PEAK_T * lu, 4))
        traffic = rec.get("hbm_bytes_per_launch")
        if traffic is not None:
            gbs = traffic / t_s / 1e9
            hbm.update(achieved=round(gbs, 2), frac=round(gbs / HBM_PEAK_GBS, 5))
    pmc = {"workload": workload, "lib_sha256": sha, "matched": rec is not None,
           "schedule": rec.get("schedule") if rec else None,
           "source": rec.get("source") if rec else None,
           "note": None if rec else ("the PMC record of this workload and build was measured under another "
                                     "schedule than this run's: PMC fields left null" if other_sched else
                                     "no rocprofv3 PMC record of this workload for this libmcpt.so "
                                     "build (summing this call's launches) in profiles/pmc_records.json: "
                                     "PMC fields left null"
                                     if world == 1 else "PMC records are single-GPU measurements")}
    refb = {"per_launch": ref_bytes, "per_sample": round(float(bytes_per_sample), 2),
            "rate_GBs": round(ref_bytes / t_s / 1e9, 1) if t_s > 0 else None}
    if bound == "hbm":
        ach = ref_bytes / t_s / 1e9 if t_s > 0 and ref_bytes > 0 else None
        roof = {"bound": "hbm", "achieved": None if ach is None else round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": None if ach is None else round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_ratio": round(traffic / ref_bytes, 3) if traffic and ref_bytes > 0 else None,
                "traffic_GBs": hbm["achieved"], "kernel_ms": round(avg_trace_ms, 3), "launches_per_call": launches,
                "valu": valu, "pmc": pmc}
        refb["note"] = ("SURVEY §8d texel-fetch model (incl. the mesh events), counted exactly by the counting "
                        "build of the same kernel: the algorithmic bytes of `achieved`")
        # which roof binds, from the same-build PMC record (advisor r05): VALU issue against the
        # measured fabric bytes.  The fabric (L2 -> memory side) counters include Infinity-Cache
        # hits (MI355X_MICROARCH.md §HBM; TCC_EA0_RDREQ_DRAM = TCC_EA0_RDREQ on gfx950), so
        # `traffic` is an upper bound on the HBM bytes, never a split of L3 and HBM
        if valu["frac"] is not None and hbm["frac"] is not None:
            roof["traffic_frac"] = hbm["frac"]
            roof["limiter"] = {"valu_issue_frac": valu["frac"], "fabric_frac": hbm["frac"],
                               "bound_by": "valu issue" if valu["frac"] > hbm["frac"] else "memory",
                               "note": ("frac prices the algorithmic bytes against the HBM peak (the north "
                                        "star's roofline); bound_by says which measured rate is closer to its "
                                        "own peak: VALU lane-instructions / 78.64 T, or fabric bytes (L3 + HBM) / 8 TB/s")}
            # the fabric's own ceiling on this access pattern (measured, not a spec figure)
            req = (rec.get("memory") or {}).get("fabric_reads")
            ceil = GATHER_CEILING_REQ_S.get(workload.split("_")[0])
            if req and ceil and t_s > 0:
                roof["limiter"]["fabric_request_ceiling"] = {
                    "walk_requests_per_s": round(req / t_s / 1e9, 2), "ceiling_requests_per_s": round(ceil / 1e9, 2),
                    "unit": "G/s", "frac": round(req / t_s / ceil, 4),
                    "source": "tools/microbench/gather_ceiling.hip (profiles/r06_gather_ceiling.json): dependent "
                              "random 64-B record chains over the same working set, one 128-B fabric request per record"}
    else:
        roof = dict(bound="valu", **{k: valu[k] for k in ("achieved", "peak", "unit", "frac", "lane_utilisation",
                                                           "useful_frac")})
        if "valu_instructions_per_launch" in valu:
            roof["valu_instructions_per_launch"] = valu["valu_instructions_per_launch"]
        roof.update(traffic=traffic, hbm=hbm, kernel_ms=round(avg_trace_ms, 3), launches_per_call=launches, pmc=pmc)
        refb["note"] = ("SURVEY §8d texel-fetch model: the bytes the reference's shader would fetch for the "
                        "same work (event counts of the counting build). Scene records are served from "
                        "LDS/L1/L2 here, so this is NOT HBM traffic and is never divided by the HBM peak")
    if rec is not None and rec.get("wave_cycle_split"):
        roof["wave_cycle_split"] = {k: round(v, 4) for k, v in rec["wave_cycle_split"].items()}
    roof["reference_equivalent_bytes"] = refb
    return roof


def run_point(args, sr, rough, S, world, barrier, stat_dev, wd):
    """Upload the point's scene, AUTO trials, warm-up, K timed steps (render + gather), the
    counting launch and rank 0's self check.  Returns this rank's figures."""
    W, H, B = args.width, args.height, args.bounces
    wd.enter("upload")
    scene = build_scene(args, rough)
    sr.upload_scene(scene)
    ipv, iv = mcpt.camera_canonical(W, H)
    stream = sr.stream   # the renderer's kernels, its D2D copy and the gather run on it
    # AUTO times its candidate schedules (per-lane / wave-coherent walk, two or four pass
    # segments per work item) on the first sizeable launches of a scene: run those before the
    # warm-up so that every warm-up and timed step uses the pick
    wd.enter("auto")
    for _ in range(mcpt.AUTO_TRIALS):
        sr.render(ipv, iv, 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
    sr.r.clear_accum()
    frame = None
    wd.enter("warmup")
    for k in range(args.warmup):
        sr.render(ipv, iv, k * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
        frame = sr.gather()
    barrier()
    wd.enter("timed")
    kernel_ms, gather_ev = [], []
    # the library keeps the HIP events of its last TIMING_RING render calls: the steps are
    # queued back to back and their kernel times read once per half ring (one wait per 32
    # steps) and after the loop, instead of a wait after every step (which exposed the launch
    # latency of short steps: C1's 0.08 ms launches)
    half = mcpt.Renderer.TIMING_RING // 2
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        sr.render(ipv, iv, k * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        frame = sr.gather()
        e1.record(stream)
        gather_ev.append((e0, e1))
        if (k - args.warmup + 1) % half == 0:
            kernel_ms.extend(sr.r.kernel_ms_back(b) + (sr.r.kernel_span_ms_back(b),) for b in reversed(range(half)))
    barrier()
    kernel_ms.extend(sr.r.kernel_ms_back(b) + (sr.r.kernel_span_ms_back(b),) for b in reversed(range(args.steps % half)))
    elapsed = time.perf_counter() - t0
    wd.enter("stats")
    sched = sr.r.schedule()   # what AUTO picked for this rank's timed launches
    launches = sr.r.last_launch_count()   # sub-launches of one timed call (segment-sum budget)
    t = torch.tensor([elapsed], dtype=torch.float64, device=stat_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    gather_ms = float(np.mean([a.elapsed_time(b) for a, b in gather_ev]))

    # reference-equivalent bytes of one launch: the counting build over the first timed pass range
    ev_local = np.zeros(len(mcpt.EVENT_NAMES), np.uint64)
    wd.enter("count")
    if not args.no_count:
        ev_local = sr.r.render_counted(ipv, iv, args.warmup * S + 1, S, 0.0, B, args.ior, mcpt.MONTECARLO)
    bytes_local = float((ev_local.astype(np.float64) * mcpt.Renderer.event_bytes()).sum())
    avg_trace_ms = float(np.mean([a for a, _, _ in kernel_ms]))
    avg_combine_ms = float(np.mean([b for _, b, _ in kernel_ms]))
    avg_span_ms = float(np.mean([c for _, _, c in kernel_ms]))
    props = torch.cuda.get_device_properties(sr.device)
    stats = torch.tensor([bytes_local, avg_trace_ms, avg_combine_ms, float(ev_local[6]), gather_ms,
                          float(sr.g.n_local), float(props.pci_domain_id), float(props.pci_bus_id),
                          float(props.pci_device_id), float(sr.device.index)], dtype=torch.float64, device=stat_dev)
    if world > 1:
        allstats = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allstats, stats)
        allstats = torch.stack(allstats).cpu().numpy()
    else:
        allstats = stats.cpu().numpy()[None]
    check = None
    wd.enter("self_check")
    if args.rank == 0 and not args.no_check:
        check = self_check(args, scene, ipv, iv, frame, args.warmup + args.steps, S, args.local_rank)
    return dict(rough=rough, elapsed=elapsed, sched=sched, launches=launches, gather_ms=gather_ms, avg_trace_ms=avg_trace_ms,
                avg_span_ms=avg_span_ms,
                avg_combine_ms=avg_combine_ms, allstats=allstats, check=check, scene=scene,
                events={n: int(v) for n, v in zip(mcpt.EVENT_NAMES, ev_local)})


class Watchdog:
    """A rank's phase stamps and its own deadline: past `deadline_s` the rank prints the phase it
    is in (and since when) to stderr and exits 124 — also when a launcher other than ours
    (torch.distributed.run) started it, which then stops the other ranks."""

    def __init__(self, rank: int, deadline_s: float):
        self.rank, self.deadline = rank, deadline_s
        self.t0 = time.time()
        self.phase, self.t_phase = "start", self.t0
        stamp(rank, "start", self.t0)
        if deadline_s is not None:   # (None: --deadline <= 0, no limit)
            threading.Thread(target=self._run, daemon=True).start()

    def enter(self, phase: str) -> None:
        self.phase, self.t_phase = phase, time.time()
        stamp(self.rank, phase, self.t0)

    def _run(self) -> None:
        while True:
            left = self.t0 + self.deadline - time.time()
            if left <= 0:
                break
            time.sleep(min(left, 1.0))
        if self.phase == "done":
            return
        print(f"bench rank {self.rank}: deadline {self.deadline:g} s reached in phase {self.phase} (entered "
              f"{time.time() - self.t_phase:.1f} s ago, t={time.time() - self.t0:.1f} s); exiting",
              file=sys.stderr, flush=True)
        os._exit(124)


def init_group(backend: str, local_rank: int, deadline_s: float) -> None:
    """The process group, with a timeout bounded by the deadline (RCCL init and collectives
    fail instead of hanging; gloo likewise)."""
    import datetime
    to = datetime.timedelta(seconds=300.0 if deadline_s is None else max(10.0, min(300.0, deadline_s)))
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=to)
    else:
        dist.init_process_group(backend, timeout=to)


def drill(args, world: int, rank: int, wd: Watchdog) -> None:
    """`--drill-stall`: the launcher's deadline and stall report on CPU.  The ranks walk PHASES
    with a gloo barrier per phase and no GPU work; rank R sleeps before phase P."""
    stall_rank, stall_phase, stall_s = args.drill_stall
    for ph in PHASES[1:-1]:
        if rank == stall_rank and ph == stall_phase:
            time.sleep(stall_s)
        wd.enter(ph)
        if ph == "init":
            init_group("gloo", 0, args.deadline)
        elif world > 1 and ph not in ("cpu_baseline",):
            dist.barrier()
    wd.enter("done")
    if rank == 0:
        print(json.dumps({"metric": "drill", "n_gpus": world, "drill": True, "phases": list(PHASES),
                          "config": args.config, "scaling": args.scaling}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))   # this process never touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    backend = os.environ.get("MCPT_DIST_BACKEND", "nccl")   # "gloo": N>1 rehearsal sharing GPUs
    wd = Watchdog(rank, args.deadline)
    if args.drill_stall is not None:
        if backend != "gloo":
            print("bench: --drill-stall needs MCPT_DIST_BACKEND=gloo", file=sys.stderr, flush=True)
            sys.exit(2)
        drill(args, world, rank, wd)
        return
    n_dev = torch.cuda.device_count()
    why = check_world(args.gpus, world, backend, n_dev, local_world)
    if why:
        print(f"bench rank {rank}: {why}; not running", file=sys.stderr, flush=True)
        sys.exit(3)
    shared = backend != "nccl" and n_dev < local_world
    if backend != "nccl":
        local_rank = local_rank % n_dev   # ranks may share a GPU
    args.world, args.rank, args.local_rank = world, rank, local_rank
    torch.cuda.set_device(local_rank)
    wd.enter("init")
    if world > 1:
        init_group(backend, local_rank, args.deadline)
        if dist.get_world_size() != args.gpus:
            print(f"bench rank {rank}: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}",
                  file=sys.stderr, flush=True)
            sys.exit(3)

    W, H, B = args.width, args.height, args.bounces
    # passes per step: strong (the default: one frame in total, split over the ranks) or weak
    # (--scaling weak, c2 / c3; c1) = one frame of samples per GPU
    S = args.spp * world if args.scaling == "weak" else args.spp
    sr = ShardedRenderer(W, H, args.band_rows, world, rank, local_rank)
    stat_dev = sr.device if backend == "nccl" else torch.device("cpu")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    points = [run_point(args, sr, rough, S, world, barrier, stat_dev, wd) for rough in args.rough_points]

    if rank == 0:
        sha = lib_sha256()
        samples_per_step = float(W) * H * S
        total_s = sum(pt["elapsed"] for pt in points)
        n_steps = args.steps * len(points)
        value = samples_per_step * n_steps / total_s / 1e6
        main_pt = max(points, key=lambda pt: pt["avg_trace_ms"])   # the dominant kernel
        for pt in points:
            a = pt["allstats"]
            pt["roof"] = roofline(workload_key(args, S, pt["rough"]), sha, pt["avg_trace_ms"], float(a[0, 0]),
                                  float(a[:, 0].sum() / max(a[:, 3].sum(), 1.0)), world, pt["launches"],
                                  bound="hbm" if args.scene in ("mesh", "mesh4") else "valu", sched=pt["sched"])
        config = {
            "workload": workload_key(args, S, main_pt["rough"] if len(points) == 1 else None)
                        + ("_rough-sweep" if len(points) > 1 else ""),
            "baseline_config": args.config.upper(),
            "scene": args.scene, "width": W, "height": H, "spp_per_step": S,
            "spp_per_gpu_step": S // world if args.scaling == "weak" else S, "bounces": B,
            "ior": args.ior, "light_intensity": args.light, "variant": "montecarlo.frag",
            "parallelism": (f"balanced row shards ({args.band_rows}-row bands) x{world} + "
                            f"{'RCCL' if backend == 'nccl' else backend} gather") if world > 1 else "single GPU",
        }
        if world > 1:
            config["backend"] = backend
            if shared:
                config["rehearsal"] = f"{world} ranks sharing {n_dev} GPU(s): checks the N>1 code path, not scaling"
        if args.config == "c3":
            config["roughness_points"] = [
                {"roughness": pt["rough"], "value": round(samples_per_step * args.steps / pt["elapsed"] / 1e6, 2),
                 "ms_per_step": round(pt["elapsed"] / args.steps * 1e3, 3),
                 "kernel_ms": round(pt["avg_trace_ms"], 3), "schedule_rank0": pt["sched"],
                 "roofline_frac": pt["roof"]["frac"], "self_check": pt["check"]} for pt in points]
        if args.target_spp:
            t_step = total_s / n_steps
            config["target_spp"] = args.target_spp
            config["time_to_target_s"] = round(args.target_spp / S * t_step, 3)
            config["time_to_target_note"] = (f"extrapolated: {args.target_spp} spp / {S} spp per step x the measured "
                                             f"{t_step * 1e3:.1f} ms per step (render + gather); not a measured run "
                                             "of the whole target")
        a = main_pt["allstats"]
        if not args.no_count:   # the counting launch's events on rank 0 (its rows; all rows at N = 1)
            main_pt["roof"]["reference_equivalent_bytes"]["events_rank0"] = main_pt["events"]
        checks = [pt["check"] for pt in points if pt["check"] is not None]
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(total_s / n_steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (reference scene {args.scene} built by the C++ scene producer; "
                    "deterministic RNG seeds)",
            "config": config,
            "kernel_ms": {"trace_avg": round(main_pt["avg_trace_ms"], 3),
                          # render lanes: consecutive launches overlap; trace_avg is
                          # each launch's period (previous render end -> its end, what the roofline
                          # divides by), span_avg its own start -> end (what a profiler's kernel
                          # duration shows, the overlapped tails counted twice)
                          "span_avg": round(main_pt["avg_span_ms"], 3),
                          "combine_avg": round(main_pt["avg_combine_ms"], 3),
                          "gather_avg": round(main_pt["gather_ms"], 3),
                          "per_rank_trace_avg": [round(float(x), 3) for x in a[:, 1]],
                          "per_rank_rows": [int(x) for x in a[:, 5]],
                          "schedule_rank0": main_pt["sched"]},
            # which physical GPU each rank rendered on (PCI domain:bus:device, from torch's device
            # properties) and the process group's size: an N-GPU line names N devices
            "devices": {"world_size": dist.get_world_size() if dist.is_initialized() else 1,
                        "per_rank_pci": [f"{int(x[6]):04x}:{int(x[7]):02x}:{int(x[8]):02x}" for x in a],
                        "per_rank_device_index": [int(x[9]) for x in a],
                        "distinct_devices": len({(int(x[6]), int(x[7]), int(x[8])) for x in a})},
            "roofline": main_pt["roof"],
            "self_check": (None if not checks else
                           {"rows": checks[0]["rows"], "passes": checks[0]["passes"],
                            "bit_equal": all(c["bit_equal"] for c in checks),
                            "channels_differing": sum(c["channels_differing"] for c in checks),
                            "points": len(checks)}),
        }
        if not args.no_cpu_baseline and world == 1:
            wd.enter("cpu_baseline")
            out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds, main_pt["rough"], scene=main_pt["scene"])
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    sr.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    wd.enter("done")
    bad = [pt["check"] for pt in points if pt["check"] is not None and not pt["check"]["bit_equal"]]
    if bad:
        sys.exit(f"self check failed: {bad}")


if __name__ == "__main__":
    main()
