"""Multi-GPU rendering: interleaved row-band shards + one gather to rank 0.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm).  Every
pixel×pass is independent and the RNG seed is a pure function of (screen_tc, pass, date),
so splitting the frame by rows is bit-identical to one GPU: each rank renders its rows for
ALL passes, into a compact local accumulator, and rank 0 gathers the shards (one RCCL
gather of fp32 RGB rows, padded to the largest shard) and scatters them back into frame
order.  Partitions: "balanced" (default; mcpt_balanced_rows: 8-row bands dealt with a
per-period rotation, leftover rows dealt singly, row counts equal within one) and "bands"
(``(y // band_rows) % world == rank``, mcpt_set_target).  No collective runs on the
data path of the render itself; the gather is the frame's only exchange step.

The gather/reassembly here is device-agnostic torch code so the N>1 path is covered by
world_size-2 ``gloo`` tests on CPU (tests/test_dist_gloo.py).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist


PARTITIONS = ("balanced", "bands")


def band_owner(H: int, band_rows: int, world: int) -> np.ndarray:
    """Owner rank of every row, interleaved bands: band (y // band_rows) % world — mcpt_set_target."""
    return (np.arange(H) // band_rows) % world


def balanced_owner(H: int, band_rows: int, world: int) -> np.ndarray:
    """Owner rank of every row, balanced partition — mcpt_balanced_rows (include/mcpt.h).

    Whole periods of `world` bands: in period j, rank r takes band j·world + (r + j) % world,
    so every rank holds every band position of a period equally often (no rank always gets
    the top band of each period); the rows after the last whole period are dealt one at a
    time with the same rotation, so row counts differ by at most one.
    """
    y = np.arange(H)
    periods = (H // band_rows) // world
    rest0 = periods * world * band_rows
    b = y // band_rows
    owner = ((b % world) - (b // world) % world) % world
    tail = y >= rest0
    owner[tail] = ((y[tail] - rest0) + periods) % world
    return owner


def local_rows(H: int, band_rows: int, world: int, rank: int, partition: str = "bands") -> np.ndarray:
    """Global row ids (increasing) owned by `rank` under `partition` ("bands": mcpt_set_target,
    "balanced": mcpt_balanced_rows)."""
    if partition not in PARTITIONS:
        raise ValueError(f"partition must be one of {PARTITIONS}")
    owner = (balanced_owner if partition == "balanced" else band_owner)(H, band_rows, world)
    return np.nonzero(owner == rank)[0]


def max_local_rows(H: int, band_rows: int, world: int, partition: str = "bands") -> int:
    return max(len(local_rows(H, band_rows, world, r, partition)) for r in range(world))


def frame_row_index(H: int, band_rows: int, world: int, partition: str = "bands") -> np.ndarray:
    """For the padded gather buffer [world, max_rows, ...]: flat source index of each frame row."""
    m = max_local_rows(H, band_rows, world, partition)
    src = np.empty(H, np.int64)
    for r in range(world):
        rows = local_rows(H, band_rows, world, r, partition)
        src[rows] = r * m + np.arange(len(rows))
    return src


class FrameGather:
    """Pre-allocated buffers + index for gathering row-band shards into a frame on `dst`.

    ``gather(local)``: local is [n_local_rows, W, 3] on this rank's device; returns the
    assembled [H, W, 3] frame on `dst` (None on other ranks).

    At world 1 the send buffer is the frame and no collective runs, unless
    ``force_collective``: then the world-1 gather goes through the process group like any other
    (the test that drives the RCCL branch on a one-GPU box, tests/test_gpu_dist.py).
    """

    def __init__(self, H: int, W: int, band_rows: int, world: int, rank: int, device: torch.device,
                 dst: int = 0, group=None, use_gather: bool = True, partition: str = "bands",
                 force_collective: bool = False):
        self.collective = world > 1 or force_collective
        self.H, self.W, self.band_rows, self.world, self.rank = H, W, band_rows, world, rank
        self.dst, self.group, self.device, self.partition = dst, group, device, partition
        self.m = max_local_rows(H, band_rows, world, partition)
        self.n_local = len(local_rows(H, band_rows, world, rank, partition))
        self.send = torch.zeros((self.m, W, 3), dtype=torch.float32, device=device)
        self.use_gather = use_gather
        if rank == dst or not use_gather:
            self.recv = torch.empty((world * self.m, W, 3), dtype=torch.float32, device=device)
            self.recv_list = list(self.recv.view(world, self.m, W, 3).unbind(0))
        else:
            self.recv, self.recv_list = None, None
        self.index = torch.as_tensor(frame_row_index(H, band_rows, world, partition), device=device)
        self.frame = (torch.empty((H, W, 3), dtype=torch.float32, device=device)
                      if rank == dst and self.collective else None)

    def gather(self, local: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        if local is not None:
            self.send[: self.n_local].copy_(local)
        if not self.collective:
            return self.send
        staged = self.device.type != "cpu" and dist.get_backend(self.group) == "gloo"
        if staged:   # rehearsal of the N>1 path on one GPU (gloo collectives need host tensors)
            send, recv = self.send.cpu(), (self.recv.cpu() if self.recv is not None else None)
            recv_list = list(recv.view(self.world, self.m, self.W, 3).unbind(0)) if recv is not None else None
        else:
            send, recv, recv_list = self.send, self.recv, self.recv_list
        if self.use_gather:
            dist.gather(send, recv_list if self.rank == self.dst else None, dst=self.dst, group=self.group)
        else:
            dist.all_gather_into_tensor(recv, send, group=self.group)
        if self.rank != self.dst:
            return None
        if staged:
            self.recv.copy_(recv)
        torch.index_select(self.recv, 0, self.index, out=self.frame)
        return self.frame


class ShardedRenderer:
    """mcpt.Renderer for this rank's rows + the RCCL gather (GPU path).

    partition "balanced" (default): mcpt_balanced_rows — equal row counts (±1) and rotated
    band positions; "bands": the plain interleaved bands of mcpt_set_target.
    """

    def __init__(self, W: int, H: int, band_rows: int = 8, world: int = 1, rank: int = 0,
                 local_rank: int = 0, group=None, partition: str = "balanced", force_collective: bool = False):
        import mcpt
        self.device = torch.device("cuda", local_rank)
        self.r = mcpt.Renderer(local_rank)
        # The renderer's kernels, the D2D copy into the send buffer and the collective are
        # ordered on ONE stream: a torch stream created here and handed to the library.  (Handing
        # over torch's default stream, handle 0, would leave the library on its own non-blocking
        # stream, and the gather would read the send buffer before the copy landed.)
        # (the greatest priority: with the library's render lanes, the combines and the gather on
        # this stream are dispatched ahead of the next render's waiting workgroups)
        self.stream = torch.cuda.Stream(self.device, priority=torch.cuda.Stream.priority_range()[1])
        self.r.set_stream(self.stream.cuda_stream)
        if partition == "bands":
            self.r.set_target(W, H, band_rows, world, rank)
        else:
            self.r.set_target_rows(W, H, local_rows(H, band_rows, world, rank, partition))
        self.W, self.H, self.band_rows, self.world, self.rank = W, H, band_rows, world, rank
        self.partition = partition
        self.g = FrameGather(H, W, band_rows, world, rank, self.device, group=group, partition=partition,
                             force_collective=force_collective)
        # the gather buffers were allocated (and zero-filled) on the caller's stream
        self.stream.wait_stream(torch.cuda.current_stream(self.device))

    def upload_scene(self, scene) -> None:
        self.r.upload_scene(scene)

    def render(self, invPV, invV, first_pass, n_passes, date=0.0, bounces=3, refract_ind=1.0, variant=0):
        self.r.render(invPV, invV, first_pass, n_passes, date, bounces, refract_ind, variant)

    def gather(self) -> Optional[torch.Tensor]:
        """Copy the local accumulator into the send buffer and gather the frame to rank 0, both
        on `self.stream` after the queued renders; the caller's current stream is then made to
        wait for it, so the returned frame is safe to use there.

        The returned tensor is a buffer this renderer reuses (the frame on rank 0, the send
        buffer at world 1): the next gather overwrites it.  That gather's writes are ordered
        after everything the caller has queued on its current stream by then (the private
        stream waits for it first), so work the caller queued that reads the previous frame
        completes before the buffer changes; keep a copy (``frame.clone()``) to hold a frame
        across gathers."""
        n = self.g.n_local
        caller = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(caller)   # the caller's reads of the previous frame come first
        with torch.cuda.stream(self.stream):
            if n:
                self.r.copy_accum_device(self.g.send.data_ptr(), n * self.W * 3 * 4)
            frame = self.g.gather(None)
        caller.wait_stream(self.stream)
        return frame

    def close(self) -> None:
        self.r.close()
