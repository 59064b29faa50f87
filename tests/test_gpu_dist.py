"""The N>1 path on the GPU: ShardedRenderer ranks (2 and 3 processes sharing cuda:0, gloo
collectives staged through the host — the only N>1 run one GPU allows; RCCL needs a GPU per
rank) render their balanced row shards for several pass ranges back to back with no host
synchronization, gather after each, and rank 0's frame must equal a one-context render of the
same passes bit for bit.  This is the ordering bench.py's timed loop relies on: the library's
kernels, its D2D copy into the send buffer and the collective must share one stream (a round-2
bug: the library ran on its own non-blocking stream and the gather read a stale buffer)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, S, steps, q):
    import sys
    sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mcpt
        from mcpt.dist import ShardedRenderer
        ipv, iv = mcpt.camera_canonical(W, H)
        sc = mcpt.Scene.reference(6)
        sr = ShardedRenderer(W, H, 8, world, rank, 0)
        sr.upload_scene(sc)
        frame = None
        for k in range(steps):   # no host synchronization between steps (as in bench.py)
            sr.render(ipv, iv, k * S + 1, S, 0.0, 8, 1.0, mcpt.MONTECARLO)
            frame = sr.gather()
        if rank == 0:
            got = frame.cpu().numpy()
            ref = mcpt.Renderer(0)
            ref.upload_scene(sc)
            ref.set_target(W, H)
            ref.render(ipv, iv, 1, steps * S, 0.0, 8, 1.0, mcpt.MONTECARLO)
            want, n = ref.read_accum()
            ref.close()
            q.put((int((got.view(np.uint32) != want.view(np.uint32)).sum()), n))
        sr.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_renderer_gather_ordered(world):
    W, H, S, steps = 640, 360, 64, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(world, _free_port(), W, H, S, steps, q), nprocs=world, join=True,
                       start_method="spawn")
    diff, n = q.get(timeout=120)
    assert n == steps * S
    assert diff == 0, f"{diff} channels of the gathered frame differ from the one-context render"


def _nccl_worker(rank, port, W, H, S, steps, q):
    """World 1 over RCCL: init_process_group("nccl", device_id=cuda:0) and FrameGather's
    collective branch (force_collective skips the world-1 shortcut), so the code path the
    driver's 8-GPU run takes executes here: the gathered frame must equal the renderer's own
    accumulator bit for bit."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "montecarlo-pathtracing_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import mcpt
        from mcpt.dist import ShardedRenderer
        ipv, iv = mcpt.camera_canonical(W, H)
        sr = ShardedRenderer(W, H, 8, 1, 0, 0, force_collective=True)
        sr.upload_scene(mcpt.Scene.reference(6))
        frame = None
        for k in range(steps):
            sr.render(ipv, iv, k * S + 1, S, 0.0, 8, 1.0, mcpt.MONTECARLO)
            frame = sr.gather()
        got = frame.cpu().numpy()
        want, n = sr.r.read_accum()
        props = torch.cuda.get_device_properties(0)
        q.put((dist.get_backend(), dist.get_world_size(), frame.data_ptr() != sr.g.send.data_ptr(),
               int((got.view(np.uint32) != want.view(np.uint32)).sum()), n, props.pci_bus_id))
        sr.close()
    finally:
        dist.destroy_process_group()


def test_rccl_gather_world1_collective():
    """The RCCL branch of FrameGather.gather (dist.gather over the nccl backend) and
    init_process_group("nccl", device_id=...) run on the one GPU of the box."""
    W, H, S, steps = 640, 360, 64, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_nccl_worker, args=(_free_port(), W, H, S, steps, q), nprocs=1, join=True,
                       start_method="spawn")
    backend, world, separate, diff, n, bus = q.get(timeout=120)
    assert backend == "nccl" and world == 1
    assert separate, "the frame must come out of the collective, not alias the send buffer"
    assert n == steps * S
    assert diff == 0, f"{diff} channels of the RCCL-gathered frame differ from the accumulator"
