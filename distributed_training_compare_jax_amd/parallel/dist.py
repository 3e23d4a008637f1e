"""Process bootstrap: one process per GPU over torch.distributed (RCCL on ROCm, gloo on CPU).

The reference is single-controller (one Python process drives every local device,
``main.py:34``); here every rank is its own process and every reference "mesh" op becomes
an explicit collective.  Ranks come from a launcher (``torchrun`` env: RANK, WORLD_SIZE,
LOCAL_RANK, MASTER_ADDR/PORT) or from :func:`spawn` (``main.py`` self-spawns when started
as a plain script, keeping the reference's one-command UX).
"""

from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default), in
# order: two streams on one queue execute as one.  A multi-rank step has more streams than that (the
# step stream, the side stream, every communicator's RCCL stream, gloo's copy streams) and kernels
# that wait on OTHER processes (RCCL's, the P2P all-reduce barrier): a barrier queued ahead of an
# unrelated collective on a shared queue blocks that collective, and across ranks this closes a
# cycle.  Measured: dp2 x tp2 with the P2P all-reduce on one GPU timed out at the default 4 queues
# and passes at 16 (profiles/r3_hw_queues.log).  So every multi-rank GPU process gets >= 16 queues.
MIN_HW_QUEUES = 16


def _ensure_hw_queues():
    cur = os.environ.get("GPU_MAX_HW_QUEUES")
    if cur is not None and cur.isdigit() and int(cur) >= MIN_HW_QUEUES:
        return
    if torch.cuda.is_initialized():
        import warnings

        warnings.warn(f"HIP was initialised before init_distributed: GPU_MAX_HW_QUEUES={cur} stays in effect "
                      f"(multi-rank steps want >= {MIN_HW_QUEUES}; set it in the launcher's environment)")
        return
    os.environ["GPU_MAX_HW_QUEUES"] = str(MIN_HW_QUEUES)


def init_distributed(device: str = "auto", timeout_s: float = 600.0) -> DistInfo:
    """Initialise (or reuse) the default process group from the environment."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1 and device != "cpu":
        _ensure_hw_queues()  # before the first HIP call of this process
    use_cuda = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
    if use_cuda:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local_rank % max(ndev, 1))
        torch.cuda.set_device(dev)
        backend = "nccl"  # = RCCL on ROCm
    else:
        dev = torch.device("cpu")
        backend = "gloo"
    # DTC_DIST_BACKEND=gloo runs several GPU ranks on ONE GPU (RCCL refuses duplicate devices):
    # the 1-GPU test box uses it to exercise the multi-rank GPU code paths (graphs + collectives).
    backend = os.environ.get("DTC_DIST_BACKEND", backend)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return DistInfo(rank, world, local_rank, dev, backend)


def staged_p2p() -> bool:
    """True when point-to-point traffic of GPU tensors must go through host memory (gloo)."""
    return is_dist() and dist.get_backend() == "gloo"


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def destroy():
    if is_dist():
        dist.destroy_process_group()


def _spawn_entry(local_rank: int, world: int, port: int, fn: Callable, args: tuple):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    fn(*args)


def spawn(fn: Callable, world: int, args: tuple = (), port: Optional[int] = None):
    """Run ``fn(*args)`` in ``world`` fresh processes (spawn start method, 127.0.0.1 rendezvous)."""
    import torch.multiprocessing as mp

    port = port or _free_port()
    mp.start_processes(_spawn_entry, args=(world, port, fn, args), nprocs=world, join=True, start_method="spawn")
