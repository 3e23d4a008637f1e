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


# Why cross-process spin waits cannot deadlock here, whatever GPU_MAX_HW_QUEUES is.
# HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default) in FIFO
# order, so two streams that share a queue execute as one, and a kernel that waits on OTHER processes
# (an RCCL collective, the P2P all-reduce barrier of parallel/p2p.py) blocks everything queued behind
# it.  That is safe as long as every blocking operation is ENQUEUED BY THE MAIN THREAD IN PROGRAM
# ORDER, which is identical on every rank (StepProgram issues graphs and collectives in one fixed
# sequence, and program.check_collective_sequences proves the ranks agree): then the globally
# earliest unfinished blocking operation has, on every participating rank, only finished or
# non-blocking work ahead of it in any queue, so it completes, and by induction every later one does
# -- a cycle would need some rank to have enqueued a later operation ahead of an earlier one.  The
# one way that order broke was gloo on GPU tensors (the one-GPU multi-rank test rig): gloo enqueues
# its device copy-back from a worker thread at an unpredictable time, behind later barriers
# (profiles/r3_hw_queues.log: dp2 x tp2 hung at 4 queues).  StepProgram.sync_comms therefore waits
# every gloo collective on GPU tensors where it is issued (the Engine sets it), and the queue count
# is left at the box default.  The in-launch LayerNorm statistics exchange (ops/ln_fused.py) waits
# only on blocks of its own grid and is enabled for single-rank runs only.
def init_distributed(device: str = "auto", timeout_s: float = 600.0, single_rank_pg: bool = False) -> DistInfo:
    """Initialise (or reuse) the default process group from the environment.

    ``single_rank_pg`` (or ``DTC_WORLD1_PG=1``): create the process group at world size 1 too, so a one-GPU
    run can drive real RCCL communicators (``TrainConfig.dp_comm_rehearsal``: the DP collective sequence
    issued on a one-rank group)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
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
    single_rank_pg = single_rank_pg or os.environ.get("DTC_WORLD1_PG", "0") == "1"
    if (world > 1 or single_rank_pg) and not dist.is_initialized():
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
