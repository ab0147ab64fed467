"""Run a function on N gloo CPU ranks (the analogue of the reference's
scripts/local.sh multi-process runs)."""
from __future__ import annotations

import os
import socket

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def run_world(fn, world: int, *args) -> None:
    mp.spawn(_entry, args=(world, free_port(), fn, args), nprocs=world, join=True)


def _entry_gpu(rank, world, port, fn, args):
    """Rank entry of run_world_gpu: every rank on GPU 0, RCCL between the
    processes (xflow_amd.parallel.dist.shared_gpu_setup)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), XFLOW_SHARED_GPU="1")
    import torch
    import torch.distributed as dist

    from xflow_amd.parallel.dist import shared_gpu_setup

    shared_gpu_setup(rank)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        fn(rank, world, *args)
        torch.cuda.synchronize(dev)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def run_world_gpu(fn, world: int, *args) -> None:
    """Run fn on `world` processes that share this box's GPU 0 and talk over
    real RCCL (socket transport between per-rank host ids): the multi-process
    GPU path on a 1-GPU box."""
    mp.spawn(_entry_gpu, args=(world, free_port(), fn, args), nprocs=world, join=True)


def _entry_gpu_gloo(rank, world, port, fn, args):
    """Rank entry of run_world_gpu_gloo: every rank on GPU 0, gloo for the
    process group (the asynchronous parameter server needs no collective
    transport: only its handshake uses the group)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
        torch.cuda.synchronize(dev)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def run_world_gpu_gloo(fn, world: int, *args) -> None:
    mp.spawn(_entry_gpu_gloo, args=(world, free_port(), fn, args), nprocs=world, join=True)
