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
