"""Loopback transport: W "virtual ranks" of the sharded step in one process,
one engine per rank on the same device, exchanging through device copies.

SURVEY.md §7.3.6: the GPU runner hands out one MI355X per call, so the
multi-GPU step (ShardedEngine / AsyncShardedEngine) is exercised at its real
per-rank shape on ONE GPU: every rank runs in its own host thread, the
all-to-alls become a barrier plus a device copy of each (source, destination)
part on the shared stream.  Everything else -- the owner-partitioned dedup
into W ranges, the counts exchange carried with the values, the owner pull of
every source's keys, the one-launch multi-source apply -- is the code that
runs over RCCL on an 8-GPU node.  Used by tools/w8_emulate.py (per-rank kernel
profile) and the bench-scale W = 8 equivalence test (tests/test_w8_loopback.py).

The bus also records the bytes of every (source, destination) part, i.e. the
per-link traffic the same step would put on the node's xGMI mesh.
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

import torch

from xflow_amd.engine import Engine
from xflow_amd.parallel.sparse_a2a import ShardedEngine


class LoopbackBus:
    """In-process all-to-all between W threads.  Each exchange: every rank
    posts its input and splits, waits for all, copies its parts in source
    order, waits again (inputs stay valid until every rank copied)."""

    def __init__(self, world: int, sync: bool = False):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.posted: List[Optional[tuple]] = [None] * world
        self.sync = sync  # synchronize the device after the copies (separate streams)
        self.link_bytes = [[0] * world for _ in range(world)]  # [src][dst], off-diagonal = links
        self.exchanges = 0

    def a2a(self, rank: int, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits) -> None:
        W = self.world
        unit = inp.element_size() * (inp[0].numel() if inp.dim() > 1 and inp.shape[0] else 1)
        if in_splits is None:
            in_splits = [inp.shape[0] // W] * W
            out_splits = [out.shape[0] // W] * W
        self.posted[rank] = (inp, [int(x) for x in in_splits], unit)
        self.barrier.wait()
        ro = 0
        for src in range(W):
            sinp, ssplits, sunit = self.posted[src]
            so = sum(ssplits[:rank])
            n = int(out_splits[src])
            if n != ssplits[rank]:
                raise RuntimeError(f"loopback: rank {rank} expects {n} rows from {src}, "
                                   f"which sends {ssplits[rank]}")
            if n:
                out[ro:ro + n].copy_(sinp[so:so + n])
                self.link_bytes[src][rank] += n * sunit
            ro += n
        if self.sync:
            torch.cuda.synchronize()
        if rank == 0:
            self.exchanges += 1
        self.barrier.wait()


def loopback_engine(bus: LoopbackBus, rank: int, engine: Engine, cls=ShardedEngine, **kw):
    """A ShardedEngine (or subclass, e.g. AsyncShardedEngine) of virtual rank
    ``rank`` whose exchanges go through ``bus``."""

    class Loopback(cls):
        def _a2a(self, out, inp, out_splits, in_splits):
            if self.drop_exchanges > 0:
                self.drop_exchanges -= 1
                return
            bus.a2a(rank, out, inp, out_splits, in_splits)

    return Loopback(engine, world=bus.world, rank=rank, **kw)


def run_ranks(bus: LoopbackBus, fn: Callable[[int], None]) -> None:
    """Run fn(rank) for every rank of ``bus`` on its own thread; re-raise the
    first failure (after releasing the other ranks from the bus barrier)."""
    errors = []

    def body(r):
        try:
            fn(r)
        except BaseException as e:  # surfaced below
            errors.append(e)
            bus.barrier.abort()

    th = [threading.Thread(target=body, args=(r,), name=f"vrank{r}") for r in range(bus.world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0]
