"""GPU-only paths: the RCCL sparse all-to-all step (a 1-rank "nccl" process
group exercises the same collectives the 8-GPU run uses), and the trainer on
the bundled data with the HIP backend vs the CPU backend."""
import os

import numpy as np
import pytest
import torch

from conftest import DATA
from dist_utils import free_port
from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig, TrainConfig
from xflow_amd.engine import Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_group(gpu_device):
    import torch.distributed as dist

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0,
                            world_size=1, device_id=gpu_device)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,slices,transport,self_exchange,pipelined",
                         [("lr", 1, "rccl", "alias", False), ("lr", 4, "rccl", "alias", False),
                          ("fm", 2, "rccl", "alias", False), ("lr", 4, "torch", "alias", False),
                          ("lr", 1, "rccl", "comm", True), ("lr", 4, "rccl", "comm", True),
                          ("fm", 1, "rccl", "comm", True), ("mvm", 2, "rccl", "comm", True)])
def test_rccl_sharded_step_equals_fused(gpu_device, nccl_group, kind, slices, transport,
                                        self_exchange, pipelined):
    """self_exchange="comm": every exchange of the 1-rank step really goes
    through RCCL (ncclSend/ncclRecv to self, grouped calls carrying the next
    batch's counts with the values, masks with the gradients) -- the code
    path of the multi-GPU step."""
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    def mk():
        return Engine(ModelConfig(kind=kind, v_dim=8), OptimConfig(),
                      EngineConfig(table_log2_cap=16, max_rows=512, max_nnz=512 * 16,
                                   max_slices=slices), device=gpu_device)

    a, b = mk(), mk()
    sh = ShardedEngine(a, transport=transport, self_exchange=self_exchange)
    assert sh.transport == transport
    keys = []
    data = [random_csr(512, 8, 300, seed=step) for step in range(4)]
    bs = [to_batch(*d, gpu_device, slice_rows=512 // slices) for d in data]
    for step, (k, rp, fg, lab) in enumerate(data):
        keys.append(k)
        nxt = bs[step + 1] if pipelined and step + 1 < len(bs) else None
        assert sh.train_step(bs[step], next_batch=nxt)
        b.train_step(to_batch(k, rp, fg, lab, gpu_device, slice_rows=512 // slices))
    if pipelined:
        assert sh.inline_prepares == 1
    allk = np.unique(np.concatenate(keys))
    np.testing.assert_allclose(a.pull(allk), b.pull(allk), rtol=1e-5, atol=1e-7)
    # sharded eval == fused eval
    k, rp, fg, lab = random_csr(512, 8, 300, seed=77)
    pa = sh.eval_step(to_batch(k, rp, fg, lab, gpu_device))
    pb = b.eval_step(to_batch(k, rp, fg, lab, gpu_device))
    torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-7)
    assert sh.bytes_moved > 0


def test_trainer_gpu_matches_cpu_on_bundled_data(gpu_device, tmp_path):
    from xflow_amd.trainer import Trainer

    preds = []
    for dev in (torch.device("cpu"), gpu_device):
        d = tmp_path / dev.type
        cfg = TrainConfig(train_prefix=os.path.join(DATA, "small_train"),
                          test_prefix=os.path.join(DATA, "small_test"), epochs=5, threads=8,
                          pred_dir=str(d), model=ModelConfig(kind="fm"),
                          engine=EngineConfig(table_log2_cap=14))
        Trainer(cfg, device=dev).train()
        preds.append(np.loadtxt(d / "pred_0_0.txt"))
    np.testing.assert_allclose(preds[0], preds[1], rtol=1e-4, atol=1e-5)


class _LocalBus:
    """In-process all-to-all between threads (one engine per 'rank' on the
    same GPU): every rank posts its input, waits for all, copies its parts."""

    def __init__(self, world):
        import threading

        self.world = world
        self.barrier = threading.Barrier(world)
        self.posted = [None] * world

    def a2a(self, rank, out, inp, out_splits, in_splits):
        W = self.world
        if in_splits is None:
            in_splits = [inp.shape[0] // W] * W
            out_splits = [out.shape[0] // W] * W
        self.posted[rank] = (inp, [int(x) for x in in_splits])
        self.barrier.wait()
        ro = 0
        for src in range(W):
            sinp, ssplits = self.posted[src]
            so = sum(ssplits[:rank])
            n = int(out_splits[src])
            assert n == ssplits[rank]
            if n:
                out[ro:ro + n].copy_(sinp[so:so + n])
            ro += n
        torch.cuda.synchronize()
        self.barrier.wait()  # everyone copied before inputs are reused


def _local_sharded(bus, rank, engine):
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    class LocalSharded(ShardedEngine):
        def _a2a(self, out, inp, out_splits, in_splits):
            bus.a2a(rank, out, inp, out_splits, in_splits)

    return LocalSharded(engine, world=bus.world, rank=rank)


@pytest.mark.parametrize("world,kind,S,pipelined,og",
                         [(2, "lr", 1, False, 0), (3, "lr", 1, False, 1), (2, "fm", 1, False, 0),
                          (8, "lr", 1, True, 0), (8, "lr", 1, True, 1), (8, "lr", 2, True, 0),
                          (4, "fm", 2, True, 0), (4, "fm", 1, True, 1), (4, "mvm", 1, True, 0),
                          (4, "mvm", 1, True, 1), (8, "fm", 1, False, 0)])
def test_owner_partitioned_multirank_on_one_gpu(gpu_device, world, kind, S, pipelined, og):
    """W in-process ranks on one GPU (threads + a local all-to-all) train the
    owner-partitioned sharded step; the union of their shards equals one
    engine trained on the concatenated batches (same check as the gloo
    multi-rank test, here through the HIP partitioned dedup, the owner
    grouping and the one-launch multi-source apply or the per-source applies
    -- og: EngineConfig.owner_group; pipelined: each step prepares the next
    batch into the other worker buffer set)."""
    import threading

    from xflow_amd.testing.hashing import owner_of

    rows, steps = 256, 3

    def mk():
        return Engine(ModelConfig(kind=kind, v_dim=4), OptimConfig(),
                      EngineConfig(table_log2_cap=16, max_rows=world * rows,
                                   max_nnz=world * rows * 16, max_slices=world * S,
                                   owner_group=og),
                      device=gpu_device)

    def data(r, s):
        return random_csr(rows, 6, 120, seed=1000 * s + r)

    bus = _LocalBus(world)
    engines = [mk() for _ in range(world)]
    errors = []

    def run(r):
        try:
            sh = _local_sharded(bus, r, engines[r])
            bs = [to_batch(*data(r, s), gpu_device, slice_rows=rows // S) for s in range(steps)]
            for s in range(steps):
                nxt = bs[s + 1] if pipelined and s + 1 < steps else None
                sh.train_step(bs[s], S=S, next_batch=nxt)
            torch.cuda.synchronize()
        except BaseException as e:  # surfaced below
            errors.append(e)
            bus.barrier.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    ref = mk()
    for s in range(steps):
        parts = [data(r, s) for r in range(world)]
        keys = np.concatenate([p[0] for p in parts])
        lab = np.concatenate([p[3] for p in parts])
        fg = np.concatenate([p[2] for p in parts])
        rp = np.concatenate([parts[0][1]] + [p[1][1:] + sum(len(q[0]) for q in parts[:i + 1])
                                             for i, p in enumerate(parts[1:])])
        ref.train_step(to_batch(keys, rp.astype(np.int32), fg, lab, gpu_device,
                                slice_rows=rows // S))
    allk, allv = [], []
    for r, e in enumerate(engines):
        assert not e.overflowed()
        k, _ = e.export_table()
        assert (owner_of(k, world) == r).all()
        allk.append(k)
        allv.append(e.pull(k))
    k = np.concatenate(allk)
    assert len(np.unique(k)) == len(k) == ref.table_size()
    np.testing.assert_allclose(np.concatenate(allv), ref.pull(k), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("staleness,self_exchange", [(1, "alias"), (1, "comm"), (2, "comm"),
                                                     (3, "alias")])
def test_async_staleness_one_on_gpu_matches_simulation(gpu_device, nccl_group, staleness,
                                                       self_exchange):
    """Config 4 on the HIP backend (1-rank RCCL group): AsyncShardedEngine ==
    the reference step whose pulls miss exactly the previous k steps' pushes.
    Also pins the owner apply's (n, z) stash: the staleness-k step applies a
    buffer after other buffers' pulls and applies, so it must re-read.  With
    self_exchange="comm" the pushes ride in the next step's key exchange
    through RCCL (one communicator, one stream)."""
    from collections import deque

    from xflow_amd.parallel.async_p2p import AsyncShardedEngine
    from xflow_amd.testing import torch_ref
    from xflow_amd.testing.hashing import normal_init

    rows, steps = 64, 6
    eng = Engine(ModelConfig(kind="lr", v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=14, max_rows=rows, max_nnz=rows * 16),
                 device=gpu_device)
    sh = AsyncShardedEngine(eng, staleness=staleness, self_exchange=self_exchange)
    data = [random_csr(rows, 6, 80, seed=1000 * s) for s in range(steps)]
    for k, rp, fg, lab in data:
        sh.train_step(to_batch(k, rp, fg, lab, gpu_device), S=1)
    sh.flush()
    torch.cuda.synchronize()
    assert sh.p2p_ops == steps
    ref = torch_ref.RefTable(1, 1, "ftrl", init_fn=lambda k, d: normal_init(k, d) * 1e-2)
    pending = deque()
    for k, rp, fg, lab in data:
        _, cur = torch_ref.compute_step(ref, "lr", k, lab, rp.astype(np.int32), rows)
        if len(pending) == staleness:
            torch_ref.apply_step(ref, pending.popleft())
        pending.append(cur)
    while pending:
        torch_ref.apply_step(ref, pending.popleft())
    keys, _ = eng.export_table()
    np.testing.assert_allclose(eng.pull(keys), ref.weights(keys, insert=False).numpy(),
                               rtol=1e-4, atol=1e-6)
