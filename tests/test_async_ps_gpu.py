"""The asynchronous parameter server on the HIP backend: several processes
share this box's GPU 0 and exchange keys, values and gradient entries through
HIP-IPC windows (fine-grained HBM), no RCCL.  The live tables equal a
one-process GPU replay of the owners' logs bit for bit, for the dense
(one slice) and the CSR (several slices) gradient exchange of every model.
(On an 8-GPU node the same windows are peer HBM over xGMI.)"""
import os

import numpy as np
import pytest
import torch

from dist_utils import run_world_gpu_gloo
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo
from xflow_amd.engine import Engine
from xflow_amd.parallel.async_ps import AsyncParameterServer, replay_logs, worker_config

pytestmark = pytest.mark.gpu
ROWS = 4096


def _cfg(kind, slices, fm_math="reference"):
    model = ModelConfig(kind=kind, v_dim=8, fm_math=fm_math)
    optim = OptimConfig(v_init_scale=1.0 if kind == "mvm" else 1e-2)
    cfg = EngineConfig(table_log2_cap=20, max_rows=ROWS, max_nnz=ROWS * 39, max_slices=slices)
    return model, optim, cfg


def _synth(fields):
    return SynthConfig(seed=11, n_fields=fields, total_features=20_000_000,
                       hash_space=20_000_000)


def _table(eng):
    keys, words = eng.export_table()
    order = np.argsort(keys)
    return keys[order], words.reshape(len(keys), -1)[order]


def _rank(rank, world, kind, fm_math, slices, k, steps, fields, out_dir):
    model, optim, cfg = _cfg(kind, slices, fm_math)
    aps = AsyncParameterServer(model, optim, cfg, torch.device("cuda", 0), staleness=k,
                               slices=slices)
    assert aps.transport.startswith("ipc")
    gen = SyntheticCriteo(aps.worker, ROWS, _synth(fields), rank=rank, slice_rows=ROWS // slices)
    bufs = [gen.alloc_batch() for _ in range(2)]
    for t in range(steps):
        b = bufs[t & 1]
        gen.next(out=b)
        assert aps.train_step(b)
    aps.close()
    keys, words = _table(aps.server)
    st = aps.stats()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), log=aps.log(), keys=keys, words=words,
             csr=st["csr"], max_staleness=st["max_staleness"])


@pytest.mark.parametrize("kind,fm_math,slices,k,fields", [
    ("lr", "reference", 1, 1, 39), ("lr", "reference", 64, 2, 39),
    ("fm", "reference", 16, 1, 39), ("fm", "standard", 8, 0, 39), ("mvm", "reference", 4, 1, 18)])
def test_async_ps_gpu_equals_log_replay(tmp_path, kind, fm_math, slices, k, fields):
    world, steps = 3, 4
    run_world_gpu_gloo(_rank, world, kind, fm_math, slices, k, steps, fields, str(tmp_path))
    dev = torch.device("cuda", 0)
    model, optim, cfg = _cfg(kind, slices, fm_math)
    live = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert bool(live[0]["csr"]) == (slices > 1)
    workers = [Engine(model, optim, worker_config(cfg), dev) for _ in range(world)]
    servers = [Engine(model, optim, cfg, dev) for _ in range(world)]
    batches = []
    for s in range(world):
        gen = SyntheticCriteo(workers[s], ROWS, _synth(fields), rank=s, slice_rows=ROWS // slices)
        batches.append([gen.next(out=gen.alloc_batch()) for _ in range(steps)])
    replay_logs([x["log"] for x in live], batches, workers, servers, k, slices)
    torch.cuda.synchronize(dev)
    for o in range(world):
        assert int(live[o]["max_staleness"]) <= k
        keys, words = _table(servers[o])
        assert np.array_equal(keys, live[o]["keys"]), f"owner {o}: key sets differ"
        assert np.array_equal(words, live[o]["words"]), f"owner {o}: state differs from replay"


def _trainer_rank(rank, world, data_dir, out_dir):
    from xflow_amd.config import TrainConfig
    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=os.path.join(data_dir, "small_train"),
                      test_prefix=os.path.join(data_dir, "small_test"), epochs=3, threads=4,
                      pred_dir=out_dir, async_ps=True, staleness=1,
                      engine=EngineConfig(table_log2_cap=14))
    t = Trainer(cfg, device=torch.device("cuda", 0))
    assert t.aps is not None and t.aps.transport.startswith("ipc")
    res = t.train()
    np.save(os.path.join(out_dir, f"keys{rank}.npy"), np.sort(t.table.export_table()[0]))
    if rank == 0:
        np.save(os.path.join(out_dir, "res.npy"), np.array([res["n"], res["ln_logloss"]]))
    t.close()


def test_async_trainer_two_gpu_processes(tmp_path):
    """The CLI's --async path (Trainer + asynchronous parameter server) on 2
    processes sharing GPU 0: both train their shard without meeting, pause at
    every epoch end, rank 0 predicts over both servers; the two shards hold
    every key a one-process run holds, each exactly once, and the prediction
    file is the reference's 200 lines."""
    from conftest import DATA

    from xflow_amd.config import TrainConfig
    from xflow_amd.trainer import Trainer

    run_world_gpu_gloo(_trainer_rank, 2, DATA, str(tmp_path))
    k = np.concatenate([np.load(tmp_path / f"keys{r}.npy") for r in range(2)])
    one = Trainer(TrainConfig(train_prefix=os.path.join(DATA, "small_train"),
                              test_prefix=os.path.join(DATA, "small_test"), epochs=1,
                              threads=4, write_pred=False, engine=EngineConfig(table_log2_cap=14)),
                  device=torch.device("cpu"))
    one.train()
    ref = np.sort(one.table.export_table()[0])
    one.close()
    assert len(k) == len(np.unique(k)) and np.array_equal(np.sort(k), ref)
    pred = np.loadtxt(tmp_path / "pred_0_0.txt")
    assert pred.shape == (200, 3) and np.all((pred[:, 0] > 0) & (pred[:, 0] < 1))
    n, ll = np.load(tmp_path / "res.npy")
    assert n == 200 and 0.3 < ll < 1.0
