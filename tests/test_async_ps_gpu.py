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
