"""The asynchronous parameter server (BASELINE config 4, parallel/async_ps.py):
workers that never lock-step.

* Live tables equal a one-process replay of the owners' logs bit for bit:
  each owner applied every (source, step) push as its log says, against the
  weights each pull saw (reference: per-push application in arrival order,
  ftrl.h:54-80).
* Bounded staleness: no worker ever pulled with more than k of its own
  pushes unapplied.
* A straggler (XFLOW_FAULT=slow_rank) does not slow the other workers: they
  run ahead of it (lead > k), which the lock-step step cannot do.

CPU backend, gloo for the handshake only; the transport is /dev/shm windows.
The GPU variant (HIP IPC windows, RCCL-free) is tests/test_async_ps_gpu.py.
"""
import os
import time

import numpy as np
import pytest
import torch

from dist_utils import run_world
from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.parallel.async_ps import AsyncParameterServer, replay_logs, worker_config

ROWS, FIELDS, VOCAB = 64, 6, 60


def _cfg(kind, slices):
    model = ModelConfig(kind=kind, v_dim=4)
    cfg = EngineConfig(table_log2_cap=14, max_rows=ROWS, max_nnz=ROWS * 16, max_slices=slices)
    return model, OptimConfig(), cfg


def _batch(rank, step, slices, device=torch.device("cpu")):
    return to_batch(*random_csr(ROWS, FIELDS, VOCAB, seed=7919 * step + rank), device,
                    slice_rows=ROWS // slices)


def _table(eng):
    keys, words = eng.export_table()
    order = np.argsort(keys)
    return keys[order], words.reshape(len(keys), -1)[order]


def _async_rank(rank, world, kind, slices, k, steps, out_dir, slow):
    if slow is not None and rank == slow[0]:
        os.environ["XFLOW_FAULT"] = f"slow_rank:{slow[0]}:{slow[1]}"
    model, optim, cfg = _cfg(kind, slices)
    aps = AsyncParameterServer(model, optim, cfg, "cpu", staleness=k, slices=slices)
    t0 = time.perf_counter()
    for t in range(steps):
        assert aps.train_step(_batch(rank, t, slices))
    aps.finish()
    elapsed = time.perf_counter() - t0
    aps.close()
    keys, words = _table(aps.server)
    st = aps.stats()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), log=aps.log(), keys=keys, words=words,
             elapsed=elapsed, max_staleness=st["max_staleness"], max_lead=st["max_lead"],
             bytes=st["bytes_moved"])


def _replay(out_dir, world, kind, slices, k, steps):
    model, optim, cfg = _cfg(kind, slices)
    logs = [np.load(os.path.join(out_dir, f"r{r}.npz"))["log"] for r in range(world)]
    workers = [Engine(model, optim, worker_config(cfg)) for _ in range(world)]
    servers = [Engine(model, optim, cfg) for _ in range(world)]
    batches = [[_batch(s, t, slices) for t in range(steps)] for s in range(world)]
    replay_logs(logs, batches, workers, servers, k, slices)
    return servers


def _check_equal(out_dir, world, servers):
    for o in range(world):
        live = np.load(os.path.join(out_dir, f"r{o}.npz"))
        keys, words = _table(servers[o])
        assert np.array_equal(keys, live["keys"]), f"owner {o}: key sets differ"
        assert np.array_equal(words, live["words"]), f"owner {o}: table state differs from replay"


@pytest.mark.parametrize("kind,slices,k,world", [("lr", 1, 1, 3), ("lr", 4, 0, 2), ("lr", 4, 2, 3),
                                                 ("fm", 2, 1, 3), ("mvm", 1, 1, 2),
                                                 # a node's eight ranks: every owner serves 7 peers
                                                 ("lr", 4, 1, 8)])
def test_async_tables_equal_log_replay(tmp_path, kind, slices, k, world):
    steps = 5
    run_world(_async_rank, world, kind, slices, k, steps, str(tmp_path), None)
    for r in range(world):
        x = np.load(tmp_path / f"r{r}.npz")
        lg = x["log"]
        # every source's pull and push of every step reached every owner, once
        assert len(lg) == 2 * world * steps
        assert int(x["max_staleness"]) <= k
        for s in range(world):
            mine = lg[lg[:, 1] == s]
            assert mine[mine[:, 0] == 0, 2].tolist() == list(range(steps))
            assert mine[mine[:, 0] == 1, 2].tolist() == list(range(steps))
    _check_equal(str(tmp_path), world, _replay(str(tmp_path), world, kind, slices, k, steps))


def test_async_straggler_does_not_stall_others(tmp_path):
    world, k, steps, slow_ms = 3, 1, 12, 60
    run_world(_async_rank, world, "lr", 2, k, steps, str(tmp_path), (2, slow_ms))
    res = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    slow_t = float(res[2]["elapsed"])
    assert slow_t >= steps * slow_ms / 1000.0
    for r in (0, 1):
        # the fast workers never waited for the straggler's pace ...
        assert float(res[r]["elapsed"]) < 0.5 * slow_t, (r, float(res[r]["elapsed"]), slow_t)
        # ... ran ahead of it by more than any lock-step bound ...
        assert int(res[r]["max_lead"]) > k
        # ... while their own pushes stayed within k of their pulls
        assert int(res[r]["max_staleness"]) <= k
    _check_equal(str(tmp_path), world, _replay(str(tmp_path), world, "lr", 2, k, steps))


def test_async_single_rank_and_eval(tmp_path):
    """World 1 (no process group): train, evaluate through the server thread,
    replay; eval pulls insert nothing."""
    model, optim, cfg = _cfg("lr", 2)
    aps = AsyncParameterServer(model, optim, cfg, "cpu", staleness=1, slices=2)
    for t in range(4):
        aps.train_step(_batch(0, t, 2))
    aps.finish()
    size = aps.server.native.table_size()
    p = aps.eval_step(_batch(0, 99, 2))
    assert p is not None and p.shape == (ROWS,) and torch.isfinite(p).all()
    assert aps.server.native.table_size() == size
    aps.close()
    lg = aps.log()
    assert (lg[:, 0] == 2).sum() == 1
    servers = [Engine(model, optim, cfg)]
    replay_logs([lg[lg[:, 0] != 2]], [[_batch(0, t, 2) for t in range(4)]],
                [Engine(model, optim, worker_config(cfg))], servers, 1, 2)
    keys, words = _table(servers[0])
    lk, lw = _table(aps.server)
    assert np.array_equal(keys, lk) and np.array_equal(words, lw)
    # eval predictions: the same as a forward over the final table
    ref = Engine(model, optim, cfg)
    ref.import_table(*aps.server.export_table())
    q = ref.eval_step(_batch(0, 99, 2))
    np.testing.assert_array_equal(p.numpy(), q.numpy())


def _ckpt_rank(rank, world, data_dir, root, out_dir, resume):
    from xflow_amd.config import TrainConfig
    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=os.path.join(data_dir, "small_train"),
                      test_prefix=os.path.join(data_dir, "small_test"), epochs=3, threads=4,
                      async_ps=True, staleness=1, write_pred=False, save_every=1,
                      engine=EngineConfig(table_log2_cap=14))
    t = Trainer(cfg, device=torch.device("cpu"))
    if resume:
        meta = t.resume(root)
        assert meta is not None and t.epoch == int(meta["epoch"])
        # the resumed server shard is the saved one, bit for bit
        saved = np.load(os.path.join(out_dir, f"ep{t.epoch}_r{rank}.npz"))
        keys, words = _table(t.table)
        assert np.array_equal(keys, saved["keys"]) and np.array_equal(words, saved["words"])
        t.train()
        np.save(os.path.join(out_dir, f"resumed_epoch_r{rank}.npy"), np.array([t.epoch]))
    else:
        cfg.checkpoint_dir = root
        t.train_epochs(2)
        keys, words = _table(t.table)
        np.savez(os.path.join(out_dir, f"ep{t.epoch}_r{rank}.npz"), keys=keys, words=words)
    t.close()


def test_async_trainer_checkpoint_resume(tmp_path):
    """Config 4 through the Trainer with versioned checkpoints: every epoch
    end pauses the servers (all pushes applied), each rank saves its shard;
    a new 2-rank job resumes from LATEST with each shard restored bit for
    bit and trains the remaining epoch."""
    from conftest import DATA

    root = str(tmp_path / "ckpt")
    run_world(_ckpt_rank, 2, DATA, root, str(tmp_path), False)
    assert os.path.exists(os.path.join(root, "LATEST"))
    run_world(_ckpt_rank, 2, DATA, root, str(tmp_path), True)
    for r in range(2):
        assert int(np.load(tmp_path / f"resumed_epoch_r{r}.npy")[0]) == 3
