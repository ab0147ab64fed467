"""The native sharded step (csrc/comm/sharded_step.cpp) against the Python
ShardedEngine step it replaces (xflow_amd/parallel/sparse_a2a.py).

On the CPU the native step runs at world 1 (the self-exchange; its RCCL
group calls need GPUs): pipelined steps (the next batch prepared mid-step),
slice groups (> 32 slices), eval steps between training steps and an empty
batch at the end must give bit-identical tables, losses and predictions.
Multi-rank native steps over RCCL are covered by
tests/test_rccl_multiprocess.py on the GPU box.
"""
import os

import numpy as np
import pytest
import torch

from dist_utils import run_world
from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Batch, Engine

ROWS, FIELDS, VOCAB, STEPS = 120, 6, 90, 4


def _worker(rank, world, out_dir, kind, slices, pipelined, native, staleness=0):
    os.environ["XFLOW_NATIVE_STEP"] = "1" if native else "0"
    from xflow_amd.parallel.async_p2p import AsyncShardedEngine
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    dev = torch.device("cpu")
    eng = Engine(ModelConfig(kind=kind, v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=14, max_rows=ROWS, max_nnz=ROWS * 16,
                              max_slices=slices))
    sh = AsyncShardedEngine(eng, staleness=staleness) if staleness else ShardedEngine(eng)
    assert sh.native_step == native
    sr = max(1, ROWS // slices)
    batches = [to_batch(*random_csr(ROWS, FIELDS, VOCAB, seed=7 * step + 1), dev, slice_rows=sr)
               for step in range(STEPS)]
    test = to_batch(*random_csr(ROWS, FIELDS, VOCAB, seed=999), dev)
    preds = []
    calls = [0]

    def prefetch():  # (the caller's device work producing the next batch)
        calls[0] += 1

    for step in range(STEPS):
        nxt = batches[step + 1] if pipelined and step + 1 < STEPS else None
        assert sh.train_step(batches[step], S=slices, next_batch=nxt, prefetch=prefetch)
        if step == 1:  # an evaluation between training steps
            preds.append(sh.eval_step(test).numpy().copy())
    preds.append(sh.eval_step(test).numpy().copy())
    empty = Batch(keys=torch.zeros(0, dtype=torch.int64), labels=torch.zeros(0),
                  row_ptr=torch.zeros(1, dtype=torch.int32), slice_rows=sr)
    assert not sh.train_step(empty, S=slices)
    assert sh.eval_step(empty) is None
    if staleness:
        sh.flush()
    keys, words = eng.export_table()
    o = np.argsort(keys)
    st = eng.read_stats()
    tag = "n" if native else "p"
    np.save(os.path.join(out_dir, f"keys_{tag}.npy"), keys[o])
    np.save(os.path.join(out_dir, f"words_{tag}.npy"), words.reshape(len(keys), -1)[o])
    np.save(os.path.join(out_dir, f"stats_{tag}.npy"), np.array([st["rows"], st["ln_loss"]]))
    np.save(os.path.join(out_dir, f"preds_{tag}.npy"), np.stack(preds))
    np.save(os.path.join(out_dir, f"counters_{tag}.npy"),
            np.array([sh.inline_prepares, sh.empty_steps, sh.bytes_moved, calls[0],
                      getattr(sh, "p2p_ops", 0)]))


@pytest.mark.parametrize("kind,slices,pipelined,staleness",
                         [("lr", 1, True, 0), ("lr", 4, False, 0), ("fm", 1, True, 0),
                          ("fm", 40, True, 0), ("mvm", 1, False, 0), ("lr", 40, True, 0),
                          # the staleness-k step (async_p2p.AsyncShardedEngine)
                          ("lr", 1, True, 1), ("fm", 4, False, 2), ("mvm", 40, True, 1)])
def test_native_step_equals_python_step(tmp_path, kind, slices, pipelined, staleness):
    for native in (False, True):
        run_world(_worker, 1, str(tmp_path), kind, slices, pipelined, native, staleness)
    for name in ("keys", "words", "stats", "preds", "counters"):
        a = np.load(tmp_path / f"{name}_p.npy")
        b = np.load(tmp_path / f"{name}_n.npy")
        assert a.shape == b.shape, name
        np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8), err_msg=name)


def _mismatch_worker(rank, world, out_dir, native):
    os.environ["XFLOW_NATIVE_STEP"] = "1" if native else "0"
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    dev = torch.device("cpu")
    eng = Engine(ModelConfig(kind="fm", v_dim=4), OptimConfig(),
                 EngineConfig(table_log2_cap=14, max_rows=ROWS, max_nnz=ROWS * 16))
    sh = ShardedEngine(eng)
    A, B, C = (to_batch(*random_csr(ROWS, FIELDS, VOCAB, seed=s), dev) for s in (3, 4, 5))
    sh.train_step(A, S=1, next_batch=B)  # B prepared ahead ...
    sh.train_step(C, S=1)                # ... but C comes first
    sh.train_step(B, S=1, next_batch=C)
    sh.train_step(C, S=1)
    keys, _ = eng.export_table()
    o = np.argsort(keys)
    tag = "n" if native else "p"
    np.save(os.path.join(out_dir, f"mk_{tag}.npy"), keys[o])
    np.save(os.path.join(out_dir, f"mv_{tag}.npy"), eng.pull(keys[o]))
    np.save(os.path.join(out_dir, f"mc_{tag}.npy"), np.array([sh.inline_prepares]))


def test_native_step_unannounced_batch(tmp_path):
    """A step on a batch other than the prepared one prepares its own (both
    implementations alike, bit for bit)."""
    for native in (False, True):
        run_world(_mismatch_worker, 1, str(tmp_path), native)
    for name in ("mk", "mv", "mc"):
        a, b = np.load(tmp_path / f"{name}_p.npy"), np.load(tmp_path / f"{name}_n.npy")
        np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8), err_msg=name)
