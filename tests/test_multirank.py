"""Multi-rank (gloo, CPU) tests of the sharded table + sparse all-to-all path.

Equivalence: one lock-step step on W ranks with S slices each equals one
single-rank step whose batch concatenates the ranks' batches as W*S ordered
slices (every slice reads the same weights; owners apply pushes in (source,
slice) order; gradients normalised per slice)."""
import os

import numpy as np
import pytest
import torch

from dist_utils import run_world
from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.testing.hashing import owner_of

ROWS, FIELDS, VOCAB, STEPS = 64, 6, 80, 3


def _batches(rank, step):
    return random_csr(ROWS, FIELDS, VOCAB, seed=1000 * step + rank)


def _make_engine(kind, slices):
    return Engine(ModelConfig(kind=kind, v_dim=4), OptimConfig(),
                  EngineConfig(table_log2_cap=14, max_rows=4 * ROWS, max_nnz=4 * ROWS * 16,
                               max_slices=4 * slices))


def _sharded_worker(rank, world, kind, slices, out_dir, pipelined=False):
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    eng = _make_engine(kind, slices)
    sh = ShardedEngine(eng)
    batches = [to_batch(*_batches(rank, step), torch.device("cpu"), slice_rows=ROWS // slices)
               for step in range(STEPS)]
    for step in range(STEPS):
        # pipelined: the next batch is prepared (dedup, counts exchange) inside
        # this step, into the other worker buffer set
        nxt = batches[step + 1] if pipelined and step + 1 < STEPS else None
        sh.train_step(batches[step], S=slices, next_batch=nxt)
    keys, words = eng.export_table()
    np.save(os.path.join(out_dir, f"keys{rank}.npy"), keys)
    vals = eng.pull(keys) if len(keys) else np.zeros((0, eng.params_per_key), np.float32)
    np.save(os.path.join(out_dir, f"vals{rank}.npy"), vals)
    st = eng.read_stats()
    np.save(os.path.join(out_dir, f"stats{rank}.npy"), np.array([st["rows"], st["ln_loss"]]))


@pytest.mark.parametrize("kind,slices,pipelined,world",
                         [("lr", 1, False, 2), ("lr", 2, False, 2), ("fm", 2, False, 2),
                          ("mvm", 1, False, 2), ("lr", 2, True, 3), ("fm", 1, True, 2),
                          # > 32 slices per rank: slice groups, (source, slice) order
                          ("lr", 64, True, 2), ("fm", 64, False, 2), ("mvm", 64, True, 2)])
def test_sharded_equals_single_rank(tmp_path, kind, slices, pipelined, world):
    run_world(_sharded_worker, world, kind, slices, str(tmp_path), pipelined)
    # single-rank replay: concatenated batches, world*slices ordered slices
    ref = _make_engine(kind, slices)
    for step in range(STEPS):
        parts = [_batches(r, step) for r in range(world)]
        keys = np.concatenate([p[0] for p in parts])
        fg = np.concatenate([p[2] for p in parts])
        lab = np.concatenate([p[3] for p in parts])
        rp = np.concatenate([parts[0][1]] + [p[1][1:] + sum(len(q[0]) for q in parts[:i + 1])
                                             for i, p in enumerate(parts[1:])])
        ref.train_step(to_batch(keys, rp.astype(np.int32), fg, lab, torch.device("cpu"),
                                slice_rows=ROWS // slices))
    allk, allv = [], []
    for r in range(world):
        k = np.load(tmp_path / f"keys{r}.npy")
        assert (owner_of(k, world) == r).all(), "a rank holds keys it does not own"
        allk.append(k)
        allv.append(np.load(tmp_path / f"vals{r}.npy"))
    k = np.concatenate(allk)
    v = np.concatenate(allv)
    assert len(np.unique(k)) == len(k)
    want = ref.pull(k)
    assert ref.table_size() == len(k)
    np.testing.assert_allclose(v, want, rtol=1e-4, atol=1e-6)
    rows = sum(np.load(tmp_path / f"stats{r}.npy")[0] for r in range(world))
    assert rows == world * ROWS * STEPS


def _ckpt_worker(rank, world, ckpt_dir, out_dir):
    from xflow_amd import checkpoint
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    eng = _make_engine("fm", 1)
    sh = ShardedEngine(eng)
    for step in range(2):
        k, rp, fg, lab = _batches(rank, step)
        sh.train_step(to_batch(k, rp, fg, lab, torch.device("cpu")))
    checkpoint.save(eng, ckpt_dir, rank, world, meta={"epoch": 1})
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"k{rank}.npy"), keys)
    np.save(os.path.join(out_dir, f"v{rank}.npy"), eng.pull(keys))


def _reload_worker(rank, world, ckpt_dir, out_dir):
    from xflow_amd import checkpoint

    eng = _make_engine("fm", 1)
    meta = checkpoint.load(eng, ckpt_dir, rank, world)
    assert meta["epoch"] == 1 and meta["world"] == 2
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"rk{rank}.npy"), keys)
    np.save(os.path.join(out_dir, f"rv{rank}.npy"), eng.pull(keys))


def test_checkpoint_reshard_2_to_1_and_3(tmp_path):
    ck = str(tmp_path / "ckpt")
    run_world(_ckpt_worker, 2, ck, str(tmp_path))
    k = np.concatenate([np.load(tmp_path / f"k{r}.npy") for r in range(2)])
    v = np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(2)])
    order = np.argsort(k)
    # world 1: one engine loads every shard
    from xflow_amd import checkpoint

    one = _make_engine("fm", 1)
    checkpoint.load(one, ck, 0, 1)
    np.testing.assert_array_equal(one.pull(k[order]), v[order])
    # world 3: keys re-sharded by the new owner function
    run_world(_reload_worker, 3, ck, str(tmp_path))
    k3 = np.concatenate([np.load(tmp_path / f"rk{r}.npy") for r in range(3)])
    v3 = np.concatenate([np.load(tmp_path / f"rv{r}.npy") for r in range(3)])
    o3 = np.argsort(k3)
    np.testing.assert_array_equal(k3[o3], k[order])
    np.testing.assert_array_equal(v3[o3], v[order])


def _trainer_worker(rank, world, data_dir, pred_dir):
    import json

    from xflow_amd.config import TrainConfig
    from xflow_amd.parallel import dist as xdist
    from xflow_amd.trainer import Trainer

    metrics = os.path.join(pred_dir, "metrics.jsonl")
    # 4 KB blocks: several blocks (steps) per epoch; rank 1 has fewer rows, so
    # it runs out of data first and joins the last steps with empty batches
    cfg = TrainConfig(train_prefix=os.path.join(data_dir, "small_train"),
                      test_prefix=os.path.join(data_dir, "small_test"), epochs=3, threads=4,
                      pred_dir=pred_dir, engine=EngineConfig(table_log2_cap=14),
                      train_block_bytes=4096 if rank == 0 else 6144, metrics_file=metrics)
    t = Trainer(cfg, device=torch.device("cpu"))
    # the training loop needs no per-block collective or host sync: the end
    # of an epoch travels in the counts exchange of the pipelined step
    calls = []
    orig = xdist.all_any
    xdist.all_any = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        t.train_epochs(cfg.epochs)
    finally:
        xdist.all_any = orig
    assert not calls, "per-block all_any in the training loop"
    assert t.sharded.empty_steps == cfg.epochs
    res = t.predict(0)
    if rank == 0:
        assert res["n"] == 200 and 0.0 < res["auc"] < 1.0
        recs = [json.loads(x) for x in open(metrics)]
        ep = [r for r in recs if r["event"] == "epoch"]
        assert len(ep) == 3 and all(r["steps"] > 3 * (i + 1) for i, r in enumerate(ep))
        # one batch per epoch is prepared in line (the first); no step waited
        assert all(r["inline_prepares"] == 1 and r["host_waits"] == 0 for r in ep), ep
        # steady state: the next batch's keys ride in the gradient exchange
        assert ep[-1]["early_key_exchanges"] >= ep[-1]["steps"] - 3 * len(ep), ep


def test_trainer_two_workers_bundled_data(tmp_path):
    from conftest import DATA

    run_world(_trainer_worker, 2, DATA, str(tmp_path))
    pred = np.loadtxt(tmp_path / "pred_0_0.txt")
    assert pred.shape == (200, 3)


def _async_worker(rank, world, out_dir, staleness=1, slices=1):
    from xflow_amd.parallel.async_p2p import AsyncShardedEngine

    eng = _make_engine("lr", slices)
    sh = AsyncShardedEngine(eng, staleness=staleness)
    bs = [to_batch(*_batches(rank, step), torch.device("cpu"), slice_rows=ROWS // slices)
          for step in range(STEPS + 2)]
    for step in range(STEPS + 2):
        # pipelined (next batch prepared inside the step) from the second step on
        nxt = bs[step + 1] if 0 < step < STEPS + 1 else None
        sh.train_step(bs[step], S=slices, next_batch=nxt)
    sh.flush()
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"akeys{rank}.npy"), keys)
    np.save(os.path.join(out_dir, f"avals{rank}.npy"), eng.pull(keys))
    assert sh.p2p_ops > 0


@pytest.mark.parametrize("staleness,slices", [(1, 1), (2, 1), (3, 1), (1, 64)])
def test_async_p2p_staleness_one_matches_simulation(tmp_path, staleness, slices):
    """AsyncShardedEngine == the reference step with pulls that miss exactly
    the previous k steps' pushes (staleness k), pushes in (source, slice)
    order (64 slices per rank: two slice groups)."""
    from collections import deque

    from xflow_amd.testing import torch_ref
    from xflow_amd.testing.hashing import normal_init

    world = 2
    run_world(_async_worker, world, str(tmp_path), staleness, slices)
    ref = torch_ref.RefTable(1, 1, "ftrl", init_fn=lambda k, d: normal_init(k, d) * 1e-2)
    pending = deque()
    for step in range(STEPS + 2):
        parts = [_batches(r, step) for r in range(world)]
        keys = np.concatenate([p[0] for p in parts])
        lab = np.concatenate([p[3] for p in parts])
        rp = np.concatenate([parts[0][1]] + [p[1][1:] + len(parts[0][0]) for p in parts[1:]])
        _, cur = torch_ref.compute_step(ref, "lr", keys, lab, rp.astype(np.int32), ROWS // slices)
        if len(pending) == staleness:
            torch_ref.apply_step(ref, pending.popleft())
        pending.append(cur)
    while pending:
        torch_ref.apply_step(ref, pending.popleft())
    k = np.concatenate([np.load(tmp_path / f"akeys{r}.npy") for r in range(world)])
    v = np.concatenate([np.load(tmp_path / f"avals{r}.npy") for r in range(world)])
    want = ref.weights(k, insert=False).numpy()
    np.testing.assert_allclose(v, want, rtol=1e-4, atol=1e-6)


def _async_trainer_worker(rank, world, data_dir, pred_dir):
    from xflow_amd.config import TrainConfig
    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=os.path.join(data_dir, "small_train"),
                      test_prefix=os.path.join(data_dir, "small_test"), epochs=2, threads=4,
                      pred_dir=pred_dir, async_p2p=True,
                      optim=OptimConfig(lambda1=0.01),
                      engine=EngineConfig(table_log2_cap=14))
    t = Trainer(cfg, device=torch.device("cpu"))
    res = t.train()
    if rank == 0:
        assert res["n"] == 200 and 0.0 < res["auc"] < 1.0


def test_trainer_async_p2p_two_workers(tmp_path):
    from conftest import DATA

    run_world(_async_trainer_worker, 2, DATA, str(tmp_path))
    assert np.loadtxt(tmp_path / "pred_0_0.txt").shape == (200, 3)


def _mismatch_worker(rank, world, out_dir, pipelined):
    """train_step(A, next_batch=B) then train_step(C): the step must drop the
    keys exchanged ahead for B and train C on its own keys."""
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    eng = _make_engine("fm", 1)
    sh = ShardedEngine(eng)
    dev = torch.device("cpu")
    A, B, C = (to_batch(*_batches(rank, s), dev, slice_rows=ROWS) for s in (0, 1, 2))
    if pipelined:
        sh.train_step(A, S=1, next_batch=B)  # (B's keys ride in A's gradient exchange)
        sh.train_step(C, S=1)                # not the announced batch
        sh.train_step(B, S=1)
    else:
        for b in (A, C, B):
            sh.train_step(b, S=1)
    keys, _ = eng.export_table()
    o = np.argsort(keys)
    np.save(os.path.join(out_dir, f"k{rank}_{int(pipelined)}.npy"), keys[o])
    np.save(os.path.join(out_dir, f"v{rank}_{int(pipelined)}.npy"), eng.pull(keys[o]))


def test_unannounced_batch_drops_early_keys(tmp_path):
    """gloo, 2 ranks: a step on a batch other than the announced next one
    equals the unpipelined sequence bit for bit."""
    for pipelined in (False, True):
        run_world(_mismatch_worker, 2, str(tmp_path), pipelined)
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"k{r}_0.npy"),
                                      np.load(tmp_path / f"k{r}_1.npy"))
        np.testing.assert_array_equal(np.load(tmp_path / f"v{r}_0.npy").view(np.uint32),
                                      np.load(tmp_path / f"v{r}_1.npy").view(np.uint32))


def _parse_worker(rank, world, data_dir, out_dir, gpu_parse, resident):
    from xflow_amd.config import TrainConfig
    from xflow_amd.trainer import Trainer

    # 4 KB blocks of variable-width rows (bundled data: fields 16/17 multi-valued):
    # several CSR blocks per epoch, the next one announced before the current trains
    cfg = TrainConfig(train_prefix=os.path.join(data_dir, "small_train"),
                      test_prefix=os.path.join(data_dir, "small_test"), epochs=3, threads=4,
                      pred_dir=out_dir, engine=EngineConfig(table_log2_cap=14),
                      train_block_bytes=4096, gpu_parse=gpu_parse, resident=resident)
    t = Trainer(cfg, device=torch.device("cpu"))
    t.train_epochs(cfg.epochs)
    t.predict(0)


@pytest.mark.parametrize("resident", [False, True])
def test_device_parse_two_workers_equals_host_parse(tmp_path, resident):
    """The device tokeniser's stream (TextStream; on the CPU backend it parses
    with reader.cpp's rules) feeds the 2-rank pipelined step -- which parses
    block t+1 before block t trains -- and the --resident cache the same
    variable-width CSR blocks as the host reader: identical models."""
    from conftest import DATA

    preds = []
    for tag, gp, res in (("host", False, False), ("dev", True, resident)):
        d = tmp_path / tag
        d.mkdir()
        run_world(_parse_worker, 2, DATA, str(d), gp, res)
        preds.append(np.loadtxt(d / "pred_0_0.txt"))
    np.testing.assert_array_equal(preds[0], preds[1])
