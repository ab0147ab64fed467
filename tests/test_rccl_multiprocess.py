"""Multi-process RCCL tests on ONE GPU (XFLOW_SHARED_GPU=1, dist_utils.run_world_gpu).

Several processes share GPU 0 and exchange keys, values, gradients and
async pushes through the native RCCL communicator (csrc/comm/rccl_comm.cpp)
and torch's RCCL process group -- real RCCL kernels moving bytes between
processes over its socket transport (each rank presents its own NCCL_HOSTID,
since RCCL refuses two ranks of one host on one device).  This is the code
path of a multi-GPU run minus xGMI: the group calls, the counts exchange with
sequence numbers, the pipelined step, the async send/recv.  Each test checks
the result against a single-process replay, as the gloo tests do
(tests/test_multirank.py); reference call sites: lr_worker.cc:170,175
(Pull/Push), ftrl.h:54-80 (server apply)."""
import os

import numpy as np
import pytest
import torch

from dist_utils import run_world_gpu
from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.testing.hashing import owner_of

pytestmark = pytest.mark.gpu

ROWS, FIELDS, VOCAB, STEPS = 512, 8, 300, 4


def _batches(rank, step):
    return random_csr(ROWS, FIELDS, VOCAB, seed=7000 * step + rank)


def _make_engine(kind, world, dev):
    return Engine(ModelConfig(kind=kind, v_dim=4), OptimConfig(),
                  EngineConfig(table_log2_cap=16, max_rows=world * ROWS,
                               max_nnz=world * ROWS * 16, max_slices=world),
                  device=dev)


def _sharded_worker(rank, world, kind, out_dir):
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    dev = torch.device("cuda", 0)
    eng = _make_engine(kind, world, dev)
    sh = ShardedEngine(eng)
    assert sh.transport == "rccl", sh.transport
    bs = [to_batch(*_batches(rank, s), dev) for s in range(STEPS)]
    for s in range(STEPS):
        sh.train_step(bs[s], next_batch=bs[s + 1] if s + 1 < STEPS else None)
    torch.cuda.synchronize(dev)
    assert not eng.overflowed()
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"k{rank}.npy"), keys)
    np.save(os.path.join(out_dir, f"v{rank}.npy"), eng.pull(keys))
    np.save(os.path.join(out_dir, f"b{rank}.npy"), np.array([sh.bytes_moved]))


@pytest.mark.parametrize("world,kind", [(2, "lr"), (4, "lr"), (2, "fm"), (3, "mvm")])
def test_rccl_processes_sharded_equals_single_engine(gpu_device, tmp_path, world, kind):
    """W processes on one GPU, pipelined sharded step over RCCL: the union of
    their table shards equals one engine trained on the concatenated batches
    as W ordered slices."""
    run_world_gpu(_sharded_worker, world, kind, str(tmp_path))
    ref = _make_engine(kind, world, gpu_device)
    for s in range(STEPS):
        parts = [_batches(r, s) for r in range(world)]
        keys = np.concatenate([p[0] for p in parts])
        fg = np.concatenate([p[2] for p in parts])
        lab = np.concatenate([p[3] for p in parts])
        rp = np.concatenate([parts[0][1]] + [p[1][1:] + sum(len(q[0]) for q in parts[:i + 1])
                                             for i, p in enumerate(parts[1:])])
        ref.train_step(to_batch(keys, rp.astype(np.int32), fg, lab, gpu_device,
                                slice_rows=ROWS))
    k = np.concatenate([np.load(tmp_path / f"k{r}.npy") for r in range(world)])
    v = np.concatenate([np.load(tmp_path / f"v{r}.npy") for r in range(world)])
    for r in range(world):
        kr = np.load(tmp_path / f"k{r}.npy")
        assert (owner_of(kr, world) == r).all(), "a rank holds keys it does not own"
        assert np.load(tmp_path / f"b{r}.npy")[0] > 0
    assert len(np.unique(k)) == len(k) == ref.table_size()
    np.testing.assert_allclose(v, ref.pull(k), rtol=1e-4, atol=1e-6)


def _async_worker(rank, world, out_dir, staleness):
    from xflow_amd.parallel.async_p2p import AsyncShardedEngine

    dev = torch.device("cuda", 0)
    eng = _make_engine("lr", world, dev)
    sh = AsyncShardedEngine(eng, staleness=staleness)
    bs = [to_batch(*_batches(rank, s), dev) for s in range(STEPS + 2)]
    for s in range(STEPS + 2):
        nxt = bs[s + 1] if 0 < s < STEPS + 1 else None
        sh.train_step(bs[s], S=1, next_batch=nxt)
    sh.flush()
    torch.cuda.synchronize(dev)
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"ak{rank}.npy"), keys)
    np.save(os.path.join(out_dir, f"av{rank}.npy"), eng.pull(keys))
    assert sh.p2p_ops > 0


@pytest.mark.parametrize("staleness", [1, 2])
def test_rccl_processes_async_staleness_matches_simulation(gpu_device, tmp_path, staleness):
    """Config 4 over RCCL between processes: pushes ride in the key exchange
    k steps later; equals the reference step whose pulls miss exactly the
    previous k steps' pushes."""
    from collections import deque

    from xflow_amd.testing import torch_ref
    from xflow_amd.testing.hashing import normal_init

    world = 2
    run_world_gpu(_async_worker, world, str(tmp_path), staleness)
    ref = torch_ref.RefTable(1, 1, "ftrl", init_fn=lambda k, d: normal_init(k, d) * 1e-2)
    pending = deque()
    for s in range(STEPS + 2):
        parts = [_batches(r, s) for r in range(world)]
        keys = np.concatenate([p[0] for p in parts])
        lab = np.concatenate([p[3] for p in parts])
        rp = np.concatenate([parts[0][1]] + [p[1][1:] + len(parts[0][0]) for p in parts[1:]])
        _, cur = torch_ref.compute_step(ref, "lr", keys, lab, rp.astype(np.int32), ROWS)
        if len(pending) == staleness:
            torch_ref.apply_step(ref, pending.popleft())
        pending.append(cur)
    while pending:
        torch_ref.apply_step(ref, pending.popleft())
    k = np.concatenate([np.load(tmp_path / f"ak{r}.npy") for r in range(world)])
    v = np.concatenate([np.load(tmp_path / f"av{r}.npy") for r in range(world)])
    np.testing.assert_allclose(v, ref.weights(k, insert=False).numpy(), rtol=1e-4, atol=1e-6)


def _trainer_worker(rank, world, data_dir, pred_dir, gpu):
    from xflow_amd.config import TrainConfig
    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=os.path.join(data_dir, "small_train"),
                      test_prefix=os.path.join(data_dir, "small_test"), epochs=3, threads=4,
                      pred_dir=pred_dir, engine=EngineConfig(table_log2_cap=14),
                      train_block_bytes=4096 if rank == 0 else 6144)
    t = Trainer(cfg, device=torch.device("cuda", 0) if gpu else torch.device("cpu"))
    if gpu:
        assert t.sharded.transport == "rccl", t.sharded.transport
    t.train()


def test_rccl_processes_trainer_equals_cpu_gloo(gpu_device, tmp_path):
    """The Trainer (CLI path) on 2 GPU processes over RCCL writes the same
    predictions as the same 2-rank job on the CPU backend over gloo."""
    from conftest import DATA
    from dist_utils import run_world

    gdir, cdir = tmp_path / "gpu", tmp_path / "cpu"
    gdir.mkdir()
    cdir.mkdir()
    run_world_gpu(_trainer_worker, 2, DATA, str(gdir), True)
    run_world(_trainer_worker, 2, DATA, str(cdir), False)
    g = np.loadtxt(gdir / "pred_0_0.txt")
    c = np.loadtxt(cdir / "pred_0_0.txt")
    assert g.shape == c.shape == (200, 3)
    np.testing.assert_allclose(g, c, rtol=1e-5, atol=1e-6)


# ---- bench scale over RCCL between processes: W = 4 x 32 768 Criteo-shaped
# rows x 39 fields x 5 pipelined steps (the loopback test's shape,
# tests/test_w8_loopback.py, now through real RCCL group calls)
BS_ROWS, BS_STEPS, BS_W = 32768, 5, 4


def _bs_batches(rank, dev, kind="lr"):
    from xflow_amd.data.synth import SynthConfig, SyntheticCriteo

    # (an MVM generator engine also fills the field ids MVM needs)
    gen_eng = Engine(ModelConfig(kind="mvm" if kind == "mvm" else "lr"), OptimConfig(),
                     EngineConfig(table_log2_cap=10, max_rows=BS_ROWS, max_nnz=BS_ROWS * 39),
                     device=dev)
    g = SyntheticCriteo(gen_eng, BS_ROWS, SynthConfig(seed=4242), rank=rank)
    out = []
    for _ in range(BS_STEPS):
        b = g.alloc_batch()
        g.next(out=b)
        out.append(b)
    return out


def _bs_engine(dev, rows, log2_cap, slices=1, kind="lr", owner_group=0):
    # ("fm_std": standard-math FM, full-row CSR entries)
    m = (ModelConfig(kind="fm", v_dim=4, fm_math="standard") if kind == "fm_std"
         else ModelConfig(kind=kind, v_dim=4))
    # (MVM live: SGD from v = 0.9, so the 39-field products stay non-zero)
    o = OptimConfig(kind="sgd", sgd_v_init=0.9) if kind == "mvm" else OptimConfig()
    return Engine(m, o,
                  EngineConfig(table_log2_cap=log2_cap, max_rows=rows, max_nnz=rows * 39,
                               max_slices=slices, owner_group=owner_group), device=dev)


def _bs_worker(rank, world, kind, out_dir):
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    dev = torch.device("cuda", 0)
    eng = _bs_engine(dev, BS_ROWS, 22, kind=kind)
    sh = ShardedEngine(eng)
    assert sh.transport == "rccl", sh.transport
    bs = _bs_batches(rank, dev)
    for s in range(BS_STEPS):
        assert sh.train_step(bs[s], S=1, next_batch=bs[s + 1] if s + 1 < BS_STEPS else None)
    torch.cuda.synchronize(dev)
    assert not eng.overflowed()
    assert sh.inline_prepares == 1 and sh.early_key_exchanges == BS_STEPS - 1
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"bk{rank}.npy"), keys)
    np.save(os.path.join(out_dir, f"bv{rank}.npy"), eng.pull(keys))


@pytest.mark.parametrize("kind", ["lr", "fm"])
def test_rccl_processes_bench_scale_equals_single_engine(gpu_device, tmp_path, kind):
    """4 processes x 32 768 Criteo-shaped rows x 39 fields x 5 pipelined steps
    over RCCL == one engine trained on the 4 ranks' batches as 4 ordered
    slices per step (rtol 1e-4)."""
    from xflow_amd.engine import Batch

    run_world_gpu(_bs_worker, BS_W, kind, str(tmp_path))
    data = [_bs_batches(r, gpu_device) for r in range(BS_W)]
    ref = _bs_engine(gpu_device, BS_W * BS_ROWS, 25, slices=BS_W, kind=kind)
    for s in range(BS_STEPS):
        keys = torch.cat([data[r][s].keys.view(39, BS_ROWS) for r in range(BS_W)],
                         dim=1).reshape(-1)
        lab = torch.cat([data[r][s].labels for r in range(BS_W)])
        ref.train_step(Batch(keys=keys.contiguous(), labels=lab, nnz_per_row=39,
                             field_major=True, slice_rows=BS_ROWS))
    k = np.concatenate([np.load(tmp_path / f"bk{r}.npy") for r in range(BS_W)])
    v = np.concatenate([np.load(tmp_path / f"bv{r}.npy") for r in range(BS_W)])
    for r in range(BS_W):
        assert (owner_of(np.load(tmp_path / f"bk{r}.npy"), BS_W) == r).all()
    assert len(np.unique(k)) == len(k) == ref.table_size()
    np.testing.assert_allclose(v, ref.pull(k), rtol=1e-4, atol=1e-6)


# ---- several Hogwild slices per rank over RCCL: the CSR exchange (only the
# touched (key, slice) entries move; reference: each slice pushes its own
# keys, lr_worker.cc:162-175)
CSR_S, CSR_STEPS = 64, 3


def _csr_worker(rank, world, kind, out_dir, owner_group=0):
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    dev = torch.device("cuda", 0)
    eng = _bs_engine(dev, BS_ROWS, 22, slices=CSR_S, kind=kind, owner_group=owner_group)
    sh = ShardedEngine(eng)
    assert sh.transport == "rccl", sh.transport
    bs = _bs_batches(rank, dev, kind)[:CSR_STEPS]
    for b in bs:
        b.slice_rows = BS_ROWS // CSR_S
    for s in range(CSR_STEPS):
        assert sh.train_step(bs[s], S=CSR_S, next_batch=bs[s + 1] if s + 1 < CSR_STEPS else None)
    torch.cuda.synchronize(dev)
    assert not eng.overflowed()
    assert sh.csr_exchanges == CSR_STEPS, sh.csr_exchanges
    keys, _ = eng.export_table()
    np.save(os.path.join(out_dir, f"ck{rank}.npy"), keys)
    np.save(os.path.join(out_dir, f"cv{rank}.npy"), eng.pull(keys))
    np.save(os.path.join(out_dir, f"cb{rank}.npy"), np.array([sh.bytes_moved]))


@pytest.mark.parametrize("kind,CSR_W,owner_group", [
    ("lr", 2, 0), ("fm", 2, 0), ("fm_std", 2, 0), ("mvm", 2, 0),
    # >= 3 sources: the owners' per-source apply order (s_apply_csr's first
    # source), and reference FM with the owner grouping configured (the CSR
    # pull keeps the pulled weights, no grouping)
    ("lr", 4, 0), ("fm", 4, 1), ("fm_std", 4, 0), ("mvm", 3, 0)])
def test_rccl_processes_csr_slices_equal_single_engine(gpu_device, tmp_path, kind, CSR_W,
                                                        owner_group):
    """W processes x 32 768 Criteo-shaped rows x 64 slices each, 3 pipelined
    steps over RCCL with the CSR gradient exchange == one engine trained on
    every rank's rows as W x 64 ordered slices per step (source 0's slices,
    then source 1's, ...); the bytes moved are the touched pairs', far below
    the dense [keys][64 x width] blocks."""
    from xflow_amd.engine import Batch

    run_world_gpu(_csr_worker, CSR_W, kind, str(tmp_path), owner_group)
    data = [_bs_batches(r, gpu_device, kind)[:CSR_STEPS] for r in range(CSR_W)]
    ref = _bs_engine(gpu_device, CSR_W * BS_ROWS, 24, slices=CSR_W * CSR_S, kind=kind)
    for s in range(CSR_STEPS):
        keys = torch.cat([data[r][s].keys.view(39, BS_ROWS) for r in range(CSR_W)],
                         dim=1).reshape(-1)
        lab = torch.cat([data[r][s].labels for r in range(CSR_W)])
        fg = (torch.cat([data[r][s].fgid.view(39, BS_ROWS) for r in range(CSR_W)], dim=1)
              .reshape(-1).contiguous() if kind == "mvm" else None)
        ref.train_step(Batch(keys=keys.contiguous(), labels=lab, fgid=fg, nnz_per_row=39,
                             field_major=True, slice_rows=BS_ROWS // CSR_S))
    assert ref.csr_steps == CSR_STEPS
    k = np.concatenate([np.load(tmp_path / f"ck{r}.npy") for r in range(CSR_W)])
    v = np.concatenate([np.load(tmp_path / f"cv{r}.npy") for r in range(CSR_W)])
    assert len(np.unique(k)) == len(k) == ref.table_size()
    np.testing.assert_allclose(v, ref.pull(k), rtol=1e-4, atol=1e-6)
    # dense per-slice blocks would move >= n_keys x 64 x width floats per step
    width = {"lr": 1, "fm": 2, "fm_std": 8, "mvm": 4}[kind]
    dense = CSR_STEPS * len(k) * CSR_S * 4 * width / CSR_W
    for r in range(CSR_W):
        assert np.load(tmp_path / f"cb{r}.npy")[0] < dense / 4
