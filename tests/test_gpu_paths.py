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


@pytest.mark.parametrize("kind,slices", [("lr", 1), ("lr", 4), ("fm", 2)])
def test_rccl_sharded_step_equals_fused(gpu_device, nccl_group, kind, slices):
    from xflow_amd.parallel.sparse_a2a import ShardedEngine

    def mk():
        return Engine(ModelConfig(kind=kind, v_dim=8), OptimConfig(),
                      EngineConfig(table_log2_cap=16, max_rows=512, max_nnz=512 * 16,
                                   max_slices=slices), device=gpu_device)

    a, b = mk(), mk()
    sh = ShardedEngine(a)
    keys = []
    for step in range(4):
        k, rp, fg, lab = random_csr(512, 8, 300, seed=step)
        keys.append(k)
        sh.train_step(to_batch(k, rp, fg, lab, gpu_device, slice_rows=512 // slices))
        b.train_step(to_batch(k, rp, fg, lab, gpu_device, slice_rows=512 // slices))
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
