"""Inference from a checkpoint (xflow_amd/serve.py): a Predictor loaded from a
training checkpoint scores the test file exactly like the trainer's own
rank-0 evaluation (pred_0_0.txt, lr_worker.cc:40-98), including after a
2-rank (sharded) training run, and the HTTP endpoint returns the same."""
import os

import numpy as np
import pytest
import torch

from conftest import DATA
from dist_utils import run_world


def _train(out, kind, device="cpu"):
    from xflow_amd.config import EngineConfig, ModelConfig, TrainConfig
    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=os.path.join(DATA, "small_train"),
                      test_prefix=os.path.join(DATA, "small_test"), epochs=3, threads=8,
                      pred_dir=str(out), model=ModelConfig(kind=kind, v_dim=4),
                      engine=EngineConfig(table_log2_cap=14), checkpoint_dir=str(out / "ck"),
                      save_every=1)
    Trainer(cfg, device=torch.device(device)).train()
    return np.loadtxt(out / "pred_0_0.txt")


def _test_text():
    with open(os.path.join(DATA, "small_test-00000"), "rb") as f:
        return f.read()


@pytest.mark.parametrize("kind", ["lr", "fm", "mvm"])
def test_predictor_equals_trainer_eval(tmp_path, kind):
    from xflow_amd.serve import Predictor

    want = _train(tmp_path, kind)
    p = Predictor(str(tmp_path / "ck"), device=torch.device("cpu"), max_rows=64)
    got = p.predict_libffm(_test_text())
    assert got.shape == (200,)
    np.testing.assert_allclose(got, want[:, 0], rtol=2e-5, atol=1e-6)


def _sharded_train(rank, world, out):
    import pathlib

    _train(pathlib.Path(out), "lr")


def test_predictor_loads_a_two_rank_checkpoint(tmp_path):
    """Shards of a 2-rank run are merged into one serving table."""
    from xflow_amd.serve import Predictor

    run_world(_sharded_train, 2, str(tmp_path))
    want = np.loadtxt(tmp_path / "pred_0_0.txt")
    p = Predictor(str(tmp_path / "ck"), device=torch.device("cpu"))
    assert p.meta["world"] == 2
    np.testing.assert_allclose(p.predict_libffm(_test_text()), want[:, 0], rtol=2e-5, atol=1e-6)


def test_http_predict(tmp_path):
    from fastapi.testclient import TestClient

    from xflow_amd.serve import Predictor, make_app

    want = _train(tmp_path, "lr")
    p = Predictor(str(tmp_path / "ck"), device=torch.device("cpu"))
    c = TestClient(make_app(p))
    assert c.get("/health").json()["keys"] == p.keys
    lines = _test_text().decode().splitlines()[:5]
    r = c.post("/predict", json={"libffm": "\n".join(lines)})
    assert r.status_code == 200
    np.testing.assert_allclose(r.json()["pctr"], want[:5, 0], rtol=2e-5, atol=1e-6)
    from xflow_amd import native

    blk = native.load().parse_libffm(("\n".join(lines) + "\n").encode())
    rp = np.asarray(blk["row_ptr"])
    keys = np.asarray(blk["keys"]).view(np.uint64)
    rows = [[int(k) for k in keys[rp[i]:rp[i + 1]]] for i in range(len(rp) - 1)]
    r2 = c.post("/predict", json={"keys": rows})
    np.testing.assert_allclose(r2.json()["pctr"], r.json()["pctr"], rtol=0, atol=0)
    assert c.post("/predict", json={}).status_code == 400


@pytest.mark.gpu
def test_predictor_gpu_equals_cpu(gpu_device, tmp_path):
    """The GPU forward serves the same predictions as the CPU backend."""
    from xflow_amd.serve import Predictor

    _train(tmp_path, "fm")
    a = Predictor(str(tmp_path / "ck"), device=gpu_device).predict_libffm(_test_text())
    b = Predictor(str(tmp_path / "ck"), device=torch.device("cpu")).predict_libffm(_test_text())
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)


def test_mvm_keys_api_needs_field_ids(tmp_path):
    """An MVM model multiplies per-field sums: scoring hashed keys without
    their field ids is refused (HTTP 400), and with them equals the libffm
    path.  The Predictor sizes its table from the shard headers."""
    from fastapi.testclient import TestClient

    from xflow_amd import checkpoint, native
    from xflow_amd.serve import Predictor, make_app

    want = _train(tmp_path, "mvm")
    p = Predictor(str(tmp_path / "ck"), device=torch.device("cpu"))
    shards = [os.path.join(p.ckpt, f) for f in os.listdir(p.ckpt) if f.endswith(".xftb")]
    assert sum(checkpoint.shard_keys(f) for f in shards) == p.keys == \
        sum(len(checkpoint.read_shard(f)[1]) for f in shards)
    c = TestClient(make_app(p))
    lines = _test_text().decode().splitlines()[:6]
    blk = native.load().parse_libffm(("\n".join(lines) + "\n").encode())
    rp = np.asarray(blk["row_ptr"])
    keys = np.asarray(blk["keys"]).view(np.uint64)
    fg = np.asarray(blk["fgid"])
    rows = [[int(k) for k in keys[rp[i]:rp[i + 1]]] for i in range(len(rp) - 1)]
    fields = [[int(g) for g in fg[rp[i]:rp[i + 1]]] for i in range(len(rp) - 1)]
    assert c.post("/predict", json={"keys": rows}).status_code == 400
    r = c.post("/predict", json={"keys": rows, "fields": fields})
    assert r.status_code == 200
    np.testing.assert_allclose(r.json()["pctr"], want[:6, 0], rtol=2e-5, atol=1e-6)
