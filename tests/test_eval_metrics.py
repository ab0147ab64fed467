"""Device-side AUC / logloss (Engine.eval_metrics, csrc/hip/kernels_eval.hip:
stable radix sort + rank sums) against the reference printer semantics
(base.h:84-110, native reference_auc) and a numpy definition."""
import os

import numpy as np
import pytest
import torch

from conftest import DATA
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig, TrainConfig
from xflow_amd.engine import Engine
from xflow_amd.metrics import reference_auc

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(name):
    return torch.device("cuda", 0) if name == "cuda" else torch.device("cpu")


def _np_metrics(p, y):
    order = np.argsort(-p, kind="stable")
    ys = y[order].astype(np.int64)  # (exact integer sums)
    tp_before = np.cumsum(ys) - ys
    area = int(tp_before[ys == 0].sum())
    return area, int(ys.sum())


@pytest.mark.parametrize("devname", DEVS)
@pytest.mark.parametrize("n,ties", [(200, False), (5000, True), (1_000_003, False)])
def test_eval_metrics_exact_area(devname, n, ties):
    dev = _dev(devname)
    if devname == "cpu" and n > 100000:
        pytest.skip("large case on the GPU only")
    rng = np.random.default_rng(n)
    p = rng.random(n).astype(np.float32) * 0.999 + 1e-6
    if ties:
        p = (np.round(p * 50) / 50 + 1e-6).astype(np.float32)
    y = (rng.random(n) < 0.3).astype(np.float32)
    e = Engine(ModelConfig(), OptimConfig(), EngineConfig(table_log2_cap=8), device=dev)
    r = e.eval_metrics(torch.from_numpy(p).to(dev), torch.from_numpy(y).to(dev))
    area, tp = _np_metrics(p, y)
    assert r["n"] == n and r["tp"] == tp and r["area"] == area
    auc = area / (tp * (n - tp))
    assert abs(r["auc"] - auc) <= 1e-6 * auc + 1e-7
    pc = np.clip(p, 1e-7, 1 - 1e-7).astype(np.float64)
    ll = -(y * np.log(pc) + (1 - y) * np.log1p(-pc)).mean()
    assert abs(r["ln_logloss"] - ll) <= 1e-9 * abs(ll)
    if n <= 5000 and not ties:  # the reference printer (float accumulators) agrees exactly
        ref = reference_auc(y.astype(np.int32), p)
        assert r["line"] == ref["line"], (r["line"], ref["line"])


@pytest.mark.parametrize("devname", DEVS)
def test_trainer_eval_on_bundled_data(devname, tmp_path):
    """Bundled data: the trainer prints the reference's line (reference_auc of
    its predictions, pred file written) and logs the device AUC, which equals
    the stable-tie definition of the same predictions."""
    import json

    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=os.path.join(DATA, "small_train"),
                      test_prefix=os.path.join(DATA, "small_test"), epochs=10, threads=8,
                      pred_dir=str(tmp_path), model=ModelConfig(kind="lr"),
                      metrics_file=str(tmp_path / "m.jsonl"),
                      engine=EngineConfig(table_log2_cap=14))
    res = Trainer(cfg, device=_dev(devname)).train()
    pred = np.loadtxt(tmp_path / "pred_0_0.txt")
    ref = reference_auc(pred[:, 2].astype(np.int32), pred[:, 0].astype(np.float32))
    assert res["line"] == ref["line"] and res["n"] == 200
    ev = [json.loads(l) for l in open(tmp_path / "m.jsonl") if '"eval"' in l][-1]
    p, y = pred[:, 0].astype(np.float32), pred[:, 2].astype(np.float32)
    area, tp = _np_metrics(p, y)
    # (pred file values are %g-rounded: equal up to the rounding's ties)
    assert abs(ev["auc_device"] - area / (tp * (200 - tp))) < 2e-3
