"""End-to-end parity with the reference's semantics on the bundled data:
an independent pure-Python oracle (xflow_amd/testing/oracle.py, written from
the reference sources) vs the engine driven by the Python trainer and by the
native C++ trainer (the code behind xflow_lr and the C API)."""
import os

import numpy as np
import pytest
import torch

from conftest import DATA
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig, TrainConfig
from xflow_amd.testing import oracle
from xflow_amd.testing.hashing import normal_init

TRAIN = os.path.join(DATA, "small_train")
TEST = os.path.join(DATA, "small_test")


def v_init(key, k):
    return float(normal_init(np.array([key], dtype=np.uint64), k)[0] * np.float32(1e-2))


def run_oracle(kind, opt, epochs, threads=8, concurrent=False, fm_math="reference",
               mvm_math="compat", v_dim=10):
    o = oracle.Oracle(kind, opt, v_dim, fm_math, mvm_math, threads, v_init, concurrent)
    o.init_push()
    tr = oracle.parse_file(TRAIN + "-00000")
    te = oracle.parse_file(TEST + "-00000")
    for _ in range(epochs):
        o.train_block(tr)
    return o.predict(te)


def run_trainer(tmp_path, kind, opt, epochs, threads=8, serial=True, fm_math="reference",
                mvm_math="compat", v_dim=10):
    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=TRAIN, test_prefix=TEST, epochs=epochs, threads=threads,
                      serial_slices=serial, pred_dir=str(tmp_path),
                      model=ModelConfig(kind=kind, v_dim=v_dim, fm_math=fm_math,
                                        mvm_math=mvm_math),
                      optim=OptimConfig(kind=opt), engine=EngineConfig(table_log2_cap=14))
    t = Trainer(cfg, device=torch.device("cpu"))
    res = t.train()
    pred = np.loadtxt(os.path.join(str(tmp_path), "pred_0_0.txt"), ndmin=2)
    return res, pred


CASES = [("lr", "ftrl", 10, "reference", "compat"),
         ("lr", "sgd", 5, "reference", "compat"),
         ("fm", "ftrl", 3, "reference", "compat"),
         ("fm", "ftrl", 3, "standard", "compat"),
         ("mvm", "ftrl", 3, "reference", "compat"),
         ("mvm", "ftrl", 2, "reference", "fixed")]


@pytest.mark.parametrize("kind,opt,epochs,fm_math,mvm_math", CASES)
def test_serial_slices_match_oracle(tmp_path, kind, opt, epochs, fm_math, mvm_math):
    want = run_oracle(kind, opt, epochs, fm_math=fm_math, mvm_math=mvm_math)
    res, pred = run_trainer(tmp_path, kind, opt, epochs, fm_math=fm_math, mvm_math=mvm_math)
    assert pred.shape[0] == len(want) == 200
    np.testing.assert_array_equal(pred[:, 2].astype(int), [w[0] for w in want])
    np.testing.assert_array_equal(pred[:, 1].astype(int), [1 - w[0] for w in want])
    np.testing.assert_allclose(pred[:, 0], [w[1] for w in want], rtol=2e-4, atol=2e-6)
    ll, auc = oracle.calculate_auc(want)
    assert abs(res["logloss_printed"] - ll) < 5e-4
    if np.ptp(pred[:, 0]) > 1e-5:  # MVM's products ~0 give pctr ~0.5: AUC = tie order
        assert abs(res["auc"] - auc) < 5e-3


def test_concurrent_slices_match_oracle(tmp_path):
    want = run_oracle("lr", "ftrl", 10, concurrent=True)
    _, pred = run_trainer(tmp_path, "lr", "ftrl", 10, serial=False)
    np.testing.assert_allclose(pred[:, 0], [w[1] for w in want], rtol=2e-4, atol=2e-6)


def test_appendix_c_anchor_native_trainer(native, tmp_path):
    """LR-FTRL, 100 epochs, 1 worker, 8 slices (SURVEY.md Appendix C:
    printed -0.7820 / AUC 0.5881 for the serial emulation)."""
    t = native.Trainer({"train_prefix": TRAIN, "test_prefix": TEST, "model": 0, "epochs": 100,
                        "threads": 8, "serial_slices": True, "pred_dir": str(tmp_path),
                        "device": -1, "verbose": False, "table_log2_cap": 14})
    t.train_epochs(100)
    r = t.predict(0)
    assert abs(r["logloss_printed"] - (-0.7820)) < 2e-3
    assert abs(r["auc"] - 0.5881) < 2e-3
    assert r["line"].startswith("logloss: ") and "\tauc = " in r["line"] and \
        r["line"].endswith("tp = 46 fp = 154")


def test_mvm_predict_compat_emits_vdim_rows_per_slice(tmp_path):
    from xflow_amd.trainer import Trainer

    cfg = TrainConfig(train_prefix=TRAIN, test_prefix=TEST, epochs=1, threads=8,
                      mvm_predict_compat=True, pred_dir=str(tmp_path),
                      model=ModelConfig(kind="mvm"), engine=EngineConfig(table_log2_cap=14))
    res = Trainer(cfg, device=torch.device("cpu")).train()
    assert res["n"] == 8 * 10  # v_multi.size() rows per slice (mvm_worker.cc:96)


# ---- the reference's default slice count: hardware_concurrency threads ----
# (lr_worker.h:40-41).  An MI355X host has far more than 32 hardware threads;
# a block of fewer rows than threads trains (and predicts) nothing
# (lr_worker.cc:190-199), a larger thread count than 32 runs as slice groups.

@pytest.mark.parametrize("threads,epochs", [(64, 10), (40, 4)])
def test_many_concurrent_slices_match_oracle(tmp_path, threads, epochs):
    want = run_oracle("lr", "ftrl", epochs, threads=threads, concurrent=True)
    res, pred = run_trainer(tmp_path, "lr", "ftrl", epochs, threads=threads, serial=False)
    assert len(want) == pred.shape[0] == (200 // threads) * threads
    np.testing.assert_allclose(pred[:, 0], [w[1] for w in want], rtol=2e-4, atol=2e-6)
    ll, _ = oracle.calculate_auc(want)
    assert abs(res["logloss_printed"] - ll) < 5e-4


def test_default_threads_on_a_256_thread_host_python_cli(tmp_path, monkeypatch, capsys):
    """`xflow_lr <train> <test> 0 10` with no --threads on a 256-thread host:
    every 200-row block has fewer rows than threads, so -- like the
    reference -- nothing is trained or predicted, and the run completes."""
    from xflow_amd import cli

    monkeypatch.setattr(os, "cpu_count", lambda: 256)
    want = run_oracle("lr", "ftrl", 10, threads=256, concurrent=True)
    assert want == []
    rc = cli.main([TRAIN, TEST, "0", "10", "--cpu", "--pred-dir", str(tmp_path),
                   "--log2-cap", "14"])
    assert rc in (0, None)
    out = capsys.readouterr().out
    assert "logloss: 0\ttp_n = 0" in out and "train end......" in out
    assert os.path.getsize(os.path.join(str(tmp_path), "pred_0_0.txt")) == 0


@pytest.mark.parametrize("hw", [256, 48])
def test_default_threads_native_cli(tmp_path, hw):
    """The native xflow_lr binary with its default thread count
    (hardware_concurrency, here XFLOW_HARDWARE_CONCURRENCY) on the bundled
    data: 256 threads train nothing; 48 threads = two slice groups per block,
    predictions equal to the oracle's."""
    import subprocess

    from xflow_amd import _build

    binp = os.path.join(_build.BUILD, "bin", "xflow_lr")
    env = dict(os.environ, XFLOW_HARDWARE_CONCURRENCY=str(hw), XFLOW_PRED_DIR=str(tmp_path))
    r = subprocess.run([binp, TRAIN, TEST, "0", "4", "--device", "-1"], cwd=str(tmp_path),
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    want = run_oracle("lr", "ftrl", 4, threads=hw, concurrent=True)
    pred = np.loadtxt(os.path.join(str(tmp_path), "pred_0_0.txt"), ndmin=2)
    if hw == 256:
        assert want == [] and pred.size == 0
        assert "tp_n = 0" in r.stdout
    else:
        assert pred.shape[0] == len(want) == (200 // hw) * hw
        np.testing.assert_allclose(pred[:, 0], [w[1] for w in want], rtol=2e-4, atol=2e-6)


def test_mvm_ftrl_liveness_pinned_at_reference_slicing(tmp_path):
    """MVM-FTRL's liveness, pinned with the oracle at the reference's own
    slicing (one 2 MB block = the whole 200-row shard, hardware_concurrency = 8
    slices, mvm_worker.cc:286-296) and init (N(0,1)*1e-2, ftrl.h:114-120):
    the 17-field product of field sums (~1e-34) is already 0 in float32
    before any push, so every prediction is exactly 0.5 -- before training
    and after (the first pushes set v from (z, n), no larger).  The engine
    reproduces it: the reference's own MVM does not learn on its own data,
    and bench rows of MVM-FTRL are labelled degenerate for the same reason."""
    o = oracle.Oracle("mvm", "ftrl", 10, "reference", "compat", 8, v_init)
    o.init_push()
    te = oracle.parse_file(TEST + "-00000")
    assert all(p == 0.5 for _, p in o.predict(te))  # dead at init
    tr = oracle.parse_file(TRAIN + "-00000")
    for _ in range(3):
        o.train_block(tr)
    assert all(p == 0.5 for _, p in o.predict(te))  # and after three epochs
    res, pred = run_trainer(tmp_path, "mvm", "ftrl", 3)
    assert np.all(pred[:, 0] == 0.5)
