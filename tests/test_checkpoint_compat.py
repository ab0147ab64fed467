"""Resume compatibility (xflow_amd/checkpoint.py check_compatible): fields
that define the table's meaning must match; hyperparameters and kernel
choices may change on resume (warning only)."""
import warnings

import numpy as np
import pytest
import torch

from helpers import random_csr, to_batch
from xflow_amd import checkpoint
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine


def _eng(model=None, optim=None):
    return Engine(model or ModelConfig(kind="fm", v_dim=4), optim or OptimConfig(),
                  EngineConfig(table_log2_cap=12, max_rows=64, max_nnz=1024))


def test_resume_with_changed_schedule_warns_and_loads(tmp_path):
    e = _eng()
    k, rp, fg, lab = random_csr(64, 6, seed=1)
    e.train_step(to_batch(k, rp, fg, lab, torch.device("cpu")))
    checkpoint.save(e, str(tmp_path), 0, 1, barrier=lambda: None)
    keys, _ = e.export_table()
    f = _eng(ModelConfig(kind="fm", v_dim=4, fm_mfma=True), OptimConfig(lambda1=1e-3, alpha=0.1))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        checkpoint.load(f, str(tmp_path), 0, 1)
    assert any("changed" in str(x.message) for x in w)
    # (the state is the same; the weights differ only through the new hyperparameters)
    assert f.table_size() == e.table_size() == len(keys)
    g = _eng(ModelConfig(kind="fm", v_dim=4, fm_mfma=True), OptimConfig())
    checkpoint.load(g, str(tmp_path), 0, 1)
    np.testing.assert_array_equal(g.pull(keys), e.pull(keys))


def test_resume_with_changed_layout_raises(tmp_path):
    e = _eng()
    checkpoint.save(e, str(tmp_path), 0, 1, barrier=lambda: None)
    with pytest.raises(ValueError, match="differs"):
        checkpoint.load(_eng(ModelConfig(kind="fm", v_dim=4, fm_math="standard")), str(tmp_path), 0, 1)
